// DeformConv2d (operators/Deformable_convolution.py:5-146): modulated DCNv2 with the reference's
// semantics (offset channels [rows | cols], p_0 = 1 + idx * stride, floor of the UNclamped p,
// corners and p clamped to the zero-padded map, sigmoid modulation, k x k stride-k conv, no bias).
//
// The contractions keep fp32-level accuracy: the forward's on the bf16 matrix cores with every
// fp32 operand split into three bf16 parts (six products per pair, split3 / mfma6 below: the
// dropped terms are below 2^-26 relative), the backward's on fp32 MFMA (v_mfma_f32_32x32x2_f32:
// exact f32 products, one rounding per step).  GEMM views, with
// M = B*Ho*Wo output pixels, N = k*k kernel points and the reduction index ordered K' = n*C + c
// (a permutation of conv.weight's c*N + n, applied to the weight copies below):
//   forward      out[o, m]   = sum_K' Wf[o, K'] * cols[K', m]
//   backward     dcols[m, c] = sum_o dout[o, m] * Wb[n, o, c]   (per n) -> dx, d_offset, d_mask
//                dWp[o,n,c]  = sum_m dout[o, m] * cols[(n,c), m]
// cols[(n,c), m] = sigmoid(mask) * sum_q g_q * x[corner_q] is never materialised: it is built per
// 32-channel K'-tile into LDS from per-(pixel, kernel point) coefficients computed once
// (k_dcn_coef), reading x channels-last (xt) so the four corner gathers of a pixel are
// contiguous channel vectors, and it is shared by every output channel of the tile.
// dx is a gather, not a scatter: the backward-data kernel writes the dcols rows, and one wave
// per input pixel sums the rows whose bilinear corners land on it (lists built by a counting sort
// on integer counters), written back as NCHW rows.  Roofline: MFMA-bound (2*M*O*C*N
// flops forward, 2x backward).
#include <hipcub/hipcub.hpp>

#include "sbod_common.h"

// The forward's contraction on the split-bf16 matrix cores (k_dcn_fwd3) unless an A/B build asks
// for the fp32-MFMA kernel (-DSBOD_DCN_FP32_FWD); the backward-data split form is a variant only
// (-DSBOD_DCN_SPLIT_BF16: measured no faster).
#ifndef SBOD_DCN_FP32_FWD
#define SBOD_DCN_SPLIT_FWD 1
#endif

namespace sbod {

typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));

#if defined(SBOD_DCN_SPLIT_BF16) || defined(SBOD_DCN_SPLIT_FWD)
// ---- split-bf16 contraction (the fp32 products on the bf16 matrix cores).  An fp32 value is the
// exact sum of three bf16 parts, x = h + m + l (h = bf16(x) round-to-nearest-even, m =
// bf16(x - h), l = x - h - m: 24 significant bits = 3 x 8, every subtraction exact).  A product
// a*b is then sum_{i,j} a_i b_j; the six terms of order <= 2^-16 relative (hh, hm, mh, hl, lh,
// mm) are kept, the three below 2^-26 (ml, lm, ll) dropped, every bf16 x bf16 product is exact
// in the MFMA's fp32 accumulation — so each K = 16 step adds its products with fp32-level error
// (<= 2^-25 relative per product from the dropped terms), as the fp32 MFMA does, at 6
// v_mfma_f32_32x32x16_bf16 (32 cycles each) per 16 K instead of 8 v_mfma_f32_32x32x2_f32 (64
// cycles each): 2.7x the fp32 matrix rate (MI355X_MICROARCH.md: fp32 MFMA runs at the fp32 vector
// rate, 1/16 of bf16).  Non-finite inputs give NaN (inf - inf in the split), not +-inf.
__device__ __forceinline__ void split3(float x, __bf16 &h, __bf16 &m, __bf16 &l) {
  h = static_cast<__bf16>(x);
  const float r = x - static_cast<float>(h);
  m = static_cast<__bf16>(r);
  l = static_cast<__bf16>(r - static_cast<float>(m));
}
struct Split8 {
  bf16x8 p[3];   // high, middle, low parts of 8 consecutive K values
};
__device__ __forceinline__ Split8 split8(const float (&v)[8]) {
  Split8 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    __bf16 h, m, l;
    split3(v[i], h, m, l);
    r.p[0][i] = h;
    r.p[1][i] = m;
    r.p[2][i] = l;
  }
  return r;
}
// acc += A[32 x 16] B[16 x 32] from the split parts: the small terms first
__device__ __forceinline__ f32x16 mfma6(const bf16x8 (&a)[3], const bf16x8 (&b)[3], f32x16 acc) {
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[2], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[2], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[1], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[1], b[0], acc, 0, 0, 0);
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[0], b[0], acc, 0, 0, 0);
  return acc;
}

#endif  // split-bf16 helpers

constexpr int kDcnThreads = 256;
constexpr int kMaxN = 49;      // k*k <= 49 (k <= 7)

// Per (pixel m, kernel point n): corner offsets in the image plane (-1 outside the original
// map: zero padding), bilinear weights g (unmodulated), mask value, and the derivative terms.
struct Coef {
  int idx[4];          // lt, rb, lb, rt
  float g[4];
  float mval;          // sigmoid(mask logit) (1 without modulation)
  float tlx, rbx, tly, rby;  // q_lt.x - p.x, q_rb.x - p.x, q_lt.y - p.y, q_rb.y - p.y (clamped p)
  int inr;             // bit 0: 0 <= p.x <= Hp-1, bit 1: 0 <= p.y <= Wp-1 (clamp passes gradient)
};
static_assert(sizeof(Coef) == 56, "Coef layout");

struct DcnShape {
  int B, C, H, W, O, k, N, stride, pad, Ho, Wo, Hp, Wp, M, K;
};

// Grid-stride zero fill of n floats (16-B stores where aligned) by every thread of a launch: the
// zero-initialised outputs of a later kernel ride along with an earlier one instead of a memset node.
__device__ __forceinline__ void zero_fill(float *p, int64_t n) {
  if (!p || n <= 0) return;
  const int64_t nthr = static_cast<int64_t>(gridDim.x) * gridDim.y * gridDim.z * blockDim.x;
  const int64_t id = (static_cast<int64_t>(blockIdx.z) * gridDim.y * gridDim.x +
                      static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t head = (reinterpret_cast<uintptr_t>(p) & 15) ? n : 0;   // unaligned: scalar stores only
  const int64_t n4 = (n - head) >> 2;
  float4 *p4 = reinterpret_cast<float4 *>(p);
  for (int64_t i = id; i < n4; i += nthr) p4[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  for (int64_t i = 4 * n4 + id; i < n; i += nthr) p[i] = 0.f;
}

__global__ __launch_bounds__(256) void k_dcn_coef(DcnShape s, const float *__restrict__ offset,
                                                  const float *__restrict__ mlog,
                                                  Coef *__restrict__ coef, uint32_t *__restrict__ tcount,
                                                  float *__restrict__ zero_out, int64_t n_zero) {
  zero_fill(zero_out, n_zero);   // the split-K forward's output, accumulated by k_dcn_fwd
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= static_cast<int64_t>(s.M) * s.N) return;
  const int n = static_cast<int>(t % s.N);
  const int m = static_cast<int>(t / s.N);
  const int HWo = s.Ho * s.Wo;
  const int b = m / HWo, pix = m - b * HWo, h = pix / s.Wo, w = pix - h * s.Wo;
  const int i = n / s.k, j = n - i * s.k;
  // p_n = arange((-(k-1))//2, (k-1)//2 + 1) (Deformable_convolution.py:93-101): floor(-(k-1)/2) = -(k/2)
  const int base = -(s.k / 2);
  const float off_x = offset[((static_cast<int64_t>(b) * 2 * s.N + n) * s.Ho + h) * s.Wo + w];
  const float off_y = offset[((static_cast<int64_t>(b) * 2 * s.N + s.N + n) * s.Ho + h) * s.Wo + w];
  const float px = static_cast<float>(1 + h * s.stride + base + i) + off_x;
  const float py = static_cast<float>(1 + w * s.stride + base + j) + off_y;
  const float fx = floorf(px), fy = floorf(py);
  const float hx = static_cast<float>(s.Hp - 1), hy = static_cast<float>(s.Wp - 1);
  const float ltx = fminf(fmaxf(fx, 0.f), hx), lty = fminf(fmaxf(fy, 0.f), hy);
  const float rbx = fminf(fmaxf(fx + 1.f, 0.f), hx), rby = fminf(fmaxf(fy + 1.f, 0.f), hy);
  const float pcx = fminf(fmaxf(px, 0.f), hx), pcy = fminf(fmaxf(py, 0.f), hy);
  Coef c;
  c.tlx = ltx - pcx;
  c.rbx = rbx - pcx;
  c.tly = lty - pcy;
  c.rby = rby - pcy;
  c.g[0] = (1.f + c.tlx) * (1.f + c.tly);   // lt   (Deformable_convolution.py:64-67)
  c.g[1] = (1.f - c.rbx) * (1.f - c.rby);   // rb
  c.g[2] = (1.f + c.tlx) * (1.f - c.rby);   // lb
  c.g[3] = (1.f - c.rbx) * (1.f + c.tly);   // rt
  const int qx[4] = {static_cast<int>(ltx), static_cast<int>(rbx), static_cast<int>(ltx), static_cast<int>(rbx)};
  const int qy[4] = {static_cast<int>(lty), static_cast<int>(rby), static_cast<int>(rby), static_cast<int>(lty)};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int yy = qx[q] - s.pad, xx = qy[q] - s.pad;   // padded -> original coordinates
    c.idx[q] = (yy >= 0 && yy < s.H && xx >= 0 && xx < s.W) ? yy * s.W + xx : -1;
  }
  if (mlog) {
    const float z = mlog[((static_cast<int64_t>(b) * s.N + n) * s.Ho + h) * s.Wo + w];
    c.mval = 1.f / (1.f + expf(-z));
  } else {
    c.mval = 1.f;
  }
  c.inr = ((px >= 0.f && px <= hx) ? 1 : 0) | ((py >= 0.f && py <= hy) ? 2 : 0);
  coef[t] = c;
  if (tcount) {   // backward: how many corner samples land on each input pixel (dx gather lists)
    const int64_t ib = static_cast<int64_t>(b) * s.H * s.W;
#pragma unroll
    for (int q = 0; q < 4; ++q)
      if (c.idx[q] >= 0) atomicAdd(tcount + ib + c.idx[q], 1u);
  }
}


// Batched transpose in [nb][R][S] -> out [nb][S][R] (64 x 64 LDS tiles); zeroes `zero` [n_zero]
// on the side (the sample counters the coefficient pass that follows increments).
__global__ __launch_bounds__(256) void k_transpose(const float *__restrict__ in, float *__restrict__ out,
                                                   int R, int S, float *__restrict__ zero, int64_t n_zero) {
  zero_fill(zero, n_zero);
  __shared__ float t[64][65];
  const int s0 = blockIdx.x * 64, r0 = blockIdx.y * 64;
  const int64_t base = static_cast<int64_t>(blockIdx.z) * R * S;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int r = r0 + i, s = s0 + tx;
    t[i][tx] = (r < R && s < S) ? in[base + static_cast<int64_t>(r) * S + s] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int s = s0 + i, r = r0 + tx;
    if (r < R && s < S) out[base + static_cast<int64_t>(s) * R + r] = t[tx][i];
  }
}

// conv.weight [O][C][N] -> the forward's Wf [O][N][C] and (training) the backward's Wb [N][O][C]
// in one pass: one block per (64-channel chunk, output channel), the chunk's 64 x N contiguous
// weights staged in LDS, each layout's rows written along c.
// With wf3 (the split-bf16 forward), Wf's three bf16 parts [3][O][N][C] are written in the same
// pass (split3 of each weight).
__global__ __launch_bounds__(256) void k_weight_layouts(const float *__restrict__ w, int O, int C, int N,
                                                        float *__restrict__ wf, float *__restrict__ wb,
                                                        __bf16 *__restrict__ wf3) {
  __shared__ float t[64][kMaxN + 1];
  const int c0 = blockIdx.x * 64, o = blockIdx.y;
  const int nc = min(64, C - c0);
  const float *src = w + (static_cast<int64_t>(o) * C + c0) * N;
  for (int e = threadIdx.x; e < nc * N; e += blockDim.x) t[e / N][e % N] = src[e];
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * N; e += blockDim.x) {
    const int n = e >> 6, cl = e & 63;
    if (cl >= nc) continue;
    const float v = t[cl][n];
    const int64_t fi = (static_cast<int64_t>(o) * N + n) * C + c0 + cl;
    wf[fi] = v;
    if (wb) wb[(static_cast<int64_t>(n) * O + o) * C + c0 + cl] = v;
#if defined(SBOD_DCN_SPLIT_BF16) || defined(SBOD_DCN_SPLIT_FWD)
    if (wf3) {
      const int64_t part = static_cast<int64_t>(O) * N * C;
      __bf16 hp, mp, lp;
      split3(v, hp, mp, lp);
      wf3[fi] = hp;
      wf3[part + fi] = mp;
      wf3[2 * part + fi] = lp;
    }
#endif
  }
}

#ifdef SBOD_DCN_SPLIT_BF16
// The backward-data B operand: Wf [O][N][C] fp32 -> wb3 [3][N][C][Op] bf16 split parts, output
// channels contiguous (the MFMA's K), zero past O (Op = O rounded up to 64).  64 x 64 tiles of
// (o, c) per kernel point through LDS.
__global__ __launch_bounds__(256) void k_wb_split(const float *__restrict__ wf, int O, int C, int N, int Op,
                                                  __bf16 *__restrict__ wb3) {
  __shared__ float t[64][65];
  const int c0 = blockIdx.x * 64, o0 = blockIdx.y * 64, n = blockIdx.z;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int o = o0 + i, c = c0 + tx;
    t[i][tx] = (o < O && c < C) ? wf[(static_cast<int64_t>(o) * N + n) * C + c] : 0.f;
  }
  __syncthreads();
  const int64_t part = static_cast<int64_t>(N) * C * Op;
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i;
    if (c >= C) continue;
    __bf16 h, m, l;
    split3(t[tx][i], h, m, l);
    __bf16 *d = wb3 + (static_cast<int64_t>(n) * C + c) * Op + o0 + tx;
    d[0] = h;
    d[part] = m;
    d[2 * part] = l;
  }
}
inline int dcn_opad(int O) { return (O + 63) / 64 * 64; }

#endif  // SBOD_DCN_SPLIT_BF16

// Bilinear combination in the reference's order: ((lt + rb) + lb) + rt, then * mask.
__device__ __forceinline__ float combine(const float g[4], float m, float x0, float x1, float x2, float x3) {
  return (((g[0] * x0 + g[1] * x1) + g[2] * x2) + g[3] * x3) * m;
}

template <int VEC>
__device__ __forceinline__ void load_vec(const float *p, bool ok, float *v) {
  if (VEC == 4) {
    const float4 t = ok ? *reinterpret_cast<const float4 *>(p) : make_float4(0.f, 0.f, 0.f, 0.f);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else {
    v[0] = ok ? *p : 0.f;
  }
}

// XCD-aware workgroup order.  The dispatcher deals workgroups to the 8 XCDs round-robin, so
// consecutive logical tiles (which share corner rows of x, dout pixel rows or a weight slice)
// would land on 8 different L2s.  Dispatch id L -> logical id: each XCD gets one contiguous
// range of logical tiles (a bijection for any total).
struct Tile3 {
  int x, y, z;
};
__device__ __forceinline__ int xcd_logical(int L, int total) {
  const int q = total >> 3, r = total & 7, x = L & 7, pos = L >> 3;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + pos;
}
// the logical id decomposed with extents (nx fastest, ny, nz)
__device__ __forceinline__ Tile3 xcd_tile(int nx, int ny, int nz) {
  const int L = static_cast<int>(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z));
  const int lam = xcd_logical(L, nx * ny * nz);
  const int x = lam % nx, rest = lam / nx;
  return Tile3{x, rest % ny, rest / ny};
}

// ----------------------------------------------------------------------------- forward
// Block: 64 pixels x 256 output channels, 4 waves x (64 channels x 64 pixels) = 2 x 2 MFMA tiles.
// K'-tiles of 32 channels of one kernel point; blockIdx.z takes a contiguous share of them
// (split-K for small maps, combined with float atomics).  One tile of gathers is in flight while
// the previous tile's MFMAs run (double-buffered LDS, one barrier per tile); the weights are
// single-buffered (loaded after the MFMAs that read them), 3 workgroups per CU.
constexpr int kFM = 64, kFKC = 32, kFLD = kFM + 2;

#ifndef SBOD_DCN_FWD_WAVES
#define SBOD_DCN_FWD_WAVES 3
#endif
template <int VEC>
__global__ __launch_bounds__(kDcnThreads, VEC == 4 ? SBOD_DCN_FWD_WAVES : 2) void k_dcn_fwd(DcnShape s, const float *__restrict__ xt,
                                                            const Coef *__restrict__ coef,
                                                            const float *__restrict__ wf,
                                                            float *__restrict__ out, int atomic_out) {
  __shared__ float s_cols[2][kFKC][kFLD];
  extern __shared__ float s_coefd[];        // dynamic [N][9][kFM]: idx[4] | g[4] | mask of each pixel
  float (*s_coef)[9][kFM] = reinterpret_cast<float (*)[9][kFM]>(s_coefd);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, l31 = lane & 31;
  const Tile3 tl = xcd_tile(gridDim.x, gridDim.y, gridDim.z);   // consecutive pixel tiles share an L2
  const int m0 = tl.x * kFM, o0 = tl.y * 256;
  const int HWo = s.Ho * s.Wo, HW = s.H * s.W;
  const int CT = (s.C + kFKC - 1) / kFKC, T = s.N * CT;
  const int t0 = static_cast<int>(static_cast<int64_t>(tl.z) * T / gridDim.z);
  const int t1 = static_cast<int>(static_cast<int64_t>(tl.z + 1) * T / gridDim.z);
  // sampler role: pixel mm, 8 channels starting at 8 * cq
  const int mm = tid & 63, cq = tid >> 6;
  // pixels past M sample a clamped pixel: their columns only reach output columns that are never
  // stored.  Every operand load below is unconditional (clamped addresses, zero selects applied
  // when the columns are stored), so the loop is straight-line code and the waits the compiler
  // places before the MFMAs cover exactly the weights they read, not the gathers in flight.
  const int ms = min(m0 + mm, s.M - 1);
  const float *xb = xt + static_cast<int64_t>(ms / HWo) * HW * s.C;
  struct Cf {
    int idx[4];
    float g[4], m;
  };
  // the block's coefficients (every kernel point of its 64 pixels) staged in LDS once: the
  // gathers then depend on LDS reads only, never on a global load in flight
  for (int e = tid; e < s.N * kFM; e += kDcnThreads) {
    const int n = e / kFM, px = e - n * kFM;
    const float *c = reinterpret_cast<const float *>(coef + static_cast<int64_t>(min(m0 + px, s.M - 1)) * s.N + n);
#pragma unroll
    for (int j = 0; j < 9; ++j) s_coef[n][j][px] = c[j];
  }
  __syncthreads();
  // K'-tile order t = channel chunk * N + kernel point: consecutive tiles sample the same 32
  // channels at the 3x3 neighbourhood's positions, so their corner lines are still in L2 (the
  // kernel-point-major order revisited every line only after N chunks' worth of other lines)
  auto load_coef = [&](int t) {   // idx, g and mask of this pixel's kernel point for tile t
    const int n = t % s.N;
    Cf c;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      c.idx[q] = __builtin_bit_cast(int, s_coef[n][q][mm]);
      c.g[q] = s_coef[n][4 + q][mm];
    }
    c.m = s_coef[n][8][mm];
    return c;
  };
  float X[4][8];
  bool xok[4][8 / VEC];
  float acur[2][16];   // one A buffer: the next tile's weights load once the MFMAs have read these
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  auto gather = [&](int t, const Cf &cf) {
    const int c0 = (t / s.N) * kFKC + 8 * cq;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float *p = xb + static_cast<int64_t>(max(cf.idx[q], 0)) * s.C;
#pragma unroll
      for (int v = 0; v < 8; v += VEC) {
        const int c = c0 + v;
        xok[q][v / VEC] = cf.idx[q] >= 0 && c < s.C;
        load_vec<VEC>(p + min(c, s.C - VEC), true, &X[q][v]);
      }
    }
  };
  auto store_cols = [&](int buf, const Cf &cf) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int v = 0; v < 8; ++v) X[q][v] = xok[q][v / VEC] ? X[q][v] : 0.f;
#pragma unroll
    for (int v = 0; v < 8; ++v)
      s_cols[buf][8 * cq + v][mm] = combine(cf.g, cf.m, X[0][v], X[1][v], X[2][v], X[3][v]);
  };
  auto load_a = [&](int t) {   // rows past O are never stored; columns past C meet zero columns
    const int ct = t / s.N, n = t - ct * s.N, c0 = ct * kFKC + 16 * h;
#pragma unroll
    for (int ri = 0; ri < 2; ++ri) {
      const int o = min(o0 + 64 * wv + 32 * ri + l31, s.O - 1);
      const float *p = wf + static_cast<int64_t>(o) * s.K + static_cast<int64_t>(n) * s.C;
#pragma unroll
      for (int v = 0; v < 16; v += VEC) load_vec<VEC>(p + min(c0 + v, s.C - VEC), true, &acur[ri][v]);
    }
  };

  if (t0 < t1) {
    Cf cf = load_coef(t0);
    gather(t0, cf);
    store_cols(0, cf);
    load_a(t0);
    __syncthreads();
    for (int t = t0; t < t1; ++t) {
      const int buf = (t - t0) & 1;
      const int tn = min(t + 1, t1 - 1);   // the last pass re-gathers its own tile into the idle buffer
      cf = load_coef(tn);
      gather(tn, cf);
      __builtin_amdgcn_sched_barrier(0);   // the prefetch stays ahead of the MFMAs
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const float b0 = s_cols[buf][16 * h + st][l31];
        const float b1 = s_cols[buf][16 * h + st][32 + l31];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(acur[0][st], b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(acur[0][st], b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(acur[1][st], b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(acur[1][st], b1, acc[1][1], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
      load_a(tn);   // L2-resident weights, in flight through the column store and barrier
      store_cols(buf ^ 1, cf);
      __syncthreads();
    }
  }
  // C/D map (gfx950, dtype independent): col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int bq = 0; bq < 2; ++bq) {
    const int m = m0 + 32 * bq + l31;
    if (m >= s.M) continue;
    const int b = m / HWo, pix = m - b * HWo;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = o0 + 64 * wv + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (o >= s.O) continue;
        float *dst = out + (static_cast<int64_t>(b) * s.O + o) * HWo + pix;
        if (atomic_out) atomicAdd(dst, acc[a][bq][r]);
        else *dst = acc[a][bq][r];
      }
  }
}

#ifdef SBOD_DCN_SPLIT_FWD
// The forward contraction on the split-bf16 matrix cores (mfma6): k_dcn_fwd's blocking, gathers,
// coefficient staging and K'-tile order, with (1) the weights' split parts precomputed
// (wf3 [3][O][N*C] bf16, written by k_weight_layouts) and loaded as 16-byte vectors of 8 consecutive channels into
// the A registers, (2) each combined column value split once by the thread that samples it and
// stored as three bf16 rows (LDS [buf][part][pixel][channel], a 40-element pitch: conflict-free
// 16-byte reads) — 48 bf16 MFMAs per K'-tile and wave instead of 64 fp32 ones at twice the cycles.
// C % 8 == 0 (16-byte weight vectors).
constexpr int kF3Pitch = 40;

__global__ __launch_bounds__(kDcnThreads, 2) void k_dcn_fwd3(DcnShape s, const float *__restrict__ xt,
                                                                            const Coef *__restrict__ coef,
                                                                            const __bf16 *__restrict__ wf3,
                                                                            float *__restrict__ out, int atomic_out) {
  __shared__ __attribute__((aligned(16))) __bf16 s_cols[2][3][kFM][kF3Pitch];
  extern __shared__ float s_coefd[];        // dynamic [N][9][kFM]: idx[4] | g[4] | mask of each pixel
  float (*s_coef)[9][kFM] = reinterpret_cast<float (*)[9][kFM]>(s_coefd);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, l31 = lane & 31;
  const Tile3 tl = xcd_tile(gridDim.x, gridDim.y, gridDim.z);
  const int m0 = tl.x * kFM, o0 = tl.y * 256;
  const int HWo = s.Ho * s.Wo, HW = s.H * s.W;
  const int CT = (s.C + kFKC - 1) / kFKC, T = s.N * CT;
  const int t0 = static_cast<int>(static_cast<int64_t>(tl.z) * T / gridDim.z);
  const int t1 = static_cast<int>(static_cast<int64_t>(tl.z + 1) * T / gridDim.z);
#ifdef SBOD_DCN_FWD3_WAVE_CHANNELS
  const int mm = tid & 63, cq = tid >> 6;   // (A/B form) a wave = 64 pixels x one channel group
#else
  // a lane quad = one pixel's 32 channels (128 contiguous bytes of xt per corner): a wave's
  // corner load touches 16 lines instead of 64, the same line no longer fetched by four waves
  const int mm = tid >> 2, cq = tid & 3;
#endif
  const int ms = min(m0 + mm, s.M - 1);
  const float *xb = xt + static_cast<int64_t>(ms / HWo) * HW * s.C;
  struct Cf {
    int idx[4];
    float g[4], m;
  };
  for (int e = tid; e < s.N * kFM; e += kDcnThreads) {
    const int n = e / kFM, px = e - n * kFM;
    const float *c = reinterpret_cast<const float *>(coef + static_cast<int64_t>(min(m0 + px, s.M - 1)) * s.N + n);
#pragma unroll
    for (int j = 0; j < 9; ++j) s_coef[n][j][px] = c[j];
  }
  __syncthreads();
  auto load_coef = [&](int t) {
    const int n = t % s.N;
    Cf c;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      c.idx[q] = __builtin_bit_cast(int, s_coef[n][q][mm]);
      c.g[q] = s_coef[n][4 + q][mm];
    }
    c.m = s_coef[n][8][mm];
    return c;
  };
  float X[4][8];
  bool xok[4][2];
  bf16x8 acur[2][2][3];   // [ri][j][part]: the next tile's weights load once the MFMAs have read these
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  auto gather = [&](int t, const Cf &cf, float (&XX)[4][8], bool (&ok)[4][2]) {
    const int c0 = (t / s.N) * kFKC + 8 * cq;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float *p = xb + static_cast<int64_t>(max(cf.idx[q], 0)) * s.C;
#pragma unroll
      for (int v = 0; v < 8; v += 4) {
        const int c = c0 + v;
        ok[q][v / 4] = cf.idx[q] >= 0 && c < s.C;
        load_vec<4>(p + min(c, s.C - 4), true, &XX[q][v]);
      }
    }
  };
  auto store_cols = [&](int buf, const Cf &cf, float (&XX)[4][8], const bool (&ok)[4][2]) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int v = 0; v < 8; ++v) XX[q][v] = ok[q][v / 4] ? XX[q][v] : 0.f;
    float col[8];
#pragma unroll
    for (int v = 0; v < 8; ++v) col[v] = combine(cf.g, cf.m, XX[0][v], XX[1][v], XX[2][v], XX[3][v]);
    const Split8 sp = split8(col);
#pragma unroll
    for (int p = 0; p < 3; ++p) *reinterpret_cast<bf16x8 *>(&s_cols[buf][p][mm][8 * cq]) = sp.p[p];
  };
  const int64_t part = static_cast<int64_t>(s.O) * s.K;
  auto load_a = [&](int t) {   // rows past O are never stored; channels past C meet zero columns
    const int ct = t / s.N, n = t - ct * s.N;
#pragma unroll
    for (int ri = 0; ri < 2; ++ri) {
      const int o = min(o0 + 64 * wv + 32 * ri + l31, s.O - 1);
      const __bf16 *pr = wf3 + static_cast<int64_t>(o) * s.K + static_cast<int64_t>(n) * s.C;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int c = min(ct * kFKC + 16 * j + 8 * h, s.C - 8);
#pragma unroll
        for (int p = 0; p < 3; ++p) acur[ri][j][p] = *reinterpret_cast<const bf16x8 *>(pr + p * part + c);
      }
    }
  };
  if (t0 < t1) {
    Cf cf = load_coef(t0);
    gather(t0, cf, X, xok);
    store_cols(0, cf, X, xok);
    load_a(t0);
    __syncthreads();
    for (int t = t0; t < t1; ++t) {
      const int buf = (t - t0) & 1;
      const int tn = min(t + 1, t1 - 1);   // the last pass re-gathers its own tile into the idle buffer
      cf = load_coef(tn);
      gather(tn, cf, X, xok);
      __builtin_amdgcn_sched_barrier(0);   // the prefetch stays ahead of the MFMAs
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bf16x8 b[2][3];
#pragma unroll
        for (int bq = 0; bq < 2; ++bq)
#pragma unroll
          for (int p = 0; p < 3; ++p) b[bq][p] = *reinterpret_cast<const bf16x8 *>(&s_cols[buf][p][32 * bq + l31][16 * j + 8 * h]);
#pragma unroll
        for (int ri = 0; ri < 2; ++ri)
#pragma unroll
          for (int bq = 0; bq < 2; ++bq) acc[ri][bq] = mfma6(acur[ri][j], b[bq], acc[ri][bq]);
      }
      __builtin_amdgcn_sched_barrier(0);
      load_a(tn);   // L2-resident weights, in flight through the column store and barrier
      store_cols(buf ^ 1, cf, X, xok);
      __syncthreads();
    }
  }
#pragma unroll
  for (int bq = 0; bq < 2; ++bq) {
    const int m = m0 + 32 * bq + l31;
    if (m >= s.M) continue;
    const int b = m / HWo, pix = m - b * HWo;
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = o0 + 64 * wv + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (o >= s.O) continue;
        float *dst = out + (static_cast<int64_t>(b) * s.O + o) * HWo + pix;
        if (atomic_out) atomicAdd(dst, acc[a][bq][r]);
        else *dst = acc[a][bq][r];
      }
  }
}
#endif  // SBOD_DCN_SPLIT_FWD

// ----------------------------------------------------------------------------- backward (data)
// Block: 64 pixels x 256 channels for ONE kernel point n (blockIdx.z).  dcols[m, n, c] =
// sum_o dout[o, m] Wb[n, o, c] on MFMA (dout staged in 32-channel chunks, Wb read straight
// from L2 with lanes along c), written as rows of the dcols buffer (128-B segments).  dx is a
// gather over those rows (k_dcn_dx_gather); the offset / mask gradients need the corner values,
// which k_dcn_bwd_weight already samples, so they are reduced there.
constexpr int kBM = 64, kBOC = 32, kBLD = kBM + 2;
#ifndef SBOD_BWD_DATA_MIN_BLOCKS
#define SBOD_BWD_DATA_MIN_BLOCKS 256
#endif
constexpr int kBwdDataMinBlocks = SBOD_BWD_DATA_MIN_BLOCKS;   // below: 32-pixel blocks

// R row halves of 32 pixels per block (R = 2: 64 pixels; R = 1: 32, for maps too small to give
// every CU a 64-pixel block)
template <int R>
__global__ __launch_bounds__(kDcnThreads, 3) void k_dcn_bwd_data(
    DcnShape s, const float *__restrict__ wb, const float *__restrict__ gout, float *__restrict__ dcols) {
  constexpr int kRM = 32 * R;                 // pixels per block
  constexpr int kLd = kDcnThreads / kRM;      // dout rows (o) per staging pass of the block
  __shared__ float s_dout[2][kBOC][kBLD];     // A operand [o][m]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, l31 = lane & 31;
  // logical order kernel point fastest: the N tiles of one pixel tile (same dout rows) run
  // back to back on one XCD
  const Tile3 tl = xcd_tile(gridDim.z, gridDim.x, gridDim.y);
  const int m0 = tl.y * kRM, cgb = tl.z * 256, n = tl.x;
  const int HWo = s.Ho * s.Wo;
  const int OT = (s.O + kBOC - 1) / kBOC;
  // Operand loads are unconditional, through wave-uniform buffer descriptors (32-bit lane offsets,
  // a scalar offset per chunk / row): dout lanes past M read a clamped pixel and rows o >= O read
  // in-range data or 0 (the descriptor's range check), both zeroed in dstage; Wb rows o >= O meet
  // a zero dout.  No branch makes the compiler wait for the prefetch before the current MFMAs.
  const auto rg = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(gout), static_cast<short>(0),
                                                    static_cast<int>(static_cast<int64_t>(s.M) * s.O * 4), 0x00020000);
  const auto rw = __builtin_amdgcn_make_buffer_rsrc(const_cast<float *>(wb), static_cast<short>(0),
                                                    static_cast<int>(static_cast<int64_t>(s.N) * s.O * s.C * 4), 0x00020000);
  constexpr int kSt = kBOC * kRM / kDcnThreads;   // staged dout elements per thread (8 or 4)
  int dvoff[kSt];   // dout element (o = oc * 32 + ol, m) at byte dvoff + oc * 32 * HWo * 4
  bool dok[kSt];
#pragma unroll
  for (int i = 0; i < kSt; ++i) {
    const int e = tid + kDcnThreads * i;
    const int ol = e / kRM, mm = e % kRM, m = min(m0 + mm, s.M - 1);
    const int b = m / HWo, pix = m - b * HWo;
    dok[i] = m0 + mm < s.M;
    dvoff[i] = ((b * s.O + ol) * HWo + pix) * 4;
  }
  float dstage[kSt];
  float bcur[2][16];   // one B buffer: the next chunk's weights load once the MFMAs have read these
  auto load_dout = [&](int oc) {
    const int so = oc * kBOC * HWo * 4;   // wave-uniform: rows o >= O read finite data or 0 (range check)
#pragma unroll
    for (int i = 0; i < kSt; ++i) {
      const bool o_ok = oc * kBOC + (tid + kDcnThreads * i) / kRM < s.O;
      const float v = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rg, dvoff[i], so, 0));
      dstage[i] = (dok[i] && o_ok) ? v : 0.f;
    }
  };
  auto store_dout = [&](int buf) {
#pragma unroll
    for (int i = 0; i < kSt; ++i) {
      const int e = tid + kDcnThreads * i;
      s_dout[buf][e / kRM][e % kRM] = dstage[i];
    }
  };
  int bvoff[2];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
    bvoff[ci] = ((16 * h) * s.C + min(cgb + 64 * wv + 32 * ci + l31, s.C - 1)) * 4;
  auto load_b = [&](int oc, float (&bb)[2][16]) {
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      // wave-uniform scalar offset; rows o >= O (their dout is zero) read the next kernel point's
      // weights or 0 past the end (the descriptor's range check)
      const int so = (n * s.O + oc * kBOC + st) * s.C * 4;
#pragma unroll
      for (int ci = 0; ci < 2; ++ci)
        bb[ci][st] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rw, bvoff[ci], so, 0));
    }
  };
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  load_dout(0);
  store_dout(0);
  load_b(0, bcur);
  __syncthreads();
  float a0[16], a1[16];
  for (int oc = 0; oc < OT; ++oc) {
    const int buf = oc & 1;
    const bool more = oc + 1 < OT;
    const int ocn = more ? oc + 1 : oc;
    load_dout(ocn);
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      a0[st] = s_dout[buf][16 * h + st][l31];
      if constexpr (R == 2) a1[st] = s_dout[buf][16 * h + st][32 + l31];
    }
    __builtin_amdgcn_sched_barrier(0);   // the prefetch stays ahead of the MFMAs
#pragma unroll
    for (int st = 0; st < 16; ++st) {
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[st], bcur[0][st], acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[st], bcur[1][st], acc[0][1], 0, 0, 0);
      if constexpr (R == 2) {
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[st], bcur[0][st], acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[st], bcur[1][st], acc[1][1], 0, 0, 0);
      }
    }
    __builtin_amdgcn_sched_barrier(0);
    load_b(ocn, bcur);   // L2-resident weights, in flight through the dout store and barrier
    if (more) store_dout(buf ^ 1);
    __syncthreads();
  }
  // epilogue: row m = 32 ri + (r&3) + 8 (r>>2) + 4 h, column c = cgb + 64 wv + 32 ci + l31
#pragma unroll
  for (int ri = 0; ri < R; ++ri)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + 32 * ri + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (m >= s.M) continue;
      float *row = dcols + (static_cast<int64_t>(m) * s.N + n) * s.C;
#pragma unroll
      for (int ci = 0; ci < 2; ++ci) {
        const int c = cgb + 64 * wv + 32 * ci + l31;
        if (c < s.C) row[c] = acc[ri][ci][r];
      }
    }
}

#ifdef SBOD_DCN_SPLIT_BF16
// The same contraction on the split-bf16 matrix cores (mfma6).  Block: 32 R pixels x 256
// channels of ONE kernel point n; K = output channels in chunks of 32.  A = dout [pixel][o]: each
// thread loads its pixel's kSt consecutive output channels (coalesced along the pixels), splits
// them and stores the three parts as one vector per part into LDS [part][pixel][o] (a 40-element
// row pitch: conflict-free 16-byte reads); B = wb3 [part][n][c][o], 16-byte loads of 8
// consecutive o straight from L2 into the MFMA registers, the next chunk's in flight through
// the current chunk's MFMAs.  The epilogue is the fp32 kernel's (dcols rows).
constexpr int kB3Pitch = 40;
template <int R>
__global__ __launch_bounds__(kDcnThreads, 2) void k_dcn_bwd_data3(
    DcnShape s, const __bf16 *__restrict__ wb3, int Op, const float *__restrict__ gout, float *__restrict__ dcols) {
  constexpr int kRM = 32 * R;                 // pixels per block
  constexpr int kSt = kBOC * kRM / kDcnThreads;   // output channels per staging thread (8 or 4)
  constexpr int kOg = kBOC / kSt;             // staging groups along o
  __shared__ __attribute__((aligned(16))) __bf16 s_a[2][3][kRM][kB3Pitch];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, l31 = lane & 31;
  const Tile3 tl = xcd_tile(gridDim.z, gridDim.x, gridDim.y);
  const int m0 = tl.y * kRM, cgb = tl.z * 256, n = tl.x;
  const int HWo = s.Ho * s.Wo;
  const int OT = (s.O + kBOC - 1) / kBOC;
  // staging role: pixel mm, output channels og * kSt .. + kSt of each chunk
  const int mm = tid % kRM, og = tid / kRM;
  static_assert(kOg * kRM == kDcnThreads, "staging covers the chunk");
  const int msc = min(m0 + mm, s.M - 1);
  const bool mok = m0 + mm < s.M;
  const int sb = msc / HWo, spix = msc - sb * HWo;
  const float *gp = gout + (static_cast<int64_t>(sb) * s.O) * HWo + spix;   // + o * HWo
  // two dout staging sets: chunk oc+2's loads are in flight while chunk oc+1's are split and stored
  // and chunk oc's MFMAs run (the split MFMAs leave too little time to cover one chunk of lead)
  float dA[kSt], dB[kSt];
  auto load_dout = [&](int oc, float (&dstage)[kSt]) {
#pragma unroll
    for (int i = 0; i < kSt; ++i) {
      const int o = oc * kBOC + og * kSt + i;
      const float v = gp[static_cast<int64_t>(min(o, s.O - 1)) * HWo];   // unconditional, clamped
      dstage[i] = (mok && o < s.O) ? v : 0.f;
    }
  };
  auto store_dout = [&](int buf, float (&dstage)[kSt]) {
    if constexpr (kSt == 8) {
      const Split8 sp = split8(dstage);
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<bf16x8 *>(&s_a[buf][p][mm][og * 8]) = sp.p[p];
    } else {
      bf16x4 v[3];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __bf16 a, b, c;
        split3(dstage[i], a, b, c);
        v[0][i] = a;
        v[1][i] = b;
        v[2][i] = c;
      }
#pragma unroll
      for (int p = 0; p < 3; ++p) *reinterpret_cast<bf16x4 *>(&s_a[buf][p][mm][og * 4]) = v[p];
    }
  };
  // B: this lane's channel rows (clamped: channels past C are never stored)
  const int64_t part = static_cast<int64_t>(s.N) * s.C * Op;
  const __bf16 *brow[2];
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
    brow[ci] = wb3 + (static_cast<int64_t>(n) * s.C + min(cgb + 64 * wv + 32 * ci + l31, s.C - 1)) * Op + 8 * h;
  bf16x8 b0[2][2][3], b1[2][2][3];   // [ci][j][part]; the next chunk's in flight a whole chunk ahead
  auto load_b = [&](int oc, bf16x8 (&bb)[2][2][3]) {
#pragma unroll
    for (int ci = 0; ci < 2; ++ci)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int p = 0; p < 3; ++p)
          bb[ci][j][p] = *reinterpret_cast<const bf16x8 *>(brow[ci] + p * part + oc * kBOC + 16 * j);
  };
  f32x16 acc[R][2];
#pragma unroll
  for (int a = 0; a < R; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  load_dout(0, dA);
  store_dout(0, dA);
  load_b(0, b0);
  load_dout(min(1, OT - 1), dA);
  __syncthreads();
  auto step = [&](int oc, bf16x8 (&bc)[2][2][3], bf16x8 (&bn)[2][2][3], float (&dcur)[kSt], float (&dnext)[kSt]) {
    const int buf = oc & 1;
    load_dout(min(oc + 2, OT - 1), dnext);
    load_b(min(oc + 1, OT - 1), bn);
    __builtin_amdgcn_sched_barrier(0);   // the prefetch stays ahead of the MFMAs
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      bf16x8 a[R][3];
#pragma unroll
      for (int ri = 0; ri < R; ++ri)
#pragma unroll
        for (int p = 0; p < 3; ++p) a[ri][p] = *reinterpret_cast<const bf16x8 *>(&s_a[buf][p][32 * ri + l31][16 * j + 8 * h]);
#pragma unroll
      for (int ri = 0; ri < R; ++ri)
#pragma unroll
        for (int ci = 0; ci < 2; ++ci) acc[ri][ci] = mfma6(a[ri], bc[ci][j], acc[ri][ci]);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (oc + 1 < OT) store_dout(buf ^ 1, dcur);
    __syncthreads();
  };
  int oc = 0;
  for (; oc + 1 < OT; oc += 2) {
    step(oc, b0, b1, dA, dB);
    step(oc + 1, b1, b0, dB, dA);
  }
  if (oc < OT) step(oc, b0, b1, dA, dB);
  // epilogue: row m = 32 ri + (r&3) + 8 (r>>2) + 4 h, column c = cgb + 64 wv + 32 ci + l31
#pragma unroll
  for (int ri = 0; ri < R; ++ri)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int m = m0 + 32 * ri + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (m >= s.M) continue;
      float *row = dcols + (static_cast<int64_t>(m) * s.N + n) * s.C;
#pragma unroll
      for (int ci = 0; ci < 2; ++ci) {
        const int c = cgb + 64 * wv + 32 * ci + l31;
        if (c < s.C) {
#ifdef SBOD_DCN_DCOLS_PLAIN
          row[c] = acc[ri][ci][r];
#else
          __builtin_nontemporal_store(acc[ri][ci][r], row + c);   // streamed: keeps dout / weights in L2
#endif
        }
      }
    }
}

#endif  // SBOD_DCN_SPLIT_BF16

// ----------------------------------------------------------------------------- backward (dx gather)
// dx[b, y, x, c] = sum over the samples (pixel m, kernel point n, corner q) whose corner q lands
// on input pixel (y, x) of  g_q(m, n) * mask(m, n) * dcols[m, n, c].  k_dcn_bwd_data writes the
// dcols rows; k_dcn_coef counted the samples per input pixel, an exclusive scan gives each pixel
// its entry range, k_dcn_dx_fill places (row, weight) entries with integer atomics on those
// counters, and k_dcn_dx_gather (one wave per input pixel) sums its rows in registers and stores
// dx once: no float atomics (the per-pixel entry order is arbitrary; fp32 sums stay within the
// tests' tolerance, as with the atomics they replace).
// Exclusive scan of the per-input-pixel sample counts into the entry cursors, in ONE launch of one
// 1024-thread block: each thread sums a contiguous segment (its loads independent, in flight
// together), the block scans the 1024 sums (wave shuffles + 16 wave totals in LDS), and each
// thread writes its segment's running offsets.  Used up to kScanOneBlock counters (8 per thread),
// where it replaces the library scan's two launches; beyond, its per-thread segments are long
// strided walks (C4 64x64: 36 us vs 2 x 4.8 us, profiles/r4_dcn_variants_b3) and hipCUB scans.
constexpr int kScanOneBlock = 8192;

__global__ __launch_bounds__(1024) void k_dcn_scan(const uint32_t *__restrict__ in, uint32_t *__restrict__ out, int n) {
  __shared__ uint32_t s_w[16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int per = (n + 1023) >> 10;
  const int b0 = min(tid * per, n), b1 = min(b0 + per, n);
  uint32_t sum = 0;
#pragma unroll 8
  for (int i = b0; i < b1; ++i) sum += in[i];
  uint32_t incl = sum;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t v = __shfl_up(incl, off, 64);
    if (lane >= off) incl += v;
  }
  if (lane == 63) s_w[wv] = incl;
  __syncthreads();
  if (wv == 0) {
    uint32_t w = lane < 16 ? s_w[lane] : 0u, wi = w;
#pragma unroll
    for (int off = 1; off < 16; off <<= 1) {
      const uint32_t v = __shfl_up(wi, off, 64);
      if (lane >= off) wi += v;
    }
    if (lane < 16) s_w[lane] = wi - w;   // exclusive: the waves before
  }
  __syncthreads();
  uint32_t run = s_w[wv] + incl - sum;
#pragma unroll 8
  for (int i = b0; i < b1; ++i) {
    const uint32_t c = in[i];
    out[i] = run;
    run += c;
  }
}

struct DxEnt {
  uint32_t row;   // m * N + n
  float w;        // g_q * mask
};

__global__ __launch_bounds__(256) void k_dcn_dx_fill(DcnShape s, const Coef *__restrict__ coef,
                                                     uint32_t *__restrict__ cur, DxEnt *__restrict__ ent,
                                                     float *__restrict__ z0, int64_t n0, float *__restrict__ z1,
                                                     int64_t n1, float *__restrict__ z2, int64_t n2) {
  // the zero-initialised gradients the later kernels accumulate into (offset, mask, weight)
  zero_fill(z0, n0);
  zero_fill(z1, n1);
  zero_fill(z2, n2);
  const int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (t >= static_cast<int64_t>(s.M) * s.N) return;
  const int m = static_cast<int>(t / s.N);
  const int64_t ib = static_cast<int64_t>(m / (s.Ho * s.Wo)) * s.H * s.W;
  const Coef cf = coef[t];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (cf.idx[q] < 0) continue;
    // cur starts at each pixel's first entry (exclusive scan of the counts) and ends at its last + 1
    const uint32_t k = atomicAdd(cur + ib + cf.idx[q], 1u);
    ent[k] = DxEnt{static_cast<uint32_t>(t), cf.g[q] * cf.mval};
  }
}

// One wave per input pixel, kGxPix pixels per block; lanes hold 4 consecutive channels (C % 4 == 0)
// or 1.  Each 64*VEC-channel pass lands in LDS and leaves as rows of dx [B][C][H][W] (kGxPix
// consecutive pixels per channel): the channels-last result is never written to HBM and
// transposed back.  After k_dcn_dx_fill, cur[tp] is the end of pixel tp's entries and cur[tp - 1]
// its start.
#ifndef SBOD_GX_PIX   // A/B knobs: pixels (waves) per block, dcols rows in flight per wave
#define SBOD_GX_PIX 8   // 8 (512 threads): 64² 211-213 vs 218-219 us, 8² 8.8 vs 10.6 us (r4_gx_ab_c1.jsonl)
#endif
#ifndef SBOD_GX_ROWS
#define SBOD_GX_ROWS 8
#endif
constexpr int kGxPix = SBOD_GX_PIX;
#ifndef SBOD_WG_TARGET   // A/B knob: k_dcn_bwd_weight's target workgroup count (pixel slices)
#define SBOD_WG_TARGET 512
#endif
constexpr int kGxRows = SBOD_GX_ROWS;

template <int VEC>
__global__ __launch_bounds__(64 * kGxPix) void k_dcn_dx_gather(int C, int HW, int ntarget,
                                                              const uint32_t *__restrict__ cur,
                                                              const DxEnt *__restrict__ ent,
                                                              const float *__restrict__ dcols, float *__restrict__ gx) {
  // row stride 64 * VEC + 8 floats: the float4 row writes stay 16-B aligned and the column reads
  // (8 pixels x 8 channels per wave) hit 64 distinct banks
  constexpr int kLd = 64 * VEC + 8;
  __shared__ __attribute__((aligned(16))) float s_t[kGxPix][kLd];
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // neighbouring input pixels (overlapping dcols rows) on one XCD
  const int tp0 = xcd_logical(blockIdx.x, gridDim.x) * kGxPix;
  const int tp = tp0 + wv;
  const bool live = tp < ntarget;
  uint32_t e0 = 0, e1 = 0;
  if (live) {
    e0 = __builtin_amdgcn_readfirstlane(tp > 0 ? cur[tp - 1] : 0u);
    e1 = __builtin_amdgcn_readfirstlane(cur[tp]);
  }
  for (int cb = 0; cb < C; cb += 64 * VEC) {   // uniform trip count: every lane loads entries
    const int c0 = min(cb + VEC * lane, C - VEC);   // lanes past C read a valid column, store nothing
    float acc[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[v] = 0.f;
    // entries 64 at a time, one per lane (one coalesced load), broadcast by readlane; eight dcols
    // rows in flight; rows summed in entry order
    for (uint32_t eb = e0; eb < e1; eb += 64) {
      const int ne = static_cast<int>(min(e1 - eb, 64u));
      const DxEnt mine = lane < ne ? ent[eb + lane] : DxEnt{0u, 0.f};
      int k = 0;
      for (; k + kGxRows <= ne; k += kGxRows) {
        float x[kGxRows][VEC], w[kGxRows];
#pragma unroll
        for (int u = 0; u < kGxRows; ++u) {
          const uint32_t row = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(mine.row), k + u));
          w[u] = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, mine.w), k + u));
          load_vec<VEC>(dcols + static_cast<int64_t>(row) * C + c0, true, x[u]);
        }
#pragma unroll
        for (int u = 0; u < kGxRows; ++u)
#pragma unroll
          for (int v = 0; v < VEC; ++v) acc[v] += w[u] * x[u][v];
      }
      for (; k < ne; ++k) {
        const uint32_t row = static_cast<uint32_t>(__builtin_amdgcn_readlane(static_cast<int>(mine.row), k));
        const float w = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, mine.w), k));
        float x[VEC];
        load_vec<VEC>(dcols + static_cast<int64_t>(row) * C + c0, true, x);
#pragma unroll
        for (int v = 0; v < VEC; ++v) acc[v] += w * x[v];
      }
    }
    if constexpr (VEC == 4)
      *reinterpret_cast<float4 *>(&s_t[wv][4 * lane]) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    else
      for (int v = 0; v < VEC; ++v) s_t[wv][VEC * lane + v] = acc[v];
    __syncthreads();
    const int nc = min(64 * VEC, C - cb);
    for (int e = threadIdx.x; e < kGxPix * 64 * VEC; e += 64 * kGxPix) {
      const int px = e % kGxPix, cl = e / kGxPix, p = tp0 + px;
      if (cl < nc && p < ntarget) {
        const int b = p / HW, pix = p - b * HW;
        gx[(static_cast<int64_t>(b) * C + cb + cl) * HW + pix] = s_t[px][cl];
      }
    }
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------- backward (weight)
// Block: one kernel point n x 64 channels (blockIdx.x), a slice of pixels (blockIdx.y), 256
// output channels (blockIdx.z): dWp[o, n, c] += sum_m dout[o, m] cols[(n, c), m], transposed to
// conv.weight's [O][C][k][k] after (accumulating in that layout directly puts the 32 lanes of an
// atomic on 32 lines, k² floats apart: the C4 8x8 backward took 0.31 ms instead of 0.17).  The mirror of
// the forward kernel: dout rows go straight from HBM into the MFMA A registers (float4 when a
// 32-pixel chunk never straddles two images), the columns are re-sampled channels-last into
// double-buffered LDS, and the next chunk's gathers are in flight during the current MFMAs.
// The same corner samples give the offset / mask gradients (Deformable_convolution.py:59-91 by
// autograd): with dcols from k_dcn_bwd_data, each pixel's partial sums over this block's 64
// channels, pm = sum dcol * raw and d/dp = sum dcol * mask * (corner-difference terms), are
// reduced over the 8 lanes holding the pixel (DPP) and added to d_offset / d_mask (C / 64
// partials per (pixel, kernel point); output-channel block 0 only).
constexpr int kWC = 64, kWMs = 32, kWLD = kWC + 2;

template <int VEC, bool AVEC, bool DOFS>   // (the scalar-channel form needs more registers: one block per CU)
#ifndef SBOD_DCN_WGRAD_WAVES
#define SBOD_DCN_WGRAD_WAVES 2
#endif
__global__ __launch_bounds__(kDcnThreads, VEC == 4 ? SBOD_DCN_WGRAD_WAVES : 1) void k_dcn_bwd_weight(
    DcnShape s, const float *__restrict__ xt, const Coef *__restrict__ coef,
    const float *__restrict__ gout, float *__restrict__ gwp, int m_slice,
    const float *__restrict__ dcols, float *__restrict__ goff, float *__restrict__ gmlog) {
  __shared__ float s_cols[2][kWMs][kWLD];      // B operand [m][c]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, l31 = lane & 31;
  const Tile3 tl = xcd_tile(gridDim.x, gridDim.y, gridDim.z);   // one pixel slice's tiles share an L2
  // kernel point fastest: the N blocks of one channel block and pixel slice (the same corner
  // lines, dout rows) run side by side on one XCD
  const int cb = tl.x / s.N, n = tl.x - cb * s.N, c0 = cb * kWC;
  const int ms0 = tl.y * m_slice, o0 = tl.z * 256;
  const int mend = min(ms0 + m_slice, s.M);
  const int HWo = s.Ho * s.Wo, HW = s.H * s.W;
  const int smm = tid >> 3, scg = (tid & 7) * 8;
  const bool oblk0 = tl.z == 0;   // offset / mask gradients from output-channel block 0 only
  const bool dow = gwp != nullptr;
  // Every operand load is unconditional (pixels past the slice read a clamped pixel and their
  // columns are stored as zeros; corners outside the map and channels past C are zeroed at the
  // store), so the loop is straight-line code: the waits before the MFMAs cover the dout rows
  // they read, not the next chunk's gathers in flight.
  struct CfW {
    int idx[4];
    float g[4], m, tlx, rbx, tly, rby;
    int inr;
  };
  // Address arithmetic.  AVEC (every 32-pixel chunk whole and inside one image): the chunk's
  // image and first pixel are wave-uniform (scalar unit), the per-lane parts (channel offsets,
  // this lane's pixel row / output channel rows) are loop-invariant 32-bit offsets, so a chunk
  // costs one 64-bit add per load instead of divisions and 64-bit multiply-adds per lane.
  int cofs[8 / VEC];   // this lane's channel offsets, clamped into the row
#pragma unroll
  for (int v = 0; v < 8; v += VEC) cofs[v / VEC] = min(c0 + scg + v, s.C - VEC);
  const int lane_cf = smm * s.N;                       // coef rows of this lane's pixel
  const int lane_dc = smm * s.N * s.C;                 // dcols rows of this lane's pixel
  int lane_o[2];                                       // dout rows (o * HWo) of this lane
#pragma unroll
  for (int ri = 0; ri < 2; ++ri) lane_o[ri] = min(o0 + 64 * wv + 32 * ri + l31, s.O - 1) * HWo;
  auto load_cf = [&](int m0) {
    const Coef *cp = AVEC ? coef + (static_cast<int64_t>(m0) * s.N + n) + lane_cf
                          : coef + static_cast<int64_t>(min(m0 + smm, mend - 1)) * s.N + n;
    const float *c = reinterpret_cast<const float *>(cp);
    float2 w[7];   // a Coef is 8-byte aligned (56 bytes)
#pragma unroll
    for (int j = 0; j < 7; ++j) w[j] = reinterpret_cast<const float2 *>(c)[j];
    return CfW{{__builtin_bit_cast(int, w[0].x), __builtin_bit_cast(int, w[0].y), __builtin_bit_cast(int, w[1].x),
                __builtin_bit_cast(int, w[1].y)},
               {w[2].x, w[2].y, w[3].x, w[3].y}, w[4].x, w[4].y, w[5].x, w[5].y, w[6].x, __builtin_bit_cast(int, w[6].y)};
  };
  float X[4][8], D[8];
  bool xok[4][8 / VEC];
  float acur[2][16], anext[2][16];
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  auto gather = [&](int m0, const CfW &cf) {
    const float *xb;
    if (AVEC) {
      xb = xt + static_cast<int64_t>(m0 / HWo) * HW * s.C;   // uniform
    } else {
      const int m = min(m0 + smm, mend - 1);
      xb = xt + static_cast<int64_t>(m / HWo) * HW * s.C;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // corner pixel * C: both factors < 2^24 (per-image sizes are validated below 2^31)
      const float *p = xb + __umul24(static_cast<uint32_t>(max(cf.idx[q], 0)), static_cast<uint32_t>(s.C));
#pragma unroll
      for (int v = 0; v < 8; v += VEC) {
        xok[q][v / VEC] = cf.idx[q] >= 0 && c0 + scg + v < s.C;
        load_vec<VEC>(p + cofs[v / VEC], true, &X[q][v]);
      }
    }
    if constexpr (DOFS) {
      const float *dr = AVEC ? dcols + (static_cast<int64_t>(m0) * s.N + n) * s.C + lane_dc
                             : dcols + (static_cast<int64_t>(min(m0 + smm, mend - 1)) * s.N + n) * s.C;
#pragma unroll
      for (int v = 0; v < 8; v += VEC) load_vec<VEC>(dr + cofs[v / VEC], true, &D[v]);
    }
  };
  // live: this chunk's offset / mask partials are added (false for the prefetch past the last).
  // The column value and the offset / mask partials use fused multiply-adds (the weight and
  // offset / mask gradients are checked to fp32 tolerance, not bit-exactly):
  //   raw = g0 X0 + g1 X1 + g2 X2 + g3 X3,
  //   d/dx = (1 + tly)(X3 - X0) + (1 - rby)(X1 - X2),  d/dy = (1 + tlx)(X2 - X0) + (1 - rbx)(X1 - X3)
  // (Deformable_convolution.py:59-91 by autograd, corners lt, rb, lb, rt).
  auto store_cols = [&](int buf, const CfW &cf, int m0, bool live) {
    const bool ok = AVEC || m0 + smm < mend;
    const float cm = cf.m;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int v = 0; v < 8; ++v) X[q][v] = (ok && xok[q][v / VEC]) ? X[q][v] : 0.f;
    float pm = 0.f, ppx = 0.f, ppy = 0.f;
    const float ay = 1.f + cf.tly, by = 1.f - cf.rby, ax = 1.f + cf.tlx, bx = 1.f - cf.rbx;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const float raw = __builtin_fmaf(cf.g[3], X[3][v], __builtin_fmaf(cf.g[2], X[2][v],
                                       __builtin_fmaf(cf.g[1], X[1][v], cf.g[0] * X[0][v])));
      s_cols[buf][smm][scg + v] = raw * cm;
      if constexpr (DOFS) {
        const float d = c0 + scg + v < s.C ? D[v] : 0.f;
        pm = __builtin_fmaf(d, raw, pm);
        ppx = __builtin_fmaf(d, __builtin_fmaf(ay, X[3][v] - X[0][v], by * (X[1][v] - X[2][v])), ppx);
        ppy = __builtin_fmaf(d, __builtin_fmaf(ax, X[2][v] - X[0][v], bx * (X[1][v] - X[3][v])), ppy);
      }
    }
    if constexpr (DOFS) {   // the 8 lanes of this pixel are lanes 8k..8k+7: quad swaps + half-row mirror
      if (live && oblk0) {
        pm += dpp_f32_or0<0xB1, 0xf>(pm);
        ppx += dpp_f32_or0<0xB1, 0xf>(ppx);
        ppy += dpp_f32_or0<0xB1, 0xf>(ppy);
        pm += dpp_f32_or0<0x4E, 0xf>(pm);
        ppx += dpp_f32_or0<0x4E, 0xf>(ppx);
        ppy += dpp_f32_or0<0x4E, 0xf>(ppy);
        pm += dpp_f32_or0<0x141, 0xf>(pm);
        ppx += dpp_f32_or0<0x141, 0xf>(ppx);
        ppy += dpp_f32_or0<0x141, 0xf>(ppy);
        if ((tid & 7) == 0 && ok) {
          const int m = m0 + smm, b = m / HWo, pix = m - b * HWo;
          if (goff) {
            atomicAdd(goff + (static_cast<int64_t>(b) * 2 * s.N + n) * HWo + pix, (cf.inr & 1) ? ppx * cm : 0.f);
            atomicAdd(goff + (static_cast<int64_t>(b) * 2 * s.N + s.N + n) * HWo + pix, (cf.inr & 2) ? ppy * cm : 0.f);
          }
          if (gmlog) atomicAdd(gmlog + (static_cast<int64_t>(b) * s.N + n) * HWo + pix, pm * cm * (1.f - cm));
        }
      }
    }
  };
  auto load_a = [&](int m0, float (&a)[2][16]) {   // dout rows; pixels past the slice meet zero columns
    const int mb = m0 + 16 * h;
    if (AVEC) {   // 32-pixel chunks inside one image, slices of whole chunks: mb + 15 < mend
      const int b = m0 / HWo;   // uniform
      const float *pb = gout + static_cast<int64_t>(b) * s.O * HWo + (mb - b * HWo);
#pragma unroll
      for (int ri = 0; ri < 2; ++ri)
#pragma unroll
        for (int v = 0; v < 16; v += 4) load_vec<4>(pb + lane_o[ri] + v, true, &a[ri][v]);
    } else {
#pragma unroll
      for (int ri = 0; ri < 2; ++ri) {
        const int o = min(o0 + 64 * wv + 32 * ri + l31, s.O - 1);
#pragma unroll
        for (int v = 0; v < 16; ++v) {
          const int m = min(mb + v, mend - 1);
          const int b = m / HWo, pix = m - b * HWo;
          a[ri][v] = gout[(static_cast<int64_t>(b) * s.O + o) * HWo + pix];
        }
      }
    }
  };

  if (ms0 < mend) {
    const int nch = (mend - ms0 + kWMs - 1) / kWMs;
    CfW cf = load_cf(ms0);
    gather(ms0, cf);
    store_cols(0, cf, ms0, true);
    load_a(ms0, acur);
    CfW cn = load_cf(ms0 + min(1, nch - 1) * kWMs);   // coefficients one chunk ahead of the gathers
    __syncthreads();
    for (int i = 0; i < nch; ++i) {
      const int buf = i & 1;
      const int mn = ms0 + min(i + 1, nch - 1) * kWMs;   // the last pass re-gathers its own chunk
      cf = cn;
      gather(mn, cf);
#ifndef SBOD_DCN_WGRAD_SINGLE_A
      load_a(mn, anext);
#endif
      cn = load_cf(ms0 + min(i + 2, nch - 1) * kWMs);
      __builtin_amdgcn_sched_barrier(0);   // the prefetch stays ahead of the MFMAs
#pragma unroll
      for (int st = 0; st < 16; ++st) {
        const float b0 = s_cols[buf][16 * h + st][l31];
        const float b1 = s_cols[buf][16 * h + st][32 + l31];
        acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(acur[0][st], b0, acc[0][0], 0, 0, 0);
        acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(acur[0][st], b1, acc[0][1], 0, 0, 0);
        acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(acur[1][st], b0, acc[1][0], 0, 0, 0);
        acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(acur[1][st], b1, acc[1][1], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
#ifdef SBOD_DCN_WGRAD_SINGLE_A
      load_a(mn, acur);   // (A/B variant) the next chunk's dout rows, once these MFMAs read theirs
      store_cols(buf ^ 1, cf, mn, i + 1 < nch);
#else
      store_cols(buf ^ 1, cf, mn, i + 1 < nch);
#pragma unroll
      for (int ri = 0; ri < 2; ++ri)
#pragma unroll
        for (int v = 0; v < 16; ++v) acur[ri][v] = anext[ri][v];
#endif
      __syncthreads();
    }
  }
  if (!dow) return;   // (offset / mask gradients only: the MFMA result is not wanted)
  // this pixel slice's partial dWp: plain stores into its own [O][N][C] plane (k_wgrad_fold sums
  // the planes in slice order: deterministic, no far atomics)
  float *gws = gwp + static_cast<int64_t>(tl.y) * s.O * s.K;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bq = 0; bq < 2; ++bq) {
      const int c = c0 + 32 * bq + l31;
      if (c >= s.C) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = o0 + 64 * wv + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (o < s.O) gws[(static_cast<int64_t>(o) * s.N + n) * s.C + c] = acc[a][bq][r];
      }
    }
}

#ifdef SBOD_DCN_SPLIT_FWD
// The weight-gradient contraction on the split-bf16 matrix cores (mfma6), for the common case
// (C % 4 == 0, 32-pixel chunks inside one image): the sampler splits each column value once into
// three bf16 rows of LDS [buf][part][channel][pixel] (pixels, the MFMA's K, contiguous; a 40-element
// pitch), and each wave splits its own dout rows (8 consecutive pixels per 16-byte pair of loads)
// right before the MFMAs.  The offset / mask gradients are the fp32 kernel's, from the same samples.
template <bool DOFS>
__global__ __launch_bounds__(kDcnThreads, 2) void k_dcn_bwd_weight3(
    DcnShape s, const float *__restrict__ xt, const Coef *__restrict__ coef,
    const float *__restrict__ gout, float *__restrict__ gwp, int m_slice,
    const float *__restrict__ dcols, float *__restrict__ goff, float *__restrict__ gmlog) {
  constexpr int VEC = 4;
  constexpr bool AVEC = true;
  __shared__ __attribute__((aligned(16))) __bf16 s_cb[2][3][kWC][kF3Pitch];   // B operand [part][c][m]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, h = lane >> 5, l31 = lane & 31;
  const Tile3 tl = xcd_tile(gridDim.x, gridDim.y, gridDim.z);   // one pixel slice's tiles share an L2
  // kernel point fastest: the N blocks of one channel block and pixel slice (the same corner
  // lines, dout rows) run side by side on one XCD
  const int cb = tl.x / s.N, n = tl.x - cb * s.N, c0 = cb * kWC;
  const int ms0 = tl.y * m_slice, o0 = tl.z * 256;
  const int mend = min(ms0 + m_slice, s.M);
  const int HWo = s.Ho * s.Wo, HW = s.H * s.W;
  const int smm = tid >> 3, scg = (tid & 7) * 8;
  const bool oblk0 = tl.z == 0;   // offset / mask gradients from output-channel block 0 only
  const bool dow = gwp != nullptr;
  // Every operand load is unconditional (pixels past the slice read a clamped pixel and their
  // columns are stored as zeros; corners outside the map and channels past C are zeroed at the
  // store), so the loop is straight-line code: the waits before the MFMAs cover the dout rows
  // they read, not the next chunk's gathers in flight.
  struct CfW {
    int idx[4];
    float g[4], m, tlx, rbx, tly, rby;
    int inr;
  };
  // Address arithmetic.  AVEC (every 32-pixel chunk whole and inside one image): the chunk's
  // image and first pixel are wave-uniform (scalar unit), the per-lane parts (channel offsets,
  // this lane's pixel row / output channel rows) are loop-invariant 32-bit offsets, so a chunk
  // costs one 64-bit add per load instead of divisions and 64-bit multiply-adds per lane.
  int cofs[8 / VEC];   // this lane's channel offsets, clamped into the row
#pragma unroll
  for (int v = 0; v < 8; v += VEC) cofs[v / VEC] = min(c0 + scg + v, s.C - VEC);
  const int lane_cf = smm * s.N;                       // coef rows of this lane's pixel
  const int lane_dc = smm * s.N * s.C;                 // dcols rows of this lane's pixel
  int lane_o[2];                                       // dout rows (o * HWo) of this lane
#pragma unroll
  for (int ri = 0; ri < 2; ++ri) lane_o[ri] = min(o0 + 64 * wv + 32 * ri + l31, s.O - 1) * HWo;
  auto load_cf = [&](int m0) {
    const Coef *cp = AVEC ? coef + (static_cast<int64_t>(m0) * s.N + n) + lane_cf
                          : coef + static_cast<int64_t>(min(m0 + smm, mend - 1)) * s.N + n;
    const float *c = reinterpret_cast<const float *>(cp);
    float2 w[7];   // a Coef is 8-byte aligned (56 bytes)
#pragma unroll
    for (int j = 0; j < 7; ++j) w[j] = reinterpret_cast<const float2 *>(c)[j];
    return CfW{{__builtin_bit_cast(int, w[0].x), __builtin_bit_cast(int, w[0].y), __builtin_bit_cast(int, w[1].x),
                __builtin_bit_cast(int, w[1].y)},
               {w[2].x, w[2].y, w[3].x, w[3].y}, w[4].x, w[4].y, w[5].x, w[5].y, w[6].x, __builtin_bit_cast(int, w[6].y)};
  };
  float X[4][8], D[8];
  bool xok[4][8 / VEC];
  float acur[2][2][8], anext[2][2][8];
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;

  auto gather = [&](int m0, const CfW &cf) {
    const float *xb;
    if (AVEC) {
      xb = xt + static_cast<int64_t>(m0 / HWo) * HW * s.C;   // uniform
    } else {
      const int m = min(m0 + smm, mend - 1);
      xb = xt + static_cast<int64_t>(m / HWo) * HW * s.C;
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      // corner pixel * C: both factors < 2^24 (per-image sizes are validated below 2^31)
      const float *p = xb + __umul24(static_cast<uint32_t>(max(cf.idx[q], 0)), static_cast<uint32_t>(s.C));
#pragma unroll
      for (int v = 0; v < 8; v += VEC) {
        xok[q][v / VEC] = cf.idx[q] >= 0 && c0 + scg + v < s.C;
        load_vec<VEC>(p + cofs[v / VEC], true, &X[q][v]);
      }
    }
    if constexpr (DOFS) {
      const float *dr = AVEC ? dcols + (static_cast<int64_t>(m0) * s.N + n) * s.C + lane_dc
                             : dcols + (static_cast<int64_t>(min(m0 + smm, mend - 1)) * s.N + n) * s.C;
#pragma unroll
      for (int v = 0; v < 8; v += VEC) load_vec<VEC>(dr + cofs[v / VEC], true, &D[v]);
    }
  };
  // live: this chunk's offset / mask partials are added (false for the prefetch past the last).
  // The column value and the offset / mask partials use fused multiply-adds (the weight and
  // offset / mask gradients are checked to fp32 tolerance, not bit-exactly):
  //   raw = g0 X0 + g1 X1 + g2 X2 + g3 X3,
  //   d/dx = (1 + tly)(X3 - X0) + (1 - rby)(X1 - X2),  d/dy = (1 + tlx)(X2 - X0) + (1 - rbx)(X1 - X3)
  // (Deformable_convolution.py:59-91 by autograd, corners lt, rb, lb, rt).
  auto store_cols = [&](int buf, const CfW &cf, int m0, bool live) {
    const bool ok = AVEC || m0 + smm < mend;
    const float cm = cf.m;
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int v = 0; v < 8; ++v) X[q][v] = (ok && xok[q][v / VEC]) ? X[q][v] : 0.f;
    float pm = 0.f, ppx = 0.f, ppy = 0.f;
    const float ay = 1.f + cf.tly, by = 1.f - cf.rby, ax = 1.f + cf.tlx, bx = 1.f - cf.rbx;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const float raw = __builtin_fmaf(cf.g[3], X[3][v], __builtin_fmaf(cf.g[2], X[2][v],
                                       __builtin_fmaf(cf.g[1], X[1][v], cf.g[0] * X[0][v])));
      __bf16 hp, mp, lp;
      split3(raw * cm, hp, mp, lp);
      s_cb[buf][0][scg + v][smm] = hp;
      s_cb[buf][1][scg + v][smm] = mp;
      s_cb[buf][2][scg + v][smm] = lp;
      if constexpr (DOFS) {
        const float d = c0 + scg + v < s.C ? D[v] : 0.f;
        pm = __builtin_fmaf(d, raw, pm);
        ppx = __builtin_fmaf(d, __builtin_fmaf(ay, X[3][v] - X[0][v], by * (X[1][v] - X[2][v])), ppx);
        ppy = __builtin_fmaf(d, __builtin_fmaf(ax, X[2][v] - X[0][v], bx * (X[1][v] - X[3][v])), ppy);
      }
    }
    if constexpr (DOFS) {   // the 8 lanes of this pixel are lanes 8k..8k+7: quad swaps + half-row mirror
      if (live && oblk0) {
        pm += dpp_f32_or0<0xB1, 0xf>(pm);
        ppx += dpp_f32_or0<0xB1, 0xf>(ppx);
        ppy += dpp_f32_or0<0xB1, 0xf>(ppy);
        pm += dpp_f32_or0<0x4E, 0xf>(pm);
        ppx += dpp_f32_or0<0x4E, 0xf>(ppx);
        ppy += dpp_f32_or0<0x4E, 0xf>(ppy);
        pm += dpp_f32_or0<0x141, 0xf>(pm);
        ppx += dpp_f32_or0<0x141, 0xf>(ppx);
        ppy += dpp_f32_or0<0x141, 0xf>(ppy);
        if ((tid & 7) == 0 && ok) {
          const int m = m0 + smm, b = m / HWo, pix = m - b * HWo;
          if (goff) {
            atomicAdd(goff + (static_cast<int64_t>(b) * 2 * s.N + n) * HWo + pix, (cf.inr & 1) ? ppx * cm : 0.f);
            atomicAdd(goff + (static_cast<int64_t>(b) * 2 * s.N + s.N + n) * HWo + pix, (cf.inr & 2) ? ppy * cm : 0.f);
          }
          if (gmlog) atomicAdd(gmlog + (static_cast<int64_t>(b) * s.N + n) * HWo + pix, pm * cm * (1.f - cm));
        }
      }
    }
  };
  auto load_a = [&](int m0, float (&a)[2][2][8]) {   // dout rows: pixels m0 + 16 j + 8 h + 0..7
    const int b = m0 / HWo;   // uniform (32-pixel chunks inside one image)
    const float *pb = gout + static_cast<int64_t>(b) * s.O * HWo + (m0 - b * HWo) + 8 * h;
#pragma unroll
    for (int ri = 0; ri < 2; ++ri)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int v = 0; v < 8; v += 4) load_vec<4>(pb + lane_o[ri] + 16 * j + v, true, &a[ri][j][v]);
  };

  if (ms0 < mend) {
    const int nch = (mend - ms0 + kWMs - 1) / kWMs;
    CfW cf = load_cf(ms0);
    gather(ms0, cf);
    store_cols(0, cf, ms0, true);
    load_a(ms0, acur);
    CfW cn = load_cf(ms0 + min(1, nch - 1) * kWMs);   // coefficients one chunk ahead of the gathers
    __syncthreads();
    for (int i = 0; i < nch; ++i) {
      const int buf = i & 1;
      const int mn = ms0 + min(i + 1, nch - 1) * kWMs;   // the last pass re-gathers its own chunk
      cf = cn;
      gather(mn, cf);
      load_a(mn, anext);
      cn = load_cf(ms0 + min(i + 2, nch - 1) * kWMs);
      __builtin_amdgcn_sched_barrier(0);   // the prefetch stays ahead of the MFMAs
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        bf16x8 bb[2][3];
#pragma unroll
        for (int bq = 0; bq < 2; ++bq)
#pragma unroll
          for (int p = 0; p < 3; ++p) bb[bq][p] = *reinterpret_cast<const bf16x8 *>(&s_cb[buf][p][32 * bq + l31][16 * j + 8 * h]);
#pragma unroll
        for (int ri = 0; ri < 2; ++ri) {
          const Split8 sa = split8(acur[ri][j]);
#pragma unroll
          for (int bq = 0; bq < 2; ++bq) acc[ri][bq] = mfma6(sa.p, bb[bq], acc[ri][bq]);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      store_cols(buf ^ 1, cf, mn, i + 1 < nch);
#pragma unroll
      for (int ri = 0; ri < 2; ++ri)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int v = 0; v < 8; ++v) acur[ri][j][v] = anext[ri][j][v];
      __syncthreads();
    }
  }
  if (!dow) return;   // (offset / mask gradients only: the MFMA result is not wanted)
  // this pixel slice's partial dWp: plain stores into its own [O][N][C] plane (k_wgrad_fold sums
  // the planes in slice order: deterministic, no far atomics)
  float *gws = gwp + static_cast<int64_t>(tl.y) * s.O * s.K;
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bq = 0; bq < 2; ++bq) {
      const int c = c0 + 32 * bq + l31;
      if (c >= s.C) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = o0 + 64 * wv + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * h;
        if (o < s.O) gws[(static_cast<int64_t>(o) * s.N + n) * s.C + c] = acc[a][bq][r];
      }
    }
}

#endif  // SBOD_DCN_SPLIT_FWD (the split weight gradient)

// A shape whose sizes are non-positive, out of range or overflow 32-bit indexing comes back with
// every field 0 (shape_ok() false): no division by a zero stride, no signed overflow in the
// products, and the size queries return 0 for it.
DcnShape make_shape(int B, int C, int H, int W, int O, int k, int stride, int pad) {
  DcnShape s{};
  if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || O <= 0 || k <= 0 || k > 7 || stride <= 0 || pad < 0 ||
      H > (1 << 30) || W > (1 << 30) || pad > (1 << 20))
    return s;
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;   // p_conv: 3x3, padding 1
  const int64_t M = static_cast<int64_t>(B) * Ho * Wo, K = static_cast<int64_t>(C) * k * k;
  if (M * k * k >= (1ll << 31) || K * O >= (1ll << 31) || static_cast<int64_t>(C) * H * W >= (1ll << 31) ||
      static_cast<int64_t>(B) * C * H * W >= (1ll << 40))
    return s;
  s.B = B; s.C = C; s.H = H; s.W = W; s.O = O; s.k = k; s.N = k * k;
  s.stride = stride; s.pad = pad;
  s.Ho = static_cast<int>(Ho);
  s.Wo = static_cast<int>(Wo);
  s.Hp = H + 2 * pad;
  s.Wp = W + 2 * pad;
  s.M = static_cast<int>(M);
  s.K = static_cast<int>(K);
  return s;
}

inline bool shape_ok(const DcnShape &s) { return s.B > 0; }

// Training state (sbod_dcn_state_bytes): what the forward derives and the backward re-uses — the
// per-(pixel, kernel point) coefficients, channels-last x, both weight layouts and the per-input-
// pixel sample counts.  The forward-only workspace is its prefix (coef, xt, wf).
struct DcnState {
  Coef *coef;
  float *xt, *wf;
#ifdef SBOD_DCN_SPLIT_FWD
  __bf16 *wf3;        // [3][O][N*C] split parts of Wf (the split-bf16 forward)
#endif
  uint32_t *tcount;   // training: [B*H*W + 1] corner samples per input pixel
#ifndef SBOD_DCN_SPLIT_BF16
  float *wb;          // training: Wb [N][O][C] (A/B build: the fp32-MFMA backward-data kernel)
#else
  __bf16 *wb3;        // training: [3][N][C][Op] split parts of the weights, o contiguous
#endif
};

// Backward scratch (sbod_dcn_scratch_bytes): dcols rows [M][N][C], the weight-gradient
// accumulator dWp [O][N][C], the per-input-pixel entry cursors and entries of the dx gather.
struct DcnScratch {
  float *dcols, *gwp;
  uint32_t *cur;
  DxEnt *ent;
  void *scan_tmp;      // hipCUB scan storage (more than kScanOneBlock counters)
  size_t scan_bytes;
};

// The weight gradient's pixel slices: one round of resident blocks (256 CUs x 2) over the
// (channel block x kernel point) x output-channel-block tiles (a partial second round would double
// the time), each slice a whole number of 32-pixel chunks.  The workspace holds one dWp plane per
// slice (carve_scratch sizes it with the weight gradient wanted, the largest count of tiles).
struct WgSplit {
  int gx, gz, slices, m_slice;
};
WgSplit wgrad_split(const DcnShape &s, bool grad_weight) {
  WgSplit w;
  w.gx = s.N * ((s.C + kWC - 1) / kWC);
  w.gz = grad_weight ? (s.O + 255) / 256 : 1;
  int slices = std::max(1, SBOD_WG_TARGET / (w.gx * w.gz));
  slices = std::max(1, std::min(slices, (s.M + kWMs - 1) / kWMs));
  int m_slice = (s.M + slices - 1) / slices;
  w.m_slice = (m_slice + kWMs - 1) / kWMs * kWMs;
  w.slices = (s.M + w.m_slice - 1) / w.m_slice;
  return w;
}

size_t dcn_scan_bytes(int64_t n) {
  if (n <= kScanOneBlock) return 0;
  size_t b = 0;
  // size query only; a failed query makes the workspace requirement unsatisfiable (loud)
  if (hipcub::DeviceScan::ExclusiveSum(nullptr, b, static_cast<uint32_t *>(nullptr), static_cast<uint32_t *>(nullptr),
                                       static_cast<int>(n)) != hipSuccess)
    return SIZE_MAX / 4;
  return b;
}

size_t carve_state(const DcnShape &s, void *base, DcnState *w, bool train) {
  char *p = static_cast<char *>(base);
  size_t off = 0;
  auto take = [&](size_t bytes) { char *r = p ? p + off : nullptr; off += align_up(bytes); return r; };
  const size_t wbytes = static_cast<size_t>(s.O) * s.K * 4;
  const size_t npix = static_cast<size_t>(s.B) * s.H * s.W;
  DcnState t{};
  t.coef = reinterpret_cast<Coef *>(take(static_cast<size_t>(s.M) * s.N * sizeof(Coef)));
  t.xt = reinterpret_cast<float *>(take(npix * s.C * 4));
  t.wf = reinterpret_cast<float *>(take(wbytes));
#ifdef SBOD_DCN_SPLIT_FWD
  t.wf3 = reinterpret_cast<__bf16 *>(take(static_cast<size_t>(s.O) * s.K * 6));
#endif
  if (train) {
    t.tcount = reinterpret_cast<uint32_t *>(take((npix + 1) * 4));
#ifndef SBOD_DCN_SPLIT_BF16
    t.wb = reinterpret_cast<float *>(take(wbytes));
#else
    t.wb3 = reinterpret_cast<__bf16 *>(take(static_cast<size_t>(3) * s.N * s.C * dcn_opad(s.O) * 2));
#endif
  }
  if (w) *w = t;
  return off;
}

size_t carve_scratch(const DcnShape &s, void *base, DcnScratch *w) {
  char *p = static_cast<char *>(base);
  size_t off = 0;
  auto take = [&](size_t bytes) { char *r = p ? p + off : nullptr; off += align_up(bytes); return r; };
  const size_t rows = static_cast<size_t>(s.M) * s.N;
  const size_t npix = static_cast<size_t>(s.B) * s.H * s.W;
  DcnScratch t{};
  t.dcols = reinterpret_cast<float *>(take(rows * s.C * 4));
  t.gwp = reinterpret_cast<float *>(take(static_cast<size_t>(wgrad_split(s, true).slices) * s.O * s.K * 4));
  t.cur = reinterpret_cast<uint32_t *>(take((npix + 1) * 4));
  t.ent = reinterpret_cast<DxEnt *>(take(rows * 4 * sizeof(DxEnt)));
  t.scan_bytes = dcn_scan_bytes(static_cast<int64_t>(npix) + 1);
  t.scan_tmp = take(t.scan_bytes);
  if (w) *w = t;
  return off;
}

// The stateless backward's workspace: the training state, then the scratch.
size_t carve_all(const DcnShape &s, void *base, DcnState *st, DcnScratch *sc) {
  const size_t a = carve_state(s, base, st, true);
  return a + carve_scratch(s, base ? static_cast<char *>(base) + a : nullptr, sc);
}

// split-K of the forward: up to 16 slices of the K' tiles (a sweep of the cap at 32x32 / 16x16 /
// 8x8, profiles/r3_dcn_split_sweep_s1.jsonl: 16 is at least as fast as 32 or 64 on every map, 7 %
// faster at 8x8), only while the pixel x output-channel tiles leave the chip under-filled
#ifndef SBOD_FWD_SPLIT_MAX   // A/B knob: the forward's split-K cap
#define SBOD_FWD_SPLIT_MAX 16
#endif
int fwd_split(const DcnShape &s) {
  const int mt = (s.M + kFM - 1) / kFM, og = (s.O + 255) / 256;
  const int T = s.N * ((s.C + kFKC - 1) / kFKC);
  int split = 1;
  while (split * 2 <= T && mt * og * split < 512 && split < SBOD_FWD_SPLIT_MAX) split *= 2;
  return split;
}

// The weight gradient's finish: dw[o][c][n] = sum over pixel slices (in slice order) of
// gwp[slice][o][n][c].  One block per (64-channel chunk, output channel): the N x 64 sums read
// along c (16-byte vectors when C % 4 == 0, the slices' loads in flight together), staged in LDS,
// written along the [c][n] rows.
template <int VEC>
__global__ __launch_bounds__(256) void k_wgrad_fold(const float *__restrict__ gwp, int slices, int64_t plane, int N,
                                                    int C, float *__restrict__ dw) {
  __shared__ float t[64][kMaxN + 1];
  const int c0 = blockIdx.x * 64, o = blockIdx.y;
  const int nc = min(64, C - c0);
  const float *src = gwp + static_cast<int64_t>(o) * N * C + c0;
  constexpr int G = 64 / VEC;   // vectors per 64-channel row
  for (int e = threadIdx.x; e < N * G; e += blockDim.x) {
    const int n = e / G, cl = (e - n * G) * VEC;
    if (cl >= nc) continue;
    float v[VEC] = {};
    const float *q = src + static_cast<int64_t>(n) * C + cl;
#pragma unroll 4
    for (int sl = 0; sl < slices; ++sl) {
      float x[VEC];
      load_vec<VEC>(q + sl * plane, true, x);
#pragma unroll
      for (int k = 0; k < VEC; ++k) v[k] += x[k];
    }
#pragma unroll
    for (int k = 0; k < VEC; ++k) t[cl + k][n] = v[k];
  }
  __syncthreads();
  float *dst = dw + (static_cast<int64_t>(o) * C + c0) * N;
  for (int e = threadIdx.x; e < nc * N; e += blockDim.x) dst[e] = t[e / N][e % N];
}

}  // namespace sbod

using namespace sbod;

// The independent branches of an eager call at a large map (the weight layouts beside the x
// transpose + coefficients; the dx scan + entry fill beside the backward-data contraction; the dx
// gather beside the weight gradient) go to a side stream, forked from and joined back into the
// caller's stream with events: C4 64x64 eager fwd+bwd 2.259-2.262 vs 2.294-2.304 ms.  Smaller maps
// do not pay for the event calls (round 4), and a captured graph keeps one stream: as parallel
// graph branches the same forks made the replay SLOWER (8x8 0.144-0.146 vs 0.124-0.125 ms, 16x16
// 0.259-0.265 vs 0.244-0.249; 64x64 equal), the branches' cross-queue edges costing more than the
// overlap.  One side stream and four events per host thread and device.
struct SideStream {
  hipStream_t s = nullptr;
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  bool ok = false;
};
constexpr int64_t kEagerForkWork = int64_t(1) << 24;   // M x O: C4's 64x64 map (B=16, O=256)
static SideStream *dcn_side(const DcnShape &s, hipStream_t hs) {
  static thread_local SideStream side[16];
  hipDevice_t dev = 0;
  if (hipStreamGetDevice(hs, &dev) != hipSuccess || dev < 0 || dev >= 16) return nullptr;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (hipStreamIsCapturing(hs, &cs) != hipSuccess) return nullptr;
  const bool capturing = cs == hipStreamCaptureStatusActive;
  SideStream &x = side[dev];
  if (!x.ok && !capturing) {
    int cur = 0;
    if (hipGetDevice(&cur) != hipSuccess) return nullptr;
    if (cur != dev && hipSetDevice(dev) != hipSuccess) return nullptr;
    bool ok = hipStreamCreateWithFlags(&x.s, hipStreamNonBlocking) == hipSuccess;
    for (auto &e : x.ev) ok = ok && hipEventCreateWithFlags(&e, hipEventDisableTiming) == hipSuccess;
    x.ok = ok;
    if (cur != dev) (void)hipSetDevice(cur);
  }
  if (!x.ok || capturing || static_cast<int64_t>(s.M) * s.O < kEagerForkWork) return nullptr;
  return &x;
}
// side stream waits for everything issued on hs so far
static bool dcn_fork(SideStream *x, int e, hipStream_t hs) {
  return hipEventRecord(x->ev[e], hs) == hipSuccess && hipStreamWaitEvent(x->s, x->ev[e], 0) == hipSuccess;
}
// hs waits for everything issued on the side stream so far
static bool dcn_join(SideStream *x, int e, hipStream_t hs) {
  return hipEventRecord(x->ev[e], x->s) == hipSuccess && hipStreamWaitEvent(hs, x->ev[e], 0) == hipSuccess;
}

static int dcn_check(const DcnShape &s, const float *x, const float *offset, const float *weight) {
  SBOD_REQUIRE(x && offset && weight && shape_ok(s),
               "sbod_dcn: bad arguments (NULL tensor, or sizes non-positive, kernel_size > 7 or "
               "beyond 32-bit indexing)");
  SBOD_REQUIRE(s.N <= kMaxN, "sbod_dcn: kernel_size %d > 7 unsupported", s.k);
  SBOD_REQUIRE(static_cast<int64_t>(s.M) * s.N < (1ll << 31) && static_cast<int64_t>(s.C) * s.H * s.W < (1ll << 31) &&
                   static_cast<int64_t>(s.O) * s.K < (1ll << 31) && s.H < 65536 * 64 && s.W < 65536,
               "sbod_dcn: sizes overflow 32-bit indexing");
  return SBOD_OK;
}

// Derives the state from the inputs: x -> channels-last xt (training: the sample counters zeroed
// on the side), the coefficients (training: the counts; split-K: the output zeroed on the side),
// the weight layouts.  Three launches.
static int dcn_derive(const DcnShape &s, const float *x, const float *offset, const float *mask_logits,
                      const float *weight, const DcnState &st, bool train, float *zero_out, int64_t n_zero_out,
                      hipStream_t hs) {
  const int64_t npix = static_cast<int64_t>(s.B) * s.H * s.W;
  const int HW = s.H * s.W;
  SideStream *side = dcn_side(s, hs);
  if (side && !dcn_fork(side, 0, hs)) return launch_status("dcn fork (derive)");
  const hipStream_t ls = side ? side->s : hs;   // the weight layouts' stream
  hipLaunchKernelGGL(k_transpose, dim3((HW + 63) / 64, (s.C + 63) / 64, s.B), dim3(256), 0, hs, x, st.xt, s.C, HW,
                     train ? reinterpret_cast<float *>(st.tcount) : nullptr, train ? npix + 1 : 0);
  SBOD_LAUNCHED("k_transpose(x)");   // x [B][C][HW] -> xt [B][HW][C]
  const int64_t nc = static_cast<int64_t>(s.M) * s.N;
  hipLaunchKernelGGL(k_dcn_coef, dim3((nc + 255) / 256), dim3(256), 0, hs, s, offset, mask_logits, st.coef,
                     train ? st.tcount : nullptr, zero_out, n_zero_out);
  SBOD_LAUNCHED("k_dcn_coef");
#ifdef SBOD_DCN_SPLIT_FWD
  __bf16 *wf3 = st.wf3;
#else
  __bf16 *wf3 = nullptr;
#endif
#ifndef SBOD_DCN_SPLIT_BF16
  hipLaunchKernelGGL(k_weight_layouts, dim3((s.C + 63) / 64, s.O), dim3(256), 0, ls, weight, s.O, s.C, s.N, st.wf,
                     train ? st.wb : nullptr, wf3);
  SBOD_LAUNCHED("k_weight_layouts");
#else
  hipLaunchKernelGGL(k_weight_layouts, dim3((s.C + 63) / 64, s.O), dim3(256), 0, ls, weight, s.O, s.C, s.N, st.wf,
                     static_cast<float *>(nullptr), wf3);
  SBOD_LAUNCHED("k_weight_layouts");
  if (train) {
    const int op = dcn_opad(s.O);
    hipLaunchKernelGGL(k_wb_split, dim3((s.C + 63) / 64, op / 64, s.N), dim3(256), 0, ls, st.wf, s.O, s.C, s.N, op,
                       st.wb3);
    SBOD_LAUNCHED("k_wb_split");
  }
#endif
  if (side && !dcn_join(side, 1, hs)) return launch_status("dcn join (derive)");
  return SBOD_OK;
}

static int dcn_forward(const DcnShape &s, const DcnState &st, float *out, int split, hipStream_t hs) {
  const dim3 grid((s.M + kFM - 1) / kFM, (s.O + 255) / 256, split);
  KernelTimer kt("k_dcn_fwd", hs);
  const size_t lds = static_cast<size_t>(s.N) * 9 * kFM * 4;   // the block's coefficients
  if (lds > 48 * 1024) {   // k >= 5: above the default dynamic-LDS limit (gfx950 has 160 KB per CU)
    const void *f = s.C % 4 == 0 ? reinterpret_cast<const void *>(k_dcn_fwd<4>) : reinterpret_cast<const void *>(k_dcn_fwd<1>);
    if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)) != hipSuccess)
      return launch_status("hipFuncSetAttribute(k_dcn_fwd LDS)");
  }
#ifdef SBOD_DCN_SPLIT_FWD
  if (s.C % 8 == 0) {
    if (lds > 48 * 1024 &&
        hipFuncSetAttribute(reinterpret_cast<const void *>(k_dcn_fwd3), hipFuncAttributeMaxDynamicSharedMemorySize,
                            static_cast<int>(lds)) != hipSuccess)
      return launch_status("hipFuncSetAttribute(k_dcn_fwd3 LDS)");
    hipLaunchKernelGGL(k_dcn_fwd3, grid, dim3(kDcnThreads), lds, hs, s, st.xt, st.coef,
                       static_cast<const __bf16 *>(st.wf3), out, split > 1 ? 1 : 0);
    SBOD_LAUNCHED("k_dcn_fwd3");
    return SBOD_OK;
  }
#endif
  if (s.C % 4 == 0)
    hipLaunchKernelGGL(k_dcn_fwd<4>, grid, dim3(kDcnThreads), lds, hs, s, st.xt, st.coef, st.wf, out, split > 1 ? 1 : 0);
  else
    hipLaunchKernelGGL(k_dcn_fwd<1>, grid, dim3(kDcnThreads), lds, hs, s, st.xt, st.coef, st.wf, out, split > 1 ? 1 : 0);
  SBOD_LAUNCHED("k_dcn_fwd");
  return SBOD_OK;
}

// The backward from a training state: with dx wanted, scan (the pixels' entry ranges) -> dx_fill
// (which also zeroes the offset / mask / weight gradients) -> bwd_data (dcols rows) -> dx gather
// (straight into [B][C][H][W]) -> bwd_weight (weight gradient into [O][C][k][k] and the offset /
// mask gradients) -> transpose of dWp; six launches for all four gradients.
static int dcn_backward(const DcnShape &s, const DcnState &st, const DcnScratch &sc, const float *grad_out,
                        float *grad_x, float *grad_offset, float *grad_mask_logits, float *grad_weight, hipStream_t hs) {
  const int npix = s.B * s.H * s.W;
  const bool need_om = grad_offset || grad_mask_logits;
  const bool need_cols = grad_x || need_om;
  SBOD_REQUIRE(!need_cols || (static_cast<int64_t>(s.M) * s.O * 4 < (1ll << 31) &&
                              static_cast<int64_t>(s.N) * s.O * s.C * 4 < (1ll << 31)),
               "sbod_dcn_bwd: grad_out / weight exceed the 2 GiB buffer-descriptor range");
  const int64_t ob = static_cast<int64_t>(s.M) * s.N;
  // with dx: the scan + entry fill (side stream) beside the backward-data contraction, joined
  // before the weight gradient (which adds into the offset / mask gradients the fill zeroes);
  // then the dx gather (side stream) beside the weight gradient, joined at the end
  SideStream *side = grad_x && need_cols ? dcn_side(s, hs) : nullptr;
  if (side && !dcn_fork(side, 0, hs)) return launch_status("dcn fork (backward)");
  const hipStream_t xs = side ? side->s : hs;   // the dx branch's stream
  if (grad_x) {   // the input pixels' entry ranges (scan of the counts the forward made)
    if (npix + 1 <= kScanOneBlock) {
      hipLaunchKernelGGL(k_dcn_scan, dim3(1), dim3(1024), 0, xs, st.tcount, sc.cur, npix + 1);
      SBOD_LAUNCHED("k_dcn_scan");
    } else {
      size_t tb = sc.scan_bytes;
      if (hipcub::DeviceScan::ExclusiveSum(sc.scan_tmp, tb, st.tcount, sc.cur, npix + 1, xs) != hipSuccess)
        return launch_status("DeviceScan(dcn dx offsets)");
    }
    hipLaunchKernelGGL(k_dcn_dx_fill, dim3((ob + 255) / 256), dim3(256), 0, xs, s, st.coef, sc.cur, sc.ent,
                       grad_offset, grad_offset ? 2 * ob : 0, grad_mask_logits, grad_mask_logits ? ob : 0,
                       nullptr, int64_t(0));
    SBOD_LAUNCHED("k_dcn_dx_fill");
  } else {
    if (grad_offset && hipMemsetAsync(grad_offset, 0, 2 * ob * 4, hs) != hipSuccess) return launch_status("memset");
    if (grad_mask_logits && hipMemsetAsync(grad_mask_logits, 0, ob * 4, hs) != hipSuccess) return launch_status("memset");
  }
  if (need_cols) {
    KernelTimer kt("k_dcn_bwd_data", hs);
    // 64-pixel blocks, or 32 when that leaves fewer blocks than CUs (C4's 8x8 map: 144 -> 288)
    const int64_t nb64 = static_cast<int64_t>((s.M + kBM - 1) / kBM) * ((s.C + 255) / 256) * s.N;
#ifndef SBOD_DCN_SPLIT_BF16
    if (nb64 >= kBwdDataMinBlocks)
      hipLaunchKernelGGL(k_dcn_bwd_data<2>, dim3((s.M + 63) / 64, (s.C + 255) / 256, s.N), dim3(kDcnThreads), 0,
                         hs, s, st.wb, grad_out, sc.dcols);
    else
      hipLaunchKernelGGL(k_dcn_bwd_data<1>, dim3((s.M + 31) / 32, (s.C + 255) / 256, s.N), dim3(kDcnThreads), 0,
                         hs, s, st.wb, grad_out, sc.dcols);
#else
    const int op = dcn_opad(s.O);
    if (nb64 >= kBwdDataMinBlocks)
      hipLaunchKernelGGL(k_dcn_bwd_data3<2>, dim3((s.M + 63) / 64, (s.C + 255) / 256, s.N), dim3(kDcnThreads), 0,
                         hs, s, static_cast<const __bf16 *>(st.wb3), op, grad_out, sc.dcols);
    else
      hipLaunchKernelGGL(k_dcn_bwd_data3<1>, dim3((s.M + 31) / 32, (s.C + 255) / 256, s.N), dim3(kDcnThreads), 0,
                         hs, s, static_cast<const __bf16 *>(st.wb3), op, grad_out, sc.dcols);
#endif
  }
  if (need_cols) SBOD_LAUNCHED("k_dcn_bwd_data");
  if (side && !(dcn_join(side, 1, hs) && dcn_fork(side, 2, hs))) return launch_status("dcn join / fork (backward)");
  if (grad_x) {
    {
      KernelTimer kt("k_dcn_dx_gather", xs);
      const dim3 grid((npix + kGxPix - 1) / kGxPix);
      if (s.C % 4 == 0)
        hipLaunchKernelGGL(k_dcn_dx_gather<4>, grid, dim3(64 * kGxPix), 0, xs, s.C, s.H * s.W, npix, sc.cur, sc.ent,
                           sc.dcols, grad_x);
      else
        hipLaunchKernelGGL(k_dcn_dx_gather<1>, grid, dim3(64 * kGxPix), 0, xs, s.C, s.H * s.W, npix, sc.cur, sc.ent,
                           sc.dcols, grad_x);
    }
    SBOD_LAUNCHED("k_dcn_dx_gather");
  }
  if (grad_weight || need_om) {
    // weight gradient, and the offset / mask gradients from the same corner samples (C / 64
    // channel-block partials added into the zeroed outputs)
    const WgSplit wg = wgrad_split(s, grad_weight != nullptr);
    const int m_slice = wg.m_slice;
    const dim3 grid(wg.gx, wg.slices, wg.gz);
    const bool avec = (s.Ho * s.Wo) % kWMs == 0;   // 32-pixel chunks never straddle images
    const float *dc = need_om ? sc.dcols : nullptr;
    {
      KernelTimer kt("k_dcn_bwd_weight", hs);
      auto go = [&](auto kern) {
        hipLaunchKernelGGL(kern, grid, dim3(kDcnThreads), 0, hs, s, st.xt, st.coef, grad_out, grad_weight ? sc.gwp : nullptr, m_slice, dc,
                           grad_offset, grad_mask_logits);
      };
#if defined(SBOD_DCN_SPLIT_FWD) && !defined(SBOD_DCN_FP32_WGRAD)
      constexpr bool split = true;   // the split-bf16 weight gradient (A/B build: -DSBOD_DCN_FP32_WGRAD)
#else
      constexpr bool split = false;
#endif
      if (dc) {
        if (s.C % 4 == 0 && avec) {
          if constexpr (split) go(k_dcn_bwd_weight3<true>);
          else go(k_dcn_bwd_weight<4, true, true>);
        } else if (s.C % 4 == 0) go(k_dcn_bwd_weight<4, false, true>);
        else go(k_dcn_bwd_weight<1, false, true>);
      } else {
        if (s.C % 4 == 0 && avec) {
          if constexpr (split) go(k_dcn_bwd_weight3<false>);
          else go(k_dcn_bwd_weight<4, true, false>);
        } else if (s.C % 4 == 0) go(k_dcn_bwd_weight<4, false, false>);
        else go(k_dcn_bwd_weight<1, false, false>);
      }
    }
    SBOD_LAUNCHED("k_dcn_bwd_weight");
    if (grad_weight) {   // the slices' dWp [O][N][C] planes summed -> conv.weight's [O][C][N]
      const dim3 fg((s.C + 63) / 64, s.O);
      const int64_t plane = static_cast<int64_t>(s.O) * s.K;
      if (s.C % 4 == 0)
        hipLaunchKernelGGL(k_wgrad_fold<4>, fg, dim3(256), 0, hs, sc.gwp, wg.slices, plane, s.N, s.C, grad_weight);
      else
        hipLaunchKernelGGL(k_wgrad_fold<1>, fg, dim3(256), 0, hs, sc.gwp, wg.slices, plane, s.N, s.C, grad_weight);
      SBOD_LAUNCHED("k_wgrad_fold");
    }
  }
  if (side && !dcn_join(side, 3, hs)) return launch_status("dcn join (backward)");
  return SBOD_OK;
}

extern "C" {

size_t sbod_dcn_workspace_bytes(int B, int C, int H, int W, int O, int k, int stride, int pad) {
  const DcnShape s = make_shape(B, C, H, W, O, k, stride, pad);
  return shape_ok(s) ? carve_all(s, nullptr, nullptr, nullptr) : 0;
}

size_t sbod_dcn_fwd_workspace_bytes(int B, int C, int H, int W, int O, int k, int stride, int pad) {
  const DcnShape s = make_shape(B, C, H, W, O, k, stride, pad);
  return shape_ok(s) ? carve_state(s, nullptr, nullptr, false) : 0;
}

size_t sbod_dcn_state_bytes(int B, int C, int H, int W, int O, int k, int stride, int pad) {
  const DcnShape s = make_shape(B, C, H, W, O, k, stride, pad);
  return shape_ok(s) ? carve_state(s, nullptr, nullptr, true) : 0;
}

size_t sbod_dcn_scratch_bytes(int B, int C, int H, int W, int O, int k, int stride, int pad) {
  const DcnShape s = make_shape(B, C, H, W, O, k, stride, pad);
  return shape_ok(s) ? carve_scratch(s, nullptr, nullptr) : 0;
}

int sbod_dcn_fwd_f32(const float *x, const float *offset, const float *mask_logits,
                     const float *weight, int B, int C, int H, int W, int O, int k, int stride,
                     int pad, float *out, void *workspace, size_t workspace_bytes, void *stream) {
  const DcnShape s = make_shape(B, C, H, W, O, k, stride, pad);
  int st = dcn_check(s, x, offset, weight);
  if (st != SBOD_OK) return st;
  SBOD_REQUIRE(out != nullptr, "sbod_dcn_fwd_f32: out is NULL");
  const size_t need = carve_state(s, nullptr, nullptr, false);
  if (workspace == nullptr || workspace_bytes < need) {
    set_error("sbod_dcn_fwd_f32: workspace %zu < %zu", workspace_bytes, need);
    return SBOD_E_WORKSPACE;
  }
  hipStream_t hs = as_stream(stream);
  DcnState w;
  carve_state(s, workspace, &w, false);
  const int split = fwd_split(s);
  st = dcn_derive(s, x, offset, mask_logits, weight, w, false, split > 1 ? out : nullptr,
                  split > 1 ? static_cast<int64_t>(s.M) * s.O : 0, hs);
  if (st != SBOD_OK) return st;
  return dcn_forward(s, w, out, split, hs);
}

int sbod_dcn_fwd_train_f32(const float *x, const float *offset, const float *mask_logits,
                           const float *weight, int B, int C, int H, int W, int O, int k, int stride,
                           int pad, float *out, void *state, size_t state_bytes, void *stream) {
  const DcnShape s = make_shape(B, C, H, W, O, k, stride, pad);
  int st = dcn_check(s, x, offset, weight);
  if (st != SBOD_OK) return st;
  SBOD_REQUIRE(out != nullptr, "sbod_dcn_fwd_train_f32: out is NULL");
  const size_t need = carve_state(s, nullptr, nullptr, true);
  if (state == nullptr || state_bytes < need) {
    set_error("sbod_dcn_fwd_train_f32: state %zu < %zu", state_bytes, need);
    return SBOD_E_WORKSPACE;
  }
  hipStream_t hs = as_stream(stream);
  DcnState w;
  carve_state(s, state, &w, true);
  const int split = fwd_split(s);
  st = dcn_derive(s, x, offset, mask_logits, weight, w, true, split > 1 ? out : nullptr,
                  split > 1 ? static_cast<int64_t>(s.M) * s.O : 0, hs);
  if (st != SBOD_OK) return st;
  return dcn_forward(s, w, out, split, hs);
}

int sbod_dcn_bwd_state_f32(const float *grad_out, int B, int C, int H, int W, int O, int k, int stride,
                           int pad, float *grad_x, float *grad_offset, float *grad_mask_logits,
                           float *grad_weight, const void *state, size_t state_bytes, void *scratch,
                           size_t scratch_bytes, void *stream) {
  const DcnShape s = make_shape(B, C, H, W, O, k, stride, pad);
  SBOD_REQUIRE(shape_ok(s) && s.N <= kMaxN, "sbod_dcn_bwd_state_f32: bad sizes");
  SBOD_REQUIRE(grad_out != nullptr, "sbod_dcn_bwd_state_f32: grad_out is NULL");
  const size_t need_st = carve_state(s, nullptr, nullptr, true), need_sc = carve_scratch(s, nullptr, nullptr);
  if (state == nullptr || state_bytes < need_st || scratch == nullptr || scratch_bytes < need_sc) {
    set_error("sbod_dcn_bwd_state_f32: state %zu < %zu or scratch %zu < %zu", state_bytes, need_st, scratch_bytes,
              need_sc);
    return SBOD_E_WORKSPACE;
  }
  DcnState w;
  DcnScratch t;
  carve_state(s, const_cast<void *>(state), &w, true);
  carve_scratch(s, scratch, &t);
  return dcn_backward(s, w, t, grad_out, grad_x, grad_offset, grad_mask_logits, grad_weight, as_stream(stream));
}

int sbod_dcn_bwd_f32(const float *x, const float *offset, const float *mask_logits,
                     const float *weight, const float *grad_out, int B, int C, int H, int W,
                     int O, int k, int stride, int pad, float *grad_x, float *grad_offset,
                     float *grad_mask_logits, float *grad_weight, void *workspace,
                     size_t workspace_bytes, void *stream) {
  const DcnShape s = make_shape(B, C, H, W, O, k, stride, pad);
  int st = dcn_check(s, x, offset, weight);
  if (st != SBOD_OK) return st;
  SBOD_REQUIRE(grad_out != nullptr, "sbod_dcn_bwd_f32: grad_out is NULL");
  const size_t need = carve_all(s, nullptr, nullptr, nullptr);
  if (workspace == nullptr || workspace_bytes < need) {
    set_error("sbod_dcn_bwd_f32: workspace %zu < %zu", workspace_bytes, need);
    return SBOD_E_WORKSPACE;
  }
  hipStream_t hs = as_stream(stream);
  DcnState w;
  DcnScratch t;
  carve_all(s, workspace, &w, &t);
  st = dcn_derive(s, x, offset, mask_logits, weight, w, true, nullptr, 0, hs);   // the state, re-derived
  if (st != SBOD_OK) return st;
  if (!mask_logits) grad_mask_logits = nullptr;
  return dcn_backward(s, w, t, grad_out, grad_x, grad_offset, grad_mask_logits, grad_weight, hs);
}

}  // extern "C"
