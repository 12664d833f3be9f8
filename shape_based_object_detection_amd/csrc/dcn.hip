// DeformConv2d (operators/Deformable_convolution.py:5-146): modulated DCNv2 with the reference's
// semantics (offset channels [rows | cols], p_0 = 1 + idx * stride, floor of the UNclamped p,
// corners and p clamped to the zero-padded map, sigmoid modulation, k x k stride-k conv, no bias).
//
// The contraction runs on fp32 MFMA (v_mfma_f32_32x32x2_f32: exact f32 products, one rounding
// per step) so results stay within fp32 tolerance of the reference.  GEMM views, with
// M = B*Ho*Wo output pixels, K = C*k*k (c-major, the flattening of conv.weight [O,C,k,k]):
//   forward      out[o, m]  = sum_K W[o, K] * cols[K, m]
//   backward     dcols[K,m] = sum_o W[o, K] * dout[o, m]   -> dx (atomics), d_offset, d_mask
//                dW[o, K]   = sum_m dout[o, m] * cols[K, m]
// cols[K, m] = sigmoid(mask) * sum_q g_q * x_pad[corner_q] is never materialised: it is built
// per K-tile into LDS from per-(pixel, kernel point) coefficients computed once (k_dcn_coef),
// so the bilinear gathers are shared by every output channel of the tile.
// Roofline: MFMA-bound (2*M*O*K flops forward, 4*M*O*K backward).
#include "sbod_common.h"

namespace sbod {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kDcnThreads = 256;
constexpr int kMaxN = 49;      // k*k <= 49 (k <= 7)

// Per (pixel m, kernel point n): corner offsets in the (b, c) plane (-1 outside the original
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

__global__ __launch_bounds__(256) void k_dcn_coef(DcnShape s, const float *__restrict__ offset,
                                                  const float *__restrict__ mlog,
                                                  Coef *__restrict__ coef) {
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
}

// Modulated sample cols[K = c*N + n, m]; the sum order of the reference (lt + rb + lb + rt) * m.
__device__ __forceinline__ float sample(const float *__restrict__ xplane, const Coef &c) {
  float v[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) v[q] = c.idx[q] >= 0 ? xplane[c.idx[q]] : 0.f;
  return (((c.g[0] * v[0] + c.g[1] * v[1]) + c.g[2] * v[2]) + c.g[3] * v[3]) * c.mval;
}

// ----------------------------------------------------------------------------- forward
// Block = 64 pixels x 256 output channels (4 waves x 64 channels, 2 x 2 tiles of 32 x 32).
constexpr int kFM = 64, kFO = 256, kFK = 32;

__global__ __launch_bounds__(kDcnThreads) void k_dcn_fwd(DcnShape s, const float *__restrict__ x,
                                                         const Coef *__restrict__ coef,
                                                         const float *__restrict__ wt,
                                                         float *__restrict__ out) {
  __shared__ float s_cols[kFK][kFM];         // B operand [k][m]
  __shared__ float s_w[kFO][kFK + 1];        // A operand [o][k]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int m0 = blockIdx.x * kFM, o0 = blockIdx.y * kFO;
  const int HW = s.H * s.W, HWo = s.Ho * s.Wo;
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  for (int k0 = 0; k0 < s.K; k0 += kFK) {
    __syncthreads();
    for (int e = tid; e < kFK * kFM; e += kDcnThreads) {
      const int kk = e / kFM, mm = e - kk * kFM;
      const int K = k0 + kk, m = m0 + mm;
      float v = 0.f;
      if (K < s.K && m < s.M) {
        const int c = K / s.N, n = K - c * s.N;
        const int b = m / HWo;
        v = sample(x + (static_cast<int64_t>(b) * s.C + c) * HW, coef[static_cast<int64_t>(m) * s.N + n]);
      }
      s_cols[kk][mm] = v;
    }
    for (int e = tid; e < kFO * kFK; e += kDcnThreads) {
      const int o = e / kFK, kk = e - o * kFK;
      const int K = k0 + kk;
      s_w[o][kk] = (o0 + o < s.O && K < s.K) ? wt[static_cast<int64_t>(o0 + o) * s.K + K] : 0.f;
    }
    __syncthreads();
#pragma unroll 4
    for (int st = 0; st < kFK / 2; ++st) {
      const int kk = 2 * st + (lane >> 5);
      const float a0 = s_w[64 * wv + (lane & 31)][kk];
      const float a1 = s_w[64 * wv + 32 + (lane & 31)][kk];
      const float b0 = s_cols[kk][lane & 31];
      const float b1 = s_cols[kk][32 + (lane & 31)];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
  }
  // C/D map (gfx950, dtype independent): col = lane & 31, row = (r&3) + 8*(r>>2) + 4*(lane>>5)
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bq = 0; bq < 2; ++bq) {
      const int m = m0 + 32 * bq + (lane & 31);
      if (m >= s.M) continue;
      const int b = m / HWo, pix = m - b * HWo;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = o0 + 64 * wv + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (o < s.O) out[(static_cast<int64_t>(b) * s.O + o) * HWo + pix] = acc[a][bq][r];
      }
    }
}

// ----------------------------------------------------------------------------- backward (data)
// Block = 64 pixels; per K-tile of 128 (4 waves x 32 rows) dcols = W^T dout over all O, then the
// epilogue turns each dcols element into dx (atomics) and per-(pixel, n) sums of d_mask and
// d_p (LDS), written once at the end (clamp masks applied, sigmoid derivative applied).
constexpr int kBM = 64, kBK = 128, kBO = 64;

__global__ __launch_bounds__(kDcnThreads) void k_dcn_bwd_data(
    DcnShape s, const float *__restrict__ x, const Coef *__restrict__ coef,
    const float *__restrict__ wt, const float *__restrict__ gout, float *__restrict__ gx,
    float *__restrict__ goff, float *__restrict__ gmlog) {
  __shared__ float s_dout[kBO][kBM];           // B operand [o][m]
  __shared__ float s_wt[kBK][kBO + 1];         // A operand [K][o]
  __shared__ float s_acc[3][kBM][kMaxN];       // d_mask, d_px, d_py per (pixel, n)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int m0 = blockIdx.x * kBM;
  const int HW = s.H * s.W, HWo = s.Ho * s.Wo;
  for (int e = tid; e < 3 * kBM * kMaxN; e += kDcnThreads) (&s_acc[0][0][0])[e] = 0.f;
  for (int K0 = 0; K0 < s.K; K0 += kBK) {
    f32x16 acc[2];
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[0][r] = acc[1][r] = 0.f;
    for (int o0 = 0; o0 < s.O; o0 += kBO) {
      __syncthreads();
      for (int e = tid; e < kBO * kBM; e += kDcnThreads) {
        const int oo = e / kBM, mm = e - oo * kBM;
        const int o = o0 + oo, m = m0 + mm;
        float v = 0.f;
        if (o < s.O && m < s.M) {
          const int b = m / HWo, pix = m - b * HWo;
          v = gout[(static_cast<int64_t>(b) * s.O + o) * HWo + pix];
        }
        s_dout[oo][mm] = v;
      }
      for (int e = tid; e < kBO * kBK; e += kDcnThreads) {
        const int oo = e / kBK, kk = e - oo * kBK;
        const int o = o0 + oo, K = K0 + kk;
        s_wt[kk][oo] = (o < s.O && K < s.K) ? wt[static_cast<int64_t>(o) * s.K + K] : 0.f;
      }
      __syncthreads();
#pragma unroll 4
      for (int st = 0; st < kBO / 2; ++st) {
        const int oo = 2 * st + (lane >> 5);
        const float a = s_wt[32 * wv + (lane & 31)][oo];
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, s_dout[oo][lane & 31], acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, s_dout[oo][32 + (lane & 31)], acc[1], 0, 0, 0);
      }
    }
    // epilogue: element (K, m) of this wave's 32 x 64 slab
#pragma unroll
    for (int bq = 0; bq < 2; ++bq) {
      const int mm = 32 * bq + (lane & 31), m = m0 + mm;
      if (m >= s.M) continue;
      const int b = m / HWo;
#pragma unroll 4
      for (int r = 0; r < 16; ++r) {
        const int K = K0 + 32 * wv + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (K >= s.K) continue;
        const int c = K / s.N, n = K - c * s.N;
        const Coef cf = coef[static_cast<int64_t>(m) * s.N + n];
        const int64_t plane = (static_cast<int64_t>(b) * s.C + c) * HW;
        float v[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = cf.idx[q] >= 0 ? x[plane + cf.idx[q]] : 0.f;
        const float dcol = acc[bq][r];
        const float raw = ((cf.g[0] * v[0] + cf.g[1] * v[1]) + cf.g[2] * v[2]) + cf.g[3] * v[3];
        const float dval = dcol * cf.mval;
        if (gx) {
#pragma unroll
          for (int q = 0; q < 4; ++q)
            if (cf.idx[q] >= 0) atomicAdd(gx + plane + cf.idx[q], dval * cf.g[q]);
        }
        const float dpx = -(1.f + cf.tly) * v[0] + (1.f - cf.rby) * v[1] - (1.f - cf.rby) * v[2] + (1.f + cf.tly) * v[3];
        const float dpy = -(1.f + cf.tlx) * v[0] + (1.f - cf.rbx) * v[1] + (1.f + cf.tlx) * v[2] - (1.f - cf.rbx) * v[3];
        atomicAdd(&s_acc[0][mm][n], dcol * raw);
        atomicAdd(&s_acc[1][mm][n], dval * dpx);
        atomicAdd(&s_acc[2][mm][n], dval * dpy);
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < kBM * s.N; e += kDcnThreads) {
    const int mm = e / s.N, n = e - mm * s.N, m = m0 + mm;
    if (m >= s.M) continue;
    const Coef cf = coef[static_cast<int64_t>(m) * s.N + n];
    const int b = m / HWo, pix = m - b * HWo;
    if (goff) {
      goff[(static_cast<int64_t>(b) * 2 * s.N + n) * HWo + pix] = (cf.inr & 1) ? s_acc[1][mm][n] : 0.f;
      goff[(static_cast<int64_t>(b) * 2 * s.N + s.N + n) * HWo + pix] = (cf.inr & 2) ? s_acc[2][mm][n] : 0.f;
    }
    if (gmlog) gmlog[(static_cast<int64_t>(b) * s.N + n) * HWo + pix] = s_acc[0][mm][n] * cf.mval * (1.f - cf.mval);
  }
}

// ----------------------------------------------------------------------------- backward (weight)
// Block = (64-wide K tile, a slice of kWSlice pixels), 256 output channels (4 waves x 64).
// dW partial sums are added with float atomics (one 64 x 64 tile per wave at the end).
constexpr int kWK = 64, kWO = 256, kWMs = 32, kWSlice = 2048;

__global__ __launch_bounds__(kDcnThreads) void k_dcn_bwd_weight(
    DcnShape s, const float *__restrict__ x, const Coef *__restrict__ coef,
    const float *__restrict__ gout, float *__restrict__ gw) {
  __shared__ float s_cols[kWMs][kWK];          // B operand [m][K]
  __shared__ float s_dout[kWO][kWMs + 1];      // A operand [o][m]
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int K0 = blockIdx.x * kWK, ms0 = blockIdx.y * kWSlice, o0 = blockIdx.z * kWO;
  const int HW = s.H * s.W, HWo = s.Ho * s.Wo;
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][b][r] = 0.f;
  const int mend = min(ms0 + kWSlice, s.M);
  for (int m0 = ms0; m0 < mend; m0 += kWMs) {
    __syncthreads();
    for (int e = tid; e < kWMs * kWK; e += kDcnThreads) {
      const int mm = e / kWK, kk = e - mm * kWK;
      const int m = m0 + mm, K = K0 + kk;
      float v = 0.f;
      if (m < mend && K < s.K) {
        const int c = K / s.N, n = K - c * s.N;
        const int b = m / HWo;
        v = sample(x + (static_cast<int64_t>(b) * s.C + c) * HW, coef[static_cast<int64_t>(m) * s.N + n]);
      }
      s_cols[mm][kk] = v;
    }
    for (int e = tid; e < kWO * kWMs; e += kDcnThreads) {
      const int oo = e / kWMs, mm = e - oo * kWMs;
      const int o = o0 + oo, m = m0 + mm;
      float v = 0.f;
      if (o < s.O && m < mend) {
        const int b = m / HWo, pix = m - b * HWo;
        v = gout[(static_cast<int64_t>(b) * s.O + o) * HWo + pix];
      }
      s_dout[oo][mm] = v;
    }
    __syncthreads();
#pragma unroll 4
    for (int st = 0; st < kWMs / 2; ++st) {
      const int mm = 2 * st + (lane >> 5);
      const float a0 = s_dout[64 * wv + (lane & 31)][mm];
      const float a1 = s_dout[64 * wv + 32 + (lane & 31)][mm];
      const float b0 = s_cols[mm][lane & 31];
      const float b1 = s_cols[mm][32 + (lane & 31)];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
  }
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int bq = 0; bq < 2; ++bq) {
      const int K = K0 + 32 * bq + (lane & 31);
      if (K >= s.K) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int o = o0 + 64 * wv + 32 * a + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (o < s.O) atomicAdd(gw + static_cast<int64_t>(o) * s.K + K, acc[a][bq][r]);
      }
    }
}

DcnShape make_shape(int B, int C, int H, int W, int O, int k, int stride, int pad) {
  DcnShape s;
  s.B = B; s.C = C; s.H = H; s.W = W; s.O = O; s.k = k; s.N = k * k;
  s.stride = stride; s.pad = pad;
  s.Ho = (H - 1) / stride + 1;   // p_conv: 3x3, padding 1, stride `stride`
  s.Wo = (W - 1) / stride + 1;
  s.Hp = H + 2 * pad;
  s.Wp = W + 2 * pad;
  s.M = B * s.Ho * s.Wo;
  s.K = C * s.N;
  return s;
}

}  // namespace sbod

using namespace sbod;

extern "C" {

size_t sbod_dcn_workspace_bytes(int B, int C, int H, int W, int O, int k, int stride, int pad) {
  const DcnShape s = make_shape(B, C, H, W, O, k, stride, pad);
  return align_up(static_cast<size_t>(s.M) * s.N * sizeof(Coef));
}

static int dcn_check(const DcnShape &s, const float *x, const float *offset, const float *weight) {
  SBOD_REQUIRE(x && offset && weight && s.B > 0 && s.C > 0 && s.H > 0 && s.W > 0 && s.O > 0 &&
                   s.k > 0 && s.stride > 0 && s.pad >= 0,
               "sbod_dcn: bad arguments");
  SBOD_REQUIRE(s.N <= kMaxN, "sbod_dcn: kernel_size %d > 7 unsupported", s.k);
  SBOD_REQUIRE(static_cast<int64_t>(s.M) * s.N < (1ll << 31) && static_cast<int64_t>(s.C) * s.H * s.W < (1ll << 31),
               "sbod_dcn: sizes overflow 32-bit indexing");
  return SBOD_OK;
}

int sbod_dcn_fwd_f32(const float *x, const float *offset, const float *mask_logits,
                     const float *weight, int B, int C, int H, int W, int O, int k, int stride,
                     int pad, float *out, void *workspace, size_t workspace_bytes, void *stream) {
  const DcnShape s = make_shape(B, C, H, W, O, k, stride, pad);
  int st = dcn_check(s, x, offset, weight);
  if (st != SBOD_OK) return st;
  SBOD_REQUIRE(out != nullptr, "sbod_dcn_fwd_f32: out is NULL");
  const size_t need = sbod_dcn_workspace_bytes(B, C, H, W, O, k, stride, pad);
  if (workspace_bytes < need) {
    set_error("sbod_dcn_fwd_f32: workspace %zu < %zu", workspace_bytes, need);
    return SBOD_E_WORKSPACE;
  }
  hipStream_t hs = as_stream(stream);
  Coef *coef = static_cast<Coef *>(workspace);
  const int64_t nc = static_cast<int64_t>(s.M) * s.N;
  hipLaunchKernelGGL(k_dcn_coef, dim3((nc + 255) / 256), dim3(256), 0, hs, s, offset, mask_logits, coef);
  SBOD_LAUNCHED("k_dcn_coef");
  hipLaunchKernelGGL(k_dcn_fwd, dim3((s.M + kFM - 1) / kFM, (s.O + kFO - 1) / kFO), dim3(kDcnThreads), 0,
                     hs, s, x, coef, weight, out);
  SBOD_LAUNCHED("k_dcn_fwd");
  return SBOD_OK;
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
  const size_t need = sbod_dcn_workspace_bytes(B, C, H, W, O, k, stride, pad);
  if (workspace_bytes < need) {
    set_error("sbod_dcn_bwd_f32: workspace %zu < %zu", workspace_bytes, need);
    return SBOD_E_WORKSPACE;
  }
  hipStream_t hs = as_stream(stream);
  Coef *coef = static_cast<Coef *>(workspace);
  const int64_t nc = static_cast<int64_t>(s.M) * s.N;
  hipLaunchKernelGGL(k_dcn_coef, dim3((nc + 255) / 256), dim3(256), 0, hs, s, offset, mask_logits, coef);
  SBOD_LAUNCHED("k_dcn_coef");
  if (grad_x || grad_offset || grad_mask_logits) {
    float *gx = grad_x;
    if (gx && hipMemsetAsync(gx, 0, static_cast<size_t>(B) * C * H * W * 4, hs) != hipSuccess)
      return launch_status("hipMemsetAsync(dcn dx)");
    hipLaunchKernelGGL(k_dcn_bwd_data, dim3((s.M + kBM - 1) / kBM), dim3(kDcnThreads), 0, hs, s, x, coef,
                       weight, grad_out, gx, grad_offset, mask_logits ? grad_mask_logits : nullptr);
    SBOD_LAUNCHED("k_dcn_bwd_data");
  }
  if (grad_weight) {
    if (hipMemsetAsync(grad_weight, 0, static_cast<size_t>(O) * s.K * 4, hs) != hipSuccess)
      return launch_status("hipMemsetAsync(dcn dw)");
    hipLaunchKernelGGL(k_dcn_bwd_weight,
                       dim3((s.K + kWK - 1) / kWK, (s.M + kWSlice - 1) / kWSlice, (s.O + kWO - 1) / kWO),
                       dim3(kDcnThreads), 0, hs, s, x, coef, grad_out, grad_weight);
    SBOD_LAUNCHED("k_dcn_bwd_weight");
  }
  return SBOD_OK;
}

}  // extern "C"
