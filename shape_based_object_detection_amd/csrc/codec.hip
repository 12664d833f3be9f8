// Box codecs (dataset/transforms.py:26-83, iou_utils.py:167-177 / 324-368).
// Element-wise, HBM-bound: 32 B per row (read 16 + write 16) + 16 B of prior.
#include "sbod_common.h"

namespace sbod {

__global__ __launch_bounds__(256) void k_codec(int op, const float *__restrict__ in,
                                               const float *__restrict__ pri, int64_t n,
                                               int64_t prow, float v0, float v1,
                                               float *__restrict__ out) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += stride) {
    Box4 x = ld4(in + 4 * i);
    Box4 p{0.f, 0.f, 0.f, 0.f};
    if (pri) p = ld4(pri + 4 * (prow > 0 ? i % prow : i));
    Box4 r;
    switch (op) {
      case SBOD_CODEC_XY_TO_CXCY:
        r = xy_to_cxcy(x);
        break;
      case SBOD_CODEC_CXCY_TO_XY:  // transforms.py:44-45 (also iou_utils.point_form)
        r = Box4{x.a - x.c / 2.f, x.b - x.d / 2.f, x.a + x.c / 2.f, x.b + x.d / 2.f};
        break;
      case SBOD_CODEC_ENCODE_TENFIVE:
        r = encode_tenfive(x, p);
        break;
      case SBOD_CODEC_DECODE_TENFIVE:  // gcxgcy_to_cxcy
        r = Box4{x.a * p.c / 10.f + p.a, x.b * p.d / 10.f + p.b, expf(x.c / 5.f) * p.c,
                 expf(x.d / 5.f) * p.d};
        break;
      case SBOD_CODEC_DECODE_TENFIVE_XY:
        r = decode_tenfive_xy(x, p);
        break;
      case SBOD_CODEC_ENCODE_VAR: {  // iou_utils.encode: x is matched xyxy
        float gx = (x.a + x.c) / 2.f - p.a, gy = (x.b + x.d) / 2.f - p.b;
        gx = gx / (v0 * p.c);
        gy = gy / (v0 * p.d);
        r = Box4{gx, gy, logf((x.c - x.a) / p.c) / v1, logf((x.d - x.b) / p.d) / v1};
        break;
      }
      default: {  // SBOD_CODEC_DECODE_VAR, iou_utils.decode
        float cx = p.a + x.a * v0 * p.c, cy = p.b + x.b * v0 * p.d;
        float w = p.c * expf(x.c * v1), h = p.d * expf(x.d * v1);
        float x1 = cx - w / 2.f, y1 = cy - h / 2.f;
        r = Box4{x1, y1, w + x1, h + y1};
      }
    }
    st4(out + 4 * i, r);
  }
}

}  // namespace sbod

extern "C" int sbod_codec_f32(int op, const float *in, const float *priors, int64_t n,
                              int64_t prior_rows, float var0, float var1, float *out, void *stream) {
  SBOD_REQUIRE(n >= 0 && in && out && op >= 0 && op <= SBOD_CODEC_DECODE_TENFIVE_XY,
               "sbod_codec_f32: bad arguments (op=%d)", op);
  SBOD_REQUIRE(priors || op <= SBOD_CODEC_CXCY_TO_XY, "sbod_codec_f32: op %d needs priors", op);
  if (n == 0) return SBOD_OK;
  int64_t blocks = (n + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(sbod::k_codec, dim3(blocks), dim3(256), 0, sbod::as_stream(stream), op, in,
                     priors, n, prior_rows, var0, var1, out);
  SBOD_LAUNCHED("k_codec");
  return SBOD_OK;
}
