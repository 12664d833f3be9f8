// Ground-truth packing: the collate_fn list-of-tensors batch
// (dataset/Datasets.py:58-86; the training loop moves each image's boxes/labels to the device,
// train_anchor.py:266-268) packed into the ragged device layout every other entry point reads:
// gt_boxes [sum G, 4] f32, gt_labels [sum G] int64, gt_offsets [B + 1] int32.
//
// The reference zero-fills per-step tensors and indexes them per image in a Python loop
// (models/SSD512.py:525-572).  Here one launch copies every image's rows: the per-image source
// pointers and the offsets travel in the kernel arguments (no pointer table in device memory, no
// host->device copy), so the packing is a single dispatch whose destination can be a
// fixed-capacity buffer that a captured hipGraph reads.
//
// Roofline: HBM-bound, 24 B per object in + 24 B out (tiny: < 30 KB at VOC sizes) — the launch
// is latency.  One workgroup per image.
#include "sbod_common.h"

namespace sbod {

SBOD_STAMP_DECL

__global__ __launch_bounds__(64) void k_gt_pack(GtPackArgs a, int n_img, int last_chunk,
                                                float *__restrict__ out_boxes,
                                                int64_t *__restrict__ out_labels,
                                                int32_t *__restrict__ out_off) {
  STAMP_BEGIN();
  const int i = blockIdx.x;
  const int r0 = a.off[i], G = a.off[i + 1] - r0;
  const float4 *src = reinterpret_cast<const float4 *>(a.boxes[i]);
  float4 *dst = reinterpret_cast<float4 *>(out_boxes) + r0;
  const bool aligned = (reinterpret_cast<uintptr_t>(a.boxes[i]) & 15) == 0;
  for (int g = threadIdx.x; g < G; g += blockDim.x) {
    if (aligned) {
      dst[g] = src[g];
    } else {
      const float *s = a.boxes[i] + 4 * g;
      dst[g] = make_float4(s[0], s[1], s[2], s[3]);
    }
    out_labels[r0 + g] = a.labels[i][g];
  }
  if (threadIdx.x == 0) {
    out_off[i] = r0;
    if (last_chunk && i == n_img - 1) out_off[n_img] = r0 + G;
  }
  STAMP_END(8, 1);
}

}  // namespace sbod

using namespace sbod;

extern "C" int sbod_gt_pack(const void *const *box_ptrs, const void *const *label_ptrs,
                            const int32_t *counts, int B, int64_t capacity, float *gt_boxes,
                            int64_t *gt_labels, int32_t *gt_offsets, void *stream) {
  SBOD_REQUIRE(B > 0 && box_ptrs && label_ptrs && counts && gt_boxes && gt_labels && gt_offsets,
               "sbod_gt_pack: bad arguments (B=%d)", B);
  int64_t total = 0;
  for (int i = 0; i < B; ++i) {
    SBOD_REQUIRE(counts[i] >= 0, "sbod_gt_pack: image %d has a negative object count", i);
    SBOD_REQUIRE(counts[i] == 0 || (box_ptrs[i] && label_ptrs[i]), "sbod_gt_pack: image %d: null rows", i);
    total += counts[i];
  }
  SBOD_REQUIRE(total <= capacity, "sbod_gt_pack: %lld objects exceed the capacity %lld",
               static_cast<long long>(total), static_cast<long long>(capacity));
  SBOD_REQUIRE(total < (int64_t(1) << 31), "sbod_gt_pack: too many objects");
  hipStream_t s = as_stream(stream);
  int32_t row = 0;
  for (int c0 = 0; c0 < B; c0 += kPackImgs) {
    const int n = B - c0 < kPackImgs ? B - c0 : kPackImgs;
    GtPackArgs a;
    for (int i = 0; i < n; ++i) {
      a.boxes[i] = static_cast<const float *>(box_ptrs[c0 + i]);
      a.labels[i] = static_cast<const int64_t *>(label_ptrs[c0 + i]);
      a.off[i] = row;
      row += counts[c0 + i];
    }
    a.off[n] = row;
    hipLaunchKernelGGL(k_gt_pack, dim3(n), dim3(64), 0, s, a, n, c0 + n == B ? 1 : 0, gt_boxes,
                       gt_labels, gt_offsets + c0);
    SBOD_LAUNCHED("k_gt_pack");
  }
  return SBOD_OK;
}

SBOD_STAMP_EXPORT(gtpack)
