"""Seeded synthetic workload recipe.

Every bench line and every parity test draws its inputs from here, so the GPU box, this
container and the golden-fixture generator see the same bytes for the same seed.  Only the
CPU ``torch.Generator`` is used (mt19937, identical across hosts for one torch version).

Recipe, per image ``i`` with seed ``s_i = seed + i``:
  * ``G ~ U{1..max_objects}``; ``xy ~ U(0, 0.7)^2``, ``wh ~ U(0.02, 0.32)^2`` → normalized xyxy;
    ``labels ~ U{1..n_classes-1}``.
  * Predictions from a generator seeded ``10000 + seed``: ``locs ~ N(0, 0.1^2)``,
    ``scores ~ N(0, 1)``; for detection workloads ``+6.0`` on the background logit
    (≈1,330 candidates per class and image above ``min_score = 0.01`` at SSD512 sizes).
"""
import torch


def make_gt(batch_size, seed=0, n_classes=21, max_objects=16):
    """Return ``(boxes, labels)``: lists of ``[G_i, 4]`` float32 xyxy and ``[G_i]`` int64 (CPU)."""
    boxes, labels = [], []
    for i in range(batch_size):
        g = torch.Generator().manual_seed(seed + i)
        n = int(torch.randint(1, max_objects + 1, (1,), generator=g).item())
        xy = torch.rand(n, 2, generator=g) * 0.7
        wh = torch.rand(n, 2, generator=g) * 0.30 + 0.02
        boxes.append(torch.cat([xy, xy + wh], dim=1).contiguous())
        labels.append(torch.randint(1, n_classes, (n,), generator=g, dtype=torch.int64))
    return boxes, labels


def make_preds(batch_size, n_priors, n_classes=21, seed=0, bg_shift=0.0):
    """Return ``(locs [B,P,4], scores [B,P,C])`` float32 on CPU."""
    g = torch.Generator().manual_seed(10000 + seed)
    locs = torch.randn(batch_size, n_priors, 4, generator=g) * 0.1
    scores = torch.randn(batch_size, n_priors, n_classes, generator=g)
    if bg_shift:
        scores[:, :, 0] += bg_shift
    return locs, scores
