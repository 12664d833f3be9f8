"""Host time of the pieces of core.detect's launch path (GPU busy with a criterion pass first,
so a blocking call shows up as a long piece)."""
import json, os, sys, time
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from shape_based_object_detection_amd import _lib as L, core  # noqa: E402
from shape_based_object_detection_amd.models import criteria as CR  # noqa: E402
from shape_based_object_detection_amd.models.priors import prior_table  # noqa: E402
dev = torch.device('cuda')
Pn = prior_table('SSD512'); P = Pn.shape[0]
pri = torch.from_numpy(Pn).to(dev)
cfg = bench.Cfg(reg_weights=1.0, device=dev, n_classes=21, reg_loss='diou', cls_loss='focal')
crit = CR.MultiBoxLoss512(priors_cxcy=pri, config=cfg)
boxes, labels, locs0, scores0, det = bench.make_batch(32, 0, dev)
locs = locs0.clone().requires_grad_(True); scores = scores0.clone().requires_grad_(True)
B, C, top_k = 32, 21, 200
res = {k: [] for k in ('alloc', 'ws', 'call', 'copy_rec', 'unbind', 'crit')}
for it in range(120):
    t = [time.perf_counter()]
    loss = crit(locs, scores, boxes, labels)          # GPU busy
    t.append(time.perf_counter())
    out_b = torch.empty(B, top_k, 4, device=dev); out_l = torch.empty(B, top_k, dtype=torch.int64, device=dev)
    out_s = torch.empty(B, top_k, device=dev); cnt = torch.empty(B, dtype=torch.int32, device=dev)
    t.append(time.perf_counter())
    nb = L.lib().sbod_detect_workspace_bytes(B, P, C); ws = core.workspace(nb, dev, 'detect')
    t.append(time.perf_counter())
    L.call('sbod_detect_f32', L.ptr(locs), L.ptr(det), B, P, C, L.ptr(pri), None, 0, 0, 0.01, 0.45, top_k, -1.0,
           0, 0, L.ptr(out_b), L.ptr(out_l), L.ptr(out_s), L.ptr(cnt), None, None, None, L.ptr(ws), nb, L.stream_of(det))
    t.append(time.perf_counter())
    ch, ev = core._count_slot(dev, B)
    ch.copy_(cnt, non_blocking=True); ev.record()
    t.append(time.perf_counter())
    full = (list(out_b.unbind(0)), list(out_l.unbind(0)), list(out_s.unbind(0)))
    t.append(time.perf_counter())
    ev.synchronize(); core._COUNT_SLOTS.setdefault((dev, B), []).append((ch, ev))
    loss.backward()
    torch.cuda.synchronize()
    if it >= 20:
        for k, (a, b) in zip(('crit', 'alloc', 'ws', 'call', 'copy_rec', 'unbind'), zip(t[:-1], t[1:])):
            res[k].append(b - a)
print(json.dumps({k: round(sorted(v)[len(v) // 2] * 1e6, 1) for k, v in res.items()}))
