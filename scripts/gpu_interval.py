#!/usr/bin/env python3
"""The step's GPU-side interval with the host out of the way (diagnostic).

Every step stream first waits on an event recorded after a spin kernel on a gate stream; N steps
are then submitted through the bench's native submit (`submit_step_program`, the same launches
as `bench.py`'s timed loop) while the GPU spins, so when the gate opens the GPU runs the N queued
steps back to back, as fast as its queues and CUs allow.  interval = (T(N2) - T(N1)) / (N2 - N1)
with T = gate end -> last stream's end (HIP events), for both chains, the criterion chain alone
(GT-list matcher, match final, loss pass, loss finish) and the detect chain alone (prepare,
segment, merge).  If both ~ criterion + detect, the two chains contend for the same CUs; if
both ~ max of the two, one chain sets the step.

    python scripts/gpu_interval.py [--n1 10] [--n2 40] [--reps 3] [--crit-streams 2] [--det-streams 2]
                                   [--batches 6] [--det-form two|one] [--finish separate|fused]
                                   [--crit-cu-reserve K [--mask spread|block]] [--shared-streams]
                                   [--detect-offset K]   (step k's detect on batch k + K)
                                   [--null-kernels N [--null-blocks M]]   (N empty kernels per step stream)
                                   (GPU_MAX_HW_QUEUES from the environment)
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from shape_based_object_detection_amd import _lib as L  # noqa: E402


def arg(name, default):
    return type(default)(sys.argv[sys.argv.index(name) + 1]) if name in sys.argv else default


def main():
    n1, n2, reps = arg('--n1', 10), arg('--n2', 40), arg('--reps', 3)
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    L.lib()
    st = bench.Step(dev, 32, 0, 1, graph=True, priority='detect', n_batches=arg('--batches', 6),
                    crit_streams=arg('--crit-streams', 2), det_streams=arg('--det-streams', 2),
                    det_form=arg('--det-form', 'two'), finish=arg('--finish', 'separate'))
    reserve = arg('--crit-cu-reserve', 0)
    if reserve > 0:
        # criterion streams on a CU-masked queue that leaves `reserve` CUs to the detect chain
        # (hipExtStreamCreateWithCUMask; the detect streams keep every CU and their priority)
        import ctypes
        hip = ctypes.CDLL('libamdhip64.so')
        ncu = torch.cuda.get_device_properties(dev).multi_processor_count
        pattern = arg('--mask', 'spread')
        off = set(range(ncu - reserve, ncu)) if pattern == 'block' else \
            {i for i in range(ncu) if i % (ncu // reserve) == ncu // reserve - 1}
        words = (ncu + 31) // 32
        mask = (ctypes.c_uint32 * words)()
        for i in range(ncu):
            if i not in off:
                mask[i // 32] |= 1 << (i % 32)
        streams_new = []
        for _ in st.cap_streams:
            h = ctypes.c_void_p()
            rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(h), ctypes.c_uint32(words), mask)
            if rc != 0:
                raise RuntimeError('hipExtStreamCreateWithCUMask: %d' % rc)
            streams_new.append(torch.cuda.ExternalStream(h.value, device=dev))
        st.cap_streams = streams_new
        st.cap_stream = streams_new[0]
    if '--shared-streams' in sys.argv:
        # each step's criterion and detect on ONE stream (the criterion's), steps over the streams
        st.det_streams = st.cap_streams
        st.det_stream = st.cap_stream
    for _ in range(4):
        st.eager_split()
    torch.cuda.synchronize()
    st.capture()
    if any(p is None for p in st.programs):
        raise RuntimeError('native step programs unavailable')
    for _ in range(2 * len(st.slots)):
        st.replay()
    torch.cuda.synchronize()
    gate = torch.cuda.Stream(dev)
    streams = st.cap_streams + st.det_streams

    # spin-kernel calibration: cycles per ms
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    with torch.cuda.stream(gate):
        e0.record(gate)
        torch.cuda._sleep(1_000_000)
        e1.record(gate)
    torch.cuda.synchronize()
    per_ms = 1_000_000 / max(e0.elapsed_time(e1), 1e-3)

    doff = arg('--detect-offset', 0)   # > 0: each step's detect reads another resident batch
    nnull, nblocks = arg('--null-kernels', 0), arg('--null-blocks', 1)

    def timed(n, parts, gate_ms):
        ev = torch.cuda.Event(enable_timing=True)
        with torch.cuda.stream(gate):
            torch.cuda._sleep(int(gate_ms * per_ms))
            ev.record(gate)
        for s in streams:
            s.wait_event(ev)
        t0 = time.perf_counter()
        for _ in range(n):
            i = st.k % len(st.slots)
            bt = st._next_batch()
            if doff and parts == 3:   # the criterion on batch i, the detect on batch i + doff
                r = L.host_ext.submit_step_program(st.programs[i], bt.boxes, bt.labels, 1)
                if r is True:
                    j = (i + doff) % len(st.slots)
                    r = L.host_ext.submit_step_program(st.programs[j], st.batches[j].boxes, st.batches[j].labels, 2)
            else:
                r = L.host_ext.submit_step_program(st.programs[i], bt.boxes, bt.labels, parts)
            if r is not True:
                raise RuntimeError('submit failed: %r' % (r,))
            for _ in range(nnull):   # empty kernels on the step's two streams (dispatch-floor probe)
                for sx in (st.cs_of(i), st.ds_of(i)):
                    if L.call('sbod_null_kernel', nblocks, sx.cuda_stream) != 0:
                        raise RuntimeError('sbod_null_kernel failed')
        host_ms = (time.perf_counter() - t0) * 1e3
        ends = []
        for s in streams:
            e = torch.cuda.Event(enable_timing=True)
            e.record(s)
            ends.append(e)
        torch.cuda.synchronize()
        gpu_ms = max(ev.elapsed_time(e) for e in ends)
        return gpu_ms, host_ms

    out = {'n1': n1, 'n2': n2, 'spin_cycles_per_ms': round(per_ms), 'crit_streams': len(st.cap_streams),
           'batches': len(st.batches), 'hw_queues': os.environ.get('GPU_MAX_HW_QUEUES'),
           'det_streams': len(st.det_streams), 'det_form': arg('--det-form', 'two'),
           'finish': arg('--finish', 'separate'), 'crit_cu_reserve': arg('--crit-cu-reserve', 0),
           'mask': arg('--mask', 'spread'), 'shared_streams': '--shared-streams' in sys.argv,
           'detect_offset': arg('--detect-offset', 0), 'null_kernels': arg('--null-kernels', 0),
           'null_blocks': arg('--null-blocks', 1), 'modes': {}}
    names = {3: 'both', 1: 'criterion', 2: 'detect'}
    for rep in range(reps):
        for parts in (3, 1, 2):
            gate_ms = 0.2 + 0.06 * n2       # > the host's submit of n2 steps (≈ 25-30 us each)
            ta, ha = timed(n1, parts, gate_ms)
            tb, hb = timed(n2, parts, gate_ms)
            rec = {'rep': rep, 'T_n1_ms': round(ta, 4), 'T_n2_ms': round(tb, 4),
                   'interval_us': round((tb - ta) / (n2 - n1) * 1e3, 2),
                   'host_submit_ms_n2': round(hb, 3), 'gate_ms': gate_ms,
                   'gated': hb < 0.9 * gate_ms}
            out['modes'].setdefault(names[parts], []).append(rec)
            print(json.dumps(dict(mode=names[parts], **rec)), flush=True)
    summ = {m: sorted(r['interval_us'] for r in v) for m, v in out['modes'].items()}
    print(json.dumps({'summary_interval_us': summ, 'crit_streams': out['crit_streams'],
                      'det_streams': out['det_streams'], 'batches': out['batches'],
                      'hw_queues': out['hw_queues'], 'det_form': out['det_form'],
                      'finish': out['finish'], 'crit_cu_reserve': out['crit_cu_reserve'],
                      'mask': out['mask'], 'shared_streams': out['shared_streams'],
                      'detect_offset': out['detect_offset'], 'null_kernels': out['null_kernels'],
                      'null_blocks': out['null_blocks']}), flush=True)


if __name__ == '__main__':
    main()
