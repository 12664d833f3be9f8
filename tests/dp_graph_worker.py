"""Rank worker for tests/test_gpu_dp_graph.py (not a test module): two ranks share cuda:0 over
gloo; each runs bench.Step's data-parallel criterion eagerly (the positive-count all-reduce
inside the criterion call) and then as the captured DPGraph (two graphs around an eager
all-reduce, the next step's matcher and all-reduce issued ahead of the current loss pass), on the
same batches over two rotations, and writes whether loss and gradients are bit-identical."""
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench as BM  # noqa: E402


def main():
    rank, world = int(os.environ['RANK']), int(os.environ['WORLD_SIZE'])
    dist.init_process_group('gloo')
    dev = torch.device('cuda', 0)
    torch.cuda.set_device(dev)
    st = BM.Step(dev, 4, rank, world, graph=True, n_batches=3)
    eager = []
    for i in range(len(st.batches)):
        loss, _ = st.eager()
        torch.cuda.synchronize()
        bt = st.batches[i]
        eager.append((loss.detach().clone(), bt.locs.grad.clone(), bt.scores.grad.clone()))
    # release the eager step's autograd graph before capturing: its AccumulateGrad nodes belong
    # to the default stream, and a capture that reuses them pulls that stream in (the runtime
    # then faults in hipStreamEndCapture)
    del loss
    torch.cuda.synchronize()
    st.capture()
    st.k = 0
    res = []
    # two rotations: from the second step on, each step's matcher and count all-reduce were
    # issued by the step before it (DPGraph.front ahead of the previous step's loss pass)
    for k in range(2 * len(st.batches)):
        i = k % len(st.batches)
        loss, _ = st.replay()
        torch.cuda.synchronize()
        bt = st.batches[i]
        e = eager[i]
        res.append({'loss_equal': bool(torch.equal(loss, e[0])), 'grad_locs_equal': bool(torch.equal(bt.locs.grad, e[1])),
                    'grad_scores_equal': bool(torch.equal(bt.scores.grad, e[2])), 'loss': float(loss)})
    with open(os.path.join(os.environ['SBOD_DP_OUT'], 'rank%d.json' % rank), 'w') as f:
        json.dump({'rank': rank, 'graph_type': type(st.slots[0][0]).__name__, 'batches': res}, f)
    dist.barrier()
    dist.destroy_process_group()


if __name__ == '__main__':
    main()
