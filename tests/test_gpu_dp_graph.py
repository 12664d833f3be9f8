"""The data-parallel step's captured criterion (bench.DPGraph: the matcher graph | an eager
positive-count all-reduce | the loss-pass graph) against the same criterion run
eagerly, two ranks sharing cuda:0 over gloo (RCCL refuses two ranks on one device): loss and both
gradients bit-identical on every batch, and the captured form is the split one."""
import json
import os

import pytest

from shape_based_object_detection_amd.launch import spawn_ranks

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_dp_split_graph_equals_eager(tmp_path):
    os.environ['SBOD_DP_OUT'] = str(tmp_path)
    try:
        rc = spawn_ranks(2, [os.path.join(HERE, 'dp_graph_worker.py')])
    finally:
        os.environ.pop('SBOD_DP_OUT', None)
    assert rc == 0, 'a rank failed (exit %s)' % rc
    for r in range(2):
        d = json.load(open(tmp_path / ('rank%d.json' % r)))
        assert d['graph_type'] == 'DPGraph'
        for b in d['batches']:
            assert b['loss_equal'] and b['grad_locs_equal'] and b['grad_scores_equal'], (r, b)
