"""bench.py's multi-GPU launch (one process per GPU, started before any GPU call) on CPU: a stub
worker joins a gloo group through the environment the launcher sets; N ranks must start, see the
same world, and only rank 0 prints the result line.  Also: bench.py refuses a --gpus that does
not match the WORLD_SIZE it runs under (no silent single-rank run)."""
import json
import os
import subprocess
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STUB = r'''
import json, os, sys
import torch, torch.distributed as dist
dist.init_process_group('gloo')
r, w = dist.get_rank(), dist.get_world_size()
assert r == int(os.environ['RANK']) == int(os.environ['LOCAL_RANK'])
assert os.environ['MASTER_ADDR'] == '127.0.0.1'
t = torch.tensor([1.0])
dist.all_reduce(t)
if r == 0:
    print(json.dumps({'world': w, 'sum': t.item(), 'argv': sys.argv[1:]}), flush=True)
dist.destroy_process_group()
'''

FAIL_STUB = r'''
import os, sys, time
if os.environ['RANK'] == '1':
    sys.exit(3)
time.sleep(60)
'''


def _run_launcher(tmp_path, stub, n, extra=()):
    script = tmp_path / 'stub.py'
    script.write_text(stub)
    code = ('import sys; sys.path.insert(0, %r)\n'
            'from shape_based_object_detection_amd.launch import spawn_ranks\n'
            'sys.exit(spawn_ranks(%d, [%r] + %r))\n' % (REPO, n, str(script), list(extra)))
    env = dict(os.environ)
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT'):
        env.pop(k, None)
    return subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=120,
                          env=env)


@pytest.mark.parametrize('n', [2, 3])
def test_spawn_ranks_starts_n_ranks_rank0_prints(tmp_path, n):
    r = _run_launcher(tmp_path, STUB, n, extra=('--steps', '5'))
    assert r.returncode == 0, r.stderr
    # gloo itself logs connection lines; the result lines are the JSON ones
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, r.stdout        # rank 0 alone prints
    d = json.loads(lines[0])
    assert d['world'] == n and d['sum'] == float(n) and d['argv'] == ['--steps', '5']


def test_spawn_ranks_propagates_failure(tmp_path):
    r = _run_launcher(tmp_path, FAIL_STUB, 2)
    assert r.returncode == 3


def test_bench_refuses_mismatched_world():
    env = dict(os.environ, WORLD_SIZE='1', RANK='0', LOCAL_RANK='0')
    r = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', '2'],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0
    assert '--gpus 2 but WORLD_SIZE=1' in r.stderr
