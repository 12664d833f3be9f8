"""One process per GPU, started by the program itself (no torchrun needed).

``spawn_ranks(n, argv)`` starts ``n`` fresh Python processes running ``argv`` with the
torch.distributed environment of a single-node job (RANK, LOCAL_RANK, WORLD_SIZE,
LOCAL_WORLD_SIZE, MASTER_ADDR=127.0.0.1, MASTER_PORT) and waits for them.  The caller must not
have touched the GPU: the children are separate processes (subprocess, never exec), and each one
initialises its own device.  If any rank fails, the others are terminated and the worst exit
status is returned.
"""
import os
import socket
import subprocess
import sys
import time


def free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def rank_env(rank, world, port, base=None):
    env = dict(os.environ if base is None else base)
    env.update({'RANK': str(rank), 'LOCAL_RANK': str(rank), 'WORLD_SIZE': str(world),
                'LOCAL_WORLD_SIZE': str(world), 'GROUP_RANK': '0', 'MASTER_ADDR': '127.0.0.1',
                'MASTER_PORT': str(port)})
    return env


def spawn_ranks(n, argv, poll_s=0.05):
    """Run ``[sys.executable] + argv`` as ``n`` ranks; returns the job's exit status."""
    port = free_port()
    procs = [subprocess.Popen([sys.executable] + list(argv), env=rank_env(r, n, port))
             for r in range(n)]
    status = 0
    try:
        live = list(procs)
        while live:
            for p in list(live):
                rc = p.poll()
                if rc is None:
                    continue
                live.remove(p)
                if rc != 0:
                    status = status or rc
                    for q in live:     # one rank failed: the job cannot complete
                        q.terminate()
            time.sleep(poll_s)
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
            p.wait()
    for p in procs:
        if p.returncode not in (0, None) and not status:
            status = p.returncode
    return status
