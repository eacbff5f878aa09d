"""bench.py's N > 1 line refuses ranks that share one GPU.

Two ranks started by hand with LOCAL_RANK 0 both bind GPU 0 of this 1-GPU box:
every rank names its GPU (PCI bus id), sees the duplicate, and the job ends
non-zero within seconds with a message naming the ranks and the GPU — before
RCCL, which would otherwise hang on two ranks of one device.  A LOCAL_RANK past
the visible GPUs ends the same way.  PSG_BENCH_SHARE_GPU=1 (the shared-GPU test
mode) is the one way to run ranks on one GPU.
"""
import os
import socket
import subprocess
import sys
import tempfile
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(world, local_ranks, extra_env=None):
    port = _port()
    procs = []
    with tempfile.TemporaryDirectory() as d:
        for r in range(world):
            env = dict(os.environ, WORLD_SIZE=str(world), RANK=str(r), LOCAL_RANK=str(local_ranks[r]),
                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                       PSG_RDZV_FILE=os.path.join(d, "rdzv"), **(extra_env or {}))
            env.pop("PSG_BENCH_SHARE_GPU", None)
            procs.append(subprocess.Popen([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world),
                                           "--steps", "2", "--warmup", "1", "--no-cpu-baseline",
                                           "--no-probe256", "--keys", str(1 << 20)],
                                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
        t0 = time.time()
        outs = []
        for p in procs:
            try:
                o, e = p.communicate(timeout=max(1.0, 90 - (time.time() - t0)))
            except subprocess.TimeoutExpired:
                p.kill()  # a rank left waiting for a peer that already exited
                o, e = p.communicate()
            outs.append((p.returncode, o, e))
        return outs, time.time() - t0


def test_two_ranks_on_one_gpu_are_refused():
    outs, secs = _launch(2, [0, 0])
    for rc, o, e in outs:
        assert rc != 0, (o, e)
        assert "one GPU per rank is required" in e and "ranks [0, 1]" in e, e[-2000:]
        assert not [l for l in o.splitlines() if l.startswith("{")], "a bench line was printed"
    assert secs < 60, secs


def test_local_rank_past_the_visible_gpus_is_refused():
    import psg
    n = psg.device_count()
    outs, secs = _launch(2, [0, n])
    rc, o, e = outs[1]
    assert rc != 0 and "GPU(s) visible" in e, e[-2000:]
    assert secs < 90, secs
