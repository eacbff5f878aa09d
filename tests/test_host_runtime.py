"""The C++ host runtime (ps:: API, local Van, slicer, merge, barriers) on CPU.

tests/_bin/kv_cluster_host runs real KVWorker / KVServer nodes with a host
request handle (test code), so no GPU is needed.  The reference's own harnesses
compiled unmodified against the runtime live in tests/_dropin/ (built by
`make -C parameter-server_amd dropin` where the reference tree exists).
"""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "_bin")
DROPIN = os.path.join(ROOT, "tests", "_dropin")


def run(path, *args, timeout=120, env=None):
    e = dict(os.environ)
    if env:
        e.update(env)
    return subprocess.run([path, *map(str, args)], capture_output=True, text=True, timeout=timeout,
                          env=e)


def _need(path):
    if not os.path.exists(path):
        pytest.skip(f"{path} not built (make -C parameter-server_amd all)")


def test_svector_semantics():
    """SVector copy/share/Slice/detach/reinterpret semantics (SVector_test.cpp)."""
    exe = os.path.join(BIN, "svector_unit")
    _need(exe)
    r = run(exe)
    assert r.returncode == 0, r.stderr[-2000:]
    assert "svector ok" in r.stdout


@pytest.mark.parametrize("ns,nw", [(1, 1), (2, 1), (3, 2), (8, 4)])
def test_host_cluster(ns, nw):
    exe = os.path.join(BIN, "kv_cluster_host")
    _need(exe)
    r = run(exe, "-ns", ns, "-nw", nw)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count(" ok") == nw


def test_num_nodes_from_environment():
    exe = os.path.join(BIN, "kv_cluster_host")
    _need(exe)
    r = run(exe, env={"PS_NUM_SERVER": "2", "PS_NUM_WORKER": "3"})
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.count(" ok") == 3


def test_dropin_connection():
    """tests/test_connection.cpp of the reference, unmodified: Start / Finalize only."""
    exe = os.path.join(DROPIN, "test_connection")
    _need(exe)
    for ns, nw in [(1, 1), (2, 3)]:
        r = run(exe, "-ns", ns, "-nw", nw)
        assert r.returncode == 0, r.stderr[-2000:]


def _has_gpu():
    try:
        import psg
        return psg.device_count() > 0
    except Exception:
        return False


def test_default_handle_fails_loudly_without_gpu():
    """The HBM store has no CPU fallback: with no GPU the server's CHECK aborts the job."""
    exe = os.path.join(DROPIN, "test_kv_app")
    _need(exe)
    if _has_gpu():
        pytest.skip("a GPU is present")
    r = run(exe, "-ns", 1, "-nw", 1, timeout=60)
    assert r.returncode != 0
    assert "value store lives in HBM" in r.stderr
