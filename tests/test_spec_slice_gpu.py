"""Unconfirmed slices (PS_SPEC_SLICE=1; parameter-server_amd/ps/kv_app.h
KVWorker::Send / Refused, KVServerDefaultHandle::Run, psg_store_run_status).

A worker that sliced an HBM key list before sends it on the bounds it had then,
without the slicer's kernel and readback.  Every server checks each key of its
slice against its own range, so a wrong bound is refused by a server (nothing
of that slice applied) and the worker re-sends those keys sliced for real; a
slice a server accepts lies in its range, so every key is still applied once,
by its own server.  The reference slices every request on the host
(src/ps/KVApp.h:515-574); the results here are the reference's, bit for bit:

* tests/harness/kv_spec_slice_device.cpp rewrites its key list in place
  between requests so that the old bounds are wrong (a Push and a Pull are
  refused and re-sent) and every Pull matches the oracle's replay of the
  program order (one worker: each key's additions come in that order);
* the benchmark's step at ns = 2 (tests/test_runs_gpu.py's oracle replay of
  the servers' arrival order) with unconfirmed slices on.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import oracle
import psg

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "_bin")
KMAX = (1 << 64) - 1


def arith(n, first, stride):
    return (np.uint64(first) + np.arange(n, dtype=np.uint64) * np.uint64(stride)).astype(np.uint64)


def run_spec(tmp_path, ns, procs, spec, num=200000):
    exe = os.path.join(BIN, "kv_spec_slice_device")
    if not os.path.exists(exe):
        pytest.skip(f"{exe} not built")
    out = tmp_path / "pull"
    env = dict(os.environ, PS_SPEC_OUT=str(out), PS_SPEC_SLICE="1" if spec else "0")
    args = [exe, "-ns", str(ns), "-nw", "1"] + (["-procs"] if procs else []) + [str(num)]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    worker = [l for l in lines if "refused" in l]
    assert len(worker) == 1, r.stdout
    return worker[0], out


def expected(num):
    """The harness's sequence replayed through the oracle (KVApp.h:446-454)."""
    orc = oracle.Store(psg.F32)
    half = KMAX // 2
    pulls = {}

    def push(k, seed):
        orc.handle(oracle.PUSH, k, oracle.synth(num, psg.F32, seed, 1, -1.0, 1.0), num)

    def pull(k, tag):
        pulls[tag] = orc.handle(oracle.PULL, k, None, num)

    k0 = arith(num, 0, KMAX // num)
    push(k0, 7)
    pull(k0, "p0a")
    push(k0, 8)
    pull(k0, "p0")
    k1 = arith(num, 1, half // num)
    push(k1, 9)
    pull(k1, "p1")
    push(k1, 10)
    pull(k1, "p1b")
    k2 = arith(num, half + 5, half // num)
    pull(k2, "p2")
    push(k2, 11)
    pull(k2, "p2b")
    return pulls


@pytest.mark.parametrize("ns,procs,spec", [(2, False, True), (2, True, True), (4, False, True), (2, False, False)])
def test_rewritten_key_list_is_refused_and_resent(tmp_path, ns, procs, spec):
    num = 200000
    worker, out = run_spec(tmp_path, ns, procs, spec, num)
    exp = expected(num)
    for tag, want in exp.items():
        got = np.fromfile(f"{out}.{tag}", dtype=np.float32)
        np.testing.assert_array_equal(got, want, err_msg=tag)
    if spec:
        # the Push of K1 on K0's bounds and the Pull of K2 on K1's: refused by
        # the servers whose slices left their ranges, then re-sent
        assert worker["refused"] >= 2, worker
    else:
        assert worker["refused"] == 0, worker


@pytest.mark.parametrize("nw,procs", [(4, False), (4, True), (8, False)])
def test_strided_runs_with_unconfirmed_slices(tmp_path, nw, procs):
    """The benchmark's step at ns = 2 with PS_SPEC_SLICE=1: the arrival-order
    replay gives every worker's last timed Pull and final Pull bit for bit."""
    import test_runs_gpu as tr
    num, repeat, ns = 300000, 12, 2
    workers, servers, tl, _ = tr.run_job(tmp_path, ns, nw, num, repeat, procs=procs, layout=0, pull_each=1,
                                         env={"PS_SPEC_SLICE": "1"})
    orc, keys, replies = tr.replay_layout0(tl, num, nw, ns)
    out = tmp_path / "pulled.f32"
    for w in workers:
        r = w["rank"]
        final = np.fromfile(f"{out}.{r}", dtype=np.float32)
        np.testing.assert_array_equal(final, orc.handle(oracle.PULL, keys[r], None, num), err_msg=f"worker {r}")
        last = np.fromfile(f"{out}.{r}.last", dtype=np.float32)
        exp = np.concatenate([replies[(w["node"], w["last_pull_ts"], s)] for s in range(ns)
                              if (w["node"], w["last_pull_ts"], s) in replies])
        np.testing.assert_array_equal(last, exp, err_msg=f"worker {r}: last timed Pull")
    assert sum(s["strided_runs"] for s in servers) > 0
