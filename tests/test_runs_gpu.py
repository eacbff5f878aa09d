"""Runs of queued Pushes through the C++ API (KVServer::OnReceive drains the
Pushes queued behind the one it takes; KVServerDefaultHandle::PushRun serves
them with psg_store_push_frames / psg_store_push_slots_frames).

nw workers push ONE key list with their own real-valued frames
(tests/harness/kv_runs_device.cpp).  The servers trace every request in the
order they handled it (PS_TRACE_REQUESTS); the test replays that order
through the oracle — the reference handle's `store[key] += vals[i]` per
request (src/ps/KVApp.h:446-454), one request after the other as its
Customer thread takes them (src/internal/Customer.cpp:52-70) — and compares
worker 0's final Pull bit for bit.  Real-valued frames make the order of
additions visible in the low bits, so a run applied out of arrival order
would fail.  The servers' store counters show the runs served in one pass.
"""
import json
import os
import subprocess

import numpy as np
import pytest

import oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "tests", "_bin")
KMAX = (1 << 64) - 1


def replay(trace_lines, num, nw, ns):
    """The oracle's store after the traced requests, in the traced order."""
    keys = np.arange(num, dtype=np.uint64) * np.uint64(KMAX // num)
    vals = {w: oracle.synth(num, oracle.F32, 7 + w, 1, -1.0, 1.0) for w in range(nw)}
    begins, ends = oracle.server_ranges(ns)
    kp, _ = oracle.slice_keys(keys, begins, ends)
    orc = oracle.Store(oracle.F32)
    for line in trace_lines:
        server, sender, _ts, push, pull, _n, _rs, _rp = map(int, line.split())
        s = (server - 8) // 2
        w = (sender - 9) // 2
        lo, hi = int(kp[s]), int(kp[s + 1])
        if push:
            orc.handle(oracle.PUSH | (oracle.PULL if pull else 0), keys[lo:hi], vals[w][lo:hi], hi - lo)
        elif pull:
            orc.handle(oracle.PULL, keys[lo:hi], None, hi - lo)
    k, v = orc.dump()
    assert np.array_equal(k, keys)
    return v


def replay_layout0(trace_lines, num, nw, ns):
    """The reference benchmark's layout (worker w sends kMaxKey / num * i + w,
    tests/test_kv_app_benchmark.cpp:47-52): the traced requests replayed in
    order through the oracle.  Returns the oracle store and every Pull's reply
    by (sender node, timestamp, server)."""
    step = np.uint64(KMAX // num)
    keys = {w: np.arange(num, dtype=np.uint64) * step + np.uint64(w) for w in range(nw)}
    vals = {w: oracle.synth(num, oracle.F32, 7 + w, 1, -1.0, 1.0) for w in range(nw)}
    begins, ends = oracle.server_ranges(ns)
    kp = {w: oracle.slice_keys(keys[w], begins, ends)[0] for w in range(nw)}
    orc = oracle.Store(oracle.F32)
    replies = {}
    for line in trace_lines:
        server, sender, ts, push, pull, n, _rs, _rp = map(int, line.split())
        s = (server - 8) // 2
        w = (sender - 9) // 2
        lo, hi = int(kp[w][s]), int(kp[w][s + 1])
        assert n == hi - lo, line
        flags = (oracle.PUSH if push else 0) | (oracle.PULL if pull else 0)
        out = orc.handle(flags, keys[w][lo:hi], vals[w][lo:hi] if push else None, hi - lo)
        if pull:
            replies[(sender, ts, s)] = out
    return orc, keys, replies


def run_job(tmp_path, ns, nw, num, repeat, key_cache=0, procs=False, env=None, layout=1, pull_each=0):
    exe = os.path.join(BIN, "kv_runs_device")
    if not os.path.exists(exe):
        pytest.skip(f"{exe} not built")
    trace = tmp_path / "trace.txt"
    out = tmp_path / "pulled.f32"
    e = dict(os.environ, PS_TRACE_REQUESTS=str(trace), PS_RUNS_OUT=str(out), **(env or {}))
    args = [exe, "-ns", str(ns), "-nw", str(nw)] + (["-procs"] if procs else []) + [
        str(num), str(repeat), str(key_cache), str(layout), str(pull_each)]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300, env=e)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    workers = [l for l in lines if "rank" in l]
    servers = [l for l in lines if "server" in l]
    assert len(workers) == nw and len(servers) == ns, r.stdout
    tl = [l for l in trace.read_text().splitlines() if l.strip()]
    got = np.fromfile(out, dtype=np.float32) if layout == 1 else None
    return workers, servers, tl, got


@pytest.mark.parametrize("ns,nw,procs", [(1, 4, False), (1, 8, False), (1, 4, True), (1, 8, True),
                                         (2, 4, False)])
def test_runs_of_pushes_match_the_arrival_order(tmp_path, ns, nw, procs):
    num, repeat = 300000, 12
    workers, servers, tl, got = run_job(tmp_path, ns, nw, num, repeat, procs=procs)
    pushes = [l for l in tl if l.split()[3] == "1"]
    assert len(pushes) == ns * nw * (repeat + 1)
    exp = replay(tl, num, nw, ns)
    np.testing.assert_array_equal(got, exp)
    runs = sum(s["runs"] for s in servers)
    in_runs = sum(int(l.split()[6]) > 1 for l in pushes)
    # the runs served in one pass are traced runs (the first, inserting Pushes
    # of a job may form a run that is served request by request)
    assert 0 < sum(s["run_frames"] for s in servers) <= in_runs, (servers, in_runs)
    assert runs > 0, "no run formed: every Push found an empty queue"


@pytest.mark.parametrize("procs", [False, True])
def test_runs_of_cached_pushes_match_the_arrival_order(tmp_path, procs):
    """LR key caching: the timed Pushes name the list by its hash, and a run of
    them is one pass over the cached stretch of slots."""
    num, nw, repeat = 300000, 6, 12
    workers, servers, tl, got = run_job(tmp_path, 1, nw, num, repeat, key_cache=1, procs=procs)
    exp = replay(tl, num, nw, 1)
    np.testing.assert_array_equal(got, exp)
    assert servers[0]["runs"] > 0


def test_runs_off_is_the_same_store(tmp_path):
    """PS_PUSH_RUNS=0: every Push handled on its own; the arrival order is
    replayed the same way and no run is formed."""
    workers, servers, tl, got = run_job(tmp_path, 1, 4, 200000, 8, env={"PS_PUSH_RUNS": "0"})
    np.testing.assert_array_equal(got, replay(tl, 200000, 4, 1))
    assert servers[0]["runs"] == 0
    assert all(l.split()[6] == "1" for l in tl)


@pytest.mark.parametrize("ns,nw,procs", [(1, 4, False), (1, 8, False), (2, 4, False), (2, 8, False),
                                         (1, 4, True), (1, 8, True), (2, 4, True), (2, 8, True)])
def test_strided_runs_match_the_arrival_order(tmp_path, ns, nw, procs):
    """The reference benchmark's own key layout, kMaxKey / num * i + rank
    (tests/test_kv_app_benchmark.cpp:47-52), with its step — a Push then a
    Pull, each waited for — on real-valued frames.  Every server's store holds
    the nw lists interleaved; the requests of distinct workers queued at a
    server (Pushes and Pulls) are served as strided runs (psg_store_run).  The
    traced arrival order replayed through the oracle gives every worker's last
    timed Pull and its final Pull bit for bit, and the servers' counters show
    the strided runs."""
    num, repeat = 300000, 12
    workers, servers, tl, _ = run_job(tmp_path, ns, nw, num, repeat, procs=procs, layout=0, pull_each=1)
    assert len([l for l in tl if l.split()[3] == "1"]) == ns * nw * (repeat + 1)
    orc, keys, replies = replay_layout0(tl, num, nw, ns)
    out = tmp_path / "pulled.f32"
    for w in workers:
        r = w["rank"]
        final = np.fromfile(f"{out}.{r}", dtype=np.float32)
        np.testing.assert_array_equal(final, orc.handle(oracle.PULL, keys[r], None, num), err_msg=f"worker {r}")
        last = np.fromfile(f"{out}.{r}.last", dtype=np.float32)
        exp = np.concatenate([replies[(w["node"], w["last_pull_ts"], s)] for s in range(ns)
                              if (w["node"], w["last_pull_ts"], s) in replies])
        np.testing.assert_array_equal(last, exp, err_msg=f"worker {r}: last timed Pull")
    in_runs = sum(int(l.split()[6]) > 1 for l in tl)
    strided = sum(s["strided_frames"] for s in servers)
    assert 0 < strided <= in_runs, (servers, in_runs)
    assert sum(s["strided_runs"] for s in servers) > 0


def test_mixed_runs_off_is_the_same_store(tmp_path):
    """PS_MIXED_RUNS=0 PSG_RUNS_STRIDED=0: the same job request by request
    (runs of one shape may form, none strided): the same values."""
    num, nw = 200000, 4
    workers, servers, tl, _ = run_job(tmp_path, 1, nw, num, 6, layout=0, pull_each=1,
                                      env={"PS_MIXED_RUNS": "0", "PSG_RUNS_STRIDED": "0"})
    orc, keys, _ = replay_layout0(tl, num, nw, 1)
    for w in workers:
        final = np.fromfile(f"{tmp_path / 'pulled.f32'}.{w['rank']}", dtype=np.float32)
        np.testing.assert_array_equal(final, orc.handle(oracle.PULL, keys[w["rank"]], None, num))
    assert sum(s["strided_runs"] for s in servers) == 0
