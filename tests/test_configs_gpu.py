"""BASELINE.json configs[2..4] at their own sizes on the one MI355X a test box has.

  configs[2]  ns = nw = 8, 256 M floats per worker: bench.py's N > 1 job with 8
              rank processes sharing the GPU (PSG_BENCH_SHARE_GPU=1 — the one-shot
              xGMI exchange kernels over hipIpc-mapped peers; RCCL refuses two
              ranks on one GPU), every rank's WHOLE pulled vector checked.
  configs[3]  LR-like keyed BSP: 10 M sorted uint64 keys, nw = ns = 4 SORTED
              shards, through psg_slice (DefaultSlicer, KVApp.h:515-574),
              psg_store_handle (KVServerDefaultHandle, KVApp.h:433-458) and
              psg_merge (the pull merge, KVApp.h:680-720), against the oracle
              doing the same on std::unordered_map.
  configs[4]  1 G fp16 dense values (one GPU holds a whole 8-shard job's model),
              Push / Pull with an integer-valued closed form.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import oracle
import psg

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module", autouse=True)
def device():
    assert psg.device_count() >= 1, "no GPU visible"
    psg.set_device(0)
    yield


def test_configs2_n8_256m_per_worker_shared_gpu():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, PSG_BENCH_SHARE_GPU="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "8",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", "8", "--keys", str(256 << 20),
           "--steps", "3", "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    assert res["n_gpus"] == 8 and res["config"]["keys_per_worker"] == 256 << 20
    assert res["config"]["shard_keys"] == 32 << 20
    assert res["parity_check"] is True, res
    assert res["config"].get("xgmi_checksum_verified") is True, res
    # the bench process bootstraps without torch: HIP / RCCL are /opt/rocm's
    libs = res["runtime_libs"]
    assert "libamdhip64" in libs and "torch" not in libs["libamdhip64"], libs


def test_configs4_f16_1g_dense():
    import argparse
    import bench
    args = argparse.Namespace(keys=1 << 30, seed=7, warmup=1, steps=3, check=1, event_every=1,
                              no_cpu_baseline=True, no_probe256=True, workload="dense-f16")
    res = bench.run(bench.GpuBackend(0, 1, 0, None, "f16"), args, 0, 1)
    assert res["parity_check"] is True, res
    assert res["parity_detail"]["device_mismatches"] == 0 and res["parity_detail"]["elements"] == 1 << 30
    assert res["dtype"] == "f16" and res["config"]["workload"].startswith("configs[4]")


def test_configs3_keyed_10m_ns4_vs_oracle():
    n, ns, nw, steps = 10_000_000, 4, 4, 2
    rng = np.random.default_rng(9)
    keys = np.unique(rng.integers(0, (1 << 64) - 1, int(n * 1.01) + 1024, dtype=np.uint64))
    keys = np.sort(rng.choice(keys, n, replace=False))
    vals = [oracle.synth(n, oracle.F32, 100 + w, 1, -1.0, 1.0) for w in range(nw)]
    begins, ends = psg.server_ranges(ns)
    st = psg.Stream()
    dk = psg.DeviceBuffer.from_numpy(keys)
    dv = [psg.DeviceBuffer.from_numpy(v) for v in vals]
    kp, _ = psg.slice_keys(dk, n, begins, ends, stream=st)
    okp = oracle.slice_keys(keys, *oracle.server_ranges(ns))
    assert okp is not None and np.array_equal(kp, okp[0])
    stores = [psg.Store(psg.SORTED, psg.F32, int(begins[s]), int(ends[s]), 0) for s in range(ns)]
    ostores = [oracle.Store(oracle.F32) for _ in range(ns)]
    for _ in range(steps):
        for w in range(nw):  # BSP: every worker's Push of the same key set, in worker order
            for s in range(ns):
                a, b = int(kp[s]), int(kp[s + 1])
                stores[s].handle(psg.PUSH, dk.ptr + 8 * a, dv[w].ptr + 4 * a, None, b - a, stream=st)
                ostores[s].handle(oracle.PUSH, keys[a:b], vals[w][a:b], b - a)
    outs, osegs = [], []
    for s in range(ns):
        a, b = int(kp[s]), int(kp[s + 1])
        o = psg.DeviceBuffer(max(b - a, 1) * 4)
        stores[s].handle(psg.PULL, dk.ptr + 8 * a, None, o, b - a, stream=st)
        outs.append((o, b - a, int(keys[a])))
        osegs.append((ostores[s].handle(oracle.PULL, keys[a:b], None, b - a), int(keys[a])))
    merged = psg.DeviceBuffer(n * 4)
    psg.merge(list(reversed(outs)), 4, merged, n, stream=st)  # replies in any order
    got = merged.download(np.float32, n, st)
    exp = oracle.merge(list(reversed(osegs)), n)
    assert np.array_equal(got, exp)  # bit-exact: same adds in the same order per key
    for s in range(ns):
        k, v = stores[s].dump()
        ok, ov = ostores[s].dump()
        order = np.argsort(ok)
        assert np.array_equal(k, ok[order]) and np.array_equal(v, ov[order])


def _bench_shared(nranks, extra, env_extra, timeout=600):
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, PSG_BENCH_SHARE_GPU="1", **env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nranks),
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "bench.py"), "--gpus", str(nranks)] + extra
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])


def test_configs4_n8_f16_1g_double_buffered_shared_gpu():
    """configs[4]: 1 G fp16 values per worker, nw = ns = 8, the step
    double-buffered on two HIP streams (chunk c's Pull while chunk c+1's Push
    runs), every rank's whole pulled vector checked against the closed form."""
    res = _bench_shared(8, ["--workload", "dense-f16", "--steps", "2", "--warmup", "1"],
                        {"PSG_BENCH_EXCHANGE": "xgmi/4"})
    assert res["parity_check"] is True and res["dtype"] == "f16", res
    assert res["config"]["keys_per_worker"] == 1 << 30 and res["n_gpus"] == 8
    assert "double-buffered" in res["config"]["exchange"], res["config"]


def test_xgmi_double_buffered_ragged_chunks():
    """3 ranks, a block of 16,004 floats in 4 chunks of 4,004 / 4,004 / 4,004 / 3,992."""
    res = _bench_shared(3, ["--keys", str(3 * 16004), "--steps", "4", "--warmup", "2"],
                        {"PSG_BENCH_EXCHANGE": "xgmi/4"}, timeout=300)
    assert res["parity_check"] is True, res
    assert "double-buffered over 4 chunks" in res["config"]["exchange"]


@pytest.mark.parametrize("exchange", ["xgmi-keyed", "xgmi-keyed-w"])
def test_configs3_keyed_cached_n4_xgmi_shared_gpu(exchange):
    """configs[3] across ranks: nw = ns = 4, 10 M sorted uint64 keys, LR key
    caching — each shard resolves its psg_slice segment once, then Push / Pull
    run as the keyed xGMI kernels on the cached slots, the Pull as reads of the
    owners' stores or as writes into every rank's output (forced each way);
    every rank's whole pulled vector is checked against the closed form of the
    pushes."""
    res = _bench_shared(4, ["--workload", "keyed-cached", "--steps", "3", "--warmup", "1"],
                        {"PSG_BENCH_EXCHANGE": exchange})
    assert res["parity_check"] is True, res
    assert res["config"]["keys_per_worker"] == 10_000_000 and res["n_gpus"] == 4
    assert "keyed xGMI" in res["config"]["exchange"], res["config"]
    assert ("as writes" in res["config"]["exchange"]) == exchange.endswith("-w"), res["config"]


@pytest.mark.parametrize("n,mode,layout", [(1, "procs", 0), (2, "procs", 0), (4, "procs", 1), (8, "threads", 0),
                                           (8, "threads", 1)])
def test_dropin_bench_line(n, mode, layout):
    """bench.py --workload dropin: ZPush / ZPull through KVWorker / KVServer at
    ns = nw = n (every node on this box's one GPU), the reference's benchmark
    key layout (0) or one shared list (1); every worker's whole pulled vector
    is checked against the closed form of its pushes (parity_check)."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "dropin", "--gpus", str(n),
                        "--dropin-mode", mode, "--dropin-layout", str(layout), "--keys", "2000000", "--steps", "5",
                        "--warmup", "2", "--no-cpu-baseline"], capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["parity_check"], line
    assert line["value"] > 0 and line["roofline"]["frac"] > 0
    assert line["config"]["servers"] == n and line["config"]["workers"] == n


@pytest.mark.parametrize("env_extra,coded", [({"PSG_BENCH_SUBSET": "0.9"}, True), ({"PSG_BENCH_STRETCHES": "16"}, True),
                                             ({"PSG_RA_IDENT": "0"}, True), ({"PSG_BENCH_STORE_EXTRA": "1"}, True),
                                             ({"PSG_BENCH_STORE_EXTRA": "2"}, False)])
def test_keyed_bench_line_store_layouts(env_extra, coded):
    """bench.py --workload keyed on the store layouts DESIGN §5.1 quotes: a random
    90 % subset of the store, a union of 16 stretches, the general path on the
    store's own list, every other / every third store key.  Parity holds (the
    pulled vector on the device, an oracle sample), the coded validation ran
    where the tiles are 1024-thread ones — at least every other store key —
    (psg_store_counters), and the roofline names the kernels that ran."""
    env = dict(os.environ, **env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--workload", "keyed", "--keys", "2000000",
                        "--steps", "6", "--warmup", "3", "--no-cpu-baseline", "--no-probe256"],
                       capture_output=True, text=True, timeout=400, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["parity_check"], line
    paths = line["keyed_paths"]
    assert (paths["coded"] > 0) == coded, paths
    kernel = line["roofline"]["kernel"]
    assert ("k_validate_code" in kernel) == coded, kernel
    # f32 Pushes of coded lists go to the lean apply (k_tile_apply) — except
    # where the general tiles keep sending them back (the store's own list
    # under PSG_RA_IDENT=0 has none: lean too)
    if coded:
        assert paths["lean"] > 0 and "k_tile_apply" in kernel, (paths, kernel)
