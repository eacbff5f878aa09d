"""The N > 1 data path of bench.py, rehearsed on CPU with world_size 2 (gloo).

bench.run() is the same orchestration the GPU job runs (shards, warmup,
barriers, max-over-ranks timing, the JSON line); only the backend differs:
here a Push is torch.distributed.reduce_scatter_tensor + the shard accumulate
and a Pull is all_gather_into_tensor — the collective pattern psg_comm_push /
psg_comm_pull issue on RCCL.  The result is checked against the oracle
replaying every worker's Push as a separate KVServerDefaultHandle request, in
worker order, on real-valued data: the reduce-scatter sums in another order,
so the bar is the north star's 1e-6 relative tolerance (plus an absolute floor
for sums that cancel to ~0).
"""
import argparse
import json
import os
import socket
import sys
import tempfile

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REL_TOL = 1e-6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class CpuCollectiveBackend:
    """bench.py backend whose Push/Pull run the RS + accumulate / AG pattern on gloo."""

    def __init__(self, rank, world, dist):
        import torch
        self.torch, self.rank, self.world, self.dist = torch, rank, world, dist

    def describe(self):
        # the fields a GPU rank reports (bench.GpuBackend.describe): here the
        # CPU process, and the gloo group in place of RCCL
        import socket
        return {"rank": self.rank, "device": "cpu", "pci_bus_id": None, "host": socket.gethostname(),
                "rccl_rank": self.dist.get_rank(), "rccl_nranks": self.dist.get_world_size()}

    def setup(self, L, seed):
        import oracle
        self.L, self.blk = L, L // self.world
        self.vals = self.torch.from_numpy(oracle.synth(L, oracle.F32, seed + self.rank, 1, -1.0, 1.0))
        self.store = self.torch.zeros(self.blk, dtype=self.torch.float32)
        self.out = self.torch.zeros(L, dtype=self.torch.float32)
        self.pushes = 0

    def push(self):
        scratch = self.torch.zeros(self.blk, dtype=self.torch.float32)
        self.dist.reduce_scatter_tensor(scratch, self.vals)
        self.store += scratch
        self.pushes += 1

    def pull(self):
        self.dist.all_gather_into_tensor(self.out, self.store)

    def new_event(self):
        return [0.0]

    def record(self, e):
        import time
        e[0] = time.perf_counter()

    def elapsed(self, a, b):
        return (b[0] - a[0]) * 1e3

    def sync(self):
        pass

    def check(self, steps_done):
        import oracle
        self.pull()
        got = self.out.numpy()
        ok = True
        for r in range(self.world):
            st = oracle.Store(oracle.F32)
            lo = r * self.blk
            for _ in range(steps_done):
                for w in range(self.world):
                    v = oracle.synth(self.L, oracle.F32, self._seed + w, 1, -1.0, 1.0)[lo:lo + self.blk]
                    st.handle(oracle.PUSH, None, v, self.blk, first_key=lo)
            exp = st.handle(oracle.PULL, None, None, self.blk, first_key=lo)
            g = got[lo:lo + self.blk]
            ok &= bool(np.all(np.abs(g - exp) <= REL_TOL * np.abs(exp) + 1e-6 * steps_done * self.world))
        return ok


def _rank_main(rank, world, port, outdir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "parameter-server_amd", "python")]
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world, init_method=f"tcp://127.0.0.1:{port}")
    import bench
    from psg_group import SocketGroup
    # bench.py's own torch-free rendezvous orchestrates; gloo carries only this
    # backend's data (the collectives RCCL carries on the GPU)
    group = SocketGroup(rank, world, path=os.path.join(outdir, "rdzv"))
    args = argparse.Namespace(keys=12288, seed=7, warmup=1, steps=3, check=1, no_cpu_baseline=True)
    res = bench.run(CpuCollectiveBackend(rank, world, dist), args, rank, world, group)
    with open(os.path.join(outdir, f"r{rank}.json"), "w") as f:
        json.dump(res, f)
    group.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_bench_distributed_path_gloo(world):
    # torch is imported only inside the rank processes: a process that loaded
    # libpsgpu.so (HIP from /opt/rocm) must not load torch's HIP runtime after it
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as d:
        port = _free_port()
        procs = [ctx.Process(target=_rank_main, args=(r, world, port, d)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=120)
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        r0 = json.load(open(os.path.join(d, "r0.json")))
        for r in range(1, world):
            assert json.load(open(os.path.join(d, f"r{r}.json"))) is None  # only rank 0 prints
    assert r0["n_gpus"] == world and r0["scaling"] == "weak"
    assert r0["parity_check"] is True
    assert r0["config"]["shard_keys"] * world == r0["config"]["keys_per_worker"]
    # value = all workers' pushed + pulled floats / max-over-ranks time
    exp = 2 * 4 * r0["config"]["keys_per_worker"] * world / (r0["ms_per_step"] * 1e-3) / 1e9
    assert abs(r0["value"] - exp) <= 1e-3 * exp + 1e-3
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config"):
        assert k in r0
    # the N > 1 line names every rank's device, GPU and communicator view
    ranks = r0["config"]["ranks"]
    assert [d["rank"] for d in ranks] == list(range(world))
    for d in ranks:
        assert {"device", "pci_bus_id", "host", "rccl_rank", "rccl_nranks"} <= set(d)
        assert d["rccl_nranks"] == world and d["rccl_rank"] == d["rank"]
    assert "distinct_gpus" in r0["config"] and "calibration_ms" in r0["config"]


def _group_rank(rank, world, port, q):
    sys.path[:0] = [os.path.join(ROOT, "parameter-server_amd", "python")]
    os.environ["MASTER_PORT"] = str(port)  # default rendezvous name: parent pid + MASTER_PORT
    from psg_group import SocketGroup
    g = SocketGroup(rank, world, timeout_s=60)
    ag = g.all_gather((rank, b"h" * rank))
    bc = g.broadcast({"uid": b"\x01\x02"} if rank == 0 else None)
    mx = g.allreduce_max([float(rank), -float(rank), 7.0])
    for _ in range(20):
        g.barrier()
    g.close()
    q.put((rank, ag, bc, mx))


@pytest.mark.parametrize("world", [2, 4])
def test_socket_group_collectives(world):
    """bench.py's torch-free rendezvous (psg_group.SocketGroup): rank-ordered
    all_gather, broadcast from rank 0, element-wise max, repeated barriers."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_group_rank, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, ag, bc, mx in res:
        assert ag == [(r, b"h" * r) for r in range(world)]
        assert bc == {"uid": b"\x01\x02"}
        assert mx == [float(world - 1), 0.0, 7.0]


def _lr_rank(rank, world, port, outdir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
    import torch
    import torch.distributed as dist
    import oracle
    dist.init_process_group("gloo", rank=rank, world_size=world, init_method=f"tcp://127.0.0.1:{port}")
    n, rounds = 6000, 4
    blk = n // world
    w = oracle.synth(blk, oracle.F32, 900 + rank, 1, -0.5, 0.5)
    m, v = np.zeros(blk), np.zeros(blk)
    out = torch.zeros(n)
    for it in range(rounds):
        g = torch.from_numpy(oracle.synth(n, oracle.F32, 1000 * it + rank, 1, -1.0, 1.0))
        merged = torch.zeros(blk)
        dist.reduce_scatter_tensor(merged, g)  # psg_comm_lr_push's collective
        oracle.lr_apply(w, merged.numpy().astype(np.float32), 0.01, m, v, float(np.float32(0.01)),
                        0.9, 0.999, 1e-8, it)
        dist.all_gather_into_tensor(out, torch.from_numpy(w))
    np.save(os.path.join(outdir, f"lr{rank}.npy"), out.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_lr_bsp_reduce_scatter_within_tolerance(world):
    """The LR BSP round as the multi-GPU path runs it (reduce-scatter of the
    workers' gradients, the SGD/Adam update on each shard, all-gather of the
    model), rehearsed on gloo, against the reference replayed with every
    worker's push merged in arrival order: the collective sums in its own
    order, so the bar is the north star's 1e-6 relative."""
    import multiprocessing as mp
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as d:
        port = _free_port()
        procs = [ctx.Process(target=_lr_rank, args=(r, world, port, d)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
        assert all(p.exitcode == 0 for p in procs)
        got = [np.load(os.path.join(d, f"lr{r}.npy")) for r in range(world)]
    n, rounds = 6000, 4
    blk = n // world
    exp = np.empty(n, np.float32)
    for s in range(world):
        w = oracle.synth(blk, oracle.F32, 900 + s, 1, -0.5, 0.5)
        m, v = np.zeros(blk), np.zeros(blk)
        for it in range(rounds):
            merged = np.zeros(blk, np.float32)
            for r in range(world):
                merged = (merged + oracle.synth(n, oracle.F32, 1000 * it + r, 1, -1.0, 1.0)[s * blk:(s + 1) * blk]
                          ).astype(np.float32)
            oracle.lr_apply(w, merged, 0.01, m, v, float(np.float32(0.01)), 0.9, 0.999, 1e-8, it)
        exp[s * blk:(s + 1) * blk] = w
    for r in range(world):
        assert np.all(np.abs(got[r] - exp) <= REL_TOL * np.abs(exp) + 1e-7), r


# ---------------------------------------------------------------------------
# The RCCL exchanges that only ever ran with one rank on the GPU box —
# psg_comm_push_keyed / _pull_keyed (configs[3]) and psg_comm_push_pull's
# bucket pipeline — rehearsed with 2-4 ranks on gloo.  The offsets come from
# the same code the RCCL path runs: the library's host-only plans
# (psg_comm_keyed_plan, psg_comm_bucket_plan) and its server ranges
# (psg_server_ranges, PostOffice.cpp:211-221); the slice is the oracle's
# DefaultSlicer restatement (KVApp.h:515-574), which the -m gpu tests pin to
# psg_slice.  Each owner applies its reduced segment with oracle.Store, the
# CPU restatement of the handle the GPU path calls (psg_store_handle).
# Integer-valued data: bit-exact (every partial sum is exact in f32);
# real-valued: the north star's 1e-6 relative (the reduce sums in its own order).
def _exchange_rank(rank, world, port, outdir, kind, data):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "parameter-server_amd", "python")]
    import torch
    import torch.distributed as dist
    import oracle
    import psg
    dist.init_process_group("gloo", rank=rank, world_size=world, init_method=f"tcp://127.0.0.1:{port}")
    mode, lo, hi = (0, 0.0, 1000.0) if data == "int" else (1, -1.0, 1.0)
    steps = 3
    if kind == "keyed":
        rng = np.random.default_rng(5)
        keys = np.unique(rng.integers(0, (1 << 64) - 1, 30000, dtype=np.uint64))
        n = len(keys)
        b, e = psg.server_ranges(world)
        ob, oe = oracle.server_ranges(world)
        assert np.array_equal(b, ob) and np.array_equal(e, oe)
        kp, _ = oracle.slice_keys(keys, b, e)
        kp = [int(x) for x in kp]
        maxseg = psg.keyed_plan(kp, world, n)
        assert all(kp[r + 1] - kp[r] <= maxseg for r in range(world))
        vals = torch.from_numpy(oracle.synth(n, oracle.F32, 50 + rank, mode, lo, hi))
        store = oracle.Store(oracle.F32)
        mine = keys[kp[rank]:kp[rank + 1]]
        for _ in range(steps):
            for r in range(world):  # one reduce per key-range segment, to its owner
                seg = vals[kp[r]:kp[r + 1]].clone()
                dist.reduce(seg, dst=r)
                if r == rank and len(mine):
                    store.handle(oracle.PUSH, mine, seg.numpy(), len(mine))
        out = torch.zeros(n, dtype=torch.float32)
        if len(mine):
            out[kp[rank]:kp[rank + 1]] = torch.from_numpy(store.handle(oracle.PULL, mine, None, len(mine)))
        for r in range(world):  # each owner broadcasts its segment into place
            view = out[kp[r]:kp[r + 1]]
            if view.numel():
                dist.broadcast(view, src=r)
    else:
        blk = 10007  # not a multiple of 64: a ragged last bucket
        L = blk * world
        vals = torch.from_numpy(oracle.synth(L, oracle.F32, 70 + rank, mode, lo, hi))
        shard = torch.zeros(blk, dtype=torch.float32)
        out = torch.zeros(L, dtype=torch.float32)
        for step, nb in enumerate([1, 3, 8][:steps]):
            offs, cnts = psg.bucket_plan(blk, nb)
            assert int(offs[0]) == 0 and int(offs[-1] + cnts[-1]) == blk
            assert all(int(offs[i + 1]) == int(offs[i] + cnts[i]) for i in range(len(offs) - 1))
            for off, cnt in zip((int(x) for x in offs), (int(x) for x in cnts)):
                for r in range(world):  # bucket b of every rank's block, reduced to its owner
                    red = vals[r * blk + off:r * blk + off + cnt].clone()
                    dist.reduce(red, dst=r)
                    if r == rank:
                        shard[off:off + cnt] += red
                for r in range(world):  # ... and broadcast back from the owner
                    view = out[r * blk + off:r * blk + off + cnt]
                    if r == rank:
                        view.copy_(shard[off:off + cnt])
                    dist.broadcast(view, src=r)
    np.save(os.path.join(outdir, f"x{rank}.npy"), out.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("data", ["int", "real"])
@pytest.mark.parametrize("world", [2, 3, 4])
@pytest.mark.parametrize("kind", ["keyed", "buckets"])
def test_rccl_exchange_plans_rehearsed_on_gloo(kind, world, data):
    import multiprocessing as mp
    sys.path[:0] = [os.path.join(ROOT, "oracle")]
    import oracle
    ctx = mp.get_context("spawn")
    with tempfile.TemporaryDirectory() as d:
        port = _free_port()
        procs = [ctx.Process(target=_exchange_rank, args=(r, world, port, d, kind, data)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(120)
        assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
        got = [np.load(os.path.join(d, f"x{r}.npy")) for r in range(world)]
    mode, lo, hi = (0, 0.0, 1000.0) if data == "int" else (1, -1.0, 1.0)
    ref = oracle.Store(oracle.F32)
    if kind == "keyed":
        keys = np.unique(np.random.default_rng(5).integers(0, (1 << 64) - 1, 30000, dtype=np.uint64))
        n = len(keys)
        for _ in range(3):  # every worker's Push, in worker order (KVApp.h:446-454)
            for w in range(world):
                ref.handle(oracle.PUSH, keys, oracle.synth(n, oracle.F32, 50 + w, mode, lo, hi), n)
        exp = ref.handle(oracle.PULL, keys, None, n)
    else:
        L = 10007 * world
        for _ in range(3):
            for w in range(world):
                ref.handle(oracle.PUSH, None, oracle.synth(L, oracle.F32, 70 + w, mode, lo, hi), L)
        exp = ref.handle(oracle.PULL, None, None, L)
    for r in range(world):
        if data == "int":
            np.testing.assert_array_equal(got[r], exp, err_msg=f"rank {r}")
        else:
            assert np.all(np.abs(got[r] - exp) <= REL_TOL * np.abs(exp) + 1e-6), r
