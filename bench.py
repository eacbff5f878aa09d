#!/usr/bin/env python3
"""Device-resident KV Push+Pull GB/s (float vals) — the BASELINE.json metric.

One step = one worker Push of its dense value vector followed by one Pull of the
same keys (tests/test_kv_app_benchmark.cpp:54-81 semantics, buffers already in
HBM, keys implicit and consecutive):

  N = 1   configs[1]: 1 server + 1 worker, L = 64 M floats.  Push is the
          KVServerDefaultHandle accumulate (src/ps/KVApp.h:446-454) as one
          streaming HIP kernel over the DENSE store; Pull is the read-back.
  N > 1   configs[2] shape, one process per GPU, rank r = worker r + server
          shard r (L / N keys): Push = RCCL reduce-scatter + the accumulate
          kernel, Pull = RCCL all-gather (psg_comm_push / psg_comm_pull), or
          the two pipelined over buckets (psg_comm_push_pull) — whichever a
          short calibration in the warm-up finds faster on this node.

value = (B * L pushed + B * L pulled) * N / (max-over-ranks time per step),
B = bytes per value (weak scaling: every worker moves L values each way at
every N).  `--workload dense-f16` runs configs[4] (f16 values, 1 B per worker).

Prints ONE JSON line on rank 0.  Launch for N > 1:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
      --master-addr 127.0.0.1 --master-port P bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "parameter-server_amd", "python"), os.path.join(ROOT, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md "Chip-level parameters"
PUSH_ACCESSES = 3      # read vals + read store + write store
PULL_ACCESSES = 2      # read store + write out

WORKLOADS = {
    # name: (dtype name, value bytes, default values per worker, description)
    "dense": ("f32", 4, 64 << 20, "configs[1]"),
    "dense-f16": ("f16", 2, 1 << 30, "configs[4]"),
    "keyed": ("f32", 4, 10_000_000, "configs[3]"),
}
# algorithmic HBM bytes per key of one keyed Push on the SORTED store:
# request key 8 + store key 8 (resolve) + value 4 + store value read/write 8
# (the resolve is fused with the apply: no slot array goes to HBM and back)
KEYED_PUSH_BYTES = 28


class GpuBackend:
    """The product path: psg C-ABI (HIP kernels + RCCL)."""

    def __init__(self, rank: int, world: int, local_rank: int, dist=None, dtype="f32",
                 keyed=False):
        import psg
        self.p = psg
        self.rank, self.world, self.dist = rank, world, dist
        self.dt = {"f32": psg.F32, "f16": psg.F16}[dtype]
        self.vb = {"f32": 4, "f16": 2}[dtype]
        self.keyed = keyed
        # PSG_BENCH_SHARE_GPU=1 (testing only): ranks share the visible GPUs
        # round-robin, and RCCL — which refuses two ranks on one GPU — is not
        # used, so the xGMI exchange path of N > 1 can run on a 1-GPU box.
        self.share_gpu = os.environ.get("PSG_BENCH_SHARE_GPU") == "1"
        psg.set_device(local_rank % psg.device_count() if self.share_gpu else local_rank)
        self.stream = psg.Stream()
        self.comm = None
        self.xgmi = None
        self.mode = "rccl"  # "rccl" (RS + AG, or pipelined when fused) or "xgmi"
        self.fused = False
        self.nbuckets = 1

    def setup(self, L: int, seed: int):
        p = self.p
        blk = L // self.world
        self.L, self.blk, self._seed = L, blk, seed
        lo = self.rank * blk
        if self.keyed:
            # configs[3]: L unique sorted uint64 keys drawn uniformly (seed 9), the same
            # key set on every worker (LR-like); each server keeps a SORTED store
            import numpy as np
            rng = np.random.default_rng(9)
            k = np.unique(rng.integers(0, (1 << 64) - 1, int(L * 1.01) + 1024, dtype=np.uint64))
            k = np.sort(rng.choice(k, L, replace=False)) if len(k) > L else k
            self.keys = p.DeviceBuffer.from_numpy(k.astype(np.uint64))
            self.begins, self.ends = p.server_ranges(self.world)
            self.store = p.Store(p.SORTED, self.dt, int(self.begins[self.rank]),
                                 int(self.ends[self.rank]), 0)
        else:
            self.store = p.Store(p.DENSE, self.dt, lo, lo + blk, blk)
        self.vals = p.DeviceBuffer(L * self.vb)
        # integer-valued 0..7 (f16 holds them and their sums exactly) / 0..999 (f32)
        self.vals.fill_synth(L, self.dt, seed + self.rank, 0, 0.0, self._hi(), self.stream)
        self.out = p.DeviceBuffer(L * self.vb)
        if self.world > 1:
            if not self.share_gpu:
                uid = [p.comm_id() if self.rank == 0 else None]
                self.dist.broadcast_object_list(uid, src=0)
                self.comm = p.Comm(uid[0], self.world, self.rank)
            self.scratch = p.DeviceBuffer(blk * self.vb)
            if not self.keyed:
                self._setup_xgmi()
        self.sync()

    def _setup_xgmi(self):
        """Map every peer's request vector and shard (hipIpc) for the one-shot
        xGMI exchange (psg_xgmi_push / _pull); a node barrier orders the phases."""
        # Every step is agreed by all ranks (all_gather of a success flag), so a
        # node where IPC mapping is unavailable falls back to RCCL everywhere
        # instead of deadlocking.
        import uuid
        p = self.p
        self.xgmi = None
        self._peer_ptrs = []
        sptr = self.store.info().vals
        try:
            mine = (p.ipc_export(self.vals.ptr), p.ipc_export(sptr))
        except Exception as e:  # noqa: BLE001
            print(f"rank {self.rank}: hipIpc export unavailable ({e}); xGMI exchange off",
                  file=sys.stderr)
            mine = None
        allh = [None] * self.world
        self.dist.all_gather_object(allh, mine)
        if any(h is None for h in allh):
            return
        tag = [uuid.uuid4().hex[:16] if self.rank == 0 else None]
        self.dist.broadcast_object_list(tag, src=0)
        vptrs, sptrs, ok = [], [], True
        try:
            for r in range(self.world):
                if r == self.rank:
                    vptrs.append(self.vals.ptr)
                    sptrs.append(sptr)
                else:
                    vptrs.append(p.ipc_open(allh[r][0]))
                    self._peer_ptrs.append(vptrs[-1])
                    sptrs.append(p.ipc_open(allh[r][1]))
                    self._peer_ptrs.append(sptrs[-1])
            x = p.Xgmi(self.world, self.rank, vptrs, sptrs)
            b = p.NodeBarrier("psg_bench_" + tag[0], self.world, self.rank)
        except Exception as e:  # noqa: BLE001
            print(f"rank {self.rank}: xGMI mapping failed ({e}); xGMI exchange off", file=sys.stderr)
            ok = False
        oks = [None] * self.world
        self.dist.all_gather_object(oks, ok)
        if not all(oks):
            for ptr in self._peer_ptrs:
                p.ipc_close(ptr)
            self._peer_ptrs = []
            return
        self.xgmi, self.node_barrier = x, b
        self.node_barrier.wait()

    def _key_pos(self):
        # the worker's DefaultSlicer on its HBM keys (psg_slice), every request
        kp, _ = self.p.slice_keys(self.keys, self.L, self.begins, self.ends, stream=self.stream)
        return kp

    def _hi(self):
        return 1000.0 if self.dt == self.p.F32 else 8.0

    # -- one phase at a time (N = 1, or the sequential RS / AG at N > 1)
    def push(self):
        if self.mode == "xgmi":
            self.xgmi.push(self.store, self.L, self.stream)
            self.stream.sync()
            self.node_barrier.wait()
            return
        if self.keyed:
            # one server: the slice is the whole request (KVWorker's DefaultSlicer
            # skips the kernel for a single range; the store's range check covers it)
            if self.comm is None:
                self.store.handle(self.p.PUSH, self.keys, self.vals, None, self.L, stream=self.stream)
            else:
                self.comm.push_keyed(self.store, self.keys, self.vals, self.L, self._key_pos(), self.stream)
        elif self.comm is None:
            self.store.handle(self.p.PUSH, None, self.vals, None, self.L, first_key=0,
                              stream=self.stream)
        else:
            self.comm.push(self.store, self.vals, self.L, self.scratch, self.stream)

    def pull(self):
        if self.mode == "xgmi":
            self.xgmi.pull(self.store, self.out, self.L, self.stream)
            self.stream.sync()
            self.node_barrier.wait()
            return
        if self.keyed:
            if self.comm is None:
                self.store.handle(self.p.PULL, self.keys, None, self.out, self.L, stream=self.stream)
            else:
                self.comm.pull_keyed(self.store, self.keys, self.out, self.L, self._key_pos(), self.stream)
        elif self.comm is None:
            self.store.handle(self.p.PULL, None, None, self.out, self.L, first_key=0,
                              stream=self.stream)
        else:
            self.comm.pull(self.store, self.out, self.L, self.stream)

    # -- both, pipelined over buckets (N > 1)
    def step(self):
        self.comm.push_pull(self.store, self.vals, self.out, self.L, self.nbuckets, self.stream)

    def _set_mode(self, cand):
        mode, nb = cand
        self.mode, self.nbuckets = mode, nb
        self.fused = mode == "rccl" and nb > 1

    def calibrate(self, dist, iters=3):
        """Pick the exchange for this node by timing each candidate a few times
        (wall clock, barrier-synced): RCCL reduce-scatter then all-gather, the
        RCCL pipelined over 4/8/16 buckets, or the one-shot xGMI kernels.  The
        max over ranks decides, so every rank picks the same."""
        if self.world == 1 or self.keyed:
            return
        import torch
        cands = [("rccl", 1), ("rccl", 4), ("rccl", 8), ("rccl", 16)] if self.comm is not None else []
        if self.xgmi is not None:
            cands.append(("xgmi", 0))
        times = []
        for cand in cands:
            self._set_mode(cand)
            self._one_step()
            self.sync()
            dist.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                self._one_step()
            self.sync()
            times.append((time.perf_counter() - t0) * 1e3 / iters)
            dist.barrier()
        t = torch.tensor(times, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        order = sorted(range(len(cands)), key=lambda i: t[i].item())
        self._set_mode(cands[order[0]])
        self.calibration = {f"{m}{'' if m == 'xgmi' else '/' + str(nb)}": round(x, 4)
                            for (m, nb), x in zip(cands, t.tolist())}
        self.pushes_in_calibration = len(cands) * (iters + 1)
        if self.mode == "xgmi":
            self.pushes_in_calibration += 1
            self.exchange_verified = self._verify_xgmi(dist)
            if not self.exchange_verified:
                rest = [cands[i] for i in order if cands[i][0] != "xgmi"]
                if not rest:
                    raise RuntimeError("xGMI exchange failed its checksum verification "
                                       "and no RCCL communicator is available")
                print("xGMI exchange failed its checksum verification; using RCCL",
                      file=sys.stderr)
                self._set_mode(rest[0])

    def _verify_xgmi(self, dist) -> bool:
        """One xGMI Push + Pull, then every rank's pulled block w must carry the
        same psg_checksum as rank w's own shard (read locally): catches a stale
        or torn cross-GPU read before the timed steps rely on the path."""
        p = self.p
        self.push()
        self.pull()
        nb = self.blk * self.vb
        mine = p.checksum(self.store.info().vals, nb, self.stream)
        got = [p.checksum(self.out.ptr + w * nb, nb, self.stream) for w in range(self.world)]
        owners = [None] * self.world
        dist.all_gather_object(owners, mine)
        ok = [None] * self.world
        dist.all_gather_object(ok, got == owners)
        return all(ok)

    def _one_step(self):
        if self.fused:
            self.step()
        else:
            self.push()
            self.pull()

    def new_event(self):
        return self.p.Event()

    def record(self, e):
        e.record(self.stream)

    def elapsed(self, a, b) -> float:
        return a.elapsed_ms(b)

    def sync(self):
        self.stream.sync()
        self.p.device_sync()

    def accumulate_probe(self, iters=10):
        """The dominant local kernel at N > 1: the shard accumulate after the
        reduce-scatter (12 B per f32 element), timed alone with HIP events."""
        if self.keyed:
            return None
        a, b = self.new_event(), self.new_event()
        self.record(a)
        for _ in range(iters):
            if self.mode == "xgmi":
                # reads the peers' (constant) request vectors and writes only this
                # rank's shard: safe to repeat without a barrier
                self.xgmi.push(self.store, self.L, self.stream)
            else:
                self.store.handle(self.p.PUSH, None, self.scratch, None, self.blk,
                                  first_key=self.rank * self.blk, stream=self.stream)
        self.record(b)
        self.sync()
        return self.elapsed(a, b) / iters

    def probe_kernel(self):
        """(name, algorithmic bytes per launch) of the kernel accumulate_probe times."""
        if self.mode == "xgmi":
            # store read + write (8 B) + one 4-B value from every rank's vector
            return ("k_xgmi_push (fused reduce of %d ranks' blocks + accumulate; "
                    "%d of them read over xGMI)" % (self.world, self.world - 1),
                    (8 + self.vb * self.world) * self.blk)
        return ("k_dense_vec<PUSH> on the shard after the reduce-scatter",
                PUSH_ACCESSES * self.vb * self.blk)

    def check(self, steps_done: int) -> bool:
        """After `steps_done` pushes every shard holds steps * sum_w vals_w
        (integer-valued, exact in f32 and in f16 at the default sizes)."""
        import numpy as np
        import oracle
        self.pull()
        self.sync()
        n = min(self.L, 1 << 20)
        npt = {self.p.F32: np.float32, self.p.F16: np.float16}[self.dt]
        got = self.out.download(npt, n, self.stream).astype(np.float64)
        exp = np.zeros(n)
        odt = {self.p.F32: oracle.F32, self.p.F16: oracle.F16}[self.dt]
        for w in range(self.world):
            s = oracle.synth(n, odt, self._seed + w, 0, 0.0, self._hi())
            exp += (s.view(np.float16) if self.dt == self.p.F16 else s).astype(np.float64)
        return bool(np.array_equal(got, exp * steps_done))


def run(backend, args, rank: int, world: int, dist=None) -> dict | None:
    L = args.keys
    assert L % world == 0, "keys must divide by the number of shards"
    backend._seed = args.seed
    backend.setup(L, args.seed)
    extra_pushes = 0
    if hasattr(backend, "calibrate") and dist is not None:
        backend.calibrate(dist)
        extra_pushes = getattr(backend, "pushes_in_calibration", 0)
    fused = getattr(backend, "fused", False)

    def barrier():
        if dist is not None:
            dist.barrier()

    def one_step():
        if fused:
            backend.step()
        else:
            backend.push()
            backend.pull()

    for _ in range(args.warmup):
        one_step()
    # Kernel times come from HIP events recorded live in the timed region, on
    # every `event_every`-th step only: a marker is not free on ROCm (each one
    # measured ~4 us of the ~0.19 ms step), so the other steps run unperturbed.
    # Sampled step k: e0 | Push k | e1 | Pull k | e2.
    every = max(1, getattr(args, "event_every", 1))
    sampled = [k for k in range(args.steps) if k % every == 0]
    evs = {k: (backend.new_event(), backend.new_event(), backend.new_event()) for k in sampled}
    backend.sync()
    barrier()
    backend.sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        e = evs.get(k)
        if e:
            backend.record(e[0])
        if fused:
            backend.step()
            if e:
                backend.record(e[1])
        else:
            backend.push()
            if e:
                backend.record(e[1])
            backend.pull()
        if e:
            backend.record(e[2])
    backend.sync()
    barrier()
    t1 = time.perf_counter()
    local_ms = (t1 - t0) * 1e3 / max(args.steps, 1)
    n_marks = max(len(sampled), 1)
    push_ms = sum(backend.elapsed(a, b) for a, b, _ in evs.values()) / n_marks
    pull_ms = sum(backend.elapsed(b, c) for _, b, c in evs.values()) / n_marks
    ms = local_ms
    acc_ms = backend.accumulate_probe() if (world > 1 and hasattr(backend, "accumulate_probe")) else None
    if dist is not None:
        import torch
        t = torch.tensor([local_ms, push_ms, pull_ms, acc_ms or 0.0], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms, push_ms, pull_ms, acc = t.tolist()
        acc_ms = acc if acc_ms is not None else None
    total_pushes = args.warmup + args.steps + extra_pushes + (10 if acc_ms is not None else 0)
    ok = None
    if args.check:
        # the accumulate probe adds the (last reduce-scatter) scratch 10 more times,
        # which breaks the closed form; only check when no probe ran
        ok = backend.check(total_pushes) if acc_ms is None else backend_check_after_probe(backend)
        if dist is not None:
            import torch
            f = torch.tensor([0 if ok else 1], dtype=torch.int32)
            dist.all_reduce(f, op=dist.ReduceOp.MAX)
            ok = f.item() == 0
    if rank != 0:
        return None
    vb = getattr(backend, "vb", 4)
    payload = 2 * vb * L * world  # pushed + pulled by all workers per step
    value_gbs = payload / (ms * 1e-3) / 1e9
    blk = L // world
    wl = getattr(args, "workload", "dense")
    res = {
        "metric": "device-resident KV Push+Pull GB/s (float vals)",
        "value": round(value_gbs, 3),
        "unit": "GB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": WORKLOADS.get(wl, ("f32",))[0],
        "data": "synthetic (integer-valued floats, seed 7+rank, generated in HBM)",
        "config": {
            "workload": (f"{WORKLOADS.get(wl, ('', 0, 0, 'configs[1]'))[3]}: "
                         + (("keyed (10 M sorted uint64 keys, SORTED store), " if wl == "keyed" else "dense, ")
                            + ("1 server + 1 worker, Push then Pull" if world == 1 else
                               f"ns=nw={world}, BSP Push/Pull (see exchange)"))),
            "keys_per_worker": L,
            "shard_keys": blk,
            "parallelism": f"ps{world}",
        },
        "push_ms": None if fused else round(push_ms, 5),
        "pull_ms": None if fused else round(pull_ms, 5),
        "parity_check": ok,
    }
    if world > 1 and hasattr(backend, "nbuckets"):
        if getattr(backend, "mode", "rccl") == "xgmi":
            res["config"]["exchange"] = "one-shot xGMI kernels (psg_xgmi push/pull, peers via hipIpc)"
        elif getattr(backend, "keyed", False):
            res["config"]["exchange"] = "RCCL grouped reduce / broadcast of the key-range segments"
        else:
            res["config"]["exchange"] = ("RCCL pipelined reduce/broadcast, %d buckets" % backend.nbuckets
                                         if fused else "RCCL reduce-scatter then all-gather")
        res["config"]["calibration_ms"] = getattr(backend, "calibration", None)
        if hasattr(backend, "exchange_verified"):
            res["config"]["xgmi_checksum_verified"] = backend.exchange_verified
    if world == 1 and getattr(backend, "keyed", False):
        res["roofline"] = roofline(KEYED_PUSH_BYTES * L, push_ms, args,
                                   "SORTED-store Push: k_tile_windows + k_resolve_apply "
                                   "(one host sync; one server, so no slicer pass)", vb)
    elif world == 1:
        res["roofline"] = roofline(PUSH_ACCESSES * vb * blk, push_ms, args,
                                   "k_dense_vec<PUSH> (store += vals)", vb)
        res["pull_roofline_frac"] = round(PULL_ACCESSES * vb * blk / (pull_ms * 1e-3) / 1e9
                                          / HBM_PEAK_GBS, 4)
    elif acc_ms is not None and hasattr(backend, "probe_kernel"):
        kname, kbytes = backend.probe_kernel()
        res["roofline"] = roofline(kbytes, acc_ms, args, kname, vb)
    elif acc_ms is not None:
        res["roofline"] = roofline(PUSH_ACCESSES * vb * blk, acc_ms, args,
                                   "k_dense_vec<PUSH> on the shard after the reduce-scatter", vb)
    else:
        res["roofline"] = None
    if world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args)
    return res


def backend_check_after_probe(backend) -> bool:
    """With the probe having re-added the scratch, check the Pull equals the shards
    (all-gather correctness) instead of the closed form."""
    import numpy as np
    backend.pull()
    backend.sync()
    npt = {backend.p.F32: np.float32, backend.p.F16: np.float16}[backend.dt]
    got = backend.out.download(npt, backend.L, backend.stream)
    _, mine = backend.store.dump()
    mine = mine.view(np.float16) if backend.dt == backend.p.F16 else mine
    lo = backend.rank * backend.blk
    return bool(np.array_equal(got[lo:lo + backend.blk], mine[:backend.blk]))


def roofline(alg_bytes: int, ms: float, args, kernel: str, vb: int) -> dict:
    achieved = alg_bytes / (ms * 1e-3) / 1e9
    # HBM bytes per launch from the committed PMC summaries (tools/pmc_summary.py):
    # the one measured on this kernel at these algorithmic bytes, if any
    traffic = None
    import glob
    for pmc in sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json"))):
        try:
            d = json.load(open(pmc))
        except Exception:
            continue
        names = [k.split("<")[0].strip() for k in str(d.get("kernel", "")).split("|")]
        if d.get("alg_bytes_per_launch") == alg_bytes and names and all(n in kernel for n in names):
            traffic = d.get("hbm_bytes_per_launch")
            break
    return {
        "kernel": kernel,
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "alg_bytes_per_launch": alg_bytes,
    }


def cpu_baseline(args) -> dict:
    """The reference handler (std::unordered_map, one thread) restated in oracle/,
    on the test_kv_app_benchmark layout: 10 M keys, 1 inserting Push, then
    `reps` steady Push + Pull.  Reported beside the GPU number, not a target."""
    import oracle
    num, reps = args.cpu_keys, args.cpu_reps
    t0 = time.perf_counter()
    first, push_s, pull_s = oracle.bench(num, reps)
    wall = time.perf_counter() - t0
    return {
        "value": round(2 * 4 * num / (push_s + pull_s) / 1e9, 4),
        "unit": "GB/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"{num} keys (kMaxKey/num*i layout), 1 inserting Push ({first:.2f} s) then "
                   f"{reps} steady Push+Pull through KVServerDefaultHandle's unordered_map loop, "
                   f"single thread, {wall:.1f} s total"),
    }


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="dense")
    ap.add_argument("--keys", type=int, default=None, help="values per worker (default by workload)")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--event-every", type=int, default=5,
                    help="record the kernel-timing HIP events on every n-th timed step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-keys", type=int, default=10_000_000)
    ap.add_argument("--cpu-reps", type=int, default=25)
    args = ap.parse_args(argv)
    dtype, _, default_keys, _ = WORKLOADS[args.workload]
    if args.keys is None:
        args.keys = default_keys

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}", file=sys.stderr)
    dist = None
    if world > 1:
        import torch  # noqa: F401  (load torch's HIP runtime before libpsgpu)
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
    backend = GpuBackend(rank, world, local_rank, dist, dtype, keyed=args.workload == "keyed")
    res = run(backend, args, rank, world, dist)
    if res is not None:
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.barrier()
    if backend.xgmi is not None:
        backend.sync()
        backend.node_barrier.wait()  # no peer still reads a buffer this rank unmaps
        backend.xgmi.close()
        for ptr in backend._peer_ptrs:
            backend.p.ipc_close(ptr)
        backend.node_barrier.close()
    if backend.comm is not None:
        backend.sync()
        backend.comm.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
