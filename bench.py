#!/usr/bin/env python3
"""Device-resident KV Push+Pull GB/s (float vals) — the BASELINE.json metric.

One step = one worker Push of its dense float vector followed by one Pull of
the same keys (tests/test_kv_app_benchmark.cpp:54-81 semantics, buffers already
in HBM, keys implicit and consecutive):

  N = 1   configs[1]: 1 server + 1 worker, L = 64 M floats.  Push is the
          KVServerDefaultHandle accumulate (src/ps/KVApp.h:446-454) as one
          streaming HIP kernel over the DENSE store; Pull is the read-back.
  N > 1   configs[3] shape, one process per GPU, rank r = worker r + server
          shard r (L / N keys): Push = RCCL reduce-scatter + the accumulate
          kernel, Pull = RCCL all-gather (psg_comm_push / psg_comm_pull).

value = (4 B * L pushed + 4 B * L pulled) * N / (max-over-ranks time per step)
(weak scaling: every worker moves L floats each way at every N).

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
F32_BYTES = 4
PUSH_BYTES_PER_ELEM = 12  # read vals + read store + write store
PULL_BYTES_PER_ELEM = 8   # read store + write out


class GpuBackend:
    """The product path: psg C-ABI (HIP kernels + RCCL)."""

    def __init__(self, rank: int, world: int, local_rank: int, dist=None):
        import psg
        self.p = psg
        self.rank, self.world, self.dist = rank, world, dist
        psg.set_device(local_rank)
        self.stream = psg.Stream()
        self.comm = None

    def setup(self, L: int, seed: int):
        p = self.p
        blk = L // self.world
        self.L, self.blk = L, blk
        lo = self.rank * blk
        self.store = p.Store(p.DENSE, p.F32, lo, lo + blk, blk)
        self.vals = p.DeviceBuffer(L * F32_BYTES)
        self.vals.fill_synth(L, p.F32, seed + self.rank, 0, 0.0, 1000.0, self.stream)
        self.out = p.DeviceBuffer(L * F32_BYTES)
        if self.world > 1:
            uid = [p.comm_id() if self.rank == 0 else None]
            self.dist.broadcast_object_list(uid, src=0)
            self.comm = p.Comm(uid[0], self.world, self.rank)
            self.scratch = p.DeviceBuffer(blk * F32_BYTES)
        self.ev = []
        self.sync()

    def push(self):
        if self.comm is None:
            self.store.handle(self.p.PUSH, None, self.vals, None, self.L, first_key=0,
                              stream=self.stream)
        else:
            self.comm.push(self.store, self.vals, self.L, self.scratch, self.stream)

    def pull(self):
        if self.comm is None:
            self.store.handle(self.p.PULL, None, None, self.out, self.L, first_key=0,
                              stream=self.stream)
        else:
            self.comm.pull(self.store, self.out, self.L, self.stream)

    def new_event(self):
        return self.p.Event()

    def record(self, e):
        e.record(self.stream)

    def elapsed(self, a, b) -> float:
        return a.elapsed_ms(b)

    def sync(self):
        self.stream.sync()
        self.p.device_sync()

    def check(self, steps_done: int) -> bool:
        """Pull result after `steps_done` pushes: every shard holds steps * sum_w vals_w
        (integer-valued floats, exact)."""
        import numpy as np
        self.pull()
        self.sync()
        got = self.out.download(np.float32, min(self.L, 1 << 20), self.stream)
        import oracle
        exp = np.zeros_like(got)
        for w in range(self.world):
            exp += oracle.synth(len(got), oracle.F32, self._seed + w, 0, 0.0, 1000.0)
        return bool(np.array_equal(got, exp * steps_done))


def run(backend, args, rank: int, world: int, dist=None) -> dict | None:
    L = args.keys
    assert L % world == 0, "keys must divide by the number of shards"
    backend._seed = args.seed
    backend.setup(L, args.seed)

    def barrier():
        if dist is not None:
            dist.barrier()

    for _ in range(args.warmup):
        backend.push()
        backend.pull()
    marks = [(backend.new_event(), backend.new_event(), backend.new_event())
             for _ in range(args.steps)]
    backend.sync()
    barrier()
    backend.sync()
    t0 = time.perf_counter()
    for a, b, c in marks:
        backend.record(a)
        backend.push()
        backend.record(b)
        backend.pull()
        backend.record(c)
    backend.sync()
    barrier()
    t1 = time.perf_counter()
    local_ms = (t1 - t0) * 1e3 / max(args.steps, 1)
    push_ms = sum(backend.elapsed(a, b) for a, b, _ in marks) / max(len(marks), 1)
    pull_ms = sum(backend.elapsed(b, c) for _, b, c in marks) / max(len(marks), 1)
    ms = local_ms
    if dist is not None:
        import torch
        t = torch.tensor([local_ms, push_ms, pull_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        ms, push_ms, pull_ms = t.tolist()
    ok = backend.check(args.warmup + args.steps) if args.check else None
    if dist is not None and args.check:
        import torch
        f = torch.tensor([0 if ok else 1], dtype=torch.int32)
        dist.all_reduce(f, op=dist.ReduceOp.MAX)
        ok = f.item() == 0
    if rank != 0:
        return None
    payload = 2 * F32_BYTES * L * world  # pushed + pulled by all workers per step
    value_gbs = payload / (ms * 1e-3) / 1e9
    blk = L // world
    # dominant kernel: the Push accumulate over this rank's shard
    push_alg = PUSH_BYTES_PER_ELEM * blk
    roof_achieved = push_alg / (push_ms * 1e-3) / 1e9 if world == 1 else None
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
        "dtype": "f32",
        "data": "synthetic (integer-valued U{0..999} floats, seed 7+rank, generated in HBM)",
        "config": {
            "workload": ("configs[1]: 1 server + 1 worker, dense Push then Pull"
                         if world == 1 else
                         f"configs[2] shape: ns=nw={world}, Push=RCCL reduce-scatter+accumulate, "
                         f"Pull=RCCL all-gather"),
            "keys_per_worker": L,
            "shard_keys": blk,
            "parallelism": f"ps{world}",
        },
        "push_ms": round(push_ms, 5),
        "pull_ms": round(pull_ms, 5),
        "parity_check": ok,
    }
    if world == 1:
        res["roofline"] = roofline(push_alg, push_ms, args)
        res["pull_roofline_frac"] = round(PULL_BYTES_PER_ELEM * blk / (pull_ms * 1e-3) / 1e9
                                          / HBM_PEAK_GBS, 4)
    else:
        res["roofline"] = None
    if world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args)
    return res


def roofline(push_alg_bytes: int, push_ms: float, args) -> dict:
    achieved = push_alg_bytes / (push_ms * 1e-3) / 1e9
    traffic = None
    pmc = os.path.join(ROOT, "profiles", "pmc_push_traffic.json")
    if os.path.exists(pmc):
        try:
            d = json.load(open(pmc))
            if d.get("keys") == args.keys:
                traffic = d.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    return {
        "kernel": "k_dense_vec<f32,PUSH> (store += vals)",
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        "alg_bytes_per_launch": push_alg_bytes,
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
        "value": round(2 * F32_BYTES * num / (push_s + pull_s) / 1e9, 4),
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
    ap.add_argument("--keys", type=int, default=64 << 20, help="floats per worker (configs[1]: 64M)")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-keys", type=int, default=10_000_000)
    ap.add_argument("--cpu-reps", type=int, default=12)
    args = ap.parse_args(argv)

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
    backend = GpuBackend(rank, world, local_rank, dist)
    res = run(backend, args, rank, world, dist)
    if res is not None:
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
