#!/usr/bin/env python3
"""Device-resident KV Push+Pull GB/s (float vals) — the BASELINE.json metric.

One step = one worker Push of its dense value vector followed by one Pull of the
same keys (tests/test_kv_app_benchmark.cpp:54-81 semantics, buffers already in
HBM, keys implicit and consecutive):

  N = 1   configs[1]: 1 server + 1 worker, L = 64 M floats.  Push is the
          KVServerDefaultHandle accumulate (src/ps/KVApp.h:446-454) as one
          streaming HIP kernel over the DENSE store; Pull is the read-back.
  N > 1   configs[2]: one process per GPU, rank r = worker r + server shard r,
          L = 256 M floats per worker (L / N keys per shard): Push = RCCL
          reduce-scatter + the accumulate kernel, Pull = RCCL all-gather
          (psg_comm_push / psg_comm_pull), the two pipelined over buckets
          (psg_comm_push_pull), or the one-shot xGMI kernels (psg_xgmi_*) —
          whichever a short calibration in the warm-up finds faster here.

value = (B * L pushed + B * L pulled) * N / (max-over-ranks time per step),
B = bytes per value (weak scaling: every worker moves L values each way at
every N).  `--workload dense-f16` runs configs[4] (f16 values, 1 G per worker),
`--workload keyed` configs[3] (10 M sorted uint64 keys, SORTED stores).

The N > 1 job is bootstrapped without torch (psg_group.SocketGroup: a loopback
star with rank 0 as the rendezvous), so libpsgpu.so runs on /opt/rocm's HIP and
RCCL at every N; the line names the libraries the process mapped.

Prints ONE JSON line on rank 0.  Launch for N > 1:
  python -m torch.distributed.run --nnodes=1 --nproc-per-node N \
      --master-addr 127.0.0.1 --master-port P bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import socket
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (os.path.join(ROOT, "parameter-server_amd", "python"), os.path.join(ROOT, "oracle")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E, MI355X_MICROARCH.md "Chip-level parameters"
# The markers that time kernels record without the system-scope release fence
# (psg_event_create_timing, hipEventDisableSystemFence: "can improve the
# accuracy of timing measurements by avoiding the cost of cache writeback and
# invalidation", hip_runtime_api.h); PSG_BENCH_EVENTS=fence for default events
TIMING_EVENTS = os.environ.get("PSG_BENCH_EVENTS", "timing") != "fence"
PUSH_ACCESSES = 3      # read vals + read store + write store
PULL_ACCESSES = 2      # read store + write out

WORKLOADS = {
    # name: (dtype name, value bytes, values per worker at N = 1, at N > 1, configs entry)
    "dense": ("f32", 4, 64 << 20, 256 << 20, "configs[1]", "configs[2]"),
    "dense-f16": ("f16", 2, 1 << 30, 1 << 30, "configs[4]", "configs[4]"),
    "keyed": ("f32", 4, 10_000_000, 10_000_000, "configs[3]", "configs[3]"),
    # configs[3] as LR_ps runs it with USE_KEY_CACHING (LRServer.h:127-142): the
    # first request resolves the key list once, later ones name it by hash and
    # run on the cached slots (psg_store_handle_slots)
    "keyed-cached": ("f32", 4, 10_000_000, 10_000_000, "configs[3] (key caching)", "configs[3] (key caching)"),
    # configs[3]'s server side as LRServer runs it in sync mode (LRServer.h:151-178):
    # one BSP round = merge the nw = 4 workers' gradient frames + the Adam update
    # (Adam.h:28-34), one kernel (psg_lr_apply_sum); a line of its own (run_lr)
    "lr": ("f32", 4, 64 << 20, 64 << 20, "LR BSP round", "LR BSP round"),
    # the drop-in API itself (run_dropin): ZPush / ZPull through KVWorker /
    # KVServer (KVServerDefaultHandle, HBM stores) at ns = nw = N, launched as
    # the reference launches its harnesses (local.py: one process per node), with
    # test_kv_app_benchmark's key layout; a line of its own
    "dropin": ("f32", 4, 10_000_000, 10_000_000, "configs[0] layout via KVWorker/KVServer",
               "configs[0] layout via KVWorker/KVServer"),
}
# algorithmic HBM bytes per key of one keyed Push on the SORTED store:
# request key 8 + store key 8 (resolve) + value 4 + store value read/write 8
# (the resolve is fused with the apply: no slot array goes to HBM and back)
KEYED_PUSH_BYTES = 28
# ... and with a cached slot list: slot 4 + value 4 + store value read/write 8
CACHED_PUSH_BYTES = 16
# ... and when that list's slots are a stretch of the store: value 4 + store value read/write 8
STRETCH_PUSH_BYTES = 12
# pushes outside warmup + steps that a run may make (calibration, verification)
BATCHED = 20  # requests per batch of the cached-stretch line's batched timing
EXTRA_PUSH_BOUND = 64


class GpuBackend:
    """The product path: psg C-ABI (HIP kernels + RCCL)."""

    def __init__(self, rank: int, world: int, local_rank: int, group=None, dtype="f32",
                 keyed=False, cached=False):
        import psg
        self.p = psg
        self.rank, self.world, self.group = rank, world, group
        self.dt = {"f32": psg.F32, "f16": psg.F16}[dtype]
        self.vb = {"f32": 4, "f16": 2}[dtype]
        self.keyed = keyed or cached
        self.cached = cached
        # PSG_BENCH_SHARE_GPU=1 (testing only): ranks share the visible GPUs
        # round-robin, and RCCL — which refuses two ranks on one GPU — is not
        # used, so the xGMI exchange path of N > 1 can run on a 1-GPU box.
        self.share_gpu = os.environ.get("PSG_BENCH_SHARE_GPU") == "1"
        ndev = psg.device_count()
        if world > 1 and not self.share_gpu and local_rank >= ndev:
            raise SystemExit(f"bench.py rank {rank}: LOCAL_RANK {local_rank} but {ndev} GPU(s) visible; one GPU per "
                             "rank is required (PSG_BENCH_SHARE_GPU=1: the shared-GPU test mode)")
        self.device = local_rank % ndev if self.share_gpu else local_rank
        psg.set_device(self.device)
        self.pci_bus_id = psg.device_pci_bus_id(self.device)
        self.host = socket.gethostname()
        if world > 1 and not self.share_gpu:
            # one GPU per rank, or the line would measure ranks sharing a device
            # (VERDICT r5 next #5): every rank names its physical GPU, and a
            # duplicate ends the job on every rank before RCCL starts
            seen = group.all_gather((self.host, self.pci_bus_id, rank))
            where = {}
            for h, pci, r in seen:
                where.setdefault((h, pci), []).append(r)
            dup = {k: v for k, v in where.items() if len(v) > 1}
            if dup:
                (h, pci), rs = next(iter(dup.items()))
                raise SystemExit(f"bench.py: ranks {rs} all run on GPU {pci} of {h}; one GPU per rank is "
                                 "required (PSG_BENCH_SHARE_GPU=1: the shared-GPU test mode)")
        self.stream = psg.Stream()
        self.comm = None
        self.xgmi = None
        self.store = None
        self.mode = "rccl"  # "rccl" (RS + AG, or pipelined when fused) or "xgmi"
        self.fused = False
        self.nbuckets = 1
        self.max_pushes = 1 << 10

    def describe(self) -> dict:
        """Where this rank ran: its HIP device, that GPU's PCI bus id and host,
        and the rank / rank count RCCL reports (psg_comm_rank) when it is up."""
        d = {"rank": self.rank, "device": self.device, "pci_bus_id": self.pci_bus_id, "host": self.host}
        if self.comm is not None:
            d["rccl_rank"], d["rccl_nranks"] = self.comm.rank()
        else:
            d["rccl_rank"] = d["rccl_nranks"] = None
        return d

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
            extra = int(os.environ.get("PSG_BENCH_STORE_EXTRA", "0"))
            if extra > 0 and self.world == 1:
                # a store that holds `extra` more keys per request key, between
                # them (the request is then every (extra+1)-th key of the store,
                # not a stretch of it: the general fused path, not the identity
                # one); inserted once with value 0 by a Pull, as operator[] does
                kk = k.astype(np.uint64)
                gaps = np.diff(kk)
                assert np.all(gaps > extra), "keys too dense for the extra store keys"
                more = [kk[:-1] + (gaps // (extra + 1)) * np.uint64(j) for j in range(1, extra + 1)]
                sk = np.unique(np.concatenate([kk] + more))
                dsk = p.DeviceBuffer.from_numpy(sk)
                tmp = p.DeviceBuffer(len(sk) * self.vb)
                self.store.handle(p.PULL, dsk, None, tmp, len(sk), stream=self.stream)
                self.sync()
                tmp.free()
                dsk.free()
                self.store_extra = extra
            nstretch = int(os.environ.get("PSG_BENCH_STRETCHES", "0"))
            if nstretch > 1 and self.world == 1:
                # the request a union of `nstretch` stretches of the store: 4096
                # store keys the request lacks sit in each of nstretch - 1 seams,
                # evenly spaced (VERDICT r4 next #4's stretch-union list); the
                # identity path fails on it, the general path's stretch tiles
                # serve it (k_validate_windows chunk_ok)
                kk = k.astype(np.uint64)
                seams = [int(L * j / nstretch) for j in range(1, nstretch)]
                more = []
                for pos in seams:
                    a, b = int(kk[pos - 1]), int(kk[pos])
                    assert b - a > 4097, "keys too dense for a seam"
                    more.append(np.arange(a + 1, a + 4097, dtype=np.uint64))
                sk = np.unique(np.concatenate([kk] + more))
                dsk = p.DeviceBuffer.from_numpy(sk)
                tmp = p.DeviceBuffer(len(sk) * self.vb)
                self.store.handle(p.PULL, dsk, None, tmp, len(sk), stream=self.stream)
                self.sync()
                tmp.free()
                dsk.free()
                self.store_stretches = nstretch
            subset = float(os.environ.get("PSG_BENCH_SUBSET", "0"))
            if 0.0 < subset < 1.0 and self.world == 1:
                # the request a random subset of the store at density `subset`:
                # L (1/subset - 1) more store keys drawn uniformly (seed 10), so
                # they fall between the request's keys at random (VERDICT r4
                # next #4's random-subset list); no tile is a stretch
                kk = k.astype(np.uint64)
                m = int(round(L * (1.0 / subset - 1.0)))
                r2 = np.random.default_rng(10)
                more = np.setdiff1d(np.unique(r2.integers(0, (1 << 64) - 1, int(m * 1.01) + 1024, dtype=np.uint64)), kk)
                more = r2.choice(more, m, replace=False) if len(more) > m else more
                sk = np.unique(np.concatenate([kk, more.astype(np.uint64)]))
                dsk = p.DeviceBuffer.from_numpy(sk)
                tmp = p.DeviceBuffer(len(sk) * self.vb)
                self.store.handle(p.PULL, dsk, None, tmp, len(sk), stream=self.stream)
                self.sync()
                tmp.free()
                dsk.free()
                self.store_subset = (subset, len(sk))
        else:
            self.store = p.Store(p.DENSE, self.dt, lo, lo + blk, blk)
        self.vals = p.DeviceBuffer(L * self.vb)
        self.vals.fill_synth(L, self.dt, seed + self.rank, 0, 0.0, self.hi(), self.stream)
        self.out = p.DeviceBuffer(L * self.vb)
        if self.cached and self.world == 1:
            # the first request of the key list: resolve it once, inserting the
            # keys (value 0, like the first Push's operator[]); later requests
            # run on the cached slots
            self.slots = p.DeviceBuffer(L * 4)
            self.store.resolve(self.keys, L, self.slots, insert=True, stream=self.stream)
            # a list that covers its range of the store resolves to a stretch of
            # slots, served without the slot stream (psg_store_handle_stretch)
            self.stretch = None if os.environ.get("PSG_BENCH_NO_STRETCH") == "1" else \
                self.store.slots_stretch(self.slots, L, stream=self.stream)
        if self.world > 1 and self.cached:
            self._setup_keyed_cached()
        elif self.world > 1:
            if self.keyed and self.share_gpu:
                raise SystemExit("the keyed N > 1 exchange runs on RCCL: one GPU per rank "
                                 "(PSG_BENCH_SHARE_GPU has no keyed path)")
            if not self.share_gpu:
                uid = self.group.broadcast(p.comm_id() if self.rank == 0 else None)
                try:
                    self.comm = p.Comm(uid, self.world, self.rank)
                except Exception as e:  # noqa: BLE001
                    print(f"rank {self.rank}: RCCL init failed ({e})", file=sys.stderr)
                    self.comm = None
                # every rank agrees: without a communicator on all of them the
                # exchange is the xGMI kernels alone
                if not all(self.group.all_gather(self.comm is not None)):
                    if self.comm is not None:
                        self.comm.close()
                    self.comm = None
                    if self.keyed:
                        raise SystemExit("the keyed N > 1 exchange needs RCCL, which failed to start")
            self.scratch = p.DeviceBuffer(blk * self.vb)
            if not self.keyed:
                self._setup_xgmi()
        self.sync()

    def hi(self) -> float:
        """Integer values 0..hi-1, so every partial sum is exact: 0..999 in f32;
        in f16 small enough that world * pushes * (hi - 1) stays <= 2048."""
        if self.dt == self.p.F32:
            return 1000.0
        return float(max(2, min(8, 2048 // (self.world * self.max_pushes) + 1)))

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
            mine = (p.ipc_export(self.vals.ptr), p.ipc_export(sptr), p.ipc_export(self.out.ptr))
        except Exception as e:  # noqa: BLE001
            print(f"rank {self.rank}: hipIpc export unavailable ({e}); xGMI exchange off",
                  file=sys.stderr)
            mine = None
        allh = self.group.all_gather(mine)
        if any(h is None for h in allh):
            return
        tag = self.group.broadcast(uuid.uuid4().hex[:16] if self.rank == 0 else None)
        vptrs, sptrs, optrs, ok = [], [], [], True
        try:
            for r in range(self.world):
                if r == self.rank:
                    vptrs.append(self.vals.ptr)
                    sptrs.append(sptr)
                    optrs.append(self.out.ptr)
                else:
                    vptrs.append(p.ipc_open(allh[r][0]))
                    self._peer_ptrs.append(vptrs[-1])
                    sptrs.append(p.ipc_open(allh[r][1]))
                    self._peer_ptrs.append(sptrs[-1])
                    optrs.append(p.ipc_open(allh[r][2]))
                    self._peer_ptrs.append(optrs[-1])
            x = p.Xgmi(self.world, self.rank, vptrs, sptrs)
            x.set_outs(optrs)
            b = p.NodeBarrier("psg_bench_" + tag, self.world, self.rank)
        except Exception as e:  # noqa: BLE001
            print(f"rank {self.rank}: xGMI mapping failed ({e}); xGMI exchange off", file=sys.stderr)
            ok = False
        if not all(self.group.all_gather(ok)):
            for ptr in self._peer_ptrs:
                p.ipc_close(ptr)
            self._peer_ptrs = []
            return
        self.xgmi, self.node_barrier = x, b
        self.node_barrier.wait()

    def _setup_keyed_cached(self):
        """configs[3] across GPUs with LR key caching: every worker pushes values
        for the same key list; shard r resolves its segment (the DefaultSlicer's,
        psg_slice) once to slots in its SORTED store, and the steady exchange is
        the keyed xGMI pair psg_xgmi_push_slots / _pull_slots over the peers'
        value vectors, stores and slot arrays (hipIpc)."""
        import uuid
        import numpy as np
        p = self.p
        kp = self._key_pos()
        self.kp = [int(x) for x in kp]
        lo, hi = self.kp[self.rank], self.kp[self.rank + 1]
        self.seg = (lo, hi - lo)
        if hi > lo:
            tmp = p.DeviceBuffer((hi - lo) * self.vb)
            # the list's first request inserts its keys (a Pull: operator[] with 0)
            self.store.handle(p.PULL, self.keys.ptr + 8 * lo, None, tmp, hi - lo, stream=self.stream)
            self.slots = p.DeviceBuffer((hi - lo) * 4)
            self.store.resolve(self.keys.ptr + 8 * lo, hi - lo, self.slots, insert=False, stream=self.stream)
        else:
            self.slots = p.DeviceBuffer(4)
        self.sync()
        sptr = self.store.info().vals
        mine = (p.ipc_export(self.vals.ptr), p.ipc_export(sptr), p.ipc_export(self.slots.ptr),
                p.ipc_export(self.out.ptr))
        allh = self.group.all_gather(mine)
        tag = self.group.broadcast(uuid.uuid4().hex[:16] if self.rank == 0 else None)
        self._peer_ptrs = []
        vptrs, sptrs, optrs, self.peer_slots = [], [], [], []
        for r in range(self.world):
            if r == self.rank:
                vptrs.append(self.vals.ptr)
                sptrs.append(sptr)
                self.peer_slots.append(self.slots.ptr)
                optrs.append(self.out.ptr)
            else:
                opened = [p.ipc_open(h) for h in allh[r]]
                self._peer_ptrs += opened
                vptrs.append(opened[0])
                sptrs.append(opened[1])
                self.peer_slots.append(opened[2])
                optrs.append(opened[3])
        self.xgmi = p.Xgmi(self.world, self.rank, vptrs, sptrs)
        self.xgmi.set_outs(optrs)
        self.node_barrier = p.NodeBarrier("psg_bench_" + tag, self.world, self.rank)
        self.seg_offs = np.array(self.kp[:-1], dtype=np.uint64)
        self.seg_ns = np.array([self.kp[w + 1] - self.kp[w] for w in range(self.world)], dtype=np.uint64)
        self.mode = "xgmi-keyed"
        self.node_barrier.wait()

    def _key_pos(self):
        # the worker's DefaultSlicer on its HBM keys (psg_slice), every request
        kp, _ = self.p.slice_keys(self.keys, self.L, self.begins, self.ends, stream=self.stream)
        return kp

    # -- one phase at a time (N = 1, or the sequential RS / AG at N > 1)
    def push(self):
        if self.mode == "xgmi-keyed":
            self.xgmi.push_slots(self.store, self.slots, self.seg[0], self.seg[1], self.stream)
            self.stream.sync()
            self.node_barrier.wait()
            return
        if self.mode == "xgmi-keyed-w":
            # the write form: no barrier between the phases (see pull)
            self.xgmi.push_slots(self.store, self.slots, self.seg[0], self.seg[1], self.stream)
            return
        if self.mode == "xgmi":
            self.xgmi.push(self.store, self.L, self.stream)
            self.stream.sync()
            self.node_barrier.wait()
            return
        if self.mode == "xgmiw":
            # the write form needs no barrier between the phases: the Pull
            # writes this rank's own shard out once its own Push is done
            self.xgmi.push(self.store, self.L, self.stream)
            return
        if self.cached and getattr(self, "stretch", None) is not None:
            self.store.handle_stretch(self.p.PUSH, self.stretch, self.vals, None, self.L, stream=self.stream)
        elif self.cached:
            self.store.handle_slots(self.p.PUSH, self.slots, self.vals, None, self.L, stream=self.stream)
        elif self.keyed:
            # one server: the slice is the whole request (KVWorker's DefaultSlicer
            # skips the kernel for a single range; the store's range check covers it)
            if self.comm is None:
                # launched without waiting for its completion word: the next
                # request queues behind it on the stream (psg_store_handle_async);
                # sync() reaps them all and raises any failure
                self.store.handle_async(self.p.PUSH, self.keys, self.vals, None, self.L, stream=self.stream)
            else:
                self.comm.push_keyed(self.store, self.keys, self.vals, self.L, self._key_pos(), self.stream)
        elif self.comm is None:
            self.store.handle(self.p.PUSH, None, self.vals, None, self.L, first_key=0,
                              stream=self.stream)
        else:
            self.comm.push(self.store, self.vals, self.L, self.scratch, self.stream)

    def pull(self):
        if self.mode == "xgmi-keyed":
            self.xgmi.pull_slots(self.store, self.peer_slots, self.seg_offs, self.seg_ns, self.out,
                                 self.stream)
            self.stream.sync()
            self.node_barrier.wait()
            return
        if self.mode == "xgmi-keyed-w":
            # this rank's segment, read through its own slots, written into every
            # rank's output; outputs complete after every rank's writes
            self.xgmi.pull_write_slots(self.store, self.slots, self.seg[0], self.seg[1], self.stream)
            self.stream.sync()
            self.node_barrier.wait()
            return
        if self.mode == "xgmi":
            self.xgmi.pull(self.store, self.out, self.L, self.stream)
            self.stream.sync()
            self.node_barrier.wait()
            return
        if self.mode == "xgmiw":
            # every rank writes its shard into every output; an output is
            # complete when all ranks' writes are (sync, then one barrier)
            self.xgmi.pull_write(self.store, self.L, self.stream)
            self.stream.sync()
            self.node_barrier.wait()
            return
        if self.cached and getattr(self, "stretch", None) is not None:
            self.store.handle_stretch(self.p.PULL, self.stretch, None, self.out, self.L, stream=self.stream)
        elif self.cached:
            self.store.handle_slots(self.p.PULL, self.slots, None, self.out, self.L, stream=self.stream)
        elif self.keyed:
            if self.comm is None:
                self.store.handle_async(self.p.PULL, self.keys, None, self.out, self.L, stream=self.stream)
            else:
                self.comm.pull_keyed(self.store, self.keys, self.out, self.L, self._key_pos(), self.stream)
        elif self.comm is None:
            self.store.handle(self.p.PULL, None, None, self.out, self.L, first_key=0,
                              stream=self.stream)
        else:
            self.comm.pull(self.store, self.out, self.L, self.stream)

    # -- both, pipelined over buckets (N > 1)
    def step(self):
        if self.mode == "xgmi":
            self._xgmi_double_buffered_step()
            return
        if self.mode == "xgmiw":
            self._xgmi_write_step()
            return
        self.comm.push_pull(self.store, self.vals, self.out, self.L, self.nbuckets, self.stream)

    def _xgmi_double_buffered_step(self):
        """configs[4]'s double-buffered step over xGMI: every chunk's Push is
        queued on the main stream; the Pull of chunk c goes on a second stream
        as soon as every rank has pushed chunk c (a node barrier per chunk), so
        it runs while the Push of chunk c + 1 is in flight.  A last barrier
        after the Pulls keeps the next step's Push off shards a peer still reads."""
        p = self.p
        if getattr(self, "stream2", None) is None:
            self.stream2 = p.Stream()
        unit = 16 // self.vb
        chunk = ((self.blk + self.nbuckets - 1) // self.nbuckets + unit - 1) // unit * unit
        bounds = [(off, min(chunk, self.blk - off)) for off in range(0, self.blk, chunk)]
        evs = getattr(self, "_db_events", [])
        while len(evs) < len(bounds):
            evs.append(p.Event())
        self._db_events = evs
        for i, (off, cnt) in enumerate(bounds):
            self.xgmi.push_range(self.store, self.L, off, cnt, self.stream)
            evs[i].record(self.stream)
        for i, (off, cnt) in enumerate(bounds):
            evs[i].sync()
            self.node_barrier.wait()  # every rank has pushed chunk i
            self.xgmi.pull_range(self.store, self.out, self.L, off, cnt, self.stream2)
        self.stream2.sync()
        self.node_barrier.wait()

    def _xgmi_write_step(self):
        """The write form double-buffered: chunk c's Push (reads the peers:
        ingress) on the main stream; chunk c's Pull as writes (egress) on a
        second stream once this rank's own Push of chunk c is done (an event,
        no barrier), so the two directions of every xGMI link carry the two
        phases at once.  One barrier per step, after both streams drain."""
        p = self.p
        if getattr(self, "stream2", None) is None:
            self.stream2 = p.Stream()
        unit = 16 // self.vb
        chunk = ((self.blk + self.nbuckets - 1) // self.nbuckets + unit - 1) // unit * unit
        bounds = [(off, min(chunk, self.blk - off)) for off in range(0, self.blk, chunk)]
        evs = getattr(self, "_db_events", [])
        while len(evs) < len(bounds):
            evs.append(p.Event())
        self._db_events = evs
        for i, (off, cnt) in enumerate(bounds):
            self.xgmi.push_range(self.store, self.L, off, cnt, self.stream)
            evs[i].record(self.stream)
            self.stream2.wait(evs[i])
            self.xgmi.pull_write_range(self.store, self.L, off, cnt, self.stream2)
        self.stream2.sync()
        self.stream.sync()
        self.node_barrier.wait()

    def _set_mode(self, cand):
        mode, nb = cand
        self.mode, self.nbuckets = mode, nb
        self.fused = nb > 1

    def calibrate(self, iters=3):
        """Pick the exchange for this node by timing each candidate a few times
        (wall clock, barrier-synced): RCCL reduce-scatter then all-gather, the
        RCCL pipelined over 4/8/16 buckets, or the one-shot xGMI kernels.  The
        max over ranks decides, so every rank picks the same."""
        self.pushes_in_calibration = 0
        if self.world == 1:
            return
        if self.keyed:
            if self.mode.startswith("xgmi-keyed"):
                self._calibrate_keyed(iters)
            return
        first = 0
        if self.comm is not None:
            self._first_collective()
            first = 1  # one Push (and Pull) outside the timing
        cands = [("rccl", 1), ("rccl", 4), ("rccl", 8), ("rccl", 16)] if self.comm is not None else []
        two_stream = [("xgmi", 2), ("xgmi", 4), ("xgmiw", 2), ("xgmiw", 4)]
        if self.xgmi is not None:
            cands += [("xgmi", 0), ("xgmiw", 0)]
            # the double-buffered steps add a second stream per rank; with every
            # rank on ONE GPU (test mode) that oversubscribes the hardware queues
            # and slows every later step ~4x (measured at N = 8), so test mode
            # times them only when forced
            if not self.share_gpu:
                cands += two_stream
        forced = os.environ.get("PSG_BENCH_EXCHANGE")  # testing: e.g. "xgmi/4", "xgmiw/2", "rccl/1"
        if forced and self.xgmi is not None:
            cands += [c for c in two_stream if c not in cands]
        if forced:
            m, _, nb = forced.partition("/")
            cands = [c for c in cands if c == (m, int(nb or 0))]
            if not cands:
                raise SystemExit(f"PSG_BENCH_EXCHANGE={forced}: not available here")
        times = []
        for cand in cands:
            self._set_mode(cand)
            self._one_step()
            self.sync()
            self.group.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                self._one_step()
            self.sync()
            times.append((time.perf_counter() - t0) * 1e3 / iters)
            self.group.barrier()
        t = self.group.allreduce_max(times)
        order = sorted(range(len(cands)), key=lambda i: t[i])
        self._set_mode(cands[order[0]])
        self.calibration = {f"{m}{'' if nb == 0 else '/' + str(nb)}": round(x, 4)
                            for (m, nb), x in zip(cands, t)}
        self.pushes_in_calibration = len(cands) * (iters + 1) + first
        if self.mode in ("xgmi", "xgmiw"):
            self.pushes_in_calibration += 1
            self.exchange_verified = self._verify_xgmi()
            if not self.exchange_verified:
                rest = [cands[i] for i in order if not cands[i][0].startswith("xgmi")]
                if not rest:
                    raise RuntimeError("xGMI exchange failed its checksum verification "
                                       "and no RCCL communicator is available")
                print("xGMI exchange failed its checksum verification; using RCCL",
                      file=sys.stderr)
                self._set_mode(rest[0])

    def _first_collective(self):
        """The first RCCL step (it also sets up the peer connections) waited for
        against PSG_COMM_TIMEOUT_S (psg_comm_sync): if it does not complete on
        every rank, every rank aborts its communicators and the exchange is the
        xGMI kernels alone — a transport that never connects ends in a fallback,
        not a hang."""
        ok = True
        self._set_mode(("rccl", 1))
        try:
            self._one_step()
            self.comm.sync(self.stream)
        except Exception as e:  # noqa: BLE001
            print(f"rank {self.rank}: first RCCL step failed ({e})", file=sys.stderr)
            ok = False
        if not all(self.group.all_gather(ok)):
            self.comm.abort()
            self.comm = None
            self.first_collective_failed = True

    def _calibrate_keyed(self, iters):
        """The key-cached xGMI exchange: the read-form Pull (psg_xgmi_pull_slots)
        or the write form (psg_xgmi_pull_write_slots), whichever runs faster
        here (max over ranks).  PSG_BENCH_EXCHANGE=xgmi-keyed / xgmi-keyed-w forces one."""
        cands = ["xgmi-keyed", "xgmi-keyed-w"]
        forced = os.environ.get("PSG_BENCH_EXCHANGE")
        if forced:
            cands = [c for c in cands if c == forced]
            if not cands:
                raise SystemExit(f"PSG_BENCH_EXCHANGE={forced}: not available here")
        times = []
        for c in cands:
            self.mode = c
            self._one_step()
            self.sync()
            self.group.barrier()
            t0 = time.perf_counter()
            for _ in range(iters):
                self._one_step()
            self.sync()
            times.append((time.perf_counter() - t0) * 1e3 / iters)
            self.group.barrier()
        t = self.group.allreduce_max(times)
        self.mode = cands[min(range(len(cands)), key=lambda i: t[i])]
        self.calibration = {c: round(x, 4) for c, x in zip(cands, t)}
        self.pushes_in_calibration = len(cands) * (iters + 1)

    def _verify_xgmi(self) -> bool:
        """One xGMI Push + Pull, then every rank's pulled block w must carry the
        same psg_checksum as rank w's own shard (read locally): catches a stale
        or torn cross-GPU read before the timed steps rely on the path."""
        p = self.p
        self.push()
        self.pull()
        nb = self.blk * self.vb
        mine = p.checksum(self.store.info().vals, nb, self.stream)
        got = [p.checksum(self.out.ptr + w * nb, nb, self.stream) for w in range(self.world)]
        owners = self.group.all_gather(mine)
        return all(self.group.all_gather(got == owners))

    def _one_step(self):
        if self.fused:
            self.step()
        else:
            self.push()
            self.pull()

    def new_event(self):
        return self.p.Event(timing=TIMING_EVENTS)

    def record(self, e):
        e.record(self.stream)

    def elapsed(self, a, b) -> float:
        return a.elapsed_ms(b)

    def sync(self):
        if self.keyed and self.store is not None:
            self.store.wait()  # the keyed requests in flight, their follow-ups and failures
        self.stream.sync()
        self.p.device_sync()

    def accumulate_probe(self, iters=10):
        """The dominant local kernel at N > 1: the shard accumulate after the
        reduce-scatter (12 B per f32 element), timed alone with HIP events.
        Runs after the parity check: it changes the shards."""
        if self.keyed:
            return None
        a, b = self.new_event(), self.new_event()
        self.record(a)
        for _ in range(iters):
            if self.mode in ("xgmi", "xgmiw"):
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
        if self.mode in ("xgmi", "xgmiw"):
            # store read + write (8 B) + one 4-B value from every rank's vector
            return ("k_xgmi_push (fused reduce of %d ranks' blocks + accumulate; "
                    "%d of them read over xGMI)" % (self.world, self.world - 1),
                    (8 + self.vb * self.world) * self.blk)
        return ("k_dense_vec<PUSH> on the shard after the reduce-scatter",
                PUSH_ACCESSES * self.vb * self.blk)

    def check(self, steps_done: int) -> dict:
        """After `steps_done` pushes every shard holds steps * sum_w vals_w
        (integer-valued, exact).  One more Pull, then:
          device  every element of the pulled vector — every rank's block, i.e.
                  the peers' shards as they arrived over the exchange — against
                  the closed form (psg_verify_synth_sum);
          oracle  a sample at the start of every block w replayed through the
                  CPU restatement of KVServerDefaultHandle (oracle.Store): each
                  worker's Push of every step as one request, in worker order."""
        import numpy as np
        import oracle
        p = self.p
        self.pull()
        self.sync()
        bad, first = p.verify_synth_sum(self.out, self.L, self.dt, self._seed, self.world,
                                        0.0, self.hi(), float(steps_done), stream=self.stream)
        npt = {p.F32: np.float32, p.F16: np.float16}[self.dt]
        odt = {p.F32: oracle.F32, p.F16: oracle.F16}[self.dt]
        m = min(self.blk, 4096)
        sample_ok = True
        for w in range(self.world):
            lo = w * self.blk
            got = self.out.download(npt, m, self.stream, offset=lo * self.vb)
            # element i of worker r's vector is synth(seed + r + i): start the
            # generator at i = lo instead of producing the whole prefix
            src = [oracle.synth(m, odt, self._seed + r + lo, 0, 0.0, self.hi()) for r in range(self.world)]
            st = oracle.Store(odt)
            for _ in range(steps_done):
                for r in range(self.world):
                    st.handle(oracle.PUSH, None, src[r], m, first_key=lo)
            exp = st.handle(oracle.PULL, None, None, m, first_key=lo)
            sample_ok &= bool(np.array_equal(got.view(np.uint16) if self.dt == p.F16 else got,
                                             exp))
        return {"ok": bad == 0 and sample_ok, "device_mismatches": bad, "first_bad": first,
                "oracle_sample_ok": sample_ok, "elements": self.L, "oracle_sample": m * self.world}

    def probe_256m(self, n=256 << 20, iters=20):
        """The north star's own target: one 256 M-float Push (and Pull) on the
        DENSE store, HIP-event timed on the kernels' stream (N = 1)."""
        p = self.p
        st = p.Store(p.DENSE, p.F32, 0, n, n)
        v, o = p.DeviceBuffer(n * 4), p.DeviceBuffer(n * 4)
        v.fill_synth(n, p.F32, self._seed, 0, 0.0, 1000.0, self.stream)
        warm = 5
        for _ in range(warm):
            st.handle(p.PUSH, None, v, None, n, stream=self.stream)
            st.handle(p.PULL, None, None, o, n, stream=self.stream)
        # The step of the workload — Push then Pull — with one event between
        # launches (~4 us of a ~0.5 ms launch); medians, so a stray slow launch
        # does not move them.  Back-to-back Pushes alone run ~10 % slower on
        # this store (measured: 0.69 vs 0.785 of HBM) and are reported beside.
        import statistics
        ev = [p.Event(timing=TIMING_EVENTS) for _ in range(2 * iters + 1)]
        ev[0].record(self.stream)
        for i in range(iters):
            st.handle(p.PUSH, None, v, None, n, stream=self.stream)
            ev[2 * i + 1].record(self.stream)
            st.handle(p.PULL, None, None, o, n, stream=self.stream)
            ev[2 * i + 2].record(self.stream)
        eb = [p.Event(timing=TIMING_EVENTS) for _ in range(iters + 1)]
        eb[0].record(self.stream)
        for i in range(iters):
            st.handle(p.PUSH, None, v, None, n, stream=self.stream)
            eb[i + 1].record(self.stream)
        self.sync()
        push_ms = statistics.median(ev[2 * i].elapsed_ms(ev[2 * i + 1]) for i in range(iters))
        pull_ms = statistics.median(ev[2 * i + 1].elapsed_ms(ev[2 * i + 2]) for i in range(iters))
        b2b_ms = statistics.median(eb[i].elapsed_ms(eb[i + 1]) for i in range(iters))
        bad, _ = p.verify_synth_sum(o, n, p.F32, self._seed, 1, 0.0, 1000.0, float(warm + iters),
                                    stream=self.stream)  # the last Pull, before the b2b Pushes
        # this process's own copy ceiling on the same two buffers: the Pull's
        # traffic is exactly a copy's (read 1 GiB, write 1 GiB), so the best of
        # a few shapes of the plain float4 streaming copy kernel (psg_copy:
        # vectors per lane in flight x blocks per CU) is what this GPU and this
        # process's page placement give the Pull (MI355X_MICROARCH.md quotes
        # 6.29 TB/s from one box; processes on one box differ by up to 10 %)
        self.sync()
        copy_shapes = {}
        for unroll, bpc in ((1, 4), (2, 2), (4, 2), (4, 3), (8, 2)):
            for _ in range(2):
                p.copy(o, v, n * 4, unroll, bpc, stream=self.stream)
            ec = [p.Event(timing=TIMING_EVENTS) for _ in range(11)]
            ec[0].record(self.stream)
            for i in range(10):
                p.copy(o, v, n * 4, unroll, bpc, stream=self.stream)
                ec[i + 1].record(self.stream)
            self.sync()
            copy_shapes[f"U{unroll}x{bpc}/CU"] = statistics.median(ec[i].elapsed_ms(ec[i + 1]) for i in range(10))
        best_shape = min(copy_shapes, key=copy_shapes.get)
        copy_ms = copy_shapes[best_shape]
        em = [p.Event(timing=TIMING_EVENTS) for _ in range(11)]
        for _ in range(2):
            p.memcpy_d2d(o, v, n * 4, stream=self.stream)
        em[0].record(self.stream)
        for i in range(10):
            p.memcpy_d2d(o, v, n * 4, stream=self.stream)
            em[i + 1].record(self.stream)
        self.sync()
        memcpy_ms = statistics.median(em[i].elapsed_ms(em[i + 1]) for i in range(10))
        st.close()
        v.free()
        o.free()
        out = {"keys": n, "push_ms": round(push_ms, 5), "pull_ms": round(pull_ms, 5),
               "parity_check": bad == 0}
        for name, ms, acc in (("push", push_ms, PUSH_ACCESSES), ("pull", pull_ms, PULL_ACCESSES)):
            gbs = acc * 4 * n / (ms * 1e-3) / 1e9
            out[f"{name}_achieved"] = round(gbs, 1)
            out[f"{name}_frac"] = round(gbs / HBM_PEAK_GBS, 4)
        out["push_back_to_back_frac"] = round(PUSH_ACCESSES * 4 * n / (b2b_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        copy_gbs = 2 * 4 * n / (copy_ms * 1e-3) / 1e9
        out["copy_ceiling"] = {"what": "psg_copy float4 streaming copy of the same 1 GiB (read + write bytes), "
                                       "best median of 5 shapes, same process and buffers",
                               "best_shape": best_shape, "ms": round(copy_ms, 5), "achieved": round(copy_gbs, 1),
                               "frac": round(copy_gbs / HBM_PEAK_GBS, 4),
                               "shapes_ms": {k: round(x, 5) for k, x in copy_shapes.items()},
                               "push_of_copy": round(out["push_achieved"] / copy_gbs, 4),
                               "pull_of_copy": round(out["pull_achieved"] / copy_gbs, 4),
                               "hipmemcpy_d2d_achieved": round(2 * 4 * n / (memcpy_ms * 1e-3) / 1e9, 1)}
        out["kernel"] = "k_dense_vec<PUSH> / <PULL>, 12 / 8 B per float"
        return out


class _LocalGroup:
    """World of one (no peers)."""
    rank, world = 0, 1

    def all_gather(self, obj):
        return [obj]

    def broadcast(self, obj=None, src=0):
        return obj

    def barrier(self):
        pass

    def allreduce_max(self, xs):
        return list(xs)

    def close(self):
        pass


def run(backend, args, rank: int, world: int, group=None) -> dict | None:
    L = args.keys
    assert L % world == 0, "keys must divide by the number of shards"
    group = group or _LocalGroup()
    backend._seed = args.seed
    backend.max_pushes = args.warmup + args.steps + EXTRA_PUSH_BOUND
    backend.setup(L, args.seed)
    extra_pushes = 0
    if hasattr(backend, "calibrate") and world > 1:
        backend.calibrate()
        extra_pushes = getattr(backend, "pushes_in_calibration", 0)
    fused = getattr(backend, "fused", False)

    def one_step():
        if fused:
            backend.step()
        else:
            backend.push()
            backend.pull()

    for _ in range(args.warmup):
        one_step()
        if getattr(backend, "keyed", False):
            # reap each warm-up step: a keyed list's windows are trusted (and its
            # identity trial decided) when its first requests are reaped, so the
            # warm-up then reaches the steady-state kernels — and loads their
            # code objects — before the timed region
            backend.sync()
    # Kernel times come from HIP events recorded live in the timed region, on
    # every `event_every`-th step only: a marker is not free on ROCm (each one
    # measured ~4 us of the ~0.19 ms step), so the other steps run unperturbed.
    # Sampled step k: e0 | Push k | e1 | Pull k | e2.
    every = max(1, getattr(args, "event_every", 1))
    sampled = [k for k in range(args.steps) if k % every == 0]
    evs = {k: (backend.new_event(), backend.new_event(), backend.new_event()) for k in sampled}
    backend.sync()
    group.barrier()
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
    group.barrier()
    t1 = time.perf_counter()
    local_ms = (t1 - t0) * 1e3 / max(args.steps, 1)
    n_marks = max(len(sampled), 1)
    push_ms = sum(backend.elapsed(a, b) for a, b, _ in evs.values()) / n_marks
    pull_ms = sum(backend.elapsed(b, c) for _, b, c in evs.values()) / n_marks
    batched = None
    if world == 1 and getattr(backend, "cached", False) and getattr(backend, "stretch", None) is not None:
        # The LR steady state's per-request cost without a marker per request
        # (VERDICT r4 next #5): BATCHED Pushes back to back, then as many Push ->
        # Pull steps, each batch between one pair of the same timing-only events.
        # A marker costs ~1-2 us on ROCm, so e0 | Push | e1 charges a ~20 us
        # Push with two of them; here they are shared by the batch.
        a, b, c = backend.new_event(), backend.new_event(), backend.new_event()
        backend.record(a)
        for _ in range(BATCHED):
            backend.push()
        backend.record(b)
        for _ in range(BATCHED):
            backend.push()
            backend.pull()
        backend.record(c)
        backend.sync()
        batched = {"requests": BATCHED, "push_ms": round(backend.elapsed(a, b) / BATCHED, 5),
                   "step_ms": round(backend.elapsed(b, c) / BATCHED, 5)}
        # ... next to the same Pushes with a marker between every two (the
        # per-request line's timing) and to the markers alone (VERDICT r5 next
        # #4): marker_ms is what one marker adds to the stream, so
        # per_request_push_ms - push_ms should equal it if markers explain the gap
        em = [backend.new_event() for _ in range(BATCHED + 1)]
        backend.record(em[0])
        for i in range(BATCHED):
            backend.push()
            backend.record(em[i + 1])
        mk = [backend.new_event() for _ in range(BATCHED + 1)]
        for e in mk:
            backend.record(e)
        backend.sync()
        batched["per_request_push_ms"] = round(sum(backend.elapsed(em[i], em[i + 1]) for i in range(BATCHED))
                                               / BATCHED, 5)
        batched["marker_ms"] = round(backend.elapsed(mk[0], mk[-1]) / BATCHED, 5)
        batched["gap_ms"] = round(batched["per_request_push_ms"] - batched["push_ms"], 5)
        extra_pushes += 3 * BATCHED
    total_pushes = args.warmup + args.steps + extra_pushes
    chk = None
    if args.check:
        # the whole pulled vector at every N, before anything else touches the shards
        chk = backend.check(total_pushes)
        if not isinstance(chk, dict):
            chk = {"ok": bool(chk)}
    acc_ms = backend.accumulate_probe() if (world > 1 and hasattr(backend, "accumulate_probe")) else None
    # every rank's device, GPU and RCCL view, gathered for the line (N > 1)
    ranks = group.all_gather(backend.describe()) if (world > 1 and hasattr(backend, "describe")) else None
    ms, push_ms, pull_ms, acc = group.allreduce_max([local_ms, push_ms, pull_ms, acc_ms or 0.0])
    acc_ms = acc if acc_ms is not None else None
    ok = None
    if chk is not None:
        oks = group.all_gather(bool(chk["ok"]))
        ok = all(oks)
    if rank != 0:
        return None
    vb = getattr(backend, "vb", 4)
    payload = 2 * vb * L * world  # pushed + pulled by all workers per step
    value_gbs = payload / (ms * 1e-3) / 1e9
    blk = L // world
    wl = getattr(args, "workload", "dense")
    spec = WORKLOADS.get(wl, WORKLOADS["dense"])
    cfg = spec[4] if world == 1 else spec[5]
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
        "dtype": spec[0],
        "data": "synthetic (integer-valued floats, seed 7+rank, generated in HBM)",
        "config": {
            "workload": (f"{cfg}: "
                         + (("keyed (10 M sorted uint64 keys, SORTED store), " if wl.startswith("keyed") else "dense, ")
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
    if chk is not None and world == 1:
        res["parity_detail"] = {k: v for k, v in chk.items() if k != "ok"}
    elif chk is not None:
        res["parity_detail"] = {"checked": "every rank's whole pulled vector on the device "
                                           "+ an oracle replay at the start of every block",
                                "elements_per_rank": L}
    if world > 1 and hasattr(backend, "nbuckets"):
        if getattr(backend, "mode", "rccl") == "xgmi" and fused:
            res["config"]["exchange"] = ("xGMI kernels double-buffered over %d chunks: chunk c's Pull on a "
                                         "second HIP stream while chunk c+1's Push runs" % backend.nbuckets)
        elif getattr(backend, "mode", "rccl") == "xgmi":
            res["config"]["exchange"] = "one-shot xGMI kernels (psg_xgmi push/pull, peers via hipIpc)"
        elif getattr(backend, "mode", "rccl") == "xgmiw" and fused:
            res["config"]["exchange"] = ("xGMI Push (reads the peers) with the Pull as writes into every "
                                         "rank's output, double-buffered over %d chunks on two HIP streams: "
                                         "the two directions of each link at once" % backend.nbuckets)
        elif getattr(backend, "mode", "rccl") == "xgmiw":
            res["config"]["exchange"] = ("xGMI Push (reads the peers) then the Pull as writes into every "
                                         "rank's output (psg_xgmi_pull_write); one barrier per step")
        elif getattr(backend, "mode", "") == "xgmi-keyed":
            res["config"]["exchange"] = ("keyed xGMI kernels on cached slots (psg_xgmi_push_slots / "
                                         "_pull_slots over the peers' values, stores and slot lists)")
        elif getattr(backend, "mode", "") == "xgmi-keyed-w":
            res["config"]["exchange"] = ("keyed xGMI kernels on cached slots, the Pull as writes "
                                         "(psg_xgmi_push_slots / _pull_write_slots into every rank's output)")
        elif getattr(backend, "keyed", False):
            res["config"]["exchange"] = "RCCL grouped reduce / broadcast of the key-range segments"
        else:
            res["config"]["exchange"] = ("RCCL pipelined reduce/broadcast, %d buckets" % backend.nbuckets
                                         if fused else "RCCL reduce-scatter then all-gather")
        res["config"]["calibration_ms"] = getattr(backend, "calibration", None)
        if getattr(backend, "first_collective_failed", False):
            res["config"]["rccl"] = ("aborted on every rank: the first collective did not complete within "
                                     "PSG_COMM_TIMEOUT_S (psg_comm_sync); xGMI kernels only")
        if hasattr(backend, "exchange_verified"):
            res["config"]["xgmi_checksum_verified"] = backend.exchange_verified
        if getattr(backend, "share_gpu", False):
            res["config"]["shared_gpu_test_mode"] = True
    if ranks is not None:
        # which device, GPU (PCI bus id, host) and RCCL rank each rank had, and
        # the exchange calibration: the first N-GPU line proves its own layout
        res["config"]["ranks"] = ranks
        res["config"]["distinct_gpus"] = len({(d.get("host"), d.get("pci_bus_id")) for d in ranks})
        res["config"].setdefault("calibration_ms", getattr(backend, "calibration", None))
    if world == 1 and getattr(backend, "cached", False) and getattr(backend, "stretch", None) is not None:
        # the cached list resolved to a stretch of slots: no slot stream, so the
        # request's bytes are those of the dense op on that stretch
        res["roofline"] = roofline(STRETCH_PUSH_BYTES * L, push_ms, args,
                                   "cached-list Push on a stretch of slots: k_dense_vec<PUSH> on "
                                   "store[first, first + n) (psg_store_handle_stretch; the list's one "
                                   "resolve found slots[i] == first + i)", vb)
        res["pull_roofline_frac"] = round(8 * L / (pull_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        res["config"]["cached_slots"] = "stretch from slot %d" % backend.stretch
        if batched:
            batched["push_frac"] = round(STRETCH_PUSH_BYTES * L / (batched["push_ms"] * 1e-3) / 1e9
                                         / HBM_PEAK_GBS, 4)
            batched["step_gbs"] = round(2 * vb * L / (batched["step_ms"] * 1e-3) / 1e9, 1)
            batched["what"] = (f"{BATCHED} Pushes back to back, then {BATCHED} Push -> Pull steps, each batch "
                               "between one pair of timing-only events: the per-request cost of a steady "
                               "request stream, dispatch included, without a marker per request; "
                               f"per_request_push_ms: {BATCHED} Pushes with a marker after each; marker_ms: "
                               f"{BATCHED + 1} markers recorded back to back with no kernel, per marker; "
                               "gap_ms = per_request_push_ms - push_ms")
            batched["per_request_push_frac"] = round(STRETCH_PUSH_BYTES * L / (batched["per_request_push_ms"]
                                                                                * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
            res["roofline"]["batched"] = batched
    elif world == 1 and getattr(backend, "cached", False):
        res["roofline"] = roofline(CACHED_PUSH_BYTES * L, push_ms, args,
                                   "cached-slot Push: k_slots_vec (store[slot] += val, slots "
                                   "from the one resolve of the key list)", vb)
        res["pull_roofline_frac"] = round(12 * L / (pull_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    elif world == 1 and getattr(backend, "keyed", False):
        # which kernels served the run's keyed requests (psg_store_counters):
        # the identity pair once the key list's windows are trusted
        paths = backend.store.counters()
        res["keyed_paths"] = paths
        if getattr(backend, "store_extra", 0):
            res["config"]["store_keys"] = (f"{backend.store_extra + 1} x the request's: the request is every "
                                           f"{backend.store_extra + 1}-th store key (PSG_BENCH_STORE_EXTRA)")
            # the least HBM a Push at this density can move per request key:
            # its key 8 + value 4, the store keys its windows span 8 (e + 1),
            # and the 4-B store values of every line it touches, read and
            # written (whole 64-B lines while 4 (e + 1) <= 64)
            e1 = backend.store_extra + 1
            res["config"]["push_min_bytes_per_key"] = 12 + 8 * e1 + 2 * min(4 * e1, 64)
        if getattr(backend, "store_subset", None):
            res["config"]["store_keys"] = (f"{backend.store_subset[1]} keys: the request is a random subset of the "
                                           f"store at density {backend.store_subset[0]} (PSG_BENCH_SUBSET)")
        if getattr(backend, "store_stretches", 0):
            res["config"]["store_keys"] = (f"the request is a union of {backend.store_stretches} stretches of the "
                                           "store (4096 store keys it lacks in each seam, PSG_BENCH_STRETCHES)")
        if paths["ident"] > 0 and paths["notident"] == 0:
            kname = ("SORTED-store Push: k_ident_check + k_ident_apply (identity request: the key "
                     "list is the stretch K[D, D + n) of the store's keys, D from its first tile's "
                     "cached window, so key i sits at slot D + i; the check — request key = store "
                     "key, 16 B/key — is the whole validation, then values only, 12 B/key; "
                     "requests in flight, each reporting completion and flags in one "
                     "kernel-written word; one server, so no slicer pass)")
        elif paths.get("lists", 0) > paths.get("coded", 0):  # most Pushes took the verified copy
            kname = ("SORTED-store Push: k_list_check + k_tile_apply_db "
                     "(the list's verified copy: the request keys compared with the copy a "
                     "learning Push of this list kept — its first lean Push at this K, "
                     "validated in full by k_validate_code — 16 B/key, no store-key lines; "
                     "tile kinds from the cached windows; then the lean apply from the lane "
                     "codes; a list that differs from its copy writes nothing and is "
                     "validated in full; requests in flight, each reporting completion and "
                     "flags in one kernel-written word; one server, so no slicer pass)")
        elif paths.get("coded", 0) == 0:
            kname = ("SORTED-store Push: k_validate_windows + k_resolve_apply "
                     "(whole-request validation before any write; each tile searches "
                     "its window in LDS; tile windows cached per key array; requests "
                     "in flight, each reporting completion and flags in one "
                     "kernel-written word; one server, so no slicer pass)")
        elif 2 * paths.get("lean", 0) > paths["coded"]:  # most coded Pushes went lean
            kname = ("SORTED-store Push: k_validate_code + k_tile_apply_db "
                     "(whole-request validation before any write, which also sorts the "
                     "tiles on trusted windows; the lean apply then takes stretches of "
                     "the store at slots lo + i and subsets of their window at places "
                     "from lane codes cached with the windows and verified each request "
                     "(a coded tile's window staged into LDS while the block's previous "
                     "tile is applied) — no key re-read, no search; a general tile, if one appears, is "
                     "applied by a follow-up on the general path and the list stays "
                     "there until the store's keys change; requests in flight, each "
                     "reporting completion and flags in one kernel-written word; one "
                     "server, so no slicer pass)")
        else:
            kname = ("SORTED-store Push: k_validate_code + k_resolve_apply "
                     "(whole-request validation before any write, which also sorts the "
                     "tiles on trusted windows: stretches of the store are applied at "
                     "slots lo + i, subsets of their window at places from lane codes "
                     "cached with the windows and verified each request — neither "
                     "re-reads its keys or searches; other tiles search their window "
                     "in LDS; requests in flight, each reporting completion and flags "
                     "in one kernel-written word; one server, so no slicer pass)")
        # the store layout the PMC summary must have been taken on (a random
        # subset moves more lines than a union of stretches)
        layout = ""
        if getattr(backend, "store_subset", None):
            layout = f"subset{backend.store_subset[0]}"
        elif getattr(backend, "store_stretches", 0):
            layout = f"stretch{backend.store_stretches}"
        elif not getattr(backend, "store_extra", 0) and not (paths["ident"] > 0 and paths["notident"] == 0):
            layout = "general"
        res["roofline"] = roofline(KEYED_PUSH_BYTES * L, push_ms, args, kname, vb,
                                   store_extra=getattr(backend, "store_extra", 0), layout=layout)
        res["pull_roofline_frac"] = round(24 * L / (pull_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
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
    if world == 1 and wl == "dense" and res.get("roofline"):
        # the 64 M store (256 MiB) stays in the 256 MiB Infinity Cache between
        # the Push and the Pull, so this fraction is IC-assisted, not pure HBM;
        # the pure-HBM figure is the 256 M north-star probe below
        store_mib = vb * blk / 2**20
        res["roofline"]["infinity_cache_assisted"] = store_mib <= 256
        res["roofline"]["store_mib"] = round(store_mib, 1)
    if (world == 1 and wl == "dense" and hasattr(backend, "probe_256m")
            and not getattr(args, "no_probe256", False)):
        res["push256_roofline"] = backend.probe_256m()
        if res.get("roofline"):
            res["roofline"]["hbm_only_frac_256m"] = res["push256_roofline"]["push_frac"]
            res["roofline"]["hbm_only_note"] = ("push256_roofline: the same Push kernel on a 1 GiB store "
                                                "(256 M floats), past the Infinity Cache")
    if world == 1 and not args.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline(args)
    res["runtime_libs"] = mapped_runtime_libs()
    res["event_markers"] = ("timing-only (hipEventDisableSystemFence)" if TIMING_EVENTS
                            else "default (system-scope fence at each record)")
    return res


def run_lr(args) -> dict:
    """The LR server's sync round on one GPU (configs[3]'s LRServer apply,
    LRServer.h:151-178 + Adam.h:28-34): `frames` gradient frames merged from 0 in
    arrival order and the Adam step over `keys` features, one launch of
    k_lr_apply_sum per step (psg_lr_apply_sum), everything resident in HBM.
    value = algorithmic HBM bytes per round (4 B per frame + weight 8 + f64
    moments 32, per feature) / ms_per_step.  Parity: the first 4096 features
    replayed round by round by the oracle's restatement (bit-exact)."""
    import numpy as np
    import psg as p
    n, frames, lr = args.keys, args.lr_frames, float(np.float32(0.01))
    p.set_device(0)
    st = p.Stream()
    w = p.Store(p.DENSE, p.F32, 0, n, n)
    init = p.DeviceBuffer(n * 4)
    init.fill_synth(n, p.F32, args.seed, 1, -0.5, 0.5, st)
    w.handle(p.PUSH, None, init, None, n, stream=st)
    grads = [p.DeviceBuffer(n * 4) for _ in range(frames)]
    for j, g in enumerate(grads):
        g.fill_synth(n, p.F32, args.seed + 100 + j, 1, -1.0, 1.0, st)
    adam = p.Adam(n, lr)
    st.sync()
    sample = 4096
    w0 = init.download(np.float32, sample)
    g0 = [g.download(np.float32, sample) for g in grads]
    init.free()
    it = 0
    for _ in range(args.warmup):
        p.lr_apply_sum(w, grads, n, 0.01, adam, it, stream=st)
        it += 1
    ev = [p.Event(timing=TIMING_EVENTS) for _ in range(args.steps + 1)]
    st.sync()
    t0 = time.perf_counter()
    ev[0].record(st)
    for i in range(args.steps):
        p.lr_apply_sum(w, grads, n, 0.01, adam, it, stream=st)
        it += 1
        ev[i + 1].record(st)
    st.sync()
    ms = (time.perf_counter() - t0) * 1e3 / args.steps
    kernel_ms = sum(ev[i].elapsed_ms(ev[i + 1]) for i in range(args.steps)) / args.steps
    per = 4 * frames + 8 + 32
    buf = p.DeviceBuffer(n * 4)
    w.handle(p.PULL, None, None, buf, n, stream=st)
    st.sync()
    got = buf.download(np.float32, sample)
    buf.free()
    # the checker: the oracle's restatement of the same rounds on the sample
    import oracle
    ref = w0.copy()
    m, v = np.zeros(sample), np.zeros(sample)
    for r in range(it):
        merged = np.zeros(sample, np.float32)
        for g in g0:
            merged = (merged + g).astype(np.float32)
        oracle.lr_apply(ref, merged, 0.01, m, v, lr, 0.9, 0.999, 1e-8, r)
    bad = int(np.count_nonzero(got.view(np.uint32) != ref.view(np.uint32)))
    # The copy ceiling of this byte mix: the same kernel's
    # loads and stores with a copy's arithmetic (psg_lr_mix_copy), timed the
    # same way in this process, after the parity sample was read (it
    # scribbles on the weights and moments).
    cev = [p.Event(timing=TIMING_EVENTS) for _ in range(args.steps + 1)]
    for _ in range(2):
        p.lr_mix_copy(w, grads, n, adam, stream=st)
    cev[0].record(st)
    for i in range(args.steps):
        p.lr_mix_copy(w, grads, n, adam, stream=st)
        cev[i + 1].record(st)
    st.sync()
    copy_ms = sum(cev[i].elapsed_ms(cev[i + 1]) for i in range(args.steps)) / args.steps
    adam.close()
    w.close()
    for g in grads:
        g.free()
    gbs = per * n / (ms * 1e-3) / 1e9
    res = {
        "metric": "device-resident LR BSP round GB/s (merge + Adam, algorithmic HBM bytes)",
        "value": round(gbs, 3), "unit": "GB/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 5), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32 merge, f64 Adam", "data": "synthetic (U(-0.5,0.5) weights, U(-1,1) gradients, generated in HBM)",
        "config": {"workload": f"LR BSP round: {frames} gradient frames merged + Adam over {n} features "
                               "(configs[3]'s LRServer sync apply, LRServer.h:151-178, Adam.h:28-34)",
                   "features": n, "frames": frames, "alg_bytes_per_feature": per},
        "parity_check": bad == 0,
        "parity_detail": {"sample": sample, "rounds": it, "mismatches": bad,
                          "oracle": "oracle.lr_apply, bit-exact restatement pinned by tests/golden/lr_ref.npz"},
        "roofline": roofline(per * n, kernel_ms, args, "k_lr_apply_sum<ADAM> (merge + Adam, one launch)", 4),
        "event_markers": ("timing-only (hipEventDisableSystemFence)" if TIMING_EVENTS
                          else "default (system-scope fence at each record)"),
        "copy_ceiling": {"kernel": "k_lr_apply_sum<ADAM, COPY> (psg_lr_mix_copy): the same loads and stores "
                                   "with a copy's arithmetic",
                         "ms": round(copy_ms, 5),
                         "gbs": round(per * n / (copy_ms * 1e-3) / 1e9, 1),
                         "frac": round(per * n / (copy_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "adam_of_copy": round(copy_ms / kernel_ms, 4)},
    }
    if not args.no_cpu_baseline:
        # the same round restated in oracle/ on one core, on a bounded sample
        cn = min(n, args.cpu_lr_features)
        rng = np.random.default_rng(args.seed)
        cw = rng.uniform(-0.5, 0.5, cn).astype(np.float32)
        cg = [rng.uniform(-1, 1, cn).astype(np.float32) for _ in range(frames)]
        cm, cv = np.zeros(cn), np.zeros(cn)
        reps = 3
        t0 = time.perf_counter()
        for r in range(reps):
            merged = np.zeros(cn, np.float32)
            for g in cg:
                merged = (merged + g).astype(np.float32)
            oracle.lr_apply(cw, merged, 0.01, cm, cv, lr, 0.9, 0.999, 1e-8, r)
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(per * cn * reps / dt / 1e9, 4), "unit": "GB/s", "cores": 1,
                               "kind": "port",
                               "sample": f"{cn} features x {reps} rounds ({frames} frames merged with numpy f32 adds, "
                                         f"then oracle.lr_apply's Adam), single thread, {dt:.1f} s",
                               "host": {"nproc": os.cpu_count(), "cpu_model": _cpu_model()}}
    res["runtime_libs"] = mapped_runtime_libs()
    return res


# algorithmic HBM bytes per key of a keyed Pull on the SORTED store: request
# key 8 + store key 8 + store value 4 + reply 4
KEYED_PULL_BYTES = 24


def run_dropin(args, n_gpus: int) -> dict:
    """The drop-in API's own line: tests/harness/
    kv_bench_dropin.cpp — HBM-resident ZPush then ZPull per step through
    KVWorker / KVServer with KVServerDefaultHandle (src/ps/KVApp.h:234-291,
    433-458), ns = nw = N, every node its own process as tests/local.py:87-114
    starts them (--dropin-mode threads: every node a thread of one process, the
    shared-GPU test mode).  Keys: test_kv_app_benchmark.cpp:47-52's
    kMaxKey/num*i + rank (--dropin-layout 0; 1: one list shared by every worker,
    the BSP shape whose Pushes a server serves as runs).  value = 2 * 4 B *
    keys * N / (max over workers of the step time).  The roofline counts each
    request's own algorithmic bytes on the general keyed path (Push 28, Pull 24
    B per key) per GPU.  Parity: every worker checks its whole pulled vector
    against the closed form of its integer-valued pushes, on the device."""
    import subprocess
    n, N = args.keys, n_gpus
    exe = os.path.join(ROOT, "tests", "_bin", "kv_bench_dropin")
    if not os.path.exists(exe):
        raise SystemExit(f"{exe} not built (make -C parameter-server_amd harness)")
    cmd = [exe, "-ns", str(N), "-nw", str(N)] + (["-procs"] if args.dropin_mode == "procs" else []) + [
        str(n), str(args.steps), str(args.warmup), str(args.dropin_layout)]
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=1200)
    wall = time.perf_counter() - t0
    if r.returncode != 0:
        raise SystemExit(f"kv_bench_dropin failed ({r.returncode}): {r.stderr[-2000:]}")
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    workers = [l for l in lines if "rank" in l]
    servers = [l for l in lines if "server" in l]
    if len(workers) != N:
        raise SystemExit(f"kv_bench_dropin: {len(workers)} worker lines for {N} workers")
    ms = max(w["ms_per_step"] for w in workers)
    gbs = 2 * 4 * n * N / (ms * 1e-3) / 1e9
    try:
        import psg as p
        gpus = max(1, min(N, p.device_count()))
    except Exception:
        gpus = 1
    # per GPU per step: its servers' N pushes and N pulls of n / N keys each
    per_gpu = (KEYED_PUSH_BYTES + KEYED_PULL_BYTES) * n * N // gpus
    roof = roofline(per_gpu, ms, args, "KVServerDefaultHandle requests (k_validate_windows / k_resolve_apply, "
                    "k_ident_*, runs: k_frames_*)", 4)
    roof["alg_bytes_note"] = (f"per GPU per step: {N} Push + {N} Pull requests of {n // N} keys per server "
                              f"x {KEYED_PUSH_BYTES} / {KEYED_PULL_BYTES} B per key, {N // gpus if gpus else N} "
                              "server(s) per GPU")
    # HBM traffic per step of this very job (every kernel of every node), from
    # the committed PMC passes at two step counts (tools/gpu_run.sh pmcdropin,
    # tools/pmc_total.py), when one was taken at this N, mode and layout
    import glob
    for f in sorted(glob.glob(os.path.join(ROOT, "profiles", f"r*_pmc_dropin_n{N}_{args.dropin_mode}_l"
                                                         f"{args.dropin_layout}.json")), reverse=True):
        try:
            d = json.load(open(f))
        except Exception:
            continue
        if d.get("alg_bytes_per_step") == per_gpu and gpus == 1:
            roof["traffic"] = d["hbm_bytes_per_step"]
            roof["traffic_source"] = os.path.relpath(f, ROOT)
            break
    res = {
        "metric": "device-resident KV Push+Pull GB/s (float vals) through KVWorker/KVServer",
        "value": round(gbs, 3), "unit": "GB/s", "n_gpus": gpus, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 5), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32", "data": "synthetic (integer-valued U{0..99} values, generated in HBM)",
        "config": {"workload": f"ns = nw = {N}, {n} keys per worker, "
                               + ("test_kv_app_benchmark's keys kMaxKey/num*i + rank" if args.dropin_layout == 0
                                  else "one key list shared by every worker (BSP: queued Pushes served as runs)"),
                   "keys": n, "servers": N, "workers": N, "mode": args.dropin_mode,
                   "api": "KVWorker::ZPush / ZPull (HBM SVectors), KVServerDefaultHandle",
                   "push_ms": round(max(w["push_ms"] for w in workers), 5),
                   "pull_ms": round(max(w["pull_ms"] for w in workers), 5)},
        "parity_check": all(w["mismatches"] == 0 for w in workers),
        "parity_detail": {"checked": "every worker's whole pulled vector vs the closed form of its pushes "
                                     "(psg_verify_synth_sum)", "mismatches": [w["mismatches"] for w in workers]},
        "roofline": roof,
        "job_wall_s": round(wall, 2),
    }
    if servers:
        # how the servers' stores served the job's requests (psg_store_counters):
        # runs in one pass (same list / strided) and the requests they held,
        # of N * N * 2 * (warmup + steps) requests in all
        tot = {k: sum(sv.get(k, 0) for sv in servers) for k in
               ("fused", "ident", "runs", "run_frames", "strided_runs", "strided_frames", "strided_single")}
        tot["requests"] = N * N * 2 * (args.warmup + args.steps)
        res["server_counters"] = tot
    if not args.no_cpu_baseline:
        import oracle
        t0 = time.perf_counter()
        f0, p0, l0 = oracle.bench(min(n, args.cpu_configs0_keys or n), 6)
        nn = min(n, args.cpu_configs0_keys or n)
        res["cpu_baseline"] = {"value": round(2 * 4 * nn / (p0 + l0) / 1e9, 4), "unit": "GB/s", "cores": 1,
                               "kind": "port",
                               "sample": (f"configs[0] layout: {nn} keys at kMaxKey/num*i through the "
                                          f"KVServerDefaultHandle unordered_map loop, 1 inserting Push ({f0:.2f} s) "
                                          f"then 6 Push+Pull, one thread, {time.perf_counter() - t0:.1f} s"),
                               "host": {"nproc": os.cpu_count(), "cpu_model": _cpu_model()}}
    return res


def roofline(alg_bytes: int, ms: float, args, kernel: str, vb: int, store_extra: int = 0,
             layout: str = "") -> dict:
    achieved = alg_bytes / (ms * 1e-3) / 1e9
    # HBM bytes per launch from the committed PMC summaries (tools/pmc_summary.py):
    # the one measured on this kernel at these algorithmic bytes and on this
    # store density (store_extra: store keys between request keys), if any
    traffic, source = None, None
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_*.json")))
    # (the newest round's summaries first: a later kernel may be described by
    # a text that also names an older one)
    files += sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_*.json")), reverse=True)
    for pmc in files:
        try:
            d = json.load(open(pmc))
        except Exception:
            continue
        names = [k.split("<")[0].strip() for k in str(d.get("kernel", "")).split("|")]
        if (d.get("alg_bytes_per_launch") == alg_bytes and d.get("store_extra", 0) == store_extra and names
                and d.get("store_layout", "") == layout and all(n in kernel for n in names)):
            traffic = d.get("hbm_bytes_per_launch")
            source = os.path.relpath(pmc, ROOT)
            break
    return {
        "kernel": kernel,
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": traffic,
        # traffic is NOT counted in this run: it is the HBM bytes per launch of
        # the committed rocprofv3 PMC summary (FETCH_SIZE x2 + WRITE_SIZE) of
        # this kernel at these algorithmic bytes
        "traffic_source": source,
        "alg_bytes_per_launch": alg_bytes,
    }


def _cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def cpu_baseline(args) -> dict:
    """The reference handler (std::unordered_map, one thread — KVServerDefaultHandle,
    src/ps/KVApp.h:433-458, runs on one Customer thread) restated in oracle/, on the
    GPU value's own workload: configs[1]'s keys 0..L-1 with the same synthetic
    values, 1 inserting Push then `reps` steady Push + Pull.  A second, labelled
    sample times configs[0]'s test_kv_app_benchmark layout (10 M keys at
    kMaxKey/num*i).  Reported beside the GPU number, not a target."""
    import oracle
    num, reps = args.cpu_keys, args.cpu_reps
    t0 = time.perf_counter()
    first, push_s, pull_s = oracle.bench_layout(num, reps, 0, 1, args.seed)
    wall = time.perf_counter() - t0
    out = {
        "value": round(2 * 4 * num / (push_s + pull_s) / 1e9, 4),
        "unit": "GB/s",
        "cores": 1,
        "kind": "port",
        "config": "configs[1] (the GPU value's workload)",
        "sample": (f"{num} keys 0..{num - 1} (configs[1] DENSE layout, values seed {args.seed}), "
                   f"1 inserting Push ({first:.2f} s) then {reps} steady Push+Pull through "
                   f"KVServerDefaultHandle's unordered_map loop, single thread, {wall:.1f} s total"),
        "host": {"nproc": os.cpu_count(), "cpu_model": _cpu_model()},
    }
    if args.cpu_configs0_keys:
        n0 = args.cpu_configs0_keys
        t0 = time.perf_counter()
        f0, p0, l0 = oracle.bench(n0, 6)
        out["configs0_sample"] = {
            "value": round(2 * 4 * n0 / (p0 + l0) / 1e9, 4), "unit": "GB/s",
            "sample": (f"configs[0] layout: {n0} keys at kMaxKey/num*i "
                       f"(test_kv_app_benchmark.cpp:47-52), 1 inserting Push ({f0:.2f} s) "
                       f"then 6 steady Push+Pull, {time.perf_counter() - t0:.1f} s"),
        }
    return out


def mapped_runtime_libs() -> dict:
    """Paths of the HIP runtime and RCCL this process mapped (the bench line says
    which ROCm the numbers come from)."""
    found = {}
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                parts = line.split()
                if len(parts) < 6:
                    continue
                path = parts[5]
                base = os.path.basename(path)
                for key in ("libamdhip64", "librccl", "libpsgpu"):
                    if base.startswith(key):
                        found.setdefault(key, os.path.realpath(path))
    except OSError:
        pass
    return found


def main(argv=None) -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="dense")
    ap.add_argument("--keys", type=int, default=None, help="values per worker (default by workload)")
    ap.add_argument("--seed", type=int, default=7)
    ap.add_argument("--check", type=int, default=1)
    ap.add_argument("--event-every", type=int, default=10,
                    help="record the kernel-timing HIP events on every n-th timed step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-probe256", action="store_true")
    ap.add_argument("--cpu-keys", type=int, default=64 << 20)
    ap.add_argument("--cpu-reps", type=int, default=12)
    ap.add_argument("--cpu-configs0-keys", type=int, default=10_000_000,
                    help="also time configs[0]'s layout at this many keys (0: skip)")
    ap.add_argument("--lr-frames", type=int, default=4, help="--workload lr: gradient frames per round (nw)")
    ap.add_argument("--cpu-lr-features", type=int, default=8 << 20,
                    help="--workload lr: features of the CPU baseline's sample")
    ap.add_argument("--dropin-mode", choices=["procs", "threads"], default="procs",
                    help="--workload dropin: one process per node (as local.py) or one thread per node")
    ap.add_argument("--dropin-layout", type=int, choices=[0, 1], default=0,
                    help="--workload dropin: 0 test_kv_app_benchmark's keys (+rank), 1 one shared list")
    args = ap.parse_args(argv)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using {world}", file=sys.stderr)
    dtype, _, keys1, keysn = WORKLOADS[args.workload][:4]
    if args.keys is None:
        args.keys = keys1 if world == 1 else keysn
    if args.workload == "lr":
        if world > 1:
            raise SystemExit("--workload lr is a one-GPU line (the N > 1 LR round is psg_comm_lr_push)")
        print(json.dumps(run_lr(args)), flush=True)
        return
    if args.workload == "dropin":
        # the job launches its own nodes (one per GPU): run it from one process
        if world > 1:
            raise SystemExit("--workload dropin launches its own ns = nw = --gpus nodes: run it as one process")
        print(json.dumps(run_dropin(args, args.gpus)), flush=True)
        return
    group = None
    if world > 1:
        from psg_group import SocketGroup
        group = SocketGroup(rank, world)
    backend = GpuBackend(rank, world, local_rank, group, dtype, keyed=args.workload == "keyed",
                         cached=args.workload == "keyed-cached")
    res = run(backend, args, rank, world, group)
    if res is not None:
        print(json.dumps(res), flush=True)
    if group is not None:
        group.barrier()
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
    if group is not None:
        group.close()


if __name__ == "__main__":
    main()
