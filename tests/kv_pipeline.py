"""The KVWorker Push / Pull / PushPull flow over ns server shards, for tests.

One request = DefaultSlicer (src/ps/KVApp.h:515-574) -> one
KVServerDefaultHandle call per non-empty slice (KVApp.h:435-456) -> for a pull,
the AddPullCB merge (KVApp.h:673-726).  Two interchangeable backends:

  OracleKV  the CPU restatement (oracle/): the checker
  GpuKV     the product C-ABI (psg_slice, psg_store_handle, psg_merge) on HIP

so a test runs the reference's own known-answer scenarios through both and
compares.
"""
from __future__ import annotations

import numpy as np

PUSH, PULL = 1, 2


class OracleKV:
    def __init__(self, ns: int):
        import oracle
        self.o = oracle
        self.ns = ns
        self.begins, self.ends = oracle.server_ranges(ns)
        self.servers = [oracle.Store(oracle.F32) for _ in range(ns)]

    def request(self, flags: int, keys: np.ndarray, vals: np.ndarray | None):
        r = self.o.slice_keys(keys, self.begins, self.ends)
        assert r is not None, "slicer CHECK"
        kp, _ = r
        segs = []
        for i in range(self.ns):
            a, b = int(kp[i]), int(kp[i + 1])
            if a == b:
                continue
            res = self.servers[i].handle(flags, keys[a:b], None if vals is None else vals[a:b],
                                         b - a)
            if flags & PULL:
                segs.append((res, int(keys[a])))
        if flags & PULL:
            # replies arrive in any order; the merge sorts them
            return self.o.merge(segs[::-1], len(keys))
        return None

    def push(self, keys, vals):
        self.request(PUSH, keys, vals)

    def pull(self, keys):
        return self.request(PULL, keys, None)

    def pushpull(self, keys, vals):
        return self.request(PUSH | PULL, keys, vals)


class GpuKV:
    """Worker + ns SORTED server stores on one GPU, all through the C-ABI."""

    def __init__(self, ns: int, kind=None):
        import psg
        self.p = psg
        self.ns = ns
        self.begins, self.ends = psg.server_ranges(ns)
        kind = psg.SORTED if kind is None else kind
        self.servers = [psg.Store(kind, psg.F32, int(self.begins[i]), int(self.ends[i]), 0)
                        for i in range(ns)]
        self.stream = psg.Stream()
        self._keys = None

    def _dev_keys(self, keys):
        if self._keys is None or self._keys[0] is not keys:
            self._keys = (keys, self.p.DeviceBuffer.from_numpy(keys, self.stream))
        return self._keys[1]

    def request(self, flags, keys, vals):
        p = self.p
        n = len(keys)
        dk = self._dev_keys(keys)
        dv = p.DeviceBuffer.from_numpy(vals, self.stream) if vals is not None else None
        kp, _ = p.slice_keys(dk, n, self.begins, self.ends, stream=self.stream)
        replies = []
        for i in range(self.ns):
            a, b = int(kp[i]), int(kp[i + 1])
            if a == b:
                continue
            out = p.DeviceBuffer((b - a) * 4) if flags & PULL else None
            self.servers[i].handle(flags, dk.ptr + 8 * a, None if dv is None else dv.ptr + 4 * a,
                                   out, b - a, stream=self.stream)
            if out is not None:
                replies.append((out, b - a, int(keys[a])))
        if flags & PULL:
            dst = p.DeviceBuffer(max(n * 4, 4))
            p.merge(replies[::-1], 4, dst, n, stream=self.stream)
            return dst.download(np.float32, n, self.stream)
        self.stream.sync()
        return None

    def push(self, keys, vals):
        self.request(PUSH, keys, vals)

    def pull(self, keys):
        return self.request(PULL, keys, None)

    def pushpull(self, keys, vals):
        return self.request(PUSH | PULL, keys, vals)


def run_kv_app(kv, keys, vals, repeat=50):
    """tests/test_kv_app.cpp:34-58 on one worker."""
    for _ in range(repeat):
        kv.push(keys, vals)
    rets = kv.pull(keys)
    outs = None
    for _ in range(repeat):
        outs = kv.pushpull(keys, vals)
    return rets, outs


def run_my(kv, keys, vals_per_customer, repeat=50):
    """tests/test_my.cpp:38-71: CC customers on the same keys, barrier between phases."""
    for v in vals_per_customer:
        for _ in range(repeat):
            kv.push(keys, v)
    rets = kv.pull(keys)
    for v in vals_per_customer:
        for _ in range(repeat):
            kv.pushpull(keys, v)
    final = kv.pull(keys)
    return rets, final
