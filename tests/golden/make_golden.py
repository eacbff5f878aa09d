"""Generate tests/golden/golden.npz — the reference's known-answer tests as data.

The reference (SovietPower/Parameter-Server) cannot be built in this image
(its Van needs protobuf 3.21 generated code and libprotobuf), so the golden
vectors are the inputs and expected outputs its own tests state:

  kv_app        tests/test_kv_app.cpp:20-61 — rank 0: num = 10000 keys
                `kMaxKey / num * i + rank`, vals = glibc `srand(rank + 7); rand() % 1000`;
                50 Push -> Pull expects 50 * vals (:56); then 50 PushPull
                expects 100 * vals (:57).
  multi_workers tests/test_kv_app_multi_workers.cpp:27-65 — customers c = 0, 1 with keys
                `kMaxKey / num * i + c`; same expectations per customer.
  my            tests/test_my.cpp:29-75 — CC = 3 customers on the SAME keys
                `kMaxKey / num * i + i`, vals 5 * (i + c); after every customer's 50
                pushes: 50 * 5 * (i * CC + CC * (CC - 1) / 2) (:52); after the 50
                PushPulls each: twice that (:71).
  slicer        DefaultSlicer (src/ps/KVApp.h:515-574) cases computed by the
                independent bisect transcription below (not by oracle/ps_oracle.cpp).

glibc rand() is called through ctypes on libc (the same generator the reference
test binaries use), independent of the oracle library.

Run:  python tests/golden/make_golden.py   (rewrites golden.npz)
"""
import bisect
import ctypes
import os

import numpy as np

KMAX = (1 << 64) - 1
HERE = os.path.dirname(os.path.abspath(__file__))

libc = ctypes.CDLL("libc.so.6")


def glibc_vals(seed, n, mod=1000):
    libc.srand(seed)
    return np.array([libc.rand() % mod for _ in range(n)], dtype=np.float32)


def ranges(ns):
    """PostOffice::GetServerRanges, src/internal/PostOffice.cpp:211-221."""
    b = [KMAX // ns * i for i in range(ns)]
    e = [KMAX // ns * (i + 1) if i != ns - 1 else KMAX for i in range(ns)]
    return b, e


def slicer(keys, ns, lens=None, nvals=None):
    """Bisect transcription of DefaultSlicer; val_pos[i] = start of slice i."""
    b, e = ranges(ns)
    keys = [int(k) for k in keys]
    pos = [0] * (ns + 1)
    pos[0] = bisect.bisect_left(keys, b[0])
    for i in range(ns):
        pos[i + 1] = bisect.bisect_left(keys, e[i], lo=pos[i])
    if pos[ns] != len(keys):
        return None
    if not keys:
        return pos, [0] * (ns + 1)
    if lens is None:
        k = (len(keys) if nvals is None else nvals) // len(keys)
        vpos = [p * k for p in pos]
    else:
        vpos = [0] * (ns + 1)
        acc = 0
        for i in range(ns):
            vpos[i] = acc
            acc += sum(lens[pos[i]:pos[i + 1]])
        vpos[ns] = acc
    return pos, vpos


def main():
    out = {}
    num, repeat = 10000, 50
    # --- test_kv_app.cpp (rank 0)
    keys = np.array([KMAX // num * i + 0 for i in range(num)], dtype=np.uint64)
    vals = glibc_vals(0 + 7, num)
    out["kv_app_keys"] = keys
    out["kv_app_vals"] = vals
    out["kv_app_rets"] = (vals * repeat).astype(np.float32)
    out["kv_app_outs"] = (vals * 2 * repeat).astype(np.float32)
    # --- test_kv_app_multi_workers.cpp (customers 0 and 1 in rank 0)
    for c in (0, 1):
        out[f"mw{c}_keys"] = np.array([KMAX // num * i + c for i in range(num)], dtype=np.uint64)
        v = glibc_vals(0 + 7, num)
        out[f"mw{c}_vals"] = v
        out[f"mw{c}_rets"] = (v * repeat).astype(np.float32)
        out[f"mw{c}_outs"] = (v * 2 * repeat).astype(np.float32)
    # --- test_my.cpp (CC = 3 customers, shared keys)
    cc = 3
    out["my_keys"] = np.array([KMAX // num * i + i for i in range(num)], dtype=np.uint64)
    for c in range(cc):
        out[f"my{c}_vals"] = np.array([5 * (i + c) for i in range(num)], dtype=np.float32)
    expect = np.array([repeat * 5 * (i * cc + cc * (cc - 1) // 2) for i in range(num)],
                      dtype=np.float64)
    out["my_rets"] = expect.astype(np.float32)
    out["my_final"] = (expect * 2).astype(np.float32)
    # --- slicer cases
    rng = np.random.default_rng(1234)
    cases = []
    for ns in (1, 2, 3, 4, 7, 8):
        k = np.unique(rng.integers(0, KMAX, size=513, dtype=np.uint64, endpoint=False))
        cases.append((k, ns, None))
        lens = rng.integers(0, 5, size=len(k)).astype(np.int32)
        cases.append((k, ns, lens))
    b8, e8 = ranges(8)
    edge = np.array(sorted({0, 1, b8[1] - 1, b8[1], b8[1] + 1, b8[4], e8[6] - 1, e8[6], KMAX - 1}),
                    dtype=np.uint64)
    cases.append((edge, 8, None))
    cases.append((np.array([5, 6, 7], dtype=np.uint64), 4, None))  # all in server 0
    for j, (k, ns, lens) in enumerate(cases):
        r = slicer(k, ns, None if lens is None else [int(x) for x in lens])
        assert r is not None
        out[f"slice{j}_keys"] = k
        out[f"slice{j}_ns"] = np.array([ns])
        out[f"slice{j}_lens"] = lens if lens is not None else np.zeros(0, dtype=np.int32)
        out[f"slice{j}_haslens"] = np.array([lens is not None])
        out[f"slice{j}_kpos"] = np.array(r[0], dtype=np.uint64)
        out[f"slice{j}_vpos"] = np.array(r[1], dtype=np.uint64)
    out["slice_ncases"] = np.array([len(cases)])
    np.savez_compressed(os.path.join(HERE, "golden.npz"), **out)
    print("wrote", os.path.join(HERE, "golden.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
