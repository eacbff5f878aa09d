"""ctypes binding of oracle/liboracle.so — TEST INFRASTRUCTURE ONLY.

The CPU restatement of the reference KV algorithms (see ps_oracle.cpp).  Only
tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, as the checker or as the timed CPU baseline; the product never does.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "liboracle.so")

F32, F64, F16, BF16 = 0, 1, 2, 3
PUSH, PULL = 1, 2
NP = {F32: np.float32, F64: np.float64, F16: np.uint16, BF16: np.uint16}

_lib = None


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} not built (make -C oracle)")
        L = C.CDLL(LIB_PATH)
        vp, u64, i32, f32, f64 = C.c_void_p, C.c_uint64, C.c_int, C.c_float, C.c_double
        L.oracle_store_new.argtypes = [i32]
        L.oracle_store_new.restype = vp
        L.oracle_store_free.argtypes = [vp]
        L.oracle_store_free.restype = None
        L.oracle_store_reserve.argtypes = [vp, u64]
        L.oracle_store_reserve.restype = None
        L.oracle_handle.argtypes = [vp, i32, vp, u64, vp, vp, u64]
        L.oracle_handle.restype = i32
        L.oracle_store_size.argtypes = [vp]
        L.oracle_store_size.restype = u64
        L.oracle_store_dump.argtypes = [vp, vp, vp]
        L.oracle_store_dump.restype = None
        L.oracle_server_ranges.argtypes = [i32, vp, vp]
        L.oracle_server_ranges.restype = None
        L.oracle_slice.argtypes = [vp, u64, vp, u64, u64, i32, vp, vp, vp, vp]
        L.oracle_slice.restype = i32
        L.oracle_merge.argtypes = [i32, C.POINTER(vp), vp, vp, i32, vp, u64]
        L.oracle_merge.restype = i32
        L.oracle_lr_apply.argtypes = [vp, vp, u64, f32, vp, vp, f64, f64, f64, f64, i32]
        L.oracle_lr_apply.restype = None
        L.oracle_synth.argtypes = [vp, u64, i32, u64, i32, f64, f64]
        L.oracle_synth.restype = None
        L.oracle_glibc_rand_mod.argtypes = [i32, i32, u64, vp]
        L.oracle_glibc_rand_mod.restype = None
        L.oracle_bench.argtypes = [u64, i32, C.POINTER(f64), C.POINTER(f64), C.POINTER(f64)]
        L.oracle_bench.restype = None
        L.oracle_bench_layout.argtypes = [u64, i32, u64, u64, u64, C.POINTER(f64),
                                          C.POINTER(f64), C.POINTER(f64)]
        L.oracle_bench_layout.restype = None
        _lib = L
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data_as(C.c_void_p)


class Store:
    """std::unordered_map<Key, V> store of KVServerDefaultHandle (KVApp.h:457)."""

    def __init__(self, dtype: int = F32):
        self.dtype = dtype
        self.h = lib().oracle_store_new(dtype)

    def handle(self, flags: int, keys, vals, n: int, first_key: int = 0):
        out = np.zeros(n, dtype=NP[self.dtype]) if flags & PULL else None
        if keys is not None:
            keys = np.ascontiguousarray(keys, dtype=np.uint64)
        if vals is not None:
            vals = np.ascontiguousarray(vals, dtype=NP[self.dtype])
        rc = lib().oracle_handle(self.h, flags, _p(keys), first_key, _p(vals), _p(out), n)
        assert rc == 0
        return out

    def size(self) -> int:
        return lib().oracle_store_size(self.h)

    def dump(self):
        n = self.size()
        k = np.empty(n, dtype=np.uint64)
        v = np.empty(n, dtype=NP[self.dtype])
        lib().oracle_store_dump(self.h, _p(k), _p(v))
        return k, v

    def __del__(self):
        try:
            lib().oracle_store_free(self.h)
        except Exception:
            pass


def server_ranges(ns: int):
    b = np.empty(ns, dtype=np.uint64)
    e = np.empty(ns, dtype=np.uint64)
    lib().oracle_server_ranges(ns, _p(b), _p(e))
    return b, e


def slice_keys(keys, begins, ends, lens=None, num_vals=None):
    """DefaultSlicer restatement; returns (key_pos, val_pos) or None on a CHECK."""
    keys = np.ascontiguousarray(keys, dtype=np.uint64)
    n = len(keys)
    ns = len(begins)
    kp = np.zeros(ns + 1, dtype=np.uint64)
    vpos = np.zeros(ns + 1, dtype=np.uint64)
    lens_a = None if lens is None else np.ascontiguousarray(lens, dtype=np.int32)
    rc = lib().oracle_slice(_p(keys), n, _p(lens_a), 0 if lens_a is None else len(lens_a),
                            n if num_vals is None else num_vals, ns,
                            _p(np.ascontiguousarray(begins, dtype=np.uint64)),
                            _p(np.ascontiguousarray(ends, dtype=np.uint64)), _p(kp), _p(vpos))
    return None if rc else (kp, vpos)


def merge(segments, dst_count: int, dtype=np.float32):
    """segments: list of (np.ndarray vals, first_key)."""
    n = len(segments)
    arrs = [np.ascontiguousarray(v, dtype=dtype) for v, _ in segments]
    ptrs = (C.c_void_p * max(n, 1))(*[a.ctypes.data for a in arrs])
    counts = np.array([len(a) for a in arrs], dtype=np.uint64)
    fks = np.array([fk for _, fk in segments], dtype=np.uint64)
    out = np.zeros(dst_count, dtype=dtype)
    rc = lib().oracle_merge(n, ptrs, _p(counts), _p(fks), np.dtype(dtype).itemsize, _p(out),
                            dst_count)
    return None if rc else out


def lr_apply(weight, merged, lr, m=None, v=None, adam_lr=0.0, beta1=0.9, beta2=0.999,
             eps=1e-8, iteration=0):
    lib().oracle_lr_apply(_p(weight), _p(merged), len(weight), lr, _p(m), _p(v), adam_lr, beta1,
                          beta2, eps, iteration)


def synth(n: int, dtype: int, seed: int, mode: int, lo: float, hi: float):
    out = np.empty(n, dtype=NP[dtype])
    lib().oracle_synth(_p(out), n, dtype, seed, mode, lo, hi)
    return out


def glibc_rand_mod(seed: int, mod: int, n: int):
    out = np.empty(n, dtype=np.float32)
    lib().oracle_glibc_rand_mod(seed, mod, n, _p(out))
    return out


def bench(num: int, reps: int):
    a, b, c = C.c_double(), C.c_double(), C.c_double()
    lib().oracle_bench(num, reps, C.byref(a), C.byref(b), C.byref(c))
    return a.value, b.value, c.value


def bench_layout(num: int, reps: int, key_base: int = 0, key_step: int = 1, seed: int = 7):
    """The handler on the GPU bench's workload (keys base + i*step, synth values)."""
    a, b, c = C.c_double(), C.c_double(), C.c_double()
    lib().oracle_bench_layout(num, reps, key_base, key_step, seed, C.byref(a), C.byref(b),
                              C.byref(c))
    return a.value, b.value, c.value
