"""ctypes binding of the psg C-ABI (include/psg.h) for tests and bench.py.

The product is the C-ABI library ``lib/libpsgpu.so`` (HIP kernels for gfx950);
this module is a thin, typed wrapper over it.  It never falls back to a CPU
path: when the library is missing, or a call fails, it raises ``PsgError``.

Functions mirror the reference interfaces named in include/psg.h (paths in the
reference repository SovietPower/Parameter-Server):
  Store.handle   -> KVServerDefaultHandle::operator()  src/ps/KVApp.h:435-456
  slice          -> KVWorker::DefaultSlicer            src/ps/KVApp.h:515-574
  merge          -> AddPullCB merge                    src/ps/KVApp.h:673-726
  server_ranges  -> PostOffice::GetServerRanges        src/internal/PostOffice.cpp:211-221
  Comm.push/pull -> BSP Push (reduce-scatter) / Pull (all-gather) over RCCL
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get(
    "PSG_LIB", os.path.join(os.path.dirname(_HERE), "lib", "libpsgpu.so"))

F32, F64, F16, BF16 = 0, 1, 2, 3
DENSE, SORTED = 0, 1
PUSH, PULL = 1, 2
RUN_ONE_BY_ONE, RUN_SAME_LIST, RUN_STRIDED = 0, 1, 2
H2D, D2H, D2D = 0, 1, 2

_NP = {F32: np.float32, F64: np.float64, F16: np.float16, BF16: np.uint16}
_ESIZE = {F32: 4, F64: 8, F16: 2, BF16: 2}

# every symbol include/psg.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "psg_abi_version", "psg_last_error", "psg_device_count", "psg_set_device", "psg_device_pci_bus_id",
    "psg_get_device", "psg_device_sync", "psg_enable_peer_access", "psg_malloc", "psg_free", "psg_host_alloc",
    "psg_host_free", "psg_host_register", "psg_host_unregister", "psg_memcpy",
    "psg_memset", "psg_copy", "psg_stream_create", "psg_stream_create_priority", "psg_stream_destroy",
    "psg_stream_sync",
    "psg_event_create", "psg_event_create_timing", "psg_event_destroy", "psg_event_record", "psg_event_sync",
    "psg_event_elapsed_ms", "psg_stream_wait_event", "psg_fill_synth", "psg_fill_keys_arith", "psg_checksum",
    "psg_verify_synth_sum",
    "psg_store_create", "psg_store_destroy", "psg_store_get_info", "psg_store_clear", "psg_store_counters",
    "psg_store_handle", "psg_store_handle_async", "psg_store_wait", "psg_sort_pairs_u64", "psg_store_resolve", "psg_store_handle_slots",
    "psg_store_slots_stretch", "psg_store_handle_stretch", "psg_store_sync", "psg_store_dump",
    "psg_key_list_hash", "psg_store_push_frames", "psg_store_push_slots_frames", "psg_store_run",
    "psg_store_run_status", "psg_store_set_key_range", "psg_server_ranges", "psg_slice", "psg_slice_hint", "psg_merge", "psg_comm_id_bytes", "psg_comm_get_id",
    "psg_comm_init", "psg_comm_destroy", "psg_comm_rank", "psg_comm_push", "psg_comm_pull",
    "psg_comm_push_pull", "psg_comm_push_keyed", "psg_comm_pull_keyed",
    "psg_comm_bucket_plan", "psg_comm_keyed_plan", "psg_comm_sync", "psg_comm_abort",
    "psg_adam_create", "psg_adam_destroy", "psg_lr_apply", "psg_lr_apply_sum", "psg_lr_mix_copy",
    "psg_comm_lr_push", "psg_xgmi_lr_push",
    "psg_ipc_handle_bytes", "psg_ipc_export", "psg_ipc_export_range", "psg_ipc_open", "psg_ipc_close", "psg_xgmi_create",
    "psg_xgmi_destroy", "psg_xgmi_push", "psg_xgmi_pull", "psg_xgmi_push_range",
    "psg_xgmi_pull_range", "psg_xgmi_set_outs", "psg_xgmi_pull_write_range", "psg_xgmi_pull_write",
    "psg_xgmi_pull_write_slots",
    "psg_xgmi_push_slots", "psg_xgmi_pull_slots", "psg_node_barrier_create",
    "psg_node_barrier_wait", "psg_node_barrier_destroy",
]


class PsgError(RuntimeError):
    def __init__(self, code: int, what: str, msg: str):
        super().__init__(f"{what} -> status {code}: {msg}")
        self.code = code


class StoreInfo(C.Structure):
    _fields_ = [("kind", C.c_int), ("dtype", C.c_int), ("key_begin", C.c_uint64),
                ("key_end", C.c_uint64), ("size", C.c_uint64), ("capacity", C.c_uint64),
                ("vals", C.c_void_p), ("keys", C.c_void_p)]


class Segment(C.Structure):
    _fields_ = [("vals", C.c_void_p), ("count", C.c_uint64), ("first_key", C.c_uint64)]


_lib = None


def lib() -> C.CDLL:
    """Load libpsgpu.so (raises if it was not built: no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise PsgError(-1, "load", f"{LIB_PATH} not built (run __graft_entry__.build())")
        L = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
        vp, u64, i32, f32, f64 = C.c_void_p, C.c_uint64, C.c_int, C.c_float, C.c_double
        sig = {
            "psg_abi_version": ([], i32), "psg_last_error": ([], C.c_char_p),
            "psg_device_count": ([C.POINTER(i32)], i32), "psg_set_device": ([i32], i32),
            "psg_device_pci_bus_id": ([i32, C.c_char_p, i32], i32),
            "psg_get_device": ([C.POINTER(i32)], i32), "psg_device_sync": ([], i32),
            "psg_enable_peer_access": ([i32, i32], i32),
            "psg_malloc": ([C.POINTER(vp), C.c_size_t], i32), "psg_free": ([vp], i32),
            "psg_host_alloc": ([C.POINTER(vp), C.c_size_t], i32), "psg_host_free": ([vp], i32),
            "psg_host_register": ([vp, C.c_size_t], i32), "psg_host_unregister": ([vp], i32),
            "psg_memcpy": ([vp, vp, C.c_size_t, i32, vp], i32),
            "psg_memset": ([vp, i32, C.c_size_t, vp], i32),
            "psg_copy": ([vp, vp, u64, i32, i32, vp], i32),
            "psg_stream_create": ([C.POINTER(vp)], i32), "psg_stream_destroy": ([vp], i32),
            "psg_stream_sync": ([vp], i32), "psg_event_create": ([C.POINTER(vp)], i32),
            "psg_event_create_timing": ([C.POINTER(vp)], i32),
            "psg_event_destroy": ([vp], i32), "psg_event_record": ([vp, vp], i32),
            "psg_event_sync": ([vp], i32),
            "psg_event_elapsed_ms": ([vp, vp, C.POINTER(f32)], i32),
            "psg_stream_wait_event": ([vp, vp], i32),
            "psg_fill_synth": ([vp, u64, i32, u64, i32, f64, f64, vp], i32),
            "psg_fill_keys_arith": ([vp, u64, u64, u64, vp], i32),
            "psg_checksum": ([vp, u64, C.POINTER(u64), vp], i32),
            "psg_verify_synth_sum": ([vp, u64, i32, u64, i32, u64, f64, f64, f64,
                                      C.POINTER(u64), C.POINTER(u64), vp], i32),
            "psg_store_create": ([i32, i32, u64, u64, u64, C.POINTER(vp)], i32),
            "psg_store_destroy": ([vp], i32),
            "psg_store_get_info": ([vp, C.POINTER(StoreInfo)], i32),
            "psg_store_clear": ([vp, vp], i32),
            "psg_store_counters": ([vp, C.POINTER(C.c_uint64), i32], i32),
            "psg_store_handle": ([vp, i32, vp, u64, vp, vp, u64, vp], i32),
            "psg_store_handle_async": ([vp, i32, vp, u64, vp, vp, u64, vp, C.POINTER(u64)], i32),
            "psg_store_wait": ([vp, u64], i32),
            "psg_sort_pairs_u64": ([vp, vp, u64, i32, vp], i32),
            "psg_store_resolve": ([vp, vp, u64, i32, vp, vp], i32),
            "psg_store_handle_slots": ([vp, i32, vp, vp, vp, u64, vp], i32),
            "psg_store_slots_stretch": ([vp, vp, u64, C.POINTER(u64), vp], i32),
            "psg_store_handle_stretch": ([vp, i32, u64, vp, vp, u64, vp], i32),
            "psg_store_sync": ([vp, vp], i32),
            "psg_store_dump": ([vp, vp, vp], i32),
            "psg_key_list_hash": ([vp, u64, C.POINTER(u64), vp], i32),
            "psg_store_push_frames": ([vp, C.POINTER(vp), u64, C.POINTER(vp), i32, u64, vp,
                                       C.POINTER(i32)], i32),
            "psg_store_push_slots_frames": ([vp, vp, u64, C.POINTER(vp), i32, u64, vp], i32),
            "psg_store_run": ([vp, i32, C.POINTER(i32), C.POINTER(vp), C.POINTER(u64), C.POINTER(vp),
                               C.POINTER(vp), vp, C.POINTER(i32)], i32),
            "psg_store_run_status": ([vp, i32, C.POINTER(i32), C.POINTER(vp), C.POINTER(u64), C.POINTER(vp),
                                      C.POINTER(vp), vp, C.POINTER(i32), C.POINTER(i32)], i32),
            "psg_slice_hint": ([vp, u64, i32, u64, vp, C.POINTER(i32)], i32),
            "psg_store_set_key_range": ([vp, u64, u64], i32),
            "psg_server_ranges": ([i32, vp, vp], i32),
            "psg_slice": ([vp, u64, vp, u64, i32, vp, vp, vp, vp, vp], i32),
            "psg_merge": ([C.POINTER(Segment), i32, i32, vp, u64, vp], i32),
            "psg_comm_id_bytes": ([], i32), "psg_comm_get_id": ([vp], i32),
            "psg_comm_bucket_plan": ([u64, i32, vp, vp, i32, C.POINTER(i32)], i32),
            "psg_comm_sync": ([vp, vp, f64], i32), "psg_comm_abort": ([vp], i32),
            "psg_comm_keyed_plan": ([vp, i32, u64, C.POINTER(u64)], i32),
            "psg_comm_init": ([vp, i32, i32, C.POINTER(vp)], i32),
            "psg_comm_destroy": ([vp], i32),
            "psg_comm_rank": ([vp, C.POINTER(i32), C.POINTER(i32)], i32),
            "psg_comm_push": ([vp, vp, vp, u64, vp, vp], i32),
            "psg_comm_pull": ([vp, vp, vp, u64, vp], i32),
            "psg_comm_push_pull": ([vp, vp, vp, vp, u64, i32, vp], i32),
            "psg_comm_push_keyed": ([vp, vp, vp, vp, u64, vp, vp], i32),
            "psg_comm_pull_keyed": ([vp, vp, vp, vp, u64, vp, vp], i32),
            "psg_adam_create": ([u64, f64, f64, f64, f64, C.POINTER(vp)], i32),
            "psg_adam_destroy": ([vp], i32),
            "psg_lr_apply": ([vp, vp, u64, f32, vp, i32, vp], i32),
            "psg_lr_apply_sum": ([vp, C.POINTER(vp), i32, i32, u64, f32, vp, i32, vp], i32),
            "psg_lr_mix_copy": ([vp, C.POINTER(vp), i32, u64, vp, vp], i32),
            "psg_comm_lr_push": ([vp, vp, vp, u64, f32, vp, i32, vp, vp], i32),
            "psg_xgmi_lr_push": ([vp, vp, u64, f32, vp, i32, vp], i32),
            "psg_ipc_handle_bytes": ([], i32), "psg_ipc_export": ([vp, vp], i32),
            "psg_ipc_export_range": ([vp, vp, C.POINTER(u64)], i32),
            "psg_ipc_open": ([vp, C.POINTER(vp)], i32), "psg_ipc_close": ([vp], i32),
            "psg_xgmi_create": ([i32, i32, C.POINTER(vp), C.POINTER(vp), C.POINTER(vp)], i32),
            "psg_xgmi_destroy": ([vp], i32), "psg_xgmi_push": ([vp, vp, u64, vp], i32),
            "psg_xgmi_pull": ([vp, vp, vp, u64, vp], i32),
            "psg_xgmi_push_range": ([vp, vp, u64, u64, u64, vp], i32),
            "psg_xgmi_pull_range": ([vp, vp, vp, u64, u64, u64, vp], i32),
            "psg_xgmi_set_outs": ([vp, C.POINTER(vp)], i32),
            "psg_xgmi_pull_write_range": ([vp, vp, u64, u64, u64, vp], i32),
            "psg_xgmi_pull_write": ([vp, vp, u64, vp], i32),
            "psg_xgmi_pull_write_slots": ([vp, vp, vp, u64, u64, vp], i32),
            "psg_xgmi_push_slots": ([vp, vp, vp, u64, u64, vp], i32),
            "psg_xgmi_pull_slots": ([vp, vp, C.POINTER(vp), vp, vp, vp, vp], i32),
            "psg_node_barrier_create": ([C.c_char_p, i32, i32, C.POINTER(vp)], i32),
            "psg_node_barrier_wait": ([vp, f64], i32), "psg_node_barrier_destroy": ([vp], i32),
        }
        for name, (args, res) in sig.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise PsgError(rc, what, lib().psg_last_error().decode(errors="replace"))


def _call(name: str, *args) -> None:
    check(getattr(lib(), name)(*args), name)


def _ptr(x) -> int | None:
    if x is None:
        return None
    if isinstance(x, DeviceBuffer):
        return x.ptr
    if isinstance(x, int):
        return x
    raise TypeError(f"expected DeviceBuffer or int device pointer, got {type(x)}")


# ---- runtime -------------------------------------------------------------------
def device_count() -> int:
    n = C.c_int(0)
    _call("psg_device_count", C.byref(n))
    return n.value


def set_device(dev: int) -> None:
    _call("psg_set_device", dev)


def device_pci_bus_id(dev: int) -> str:
    """The PCI bus id of GPU `dev` (psg_device_pci_bus_id)."""
    buf = C.create_string_buffer(64)
    _call("psg_device_pci_bus_id", dev, buf, 64)
    return buf.value.decode()


def device_sync() -> None:
    _call("psg_device_sync")


class Stream:
    def __init__(self, null: bool = False):
        self.handle = C.c_void_p(None)
        if not null:
            _call("psg_stream_create", C.byref(self.handle))

    @property
    def ptr(self):
        return self.handle.value

    def sync(self) -> None:
        _call("psg_stream_sync", self.handle)

    def wait(self, ev: "Event") -> None:
        """Later work on this stream waits for `ev`."""
        _call("psg_stream_wait_event", self.handle, ev.handle)

    def close(self) -> None:
        if self.handle.value:
            _call("psg_stream_destroy", self.handle)
            self.handle = C.c_void_p(None)


def _s(stream) -> int | None:
    return None if stream is None else stream.ptr


class Event:
    """A HIP event; ``timing=True``: a timing-only marker (psg_event_create_timing,
    no system-scope fence at its record)."""

    def __init__(self, timing: bool = False):
        self.handle = C.c_void_p(None)
        _call("psg_event_create_timing" if timing else "psg_event_create", C.byref(self.handle))

    def record(self, stream=None) -> None:
        _call("psg_event_record", self.handle, _s(stream))

    def sync(self) -> None:
        _call("psg_event_sync", self.handle)

    def elapsed_ms(self, end: "Event") -> float:
        ms = C.c_float(0)
        _call("psg_event_elapsed_ms", self.handle, end.handle, C.byref(ms))
        return ms.value

    def close(self) -> None:
        if self.handle.value:
            _call("psg_event_destroy", self.handle)
            self.handle = C.c_void_p(None)


class DeviceBuffer:
    """Raw HBM allocation (psg_malloc) of ``nbytes``; numpy upload/download."""

    def __init__(self, nbytes: int):
        self.nbytes = int(nbytes)
        h = C.c_void_p(None)
        _call("psg_malloc", C.byref(h), C.c_size_t(self.nbytes))
        self.ptr = h.value or 0

    @classmethod
    def from_numpy(cls, a: np.ndarray, stream=None) -> "DeviceBuffer":
        a = np.ascontiguousarray(a)
        b = cls(max(a.nbytes, 1))
        b.upload(a, stream)
        return b

    def upload(self, a: np.ndarray, stream=None, offset: int = 0) -> None:
        a = np.ascontiguousarray(a)
        assert offset + a.nbytes <= self.nbytes
        if a.nbytes:
            _call("psg_memcpy", C.c_void_p(self.ptr + offset), a.ctypes.data_as(C.c_void_p),
                  C.c_size_t(a.nbytes), H2D, _s(stream))
            Stream.sync(stream) if stream is not None else device_sync()

    def download(self, dtype, count: int, stream=None, offset: int = 0) -> np.ndarray:
        out = np.empty(count, dtype=dtype)
        if out.nbytes:
            assert offset + out.nbytes <= self.nbytes
            _call("psg_memcpy", out.ctypes.data_as(C.c_void_p), C.c_void_p(self.ptr + offset),
                  C.c_size_t(out.nbytes), D2H, _s(stream))
            Stream.sync(stream) if stream is not None else device_sync()
        return out

    def fill_synth(self, n: int, dtype: int, seed: int, mode: int, lo: float, hi: float,
                   stream=None) -> None:
        _call("psg_fill_synth", C.c_void_p(self.ptr), n, dtype, seed, mode, lo, hi, _s(stream))

    def free(self) -> None:
        if self.ptr:
            _call("psg_free", C.c_void_p(self.ptr))
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def copy(dst, src, nbytes: int, unroll: int = 1, blocks_per_cu: int = 4, stream=None) -> None:
    """psg_copy: the streaming float4 copy kernel (the Pull's copy ceiling)."""
    _call("psg_copy", C.c_void_p(_ptr(dst)), C.c_void_p(_ptr(src)), nbytes, unroll, blocks_per_cu, _s(stream))


def memcpy_d2d(dst, src, nbytes: int, stream=None) -> None:
    """Device-to-device copy (psg_memcpy, kind 2), stream-ordered."""
    _call("psg_memcpy", C.c_void_p(_ptr(dst)), C.c_void_p(_ptr(src)), nbytes, 2, _s(stream))


def checksum(ptr, nbytes: int, stream=None) -> int:
    """psg_checksum of a device range (synchronises the stream)."""
    h = C.c_uint64(0)
    _call("psg_checksum", C.c_void_p(_ptr(ptr)), C.c_uint64(nbytes), C.byref(h), _s(stream))
    return h.value


def verify_synth_sum(ptr, n: int, dtype: int, seed0: int, nseeds: int, lo: float, hi: float,
                     scale: float, offset: int = 0, stream=None):
    """psg_verify_synth_sum: (mismatches, first mismatching index or None)."""
    bad, first = C.c_uint64(0), C.c_uint64(0)
    _call("psg_verify_synth_sum", C.c_void_p(_ptr(ptr)), n, dtype, seed0, nseeds, offset, lo, hi,
          scale, C.byref(bad), C.byref(first), _s(stream))
    return bad.value, (None if first.value == (1 << 64) - 1 else first.value)


def key_list_hash(keys, n: int, stream=None) -> int:
    """psg_key_list_hash: the LR key-cache hash of a device key list."""
    h = C.c_uint64(0)
    _call("psg_key_list_hash", C.c_void_p(_ptr(keys)), n, C.byref(h), _s(stream))
    return h.value


def checksum_host(a: np.ndarray) -> int:
    """The same checksum computed with numpy (for tests)."""
    w = np.ascontiguousarray(a).view(np.uint64)
    with np.errstate(over="ignore"):
        x = w ^ (np.arange(len(w), dtype=np.uint64) * np.uint64(0x9E3779B97F4A7C15))
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        x = x ^ (x >> np.uint64(31))
        return int(x.sum(dtype=np.uint64))


# ---- value store ----------------------------------------------------------------
class Store:
    """One server shard's value store in HBM (psg_store_*)."""

    def __init__(self, kind: int, dtype: int, key_begin: int, key_end: int, capacity: int):
        self.h = C.c_void_p(None)
        _call("psg_store_create", kind, dtype, key_begin, key_end, capacity, C.byref(self.h))
        self.dtype = dtype
        self.esize = _ESIZE[dtype]

    def info(self) -> StoreInfo:
        i = StoreInfo()
        _call("psg_store_get_info", self.h, C.byref(i))
        return i

    def counters(self) -> dict:
        """How the store served its keyed requests (psg_store_counters)."""
        c = (C.c_uint64 * 14)()
        _call("psg_store_counters", self.h, c, 14)
        return {"fused": c[0], "ident": c[1], "notident": c[2], "ordered": c[3], "runs": c[4],
                "run_frames": c[5], "coded": c[6], "lean": c[7], "lean_partial": c[8],
                "strided_runs": c[9], "strided_frames": c[10], "lists": c[11], "notlist": c[12], "strided_single": c[13]}

    def handle(self, flags: int, keys, vals, out, n: int, first_key: int = 0, stream=None) -> None:
        _call("psg_store_handle", self.h, flags, _ptr(keys), first_key, _ptr(vals), _ptr(out), n,
              _s(stream))

    def handle_async(self, flags: int, keys, vals, out, n: int, first_key: int = 0, stream=None) -> int:
        """Launch without waiting (psg_store_handle_async); returns the ticket (0: done)."""
        t = C.c_uint64(0)
        _call("psg_store_handle_async", self.h, flags, _ptr(keys), first_key, _ptr(vals), _ptr(out), n,
              _s(stream), C.byref(t))
        return t.value

    def wait(self, ticket: int = 0) -> None:
        """Complete the requests in flight up to `ticket` (0: all); raises the first failure."""
        _call("psg_store_wait", self.h, ticket)

    def push_frames(self, keys, vals, n: int, first_key: int = 0, stream=None) -> bool:
        """A run of len(vals) Pushes on one key list (psg_store_push_frames):
        keys is a list of device key arrays (one per request) or None for a
        dense run; returns True when one pass served the run."""
        k = len(vals)
        kp = None if keys is None else (C.c_void_p * k)(*[_ptr(x) for x in keys])
        vp_ = (C.c_void_p * k)(*[_ptr(x) for x in vals])
        fused = C.c_int(0)
        _call("psg_store_push_frames", self.h, kp, first_key, vp_, k, n, _s(stream), C.byref(fused))
        return bool(fused.value)

    def run(self, ops, keys, ns, vals, outs, stream=None) -> int:
        """A run of queued requests (psg_store_run): ops[j] PUSH / PULL bits,
        keys[j] device key arrays of ns[j] keys, vals[j] / outs[j] device arrays
        (None where the request does not push / pull).  Returns PSG_RUN_*."""
        k = len(ops)
        ov = (C.c_int * k)(*ops)
        kp = (C.c_void_p * k)(*[_ptr(x) for x in keys])
        nv = (C.c_uint64 * k)(*ns)
        vp_ = (C.c_void_p * k)(*[_ptr(x) for x in vals])
        op_ = (C.c_void_p * k)(*[_ptr(x) for x in outs])
        served = C.c_int(0)
        _call("psg_store_run", self.h, k, ov, kp, nv, vp_, op_, _s(stream), C.byref(served))
        return served.value

    def push_slots_frames(self, slots, vals, n: int, first: int = 0, stream=None) -> None:
        """A run of len(vals) Pushes on a cached slot list, or (slots None) on
        the stretch [first, first + n) (psg_store_push_slots_frames)."""
        k = len(vals)
        vp_ = (C.c_void_p * k)(*[_ptr(x) for x in vals])
        _call("psg_store_push_slots_frames", self.h, _ptr(slots), first, vp_, k, n, _s(stream))

    def resolve(self, keys, n: int, slots, insert: bool = True, stream=None) -> None:
        _call("psg_store_resolve", self.h, _ptr(keys), n, int(insert), _ptr(slots), _s(stream))

    def handle_slots(self, flags: int, slots, vals, out, n: int, stream=None) -> None:
        _call("psg_store_handle_slots", self.h, flags, _ptr(slots), _ptr(vals), _ptr(out), n,
              _s(stream))

    def slots_stretch(self, slots, n: int, stream=None):
        """The first slot when slots[i] == slots[0] + i for every i, else None
        (psg_store_slots_stretch)."""
        f = C.c_uint64(0)
        _call("psg_store_slots_stretch", self.h, _ptr(slots), n, C.byref(f), _s(stream))
        return None if f.value == (1 << 64) - 1 else f.value

    def handle_stretch(self, flags: int, first: int, vals, out, n: int, stream=None) -> None:
        _call("psg_store_handle_stretch", self.h, flags, first, _ptr(vals), _ptr(out), n, _s(stream))

    def sync(self, stream=None) -> None:
        """Wait for the stream's enqueued work through the store's polled word
        (psg_store_sync)."""
        _call("psg_store_sync", self.h, _s(stream))

    def clear(self, stream=None) -> None:
        _call("psg_store_clear", self.h, _s(stream))

    def dump(self):
        i = self.info()
        keys = np.empty(i.size, dtype=np.uint64)
        vals = np.empty(i.size, dtype=_NP[self.dtype])
        _call("psg_store_dump", self.h, keys.ctypes.data_as(C.c_void_p),
              vals.ctypes.data_as(C.c_void_p))
        return keys, vals

    def close(self) -> None:
        if self.h.value:
            _call("psg_store_destroy", self.h)
            self.h = C.c_void_p(None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---- worker side --------------------------------------------------------------
def server_ranges(ns: int):
    b = np.empty(ns, dtype=np.uint64)
    e = np.empty(ns, dtype=np.uint64)
    _call("psg_server_ranges", ns, b.ctypes.data_as(C.c_void_p), e.ctypes.data_as(C.c_void_p))
    return b, e


def slice_keys(keys, n: int, begins: np.ndarray, ends: np.ndarray, lens=None, num_vals=None,
               stream=None):
    ns = len(begins)
    begins = np.ascontiguousarray(begins, dtype=np.uint64)
    ends = np.ascontiguousarray(ends, dtype=np.uint64)
    kp = np.empty(ns + 1, dtype=np.uint64)
    vp = np.empty(ns + 1, dtype=np.uint64)
    _call("psg_slice", _ptr(keys), n, _ptr(lens), n if num_vals is None else num_vals, ns,
          begins.ctypes.data_as(C.c_void_p), ends.ctypes.data_as(C.c_void_p),
          kp.ctypes.data_as(C.c_void_p), vp.ctypes.data_as(C.c_void_p), _s(stream))
    return kp, vp


def merge(segments, elem_size: int, dst, dst_count: int, stream=None) -> None:
    """segments: list of (device ptr or DeviceBuffer, count, first_key)."""
    arr = (Segment * max(len(segments), 1))()
    for i, (p, cnt, fk) in enumerate(segments):
        arr[i].vals = _ptr(p)
        arr[i].count = cnt
        arr[i].first_key = fk
    _call("psg_merge", arr, len(segments), elem_size, _ptr(dst), dst_count, _s(stream))


# ---- multi-GPU ------------------------------------------------------------------
def comm_id() -> bytes:
    n = lib().psg_comm_id_bytes()
    buf = C.create_string_buffer(n)
    _call("psg_comm_get_id", buf)
    return buf.raw


def sort_pairs_u64(keys, vals, n: int, bits: int = 64, stream=None) -> None:
    """Stable device radix sort of (keys, vals) by the low `bits` of the key, in place."""
    _call("psg_sort_pairs_u64", _ptr(keys), _ptr(vals), n, bits, _s(stream))


def bucket_plan(blk: int, nbuckets: int):
    """(offsets, counts) of psg_comm_push_pull's buckets over a block of blk
    elements (host-only: the same numbers the RCCL pipeline uses)."""
    offs = np.zeros(max(nbuckets, 1), np.uint64)
    cnts = np.zeros(max(nbuckets, 1), np.uint64)
    nb = C.c_int(0)
    _call("psg_comm_bucket_plan", blk, nbuckets, offs.ctypes.data_as(C.c_void_p),
          cnts.ctypes.data_as(C.c_void_p), len(offs), C.byref(nb))
    return offs[:nb.value].copy(), cnts[:nb.value].copy()


def keyed_plan(key_pos, nranks: int, n: int) -> int:
    """psg_comm_push_keyed's check of the slicer bounds; returns the longest segment."""
    kp = np.ascontiguousarray(key_pos, dtype=np.uint64)
    m = C.c_uint64(0)
    _call("psg_comm_keyed_plan", kp.ctypes.data_as(C.c_void_p), nranks, n, C.byref(m))
    return m.value


class Comm:
    def __init__(self, uid: bytes, nranks: int, rank: int):
        self.h = C.c_void_p(None)
        buf = C.create_string_buffer(uid, len(uid))
        _call("psg_comm_init", buf, nranks, rank, C.byref(self.h))

    def rank(self) -> tuple:
        """(this rank, ranks in the communicator) as RCCL reports them (psg_comm_rank)."""
        r, n = C.c_int(0), C.c_int(0)
        _call("psg_comm_rank", self.h, C.byref(r), C.byref(n))
        return r.value, n.value

    def sync(self, stream=None, timeout_s: float = 0.0) -> None:
        """Wait for the queued collectives, at most timeout_s; aborts them and raises on a timeout."""
        _call("psg_comm_sync", self.h, _s(stream), timeout_s)

    def abort(self) -> None:
        _call("psg_comm_abort", self.h)

    def push(self, shard: Store, vals, n_total: int, scratch=None, stream=None) -> None:
        _call("psg_comm_push", self.h, shard.h, _ptr(vals), n_total, _ptr(scratch), _s(stream))

    def pull(self, shard: Store, out, n_total: int, stream=None) -> None:
        _call("psg_comm_pull", self.h, shard.h, _ptr(out), n_total, _s(stream))

    def push_pull(self, shard: Store, vals, out, n_total: int, nbuckets: int, stream=None) -> None:
        _call("psg_comm_push_pull", self.h, shard.h, _ptr(vals), _ptr(out), n_total, nbuckets,
              _s(stream))

    def push_keyed(self, shard: Store, keys, vals, n: int, key_pos, stream=None) -> None:
        kp = np.ascontiguousarray(key_pos, dtype=np.uint64)
        _call("psg_comm_push_keyed", self.h, shard.h, _ptr(keys), _ptr(vals), n,
              kp.ctypes.data_as(C.c_void_p), _s(stream))

    def lr_push(self, weights: Store, grads, n_total: int, lr: float, adam=None, iteration=0,
                scratch=None, stream=None) -> None:
        _call("psg_comm_lr_push", self.h, weights.h, _ptr(grads), n_total, lr,
              adam.h if adam else None, iteration, _ptr(scratch), _s(stream))

    def pull_keyed(self, shard: Store, keys, out, n: int, key_pos, stream=None) -> None:
        kp = np.ascontiguousarray(key_pos, dtype=np.uint64)
        _call("psg_comm_pull_keyed", self.h, shard.h, _ptr(keys), _ptr(out), n,
              kp.ctypes.data_as(C.c_void_p), _s(stream))

    def close(self) -> None:
        if self.h.value:
            _call("psg_comm_destroy", self.h)
            self.h = C.c_void_p(None)


# ---- LR -----------------------------------------------------------------------
class Adam:
    def __init__(self, n: int, lr: float, beta1=0.9, beta2=0.999, eps=1e-8):
        self.h = C.c_void_p(None)
        _call("psg_adam_create", n, lr, beta1, beta2, eps, C.byref(self.h))

    def close(self) -> None:
        if self.h.value:
            _call("psg_adam_destroy", self.h)
            self.h = C.c_void_p(None)


def lr_apply(weights: Store, merged, n: int, lr: float, adam: Adam | None, iteration: int,
             stream=None) -> None:
    _call("psg_lr_apply", weights.h, _ptr(merged), n, lr, adam.h if adam else None, iteration,
          _s(stream))


def lr_apply_sum(weights: Store, grads, n: int, lr: float, adam: Adam | None, iteration: int,
                 from_zero: bool = True, stream=None) -> None:
    """psg_lr_apply_sum: merge `grads` (device buffers / pointers, in order) and apply."""
    arr = (C.c_void_p * max(len(grads), 1))(*[_ptr(g) for g in grads])
    _call("psg_lr_apply_sum", weights.h, arr, len(grads), int(from_zero), n, lr,
          adam.h if adam else None, iteration, _s(stream))


def lr_mix_copy(weights: Store, grads, n: int, adam: Adam, stream=None) -> None:
    """psg_lr_mix_copy: the Adam apply's loads and stores with a copy's arithmetic
    (measurement only: it scribbles on the weights and moments)."""
    arr = (C.c_void_p * max(len(grads), 1))(*[_ptr(g) for g in grads])
    _call("psg_lr_mix_copy", weights.h, arr, len(grads), n, adam.h, _s(stream))


# ---- one-shot xGMI exchange ----------------------------------------------------------
def ipc_export(ptr) -> bytes:
    n = lib().psg_ipc_handle_bytes()
    buf = C.create_string_buffer(n)
    _call("psg_ipc_export", C.c_void_p(_ptr(ptr)), buf)
    return buf.raw


def ipc_open(handle: bytes) -> int:
    p = C.c_void_p(None)
    _call("psg_ipc_open", C.create_string_buffer(handle, len(handle)), C.byref(p))
    return p.value


def ipc_close(ptr: int) -> None:
    _call("psg_ipc_close", C.c_void_p(ptr))


class Xgmi:
    """psg_xgmi over peer pointers (own rank: local pointers; others: ipc_open'd)."""

    def __init__(self, nranks: int, rank: int, vals_ptrs, store_ptrs):
        self.h = C.c_void_p(None)
        V = (C.c_void_p * nranks)(*vals_ptrs)
        S = (C.c_void_p * nranks)(*store_ptrs)
        _call("psg_xgmi_create", nranks, rank, V, S, C.byref(self.h))

    def push(self, shard: Store, n_total: int, stream=None) -> None:
        _call("psg_xgmi_push", self.h, shard.h, n_total, _s(stream))

    def pull(self, shard: Store, out, n_total: int, stream=None) -> None:
        _call("psg_xgmi_pull", self.h, shard.h, _ptr(out), n_total, _s(stream))

    def push_range(self, shard: Store, n_total: int, off: int, cnt: int, stream=None) -> None:
        _call("psg_xgmi_push_range", self.h, shard.h, n_total, off, cnt, _s(stream))

    def pull_range(self, shard: Store, out, n_total: int, off: int, cnt: int, stream=None) -> None:
        _call("psg_xgmi_pull_range", self.h, shard.h, _ptr(out), n_total, off, cnt, _s(stream))

    def set_outs(self, out_ptrs) -> None:
        """Every rank's Pull output buffer, mapped here (own rank: local pointer)."""
        O = (C.c_void_p * len(out_ptrs))(*[_ptr(p) for p in out_ptrs])
        _call("psg_xgmi_set_outs", self.h, O)

    def pull_write(self, shard: Store, n_total: int, stream=None) -> None:
        _call("psg_xgmi_pull_write", self.h, shard.h, n_total, _s(stream))

    def pull_write_range(self, shard: Store, n_total: int, off: int, cnt: int, stream=None) -> None:
        _call("psg_xgmi_pull_write_range", self.h, shard.h, n_total, off, cnt, _s(stream))

    def pull_write_slots(self, shard: Store, slots, seg_off: int, seg_n: int, stream=None) -> None:
        _call("psg_xgmi_pull_write_slots", self.h, shard.h, _ptr(slots), seg_off, seg_n, _s(stream))

    def push_slots(self, shard: Store, slots, seg_off: int, seg_n: int, stream=None) -> None:
        _call("psg_xgmi_push_slots", self.h, shard.h, _ptr(slots), seg_off, seg_n, _s(stream))

    def pull_slots(self, shard: Store, peer_slots, seg_offs, seg_ns, out, stream=None) -> None:
        w = len(peer_slots)
        sl = (C.c_void_p * w)(*[_ptr(p) for p in peer_slots])
        offs = np.ascontiguousarray(seg_offs, dtype=np.uint64)
        ns = np.ascontiguousarray(seg_ns, dtype=np.uint64)
        _call("psg_xgmi_pull_slots", self.h, shard.h, sl, offs.ctypes.data_as(C.c_void_p),
              ns.ctypes.data_as(C.c_void_p), _ptr(out), _s(stream))

    def lr_push(self, weights: Store, n_total: int, lr: float, adam=None, iteration=0,
                stream=None) -> None:
        _call("psg_xgmi_lr_push", self.h, weights.h, n_total, lr, adam.h if adam else None,
              iteration, _s(stream))

    def close(self) -> None:
        if self.h.value:
            _call("psg_xgmi_destroy", self.h)
            self.h = C.c_void_p(None)


class NodeBarrier:
    def __init__(self, name: str, nranks: int, rank: int):
        self.h = C.c_void_p(None)
        _call("psg_node_barrier_create", name.encode(), nranks, rank, C.byref(self.h))

    def wait(self, timeout_s: float = 120.0) -> None:
        _call("psg_node_barrier_wait", self.h, timeout_s)

    def close(self) -> None:
        if self.h.value:
            _call("psg_node_barrier_destroy", self.h)
            self.h = C.c_void_p(None)
