"""Identity requests on the SORTED store (csrc/psg_store.hip, k_ident_check /
k_ident_apply): a key list whose every tile holds exactly the store keys of its
cached window is served at the slots those windows give, without a validation
pass or a search.  Every case is checked bit for bit against the oracle (the
restatement of KVApp.h:446-454), and psg_store_counters shows which path ran:
the identity path where it applies, the general path where it does not —
including a list that is trusted but turns out not to be one (it writes
nothing and is served again on the general path).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle
import psg

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
KMAX = (1 << 64) - 1
NPT = {psg.F32: np.float32, psg.F64: np.float64, psg.F16: np.uint16, psg.BF16: np.uint16}
ES = {psg.F32: 4, psg.F64: 8, psg.F16: 2, psg.BF16: 2}
ALL = psg.PUSH | psg.PULL


@pytest.fixture(scope="module", autouse=True)
def device():
    assert psg.device_count() >= 1, "no GPU visible"
    psg.set_device(0)
    yield


def dev(a):
    return psg.DeviceBuffer.from_numpy(a)


def populated(dtype, n_univ, seed):
    rng = np.random.default_rng(seed)
    univ = np.unique(rng.integers(0, KMAX, n_univ, dtype=np.uint64))
    st = psg.Store(psg.SORTED, dtype, 0, KMAX, 0)
    orc = oracle.Store(dtype)
    v0 = oracle.synth(len(univ), dtype, seed, 1, -1.0, 1.0)
    st.handle(psg.PUSH, dev(univ), dev(v0), None, len(univ))
    orc.handle(oracle.PUSH, univ, v0, len(univ))
    return rng, univ, st, orc


def request(st, orc, dtype, flags, dk, k, seed, off=0):
    """One request; off > 0 places the values and the reply off 16-B alignment."""
    n = len(k)
    v = oracle.synth(n, dtype, seed, 1, -1.0, 1.0)
    dv = psg.DeviceBuffer(off + n * ES[dtype])
    out = psg.DeviceBuffer(off + n * ES[dtype])
    if flags & psg.PUSH:
        dv.upload(v, offset=off)
    st.handle(flags, dk, dv.ptr + off if flags & psg.PUSH else None, out.ptr + off if flags & psg.PULL else None, n)
    exp = orc.handle(flags, k, v if flags & psg.PUSH else None, n)
    if flags & psg.PULL:
        np.testing.assert_array_equal(out.download(NPT[dtype], n, offset=off), exp, err_msg=f"flags {flags}")


def same_store(st, orc, dtype):
    gk, gv = st.dump()
    ok, ov = orc.dump()
    np.testing.assert_array_equal(gk, ok)
    np.testing.assert_array_equal(gv.view(NPT[dtype]), ov)


@pytest.mark.parametrize("dtype", [psg.F32, psg.F64, psg.F16, psg.BF16])
def test_identity_requests_whole_store_and_stretches(dtype):
    """The whole key list and contiguous stretches of it (windows starting at
    any slot: aligned and unaligned, partial last units), every op, repeated:
    after the first request trusts the windows, the rest are identity requests."""
    rng, univ, st, orc = populated(dtype, 300000, 41)
    cases = [univ, univ[1:], univ[3:250001], univ[4096:4096 + 8192], univ[777:778 + 5000]]
    for j, k in enumerate(cases):
        dk = dev(k)
        c0 = st.counters()
        for r, flags in enumerate([psg.PUSH, ALL, psg.PULL, psg.PUSH, ALL, psg.PULL]):
            request(st, orc, dtype, flags, dk, k, 100 * j + r)
        c1 = st.counters()
        # the first request searched and trusted the windows; the other five
        # were identity requests, none of which fell back
        assert c1["ident"] - c0["ident"] == 5, (j, c0, c1)
        assert c1["notident"] == c0["notident"], (j, c0, c1)
    same_store(st, orc, dtype)


def test_identity_misaligned_value_buffers():
    """Request values and replies that are not 16-B aligned take the
    per-element form of the same kernels."""
    dtype = psg.F32
    rng, univ, st, orc = populated(dtype, 100000, 43)
    k = univ[8:60008]
    dk = dev(k)
    for r, flags in enumerate([ALL, ALL, psg.PUSH, psg.PULL, ALL]):
        request(st, orc, dtype, flags, dk, k, 300 + r, off=4)
    assert st.counters()["ident"] >= 4
    same_store(st, orc, dtype)


def test_trusted_list_that_is_not_an_identity_list():
    """A sparse subset of the store (every other key): its windows are trusted
    after the first request, the identity attempt fails, writes nothing and the
    request runs again on the general path; later requests on that list stay on
    the general path until K changes."""
    dtype = psg.F32
    rng, univ, st, orc = populated(dtype, 200000, 47)
    k = univ[::2].copy()
    dk = dev(k)
    for r, flags in enumerate([psg.PUSH, ALL, psg.PULL, psg.PUSH, ALL]):
        request(st, orc, dtype, flags, dk, k, 500 + r)
    c = st.counters()
    assert c["ident"] == 1 and c["notident"] == 1, c
    same_store(st, orc, dtype)


@pytest.mark.parametrize("change", ["absent", "inner", "swap", "repeat", "ends"])
def test_identity_list_rewritten_under_the_same_pointer(change):
    """The worker rewrites its key buffer between requests (psg.h allows it):
    an absent key, inner keys replaced, two keys swapped, a key repeated, or the
    ends moved.  The identity attempt on the rewritten list fails (a window end
    or a key does not match), writes nothing, and the general path applies the
    request exactly — inserting, or walking the keys in arrival order."""
    dtype = psg.F32
    rng, univ, st, orc = populated(dtype, 200000, 53)
    n = 120000
    k = univ[5000:5000 + n].copy()
    dk = dev(k)
    for r in range(3):
        request(st, orc, dtype, ALL, dk, k, 700 + r)
    assert st.counters()["ident"] == 2
    bad = k.copy()
    # keys strictly between two neighbours of the list: absent from the store
    mid = k[:-1] + (k[1:] - k[:-1]) // np.uint64(2)
    if change == "absent":
        bad[n // 3] = mid[n // 3 - 1]
    elif change == "inner":
        bad[100:200] = mid[99:199]
    elif change == "swap":
        bad[n // 2], bad[n // 2 + 1] = bad[n // 2 + 1], bad[n // 2]
    elif change == "repeat":
        bad[n // 4 + 1] = bad[n // 4]
    else:
        bad = univ[5001:5001 + n].copy()
    dk.upload(bad)
    for r, flags in enumerate([psg.PUSH, ALL, psg.PULL]):
        request(st, orc, dtype, flags, dk, bad, 800 + r)
    dk.upload(k)
    for r, flags in enumerate([ALL, psg.PULL]):
        request(st, orc, dtype, flags, dk, k, 900 + r)
    same_store(st, orc, dtype)


@pytest.mark.parametrize("depth", [1, 8, 40])
def test_identity_requests_in_flight_with_a_failure_in_the_middle(depth):
    """Identity requests in flight (psg_store_handle_async), one of which is
    not (a trusted list with a hole, used for the first time as one): it writes nothing and
    raises the pending word, every later request in flight is gated, and the
    wait serves them all in their order — bit-exact against the oracle."""
    dtype = psg.F32
    rng, univ, st, orc = populated(dtype, 100000, 59)
    n = 50000
    lists = []
    for j in range(3):
        k = univ[j * 10000:j * 10000 + n].copy()
        lists.append((k, dev(k)))
    for k, dk in lists:  # trust every list's windows
        request(st, orc, dtype, psg.PULL, dk, k, 1)
    # a stretch with one key left out: its windows are trusted after one
    # request, but the tile with the hole is one key short of its window
    odd = np.delete(univ[15000:15000 + n + 1], n // 2)
    dodd = dev(odd)
    request(st, orc, dtype, psg.PULL, dodd, odd, 2)
    reqs, pending = [], []
    for j in range(30):
        if j == 13:
            k, dk = odd, dodd
        else:
            k, dk = lists[j % 3]
        flags = [psg.PUSH, ALL, psg.PULL][j % 3]
        v = oracle.synth(n, dtype, 1000 + j, 1, -1.0, 1.0)
        dv = dev(v)
        out = psg.DeviceBuffer(n * 4) if flags & psg.PULL else None
        t = st.handle_async(flags, dk, dv if flags & psg.PUSH else None, out, n)
        exp = orc.handle(flags, k, v if flags & psg.PUSH else None, n)
        reqs.append((dv, out, exp))
        pending.append(t)
        if len(pending) >= depth:
            st.wait(pending.pop(0))
    st.wait()
    psg.device_sync()
    for j, (_, out, exp) in enumerate(reqs):
        if out is not None:
            np.testing.assert_array_equal(out.download(np.float32, n), exp, err_msg=f"request {j}")
    same_store(st, orc, dtype)
    c = st.counters()
    assert c["ident"] > 0 and c["notident"] == 1, c


def test_identity_switch_off_matches():
    """PSG_RA_IDENT=0 (read once per process) turns the identity kernels off:
    the same sequence in a fresh process, bit-exact, with no identity request."""
    child = r"""
import sys, numpy as np
sys.path[:0] = {paths!r}
import oracle, psg
psg.set_device(0)
rng = np.random.default_rng(61)
univ = np.unique(rng.integers(0, (1 << 64) - 1, 100000, dtype=np.uint64))
st, orc = psg.Store(psg.SORTED, psg.F32, 0, (1 << 64) - 1, 0), oracle.Store()
dk = psg.DeviceBuffer.from_numpy(univ)
n = len(univ)
out = psg.DeviceBuffer(n * 4)
for j in range(5):
    v = oracle.synth(n, psg.F32, 70 + j, 1, -1.0, 1.0)
    st.handle(psg.PUSH | psg.PULL, dk, psg.DeviceBuffer.from_numpy(v), out, n)
    assert np.array_equal(out.download(np.float32, n), orc.handle(oracle.PUSH | oracle.PULL, univ, v, n)), j
print(st.counters()["ident"])
"""
    paths = [os.path.join(os.path.dirname(HERE), "parameter-server_amd", "python"),
             os.path.join(os.path.dirname(HERE), "oracle")]
    # the first request inserts into the empty store (two-pass), the second
    # searches and trusts the windows, the last three are identity requests
    for env_val, want in (("0", "0"), ("1", "3")):
        env = dict(os.environ, PSG_RA_IDENT=env_val)
        r = subprocess.run([sys.executable, "-c", child.format(paths=paths)], env=env,
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        assert r.stdout.strip().splitlines()[-1] == want, (env_val, r.stdout)


@pytest.mark.parametrize("dtype", [psg.F32, psg.F64, psg.F16, psg.BF16])
def test_cached_slot_list_served_as_a_stretch(dtype):
    """psg_store_slots_stretch finds a resolved slot list that is a stretch of
    the store (slots[i] == first + i) — the whole list, any contiguous part of
    it — and nothing else (a sparse list, a list with an absent key);
    psg_store_handle_stretch then serves it without the slot stream, bit-exact
    against the oracle, at aligned and unaligned first slots and value buffers."""
    rng, univ, st, orc = populated(dtype, 120000, 67)
    for lo, hi in [(0, len(univ)), (3, 70003), (4096, 4096 + 8191), (len(univ) - 1, len(univ))]:
        k = univ[lo:hi]
        n = len(k)
        slots = psg.DeviceBuffer(n * 4)
        st.resolve(dev(k), n, slots, insert=False)
        first = st.slots_stretch(slots, n)
        assert first == lo, (lo, hi, first)
        for off in (0, 4):
            for r, flags in enumerate([psg.PUSH, ALL, psg.PULL]):
                v = oracle.synth(n, dtype, 40 * lo + 10 * off + r, 1, -1.0, 1.0)
                dv = psg.DeviceBuffer(off + n * ES[dtype])
                out = psg.DeviceBuffer(off + n * ES[dtype])
                dv.upload(v, offset=off)
                st.handle_stretch(flags, first, dv.ptr + off if flags & psg.PUSH else None,
                                  out.ptr + off if flags & psg.PULL else None, n)
                exp = orc.handle(flags, k, v if flags & psg.PUSH else None, n)
                if flags & psg.PULL:
                    np.testing.assert_array_equal(out.download(NPT[dtype], n, offset=off), exp)
    same_store(st, orc, dtype)
    # not stretches: every other key; a key the store lacks (slot UINT32_MAX)
    k = univ[::2].copy()
    slots = psg.DeviceBuffer(len(k) * 4)
    st.resolve(dev(k), len(k), slots, insert=False)
    assert st.slots_stretch(slots, len(k)) is None
    k = univ[100:200].copy()
    k[50] = k[49] + (k[50] - k[49]) // np.uint64(2)
    slots = psg.DeviceBuffer(len(k) * 4)
    st.resolve(dev(k), len(k), slots, insert=False)
    assert st.slots_stretch(slots, len(k)) is None
    # a stretch past the store is refused
    with pytest.raises(psg.PsgError) as ei:
        st.handle_stretch(psg.PULL, len(univ) - 5, None, psg.DeviceBuffer(40), 10)
    assert ei.value.code == 4


def test_store_sync_returns_with_the_reply_in_memory():
    """psg_store_sync: after a stretch Pull into pinned host memory on a user
    stream, the reply is readable as soon as the call returns (no other wait);
    with keyed requests in flight it reaps them first; with nothing enqueued
    it returns at once."""
    import ctypes as C
    rng, univ, st, orc = populated(psg.F32, 200000, 71)
    n = len(univ)
    slots = psg.DeviceBuffer(n * 4)
    st.resolve(dev(univ), n, slots, insert=False)
    first = st.slots_stretch(slots, n)
    assert first == 0
    s = psg.Stream()
    host = C.c_void_p(None)
    psg._call("psg_host_alloc", C.byref(host), C.c_size_t(n * 4))
    try:
        view = np.ctypeslib.as_array((C.c_float * n).from_address(host.value))
        st.sync(s)  # nothing enqueued
        for r in range(3):
            v = oracle.synth(n, psg.F32, 900 + r, 1, -1.0, 1.0)
            dv = dev(v)
            view[:] = np.nan
            st.handle_stretch(ALL, first, dv, host.value, n, s)
            st.sync(s)
            exp = orc.handle(ALL, univ, v, n)
            np.testing.assert_array_equal(view, exp)
        # a keyed request in flight on another stream is reaped first
        v = oracle.synth(n, psg.F32, 950, 1, -1.0, 1.0)
        dk, dv = dev(univ), dev(v)  # held until the request is reaped
        st.handle_async(psg.PUSH, dk, dv, None, n)
        orc.handle(psg.PUSH, univ, v, n)
        st.sync(s)
        same_store(st, orc, psg.F32)
    finally:
        psg._call("psg_host_free", host)
        s.close()


def stretch_union(univ, m, gap, start=0):
    """m stretches of the sorted store keys univ with `gap` store keys left out
    between consecutive ones: a key list that is not one stretch of the store
    (the identity request fails on it) but whose tiles mostly are."""
    n = len(univ)
    per = (n - start - gap * (m - 1)) // m
    parts = [univ[start + j * (per + gap): start + j * (per + gap) + per] for j in range(m)]
    return np.concatenate(parts)


@pytest.mark.parametrize("dtype", [psg.F32, psg.F16])
@pytest.mark.parametrize("m", [2, 16, 64])
def test_stretch_union_lists_take_stretch_tiles(dtype, m):
    """A key list made of m disjoint stretches of the store:
    the identity attempt fails once; afterwards the general path's validation
    pass marks every tile that is a stretch of the store (k_validate_windows,
    chunk_ok) and k_resolve_apply serves those at slots lo + i without a key
    re-read — seam tiles take the search.  Synchronous and in flight, every op,
    bit-exact against the oracle."""
    rng, univ, st, orc = populated(dtype, 400000, 91 + m)
    k = stretch_union(univ, m, 100, start=7)
    n = len(k)
    dk = dev(k)
    for r, flags in enumerate([psg.PUSH, ALL, psg.PULL, psg.PUSH, ALL, psg.PUSH]):
        request(st, orc, dtype, flags, dk, k, 1000 * m + r)
    c = st.counters()
    assert c["notident"] == 1, c
    reqs, pending = [], []
    for j in range(12):
        flags = [psg.PUSH, ALL, psg.PUSH, psg.PULL][j % 4]
        v = oracle.synth(n, dtype, 2000 * m + j, 1, -1.0, 1.0)
        dv = dev(v)
        out = psg.DeviceBuffer(n * ES[dtype]) if flags & psg.PULL else None
        pending.append(st.handle_async(flags, dk, dv if flags & psg.PUSH else None, out, n))
        reqs.append((dv, out, orc.handle(flags, k, v if flags & psg.PUSH else None, n)))
        if len(pending) > 4:
            st.wait(pending.pop(0))
    st.wait()
    psg.device_sync()
    for j, (_, out, exp) in enumerate(reqs):
        if out is not None:
            np.testing.assert_array_equal(out.download(NPT[dtype], n), exp, err_msg=f"request {j}")
    same_store(st, orc, dtype)


def test_stretch_union_list_with_a_key_out_of_range_is_rejected():
    """A stretch-union list whose last key lies outside the shard's range: the
    validation pass rejects the whole request (PSG_ERR_RANGE) and no tile —
    stretch tiles included — writes anything."""
    dtype = psg.F32
    rng = np.random.default_rng(97)
    ke = 1 << 62
    univ = np.unique(rng.integers(0, ke, 200000, dtype=np.uint64))
    st = psg.Store(psg.SORTED, dtype, 0, ke, 0)
    orc = oracle.Store(dtype)
    v0 = oracle.synth(len(univ), dtype, 3, 1, -1.0, 1.0)
    st.handle(psg.PUSH, dev(univ), dev(v0), None, len(univ))
    orc.handle(oracle.PUSH, univ, v0, len(univ))
    k = stretch_union(univ, 8, 50)
    dk = dev(k)
    for r in range(3):
        request(st, orc, dtype, psg.PUSH, dk, k, 40 + r)
    bad = np.concatenate([k, np.array([ke + 5], np.uint64)])
    v = oracle.synth(len(bad), dtype, 77, 1, -1.0, 1.0)
    with pytest.raises(psg.PsgError) as ei:
        st.handle(psg.PUSH, dev(bad), dev(v), None, len(bad))
    assert ei.value.code == 4
    same_store(st, orc, dtype)
    request(st, orc, dtype, ALL, dk, k, 50)
    same_store(st, orc, dtype)


def test_stretch_tiles_switch_off_matches():
    """PSG_RA_MIDENT=0 (read once per process) keeps every tile on the search
    path: the same stretch-union sequence in fresh processes, both bit-exact."""
    child = r"""
import sys, numpy as np
sys.path[:0] = {paths!r}
import oracle, psg
psg.set_device(0)
rng = np.random.default_rng(63)
univ = np.unique(rng.integers(0, (1 << 64) - 1, 300000, dtype=np.uint64))
st, orc = psg.Store(psg.SORTED, psg.F32, 0, (1 << 64) - 1, 0), oracle.Store()
st.handle(psg.PUSH, psg.DeviceBuffer.from_numpy(univ), psg.DeviceBuffer.from_numpy(np.ones(len(univ), np.float32)), None, len(univ))
orc.handle(oracle.PUSH, univ, np.ones(len(univ), np.float32), len(univ))
k = np.concatenate([univ[j * 30000 + 11: j * 30000 + 29000] for j in range(10)])
dk = psg.DeviceBuffer.from_numpy(k)
n = len(k)
out = psg.DeviceBuffer(n * 4)
for j in range(6):
    v = oracle.synth(n, psg.F32, 70 + j, 1, -1.0, 1.0)
    st.handle(psg.PUSH | psg.PULL, dk, psg.DeviceBuffer.from_numpy(v), out, n)
    assert np.array_equal(out.download(np.float32, n), orc.handle(oracle.PUSH | oracle.PULL, k, v, n)), j
gk, gv = st.dump()
ok, ov = orc.dump()
assert np.array_equal(gk, ok) and np.array_equal(gv, ov)
print("ok")
"""
    paths = [os.path.join(os.path.dirname(HERE), "parameter-server_amd", "python"),
             os.path.join(os.path.dirname(HERE), "oracle")]
    for env_val in ("0", "1"):
        env = dict(os.environ, PSG_RA_MIDENT=env_val)
        r = subprocess.run([sys.executable, "-c", child.format(paths=paths)], env=env,
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        assert r.stdout.strip().splitlines()[-1] == "ok"
