"""A run of queued Pushes on one key list served in one pass
(psg_store_push_frames / psg_store_push_slots_frames, csrc/psg_frames.hip).

The reference server handles the k Pushes one after the other
(src/internal/Customer.cpp:52-70, src/ps/KVApp.h:446-454); every case here
replays exactly that sequence through the oracle — request j's values added
after request j-1's — on real-valued data, so a different order of additions
would show in the low bits.  psg_store_counters and the `fused` return say
which path served the run: one pass where the lists are one list, request by
request where they are not (a list that differs, an absent key, keys out of
order), with the same bits either way.
"""
import numpy as np
import pytest

import oracle
import psg

pytestmark = pytest.mark.gpu

KMAX = (1 << 64) - 1
NPT = {psg.F32: np.float32, psg.F64: np.float64, psg.F16: np.uint16, psg.BF16: np.uint16}
ES = {psg.F32: 4, psg.F64: 8, psg.F16: 2, psg.BF16: 2}
DTYPES = [psg.F32, psg.F64, psg.F16, psg.BF16]


@pytest.fixture(scope="module", autouse=True)
def device():
    assert psg.device_count() >= 1, "no GPU visible"
    psg.set_device(0)
    yield


def dev(a):
    return psg.DeviceBuffer.from_numpy(np.ascontiguousarray(a))


def frames(dtype, n, k, seed):
    return [oracle.synth(n, dtype, seed + j, 1, -1.0, 1.0) for j in range(k)]


def same_store(st, orc, dtype):
    gk, gv = st.dump()
    ok, ov = orc.dump()
    np.testing.assert_array_equal(gk, ok)
    np.testing.assert_array_equal(gv.view(NPT[dtype]), ov)


def populated(dtype, n_univ, seed):
    rng = np.random.default_rng(seed)
    univ = np.unique(rng.integers(0, KMAX, n_univ, dtype=np.uint64))
    st = psg.Store(psg.SORTED, dtype, 0, KMAX, 0)
    orc = oracle.Store(dtype)
    v0 = oracle.synth(len(univ), dtype, seed, 1, -1.0, 1.0)
    st.handle(psg.PUSH, dev(univ), dev(v0), None, len(univ))
    orc.handle(oracle.PUSH, univ, v0, len(univ))
    return rng, univ, st, orc


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("k", [2, 3, 5, 8, 16])
def test_dense_run_matches_requests_in_order(dtype, k):
    """A dense run on a DENSE store: store += v_0, then v_1, ... (each add
    rounded to the store's dtype), at an unaligned offset with a ragged tail."""
    cap = 1 << 20
    st = psg.Store(psg.DENSE, dtype, 0, cap, cap)
    orc = oracle.Store(dtype)
    base = oracle.synth(cap, dtype, 3, 1, -1.0, 1.0)
    st.handle(psg.PUSH, None, dev(base), None, cap)
    orc.handle(oracle.PUSH, None, base, cap, first_key=0)
    for first, n in [(0, cap), (5, 100003), (1 << 16, 1 << 18)]:
        vs = frames(dtype, n, k, 100 + first)
        assert st.push_frames(None, [dev(v) for v in vs], n, first_key=first)
        for v in vs:
            orc.handle(oracle.PUSH, None, v, n, first_key=first)
    psg.device_sync()
    same_store(st, orc, dtype)
    assert st.counters()["runs"] == 3


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("k", [2, 4, 8])
def test_sorted_run_on_a_stretch_of_the_store(dtype, k):
    """Every worker sends its own copy of one key list (distinct device
    pointers) that is a stretch of the store — the whole store, a stretch at
    an odd slot, a short one: one pass (frames_base / check / apply)."""
    rng, univ, st, orc = populated(dtype, 200000, 11)
    for j, keys in enumerate([univ, univ[3:150001], univ[1001:1001 + 777]]):
        n = len(keys)
        dks = [dev(keys) for _ in range(k)]
        vs = frames(dtype, n, k, 50 + 10 * j)
        assert st.push_frames(dks, [dev(v) for v in vs], n), f"case {j} not served in one pass"
        for v in vs:
            orc.handle(oracle.PUSH, keys, v, n)
    same_store(st, orc, dtype)
    c = st.counters()
    assert c["runs"] == 3 and c["run_frames"] == 3 * k


@pytest.mark.parametrize("dtype", [psg.F32, psg.F16])
def test_sorted_run_on_a_sparse_list_takes_the_slot_form(dtype):
    """Lists that are one list but not a stretch of the store (every 3rd key,
    a random subset): list 0 resolved to slots once, the others checked
    against it, one pass over the slots."""
    rng, univ, st, orc = populated(dtype, 120000, 12)
    k = 5
    for j, keys in enumerate([univ[::3], np.sort(rng.choice(univ, 30001, replace=False))]):
        n = len(keys)
        dks = [dev(keys) for _ in range(k)]
        vs = frames(dtype, n, k, 70 + 10 * j)
        assert st.push_frames(dks, [dev(v) for v in vs], n)
        for v in vs:
            orc.handle(oracle.PUSH, keys, v, n)
    same_store(st, orc, dtype)
    assert st.counters()["runs"] == 2


def test_runs_that_are_not_one_list_are_served_request_by_request():
    """A list that differs from the others in one key (last, first, middle), a
    list with a key the store lacks, and keys out of order: no one-pass form
    applies; the run is served request by request with the reference's
    result — absent keys inserted, the out-of-order list in arrival order —
    and a failed check has written nothing."""
    dtype = psg.F32
    rng, univ, st, orc = populated(dtype, 100000, 13)
    base = univ[10:60010]
    n = len(base)
    last = base.copy()
    last[-1] = univ[60010]  # present, ascending, differs in the last key
    first = base.copy()
    first[0] = univ[9]  # ... in the first key
    shifted = univ[11:60011]  # another stretch of the store
    absent = base.copy()
    absent[n // 2] = base[n // 2] + np.uint64(1)  # a key the store lacks
    shuffled = base.copy()
    shuffled[[5, 6]] = shuffled[[6, 5]]  # out of order
    cases = [[base, base, last, base], [base, first, base], [base, shifted], [base, absent, base],
             [absent, base], [base, shuffled, base]]
    for ci, lists in enumerate(cases):
        vs = frames(dtype, n, len(lists), 200 + 10 * ci)
        fused = st.push_frames([dev(l) for l in lists], [dev(v) for v in vs], n)
        assert not fused, f"case {ci}: lists differ, yet served in one pass"
        for l, v in zip(lists, vs):
            orc.handle(oracle.PUSH, l, v, n)
        same_store(st, orc, dtype)
    assert st.counters()["runs"] == 0


def test_one_frame_and_the_ab_switch_are_plain_requests():
    dtype = psg.F32
    rng, univ, st, orc = populated(dtype, 50000, 14)
    v = frames(dtype, len(univ), 1, 300)[0]
    assert not st.push_frames([dev(univ)], [dev(v)], len(univ))
    orc.handle(oracle.PUSH, univ, v, len(univ))
    same_store(st, orc, dtype)


@pytest.mark.parametrize("k", [2, 3, 8, 16])
def test_cached_slot_and_stretch_runs(k):
    """LR key caching: a run on a cached slot list (sparse: scalar RMWs; a
    stretch: 16-B RMWs) and on a stretch of slots, against k requests."""
    dtype = psg.F32
    rng, univ, st, orc = populated(dtype, 80000, 15)
    for keys in [univ[::2], univ[100:70100]]:
        n = len(keys)
        dk = dev(keys)
        slots = psg.DeviceBuffer(n * 4)
        st.resolve(dk, n, slots, insert=False)
        first = st.slots_stretch(slots, n)
        vs = frames(dtype, n, k, 400 + k)
        st.push_slots_frames(slots, [dev(v) for v in vs], n)
        for v in vs:
            orc.handle(oracle.PUSH, keys, v, n)
        if first is not None:
            vs = frames(dtype, n, k, 500 + k)
            st.push_slots_frames(None, [dev(v) for v in vs], n, first=first)
            for v in vs:
                orc.handle(oracle.PUSH, keys, v, n)
        st.sync()
    same_store(st, orc, dtype)
