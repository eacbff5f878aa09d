"""Lean Pushes validated against their list's verified copy (csrc/psg_store.hip,
k_list_check).

A keyed Push whose list is a subset of the store (coded tiles) is validated
against the store keys at its coded places (k_validate_code: 8 / density B of
store-key lines and the lane codes per key).  Once a learning request of the
list has been validated in full against this K and served lean, its keys are
kept as the list's verified copy, and a later Push of the same device array is
validated by comparing it with that copy (16 B per key, two streams); keys
equal to a list validated against this very K are in range, ascending and at
the cached places.  Every case is bit-exact against the oracle (the
restatement of src/ps/KVApp.h:446-454), and a list that is NOT its copy any
more — rewritten in place, with a key out of range, out of order — wrote
nothing on the copy path and is served with the full validation: the store
sees exactly the reference's sequence, and a rejected request leaves it
unchanged.
"""
import numpy as np
import pytest

import oracle
import psg

pytestmark = pytest.mark.gpu

KMAX = (1 << 64) - 1
ALL = psg.PUSH | psg.PULL


@pytest.fixture(scope="module", autouse=True)
def device():
    assert psg.device_count() >= 1, "no GPU visible"
    psg.set_device(0)
    yield


def dev(a):
    return psg.DeviceBuffer.from_numpy(a)


def populated(n_univ, seed, key_end=KMAX):
    rng = np.random.default_rng(seed)
    univ = np.unique(rng.integers(0, key_end, n_univ, dtype=np.uint64))
    st = psg.Store(psg.SORTED, psg.F32, 0, key_end, 0)
    orc = oracle.Store(psg.F32)
    v0 = oracle.synth(len(univ), psg.F32, seed, 1, -1.0, 1.0)
    st.handle(psg.PUSH, dev(univ), dev(v0), None, len(univ))
    orc.handle(oracle.PUSH, univ, v0, len(univ))
    return rng, univ, st, orc


def subset_n(rng, univ, n):
    """n keys of univ drawn at random (sorted): a subset at density n / len(univ)"""
    return np.sort(rng.choice(univ, n, replace=False))


def push(st, orc, dk, k, seed, flags=psg.PUSH):
    n = len(k)
    v = oracle.synth(n, psg.F32, seed, 1, -1.0, 1.0)
    out = psg.DeviceBuffer(n * 4) if flags & psg.PULL else None
    st.handle(flags, dk, dev(v), out, n)
    exp = orc.handle(flags, k, v, n)
    if out is not None:
        np.testing.assert_array_equal(out.download(np.float32, n), exp)


def same_store(st, orc):
    gk, gv = st.dump()
    ok, ov = orc.dump()
    np.testing.assert_array_equal(gk, ok)
    np.testing.assert_array_equal(gv.view(np.float32), ov)


@pytest.mark.parametrize("density", [0.9, 0.75, 0.7])
def test_repeated_subset_push_takes_the_verified_copy(density):
    rng, univ, st, orc = populated(400000, 11 + int(100 * density))
    k = subset_n(rng, univ, int(len(univ) * density))
    dk = dev(k)
    for r in range(8):
        push(st, orc, dk, k, 100 + r, flags=psg.PUSH if r % 3 else ALL)
    same_store(st, orc)
    c = st.counters()
    assert c["lists"] >= 4 and c["notlist"] == 0, c


def test_list_rewritten_in_place_is_validated_in_full():
    """The same device array, rewritten with another subset of the same length
    (a caller that reuses its buffer): the copy path rejects it, nothing is
    written, the full validation serves it; later Pushes at this K generation
    take the full validation (no copy attempt), and still match."""
    rng, univ, st, orc = populated(300000, 21)
    n = int(len(univ) * 0.9)
    k1 = subset_n(rng, univ, n)
    dk = dev(k1)
    for r in range(4):
        push(st, orc, dk, k1, 200 + r)
    assert st.counters()["lists"] >= 1
    k2 = subset_n(rng, univ, n)
    dk.upload(k2)
    psg.device_sync()
    for r in range(3):
        push(st, orc, dk, k2, 300 + r, flags=ALL if r == 1 else psg.PUSH)
    same_store(st, orc)
    c = st.counters()
    assert c["notlist"] == 1, c


def test_rewritten_list_with_a_key_out_of_range_is_rejected_unchanged():
    end = 1 << 62
    rng, univ, st, orc = populated(200000, 31, key_end=end)
    n = int(len(univ) * 0.9)
    k = subset_n(rng, univ, n)
    dk = dev(k)
    for r in range(4):
        push(st, orc, dk, k, 400 + r)
    assert st.counters()["lists"] >= 1
    bad = k.copy()
    bad[-1] = np.uint64(end + 12345)  # still ascending, outside the shard
    dk.upload(bad)
    psg.device_sync()
    v = oracle.synth(n, psg.F32, 499, 1, -1.0, 1.0)
    with pytest.raises(psg.PsgError):
        st.handle(psg.PUSH, dk, dev(v), None, n)
    same_store(st, orc)  # nothing applied
    assert st.counters()["notlist"] == 1


def test_rewritten_list_out_of_order_takes_the_order_preserving_path():
    rng, univ, st, orc = populated(200000, 41)
    n = int(len(univ) * 0.9)
    k = subset_n(rng, univ, n)
    dk = dev(k)
    for r in range(4):
        push(st, orc, dk, k, 500 + r)
    sw = k.copy()
    sw[[1000, 1001]] = sw[[1001, 1000]]
    dk.upload(sw)
    psg.device_sync()
    push(st, orc, dk, sw, 600, flags=ALL)
    same_store(st, orc)
    assert st.counters()["notlist"] == 1


def test_a_new_key_generation_relearns_the_copy():
    """An insert changes K: the copy is stale (validated against the old K), the
    next Push learns again and the ones after it take the copy."""
    rng, univ, st, orc = populated(200000, 51)
    n = int(len(univ) * 0.8)
    k = subset_n(rng, univ, n)
    dk = dev(k)
    for r in range(4):
        push(st, orc, dk, k, 700 + r)
    before = st.counters()["lists"]
    fresh = np.setdiff1d(univ[::1000] + np.uint64(1), univ)
    push(st, orc, dev(fresh), fresh, 800)  # inserts
    for r in range(4):
        push(st, orc, dk, k, 900 + r)
    same_store(st, orc)
    assert st.counters()["lists"] >= before + 2


def test_requests_in_flight_on_the_verified_copy():
    rng, univ, st, orc = populated(300000, 61)
    n = int(len(univ) * 0.9)
    k = subset_n(rng, univ, n)
    dk = dev(k)
    for r in range(3):
        push(st, orc, dk, k, 1000 + r)
    pend, outs = [], []
    for j in range(12):
        flags = [psg.PUSH, ALL, psg.PUSH, psg.PULL][j % 4]
        v = oracle.synth(n, psg.F32, 1100 + j, 1, -1.0, 1.0)
        dv = dev(v)
        out = psg.DeviceBuffer(n * 4) if flags & psg.PULL else None
        pend.append((st.handle_async(flags, dk, dv if flags & psg.PUSH else None, out, n), dv))
        outs.append((out, orc.handle(flags, k, v if flags & psg.PUSH else None, n)))
        if len(pend) > 4:
            st.wait(pend.pop(0)[0])
    st.wait()
    psg.device_sync()
    for out, exp in outs:
        if out is not None:
            np.testing.assert_array_equal(out.download(np.float32, n), exp)
    same_store(st, orc)
    assert st.counters()["lists"] >= 6
