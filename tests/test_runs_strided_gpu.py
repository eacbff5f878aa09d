"""Runs of queued requests on interleaved key lists (psg_store_run,
csrc/psg_runs.hip).

The reference server takes its queued requests one at a time
(src/internal/Customer.cpp:52-70) and serves each with its own loop
(src/ps/KVApp.h:446-454).  In the reference benchmark's key layout
(tests/test_kv_app_benchmark.cpp:47-52: worker r sends kMaxKey / num * i + r)
the lists of nw workers interleave in every server's store with period nw, so
the requests queued at a server are distinct phases of one period: pairwise
disjoint, and one pass over the slots they span serves them.  Every case here
replays the run's requests in order through the oracle — Pushes, Pulls and
PushPulls, real-valued so any misplaced or doubled add shows in the bits — and
compares the store and every reply bit for bit; `served` and the store
counters say which path ran.  Runs that are not strided (overlapping lists,
absent keys, a list that leaves its phase part-way, a period above 64) are
served request by request with the same result, and a rejected pass has
written nothing.
"""
import numpy as np
import pytest

import oracle
import psg

pytestmark = pytest.mark.gpu

KMAX = (1 << 64) - 1
NPT = {psg.F32: np.float32, psg.F64: np.float64, psg.F16: np.uint16, psg.BF16: np.uint16}
DTYPES = [psg.F32, psg.F64, psg.F16, psg.BF16]
PUSH, PULL = psg.PUSH, psg.PULL


@pytest.fixture(scope="module", autouse=True)
def device():
    assert psg.device_count() >= 1, "no GPU visible"
    psg.set_device(0)
    yield


def dev(a):
    return psg.DeviceBuffer.from_numpy(np.ascontiguousarray(a))


def layout(num, P, head=0, tail=0, seed=0):
    """The benchmark's keys for P workers: list r = step * i + r (i < num),
    plus `head` keys below and `tail` keys above the interleaved block."""
    step = KMAX // (num + head + tail + 4)
    base = np.uint64(step * (head + 1))
    lists = [base + np.arange(num, dtype=np.uint64) * np.uint64(step) + np.uint64(r) for r in range(P)]
    extra = []
    if head:
        extra.append(np.arange(head, dtype=np.uint64) * np.uint64(step) + np.uint64(7))
    if tail:
        extra.append(base + np.uint64(step) * np.uint64(num) + np.arange(tail, dtype=np.uint64) * np.uint64(step))
    return lists, extra


def populated(dtype, lists, extra, seed):
    """A SORTED store holding every list (and the extra keys), filled with
    real-valued data by one Push per list — the same on the oracle."""
    st = psg.Store(psg.SORTED, dtype, 0, KMAX, 0)
    orc = oracle.Store(dtype)
    for j, l in enumerate(list(lists) + list(extra)):
        v = oracle.synth(len(l), dtype, seed + j, 1, -1.0, 1.0)
        st.handle(PUSH, dev(l), dev(v), None, len(l))
        orc.handle(oracle.PUSH, l, v, len(l))
    return st, orc


def same_store(st, orc, dtype):
    gk, gv = st.dump()
    ok, ov = orc.dump()
    np.testing.assert_array_equal(gk, ok)
    np.testing.assert_array_equal(gv.view(NPT[dtype]), ov)


def run_both(st, orc, dtype, reqs, seed):
    """reqs: [(op, keys)] in arrival order.  Serves them as one run on the GPU
    and one by one on the oracle; compares every Pull reply.  Returns served."""
    k = len(reqs)
    ops, dkeys, ns, dvals, douts, hv = [], [], [], [], [], []
    for j, (op, keys) in enumerate(reqs):
        # keys: a host array (uploaded for this run), or (host array, device
        # copy) for a list the caller keeps in HBM from run to run, as a
        # worker does (the store learns lists by their device pointer)
        keys, dk = keys if isinstance(keys, tuple) else (keys, dev(keys))
        n = len(keys)
        v = oracle.synth(n, dtype, seed + j, 1, -1.0, 1.0) if op & PUSH else None
        ops.append(op)
        dkeys.append(dk)
        ns.append(n)
        dvals.append(dev(v) if v is not None else None)
        douts.append(psg.DeviceBuffer(n * np.dtype(NPT[dtype]).itemsize) if op & PULL else None)
        hv.append(v)
    served = st.run(ops, dkeys, ns, dvals, douts)
    for j, (op, keys) in enumerate(reqs):
        keys = keys[0] if isinstance(keys, tuple) else keys
        exp = orc.handle(op, keys, hv[j], len(keys))
        if op & PULL:
            got = douts[j].download(NPT[dtype], len(keys))
            np.testing.assert_array_equal(got, exp, err_msg=f"reply of request {j}")
    return served


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("P", [2, 4, 8])
def test_interleaved_pushes_are_one_pass(dtype, P):
    """P workers' Pushes, arriving in a shuffled order, on the benchmark's
    interleaved lists: one strided pass, bit for bit the k requests."""
    num = 50001
    lists, extra = layout(num, P, head=3, tail=5)
    st, orc = populated(dtype, lists, extra, 10)
    rng = np.random.default_rng(P)
    for rep in range(3):
        order = rng.permutation(P)
        served = run_both(st, orc, dtype, [(PUSH, lists[r]) for r in order], 100 + 10 * rep)
        assert served == psg.RUN_STRIDED
    same_store(st, orc, dtype)
    c = st.counters()
    assert c["strided_runs"] == 3 and c["strided_frames"] == 3 * P


@pytest.mark.parametrize("dtype", [psg.F32, psg.F16])
@pytest.mark.parametrize("P", [4, 8])
def test_mixed_pushes_pulls_and_pushpulls(dtype, P):
    """A run mixing Pushes, Pulls and PushPulls of distinct workers (some
    phases absent: k < P), the lists of unequal length (the last row ragged):
    one pass; every Pull reads the value the sequence gives it."""
    num = 40000
    lists, extra = layout(num, P, head=1)
    # ragged: the last two phases one key shorter (the last row of the store
    # holds the first P - 2 phases only, so the layout stays strided)
    lists = [l if r < P - 2 else l[:-1] for r, l in enumerate(lists)]
    st, orc = populated(dtype, lists, extra, 20)
    rng = np.random.default_rng(7 * P)
    for rep in range(4):
        k = P if rep % 2 == 0 else P - 1
        phases = rng.permutation(P)[:k]
        reqs = [(int(rng.choice([PUSH, PULL, PUSH | PULL])), lists[r]) for r in phases]
        assert run_both(st, orc, dtype, reqs, 300 + 10 * rep) == psg.RUN_STRIDED
    same_store(st, orc, dtype)


def test_pull_only_run_is_one_checked_pass():
    dtype = psg.F32
    P = 8
    lists, extra = layout(30000, P)
    st, orc = populated(dtype, lists, extra, 30)
    assert run_both(st, orc, dtype, [(PULL, lists[r]) for r in [3, 0, 7, 1]], 400) == psg.RUN_STRIDED
    same_store(st, orc, dtype)


def test_same_list_runs_still_take_the_frames_pass():
    """Pushes of nw workers on ONE list (a BSP round): the same-list pass, each
    key's values added in arrival order."""
    dtype = psg.F32
    lists, extra = layout(60000, 4)
    st, orc = populated(dtype, lists, extra, 40)
    for rep in range(2):
        assert run_both(st, orc, dtype, [(PUSH, lists[1])] * 5, 500 + 10 * rep) == psg.RUN_SAME_LIST
    # and after interleaved runs (the hint) still
    assert run_both(st, orc, dtype, [(PUSH, lists[r]) for r in range(4)], 520) == psg.RUN_STRIDED
    assert run_both(st, orc, dtype, [(PUSH, lists[2])] * 3, 530) == psg.RUN_SAME_LIST
    assert run_both(st, orc, dtype, [(PUSH, lists[r]) for r in (2, 0)], 540) == psg.RUN_STRIDED
    same_store(st, orc, dtype)
    assert st.counters()["runs"] == 3


def test_runs_that_are_not_strided_are_served_request_by_request():
    """Overlapping lists (a worker's Push and its Pull), a list with an absent
    key (inserted), a list that leaves its phase part-way, and a period above
    64: request by request, the sequence's result, and the failed passes have
    written nothing (the store matches the oracle after every run)."""
    dtype = psg.F32
    P = 4
    lists, extra = layout(20000, P)
    st, orc = populated(dtype, lists, extra, 50)
    n = len(lists[0])
    absent = lists[2].copy()
    absent[n // 2] += np.uint64(P)  # between two rows: not in the store
    leaves = lists[3].copy()
    leaves[n - 7] = lists[0][n - 7]  # phase 0 instead of 3, near the end
    leaves[n - 7:].sort()
    cases = [
        [(PUSH, lists[0]), (PULL, lists[0])],
        [(PUSH, lists[0]), (PUSH | PULL, lists[1]), (PUSH, lists[0])],
        [(PUSH, lists[1]), (PUSH, absent), (PULL, lists[0])],
        [(PUSH, lists[0]), (PUSH, lists[1]), (PUSH, leaves)],
        [(PULL, lists[0]), (PULL, leaves)],
    ]
    for ci, reqs in enumerate(cases):
        served = run_both(st, orc, dtype, reqs, 600 + 10 * ci)
        assert served == psg.RUN_ONE_BY_ONE, f"case {ci} served as {served}"
        same_store(st, orc, dtype)
    # the insert changed K: the interleaved lists (one of them now with an extra
    # key in its phase's rows? no: the absent key sits between rows) — lists 0,1
    # are no longer strided across the inserted key's row; served one by one or
    # strided, the result is the sequence's
    run_both(st, orc, dtype, [(PUSH, lists[0]), (PUSH, lists[1])], 700)
    same_store(st, orc, dtype)


def test_wide_period_is_not_strided():
    """Lists interleaved with period 80 (> 64 phases): request by request."""
    dtype = psg.F32
    lists, extra = layout(5000, 80)
    st, orc = populated(dtype, lists, [], 60)
    served = run_both(st, orc, dtype, [(PUSH, lists[r]) for r in (5, 9, 70)], 800)
    assert served == psg.RUN_ONE_BY_ONE
    same_store(st, orc, dtype)


def test_a_rejected_request_stops_the_run():
    """A key outside the store's range: the run is served one by one up to
    that request, which fails with PSG_ERR_RANGE; the requests before it are
    applied, the failing one wrote nothing."""
    dtype = psg.F32
    P = 4
    lists, _ = layout(10000, P)
    hi = int(lists[P - 1][-1]) + 1
    st = psg.Store(psg.SORTED, dtype, 0, hi, 0)
    orc = oracle.Store(dtype)
    for j, l in enumerate(lists):
        v = oracle.synth(len(l), dtype, 70 + j, 1, -1.0, 1.0)
        st.handle(PUSH, dev(l), dev(v), None, len(l))
        orc.handle(oracle.PUSH, l, v, len(l))
    bad = lists[2].copy()
    bad[-1] = np.uint64(hi + 5)
    v0 = oracle.synth(len(lists[0]), dtype, 900, 1, -1.0, 1.0)
    v1 = oracle.synth(len(bad), dtype, 901, 1, -1.0, 1.0)
    with pytest.raises(psg.PsgError):
        st.run([PUSH, PUSH], [dev(lists[0]), dev(bad)], [len(lists[0]), len(bad)], [dev(v0), dev(v1)], [None, None])
    orc.handle(oracle.PUSH, lists[0], v0, len(lists[0]))
    same_store(st, orc, dtype)


def test_a_learnt_list_on_its_own_takes_the_strided_pass():
    """After a strided run, a request of one of its lists on its own (the
    first of a step to reach its server) is a strided pass too — its phase's
    slots of the rows — bit for bit the request; a list the store has not
    seen in a strided run is served as one request."""
    dtype = psg.F32
    P = 4
    lists, extra = layout(40000, P, head=2)
    st, orc = populated(dtype, lists, extra, 90)
    kept = [(l, dev(l)) for l in lists]
    assert run_both(st, orc, dtype, [(PUSH, kept[r]) for r in (1, 3, 0, 2)], 900) == psg.RUN_STRIDED
    for j, (op, r) in enumerate([(PUSH, 2), (PULL, 0), (PUSH | PULL, 3), (PULL, 2)]):
        assert run_both(st, orc, dtype, [(op, kept[r])], 910 + 10 * j) == psg.RUN_STRIDED
    # the same keys at another device address: not learnt, one request
    assert run_both(st, orc, dtype, [(PUSH, lists[1])], 980) == psg.RUN_ONE_BY_ONE
    assert run_both(st, orc, dtype, [(PUSH, extra[0])], 990) == psg.RUN_ONE_BY_ONE
    same_store(st, orc, dtype)
    c = st.counters()
    assert c["strided_single"] == 4 and c["strided_runs"] == 1, c
