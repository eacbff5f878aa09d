"""Parity of the HIP path (through the psg C-ABI) with the CPU oracle.

Bar: bit-exact for every integer / index result and for the float sums of the
reference's integer-valued test data; real-valued f32 sums are also bit-exact
here because both sides add the same two operands in the same order per
request (the tolerance the north star allows, 1e-6 relative, is asserted where
orders may differ: tests/test_dist.py).
"""
import os

import numpy as np
import pytest

import oracle
import psg
from kv_pipeline import GpuKV, run_kv_app, run_my

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "golden.npz"))
KMAX = (1 << 64) - 1
NPT = {psg.F32: np.float32, psg.F64: np.float64, psg.F16: np.uint16, psg.BF16: np.uint16}
ES = {psg.F32: 4, psg.F64: 8, psg.F16: 2, psg.BF16: 2}


@pytest.fixture(scope="module", autouse=True)
def device():
    assert psg.device_count() >= 1, "no GPU visible"
    psg.set_device(0)
    yield


def dev(a):
    return psg.DeviceBuffer.from_numpy(a)


def synth(n, dtype, seed, mode=0, lo=0.0, hi=1000.0):
    return oracle.synth(n, dtype, seed, mode, lo, hi)


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("dtype", [psg.F32, psg.F64, psg.F16, psg.BF16])
@pytest.mark.parametrize("mode", [0, 1])
def test_synth_generator_bitexact(dtype, mode):
    n = 100003
    b = psg.DeviceBuffer(n * ES[dtype])
    lo, hi = (0.0, 1000.0) if mode == 0 else (-1.0, 1.0)
    b.fill_synth(n, dtype, 77, mode, lo, hi)
    got = b.download(NPT[dtype], n)
    np.testing.assert_array_equal(got, oracle.synth(n, dtype, 77, mode, lo, hi))


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("dtype", [psg.F32, psg.F64, psg.F16, psg.BF16])
@pytest.mark.parametrize("n,off", [(1, 0), (3, 1), (1000, 0), (4099, 5), (65536, 3), (262147, 0)])
def test_dense_requests_vs_oracle(dtype, n, off):
    kb = 1000
    cap = n + off + 7
    st = psg.Store(psg.DENSE, dtype, kb, kb + cap + 100, cap)
    orc = oracle.Store(dtype)
    mode = 1 if dtype in (psg.F32, psg.F64) else 0
    v1 = synth(n, dtype, 1, mode, -1.0 if mode else 0.0, 1.0 if mode else 1000.0)
    v2 = synth(n, dtype, 2, mode, -1.0 if mode else 0.0, 1.0 if mode else 1000.0)
    d1, d2 = dev(v1), dev(v2)
    out = psg.DeviceBuffer(n * ES[dtype])
    fk = kb + off
    st.handle(psg.PUSH, None, d1, None, n, first_key=fk)
    orc.handle(oracle.PUSH, None, v1, n, first_key=fk)
    st.handle(psg.PUSH | psg.PULL, None, d2, out, n, first_key=fk)
    exp = orc.handle(oracle.PUSH | oracle.PULL, None, v2, n, first_key=fk)
    np.testing.assert_array_equal(out.download(NPT[dtype], n), exp)
    st.handle(psg.PULL, None, None, out, n, first_key=fk)
    exp = orc.handle(oracle.PULL, None, None, n, first_key=fk)
    np.testing.assert_array_equal(out.download(NPT[dtype], n), exp)
    # untouched slots stayed zero
    _, vals = st.dump()
    assert not np.any(vals[:off].view(np.uint8)) and not np.any(vals[off + n:].view(np.uint8))


def test_dense_full_size_64m_integer_exact():
    """configs[1] size: 64 M floats, integer-valued, so every sum is exact."""
    n = 64 << 20
    st = psg.Store(psg.DENSE, psg.F32, 0, n, n)
    v = psg.DeviceBuffer(n * 4)
    v.fill_synth(n, psg.F32, 7, 0, 0.0, 1000.0)
    out = psg.DeviceBuffer(n * 4)
    for _ in range(3):
        st.handle(psg.PUSH, None, v, None, n)
    st.handle(psg.PULL, None, None, out, n)
    host_v = v.download(np.float32, n)
    np.testing.assert_array_equal(out.download(np.float32, n), host_v * 3)
    st.handle(psg.PUSH | psg.PULL, None, v, out, n)
    np.testing.assert_array_equal(out.download(np.float32, n), host_v * 4)
    # spot check against the generator's restatement
    np.testing.assert_array_equal(host_v[:4096], oracle.synth(4096, oracle.F32, 7, 0, 0.0, 1000.0))


def test_dense_keyed_requests():
    kb = 50
    st = psg.Store(psg.DENSE, psg.F32, kb, 10_000, 4096)
    orc = oracle.Store()
    rng = np.random.default_rng(3)
    keys = np.unique(rng.integers(kb, kb + 4096, 1500)).astype(np.uint64)
    v = rng.uniform(-1, 1, len(keys)).astype(np.float32)
    out = psg.DeviceBuffer(len(keys) * 4)
    st.handle(psg.PUSH | psg.PULL, dev(keys), dev(v), out, len(keys))
    exp = orc.handle(oracle.PUSH | oracle.PULL, keys, v, len(keys))
    np.testing.assert_array_equal(out.download(np.float32, len(keys)), exp)
    with pytest.raises(psg.PsgError) as ei:
        st.handle(psg.PUSH, dev(np.array([kb + 5000], np.uint64)), dev(v[:1]), None, 1)
    assert ei.value.code == 4  # PSG_ERR_RANGE


# ---------------------------------------------------------------------------
def _sorted_sequence(n_univ, seed):
    rng = np.random.default_rng(seed)
    univ = np.unique(rng.integers(1 << 40, 1 << 62, n_univ, dtype=np.uint64))
    reqs = []
    for r in range(8):
        k = np.sort(rng.choice(univ, size=rng.integers(1, len(univ)), replace=False))
        flags = [psg.PUSH, psg.PULL, psg.PUSH | psg.PULL][r % 3]
        reqs.append((flags, k.astype(np.uint64), rng.uniform(-1, 1, len(k)).astype(np.float32)))
    reqs.append((psg.PUSH, univ, rng.uniform(-1, 1, len(univ)).astype(np.float32)))
    reqs.append((psg.PUSH | psg.PULL, univ, rng.uniform(-1, 1, len(univ)).astype(np.float32)))
    return reqs


@pytest.mark.parametrize("dtype", [psg.F32, psg.F64, psg.F16, psg.BF16])
@pytest.mark.parametrize("n_univ,seed", [(50, 1), (5000, 2), (300000, 3)])
def test_sorted_store_vs_oracle(n_univ, seed, dtype):
    """Every dtype through the fused resolve + apply: f32 takes the 16-B vector
    paths, f64 / f16 / bf16 the scalar ones."""
    st = psg.Store(psg.SORTED, dtype, 0, KMAX, 0)
    orc = oracle.Store(dtype)
    for j, (flags, k, _) in enumerate(_sorted_sequence(n_univ, seed)):
        n = len(k)
        v = synth(n, dtype, 1000 * seed + j, 1, -1.0, 1.0)
        out = psg.DeviceBuffer(n * ES[dtype]) if flags & psg.PULL else None
        st.handle(flags, dev(k), dev(v) if flags & psg.PUSH else None, out, n)
        exp = orc.handle(flags, k, v if flags & psg.PUSH else None, n)
        if out is not None:
            np.testing.assert_array_equal(out.download(NPT[dtype], n), exp)
    gk, gv = st.dump()
    ok, ov = orc.dump()
    np.testing.assert_array_equal(gk, ok)  # pulls of absent keys inserted them too
    np.testing.assert_array_equal(gv.view(NPT[dtype]), ov)  # f16 as bits, like the oracle


def test_sorted_store_benchmark_layout():
    """test_kv_app_benchmark keys (kMaxKey/num*i + rank): first Push inserts, then dense fast path."""
    num = 1 << 20
    keys = (np.arange(num, dtype=np.uint64) * np.uint64(KMAX // num)).astype(np.uint64)
    st = psg.Store(psg.SORTED, psg.F32, 0, KMAX, 0)
    v = psg.DeviceBuffer(num * 4)
    v.fill_synth(num, psg.F32, 9, 0, 0.0, 1000.0)
    dk = dev(keys)
    for _ in range(3):
        st.handle(psg.PUSH, dk, v, None, num)
    out = psg.DeviceBuffer(num * 4)
    st.handle(psg.PULL, dk, None, out, num)
    np.testing.assert_array_equal(out.download(np.float32, num), v.download(np.float32, num) * 3)
    assert st.info().size == num


def test_sorted_resolve_and_slot_requests():
    rng = np.random.default_rng(11)
    keys = np.unique(rng.integers(0, 1 << 63, 20000, dtype=np.uint64))
    n = len(keys)
    st = psg.Store(psg.SORTED, psg.F32, 0, KMAX, 0)
    orc = oracle.Store()
    slots = psg.DeviceBuffer(n * 4)
    st.resolve(dev(keys), n, slots, insert=True)  # inserts, like operator[]
    s = slots.download(np.uint32, n)
    assert sorted(s.tolist()) == list(range(n))
    v = rng.uniform(-1, 1, n).astype(np.float32)
    out = psg.DeviceBuffer(n * 4)
    for _ in range(2):
        st.handle_slots(psg.PUSH | psg.PULL, slots, dev(v), out, n)
        exp = orc.handle(oracle.PUSH | oracle.PULL, keys, v, n)
        np.testing.assert_array_equal(out.download(np.float32, n), exp)
    # resolve without insert: absent keys -> UINT32_MAX
    more = np.array([keys[0], keys[0] + 1], dtype=np.uint64)
    st.resolve(dev(more), 2, slots, insert=False)
    s2 = slots.download(np.uint32, 2)
    assert s2[1] == 0xFFFFFFFF and s2[0] != 0xFFFFFFFF


def test_sorted_sparse_requests_use_global_search():
    """A request far sparser than the store leaves windows wider than the LDS
    window (2 * block * 4 keys: 8192 at the default 1024-thread block): the
    resolve falls back to global searches.  Stride 10007 over 2 M keys spans
    ~40 M key positions per 4096-key tile, past the window at any block size."""
    rng = np.random.default_rng(31)
    univ = np.unique(rng.integers(0, 1 << 63, 2_000_000, dtype=np.uint64))
    st = psg.Store(psg.SORTED, psg.F32, 0, KMAX, 0)
    orc = oracle.Store()
    v = rng.uniform(-1, 1, len(univ)).astype(np.float32)
    st.handle(psg.PUSH, dev(univ), dev(v), None, len(univ))
    orc.handle(oracle.PUSH, univ, v, len(univ))
    for stride in (997, 10007):
        k = univ[::stride].copy()
        k2 = np.sort(np.concatenate([k, k[:-1] + 1]))  # half of them absent
        k2 = np.unique(k2)
        vv = rng.uniform(-1, 1, len(k2)).astype(np.float32)
        out = psg.DeviceBuffer(len(k2) * 4)
        st.handle(psg.PUSH | psg.PULL, dev(k2), dev(vv), out, len(k2))
        exp = orc.handle(oracle.PUSH | oracle.PULL, k2, vv, len(k2))
        np.testing.assert_array_equal(out.download(np.float32, len(k2)), exp)
    gk, gv = st.dump()
    ok, ov = orc.dump()
    np.testing.assert_array_equal(gk, ok)
    np.testing.assert_array_equal(gv, ov)


def test_sorted_extreme_keys_and_empty_request():
    st = psg.Store(psg.SORTED, psg.F32, 0, KMAX, 0)
    keys = np.array([0, 1, KMAX - 2, KMAX - 1], dtype=np.uint64)
    v = np.array([1, 2, 3, 4], np.float32)
    out = psg.DeviceBuffer(16)
    st.handle(psg.PUSH | psg.PULL, dev(keys), dev(v), out, 4)
    np.testing.assert_array_equal(out.download(np.float32, 4), v)
    st.handle(psg.PUSH, None, None, None, 0)  # n = 0: no-op
    assert st.info().size == 4


def test_sorted_duplicate_keys_apply_in_arrival_order():
    """The reference's loop (KVApp.h:446-454) adds each occurrence of a key in
    turn and a PushPull answers each occurrence with the running value."""
    st = psg.Store(psg.SORTED, psg.F32, 0, KMAX, 0)
    orc = oracle.Store()
    k = np.array([5, 7, 7, 9], np.uint64)
    v = np.array([1.0, 2.0, 3.0, 4.0], np.float32)
    out = psg.DeviceBuffer(16)
    for flags in (psg.PUSH, psg.PUSH | psg.PULL, psg.PULL):
        st.handle(flags, dev(k), dev(v), out, 4)
        exp = orc.handle(flags, k, v if flags & psg.PUSH else None, 4)
        if flags & psg.PULL:
            np.testing.assert_array_equal(out.download(np.float32, 4), exp)
    np.testing.assert_array_equal(out.download(np.float32, 4), [2.0, 10.0, 10.0, 8.0])


def _disorder(univ, bad, rng):
    k = univ.copy()
    if bad == "duplicate_last_tile":
        k[-3] = k[-4]
    elif bad == "unsorted_middle":
        k[30000], k[30001] = k[30001], k[30000]
    elif bad == "duplicate_adjacent_lanes":
        k[4100] = k[4099]  # the last key of lane 0 and the first of lane 1, second tile
    elif bad == "duplicate_adjacent_waves":
        k[4096 + 256] = k[4096 + 255]  # the last key of wave 0 and the first of wave 1
    elif bad == "shuffled":
        rng.shuffle(k)
    elif bad == "hot_keys":  # a few keys repeated many times, the rest once
        k[rng.integers(0, len(k), len(k) // 4)] = k[rng.integers(0, 16, len(k) // 4)]
    elif bad == "reversed":
        k = k[::-1].copy()
    return k


@pytest.mark.parametrize("flags", [psg.PUSH, psg.PUSH | psg.PULL, psg.PULL])
@pytest.mark.parametrize("bad", ["duplicate_last_tile", "unsorted_middle", "duplicate_adjacent_lanes",
                                 "duplicate_adjacent_waves", "shuffled", "hot_keys", "reversed"])
def test_sorted_out_of_order_request_on_a_populated_store(bad, flags):
    """Keys out of order or repeated — wherever the break sits: the last of many
    tiles, between lanes, between waves — are detected by the fast path's
    checks (k_validate_windows; a Pull inside k_resolve_apply), which then
    write nothing; the request is served by the order-preserving path (stable
    device sort by slot + one lane per key) bit-exactly like the reference's
    sequential loop, and absent keys among them are inserted once."""
    rng = np.random.default_rng(41)
    kb, ke = 1000, 1 << 62
    univ = np.unique(rng.integers(kb, ke, 60000, dtype=np.uint64))
    st = psg.Store(psg.SORTED, psg.F32, kb, ke, 0)
    orc = oracle.Store()
    v0 = rng.uniform(-1, 1, len(univ)).astype(np.float32)
    st.handle(psg.PUSH, dev(univ[::2]), dev(v0[::2]), None, len(univ[::2]))  # half present
    orc.handle(oracle.PUSH, univ[::2], v0[::2], len(univ[::2]))
    k = _disorder(univ, bad, rng)
    n = len(k)
    v = rng.uniform(-1, 1, n).astype(np.float32)
    out = psg.DeviceBuffer(n * 4) if flags & psg.PULL else None
    for _ in range(2):
        st.handle(flags, dev(k), dev(v) if flags & psg.PUSH else None, out, n)
        exp = orc.handle(flags, k, v if flags & psg.PUSH else None, n)
        if out is not None:
            np.testing.assert_array_equal(out.download(np.float32, n), exp)
    gk, gv = st.dump()
    ok, ov = orc.dump()
    np.testing.assert_array_equal(gk, ok)
    np.testing.assert_array_equal(gv, ov)
    # and the fast path still serves sorted requests afterwards
    st.handle(psg.PUSH, dev(univ), dev(np.ones(len(univ), np.float32)), None, len(univ))
    orc.handle(oracle.PUSH, univ, np.ones(len(univ), np.float32), len(univ))
    np.testing.assert_array_equal(st.dump()[1], orc.dump()[1])


@pytest.mark.parametrize("where", ["none", "tile_0", "tile_500", "last_tile"])
def test_out_of_order_pushpull_at_scale(where):
    """A 4 M-key PushPull (about a thousand 4096-key tiles) on a store holding
    half the keys, with a pair out of order and a repeat in tile `where`: the
    fast path's checks catch it wherever it sits and write nothing, and the
    order-preserving path serves the whole request (inserting the absent keys)
    — bit-exact against the oracle, replies and store, twice in a row."""
    rng = np.random.default_rng(5)
    univ = np.unique(rng.integers(0, KMAX, 4_200_000, dtype=np.uint64))[:4_000_000]
    st = psg.Store(psg.SORTED, psg.F32, 0, KMAX, 0)
    orc = oracle.Store()
    half = univ[::2].copy()
    w = rng.uniform(-1, 1, len(half)).astype(np.float32)
    st.handle(psg.PUSH, dev(half), dev(w), None, len(half))
    orc.handle(oracle.PUSH, half, w, len(half))
    k = univ.copy()
    pos = {"none": None, "tile_0": 100, "tile_500": 500 * 4096 + 7, "last_tile": len(k) - 3}[where]
    if pos is not None:
        k[pos], k[pos + 1] = k[pos + 1], k[pos]
        k[pos + 2] = k[pos - 5]  # and a repeat
    n = len(k)
    v = rng.uniform(-1, 1, n).astype(np.float32)
    out = psg.DeviceBuffer(n * 4)
    for _ in range(2):
        st.handle(psg.PUSH | psg.PULL, dev(k), dev(v), out, n)
        exp = orc.handle(oracle.PUSH | oracle.PULL, k, v, n)
        np.testing.assert_array_equal(out.download(np.float32, n), exp)
    gk, gv = st.dump()
    ok, ov = orc.dump()
    o = np.argsort(ok)
    np.testing.assert_array_equal(gk, ok[o])
    np.testing.assert_array_equal(gv, ov[o])


@pytest.mark.parametrize("flags", [psg.PUSH, psg.PUSH | psg.PULL, psg.PULL])
def test_sorted_out_of_range_request_leaves_a_populated_store_unchanged(flags):
    """A key outside the shard's range rejects the request as a whole
    (k_validate_windows reads every key before k_resolve_apply writes): the
    store keeps exactly what it held, even when the bad key is the last of
    many tiles and the request is also out of order."""
    rng = np.random.default_rng(41)
    kb, ke = 1000, 1 << 62
    univ = np.unique(rng.integers(kb, ke, 60000, dtype=np.uint64))
    st = psg.Store(psg.SORTED, psg.F32, kb, ke, 0)
    st.handle(psg.PUSH, dev(univ), dev(rng.uniform(-1, 1, len(univ)).astype(np.float32)), None, len(univ))
    k0, v0 = st.dump()
    for variant in ("last", "last_and_unsorted"):
        k = univ.copy()
        k[-1] = ke + 5
        if variant == "last_and_unsorted":
            k[100], k[101] = k[101], k[100]
        n = len(k)
        out = psg.DeviceBuffer(n * 4) if flags & psg.PULL else None
        with pytest.raises(psg.PsgError) as ei:
            st.handle(flags, dev(k), dev(np.ones(n, np.float32)), out, n)
        assert ei.value.code == 4
        k1, v1 = st.dump()
        np.testing.assert_array_equal(k1, k0)
        np.testing.assert_array_equal(v1, v0)
    st.handle(psg.PUSH, dev(univ), dev(np.ones(len(univ), np.float32)), None, len(univ))
    np.testing.assert_array_equal(st.dump()[1], (v0 + np.float32(1)).astype(np.float32))


@pytest.mark.parametrize("dtype", [psg.F32, psg.F64, psg.F16, psg.BF16])
@pytest.mark.parametrize("kind", ["sorted_empty", "sorted_populated", "dense"])
def test_shuffled_and_repeated_keys_all_dtypes(dtype, kind):
    """Requests with shuffled keys and runs of duplicates, in all four dtypes,
    on an empty SORTED store (the first request inserts), a populated one, and
    a DENSE store addressed by keys: Push, PushPull and Pull bit-exact against
    oracle.Store, the sequential unordered_map loop of KVApp.h:446-454."""
    rng = np.random.default_rng(7 + dtype)
    if kind == "dense":
        kb, cap = 100, 50000
        st = psg.Store(psg.DENSE, dtype, kb, kb + cap, cap)
        univ = np.arange(kb, kb + cap, dtype=np.uint64)
    else:
        st = psg.Store(psg.SORTED, dtype, 0, KMAX, 0)
        univ = np.unique(rng.integers(0, KMAX, 80000, dtype=np.uint64))
    orc = oracle.Store(dtype)
    if kind != "sorted_empty":
        w = synth(len(univ), dtype, 5, 1, -1.0, 1.0)
        st.handle(psg.PUSH, dev(univ), dev(w), None, len(univ))
        orc.handle(oracle.PUSH, univ, w, len(univ))
    for j in range(6):
        n = int(rng.integers(1, 120000))
        k = rng.choice(univ, n, replace=True)  # repeats, any order
        if j % 2:
            k[: n // 3] = k[0]  # a long run of one key
            rng.shuffle(k)
        flags = [psg.PUSH, psg.PUSH | psg.PULL, psg.PULL][j % 3]
        v = synth(n, dtype, 100 + j, 1, -1.0, 1.0)
        out = psg.DeviceBuffer(n * ES[dtype]) if flags & psg.PULL else None
        st.handle(flags, dev(k), dev(v) if flags & psg.PUSH else None, out, n)
        exp = orc.handle(flags, k, v if flags & psg.PUSH else None, n)
        if out is not None:
            np.testing.assert_array_equal(out.download(NPT[dtype], n), exp, err_msg=f"request {j}")
    gk, gv = st.dump()
    ok, ov = orc.dump()
    if kind == "dense":  # every slot of a DENSE store exists; the untouched ones stay 0
        g = gv.view(NPT[dtype])
        idx = (ok - np.uint64(kb)).astype(np.int64)
        np.testing.assert_array_equal(g[idx], ov.view(NPT[dtype]))
        rest = np.ones(len(g), bool)
        rest[idx] = False
        assert not np.any(g[rest].view(np.uint8))
    else:
        np.testing.assert_array_equal(gk, ok)
        np.testing.assert_array_equal(gv.view(NPT[dtype]), ov)


@pytest.mark.parametrize("n", [1, 17, 4096, 4097, 100003, 3_000_000])
@pytest.mark.parametrize("bits", [8, 20, 64])
def test_device_radix_sort_is_stable(n, bits):
    """psg_sort.hip against numpy's stable argsort on the low `bits` of the key."""
    rng = np.random.default_rng(n + bits)
    k = rng.integers(0, 1 << 63, n, dtype=np.uint64) | (rng.integers(0, 2, n, dtype=np.uint64) << np.uint64(63))
    if n > 100:
        k[: n // 5] = k[0]  # many equal keys: stability matters
    v = np.arange(n, dtype=np.uint32)
    dk, dv = dev(k), dev(v)
    psg.sort_pairs_u64(dk, dv, n, bits)
    psg.device_sync()
    key = k & np.uint64((1 << bits) - 1) if bits < 64 else k
    order = np.argsort(key, kind="stable")
    np.testing.assert_array_equal(dv.download(np.uint32, n), v[order])
    np.testing.assert_array_equal(dk.download(np.uint64, n), k[order])


@pytest.mark.parametrize("depth", [1, 4, 40])
def test_async_requests_with_absent_keys_replay_in_order(depth):
    """psg_store_handle_async: a stream of requests in flight on a populated
    store, many of which carry a few absent keys (or keys out of order).  Each
    such request raises the store's pending word; every request launched
    behind it writes nothing and reports itself gated; the wait inserts the
    keys and replays them in order.  The whole sequence — Push, PushPull and
    Pull mixed — is bit-exact against the oracle, with at most `depth`
    requests in flight."""
    rng = np.random.default_rng(99 + depth)
    univ = np.unique(rng.integers(0, KMAX, 200000, dtype=np.uint64))
    st = psg.Store(psg.SORTED, psg.F32, 0, KMAX, 0)
    orc = oracle.Store()
    base = univ[: len(univ) // 2]
    w = rng.uniform(-1, 1, len(base)).astype(np.float32)
    st.handle(psg.PUSH, dev(base), dev(w), None, len(base))
    orc.handle(oracle.PUSH, base, w, len(base))
    reqs, pending = [], []
    for j in range(60):
        if j % 5 == 0:  # a few keys the store has not seen yet
            extra = rng.choice(univ[len(univ) // 2:], 7, replace=False)
            k = np.unique(np.concatenate([base[j * 100:(j + 1) * 100 + 5000], extra]))
        elif j % 11 == 3:  # out of order
            k = base[j * 50:j * 50 + 3000].copy()
            rng.shuffle(k)
        else:
            k = base[(j * 997) % 50000:(j * 997) % 50000 + 20000]
        flags = [psg.PUSH, psg.PUSH | psg.PULL, psg.PULL][j % 3]
        v = rng.uniform(-1, 1, len(k)).astype(np.float32)
        dk, dv = dev(k), dev(v)
        out = psg.DeviceBuffer(len(k) * 4) if flags & psg.PULL else None
        t = st.handle_async(flags, dk, dv if flags & psg.PUSH else None, out, len(k))
        exp = orc.handle(flags, k, v if flags & psg.PUSH else None, len(k))
        reqs.append((dk, dv, out, exp, len(k)))
        pending.append(t)
        if len(pending) >= depth:
            st.wait(pending.pop(0))
    st.wait()
    psg.device_sync()
    for j, (_, _, out, exp, n) in enumerate(reqs):
        if out is not None:
            np.testing.assert_array_equal(out.download(np.float32, n), exp, err_msg=f"request {j}")
    gk, gv = st.dump()
    ok, ov = orc.dump()
    np.testing.assert_array_equal(gk, ok)
    np.testing.assert_array_equal(gv, ov)


def test_async_pull_replies_on_two_streams_are_in_memory_after_wait():
    """psg_store_wait promises every reaped Pull's reply is in memory.  Pulls
    in flight on stream A, then on stream B (the switch reaps A's requests),
    then wait(): each reply is read by a copy on a THIRD stream, ordered with
    neither, with no device synchronisation in between."""
    rng = np.random.default_rng(5)
    k = np.unique(rng.integers(0, KMAX, 300000, dtype=np.uint64))
    n = len(k)
    st = psg.Store(psg.SORTED, psg.F32, 0, KMAX, 0)
    orc = oracle.Store()
    dk = dev(k)
    sa, sb, sc = psg.Stream(), psg.Stream(), psg.Stream()
    outs, exps = [], []
    for rep in range(8):
        v = rng.uniform(-1, 1, n).astype(np.float32)
        st.handle(psg.PUSH, dk, dev(v), None, n, stream=sa)
        orc.handle(oracle.PUSH, k, v, n)
        for s in (sa, sa, sb, sb):
            out = psg.DeviceBuffer(n * 4)
            st.handle_async(psg.PULL, dk, None, out, n, stream=s)
            outs.append(out)
            exps.append(orc.handle(oracle.PULL, k, None, n))
        st.wait()
        for out, exp in zip(outs, exps):
            np.testing.assert_array_equal(out.download(np.float32, n, stream=sc), exp)
        outs.clear()
        exps.clear()


def test_async_request_failure_is_reported_by_wait():
    st = psg.Store(psg.SORTED, psg.F32, 0, 1 << 40, 0)
    k = np.arange(1000, dtype=np.uint64) * 7
    st.handle(psg.PUSH, dev(k), dev(np.ones(1000, np.float32)), None, 1000)
    bad = k.copy()
    bad[-1] = 1 << 41  # outside [0, 2^40)
    dk, db = dev(k), dev(bad)
    ones = dev(np.ones(1000, np.float32))
    t1 = st.handle_async(psg.PUSH, db, ones, None, 1000)
    t2 = st.handle_async(psg.PUSH, dk, ones, None, 1000)
    assert t1 and t2 > t1
    with pytest.raises(psg.PsgError) as ei:
        st.wait(t2)
    assert ei.value.code == 4
    st.wait()  # reported once
    np.testing.assert_array_equal(st.dump()[1], np.full(1000, 2.0, np.float32))


@pytest.mark.parametrize("dtype", [psg.F32, psg.F64])
def test_sorted_window_cache_transitions(dtype):
    """The store-key windows are cached per request key array and trusted once
    a request confirmed them; k_resolve_apply re-checks every cached window
    against its tile's first and last key and searches a stale one inline.
    One key buffer is reused with changing contents through every transition
    — repeats (trusted, no pre-pass), new keys under the same pointer (stale
    windows), inner keys changed with the ends kept, absent keys (an insert
    changes K's generation), keys alternating under one pointer, a rejected
    Pull on trusted windows — each request checked against the oracle."""
    rng = np.random.default_rng(123)
    univ = np.unique(rng.integers(1 << 20, 1 << 62, 400000, dtype=np.uint64))
    st = psg.Store(psg.SORTED, dtype, 0, KMAX, 0)
    orc = oracle.Store(dtype)
    v0 = synth(len(univ), dtype, 5, 1, -1.0, 1.0)
    st.handle(psg.PUSH, dev(univ), dev(v0), None, len(univ))
    orc.handle(oracle.PUSH, univ, v0, len(univ))
    n = 150000
    a = np.sort(rng.choice(univ, n, replace=False))
    b = np.sort(rng.choice(univ, n, replace=False))
    inner = a.copy()
    inner[1:-1] = np.sort(rng.choice(univ[(univ > a[0]) & (univ < a[-1])], n - 2, replace=False))
    fresh = np.unique(np.concatenate([a[: n // 2], rng.integers(1 << 20, 1 << 62, n, dtype=np.uint64)]))[:n]
    dk = psg.DeviceBuffer(n * 8)
    dv = psg.DeviceBuffer(n * ES[dtype])
    out = psg.DeviceBuffer(n * ES[dtype])
    seq = [a, a, a, b, b, b, inner, inner, a, fresh, fresh, a, b, a, b, a, a]
    for j, k in enumerate(seq):
        flags = [psg.PUSH | psg.PULL, psg.PULL, psg.PUSH][j % 3]
        v = synth(n, dtype, 900 + j, 1, -1.0, 1.0)
        dk.upload(k)
        dv.upload(v)
        st.handle(flags, dk, dv if flags & psg.PUSH else None, out if flags & psg.PULL else None, n)
        exp = orc.handle(flags, k, v if flags & psg.PUSH else None, n)
        if flags & psg.PULL:
            np.testing.assert_array_equal(out.download(NPT[dtype], n), exp, err_msg=f"request {j}")
    # a Pull with one unsorted pair on trusted windows: k_resolve_apply's own
    # check catches it and the order-preserving path answers it; the store is
    # unchanged, and the trusted windows still serve the sorted list after
    dk.upload(a)
    st.handle(psg.PULL, dk, None, out, n)
    st.handle(psg.PULL, dk, None, out, n)
    bad = a.copy()
    bad[n // 2], bad[n // 2 + 1] = bad[n // 2 + 1], bad[n // 2]
    dk.upload(bad)
    k0, s0 = st.dump()
    st.handle(psg.PULL, dk, None, out, n)
    np.testing.assert_array_equal(out.download(NPT[dtype], n), orc.handle(oracle.PULL, bad, None, n))
    k1, s1 = st.dump()
    np.testing.assert_array_equal(k1, k0)
    np.testing.assert_array_equal(s1, s0)
    dk.upload(a)
    st.handle(psg.PULL, dk, None, out, n)
    np.testing.assert_array_equal(out.download(NPT[dtype], n), orc.handle(oracle.PULL, a, None, n))
    gk, gv = st.dump()
    ok, ov = orc.dump()
    np.testing.assert_array_equal(gk, ok)
    np.testing.assert_array_equal(gv.view(NPT[dtype]), ov)


@pytest.mark.parametrize("flags", [psg.PUSH, psg.PUSH | psg.PULL])
@pytest.mark.parametrize("dtype", [psg.F32, psg.F64])
def test_push_out_of_order_after_an_ascending_prefix(flags, dtype):
    """A keyed Push / PushPull that ascends for a while and then goes out of
    order (the validation pass rejects it before any write and the
    order-preserving path serves it whole, in arrival order).  Bit-exact
    against the sequential oracle (KVApp.h:446-454) with the disorder at many
    positions — inside the first 4096-key tile, at tile edges, near the end —
    the rest repeating keys of the ascending part, absent keys on both sides
    (a half-populated store), and some requests in flight; the whole store
    compared after."""
    rng = np.random.default_rng(4242 + dtype + flags)
    univ = np.unique(rng.integers(1 << 20, 1 << 62, 300000, dtype=np.uint64))
    st = psg.Store(psg.SORTED, dtype, 0, KMAX, 0)
    orc = oracle.Store(dtype)
    half = univ[::2].copy()
    w = synth(len(half), dtype, 3, 1, -1.0, 1.0)
    st.handle(psg.PUSH, dev(half), dev(w), None, len(half))
    orc.handle(oracle.PUSH, half, w, len(half))
    outs, keep = [], []
    cuts = [10, 4095, 4096, 4097, 12288, 50000, 99990]
    for j, cut in enumerate(cuts):
        n = 100000
        k = np.sort(rng.choice(univ, n, replace=False))
        tail = k[cut:].copy()
        rng.shuffle(tail)
        k[cut:] = tail
        k[-3:] = k[:3]  # the rest repeats keys of the prefix
        v = synth(n, dtype, 50 + j, 1, -1.0, 1.0)
        out = psg.DeviceBuffer(n * ES[dtype]) if flags & psg.PULL else None
        dk, dv = dev(k), dev(v)
        keep.append((dk, dv))  # a request in flight reads them until it is reaped
        if j % 2:
            st.handle_async(flags, dk, dv, out, n)
        else:
            st.handle(flags, dk, dv, out, n)
        exp = orc.handle(flags, k, v, n)
        if out is not None:
            outs.append((out, exp, j))
    st.wait()
    psg.device_sync()
    for out, exp, j in outs:
        np.testing.assert_array_equal(out.download(NPT[dtype], len(exp)), exp, err_msg=f"request {j}")
    gk, gv = st.dump()
    ok, ov = orc.dump()
    np.testing.assert_array_equal(gk, ok)
    np.testing.assert_array_equal(gv.view(NPT[dtype]), ov)
    assert st.counters()["ordered"] >= len(cuts), st.counters()


def test_unsorted_push_with_a_key_outside_between_in_range_ends_leaves_the_store_unchanged():
    """A key outside the shard between two in-range ends (so the request is
    also out of order) rejects the whole request: PSG_ERR_RANGE, nothing
    applied."""
    rng = np.random.default_rng(77)
    kb, ke = 1000, 1 << 62
    univ = np.unique(rng.integers(kb, ke, 50000, dtype=np.uint64))
    st = psg.Store(psg.SORTED, psg.F32, kb, ke, 0)
    st.handle(psg.PUSH, dev(univ), dev(rng.uniform(-1, 1, len(univ)).astype(np.float32)), None, len(univ))
    k0, v0 = st.dump()
    k = univ.copy()
    k[10] = ke + 7
    with pytest.raises(psg.PsgError) as ei:
        st.handle(psg.PUSH, dev(k), dev(np.ones(len(k), np.float32)), None, len(k))
    assert ei.value.code == 4
    k1, v1 = st.dump()
    np.testing.assert_array_equal(k1, k0)
    np.testing.assert_array_equal(v1, v0)


def test_sorted_list_across_the_sparse_threshold():
    """One key list served while its store grows from exactly its keys to 3x
    as many: the resolve-and-apply launch switches from 1024- to 256-thread
    tiles (ra_block: a request sparse in the store), its window-cache entry is
    searched again for the new tiles, and every request — synchronous and in
    flight, on both sides of the switch — matches the oracle, as does the whole
    store after."""
    rng = np.random.default_rng(2024)
    univ = np.unique(rng.integers(1 << 20, 1 << 62, 330000, dtype=np.uint64))
    a = np.sort(rng.choice(univ, 100000, replace=False))
    rest = np.setdiff1d(univ, a)
    st = psg.Store(psg.SORTED, psg.F32, 0, KMAX, 0)
    orc = oracle.Store()
    dk = dev(a)
    n = len(a)
    keep = []
    for phase in range(2):
        if phase == 1:  # the store grows past 1.5x the list: the sparse tiles
            v = rng.uniform(-1, 1, len(rest)).astype(np.float32)
            st.handle(psg.PUSH, dev(rest), dev(v), None, len(rest))
            orc.handle(oracle.PUSH, rest, v, len(rest))
        for j in range(6):
            flags = [psg.PUSH, psg.PUSH | psg.PULL, psg.PULL][j % 3]
            v = rng.uniform(-1, 1, n).astype(np.float32)
            dv = dev(v)
            out = psg.DeviceBuffer(n * 4) if flags & psg.PULL else None
            keep.append((dv, out))
            if j >= 3:
                st.handle_async(flags, dk, dv if flags & psg.PUSH else None, out, n)
            else:
                st.handle(flags, dk, dv if flags & psg.PUSH else None, out, n)
            exp = orc.handle(flags, a, v if flags & psg.PUSH else None, n)
            if out is not None:
                keep.append((out, exp, f"phase {phase} request {j}"))
        st.wait()
    psg.device_sync()
    for item in keep:
        if len(item) == 3:
            out, exp, what = item
            np.testing.assert_array_equal(out.download(np.float32, n), exp, err_msg=what)
    gk, gv = st.dump()
    ok, ov = orc.dump()
    np.testing.assert_array_equal(gk, ok)
    np.testing.assert_array_equal(gv, ov)


@pytest.mark.parametrize("every", [2, 3, 5, 40])
def test_sorted_requests_sparse_in_the_store(every):
    """A request that asks for every `every`-th key of a larger store: its
    tiles' windows of store keys exceed the LDS window (k_resolve_apply then
    streams each window through LDS in chunks; past 16 chunks, every 40th key,
    it searches each key in HBM).  Push, PushPull and Pull in flight and
    synchronous, against the oracle, then the whole store."""
    rng = np.random.default_rng(1000 + every)
    univ = np.unique(rng.integers(1 << 20, 1 << 62, 600000, dtype=np.uint64))
    st = psg.Store(psg.SORTED, psg.F32, 0, KMAX, 0)
    orc = oracle.Store()
    v0 = rng.uniform(-1, 1, len(univ)).astype(np.float32)
    st.handle(psg.PUSH, dev(univ), dev(v0), None, len(univ))
    orc.handle(oracle.PUSH, univ, v0, len(univ))
    k = univ[1::every].copy()
    n = len(k)
    dk = dev(k)
    outs = []
    for j in range(12):
        flags = [psg.PUSH, psg.PUSH | psg.PULL, psg.PULL][j % 3]
        v = rng.uniform(-1, 1, n).astype(np.float32)
        out = psg.DeviceBuffer(n * 4) if flags & psg.PULL else None
        if j < 6:
            st.handle(flags, dk, dev(v) if flags & psg.PUSH else None, out, n)
        else:
            st.handle_async(flags, dk, dev(v) if flags & psg.PUSH else None, out, n)
        exp = orc.handle(flags, k, v if flags & psg.PUSH else None, n)
        if out is not None:
            outs.append((out, exp, j))
    st.wait()
    psg.device_sync()
    for out, exp, j in outs:
        np.testing.assert_array_equal(out.download(np.float32, n), exp, err_msg=f"request {j}")
    gk, gv = st.dump()
    ok, ov = orc.dump()
    np.testing.assert_array_equal(gk, ok)
    np.testing.assert_array_equal(gv, ov)
    # the list is not a stretch of the store: at most one identity attempt
    # (rejected), never one per request in flight
    c = st.counters()
    assert c["ident"] <= 1 and c["notident"] <= 1, c


def test_dense_keyed_out_of_range_rejected_out_of_order_applied():
    st = psg.Store(psg.DENSE, psg.F32, 100, 100000, 5000)
    base = np.arange(5000, dtype=np.float32)
    st.handle(psg.PUSH, None, dev(base), None, 5000, first_key=100)
    keys = np.arange(100, 5100, dtype=np.uint64)
    keys[-1] = 5100  # one slot past the store
    with pytest.raises(psg.PsgError) as ei:
        st.handle(psg.PUSH, dev(keys), dev(np.ones(5000, np.float32)), None, 5000)
    assert ei.value.code == 4
    np.testing.assert_array_equal(st.dump()[1], base)
    # out of order and repeated keys are applied in arrival order, like the
    # reference's loop, on the DENSE store too
    keys = np.arange(100, 5100, dtype=np.uint64)
    keys[10], keys[11] = keys[11], keys[10]
    keys[20] = keys[21]
    ones = np.ones(5000, np.float32)
    out = psg.DeviceBuffer(5000 * 4)
    st.handle(psg.PUSH | psg.PULL, dev(keys), dev(ones), out, 5000)
    orc = oracle.Store()
    orc.handle(oracle.PUSH, np.arange(100, 5100, dtype=np.uint64), base, 5000)
    np.testing.assert_array_equal(out.download(np.float32, 5000), orc.handle(oracle.PUSH | oracle.PULL, keys, ones, 5000))
    np.testing.assert_array_equal(st.dump()[1], orc.dump()[1][np.argsort(orc.dump()[0])])


_RA_BLOCK_CHILD = """
import sys, numpy as np
sys.path[:0] = {paths!r}
import oracle, psg
psg.set_device(0)
rng = np.random.default_rng(77)
univ = np.unique(rng.integers(0, 1 << 63, 200000, dtype=np.uint64))
for dt in (psg.F32, psg.F64, psg.F16, psg.BF16):
    st, orc = psg.Store(psg.SORTED, dt, 0, (1 << 64) - 1, 0), oracle.Store(dt)
    for j in range(6):
        k = np.sort(rng.choice(univ, int(rng.integers(1, len(univ))), replace=False)) if j % 2 else univ
        v = oracle.synth(len(k), dt, 500 + j, 1, -1.0, 1.0)
        n = len(k)
        out = psg.DeviceBuffer(n * 8)
        st.handle(psg.PUSH | psg.PULL, psg.DeviceBuffer.from_numpy(k), psg.DeviceBuffer.from_numpy(v), out, n)
        exp = orc.handle(oracle.PUSH | oracle.PULL, k, v, n)
        got = out.download({{psg.F32: np.float32, psg.F64: np.float64}}.get(dt, np.uint16), n)
        assert np.array_equal(got, exp), (dt, j)
print("ok")
"""


@pytest.mark.parametrize("block,knobs", [(256, {}), (512, {}), (1024, {}),
                                         (1024, {"PSG_WIN_CACHE": "0"}), (1024, {"PSG_SYNC_POLL": "0"})])
def test_sorted_store_every_block_size(block, knobs):
    """PSG_RA_BLOCK is read once per process: each block size of the fused
    validate / resolve / apply kernels gets a fresh process, every dtype.  So
    do the A/B switches: windows searched on every request (no window cache)
    and the stream synchronised instead of the kernel's completion word."""
    import subprocess
    import sys
    paths = [os.path.join(os.path.dirname(HERE), "parameter-server_amd", "python"),
             os.path.join(os.path.dirname(HERE), "oracle")]
    env = dict(os.environ, PSG_RA_BLOCK=str(block), **knobs)
    r = subprocess.run([sys.executable, "-c", _RA_BLOCK_CHILD.format(paths=paths)], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip().endswith("ok"), r.stderr[-2000:]


def test_dense_store_resolve_slots():
    st = psg.Store(psg.DENSE, psg.F32, 100, 1000, 500)
    keys = np.array([100, 150, 599], np.uint64)
    slots = psg.DeviceBuffer(12)
    st.resolve(dev(keys), 3, slots)
    assert slots.download(np.uint32, 3).tolist() == [0, 50, 499]
    with pytest.raises(psg.PsgError):
        st.resolve(dev(np.array([100, 600], np.uint64)), 2, slots)


def test_sorted_small_out_of_order_and_out_of_range():
    st = psg.Store(psg.SORTED, psg.F32, 100, 200, 0)
    v = dev(np.ones(3, np.float32))
    st.handle(psg.PUSH, dev(np.array([150, 120, 160], np.uint64)), v, None, 3)  # the first request: two-pass form
    st.handle(psg.PUSH, dev(np.array([160, 150, 150], np.uint64)), v, None, 3)  # fused form
    k, vals = st.dump()
    assert k.tolist() == [120, 150, 160] and vals.tolist() == [1.0, 3.0, 2.0]
    with pytest.raises(psg.PsgError) as ei:
        st.handle(psg.PUSH, dev(np.array([150, 199, 200], np.uint64)), v, None, 3)
    assert ei.value.code == 4


# ---------------------------------------------------------------------------
def test_slice_golden_cases():
    for j in range(int(G["slice_ncases"][0])):
        keys = G[f"slice{j}_keys"]
        ns = int(G[f"slice{j}_ns"][0])
        haslens = bool(G[f"slice{j}_haslens"][0])
        b, e = psg.server_ranges(ns)
        lens = dev(G[f"slice{j}_lens"]) if haslens else None
        kp, vp = psg.slice_keys(dev(keys), len(keys), b, e, lens=lens,
                                num_vals=None if haslens else len(keys))
        np.testing.assert_array_equal(kp, G[f"slice{j}_kpos"], err_msg=f"case {j}")
        np.testing.assert_array_equal(vp, G[f"slice{j}_vpos"], err_msg=f"case {j}")


@pytest.mark.parametrize("n,ns", [(1, 1), (1000, 3), (1 << 20, 8), (10_000_000, 4)])
def test_slice_vs_oracle_large(n, ns):
    rng = np.random.default_rng(n + ns)
    keys = np.unique(rng.integers(0, KMAX, n, dtype=np.uint64))
    lens = rng.integers(0, 4, len(keys)).astype(np.int32)
    b, e = psg.server_ranges(ns)
    dk = dev(keys)
    kp, vp = psg.slice_keys(dk, len(keys), b, e, lens=dev(lens))
    okp, ovp = oracle.slice_keys(keys, b, e, lens)
    np.testing.assert_array_equal(kp, okp)
    np.testing.assert_array_equal(vp, ovp)
    kp2, vp2 = psg.slice_keys(dk, len(keys), b, e, num_vals=2 * len(keys))
    okp2, ovp2 = oracle.slice_keys(keys, b, e, num_vals=2 * len(keys))
    np.testing.assert_array_equal(kp2, okp2)
    np.testing.assert_array_equal(vp2, ovp2)


@pytest.mark.parametrize("ns", [2, 4, 8])
def test_slice_of_a_rewritten_array_is_searched_again(ns):
    """The slicer confirms the bounds an array had at its last slice in one
    round (psg_slice's hints); an array rewritten in place — bounds moved by
    a few keys, by many, or not at all — still slices as the oracle does."""
    rng = np.random.default_rng(ns)
    n = 200_000
    b, e = psg.server_ranges(ns)
    dk = psg.DeviceBuffer(n * 8)
    for trial in range(6):
        if trial % 3 == 2:
            keys = np.sort(rng.integers(0, KMAX, n, dtype=np.uint64))  # everything moves
        elif trial % 3 == 1:
            keys = keys.copy()
            keys[:7] = np.sort(rng.integers(0, int(b[1]) if ns > 1 else 1 << 60, 7, dtype=np.uint64))
            keys = np.sort(keys)  # a few keys move across the first bound
        else:
            keys = np.sort(rng.integers(0, KMAX, n, dtype=np.uint64)) if trial == 0 else keys
        dk.upload(keys)
        psg.device_sync()
        for _ in range(2):  # the second slice of the same contents takes the hints
            kp, _ = psg.slice_keys(dk, n, b, e)
            okp, _ = oracle.slice_keys(keys, b, e)
            np.testing.assert_array_equal(kp, okp, err_msg=f"trial {trial}")


def test_slice_rejects_key_past_last_range():
    b, e = psg.server_ranges(4)
    with pytest.raises(psg.PsgError):
        psg.slice_keys(dev(np.array([3, KMAX], np.uint64)), 2, b, e)


@pytest.mark.parametrize("esize,dtype", [(4, np.float32), (2, np.uint16), (8, np.float64)])
def test_merge_vs_oracle(esize, dtype):
    rng = np.random.default_rng(esize)
    counts = [0, 1, 7, 1000, 4096, 33, 100003]
    segs_host = [(rng.integers(0, 1 << 15, c).astype(dtype), int(rng.integers(0, KMAX, dtype=np.uint64)))
                 for c in counts]
    total = sum(counts)
    segs_dev = [(dev(a) if len(a) else psg.DeviceBuffer(0), len(a), fk) for a, fk in segs_host]
    dst = psg.DeviceBuffer(total * esize + 16)
    psg.merge(segs_dev, esize, dst, total)
    exp = oracle.merge(segs_host, total, dtype=dtype)
    np.testing.assert_array_equal(dst.download(dtype, total), exp)
    # misaligned destination (byte offset not a multiple of 16)
    psg.merge(segs_dev, esize, dst.ptr + esize, total)
    np.testing.assert_array_equal(dst.download(dtype, total, offset=esize), exp)


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("ns", [1, 2, 4])
def test_kat_test_kv_app_on_gpu(ns):
    """tests/test_kv_app.cpp:20-61 through GPU slice + SORTED stores + GPU merge."""
    rets, outs = run_kv_app(GpuKV(ns), G["kv_app_keys"], G["kv_app_vals"])
    np.testing.assert_array_equal(rets, G["kv_app_rets"])
    np.testing.assert_array_equal(outs, G["kv_app_outs"])


def test_kat_test_my_on_gpu():
    rets, final = run_my(GpuKV(3), G["my_keys"], [G[f"my{c}_vals"] for c in range(3)])
    np.testing.assert_array_equal(rets, G["my_rets"])
    np.testing.assert_array_equal(final, G["my_final"])


def test_kat_multi_workers_on_gpu():
    kv = GpuKV(2)
    for c in (0, 1):
        rets, outs = run_kv_app(kv, G[f"mw{c}_keys"], G[f"mw{c}_vals"])
        np.testing.assert_array_equal(rets, G[f"mw{c}_rets"])
        np.testing.assert_array_equal(outs, G[f"mw{c}_outs"])


# ---------------------------------------------------------------------------
@pytest.mark.parametrize("adam", [False, True])
def test_lr_apply_bitexact(adam):
    n = 100003
    rng = np.random.default_rng(8)
    w0 = rng.uniform(-0.5, 0.5, n).astype(np.float32)
    st = psg.Store(psg.DENSE, psg.F32, 0, n, n)
    st.handle(psg.PUSH, None, dev(w0), None, n)
    # LRServer constructs Adam from its float learning_rate_ (LRServer.h:83-84), so the
    # Adam learning rate is the f32 0.01 widened to double, as the oracle gets it.
    a = psg.Adam(n, float(np.float32(0.01))) if adam else None
    w = w0.copy()
    m = np.zeros(n) if adam else None
    v = np.zeros(n) if adam else None
    for it in range(4):
        merged = rng.uniform(-1, 1, n).astype(np.float32)
        psg.lr_apply(st, dev(merged), n, 0.01, a, it)
        oracle.lr_apply(w, merged, 0.01, m, v, float(np.float32(0.01)), 0.9, 0.999, 1e-8, it)
    _, got = st.dump()
    np.testing.assert_array_equal(got, w)


@pytest.mark.parametrize("force", [False, True])
def test_comm_keyed_single_rank(force, monkeypatch):
    """Keyed BSP Push/Pull (grouped RCCL reduce / broadcast) into a SORTED shard."""
    if force:
        monkeypatch.setenv("PSG_COMM_FORCE_COLLECTIVE", "1")
    c = psg.Comm(psg.comm_id(), 1, 0)
    rng = np.random.default_rng(21)
    keys = np.unique(rng.integers(0, KMAX, 200000, dtype=np.uint64))
    n = len(keys)
    v = rng.uniform(-1, 1, n).astype(np.float32)
    st = psg.Store(psg.SORTED, psg.F32, 0, KMAX, 0)
    dk, dv = dev(keys), dev(v)
    b, e = psg.server_ranges(1)
    kp, _ = psg.slice_keys(dk, n, b, e)
    orc = oracle.Store()
    out = psg.DeviceBuffer(n * 4)
    for _ in range(3):
        c.push_keyed(st, dk, dv, n, kp)
        orc.handle(oracle.PUSH, keys, v, n)
    c.pull_keyed(st, dk, out, n, kp)
    np.testing.assert_array_equal(out.download(np.float32, n), orc.handle(oracle.PULL, keys, None, n))
    c.close()


@pytest.mark.parametrize("force", [False, True])
@pytest.mark.parametrize("dtype,n", [(psg.F32, 1 << 20), (psg.F32, 1000003), (psg.F16, 65600)])
def test_comm_single_rank_push_pull(force, dtype, n, monkeypatch):
    """force=True runs the RCCL reduce-scatter / all-gather and the pipelined
    grouped reduce / broadcast even with one rank (they degenerate to copies),
    so the collective calls themselves execute on the MI355X."""
    if force:
        monkeypatch.setenv("PSG_COMM_FORCE_COLLECTIVE", "1")
    c = psg.Comm(psg.comm_id(), 1, 0)
    st = psg.Store(psg.DENSE, dtype, 0, n, n)
    v = psg.DeviceBuffer(n * ES[dtype])
    v.fill_synth(n, dtype, 3, 0, 0.0, 100.0)
    out = psg.DeviceBuffer(n * ES[dtype])
    orc = oracle.Store(dtype)
    hv = oracle.synth(n, dtype, 3, 0, 0.0, 100.0)
    c.push(st, v, n)
    c.push(st, v, n)
    c.pull(st, out, n)
    orc.handle(oracle.PUSH, None, hv, n)
    orc.handle(oracle.PUSH, None, hv, n)
    np.testing.assert_array_equal(out.download(NPT[dtype], n), orc.handle(oracle.PULL, None, None, n))
    for nb in (1, 3, 8):
        c.push_pull(st, v, out, n, nb)
        exp = orc.handle(oracle.PUSH | oracle.PULL, None, hv, n)
        np.testing.assert_array_equal(out.download(NPT[dtype], n), exp, err_msg=f"nbuckets={nb}")
    c.close()


def test_comm_sync_and_abort(monkeypatch):
    """psg_comm_sync waits for the queued collectives against a deadline;
    psg_comm_abort (what every rank calls when one rank's first collective did
    not complete) makes every later collective fail with PSG_ERR_COMM."""
    monkeypatch.setenv("PSG_COMM_FORCE_COLLECTIVE", "1")
    c = psg.Comm(psg.comm_id(), 1, 0)
    n = 1 << 16
    st = psg.Store(psg.DENSE, psg.F32, 0, n, n)
    v = dev(np.ones(n, np.float32))
    s = psg.Stream()
    c.push(st, v, n, stream=s)
    c.sync(s, 30.0)
    np.testing.assert_array_equal(st.dump()[1], np.ones(n, np.float32))
    c.abort()
    with pytest.raises(psg.PsgError) as ei:
        c.push(st, v, n, stream=s)
    assert ei.value.code == 5
    c.close()


_NEVER_JOINS = r"""
import sys, time
sys.path.insert(0, sys.argv[1])
import psg
psg.set_device(0)
uid = psg.comm_id()
t0 = time.monotonic()
try:
    psg.Comm(uid, 2, 0)  # rank 1 of this world-2 communicator never joins
    print("JOINED")
except psg.PsgError as e:
    print("FAILED", e.code, round(time.monotonic() - t0, 2), str(e))
"""


def test_comm_init_with_a_rank_that_never_joins_fails_within_the_deadline():
    """psg_comm_init meets the other ranks on a non-blocking probe communicator
    polled against PSG_COMM_TIMEOUT_S: a world-2 communicator whose rank 1
    never arrives fails with PSG_ERR_COMM after the deadline instead of
    hanging the job (run in a child process, under a hard limit of its own)."""
    import subprocess
    import sys
    env = dict(os.environ, PSG_COMM_TIMEOUT_S="6")
    r = subprocess.run([sys.executable, "-c", _NEVER_JOINS, os.path.dirname(psg.__file__)],
                       env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [x for x in r.stdout.splitlines() if x.startswith(("FAILED", "JOINED"))][-1]
    words = line.split()
    assert words[0] == "FAILED" and int(words[1]) == 5, line
    assert 5.0 <= float(words[2]) <= 40.0, line  # the deadline, not a hang
    assert "did not join" in line


@pytest.mark.parametrize("nbytes", [0, 8, 4096, 8 * 1000003])
def test_checksum_matches_host(nbytes):
    """psg_checksum (the exchange self-check bench.py runs after choosing the
    xGMI path) equals its numpy restatement, and moves with one changed word."""
    a = np.random.default_rng(5).integers(0, 1 << 63, nbytes // 8, dtype=np.uint64)
    b = psg.DeviceBuffer(max(nbytes, 8))
    b.upload(a)
    assert psg.checksum(b, nbytes) == psg.checksum_host(a)
    if nbytes >= 16:
        a[1] ^= np.uint64(1)
        b.upload(a)
        assert psg.checksum(b, nbytes) == psg.checksum_host(a)
        # swapped words change it (position-keyed)
        a[[0, 1]] = a[[1, 0]]
        b.upload(a)
        assert psg.checksum(b, nbytes) == psg.checksum_host(a)
