"""The CPU oracle pinned against the reference's own known-answer tests.

Golden data: tests/golden/golden.npz (made by tests/golden/make_golden.py from
the reference tests' inputs and CHECK expectations).  No GPU needed.
"""
import ctypes
import os

import numpy as np
import pytest

import oracle
from kv_pipeline import OracleKV, run_kv_app, run_my

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "golden.npz"))
KMAX = (1 << 64) - 1


def test_glibc_rand_matches_golden():
    # the oracle's glibc rand draw == the fixture's (srand(rank + 7); rand() % 1000)
    np.testing.assert_array_equal(oracle.glibc_rand_mod(7, 1000, 10000), G["kv_app_vals"])


@pytest.mark.parametrize("ns", [1, 2, 3, 4, 8])
def test_kat_test_kv_app(ns):
    """tests/test_kv_app.cpp:20-61: 50 Push -> 50*vals; 50 PushPull -> 100*vals."""
    keys, vals = G["kv_app_keys"], G["kv_app_vals"]
    rets, outs = run_kv_app(OracleKV(ns), keys, vals)
    np.testing.assert_array_equal(rets, G["kv_app_rets"])
    np.testing.assert_array_equal(outs, G["kv_app_outs"])
    # the reference's own tolerance check, :54-58
    assert np.abs(rets - vals * 50).sum() / 50 < 1e-5


@pytest.mark.parametrize("ns", [1, 4])
def test_kat_multi_workers(ns):
    """tests/test_kv_app_multi_workers.cpp:27-65: two customers, disjoint keys, one server set."""
    kv = OracleKV(ns)
    for c in (0, 1):
        rets, outs = run_kv_app(kv, G[f"mw{c}_keys"], G[f"mw{c}_vals"])
        np.testing.assert_array_equal(rets, G[f"mw{c}_rets"])
        np.testing.assert_array_equal(outs, G[f"mw{c}_outs"])


@pytest.mark.parametrize("ns", [1, 3])
def test_kat_test_my(ns):
    """tests/test_my.cpp:29-75: 3 customers accumulate into the same keys."""
    rets, final = run_my(OracleKV(ns), G["my_keys"], [G[f"my{c}_vals"] for c in range(3)])
    np.testing.assert_array_equal(rets, G["my_rets"])
    np.testing.assert_array_equal(final, G["my_final"])


def test_slicer_golden():
    for j in range(int(G["slice_ncases"][0])):
        keys = G[f"slice{j}_keys"]
        ns = int(G[f"slice{j}_ns"][0])
        lens = G[f"slice{j}_lens"] if bool(G[f"slice{j}_haslens"][0]) else None
        b, e = oracle.server_ranges(ns)
        r = oracle.slice_keys(keys, b, e, lens)
        assert r is not None
        np.testing.assert_array_equal(r[0], G[f"slice{j}_kpos"], err_msg=f"case {j}")
        np.testing.assert_array_equal(r[1], G[f"slice{j}_vpos"], err_msg=f"case {j}")


def test_server_ranges():
    for ns in (1, 2, 3, 8):
        b, e = oracle.server_ranges(ns)
        assert b[0] == 0 and e[-1] == KMAX
        for i in range(1, ns):
            assert e[i - 1] == b[i] == KMAX // ns * i


def test_slicer_check_failures():
    b, e = oracle.server_ranges(4)
    # key == kMaxKey is past the last range (CHECK_EQ(pos[n], size), KVApp.h:544)
    assert oracle.slice_keys(np.array([1, KMAX], dtype=np.uint64), b, e) is None
    # vals not a multiple of keys (KVApp.h:551)
    assert oracle.slice_keys(np.array([1, 2], dtype=np.uint64), b, e, num_vals=3) is None
    # non-adjacent ranges (KVApp.h:531)
    e2 = e.copy()
    e2[0] -= 1
    assert oracle.slice_keys(np.array([1], dtype=np.uint64), b, e2) is None
    # empty request: all slices empty
    kp, vp = oracle.slice_keys(np.zeros(0, dtype=np.uint64), b, e)
    assert kp.tolist() == [0] * 5


def test_slicer_k_values_per_key():
    b, e = oracle.server_ranges(2)
    keys = np.array([1, 2, KMAX // 2 + 5], dtype=np.uint64)
    kp, vp = oracle.slice_keys(keys, b, e, num_vals=6)
    assert kp.tolist() == [0, 2, 3] and vp.tolist() == [0, 4, 6]


def test_merge_orders_by_first_key():
    segs = [(np.array([5, 6], np.float32), 100), (np.array([1, 2, 3], np.float32), 7),
            (np.array([9], np.float32), 1000)]
    np.testing.assert_array_equal(oracle.merge(segs, 6), [1, 2, 3, 5, 6, 9])
    assert oracle.merge(segs, 7) is None  # "lost some servers?" (KVApp.h:691)


def test_pull_inserts_absent_keys_as_zero():
    s = oracle.Store()
    out = s.handle(oracle.PULL, np.array([3, 9], np.uint64), None, 2)
    assert out.tolist() == [0, 0] and s.size() == 2


def test_pushpull_returns_post_update_value():
    s = oracle.Store()
    k = np.array([1, 2], np.uint64)
    s.handle(oracle.PUSH, k, np.array([1, 2], np.float32), 2)
    out = s.handle(oracle.PUSH | oracle.PULL, k, np.array([10, 20], np.float32), 2)
    assert out.tolist() == [11, 22]


def _splitmix(x):
    m = (1 << 64) - 1
    x = (x + 0x9E3779B97F4A7C15) & m
    x = ((x ^ (x >> 30)) * 0xBF58476D1CE4E5B9) & m
    x = ((x ^ (x >> 27)) * 0x94D049BB133111EB) & m
    return x ^ (x >> 31)


def test_synth_generator_restatement():
    n, seed = 257, 123456789
    ref_int = np.array([np.floor((_splitmix(seed + i) >> 40) * 1000.0 / 16777216.0)
                        for i in range(n)], dtype=np.float32)
    np.testing.assert_array_equal(oracle.synth(n, oracle.F32, seed, 0, 0.0, 1000.0), ref_int)
    ref_real = np.array([-1.0 + ((_splitmix(seed + i) >> 40) / 16777216.0) * 2.0
                         for i in range(n)]).astype(np.float32)
    np.testing.assert_array_equal(oracle.synth(n, oracle.F32, seed, 1, -1.0, 1.0), ref_real)


def test_half_conversions_round_to_nearest_even():
    v = np.array([0.1, 1.0 / 3, 65504.0, 1e-7, -2.5e-5, 70000.0, 3.14159], dtype=np.float32)
    s = oracle.Store(oracle.F16)
    k = np.arange(len(v), dtype=np.uint64)
    h = v.astype(np.float16).view(np.uint16)  # numpy f32 -> f16 is RNE
    s.handle(oracle.PUSH, k, h, len(v))
    _, got = s.dump()
    np.testing.assert_array_equal(got, h)
    # f16 accumulate: f32 add, one RNE rounding
    s.handle(oracle.PUSH, k, h, len(v))
    _, got2 = s.dump()
    exp = (h.view(np.float16).astype(np.float32) * 2).astype(np.float16).view(np.uint16)
    np.testing.assert_array_equal(got2, exp)


def test_bf16_conversion():
    v = np.array([1.0, 1.00390625, 1.01171875, -3.3, 1e30], dtype=np.float32)
    s = oracle.Store(oracle.BF16)
    k = np.arange(len(v), dtype=np.uint64)
    u = v.view(np.uint32)
    rne = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    s.handle(oracle.PUSH, k, rne, len(v))
    _, got = s.dump()
    np.testing.assert_array_equal(got, rne)


def test_lr_apply_matches_reference_formula():
    """LRServer.h:171-177 + Adam.h:28-34, restated in pure Python doubles."""
    import math
    rng = np.random.default_rng(5)
    n = 64
    w = rng.uniform(-0.5, 0.5, n).astype(np.float32)
    merged = rng.uniform(-1, 1, n).astype(np.float32)
    lr = np.float32(0.01)
    m = np.zeros(n)
    v = np.zeros(n)
    w_or = w.copy()
    m_or, v_or = m.copy(), v.copy()
    for it in range(3):
        oracle.lr_apply(w_or, merged, float(lr), m_or, v_or, float(lr), 0.9, 0.999, 1e-8, it)
        for i in range(n):
            g = float(np.float32(lr * merged[i]))
            m[i] = 0.9 * m[i] + (1 - 0.9) * g
            v[i] = 0.999 * v[i] + (1 - 0.999) * g * g
            mh = m[i] / (1 - math.pow(0.9, it + 1))
            vh = v[i] / (1 - math.pow(0.999, it + 1))
            g = float(lr) * mh / (math.sqrt(vh) + 1e-8)
            w[i] = np.float32(float(w[i]) - g)
    np.testing.assert_array_equal(w_or, w)
    np.testing.assert_array_equal(m_or, m)


def test_cpu_baseline_runs():
    first, push, pull = oracle.bench(20000, 2)
    assert first > 0 and push > 0 and pull > 0


@pytest.mark.parametrize("dtype", [oracle.F32, oracle.F64, oracle.F16, oracle.BF16])
def test_out_of_order_and_repeated_keys_follow_the_sequential_loop(dtype):
    """oracle.Store on requests with keys in any order and repeated — the
    semantics the GPU's order-preserving path is checked against — equals a
    pure-Python replay of KVApp.h:446-454 (`store[key] += vals[i]` per
    occurrence, a PushPull answering the running value), addition by addition
    in the element type (f16 / bf16: each sum rounded once from f32, RNE)."""
    rng = np.random.default_rng(3 + dtype)
    keys = rng.integers(0, 50, 400).astype(np.uint64)
    vals = oracle.synth(400, dtype, 11, 1, -1.0, 1.0)
    np_t = {oracle.F32: np.float32, oracle.F64: np.float64}.get(dtype)

    def add(a, b):
        if np_t is not None:
            return np_t(np_t(a) + np_t(b))
        # f16 / bf16 bits: widen to f32, add, round once to the 16-bit type
        fa, fb = _half_to_f32(a, dtype), _half_to_f32(b, dtype)
        return _f32_to_half(np.float32(fa + fb), dtype)

    zero = np_t(0) if np_t is not None else np.uint16(0)
    ref, outs = {}, []
    for flags in (oracle.PUSH, oracle.PUSH | oracle.PULL, oracle.PULL):
        o = []
        for k, v in zip(keys.tolist(), vals):
            if flags & oracle.PUSH:
                ref[k] = add(ref.get(k, zero), v)
            if flags & oracle.PULL:
                o.append(ref.setdefault(k, zero))
        outs.append(np.array(o))
    st = oracle.Store(dtype)
    got = [st.handle(f, keys, vals if f & oracle.PUSH else None, 400)
           for f in (oracle.PUSH, oracle.PUSH | oracle.PULL, oracle.PULL)]
    np.testing.assert_array_equal(got[1], outs[1].astype(got[1].dtype))
    np.testing.assert_array_equal(got[2], outs[2].astype(got[2].dtype))
    k, v = st.dump()
    assert sorted(k.tolist()) == sorted(ref)
    exp = np.array([ref[int(x)] for x in k]).astype(v.dtype)
    np.testing.assert_array_equal(v, exp)


def _half_to_f32(bits, dtype):
    b = np.uint16(bits)
    if dtype == oracle.F16:
        return np.float32(b.view(np.float16))
    return np.array([np.uint32(b) << np.uint32(16)], np.uint32).view(np.float32)[0]


def _f32_to_half(x, dtype):
    if dtype == oracle.F16:
        return np.float16(x).view(np.uint16)
    u = int(np.array([x], np.float32).view(np.uint32)[0])
    if (u & 0x7F800000) == 0x7F800000 and (u & 0x7FFFFF):  # NaN
        return np.uint16((u >> 16) | 0x40)
    r = u + 0x7FFF + ((u >> 16) & 1)  # round to nearest even
    return np.uint16((r >> 16) & 0xFFFF)


LRG = np.load(os.path.join(HERE, "golden", "lr_ref.npz"))


@pytest.mark.parametrize("case", [str(c) for c in LRG["cases"]])
def test_lr_apply_matches_the_reference_adam(case):
    """oracle.lr_apply against LR rounds computed by the REFERENCE's own Adam
    (tests/src/Adam.h compiled where it lies into oracle/_ref/ref_lr_driver,
    run inside LRServer's apply loop, LRServer.h:171-177; fixture written by
    tests/golden/make_lr_golden.py): bit for bit, round by round."""
    w = LRG[f"{case}_w0"].copy()
    lr = float(LRG[f"{case}_lr"][0])
    adam = bool(LRG[f"{case}_adam"][0])
    n = len(w)
    m = np.zeros(n) if adam else None
    v = np.zeros(n) if adam else None
    for r, it in enumerate(LRG[f"{case}_iters"]):
        oracle.lr_apply(w, LRG[f"{case}_merged"][r], lr, m, v, lr, 0.9, 0.999, 1e-8, int(it))
        np.testing.assert_array_equal(w, LRG[f"{case}_out"][r], err_msg=f"{case} round {r}")
