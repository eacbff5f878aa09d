"""Coded tiles on the SORTED store (csrc/psg_store.hip, k_validate_code): a Push
on trusted windows whose tiles are subsets of their windows is resolved in its
validation pass, and the lean apply (k_tile_apply_db; f32) or k_resolve_apply
serves those tiles from the lane codes — no request key re-read, no window,
no search; a general tile met by the lean apply is applied by a follow-up.  A list that is a random subset
of the store's keys takes that path; tiles with absent
keys, with keys too far apart for a code, or with windows wider than 8192 keys
take the general path in the same request.  Every case is bit-exact against
the oracle (the restatement of KVApp.h:446-454), synchronous and in flight.
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


def request(st, orc, dtype, flags, dk, k, seed):
    n = len(k)
    v = oracle.synth(n, dtype, seed, 1, -1.0, 1.0)
    out = psg.DeviceBuffer(n * ES[dtype]) if flags & psg.PULL else None
    st.handle(flags, dk, dev(v) if flags & psg.PUSH else None, out, n)
    exp = orc.handle(flags, k, v if flags & psg.PUSH else None, n)
    if flags & psg.PULL:
        np.testing.assert_array_equal(out.download(NPT[dtype], n), exp, err_msg=f"flags {flags}")


def same_store(st, orc, dtype):
    gk, gv = st.dump()
    ok, ov = orc.dump()
    np.testing.assert_array_equal(gk, ok)
    np.testing.assert_array_equal(gv.view(NPT[dtype]), ov)


def subset(rng, univ, density):
    """a random subset of the store keys univ at `density` (sorted)"""
    pick = rng.random(len(univ)) < density
    return univ[pick]


def run_sequence(st, orc, dtype, k, seed, inflight=True):
    """Pushes, PushPulls and Pulls of k, synchronous first (the windows become
    trusted), then in flight, every reply and the store checked"""
    dk = dev(k)
    n = len(k)
    for r, flags in enumerate([psg.PUSH, ALL, psg.PULL, psg.PUSH, ALL, psg.PUSH]):
        request(st, orc, dtype, flags, dk, k, seed + r)
    if inflight:
        reqs, pending = [], []
        for j in range(10):
            flags = [psg.PUSH, ALL, psg.PUSH, psg.PULL][j % 4]
            v = oracle.synth(n, dtype, seed + 100 + j, 1, -1.0, 1.0)
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


@pytest.mark.parametrize("dtype", [psg.F32, psg.F16, psg.F64])
@pytest.mark.parametrize("density", [0.9, 0.7])
def test_random_subset_lists_take_coded_tiles(dtype, density):
    """A random subset of the store's keys: no tile is a stretch, every tile's
    keys are in the store — coded tiles, bit-exact, and the coded validation
    ran for the Pushes on trusted windows (psg_store_counters)."""
    rng, univ, st, orc = populated(dtype, 300000, 71 + int(density * 10))
    k = subset(rng, univ, density)
    run_sequence(st, orc, dtype, k, 500)
    c = st.counters()
    # (f32: once a Push of the list has been validated in full and served
    # lean, its verified copy validates the later ones: k_list_check)
    assert c["coded"] + c["lists"] >= 4, c
    assert c["ident"] == 0 or c["notident"] >= 1, c


def test_coded_tiles_beside_absent_keys_and_wide_gaps():
    """One list whose tiles are of every kind: coded (90 % and 80 % subsets),
    general with absent keys (inserted by the follow-up, like operator[]),
    general with a lane whose keys are too far apart for its code (a run of 40
    store keys left out of a 95 % subset), general with windows wider than
    8192 keys (every 3rd and every 25th store key), a stretch, and a short tail
    tile.  (The store holds under 1.5 keys per request key, so the request
    takes 1024-thread tiles, whose Pushes are coded.)"""
    dtype = psg.F32
    rng, univ, st, orc = populated(dtype, 400000, 83)
    holed = subset(rng, univ[100000:140000], 0.95)
    for at in (5000, 17000, 29000):
        lo_key, hi_key = univ[100000 + at], univ[100000 + at + 40]
        holed = holed[(holed < lo_key) | (holed >= hi_key)]
    parts = [
        subset(rng, univ[:100000], 0.9),
        holed,
        univ[140000:180000:25],
        univ[180000:210000:3],
        univ[210000:300000],
        subset(rng, univ[300000:396000], 0.8),
    ]
    k = np.concatenate(parts)
    # absent keys: just above store keys of the last part
    fresh = np.setdiff1d(univ[300001:396000:997] + np.uint64(1), univ)
    k = np.unique(np.concatenate([k, fresh, univ[396000:396000 + 3001]]))
    assert len(univ) < 1.5 * len(k)
    run_sequence(st, orc, dtype, k, 900)
    c = st.counters()
    assert c["coded"] >= 4, c
    # the first lean apply met the general tiles: a follow-up, then the list
    # stays on k_resolve_apply
    assert c["lean"] >= 1 and c["lean_partial"] >= 1, c
    # new absent keys in a list whose other keys were coded
    more = np.setdiff1d(univ[5:100000:13] + np.uint64(3), univ)
    k2 = np.unique(np.concatenate([k, more]))
    run_sequence(st, orc, dtype, k2, 1300, inflight=False)


@pytest.mark.parametrize("n_keys", [1, 3, 4095, 4097, 8193, 50001])
def test_coded_tiles_ragged_sizes(n_keys):
    """Lists of 1, 3, 4095, 4097, 8193 and 50001 keys, each a random 90 % of
    its store: tail lanes with fewer than 4 keys, tail tiles of one lane."""
    dtype = psg.F32
    m = int(np.ceil(n_keys / 0.9)) + 1
    rng, univ, st, orc = populated(dtype, m, 101 + n_keys)
    k = np.sort(rng.choice(univ, n_keys, replace=False))
    run_sequence(st, orc, dtype, k, 40 + n_keys, inflight=n_keys > 3)
    if n_keys >= 4095:
        c = st.counters()
        assert c["coded"] >= 1 and c["lean"] >= 1, c


def test_coded_list_rewritten_shifted_under_the_same_pointer():
    """A trusted subset list rewritten in place, shifted by one key (its first
    key dropped, a store key appended): every tile's cached window then holds
    one key of the tile before it.  A coded tile rewrites its whole window of
    values, so it must not be coded on such a window (k_validate_code requires
    the window to be exactly the tile's); the Pushes, synchronous and in
    flight, stay bit-exact."""
    dtype = psg.F32
    rng, univ, st, orc = populated(dtype, 300000, 57)
    k = subset(rng, univ[:-10], 0.9)
    dk = dev(k)
    n = len(k)
    for r, flags in enumerate([psg.PUSH, ALL, psg.PUSH, psg.PUSH]):
        request(st, orc, dtype, flags, dk, k, 600 + r)
    assert st.counters()["coded"] >= 1
    k2 = np.concatenate([k[1:], univ[-5:-4]])
    dk.upload(k2)
    run_sequence(st, orc, dtype, k2, 700)


def test_coded_list_with_a_key_out_of_range_is_rejected():
    """A subset list plus one key past the shard's range: the coded validation
    rejects the whole request (PSG_ERR_RANGE) and no tile writes anything."""
    dtype = psg.F32
    rng = np.random.default_rng(97)
    ke = 1 << 62
    univ = np.unique(rng.integers(0, ke, 200000, dtype=np.uint64))
    st = psg.Store(psg.SORTED, dtype, 0, ke, 0)
    orc = oracle.Store(dtype)
    v0 = oracle.synth(len(univ), dtype, 3, 1, -1.0, 1.0)
    st.handle(psg.PUSH, dev(univ), dev(v0), None, len(univ))
    orc.handle(oracle.PUSH, univ, v0, len(univ))
    k = subset(rng, univ, 0.85)
    dk = dev(k)
    for r in range(4):
        request(st, orc, dtype, psg.PUSH, dk, k, 40 + r)
    assert st.counters()["coded"] >= 1
    # the trusted list rewritten under the same pointer with its last key past
    # the range: its Push is validated by the coded pass, which must reject it
    n = len(k)
    dk.upload(np.array([ke + 5], np.uint64), offset=(n - 1) * 8)
    before = st.counters()["coded"]
    v = oracle.synth(n, dtype, 77, 1, -1.0, 1.0)
    with pytest.raises(psg.PsgError) as ei:
        st.handle(psg.PUSH, dk, dev(v), None, n)
    assert ei.value.code == 4
    assert st.counters()["coded"] == before + 1
    same_store(st, orc, dtype)
    dk.upload(k[-1:], offset=(n - 1) * 8)
    request(st, orc, dtype, ALL, dk, k, 50)
    same_store(st, orc, dtype)


def test_coded_list_out_of_order_is_served_in_arrival_order():
    """Two keys of a subset list swapped: not rejected (§7 of DESIGN.md) but
    served in arrival order by the order-preserving path; the store equals the
    oracle's sequential replay."""
    dtype = psg.F32
    rng, univ, st, orc = populated(dtype, 200000, 61)
    k = subset(rng, univ, 0.9)
    dk = dev(k)
    for r in range(4):
        request(st, orc, dtype, psg.PUSH, dk, k, 10 + r)
    # the trusted list rewritten under the same pointer with two keys swapped:
    # the coded pass sees them out of order
    bad = k.copy()
    bad[5000], bad[5001] = bad[5001], bad[5000]
    dk.upload(bad[5000:5002], offset=5000 * 8)
    ordered = st.counters()["ordered"]
    request(st, orc, dtype, psg.PUSH, dk, bad, 30)
    assert st.counters()["ordered"] > ordered
    same_store(st, orc, dtype)
    request(st, orc, dtype, ALL, dk, bad, 31)
    dk.upload(k[5000:5002], offset=5000 * 8)
    request(st, orc, dtype, ALL, dk, k, 32)
    same_store(st, orc, dtype)


def test_coded_tiles_switch_off_matches():
    """PSG_RA_CODED=0 (read once per process) keeps the stretch check alone:
    the same random-subset sequence in fresh processes, both bit-exact."""
    child = r"""
import sys, numpy as np
sys.path[:0] = {paths!r}
import oracle, psg
psg.set_device(0)
rng = np.random.default_rng(67)
univ = np.unique(rng.integers(0, (1 << 64) - 1, 300000, dtype=np.uint64))
st, orc = psg.Store(psg.SORTED, psg.F32, 0, (1 << 64) - 1, 0), oracle.Store()
st.handle(psg.PUSH, psg.DeviceBuffer.from_numpy(univ), psg.DeviceBuffer.from_numpy(np.ones(len(univ), np.float32)), None, len(univ))
orc.handle(oracle.PUSH, univ, np.ones(len(univ), np.float32), len(univ))
k = univ[rng.random(len(univ)) < 0.85]
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
print("ok", st.counters()["coded"])
"""
    paths = [os.path.join(os.path.dirname(HERE), "parameter-server_amd", "python"),
             os.path.join(os.path.dirname(HERE), "oracle")]
    coded = {}
    for env_val in ("0", "1"):
        env = dict(os.environ, PSG_RA_CODED=env_val)
        r = subprocess.run([sys.executable, "-c", child.format(paths=paths)], env=env,
                           capture_output=True, text=True, timeout=120)
        assert r.returncode == 0, r.stderr[-2000:]
        last = r.stdout.strip().splitlines()[-1].split()
        assert last[0] == "ok"
        coded[env_val] = int(last[1])
    assert coded["0"] == 0 and coded["1"] >= 1, coded


def test_partial_lean_apply_with_requests_in_flight_behind_it():
    """The first lean apply (k_tile_apply) of a list whose seam tiles are
    general leaves those to a follow-up (W_PARTIAL) that runs only when the
    request is reaped — after the requests launched behind it have validated
    their own tiles.  Each request keeps its own tile words (one set per ring
    slot), so the follow-up applies exactly the seam tiles: a burst of requests
    in flight right after the list's windows are trusted, bit-exact."""
    dtype = psg.F32
    rng, univ, st, orc = populated(dtype, 400000, 113)
    # 16 stretches with 200 store keys left out at each seam; a 90 % subset
    # in the middle
    parts = [univ[j * 24000: j * 24000 + 23800] for j in range(16)]
    parts[8] = subset(rng, parts[8], 0.9)
    k = np.concatenate(parts)
    dk = dev(k)
    n = len(k)
    request(st, orc, dtype, psg.PUSH, dk, k, 1)   # windows searched, then trusted
    request(st, orc, dtype, psg.PUSH, dk, k, 2)   # the identity trial fails once
    reqs, pending = [], []
    for j in range(12):
        flags = [psg.PUSH, psg.PUSH, ALL, psg.PULL][j % 4]
        v = oracle.synth(n, dtype, 300 + j, 1, -1.0, 1.0)
        dv = dev(v)
        out = psg.DeviceBuffer(n * 4) if flags & psg.PULL else None
        pending.append(st.handle_async(flags, dk, dv if flags & psg.PUSH else None, out, n))
        reqs.append((dv, out, orc.handle(flags, k, v if flags & psg.PUSH else None, n)))
    st.wait()
    psg.device_sync()
    for j, (_, out, exp) in enumerate(reqs):
        if out is not None:
            np.testing.assert_array_equal(out.download(np.float32, n), exp, err_msg=f"request {j}")
    same_store(st, orc, dtype)
    c = st.counters()
    assert c["coded"] >= 1
    # the Pushes after the trial went lean; the first met the seam tiles
    assert c["lean"] >= 1 and c["lean_partial"] >= 1, c


def test_lean_apply_with_many_tiles_per_block():
    """A list of ~3 M keys (more tiles than the lean apply's blocks: each block
    serves several) made of 12 stretches of the store, 300 store keys left out
    at each seam (a seam tile's window spans both sides: coded), so every
    Push after the trial is lean — every wave of a block on every tile; then
    requests in flight.  Found a
    race (a block's first wave marking a tile done before its last wave read
    the tile's kind) that under-applied whole waves: bit-exact now."""
    dtype = psg.F32
    rng, univ, st, orc = populated(dtype, 3300000, 127)
    per = len(univ) // 12
    k = np.concatenate([univ[j * per: (j + 1) * per - 300] for j in range(12)])
    run_sequence(st, orc, dtype, k, 800)
    c = st.counters()
    assert c["lean"] >= 1 and c["lean_partial"] == 0, c


def test_lean_apply_coded_tiles_many_per_block():
    """A random 90 % subset of a 3.3 M-key store (~730 coded tiles, more than
    the lean apply's blocks): a block stages its next coded tile's window into
    its second LDS buffer while it applies the current one — Pushes, PushPulls
    and Pulls, then in flight, bit-exact."""
    dtype = psg.F32
    rng, univ, st, orc = populated(dtype, 3300000, 131)
    k = subset(rng, univ, 0.9)
    run_sequence(st, orc, dtype, k, 1700)
    c = st.counters()
    assert c["lean"] >= 1 and c["lean_partial"] == 0, c
