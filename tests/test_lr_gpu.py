"""The LR server's BSP round as ONE fused kernel, single- and multi-GPU.

Reference: LRServer::RequestHandle merges the round's gradient pushes in
arrival order from 0 (tests/src/LRServer.h:155-160), then applies SGD / Adam
with f32 -> f64 promotions (:171-177, tests/src/Adam.h:28-34).  The oracle
replays exactly that (oracle.lr_apply on the sequentially merged f32 vector).
  psg_lr_apply_sum   merge + apply in one pass over the gradient frames
  psg_comm_lr_push   RCCL reduce-scatter, then the fused apply (one rank here,
                     the collective forced so RCCL itself runs)
  psg_xgmi_lr_push   every rank reads block r of all ranks' gradients in place
                     (hipIpc) and applies — bit-exact against the rank-order replay
"""
import multiprocessing as mp
import os
import sys
import uuid

import numpy as np
import pytest

import oracle
import psg

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LR = float(np.float32(0.01))  # LRServer's float learning_rate_, widened for Adam (LRServer.h:83-84)


def dev(a):
    return psg.DeviceBuffer.from_numpy(a)


def replay(w, grads_per_round, adam, from_zero=True, start_it=0):
    """The reference round by round: merge (f32, in order), then the update."""
    n = len(w)
    m = np.zeros(n) if adam else None
    v = np.zeros(n) if adam else None
    for it, grads in enumerate(grads_per_round):
        merged = np.zeros(n, np.float32) if from_zero else grads[0].copy()
        for g in (grads if from_zero else grads[1:]):
            merged = (merged + g).astype(np.float32)
        oracle.lr_apply(w, merged, 0.01, m, v, LR, 0.9, 0.999, 1e-8, start_it + it)
    return w


@pytest.fixture(scope="module", autouse=True)
def device():
    assert psg.device_count() >= 1, "no GPU visible"
    psg.set_device(0)
    yield


# layout: None = SGD; 0/1/2 = Adam with that moment layout (psg_lr.hip:
# two arrays, blocked per 128 features, the QUAD runs per 256)
@pytest.mark.parametrize("layout", [None, 1, 0, 2])
@pytest.mark.parametrize("n,ng,from_zero", [(100003, 1, False), (100003, 4, True), (4096, 16, True),
                                            (7, 3, True), (262144, 2, False), (1000, 5, True)])
def test_lr_apply_sum_bitexact(n, ng, from_zero, layout, monkeypatch):
    adam = layout is not None
    if adam:
        monkeypatch.setenv("PSG_ADAM_LAYOUT", str(layout))
    rng = np.random.default_rng(n + ng)
    w0 = rng.uniform(-0.5, 0.5, n).astype(np.float32)
    st = psg.Store(psg.DENSE, psg.F32, 0, n, n)
    st.handle(psg.PUSH, None, dev(w0), None, n)
    a = psg.Adam(n, LR) if adam else None
    rounds = [[rng.uniform(-1, 1, n).astype(np.float32) for _ in range(ng)] for _ in range(3)]
    for it, grads in enumerate(rounds):
        bufs = [dev(g) for g in grads]
        psg.lr_apply_sum(st, bufs, n, 0.01, a, it, from_zero=from_zero)
    _, got = st.dump()
    exp = replay(w0.copy(), rounds, adam, from_zero)
    np.testing.assert_array_equal(got, exp)


def test_lr_apply_sum_misaligned_gradient_takes_the_scalar_path():
    n = 1001
    rng = np.random.default_rng(3)
    w0 = rng.uniform(-0.5, 0.5, n).astype(np.float32)
    g = rng.uniform(-1, 1, n + 1).astype(np.float32)
    st = psg.Store(psg.DENSE, psg.F32, 0, n, n)
    st.handle(psg.PUSH, None, dev(w0), None, n)
    b = dev(g)
    psg.lr_apply_sum(st, [b.ptr + 4], n, 0.01, None, 0)  # 4-B aligned only
    _, got = st.dump()
    np.testing.assert_array_equal(got, replay(w0.copy(), [[g[1:]]], False))


def test_lr_apply_sum_rejects_bad_arguments():
    st = psg.Store(psg.DENSE, psg.F32, 0, 16, 16)
    g = psg.DeviceBuffer(64)
    with pytest.raises(psg.PsgError):
        psg.lr_apply_sum(st, [g] * 17, 16, 0.01, None, 0)  # more than 16 frames in one pass
    with pytest.raises(psg.PsgError):
        psg.lr_apply_sum(st, [g], 17, 0.01, None, 0)  # past the store's slots
    f16 = psg.Store(psg.DENSE, psg.F16, 0, 16, 16)
    with pytest.raises(psg.PsgError):
        psg.lr_apply_sum(f16, [g], 16, 0.01, None, 0)


@pytest.mark.parametrize("force", [False, True])
@pytest.mark.parametrize("adam", [False, True])
def test_comm_lr_push_single_rank(force, adam, monkeypatch):
    if force:
        monkeypatch.setenv("PSG_COMM_FORCE_COLLECTIVE", "1")
    n = 1 << 20
    c = psg.Comm(psg.comm_id(), 1, 0)
    rng = np.random.default_rng(5)
    w0 = rng.uniform(-0.5, 0.5, n).astype(np.float32)
    st = psg.Store(psg.DENSE, psg.F32, 0, n, n)
    st.handle(psg.PUSH, None, dev(w0), None, n)
    a = psg.Adam(n, LR) if adam else None
    rounds = [[rng.uniform(-1, 1, n).astype(np.float32)] for _ in range(3)]
    for it, (g,) in enumerate(rounds):
        c.lr_push(st, dev(g), n, 0.01, a, it)
    out = psg.DeviceBuffer(n * 4)
    c.pull(st, out, n)
    np.testing.assert_array_equal(out.download(np.float32, n), replay(w0.copy(), rounds, adam))
    c.close()


def _xgmi_lr_rank(rank, world, n, rounds, adam, name, q_in, q_out):
    try:
        _xgmi_lr_rank_body(rank, world, n, rounds, adam, name, q_in, q_out)
    except BaseException:  # report instead of leaving the peers and the parent waiting
        import traceback
        q_out.put(("err", rank, traceback.format_exc()))
        raise


def _xgmi_lr_rank_body(rank, world, n, rounds, adam, name, q_in, q_out):
    for p in (os.path.join(ROOT, "parameter-server_amd", "python"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    import psg
    psg.set_device(rank % psg.device_count())
    blk = n // world
    grads = psg.DeviceBuffer(n * 4)
    w = psg.Store(psg.DENSE, psg.F32, rank * blk, (rank + 1) * blk, blk)
    w0 = psg.DeviceBuffer(blk * 4)
    w0.fill_synth(blk, psg.F32, 900 + rank, 1, -0.5, 0.5)
    w.handle(psg.PUSH, None, w0, None, blk, first_key=rank * blk)  # 0 + w0 = w0
    a = psg.Adam(blk, LR) if adam else None
    sptr = w.info().vals
    psg.device_sync()
    q_out.put(("h", rank, psg.ipc_export(grads.ptr), psg.ipc_export(sptr)))
    handles = q_in.get(timeout=60)
    gptrs = [grads.ptr if r == rank else psg.ipc_open(handles[r][0]) for r in range(world)]
    sptrs = [sptr if r == rank else psg.ipc_open(handles[r][1]) for r in range(world)]
    x = psg.Xgmi(world, rank, gptrs, sptrs)
    bar = psg.NodeBarrier(name, world, rank)
    out = psg.DeviceBuffer(n * 4)
    for it in range(rounds):
        grads.fill_synth(n, psg.F32, 1000 * it + rank, 1, -1.0, 1.0)
        psg.device_sync()
        bar.wait(30.0)  # every rank's gradient is written
        x.lr_push(w, n, 0.01, a, it)
        psg.device_sync()
        bar.wait(30.0)  # every shard is updated
        x.pull(w, out, n)
        psg.device_sync()
        bar.wait(30.0)  # nobody overwrites a gradient a peer still reads
    got = out.download(np.float32, n)
    bar.wait(30.0)
    x.close()
    for r in range(world):
        if r != rank:
            psg.ipc_close(gptrs[r])
            psg.ipc_close(sptrs[r])
    bar.close()
    q_out.put(("r", rank, got))


@pytest.mark.parametrize("world,adam", [(2, True), (3, False)])
def test_xgmi_lr_push_multiprocess(world, adam):
    n = 3 * 64 * 16384  # divisible by 2 and 3, 16-B blocks; shards of 8-12 MB
    rounds = 3
    ctx = mp.get_context("spawn")
    q_out = ctx.Queue()
    q_in = [ctx.Queue() for _ in range(world)]
    name = "psg_xlr_" + uuid.uuid4().hex[:12]
    procs = [ctx.Process(target=_xgmi_lr_rank, args=(r, world, n, rounds, adam, name, q_in[r], q_out))
             for r in range(world)]
    for p in procs:
        p.start()
    def get():
        msg = q_out.get(timeout=100)
        assert msg[0] != "err", f"rank {msg[1]} failed:\n{msg[2]}"
        return msg

    try:
        handles = {}
        for _ in range(world):
            _, r, hg, hs = get()
            handles[r] = (hg, hs)
        for r in range(world):
            q_in[r].put(handles)
        results = {}
        for _ in range(world):
            _, r, got = get()
            results[r] = got
    finally:
        for p in procs:
            p.join(30)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    blk = n // world
    w0 = np.concatenate([oracle.synth(blk, oracle.F32, 900 + r, 1, -0.5, 0.5) for r in range(world)])
    g = [[oracle.synth(n, oracle.F32, 1000 * it + r, 1, -1.0, 1.0) for r in range(world)]
         for it in range(rounds)]
    exp = np.empty(n, np.float32)
    for s in range(world):  # shard s: its block of every rank's gradient, merged in rank order
        rs = [[x[s * blk:(s + 1) * blk] for x in gr] for gr in g]
        exp[s * blk:(s + 1) * blk] = replay(w0[s * blk:(s + 1) * blk].copy(), rs, adam)
    for r in range(world):
        np.testing.assert_array_equal(results[r], exp, err_msg=f"rank {r}'s pulled model")


LRG = np.load(os.path.join(ROOT, "tests", "golden", "lr_ref.npz"))


@pytest.mark.parametrize("layout", [1, 2])
@pytest.mark.parametrize("fused", [False, True])
@pytest.mark.parametrize("case", [str(c) for c in LRG["cases"]])
def test_lr_apply_matches_the_reference_adam(case, fused, layout, monkeypatch):
    """psg_lr_apply (the merged frame) and psg_lr_apply_sum (the merge fused in)
    against rounds computed by the REFERENCE's own Adam (tests/src/Adam.h,
    compiled where it lies, inside LRServer's apply loop; fixture
    tests/golden/make_lr_golden.py): bit for bit, round by round, SGD and Adam,
    repeated and skipped iterations; the Adam moments in two layouts."""
    monkeypatch.setenv("PSG_ADAM_LAYOUT", str(layout))
    w0 = LRG[f"{case}_w0"]
    n = len(w0)
    lr = float(LRG[f"{case}_lr"][0])
    st = psg.Store(psg.DENSE, psg.F32, 0, n, n)
    st.handle(psg.PUSH, None, dev(w0), None, n)
    a = psg.Adam(n, lr) if LRG[f"{case}_adam"][0] else None
    for r, it in enumerate(LRG[f"{case}_iters"]):
        g = dev(LRG[f"{case}_merged"][r])
        if fused:
            psg.lr_apply_sum(st, [g], n, lr, a, int(it))
        else:
            psg.lr_apply(st, g, n, lr, a, int(it))
        _, got = st.dump()
        np.testing.assert_array_equal(got, LRG[f"{case}_out"][r], err_msg=f"{case} round {r}")
