"""The reference's LR_ps.cpp (tests/LR_ps.cpp with tests/src/LR{Server,Worker}.h,
compiled UNMODIFIED against this runtime by `make -C parameter-server_amd dropin`)
trains end to end on our KVWorker / KVServer / Customer / Van.

The a9a archive it was written for ships as a 7z file (tests/LR samples.7z) that
nothing here can unpack, so the data are synthetic in the same libsvm text
format DataLoader reads (tests/src/DataLoader.h:145-170): 123 binary features,
~14 active per sample (the a9a encoding), labels from a hidden linear model.

Checks: the job (one process per node, like local.py) exits cleanly in sync BSP mode with Adam (local.py's own LR
settings, tests/local.py:70-84), with and without USE_KEY_CACHING (the worker
then sends a 1-key hash, LRWorker.h:214-219, which the server resolves,
LRServer.h:127-142); the server's saved model has the layout of
LRServer::SaveModel (LRServer.h:107-115); and it equals a numpy replay of the
same BSP training within 1e-4 relative (the server's merge adds the workers'
gradients in arrival order, and the workers' f32 dot products are
order-sensitive, so bit-equality is not the bar here — the model's update
itself is pinned bit-exactly by tests/test_lr_gpu.py and the KATs).
"""
import os
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "_dropin", "LR_ps")
NF, NW, ITERS = 123, 4, 6


def _write_data(d, rng):
    wtrue = rng.normal(0, 1, NF)

    def samples(m):
        X = np.zeros((m, NF), np.float32)
        for r in range(m):
            X[r, rng.choice(NF, 14, replace=False)] = 1.0
        y = (X @ wtrue + rng.normal(0, 0.5, m) > 0).astype(int)
        return X, y

    def dump(path, X, y):
        with open(path, "w") as f:
            for xr, lab in zip(X, y):
                idx = np.nonzero(xr)[0]
                f.write(("+1" if lab else "-1") + "".join(f" {i + 1}:1" for i in idx) + "\n")

    os.makedirs(os.path.join(d, "train"))
    os.makedirs(os.path.join(d, "test"))
    os.makedirs(os.path.join(d, "model"))
    parts = []
    for w in range(NW):
        X, y = samples(300)
        dump(os.path.join(d, "train", f"worker-0{w}"), X, y)
        parts.append((X, y))
    Xt, yt = samples(400)
    dump(os.path.join(d, "test", "full"), Xt, yt)
    return parts


def _init_weight(seed=0):
    """InitWeight (LRServer.h:36-46): srand(seed); w = rand()/RAND_MAX - 0.5 (float)."""
    import ctypes
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(seed)
    RAND_MAX = 2147483647
    return np.array([np.float32(np.float32(libc.rand()) / np.float32(RAND_MAX)) - np.float32(0.5)
                     for _ in range(NF)], np.float32)


def _replay(parts, odd_it, lr=0.01, C=1.0):
    """Full-batch BSP as LR_ps runs it with BATCH_SIZE=-1: each round every worker
    pulls the same weights, computes its gradient (LRWorker.h:79-88), the server
    merges the pushes and applies Adam (LRServer.h:155-177, Adam.h:28-34).

    BATCH_SIZE=-1: DataLoader::GetNextBatch hands out the whole set twice per
    epoch before it wraps (DataLoader.h:178-193), so a Train() call is two BSP
    rounds, and worker 0's second push carries cmd = 1.  The server advances
    Adam's iteration when it handles that push (LRServer.h:193-195) — before
    the round's apply unless worker 0's push is the round's last to arrive.
    odd_it[k] is the iteration round 2k+1 applied with (k or k + 1)."""
    w = _init_weight(0)
    m, v = np.zeros(NF), np.zeros(NF)
    for rnd in range(2 * ITERS):
        it = rnd // 2 if rnd % 2 == 0 else odd_it[rnd // 2]
        merged = np.zeros(NF, np.float32)
        for X, y in parts:
            z = (X.astype(np.float64) @ w.astype(np.float64)).astype(np.float32)
            s = 1.0 / (1.0 + np.exp(-z.astype(np.float64)))
            g = ((s - y)[:, None] * X).sum(0) / len(y) + C * w.astype(np.float64) / len(y)
            merged = (merged + g.astype(np.float32)).astype(np.float32)
        grad = (np.float32(lr) * merged).astype(np.float64)
        m = 0.9 * m + (1 - 0.9) * grad
        v = 0.999 * v + (1 - 0.999) * grad * grad
        grad = float(np.float32(lr)) * (m / (1 - 0.9 ** (it + 1))) / (np.sqrt(v / (1 - 0.999 ** (it + 1))) + 1e-8)
        w = (w.astype(np.float64) - grad).astype(np.float32)
    return w


def _closest_replay(parts, got, nw):
    """With one worker the iteration pattern is fixed; with several, the replay
    of whichever arrival pattern the run had (2^ITERS candidates) must match."""
    if nw == 1:
        return _replay(parts, [k for k in range(ITERS)])
    best = None
    for mask in range(1 << ITERS):
        e = _replay(parts, [k + ((mask >> k) & 1) for k in range(ITERS)])
        d = np.max(np.abs(e - got))
        if best is None or d < best[0]:
            best = (d, e)
    return best[1]


@pytest.mark.parametrize("nw,key_cache", [(1, False), (4, False), (4, True)])
def test_reference_lr_ps_trains_on_this_runtime(tmp_path, nw, key_cache):
    _run_lr_ps(tmp_path, nw, key_cache)


@pytest.mark.gpu
@pytest.mark.parametrize("nw,key_cache", [(4, False), (4, True)])
def test_reference_lr_ps_trains_on_the_mi355x_box(tmp_path, nw, key_cache):
    """The same unmodified LR_ps.cpp on the GPU box: every node process then
    opens the GPU (node k of each role on GPU k % ngpu), its large frames come
    from the pinned pool and the Van runs with HIP up; the reference's own
    LRServer handle is a host handle (SetRequestHandle), so the model math
    stays the reference's, and the replay bar is the same."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "parameter-server_amd", "python"))
    import psg
    assert psg.device_count() >= 1, "no GPU visible"
    _run_lr_ps(tmp_path, nw, key_cache)


def _run_lr_ps(tmp_path, nw, key_cache):
    if not os.path.exists(EXE):
        pytest.skip(f"{EXE} not built (needs the reference tree)")
    rng = np.random.default_rng(12)
    parts = _write_data(str(tmp_path), rng)[:nw]
    env = dict(os.environ, DATA_DIR=str(tmp_path), NUM_FEATURE=str(NF), ITERATION=str(ITERS),
               BATCH_SIZE="-1", TEST_PERIOD="0", SYNC_MODE="0", LEARNING_RATE="0.01", C="1",
               USE_ADAM="1")
    if key_cache:
        env["USE_KEY_CACHING"] = "1"
    # one process per node, as local.py launches it: the server's InitWeight
    # (srand(0); rand()...) must not share libc's generator with the workers'
    # srand(rank) / rand() (LR_ps.cpp:22, :71), which threads of one process would
    r = subprocess.run([EXE, "-ns", "1", "-nw", str(nw), "-procs"], cwd=str(tmp_path), env=env,
                       capture_output=True, text=True, timeout=240)
    if key_cache and r.returncode != 0 and "LRServer.h:145" in r.stdout + r.stderr \
            and "(1 vs. %d) Unmatched keys" % NF in r.stdout + r.stderr:
        # The reference's own defect: LRServer::use_key_cache_ (LRServer.h:236)
        # is never assigned — only the worker reads USE_KEY_CACHING
        # (LRWorker.h:42) — and `new lr::LRServer()` (LR_ps.cpp:14) leaves it
        # as whatever the heap held.  When that byte is 0 the server takes the
        # worker's 1-key hash request for a full list and fails its CHECK
        # (LRServer.h:145), as the reference would.  The key-cache protocol
        # itself is pinned by this runtime's KVServerLRHandle
        # (tests/test_dropin_gpu.py, lr_sync_gpu).
        pytest.xfail("reference LRServer reads its uninitialised use_key_cache_ (LRServer.h:127, :236)")
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    with open(os.path.join(tmp_path, "model", "lr_ps")) as f:
        toks = f.read().split()
    assert int(toks[0]) == ITERS and int(toks[1]) == NF
    got = np.array([float(t) for t in toks[2:]], np.float32)
    assert len(got) == NF
    exp = _closest_replay(parts, got, nw)
    np.testing.assert_allclose(got, exp, rtol=1e-4, atol=1e-6)
    for w in range(nw):
        assert os.path.exists(os.path.join(tmp_path, "model", f"worker-0{w}"))
