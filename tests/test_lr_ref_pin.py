"""LR parity pinned by the reference's own code.

tests/harness_ref/lr_ref_pin.cpp drives one of two servers with the same worker
requests (Pull, then Push of a gradient; cmd = 1 on an epoch's last batch,
LRWorker.h:188-210):
  ref  the reference's lr::LRServer (tests/src/LRServer.h:122-207 with
       Adam.h:28-34), compiled from the reference tree as it lies;
  gpu  this runtime's KVServerLRHandle, model and merge in HBM.
It prints the model worker 0 pulls at the end, bit for bit.

CPU: the reference server's model equals the oracle's replay (oracle.lr_apply,
the restatement the GPU LR kernels are checked against) bit for bit — the
oracle's LR update is pinned by the reference itself run here.
GPU: the HBM handle's model equals the reference server's bit for bit, real-
valued gradients with one worker (sync and async), dyadic ones (exact in any
merge order) with three, SGD and Adam, 123 and 200,000 features.
"""
import ctypes
import math
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "_dropin", "lr_ref_pin")
LR = 0.01
EPOCHS, BATCHES = 3, 4


def _run(tmp_path, mode, nw, n, adam, sync, grad, full=False):
    if not os.path.exists(EXE):
        pytest.skip(f"{EXE} not built (needs the reference tree)")
    os.makedirs(os.path.join(tmp_path, "model"), exist_ok=True)
    env = dict(os.environ, PIN_MODE=mode, PIN_GRAD=grad, NUM_FEATURE=str(n), LEARNING_RATE=str(LR),
               SYNC_MODE="0" if sync else "1", ITERATION=str(EPOCHS), DATA_DIR=str(tmp_path),
               PIN_EPOCHS=str(EPOCHS), PIN_BATCHES=str(BATCHES))
    env.pop("USE_ADAM", None)
    env.pop("USE_OLD_MODEL", None)
    if adam:
        env["USE_ADAM"] = "1"
    if mode == "gpu":
        # a recycled HBM block starts as NaN: a reply read before its kernel
        # wrote it cannot pass as an older reply's plausible values
        env["PS_POOL_POISON"] = "1"
    r = subprocess.run([EXE, "-ns", "1", "-nw", str(nw)], env=env,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    models = {}
    for l in r.stdout.splitlines():
        parts = l.split()
        if parts and parts[0] == "MODEL":
            assert int(parts[2]) == n
            models[int(parts[1])] = np.array([int(x, 16) for x in parts[3:]], dtype=np.uint32).view(np.float32)
        elif parts and parts[0] == "SERVER_MODEL":
            assert int(parts[1]) == n
            models["server"] = np.array([int(x, 16) for x in parts[2:]], dtype=np.uint32).view(np.float32)
    assert sorted(k for k in models if k != "server") == list(range(nw)), r.stdout[-2000:]
    if full:
        return models
    return models[0]


def _init_weight(n, seed=0):
    """LRServer.h:36-46 InitWeight: srand(seed); w = rand() / RAND_MAX - 0.5 in float."""
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(seed)
    return np.array([np.float32(np.float32(libc.rand()) / np.float32(2147483647)) - np.float32(0.5)
                     for _ in range(n)], np.float32)


def _grad(real, rank, e, b, n):
    """grad_of of lr_ref_pin.cpp."""
    if real:
        return np.array([np.float32(math.sin(0.37 * i + 1.3 * e + 0.71 * b + 2.9 * rank)) * np.float32(0.8)
                         for i in range(n)], np.float32)
    i = np.arange(n)
    return ((((i * 7 + rank * 3 + e * 5 + b) % 11) - 5) / 64.0).astype(np.float32)


def _oracle_replay(n, nw, adam, sync, real):
    """The oracle's LR update over the harness's requests (one worker, or sync
    mode on dyadic gradients: the round's merge is then order-free).  With one
    worker its cmd = 1 push is always the round's last, so an epoch's rounds
    apply with iteration = epoch (LRServer.h:193-195)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    w = _init_weight(n)
    m = np.zeros(n) if adam else None
    v = np.zeros(n) if adam else None
    alr = float(np.float32(LR)) if adam else 0.0
    for e in range(EPOCHS):
        for b in range(BATCHES):
            groups = [list(range(nw))] if sync else [[k] for k in range(nw)]
            for grp in groups:
                merged = np.zeros(n, np.float32)
                for k in grp:
                    merged = (merged + _grad(real, k, e, b, n)).astype(np.float32)
                oracle.lr_apply(w, merged, LR, m, v, alr, 0.9, 0.999, 1e-8, e)
    return w


@pytest.mark.parametrize("adam,sync", [(True, True), (False, True), (True, False)])
def test_reference_lr_server_equals_the_oracle_replay(tmp_path, adam, sync):
    n = 123
    got = _run(tmp_path, "ref", 1, n, adam, sync, "real")
    want = _oracle_replay(n, 1, adam, sync, True)
    bad = np.nonzero(got.view(np.uint32) != want.view(np.uint32))[0]
    assert bad.size == 0, f"feature {bad[0]}: reference {got[bad[0]]!r} oracle {want[bad[0]]!r}"


def test_reference_lr_server_three_workers_sgd_equals_the_oracle_replay(tmp_path):
    n = 123
    got = _run(tmp_path, "ref", 3, n, False, True, "dyadic")
    want = _oracle_replay(n, 3, False, True, False)
    assert np.array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("nw,n,adam,sync,grad", [
    (1, 123, True, True, "real"),
    (1, 123, False, True, "real"),
    (1, 123, True, False, "real"),
    (1, 200000, True, True, "real"),
    (3, 200000, False, True, "dyadic"),
    (3, 123, False, True, "dyadic"),
])
def test_hbm_lr_handle_equals_the_reference_lr_server(tmp_path, nw, n, adam, sync, grad):
    want = _run(os.path.join(tmp_path, "ref"), "ref", nw, n, adam, sync, grad)
    models = _run(os.path.join(tmp_path, "gpu"), "gpu", nw, n, adam, sync, grad, full=True)
    got = models[0]
    bad = np.nonzero(got.view(np.uint32) != want.view(np.uint32))[0]
    if bad.size and (nw == 1 or grad == "dyadic"):
        # which side is wrong: both against the oracle's replay (exact here)
        orc = _oracle_replay(n, nw, adam, sync, grad == "real")
        nref = int(np.count_nonzero(want.view(np.uint32) != orc.view(np.uint32)))
        ngpu = int(np.count_nonzero(got.view(np.uint32) != orc.view(np.uint32)))
        pytest.fail(f"{bad.size} features differ; first {bad[0]}: HBM handle {got[bad[0]]!r} reference LRServer "
                    f"{want[bad[0]]!r}; against the oracle replay: reference run {nref} differ, HBM run {ngpu} "
                    f"differ; " + _diagnose(models, want, nw, grad))
    assert bad.size == 0, (f"{bad.size} features differ; first {bad[0]}: HBM handle {got[bad[0]]!r} "
                           f"reference LRServer {want[bad[0]]!r}; " + _diagnose(models, want, nw, grad))
    # every worker's final Pull, and the server's own model, are the reference's
    for k, m in models.items():
        assert np.array_equal(m.view(np.uint32), want.view(np.uint32)), f"{k}: " + _diagnose(models, want, nw, grad)


def _diagnose(models, want, nw, grad):
    """Which copies of the model differ from the reference's, where, and — for
    dyadic gradients — the differences in units of lr/64 next to each BSP
    round's merged gradient at the first few differing features (a missing or
    repeated round shows as a row that matches)."""
    out = []
    for k, m in sorted(models.items(), key=lambda kv: str(kv[0])):
        b = np.nonzero(m.view(np.uint32) != want.view(np.uint32))[0]
        out.append(f"{k}: {b.size} differ" + (f" in [{b[0]}, {b[-1]}]" if b.size else ""))
    m0 = models[0]
    b = np.nonzero(m0.view(np.uint32) != want.view(np.uint32))[0]
    if b.size and grad == "dyadic":
        for i in b[:4]:
            d = (float(m0[i]) - float(want[i])) / LR * 64
            rounds = {(e, bb): int(sum(((i * 7 + r * 3 + e * 5 + bb) % 11) - 5 for r in range(nw)))
                      for e in range(EPOCHS) for bb in range(BATCHES)}
            out.append(f"feature {i}: (got - want) = {d:+.3f} lr/64; merged per (epoch, batch): {rounds}")
    return "; ".join(out)
