#!/usr/bin/env python3
"""Writes tests/golden/lr_ref.npz: LR apply rounds computed by the REFERENCE's
own Adam (tests/src/Adam.h, compiled where it lies by oracle/Makefile into
oracle/_ref/ref_lr_driver) inside LRServer's apply loop (LRServer.h:171-177).

Run here, where /root/reference exists (`make -C oracle` first); the fixture is
committed, so the tests never need the reference.  Inputs are seeded numpy
draws: weights in [-0.5, 0.5), merged gradients in [-2, 2) with zeros, tiny
and large values mixed in, and iteration patterns that repeat and skip (the
sync server advances its iteration by arrival order, LRServer.h:193-195).
"""
import os
import subprocess
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_lr_driver")

CASES = [  # name, n, use_adam, learning_rate, iterations of the rounds
    ("sgd", 4099, 0, 0.01, [0, 0, 1, 1, 2, 3]),
    ("adam", 4099, 1, 0.01, [0, 0, 1, 1, 2, 3]),
    ("adam_lr05", 1031, 1, 0.05, [0, 1, 2, 3, 4, 5, 6, 7]),
    ("adam_skips", 777, 1, 0.001, [0, 2, 2, 5, 9]),
]


def run_case(name, n, adam, lr, iters, rng):
    w0 = rng.uniform(-0.5, 0.5, n).astype(np.float32)
    merged = rng.uniform(-2.0, 2.0, (len(iters), n)).astype(np.float32)
    merged[:, ::97] = 0.0
    merged[:, 1::101] = np.float32(1e-30)
    merged[:, 2::103] = np.float32(3e4)
    with tempfile.TemporaryDirectory() as d:
        fin, fout = os.path.join(d, "in.bin"), os.path.join(d, "out.bin")
        with open(fin, "wb") as f:
            f.write(np.array([n, len(iters), adam], np.int32).tobytes())
            f.write(np.array([lr], np.float32).tobytes())
            f.write(w0.tobytes())
            for it, g in zip(iters, merged):
                f.write(np.array([it], np.int32).tobytes())
                f.write(g.tobytes())
        subprocess.run([DRIVER, fin, fout], check=True)
        out = np.fromfile(fout, np.float32).reshape(len(iters), n)
    return {f"{name}_w0": w0, f"{name}_merged": merged, f"{name}_iters": np.array(iters, np.int32),
            f"{name}_lr": np.array([lr], np.float32), f"{name}_adam": np.array([adam], np.int32),
            f"{name}_out": out}


def main():
    if not os.path.exists(DRIVER):
        raise SystemExit(f"{DRIVER} not built: make -C oracle (needs /root/reference)")
    rng = np.random.default_rng(2024)
    data = {"cases": np.array([c[0] for c in CASES])}
    for c in CASES:
        data.update(run_case(*c, rng))
    np.savez_compressed(os.path.join(HERE, "lr_ref.npz"), **data)
    print("wrote", os.path.join(HERE, "lr_ref.npz"), {k: v.shape for k, v in data.items()})


if __name__ == "__main__":
    main()
