#!/usr/bin/env python3
"""Find the BSP round at which the HBM LR handle's model first goes wrong.

Runs tests/_dropin/lr_ref_pin in gpu mode (3 workers, 200,000 features, SGD,
BSP, dyadic gradients — the case GPUTEST_r03 caught) with PIN_TRACE, so worker
0 prints the last TRACE features of every Pull reply: the model after each
round.  Against the oracle's trajectory (oracle.lr_apply, the restatement the
reference's own LRServer is pinned to) it reports, for the first run whose
final model is wrong, the first round whose model differs, where, and the
difference in units of lr/64 beside every round's merged gradient.
usage: lr_pin_trace.py [TRIES] [TRACE]
"""
import json
import math
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle  # noqa: E402
import test_lr_ref_pin as t  # noqa: E402

NW, N = 3, 200000


def trajectory():
    w = t._init_weight(N)
    out = {}
    for e in range(t.EPOCHS):
        for b in range(t.BATCHES):
            out[(e, b)] = w.copy()  # what the Pull at the start of batch (e, b) returns
            merged = np.zeros(N, np.float32)
            for k in range(NW):
                merged = (merged + t._grad(False, k, e, b, N)).astype(np.float32)
            oracle.lr_apply(w, merged, t.LR, None, None, 0.0, 0.9, 0.999, 1e-8, e)
    out["final"] = w.copy()
    return out


def merged_at(i):
    return {f"{e},{b}": int(sum(((i * 7 + r * 3 + e * 5 + b) % 11) - 5 for r in range(NW)))
            for e in range(t.EPOCHS) for b in range(t.BATCHES)}


def main():
    tries = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    trace = int(sys.argv[2]) if len(sys.argv) > 2 else 30000
    traj = trajectory()
    for k in range(tries):
        with tempfile.TemporaryDirectory() as d:
            os.makedirs(os.path.join(d, "model"), exist_ok=True)
            env = dict(os.environ, PIN_MODE="gpu", PIN_GRAD="dyadic", NUM_FEATURE=str(N), LEARNING_RATE=str(t.LR),
                       SYNC_MODE="0", ITERATION=str(t.EPOCHS), DATA_DIR=d, PIN_EPOCHS=str(t.EPOCHS),
                       PIN_BATCHES=str(t.BATCHES), PIN_TRACE=str(trace), PS_POOL_POISON="1")
            env.pop("USE_ADAM", None)
            r = subprocess.run([t.EXE, "-ns", "1", "-nw", str(NW)], env=env, capture_output=True, text=True,
                               timeout=240)
        if r.returncode != 0:
            print(f"try {k}: rc {r.returncode}", r.stderr[-1500:])
            return 2
        pulls, models = {}, {}
        for line in r.stdout.splitlines():
            p = line.split()
            if p and p[0] == "PULL":
                first = int(p[3])
                pulls[(int(p[1]), int(p[2]))] = (first, np.array([int(x, 16) for x in p[4:]], np.uint32).view(np.float32))
            elif p and p[0] == "MODEL":
                models[int(p[1])] = np.array([int(x, 16) for x in p[3:]], np.uint32).view(np.float32)
            elif p and p[0] == "SERVER_MODEL":
                models["server"] = np.array([int(x, 16) for x in p[2:]], np.uint32).view(np.float32)
        fin = {str(m): int(np.count_nonzero(v.view(np.uint32) != traj["final"].view(np.uint32)))
               for m, v in models.items()}
        print(f"try {k}: final models differing from the oracle (features): {fin}", flush=True)
        if not any(fin.values()):
            continue
        report = {"try": k, "final": fin}
        for key in sorted(pulls):
            first, got = pulls[key]
            want = traj[key][first:]
            bad = np.nonzero(got.view(np.uint32) != want.view(np.uint32))[0]
            if bad.size:
                i = int(first + bad[0])
                d = [(float(got[j]) - float(want[j])) / t.LR * 64 for j in bad[:4]]
                report["first_wrong_pull"] = {"epoch_batch": key, "differing": int(bad.size),
                                              "range": [int(first + bad[0]), int(first + bad[-1])],
                                              "diff_lr_over_64": [round(x, 3) for x in d],
                                              "merged_per_round_at_first": merged_at(i),
                                              "merged_per_round_at_next": merged_at(i + 1)}
                break
        print(json.dumps(report), flush=True)
        os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
        json.dump(report, open(os.path.join(ROOT, "gpurun_out", "lr_pin_trace.json"), "w"), indent=1)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
