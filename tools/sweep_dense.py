#!/usr/bin/env python3
"""Sweep the dense accumulate kernel's launch/unroll/cache-policy knobs on the GPU.

Each configuration runs bench.py in its own process (the knobs are read once
per process from PSG_DENSE_UNROLL / PSG_DENSE_NT / PSG_DENSE_BPC).
  PSG_DENSE_NT bit 0: non-temporal request/reply streams; bit 1: non-temporal store.
usage: sweep_dense.py KEYS [UNROLLS] [NTS] [BPCS] [OP]     e.g. 67108864 1,2,4 1,2,3 2,4,8
OP = "all" (default: the knobs apply to Push and Pull) or "pull" (the Pull alone,
PSG_DENSE_PULL_*; the Push keeps its defaults).
SWEEP_ARGS (env) adds bench.py arguments, e.g. "--workload dense-f16".
Writes a table to stdout and gpurun_out/sweep_dense_<KEYS>.json.
"""
import itertools
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def ints(s):
    return [int(x) for x in s.split(",")]


keys = int(sys.argv[1]) if len(sys.argv) > 1 else 64 << 20
unrolls = ints(sys.argv[2]) if len(sys.argv) > 2 else [1, 2, 4, 8]
nts = ints(sys.argv[3]) if len(sys.argv) > 3 else [0, 1]
bpcs = ints(sys.argv[4]) if len(sys.argv) > 4 else [4, 8, 16]
op = sys.argv[5] if len(sys.argv) > 5 else "all"
pre = "PSG_DENSE_PULL_" if op == "pull" else "PSG_DENSE_"
rows = []
for unroll, nt, bpc in itertools.product(unrolls, nts, bpcs):
    env = dict(os.environ, **{pre + "UNROLL": str(unroll), pre + "NT": str(nt), pre + "BPC": str(bpc)})
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--check", "0",
           "--steps", "30", "--warmup", "3", "--keys", str(keys)] + os.environ.get("SWEEP_ARGS", "").split()
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    if r.returncode != 0:
        print("FAILED", unroll, nt, bpc, r.stderr[-400:], flush=True)
        sys.exit(r.returncode)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    row = dict(keys=keys, op=op, unroll=unroll, nt=nt, bpc=bpc, push_ms=d["push_ms"], pull_ms=d["pull_ms"],
               push_frac=d["roofline"]["frac"], pull_frac=d["pull_roofline_frac"], value=d["value"])
    rows.append(row)
    print(json.dumps(row), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(rows, open(os.path.join(ROOT, "gpurun_out", f"sweep_dense_{keys}_{op}.json"), "w"), indent=1)
best = max(rows, key=lambda r: r["value"])
print("BEST", json.dumps(best))
