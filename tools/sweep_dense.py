#!/usr/bin/env python3
"""Sweep the dense accumulate kernel's launch/unroll/cache-policy knobs on the GPU.

Each configuration runs bench.py in its own process (the knobs are read once
per process from PSG_DENSE_UNROLL / PSG_DENSE_NT / PSG_DENSE_BPC).  Writes a
table to stdout and gpurun_out/sweep_dense.json.
"""
import itertools
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
keys = int(sys.argv[1]) if len(sys.argv) > 1 else 64 << 20
rows = []
for unroll, nt, bpc in itertools.product([1, 2, 4, 8], [0, 1], [4, 8, 16]):
    env = dict(os.environ, PSG_DENSE_UNROLL=str(unroll), PSG_DENSE_NT=str(nt), PSG_DENSE_BPC=str(bpc))
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--no-cpu-baseline", "--check", "0",
           "--steps", "30", "--warmup", "3", "--keys", str(keys)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=120)
    if r.returncode != 0:
        print("FAILED", unroll, nt, bpc, r.stderr[-400:], flush=True)
        sys.exit(r.returncode)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    row = dict(unroll=unroll, nt=nt, bpc=bpc, push_ms=d["push_ms"], pull_ms=d["pull_ms"],
               push_frac=d["roofline"]["frac"], pull_frac=d["pull_roofline_frac"], value=d["value"])
    rows.append(row)
    print(json.dumps(row), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(rows, open(os.path.join(ROOT, "gpurun_out", f"sweep_dense_{keys}.json"), "w"), indent=1)
best = max(rows, key=lambda r: r["value"])
print("BEST", json.dumps(best))
