#!/usr/bin/env python3
"""Back-to-back dense Pushes at 256 M floats under the dense kernel's knobs.

Consecutive Pushes into one store are what a server sees when several workers
push in a row; they ran at 0.70 of HBM against 0.78 inside a Push-then-Pull
step.  Each configuration runs in its own process (PSG_DENSE_* are read once).
usage: sweep_b2b.py [UNROLLS] [NTS] [BPCS]      e.g. 1,2 1,3 1,2,4,8
"""
import itertools
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, statistics
sys.path.insert(0, %r)
import psg
psg.set_device(0)
n = 256 << 20
st = psg.Store(psg.DENSE, psg.F32, 0, n, n)
v = psg.DeviceBuffer(n * 4)
v.fill_synth(n, psg.F32, 7, 0, 0.0, 1000.0)
s = psg.Stream()
for _ in range(3):
    st.handle(psg.PUSH, None, v, None, n, stream=s)
ev = [psg.Event() for _ in range(21)]
ev[0].record(s)
for i in range(20):
    st.handle(psg.PUSH, None, v, None, n, stream=s)
    ev[i + 1].record(s)
s.sync()
ms = statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(20))
print(ms)
""" % os.path.join(ROOT, "parameter-server_amd", "python")


def ints(x):
    return [int(t) for t in x.split(",")]


unrolls = ints(sys.argv[1]) if len(sys.argv) > 1 else [1, 2]
nts = ints(sys.argv[2]) if len(sys.argv) > 2 else [1, 3]
bpcs = ints(sys.argv[3]) if len(sys.argv) > 3 else [1, 2, 4, 8]
rows = []
for u, nt, bpc in itertools.product(unrolls, nts, bpcs):
    env = dict(os.environ, PSG_DENSE_UNROLL=str(u), PSG_DENSE_NT=str(nt), PSG_DENSE_BPC=str(bpc))
    r = subprocess.run([sys.executable, "-c", CHILD], env=env, capture_output=True, text=True, timeout=120)
    if r.returncode != 0:
        print("FAILED", u, nt, bpc, r.stderr[-300:], flush=True)
        sys.exit(1)
    ms = float(r.stdout.strip().splitlines()[-1])
    row = dict(unroll=u, nt=nt, bpc=bpc, push_ms=ms, frac=round(12 * (256 << 20) / (ms * 1e-3) / 8e12, 4))
    rows.append(row)
    print(json.dumps(row), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(rows, open(os.path.join(ROOT, "gpurun_out", "sweep_b2b_256M.json"), "w"), indent=1)
print("BEST", json.dumps(max(rows, key=lambda r: r["frac"])))
