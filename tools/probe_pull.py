#!/usr/bin/env python3
"""Where the 256 M-float Pull's run-to-run spread comes from.

The Pull (read store, write reply) measures 0.68..0.81 of HBM across
processes with the same kernel and knobs.  Each process here times, on one
store, back-to-back Pulls and Pushes with the reply / request placed at a few
byte offsets inside one larger allocation, so the placement of the request
and reply streams relative to the store can be told apart from the process.
usage: probe_pull.py [PROCESSES]
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CHILD = r"""
import sys, statistics, json
sys.path.insert(0, %r)
import psg
psg.set_device(0)
n = 256 << 20
st = psg.Store(psg.DENSE, psg.F32, 0, n, n)
slack = 16 << 20
vb = psg.DeviceBuffer(n * 4 + slack)
o = psg.DeviceBuffer(n * 4 + slack)
vb.fill_synth((n * 4 + slack) // 4, psg.F32, 7, 0, 0.0, 1000.0)
s = psg.Stream()
frac = lambda ms, b: round(b * n / (ms * 1e-3) / 8e12, 4)


def med(op, reps=20):
    for _ in range(3):
        op()
    ev = [psg.Event() for _ in range(reps + 1)]
    ev[0].record(s)
    for i in range(reps):
        op()
        ev[i + 1].record(s)
    s.sync()
    return statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(reps))


res = {}
for off in (0, 16384, 65536, 262144, (1 << 20) + 65536):
    out, v = o.ptr + off, vb.ptr + off
    pull = med(lambda: st.handle(psg.PULL, None, None, out, n, stream=s))
    push = med(lambda: st.handle(psg.PUSH, None, v, None, n, stream=s))
    res[off] = {"pull_b2b": frac(pull, 8), "push_b2b": frac(push, 12)}
print(json.dumps({"store": st.info().vals, "out": o.ptr, "res": res}))
""" % os.path.join(ROOT, "parameter-server_amd", "python")

procs = int(sys.argv[1]) if len(sys.argv) > 1 else 4
rows = []
for k in range(procs):
    r = subprocess.run([sys.executable, "-c", CHILD], capture_output=True, text=True, timeout=120)
    if r.returncode != 0:
        print("FAILED", r.stderr[-400:], flush=True)
        sys.exit(1)
    d = json.loads(r.stdout.strip().splitlines()[-1])
    rows.append(d)
    print(json.dumps(d), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
json.dump(rows, open(os.path.join(ROOT, "gpurun_out", "probe_pull_256M.json"), "w"), indent=1)
