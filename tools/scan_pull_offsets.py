#!/usr/bin/env python3
"""Pull rate at 256 M floats against the reply buffer's byte offset (4 KiB steps)."""
import sys, statistics, json, os
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "parameter-server_amd", "python"))
import psg
psg.set_device(0)
n = 256 << 20
st = psg.Store(psg.DENSE, psg.F32, 0, n, n)
slack = 4 << 20
o = psg.DeviceBuffer(n * 4 + slack)
s = psg.Stream()
def med(op, reps=10):
    for _ in range(2): op()
    ev = [psg.Event() for _ in range(reps + 1)]
    ev[0].record(s)
    for i in range(reps):
        op(); ev[i + 1].record(s)
    s.sync()
    return statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(reps))
res = []
for k in list(range(0, 128)) + [256, 384, 512, 640, 768, 896]:
    off = k * 4096
    ms = med(lambda: st.handle(psg.PULL, None, None, o.ptr + off, n, stream=s))
    res.append((off, round(8 * n / (ms * 1e-3) / 8e12, 4)))
print(json.dumps({"store": st.info().vals, "out": o.ptr, "res": res}))
