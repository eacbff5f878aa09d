#!/usr/bin/env python3
"""One kernel, launched alone, for a rocprofv3 --pmc pass (tools/gpu_run.sh
pmcpull / pmcadam; tools/pmc_summary.py turns two passes into HBM bytes per
launch).

  pull256  k_dense_vec<PULL> on a 256 M-float DENSE store (8 B / element
           algorithmic: store read + reply write), after 3 warm Pushes
  adam64   k_lr_apply_sum<ADAM> on 64 M features with 4 gradient frames
           (4 x 4 B + weight 8 B + f64 moments 32 B = 56 B / feature)

usage: pmc_targets.py pull256|adam64 [LAUNCHES]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parameter-server_amd", "python"))
import psg  # noqa: E402

what = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
psg.set_device(0)
s = psg.Stream()
if what == "pull256":
    n = 256 << 20
    st = psg.Store(psg.DENSE, psg.F32, 0, n, n)
    v, o = psg.DeviceBuffer(n * 4), psg.DeviceBuffer(n * 4)
    v.fill_synth(n, psg.F32, 7, 0, 0.0, 1000.0, s)
    for _ in range(3):
        st.handle(psg.PUSH, None, v, None, n, stream=s)
    for _ in range(reps):
        st.handle(psg.PULL, None, None, o, n, stream=s)
elif what == "adam64":
    n = 64 << 20
    w = psg.Store(psg.DENSE, psg.F32, 0, n, n)
    grads = [psg.DeviceBuffer(n * 4) for _ in range(4)]
    for j, g in enumerate(grads):
        g.fill_synth(n, psg.F32, 100 + j, 1, -1.0, 1.0, s)
    a = psg.Adam(n, 0.01)
    for it in range(reps):
        psg.lr_apply_sum(w, grads, n, 0.01, a, it, stream=s)
else:
    raise SystemExit(f"unknown target {what}")
s.sync()
psg.device_sync()
print("done", what, reps)
