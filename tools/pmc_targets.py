#!/usr/bin/env python3
"""One kernel, launched alone, for a rocprofv3 --pmc pass (tools/gpu_run.sh
pmcpull / pmcadam; tools/pmc_summary.py turns two passes into HBM bytes per
launch).

  pull256  k_dense_vec<PULL> on a 256 M-float DENSE store (8 B / element
           algorithmic: store read + reply write), after 3 warm Pushes
  adam64   k_lr_apply_sum<ADAM> on 64 M features with 4 gradient frames
           (4 x 4 B + weight 8 B + f64 moments 32 B = 56 B / feature)

  frames8/4       a run of 8 (4) dense Pushes, 64 M floats (k_frames_apply: 8 + 4k B / element)
  frames_keyed8/4 a run of 8 (4) Pushes of one 10 M-key list = the SORTED store (16 + 12k B / key)
  frames_cached8/4 a run of 8 (4) Pushes on a cached stretch of slots (8 + 4k B / key)

  strided4push / strided4pull / strided8push / strided8pull
                  a run of P = 4 (8) requests on the reference benchmark's
                  interleaved lists (kMaxKey/num*i + r), 10 M store keys in all —
                  one server's share of the drop-in line at ns = nw = P:
                  k_run_pass check + apply (28 B / key) / the checked Pull
                  pass (24 B / key), psg_store_run

usage: pmc_targets.py TARGET [LAUNCHES]
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
elif what in ("frames8", "frames4"):
    # a run of k dense Pushes on a 64 M-float DENSE store (k_frames_apply):
    # store 8 + 4k B / element
    k = int(what[-1])
    n = 64 << 20
    st = psg.Store(psg.DENSE, psg.F32, 0, n, n)
    vs = [psg.DeviceBuffer(n * 4) for _ in range(k)]
    for j, v in enumerate(vs):
        v.fill_synth(n, psg.F32, 7 + j, 0, 0.0, 100.0, s)
    for _ in range(reps):
        st.push_frames(None, vs, n, stream=s)
elif what in ("frames_keyed8", "frames_keyed4"):
    # a run of k Pushes of one 10 M-key list (k copies of it) that is the whole
    # SORTED store: k_frames_base + k_frames_check (store key 8 + 8 per list) +
    # k_frames_apply (store value 8 + 4 per frame): 16 + 12k B / key
    import numpy as np
    k = int(what[-1])
    n = 10_000_000
    rng = np.random.default_rng(9)
    keys = np.unique(rng.integers(0, (1 << 64) - 1, n + 4096, dtype=np.uint64))[:n]
    st = psg.Store(psg.SORTED, psg.F32, 0, (1 << 64) - 1, 0)
    dks = [psg.DeviceBuffer.from_numpy(keys, s) for _ in range(k)]
    vs = [psg.DeviceBuffer(n * 4) for _ in range(k)]
    for j, v in enumerate(vs):
        v.fill_synth(n, psg.F32, 7 + j, 0, 0.0, 100.0, s)
    st.handle(psg.PUSH, dks[0], vs[0], None, n, stream=s)
    for _ in range(reps):
        assert st.push_frames(dks, vs, n, stream=s)
elif what in ("frames_cached8", "frames_cached4"):
    # a run of k Pushes on a cached list that is a stretch of slots
    # (psg_store_push_slots_frames, k_frames_apply): 8 + 4k B / key
    import numpy as np
    k = int(what[-1])
    n = 10_000_000
    rng = np.random.default_rng(9)
    keys = np.unique(rng.integers(0, (1 << 64) - 1, n + 4096, dtype=np.uint64))[:n]
    st = psg.Store(psg.SORTED, psg.F32, 0, (1 << 64) - 1, 0)
    dk = psg.DeviceBuffer.from_numpy(keys, s)
    slots = psg.DeviceBuffer(n * 4)
    st.resolve(dk, n, slots, insert=True, stream=s)
    first = st.slots_stretch(slots, n, stream=s)
    vs = [psg.DeviceBuffer(n * 4) for _ in range(k)]
    for j, v in enumerate(vs):
        v.fill_synth(n, psg.F32, 7 + j, 0, 0.0, 100.0, s)
    for _ in range(reps):
        st.push_slots_frames(None, vs, n, first=first, stream=s)
elif what.startswith("strided"):
    import numpy as np
    P = int(what[7])
    op = psg.PUSH if what.endswith("push") else psg.PULL
    n = 10_000_000 // P
    step = np.uint64(((1 << 64) - 1) // n)
    lists = [np.arange(n, dtype=np.uint64) * step + np.uint64(r) for r in range(P)]
    st = psg.Store(psg.SORTED, psg.F32, 0, (1 << 64) - 1, 0)
    dks = [psg.DeviceBuffer.from_numpy(l, s) for l in lists]
    vs = [psg.DeviceBuffer(n * 4) for _ in range(P)]
    outs = [psg.DeviceBuffer(n * 4) for _ in range(P)]
    for j, v in enumerate(vs):
        v.fill_synth(n, psg.F32, 7 + j, 0, 0.0, 100.0, s)
    for j in range(P):
        st.handle(psg.PUSH, dks[j], vs[j], None, n, stream=s)
    order = list(range(P))[::-1]
    for _ in range(reps):
        served = st.run([op] * P, [dks[j] for j in order], [n] * P,
                        [vs[j] if op == psg.PUSH else None for j in order],
                        [outs[j] if op == psg.PULL else None for j in order], stream=s)
        assert served == psg.RUN_STRIDED, served
else:
    raise SystemExit(f"unknown target {what}")
s.sync()
psg.device_sync()
print("done", what, reps)
