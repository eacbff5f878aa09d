"""Stress: a 10 M-key SORTED store, requests of the store's own list (or a
subset) in flight like bench.py's keyed line; checks the store after each
burst against the closed form (values all 1.0)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "parameter-server_amd", "python")]
import psg
psg.set_device(0)
L = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
burst = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rng = np.random.default_rng(9)
k = np.unique(rng.integers(0, (1 << 64) - 1, int(L * 1.01) + 1024, dtype=np.uint64))
k = np.sort(rng.choice(k, L, replace=False))
st = psg.Store(psg.SORTED, psg.F32, 0, (1 << 64) - 1, 0)
s = psg.Stream()
dk = psg.DeviceBuffer.from_numpy(k)
ones = psg.DeviceBuffer.from_numpy(np.ones(L, np.float32))
out = psg.DeviceBuffer(L * 4)
total = 0
for rnd in range(6):
    for j in range(burst):
        st.handle_async(psg.PUSH, dk, ones, None, L, stream=s)
        total += 1
        if j % 2 == 1:
            st.handle_async(psg.PULL, dk, None, out, L, stream=s)
    st.wait()
    psg.device_sync()
    gk, gv = st.dump()
    bad = np.flatnonzero(gv.view(np.float32) != total)
    print("round", rnd, "pushes", total, "bad", len(bad), "first", bad[:5].tolist(),
          "vals", gv.view(np.float32)[bad[:5]].tolist(), "tiles", sorted(set((bad // 4096).tolist()))[:10],
          st.counters(), flush=True)
