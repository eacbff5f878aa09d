#!/usr/bin/env python3
"""Roofline of the fused LR BSP round (psg_lr_apply_sum, k_lr_apply_sum).

One launch = LRServer's sync round (tests/src/LRServer.h:151-178) on n features:
merge the round's ng gradient frames from 0 in arrival order, then
weight -= lr * merge (SGD) or the Adam step (tests/src/Adam.h:28-34).
Algorithmic HBM bytes per feature: 4 per gradient frame + weight read/write 8,
+ Adam's f64 moments m and v read/write 32.  HIP-event medians over 20
launches on the kernel's stream (timing-only markers: psg_event_create_timing).
usage: bench_lr.py [N_FEATURES ...]      default 10000000 67108864
Writes one JSON line per case and gpurun_out/bench_lr.json.
"""
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "parameter-server_amd", "python"))
import psg  # noqa: E402

HBM_PEAK_GBS = 8000.0


def case(n, ng, adam, reps=20):
    s = psg.Stream()
    w = psg.Store(psg.DENSE, psg.F32, 0, n, n)
    grads = [psg.DeviceBuffer(n * 4) for _ in range(ng)]
    for j, g in enumerate(grads):
        g.fill_synth(n, psg.F32, 100 + j, 1, -1.0, 1.0, s)
    a = psg.Adam(n, 0.01) if adam else None
    it = 0
    for _ in range(3):
        psg.lr_apply_sum(w, grads, n, 0.01, a, it, stream=s)
        it += 1
    ev = [psg.Event(timing=True) for _ in range(reps + 1)]  # timing-only markers, as bench.py
    ev[0].record(s)
    for i in range(reps):
        psg.lr_apply_sum(w, grads, n, 0.01, a, it, stream=s)
        it += 1
        ev[i + 1].record(s)
    s.sync()
    ms = statistics.median(ev[i].elapsed_ms(ev[i + 1]) for i in range(reps))
    per = 4 * ng + 8 + (32 if adam else 0)
    gbs = per * n / (ms * 1e-3) / 1e9
    if a:
        a.close()
    w.close()
    for g in grads:
        g.free()
    return {"features": n, "grads": ng, "update": "adam" if adam else "sgd", "ms": round(ms, 5),
            "alg_bytes_per_feature": per, "achieved_gbs": round(gbs, 1), "frac": round(gbs / HBM_PEAK_GBS, 4)}


def main():
    psg.set_device(0)
    sizes = [int(x) for x in sys.argv[1:]] or [10_000_000, 64 << 20]
    rows = []
    for n in sizes:
        for ng in (1, 4):
            for adam in (False, True):
                r = case(n, ng, adam)
                rows.append(r)
                print(json.dumps(r), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    json.dump(rows, open(os.path.join(ROOT, "gpurun_out", "bench_lr.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
