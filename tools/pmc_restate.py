#!/usr/bin/env python3
"""Restate the keyed PMC summaries with the round-5 per-shape calibration
(profiles/r5_pmc_calibration.json): every read shape those kernels use counts
exactly 64 B of FETCH_SIZE per 128-B line (so the x2 of tools/pmc_summary.py
holds for them too), and WRITE_SIZE counts 32/64-B write granules.  The bytes
per launch therefore stand; this records, per summary, the shapes its kernels
use, their calibrated factors and the resulting ratio.
usage: pmc_restate.py OUT_JSON SUMMARY.json ...
"""
import json
import sys

calib = json.load(open("profiles/r5_pmc_calibration.json"))["shapes"]
# the access shapes of each kernel (csrc/psg_store.hip, psg_dense.hip)
SHAPES = {
    "k_validate_windows": ["p_rd16"],
    "k_resolve_apply": ["p_rd16", "p_rd8", "p_rd4", "p_gather4", "p_wr16", "p_span32", "p_scatter4", "p_rmw4"],
    "k_ident_check": ["p_rd16"],
    "k_ident_apply": ["p_rd16", "p_wr16"],
    "k_slots_vec": ["p_rd16", "p_gather4", "p_wr16", "p_scatter4", "p_rmw4"],
    "k_dense_vec": ["p_rd16", "p_wr16"],
    "k_lr_apply_sum": ["p_rd16", "p_wr16"],
}
out = {"calibration": "profiles/r5_pmc_calibration.json", "summaries": []}
for f in sys.argv[2:]:
    s = json.load(open(f))
    kernels = [k for k in SHAPES if k in s["kernel"]]
    shapes = sorted({x for k in kernels for x in SHAPES[k]})
    rf = {x: calib[x].get("fetch_factor") for x in shapes if calib[x].get("fetch_factor")}
    wf = {x: calib[x].get("write_factor") for x in shapes if calib[x].get("write_factor")}
    read_ok = all(abs(v - 2.0) < 1e-3 for v in rf.values())
    out["summaries"].append({
        "file": f, "kernel": s["kernel"], "kernels": kernels, "read_shapes": rf, "write_shapes": wf,
        "fetch_x2_validated": read_ok,
        "hbm_bytes_per_launch": s["hbm_bytes_per_launch"], "alg_bytes_per_launch": s["alg_bytes_per_launch"],
        "traffic_over_alg": s["traffic_over_alg"],
        "note": "reads: 2 x FETCH_SIZE = lines read for every shape listed; writes: WRITE_SIZE = "
                "granules written (exact for whole 32/64-B granules; a partly written granule counts whole)"})
json.dump(out, open(sys.argv[1], "w"), indent=1)
for e in out["summaries"]:
    print(e["file"], e["fetch_x2_validated"], round(e["traffic_over_alg"], 4))
