#!/usr/bin/env python3
"""The gfx950 HBM counter calibration table from the `pmccalib` passes of
tools/gpu_run.sh over tools/_bin/probe_pmc_shapes (make -C tools).

usage: pmc_calib.py PASS_DIR OUT_JSON

For each access shape: the median per launch of FETCH_SIZE and WRITE_SIZE
(KiB), of the raw request counters (TCC_EA0_RDREQ, _RDREQ_32B, TCC_BUBBLE,
TCC_EA0_WRREQ, _WRREQ_64B), the kernel time, and the bytes the shape is known
to move: 128-B lines read (every line of the 512 MiB region, or a line per
gathered value) and bytes written.  Then
  fetch_factor = line bytes read / (FETCH_SIZE * 1024)
  write_factor = bytes written  / (WRITE_SIZE * 1024)
and the same from the raw counters.  A factor of 2 for every read shape
confirms the guide's "FETCH_SIZE = half the bytes" beyond wide streaming
reads; any other value is the correction that shape needs.
"""
import csv
import glob
import json
import os
import statistics
import sys

MIB = 1 << 20
REGION = 512 * MIB
LINES = REGION // 128
# shape -> (line bytes read, bytes written, what it stands for)
SHAPES = {
    "p_rd16": (REGION, 0, "16-B coalesced loads (the guide's calibrated case)"),
    "p_rd8": (REGION, 0, "8-B coalesced loads (request keys)"),
    "p_rd4": (REGION, 0, "4-B coalesced loads (request values)"),
    "p_rd4_half": (REGION, 0, "4-B loads of every other word (a sparse request's store values)"),
    "p_gather4": (REGION, 0, "one 4-B load per line, random lines (scattered store values)"),
    "p_gather8": (REGION, 0, "one 8-B load per line, random lines (scattered store keys)"),
    "p_wr16": (0, REGION, "16-B coalesced stores (the guide's calibrated case)"),
    "p_wr4": (0, REGION, "4-B coalesced stores"),
    "p_wr4_half": (0, REGION // 2, "4-B stores to every other word (lines half written)"),
    "p_span32": (0, REGION // 2, "32-B spans at a 64-B stride (lines half written)"),
    "p_scatter4": (0, LINES * 4, "one 4-B store per line, random lines"),
    "p_rmw4": (REGION, LINES * 4, "one 4-B load + store per line, random lines (a sparse slot RMW)"),
}


def rows(d):
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            yield from csv.DictReader(fh)


def per_launch(d, counter):
    """{shape: median over launches of the counter (summed over its rows)}"""
    acc = {}
    for r in rows(d):
        k = r["Kernel_Name"].split("(")[0]
        if k not in SHAPES or r["Counter_Name"] != counter:
            continue
        key = (k, r["Dispatch_Id"])
        acc[key] = acc.get(key, 0.0) + float(r["Counter_Value"])
    out = {}
    for (k, _), v in acc.items():
        out.setdefault(k, []).append(v)
    return {k: statistics.median(v) for k, v in out.items()}


def kernel_us(d):
    t = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                k = r["Kernel_Name"].split("(")[0]
                if k in SHAPES:
                    t.setdefault(k, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: statistics.median(v) for k, v in t.items()}


def main():
    d, out = sys.argv[1], sys.argv[2]
    fetch = per_launch(os.path.join(d, "fetch"), "FETCH_SIZE")
    write = per_launch(os.path.join(d, "write"), "WRITE_SIZE")
    rd = per_launch(os.path.join(d, "rdreq"), "TCC_EA0_RDREQ_sum")
    rd32 = per_launch(os.path.join(d, "rdreq"), "TCC_EA0_RDREQ_32B_sum")
    bub = per_launch(os.path.join(d, "rdreq"), "TCC_BUBBLE_sum")
    wr = per_launch(os.path.join(d, "wrreq"), "TCC_EA0_WRREQ_sum")
    wr64 = per_launch(os.path.join(d, "wrreq"), "TCC_EA0_WRREQ_64B_sum")
    us = kernel_us(os.path.join(d, "trace"))
    table = {}
    for k, (rbytes, wbytes, what) in SHAPES.items():
        e = {"shape": what, "line_bytes_read": rbytes, "bytes_written": wbytes,
             "fetch_size_bytes": fetch.get(k, 0) * 1024, "write_size_bytes": write.get(k, 0) * 1024,
             "rdreq": rd.get(k), "rdreq_32b": rd32.get(k), "bubble": bub.get(k), "wrreq": wr.get(k),
             "wrreq_64b": wr64.get(k), "kernel_us": us.get(k)}
        if rbytes and e["fetch_size_bytes"]:
            e["fetch_factor"] = rbytes / e["fetch_size_bytes"]
            e["rdreq_bytes_per_line"] = (e["rdreq"] or 0) / LINES
        if wbytes and e["write_size_bytes"]:
            e["write_factor"] = wbytes / e["write_size_bytes"]
            e["wrreq_per_line"] = (e["wrreq"] or 0) / LINES
        if us.get(k):
            e["moved_tb_s"] = (rbytes + wbytes) / (us[k] * 1e-6) / 1e12
        table[k] = e
    res = {"what": "gfx950 FETCH_SIZE / WRITE_SIZE against known bytes per access shape "
                   "(tools/probe_pmc_shapes.hip, 512 MiB per shape, median of 3 launches)",
           "shapes": table}
    json.dump(res, open(out, "w"), indent=1)
    for k, e in table.items():
        print(f"{k:11s} fetch {e['fetch_size_bytes'] / MIB:9.1f} MiB  factor {e.get('fetch_factor', float('nan')):6.3f}"
              f"  write {e['write_size_bytes'] / MIB:8.1f} MiB  factor {e.get('write_factor', float('nan')):6.3f}"
              f"  rdreq/line {e.get('rdreq_bytes_per_line', float('nan')):5.2f}  32B {e['rdreq_32b']}  bubble {e['bubble']}"
              f"  wrreq {e['wrreq']} 64B {e['wrreq_64b']}  {e['kernel_us'] or 0:8.1f} us")


if __name__ == "__main__":
    main()
