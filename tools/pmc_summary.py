#!/usr/bin/env python3
"""Per-launch HBM traffic of one kernel from two rocprofv3 --pmc passes.

usage: pmc_summary.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR KEYS OUT_JSON [ALG_BYTES_PER_KEY]

KERNEL_SUBSTR may name several kernels separated by '|' (the launches of one
request): their per-launch medians are added.  ALG_BYTES_PER_KEY defaults to
12 (the dense Push).

FETCH_DIR / WRITE_DIR are the -d output directories of
  rocprofv3 --pmc FETCH_SIZE --output-format csv ...
  rocprofv3 --pmc WRITE_SIZE --output-format csv ...
(separate passes: FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2, MI355X_MICROARCH.md
"rocprofv3 PMC slots").  Units are KiB.  gfx950 correction, calibrated for
every access shape the store kernels use (tools/probe_pmc_shapes.hip,
profiles/r5_pmc_calibration.json): a read costs one TCC_EA0_RDREQ per 128-B
line it touches and FETCH_SIZE counts 64 B of it — 16-, 8- and 4-B coalesced
loads, every-other-word loads and 4- / 8-B gathers of one value per line alike
— so 2 x FETCH_SIZE is the bytes of the lines read; WRITE_SIZE counts each
write request's granule (64 B when whole 64-B halves are written, else 32 B):
the bytes written for whole granules, the granules touched for partial ones
(a lone 4-B store counts 32 B, a half-written 64-B half counts 64).
  hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024   per launch (median).
"""
import csv
import glob
import json
import os
import statistics
import sys


def read_counter(d, kernel_sub, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if kernel_sub not in row.get("Kernel_Name", ""):
                    continue
                if row.get("Counter_Name") != counter:
                    continue
                key = row.get("Dispatch_Id") or row.get("Correlation_Id") or str(len(vals))
                vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return list(vals.values())


def main():
    fdir, wdir, ksubs, keys, out = sys.argv[1:6]
    per_key = int(sys.argv[6]) if len(sys.argv) > 6 else 12
    f = w = 0.0
    launches = []
    for ksub in ksubs.split("|"):
        fetch = read_counter(fdir, ksub, "FETCH_SIZE")
        write = read_counter(wdir, ksub, "WRITE_SIZE")
        if not fetch or not write:
            print("no counter rows found for", ksub, len(fetch), len(write))
            sys.exit(1)
        f += statistics.median(fetch)
        w += statistics.median(write)
        launches.append([len(fetch), len(write)])
    hbm = (2 * f + w) * 1024
    alg = per_key * int(keys)
    res = {
        "kernel": ksubs,
        "keys": int(keys),
        "fetch_size_kib_median": f,
        "write_size_kib_median": w,
        "launches": launches,
        "correction": "gfx950: FETCH_SIZE x2 = 128-B lines read, WRITE_SIZE x1 = 32/64-B write granules; "
                      "validated per access shape (profiles/r5_pmc_calibration.json); KiB -> bytes",
        "hbm_bytes_per_launch": int(hbm),
        "alg_bytes_per_launch": alg,
        "traffic_over_alg": hbm / alg,
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
