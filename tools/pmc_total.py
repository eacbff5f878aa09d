#!/usr/bin/env python3
"""HBM traffic per step of a whole job (every kernel of every process), from
rocprofv3 --pmc passes of the same job at two step counts: the difference
cancels the start-up, warm-up and check kernels (inserts, searches, the
parity check), leaving (hi - lo) timed steps of steady-state requests.

usage: pmc_total.py FETCH_LO WRITE_LO FETCH_HI WRITE_HI STEPS_LO STEPS_HI ALG_BYTES_PER_STEP OUT_JSON [NOTE]

Each argument directory holds the counter_collection CSVs of one pass (one
file per process).  gfx950 correction as tools/pmc_summary.py: 2 x FETCH_SIZE
is the bytes of the 128-B lines read, WRITE_SIZE the 32/64-B write granules
(profiles/r5_pmc_calibration.json); KiB -> bytes."""
import csv
import glob
import json
import os
import sys


def total(d, counter):
    s, n = 0.0, 0
    by = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                key = (f, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                by[key] = by.get(key, 0.0) + float(row["Counter_Value"])
    for v in by.values():
        s += v
        n += 1
    return s, n


def main():
    flo, wlo, fhi, whi = sys.argv[1:5]
    slo, shi = int(sys.argv[5]), int(sys.argv[6])
    alg = int(sys.argv[7])
    out = sys.argv[8]
    note = sys.argv[9] if len(sys.argv) > 9 else ""
    (f0, n0), (w0, _) = total(flo, "FETCH_SIZE"), total(wlo, "WRITE_SIZE")
    (f1, n1), (w1, _) = total(fhi, "FETCH_SIZE"), total(whi, "WRITE_SIZE")
    steps = shi - slo
    hbm = ((2 * f1 + w1) - (2 * f0 + w0)) * 1024 / steps
    res = {"what": "HBM bytes per timed step of the whole job (every kernel): passes at %d and %d steps, "
                   "differenced" % (slo, shi),
           "note": note,
           "dispatches": [n0, n1],
           "correction": "gfx950: FETCH_SIZE x2 = 128-B lines read, WRITE_SIZE x1 = 32/64-B write granules "
                         "(profiles/r5_pmc_calibration.json); KiB -> bytes",
           "hbm_bytes_per_step": int(hbm), "alg_bytes_per_step": alg, "traffic_over_alg": hbm / alg}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
