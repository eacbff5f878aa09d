"""GPU busy time in a rocprofv3 --kernel-trace CSV: the union of kernel
intervals over the last part of the trace (the timed steps), against its wall
span, and the kernels' summed duration (> busy when kernels overlap on
streams).  usage: trace_busy.py trace.csv [fraction_of_trace_to_skip]
Also prints VGPR / scratch per kernel name."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.3
rows = rows[int(len(rows) * skip):]
iv = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
busy, cur_s, cur_e = 0, None, None
for s, e in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
span = max(e for _, e in iv) - iv[0][0]
summed = sum(e - s for s, e in iv)
print(f"kernels {len(iv)}  span {span/1e3:.1f} us  busy {busy/1e3:.1f} us ({busy/span:.3f})  summed {summed/1e3:.1f} us")
seen = {}
for r in rows:
    n = r["Kernel_Name"]
    n = n[:n.find("(")] if "(" in n else n
    seen.setdefault(n, (r["VGPR_Count"], r["Accum_VGPR_Count"], r["Scratch_Size"], r["LDS_Block_Size"]))
for n, (v, a, sc, lds) in seen.items():
    print(f"  {n[-70:]:70s} vgpr {v} agpr {a} scratch {sc} lds {lds}")
