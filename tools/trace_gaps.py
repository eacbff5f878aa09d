"""Print the last kernels of a rocprofv3 --kernel-trace CSV in start order,
with each kernel's duration and the idle gap before it (us)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
last = int(sys.argv[2]) if len(sys.argv) > 2 else 24
prev = None
out = []
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    out.append((r["Kernel_Name"][:58], (e - s) / 1e3, (s - prev) / 1e3 if prev else 0.0, r["Grid_Size_X"]))
    prev = e
for name, dur, gap, grid in out[-last:]:
    print(f"{name:58s} dur {dur:8.2f}  gap {gap:8.2f}  grid {grid}")
