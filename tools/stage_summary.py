"""Per-stage host times from PS_STAGE_TIMES=1 output ("[stage] node=N name T ms
B MB" lines, internal/stage_time.h): count, mean, median and 90th percentile
per (role, stage), skipping the first `skip` lines of each (the warm-up).
usage: stage_summary.py LOG [skip]"""
import collections
import re
import statistics
import sys

skip = int(sys.argv[2]) if len(sys.argv) > 2 else 20
by = collections.defaultdict(list)
pat = re.compile(r"\[stage\] node=(\d+) (\S+) ([\d.]+) ms")
for line in open(sys.argv[1], errors="replace"):
    m = pat.search(line)
    if m:
        node, name, ms = int(m.group(1)), m.group(2), float(m.group(3))
        role = "server" if node % 2 == 0 and node > 1 else "worker"
        by[(role, name)].append(ms)
for (role, name), v in sorted(by.items()):
    v = v[skip:] if len(v) > skip * 2 else v
    if not v:
        continue
    q = sorted(v)
    print(f"{role:6s} {name:34s} n {len(v):5d}  mean {statistics.mean(v) * 1e3:8.1f} us  "
          f"p50 {q[len(q) // 2] * 1e3:8.1f}  p90 {q[int(len(q) * 0.9)] * 1e3:8.1f}")
