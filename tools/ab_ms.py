"""Summarise a tools/ab.sh output of kv_bench_dropin lines: per variant, the
step time of each round (max over the workers' lines).
usage: ab_ms.py OUT..."""
import collections
import json
import re
import sys

for f in sys.argv[1:]:
    d = collections.defaultdict(list)
    for line in open(f):
        m = re.match(r"\[(.*?)\] r(\d+) (\{.*)", line)
        if m:
            d[(m.group(1), m.group(2))].append(json.loads(m.group(3))["ms_per_step"])
    agg = collections.defaultdict(list)
    for (v, _), ms in d.items():
        agg[v].append(max(ms))
    print(f)
    for v, ms in agg.items():
        print(f"  {v or '(defaults)':32s} {' '.join('%.3f' % x for x in ms)}   median {sorted(ms)[len(ms) // 2]:.3f}")
