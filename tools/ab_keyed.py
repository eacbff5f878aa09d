"""Summarise a tools/ab.sh output of bench.py keyed lines: value, Push and Pull fractions per variant and round.
usage: ab_keyed.py OUT..."""
import json,re,sys
for f in sys.argv[1:]:
    for l in open(f):
        m=re.match(r"\[(.*?)\] r(\d+) (\{.*)",l)
        if m:
            d=json.loads(m.group(3)); print(f"{m.group(1):45s} {m.group(2)} {d['value']:9.1f} push {d['roofline']['frac']:.4f} pull {d.get('pull_roofline_frac')}")
