#!/bin/bash
# bench.py --workload keyed lines under env variants, interleaved over rounds.
# usage: tools/r5_keyed_env_ab.sh OUT rounds variant...   ("" = defaults)
out=${1:-gpurun_out/r5_keyed_env_ab.txt}
rounds=${2:-2}
shift 2
: > "$out"
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    line=$(env $v timeout -k 10 300 python bench.py --workload keyed --steps 30 --warmup 5 --no-cpu-baseline --no-probe256 2>/dev/null | tail -1) || exit 1
    python3 - "$v" "$line" >> "$out" <<'PY'
import json, sys
v, line = sys.argv[1], sys.argv[2]
d = json.loads(line)
r = d.get("roofline") or {}
print(f"[{v or 'default'}] value {d['value']:.1f} GB/s  push_frac {r.get('frac')}  pull_frac {d.get('pull_roofline_frac')}  parity {d.get('parity_check')}")
PY
  done
done
