#!/bin/bash
# Keyed Push on the general path with and without stretch tiles (round 5,
# k_validate_windows chunk_ok): bench.py --workload keyed lines, interleaved.
# usage: tools/r5_keyed_ab.sh OUT [rounds]
out=${1:-gpurun_out/r5_keyed_ab.txt}
rounds=${2:-2}
: > "$out"
for r in $(seq 1 $rounds); do
  for v in "PSG_RA_IDENT=0" "PSG_RA_IDENT=0 PSG_RA_MIDENT=0" "PSG_BENCH_STRETCHES=16" "PSG_BENCH_STRETCHES=16 PSG_RA_MIDENT=0" \
           "PSG_BENCH_STRETCHES=64" "PSG_BENCH_STRETCHES=64 PSG_RA_MIDENT=0" "PSG_BENCH_STORE_EXTRA=1" "PSG_BENCH_STORE_EXTRA=1 PSG_RA_MIDENT=0" ""; do
    line=$(env $v timeout -k 10 300 python bench.py --workload keyed --steps 30 --warmup 5 --no-cpu-baseline --no-probe256 2>/dev/null | tail -1) || exit 1
    python3 - "$v" "$line" >> "$out" <<'PY'
import json, sys
v, line = sys.argv[1], sys.argv[2]
d = json.loads(line)
r = d.get("roofline") or {}
print(f"[{v or 'default'}] value {d['value']:.1f} GB/s  push_frac {r.get('frac')}  pull_frac {d.get('pull_roofline_frac')}  "
      f"paths {d.get('keyed_paths')}  parity {d.get('parity_check')}")
PY
  done
done
