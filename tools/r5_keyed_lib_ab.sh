#!/bin/bash
# Keyed Push lines under two builds of libpsgpu (PSG_LIB), interleaved: the
# candidate (lib/libpsgpu.so) against a baseline build (tools/_bin/libpsgpu_head.so).
# usage: tools/r5_keyed_lib_ab.sh OUT [rounds] [variant ...]
out=${1:-gpurun_out/r5_keyed_lib_ab.txt}
rounds=${2:-2}
shift 2
vars=("$@")
[ ${#vars[@]} -eq 0 ] && vars=("PSG_RA_IDENT=0" "PSG_BENCH_STRETCHES=16" "PSG_BENCH_STRETCHES=64")
: > "$out"
for r in $(seq 1 $rounds); do
  for v in "${vars[@]}"; do
    for lib in tools/_bin/libpsgpu_head.so parameter-server_amd/lib/libpsgpu.so; do
      line=$(env $v PSG_LIB=$lib timeout -k 10 300 python bench.py --workload keyed --steps 30 --warmup 5 --no-cpu-baseline --no-probe256 2>/dev/null | tail -1) || exit 1
      python3 - "$v" "$lib" "$line" >> "$out" <<'PY'
import json, sys
v, lib, line = sys.argv[1], sys.argv[2], sys.argv[3]
d = json.loads(line)
r = d.get("roofline") or {}
print(f"[{v or 'default'}] {lib.split('/')[-1]:20s} value {d['value']:.1f} GB/s  push_frac {r.get('frac')}  "
      f"pull_frac {d.get('pull_roofline_frac')}  parity {d.get('parity_check')}")
PY
    done
  done
done
