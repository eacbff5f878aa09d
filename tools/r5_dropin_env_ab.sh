#!/bin/bash
# The drop-in HBM line (kv_bench_dropin, N = 1, threads and processes) under
# env variants, interleaved over rounds.
# usage: tools/r5_dropin_env_ab.sh OUT rounds variant...   ("" = defaults)
out=${1:-gpurun_out/r5_dropin_env_ab.txt}
rounds=${2:-2}
shift 2
: > "$out"
for r in $(seq 1 $rounds); do
  for v in "$@"; do
    for mode in "" "-procs"; do
      line=$(env $v timeout -k 10 120 tests/_bin/kv_bench_dropin -ns 1 -nw 1 $mode 10000000 30 5 0 2>/dev/null | grep rank) || exit 1
      echo "[$v] [$mode] $line" >> "$out"
    done
  done
done
