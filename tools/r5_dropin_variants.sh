#!/bin/bash
# test_kv_app_benchmark (configs[0]'s harness) under host-path switches, two
# runs each, with the runtime's stage times: where a cold request's time goes.
# usage: tools/r5_dropin_variants.sh <out> [variant ...]  (a variant is an env
# assignment list, "" = defaults; "-procs" in a variant runs process mode)
out=${1:-gpurun_out/r5_dropin_variants.txt}
shift
exe=tests/_dropin/test_kv_app_benchmark
: > "$out"
for v in "$@"; do
  for i in 1 2; do
    echo "=== [$v] run $i" >> "$out"
    mode=""; envs=""
    for w in $v; do if [ "$w" = "-procs" ]; then mode="-procs"; else envs="$envs $w"; fi; done
    env $envs PS_STAGE_TIMES=1 timeout -k 10 120 $exe -ns 1 -nw 1 $mode 2>&1 | grep -E "average time|worker\.|server\.handle|van.recv [0-9]*[1-9]\.[0-9]* ms" | grep -v "^\[W" >> "$out" || exit 1
  done
done
