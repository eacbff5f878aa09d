#!/bin/bash
# configs[0]'s own harness (the reference's test_kv_app_benchmark.cpp, built
# unmodified) timed with the runtime's host stage timer (PS_STAGE_TIMES=1,
# internal/stage_time.h), threads and processes, ns = nw = 1, three runs each.
# usage: tools/r5_dropin_stages.sh <out file>
out=${1:-gpurun_out/r5_dropin_stages.txt}
exe=tests/_dropin/test_kv_app_benchmark
: > "$out"
for mode in threads procs; do
  for i in 1 2 3; do
    echo "=== $mode run $i" >> "$out"
    extra=""; [ $mode = procs ] && extra="-procs"
    PS_STAGE_TIMES=1 timeout -k 10 120 $exe -ns 1 -nw 1 $extra 2>&1 | grep -E "average time|^\[stage\]" | grep -v "^\[W" >> "$out" || exit 1
  done
done
