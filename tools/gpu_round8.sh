#!/bin/bash
# GPU pass 8: bench lines for DESIGN.md (64M, 256M, f16 1B, keyed) + kernel stats.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
for spec in "dense64:" "dense256:--keys 268435456 --steps 20" "f16:--workload dense-f16 --steps 20" "keyed:--workload keyed"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 python3 bench.py --no-cpu-baseline $args > gpurun_out/bench_$name.json 2> gpurun_out/bench_$name.err
  rc=$?; echo "bench $name rc=$rc"; cat gpurun_out/bench_$name.json; stop_on_crash $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof256 -o run --output-format csv -- python3 bench.py --keys 268435456 --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/prof256.log 2>&1
rc=$?; echo "rocprof 256 rc=$rc"; stop_on_crash $rc
exit 0
