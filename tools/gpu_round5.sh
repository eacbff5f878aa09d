#!/bin/bash
# GPU pass 5: tests, keyed bench, pull sweep at 256M.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
timeout -k 10 900 python3 -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log; stop_on_crash $rc
timeout -k 10 300 python3 bench.py --workload keyed --no-cpu-baseline > gpurun_out/bench_keyed.json 2> gpurun_out/bench_keyed.err
rc=$?; echo "bench keyed rc=$rc"; cat gpurun_out/bench_keyed.json; tail -3 gpurun_out/bench_keyed.err; stop_on_crash $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_keyed -o run --output-format csv -- python3 bench.py --workload keyed --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/prof_keyed.log 2>&1
rc=$?; echo "rocprof keyed rc=$rc"; stop_on_crash $rc
timeout -k 10 900 python3 tools/sweep_dense.py 268435456 1,2,4,8 1,3 2,4,8,16 > gpurun_out/sweep256b.log 2>&1
rc=$?; echo "sweep256 rc=$rc"; grep BEST gpurun_out/sweep256b.log; stop_on_crash $rc
exit 0
