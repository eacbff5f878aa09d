#!/bin/bash
# GPU pass 6: tests, keyed bench + profile, e2e harness (pinned host frames).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
timeout -k 10 900 python3 -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log; stop_on_crash $rc
timeout -k 10 300 python3 bench.py --workload keyed --no-cpu-baseline > gpurun_out/bench_keyed.json 2> gpurun_out/bench_keyed.err
rc=$?; echo "bench keyed rc=$rc"; cat gpurun_out/bench_keyed.json; stop_on_crash $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_keyed -o run --output-format csv -- python3 bench.py --workload keyed --no-cpu-baseline --steps 10 --warmup 2 > gpurun_out/prof_keyed.log 2>&1
rc=$?; echo "rocprof keyed rc=$rc"; stop_on_crash $rc
timeout -k 10 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 10000000 10 > gpurun_out/e2e_1x1.log 2>&1
rc=$?; echo "e2e rc=$rc"; tail -1 gpurun_out/e2e_1x1.log; stop_on_crash $rc
timeout -k 10 300 tests/_dropin/test_kv_app_benchmark -ns 1 -nw 1 > gpurun_out/dropin_bench.log 2>&1
rc=$?; echo "dropin bench rc=$rc"; grep -v '^\[' gpurun_out/dropin_bench.log; stop_on_crash $rc
exit 0
