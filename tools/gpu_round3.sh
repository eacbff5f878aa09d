#!/bin/bash
# GPU pass 3: full GPU test suite (kernels + drop-in harnesses + device-frame harness), bench.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
timeout -k 10 900 python3 -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log; stop_on_crash $rc
timeout -k 10 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 10000000 10 > gpurun_out/e2e_1x1.log 2>&1
rc=$?; echo "e2e rc=$rc"; cat gpurun_out/e2e_1x1.log | tail -3; stop_on_crash $rc
timeout -k 10 300 tests/_dropin/test_kv_app_benchmark -ns 1 -nw 1 > gpurun_out/dropin_bench.log 2>&1
rc=$?; echo "dropin bench rc=$rc"; grep average gpurun_out/dropin_bench.log; stop_on_crash $rc
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; stop_on_crash $rc
exit 0
