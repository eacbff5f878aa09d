#!/bin/bash
# GPU pass 18: background pinning of host blocks — drop-in tests, e2e 10M (both modes), reference benchmark.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; stop_on_crash $rc; return $rc; }
step 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dropin_gpu.py > gpurun_out/pytest_p18.log 2>&1 || { tail -20 gpurun_out/pytest_p18.log; exit 1; }
tail -1 gpurun_out/pytest_p18.log
step 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 10000000 20 > gpurun_out/e2e_threads_10M.log 2>&1 || exit 1
grep '^{' gpurun_out/e2e_threads_10M.log
step 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 -procs 10000000 20 > gpurun_out/e2e_procs_10M.log 2>&1 || exit 1
grep '^{' gpurun_out/e2e_procs_10M.log
for i in 1 2; do
step 300 tests/_dropin/test_kv_app_benchmark -ns 1 -nw 1 > gpurun_out/bench_ref_threads.log 2>&1 || exit 1
grep average gpurun_out/bench_ref_threads.log | grep -v "^\["
done
step 300 tests/_dropin/test_kv_app_benchmark -ns 1 -nw 1 -procs > gpurun_out/bench_ref_procs.log 2>&1 || exit 1
grep average gpurun_out/bench_ref_procs.log | grep -v "^\["
exit 0
