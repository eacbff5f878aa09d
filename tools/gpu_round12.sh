#!/bin/bash
# GPU pass 12: process mode (TCP control plane, hipIpc HBM frames) on the MI355X:
# drop-in tests incl. -procs, then the 10M-key e2e harness in both modes.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_dropin_gpu.py tests/test_host_runtime.py > gpurun_out/pytest_p12.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|ERROR" gpurun_out/pytest_p12.log | tail -40; stop_on_crash $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 10000000 20 > gpurun_out/e2e_threads_10M.log 2>&1
rc=$?; echo "e2e threads rc=$rc"; cat gpurun_out/e2e_threads_10M.log | tail -3; stop_on_crash $rc
timeout -k 10 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 -procs 10000000 20 > gpurun_out/e2e_procs_10M.log 2>&1
rc=$?; echo "e2e procs rc=$rc"; cat gpurun_out/e2e_procs_10M.log | tail -3; stop_on_crash $rc
exit 0
