#!/bin/bash
# GPU pass 16: shared-memory host frames in process mode — drop-in suite, e2e 10M in both
# modes, and the reference's benchmark program in both modes.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
df -h /dev/shm | tail -1
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dropin_gpu.py tests/test_host_runtime.py > gpurun_out/pytest_p16.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_p16.log; stop_on_crash $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 10000000 20 > gpurun_out/e2e_threads_10M.log 2>&1 || exit 1
grep '^{' gpurun_out/e2e_threads_10M.log
PS_VAN_STATS=1 timeout -k 10 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 -procs 10000000 20 > gpurun_out/e2e_procs_10M.log 2>&1 || { tail gpurun_out/e2e_procs_10M.log; exit 1; }
grep '^{\|van stats' gpurun_out/e2e_procs_10M.log
timeout -k 10 300 tests/_dropin/test_kv_app_benchmark -ns 1 -nw 1 > gpurun_out/bench_ref_threads.log 2>&1 || exit 1
grep "average" gpurun_out/bench_ref_threads.log | grep -v "^\["
timeout -k 10 300 tests/_dropin/test_kv_app_benchmark -ns 1 -nw 1 -procs > gpurun_out/bench_ref_procs.log 2>&1 || exit 1
grep "average" gpurun_out/bench_ref_procs.log | grep -v "^\["
ls /dev/shm | grep -c "^psg\." || true
exit 0
