#!/bin/bash
# GPU pass 10: checksum + shared-GPU N=2 bench test; Pull-only launch sweeps at 64M / 256M.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k checksum tests/test_xgmi.py > gpurun_out/pytest_p10.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -12 gpurun_out/pytest_p10.log; stop_on_crash $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python3 tools/sweep_dense.py 268435456 1,2,4,8 1,2,3,0 2,4,8 pull > gpurun_out/sweep_pull_256M.log 2>&1
rc=$?; echo "sweep256 rc=$rc"; tail -2 gpurun_out/sweep_pull_256M.log; stop_on_crash $rc
timeout -k 10 600 python3 tools/sweep_dense.py 67108864 1,2,4 1,2,3,0 2,4,8 pull > gpurun_out/sweep_pull_64M.log 2>&1
rc=$?; echo "sweep64 rc=$rc"; tail -2 gpurun_out/sweep_pull_64M.log; stop_on_crash $rc
exit 0
