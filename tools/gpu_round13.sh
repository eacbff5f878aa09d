#!/bin/bash
# GPU pass 13: RCCL communicator bootstrapped through the control plane (both modes),
# then the whole GPU suite once.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_dropin_gpu.py -k "rccl_comm" > gpurun_out/pytest_p13a.log 2>&1
rc=$?; echo "comm rc=$rc"; tail -5 gpurun_out/pytest_p13a.log; stop_on_crash $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/pytest_p13.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -5 gpurun_out/pytest_p13.log; stop_on_crash $rc
exit 0
