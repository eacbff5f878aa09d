#!/bin/bash
# GPU pass 15: e2e request latency with spin-then-block hand-offs (PS_SPIN_US) vs plain blocking.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_dropin_gpu.py > gpurun_out/pytest_p15.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_p15.log; stop_on_crash $rc
[ $rc -ne 0 ] && exit $rc
for n in 100000 10000000; do for sp in 0 50; do
  PS_SPIN_US=$sp timeout -k 10 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 $n 50 > gpurun_out/e2e.log 2>&1 || { tail gpurun_out/e2e.log; exit 1; }
  echo "n=$n spin=$sp threads $(grep '^{' gpurun_out/e2e.log)"
  PS_SPIN_US=$sp timeout -k 10 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 -procs $n 50 > gpurun_out/e2e.log 2>&1 || { tail gpurun_out/e2e.log; exit 1; }
  echo "n=$n spin=$sp procs $(grep '^{' gpurun_out/e2e.log)"
done; done
exit 0
