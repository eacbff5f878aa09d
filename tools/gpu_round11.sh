#!/bin/bash
# GPU pass 11: xGMI tests (incl. the shared-GPU N=2 bench with checksum verification);
# bench at 256M f32 and 1B f16 with the new Pull launch shape.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_xgmi.py > gpurun_out/pytest_p11.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_p11.log; stop_on_crash $rc
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python3 bench.py --keys 268435456 --no-cpu-baseline > gpurun_out/bench_256M.json 2> gpurun_out/bench_256M.err
rc=$?; echo "bench256 rc=$rc"; cat gpurun_out/bench_256M.json; stop_on_crash $rc
timeout -k 10 300 python3 bench.py --workload dense-f16 --no-cpu-baseline > gpurun_out/bench_f16.json 2> gpurun_out/bench_f16.err
rc=$?; echo "benchf16 rc=$rc"; cat gpurun_out/bench_f16.json; stop_on_crash $rc
timeout -k 10 300 python3 bench.py --no-cpu-baseline > gpurun_out/bench_64M.json 2> gpurun_out/bench_64M.err
rc=$?; echo "bench64 rc=$rc"; cat gpurun_out/bench_64M.json; stop_on_crash $rc
exit 0
