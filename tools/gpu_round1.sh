#!/bin/bash
# First GPU pass: smoke, GPU parity tests, bench, rocprof stats, dense sweep.
# Every GPU step has its own time limit; a crash/timeout code stops the script.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() {  # $1 = exit code of the previous GPU step
  case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac
}
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; stop_on_crash $rc
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; stop_on_crash $rc
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; stop_on_crash $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; stop_on_crash $rc
timeout -k 10 600 python3 tools/sweep_dense.py > gpurun_out/sweep.log 2>&1
rc=$?; echo "sweep rc=$rc"; tail -3 gpurun_out/sweep.log; stop_on_crash $rc
exit 0
