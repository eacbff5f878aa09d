#!/bin/bash
# GPU pass 9 (re-entry check): tests, smoke, default bench line.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
timeout -k 10 900 python3 -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log; stop_on_crash $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/smoke.log; stop_on_crash $rc
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; stop_on_crash $rc
exit 0
