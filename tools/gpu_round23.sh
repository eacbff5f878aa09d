#!/bin/bash
# GPU pass 23 (evidence refresh): GPU suite, smoke, default bench line with the CPU
# baseline and its rocprof kernel stats, the keyed bench line, and the C++ API
# end to end (10 M keys, threads and processes).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; stop_on_crash $rc; return $rc; }
rm -rf gpurun_out/prof64
step 600 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/pytest_final.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/pytest_final.log
step 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/smoke.log
step 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; echo "bench rc=$?"; cat gpurun_out/bench.json
step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/prof64.json 2>&1; echo "prof64 rc=$?"
step 300 python3 bench.py --workload keyed --no-cpu-baseline > gpurun_out/bench_keyed.json 2> gpurun_out/bench_keyed.err; echo "keyed rc=$?"; cat gpurun_out/bench_keyed.json
step 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 10000000 20 > gpurun_out/e2e_threads_10M.log 2>&1; echo "e2e threads rc=$?"; head -1 gpurun_out/e2e_threads_10M.log
step 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 -procs 10000000 20 > gpurun_out/e2e_procs_10M.log 2>&1; echo "e2e procs rc=$?"; head -1 gpurun_out/e2e_procs_10M.log
