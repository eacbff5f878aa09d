#!/bin/bash
# GPU pass 19: single-server slice shortcut — GPU suite, keyed bench, e2e 10M / 100K.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; stop_on_crash $rc; return $rc; }
step 900 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/pytest_p19.log 2>&1 || { tail -30 gpurun_out/pytest_p19.log; exit 1; }
tail -1 gpurun_out/pytest_p19.log
step 300 python3 bench.py --workload keyed --no-cpu-baseline > gpurun_out/bench_keyed.json 2>gpurun_out/bench_keyed.err || exit 1
cat gpurun_out/bench_keyed.json
for n in 100000 10000000; do
step 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 $n 50 > gpurun_out/e2e.log 2>&1 || exit 1
echo "n=$n $(grep '^{' gpurun_out/e2e.log)"
done
exit 0
