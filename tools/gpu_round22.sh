#!/bin/bash
# GPU pass 22: keyed (SORTED store) evidence after the LDS-DMA window staging:
# bench line, rocprof kernel stats, PMC HBM traffic of the Push request.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; stop_on_crash $rc; return $rc; }
rm -rf gpurun_out/profkeyed gpurun_out/pmc_kf gpurun_out/pmc_kw
step 600 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/pytest_final.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/pytest_final.log
step 300 python3 bench.py --workload keyed --no-cpu-baseline > gpurun_out/bench_keyed.json 2> gpurun_out/bench_keyed.err; echo "bench rc=$?"; cat gpurun_out/bench_keyed.json
step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profkeyed -o run --output-format csv -- python3 bench.py --workload keyed --no-cpu-baseline > gpurun_out/profkeyed.json 2>&1; echo "profkeyed rc=$?"
K="--workload keyed --no-cpu-baseline --check 0 --steps 5 --warmup 1"
step 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_kf -o run -- python3 bench.py $K > gpurun_out/pmc_kf.log 2>&1; echo "pmc kf rc=$?"
step 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_kw -o run -- python3 bench.py $K > gpurun_out/pmc_kw.log 2>&1; echo "pmc kw rc=$?"
python3 tools/pmc_summary.py gpurun_out/pmc_kf gpurun_out/pmc_kw "k_tile_windows|k_resolve_apply<0, 1," 10000000 gpurun_out/pmc_keyed_push_traffic.json 28
python3 tools/pmc_summary.py gpurun_out/pmc_kf gpurun_out/pmc_kw "k_resolve_apply<0, 1," 10000000 gpurun_out/pmc_keyed_apply_traffic.json 28
cat gpurun_out/pmc_keyed_push_traffic.json gpurun_out/pmc_keyed_apply_traffic.json | grep -E "traffic_over|hbm_bytes"
