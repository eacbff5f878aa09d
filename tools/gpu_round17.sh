#!/bin/bash
# GPU pass 17 (evidence refresh): GPU suite, smoke, default bench line, rocprof kernel stats of the
# default / keyed / 256M bench, PMC HBM traffic of the keyed request and the 256M Push, and the
# reference's benchmark program in both launch modes.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; stop_on_crash $rc; return $rc; }
step 900 python3 -u -m pytest -q --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/pytest_final.log 2>&1
echo "pytest rc=$?"; tail -2 gpurun_out/pytest_final.log
step 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/smoke.log
step 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; echo "bench rc=$?"; cat gpurun_out/bench.json
step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/prof64.json 2>&1; echo "prof64 rc=$?"
step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/profkeyed -o run --output-format csv -- python3 bench.py --workload keyed --no-cpu-baseline > gpurun_out/profkeyed.json 2>&1; echo "profkeyed rc=$?"
step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof256 -o run --output-format csv -- python3 bench.py --keys 268435456 --no-cpu-baseline --steps 20 > gpurun_out/prof256.json 2>&1; echo "prof256 rc=$?"
K="--workload keyed --no-cpu-baseline --check 0 --steps 5 --warmup 1"
step 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_kf -o run -- python3 bench.py $K > gpurun_out/pmc_kf.log 2>&1; echo "pmc kf rc=$?"
step 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_kw -o run -- python3 bench.py $K > gpurun_out/pmc_kw.log 2>&1; echo "pmc kw rc=$?"
python3 tools/pmc_summary.py gpurun_out/pmc_kf gpurun_out/pmc_kw "k_tile_windows|k_resolve_apply<0, 1>" 10000000 gpurun_out/pmc_keyed_push_traffic.json 28
D="--keys 268435456 --no-cpu-baseline --check 0 --steps 5 --warmup 1"
step 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_df -o run -- python3 bench.py $D > gpurun_out/pmc_df.log 2>&1; echo "pmc df rc=$?"
step 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_dw -o run -- python3 bench.py $D > gpurun_out/pmc_dw.log 2>&1; echo "pmc dw rc=$?"
python3 tools/pmc_summary.py gpurun_out/pmc_df gpurun_out/pmc_dw "k_dense_vec<0, 1," 268435456 gpurun_out/pmc_push256_traffic.json 12
step 300 tests/_dropin/test_kv_app_benchmark -ns 1 -nw 1 > gpurun_out/bench_ref_threads.log 2>&1; grep average gpurun_out/bench_ref_threads.log | grep -v "^\["
step 300 tests/_dropin/test_kv_app_benchmark -ns 1 -nw 1 -procs > gpurun_out/bench_ref_procs.log 2>&1; grep average gpurun_out/bench_ref_procs.log | grep -v "^\["
exit 0
