set -u
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
PSG_BENCH_STORE_EXTRA=1 timeout -k 10 300 python3 bench.py --workload keyed --no-cpu-baseline > gpurun_out/bench_sparse.json 2> gpurun_out/bench_sparse.err || exit $?
cat gpurun_out/bench_sparse.json
rm -rf gpurun_out/prof_sparse
PSG_BENCH_STORE_EXTRA=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sparse -o run --output-format csv -- python3 bench.py --workload keyed --no-cpu-baseline --steps 20 > gpurun_out/prof_sparse.json 2>&1 || exit $?
f=$(find gpurun_out/prof_sparse -name "*kernel_stats.csv" | head -1); cut -c1-220 "$f" | head -12
