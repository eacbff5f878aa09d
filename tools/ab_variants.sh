# kernel traces of the keyed bench with experimental builds of libpsgpu (abtmp/lib_*.so)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in "$@"; do
  rm -rf gpurun_out/v_$v
  PSG_SYNC_POLL=${POLL:-1} PSG_LIB=$PWD/abtmp/lib_$v.so timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/v_$v -o run -- python3 bench.py --workload keyed --no-cpu-baseline --no-probe256 --steps 10 --warmup 2 > gpurun_out/v_$v.json 2>&1; echo "$v rc=$?"
  python3 tools/trace_gaps.py gpurun_out/v_$v/run_kernel_trace.csv 7 | head -4
done
