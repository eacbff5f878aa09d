#!/bin/bash
# GPU pass 2: parity tests, dense-kernel sweep at 64M and 256M, PMC traffic, kernel stats.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
timeout -k 10 900 python3 -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; stop_on_crash $rc
timeout -k 10 600 python3 tools/sweep_dense.py 67108864 1,2,4 1,2,3 1,2,4,8 > gpurun_out/sweep64.log 2>&1
rc=$?; echo "sweep64 rc=$rc"; grep BEST gpurun_out/sweep64.log; stop_on_crash $rc
timeout -k 10 600 python3 tools/sweep_dense.py 268435456 1,2,4 1,2,3 2,4,8 > gpurun_out/sweep256.log 2>&1
rc=$?; echo "sweep256 rc=$rc"; grep BEST gpurun_out/sweep256.log; stop_on_crash $rc
B="bench.py --no-cpu-baseline --check 0 --steps 5 --warmup 1"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 $B > gpurun_out/pmc_fetch.log 2>&1
rc=$?; echo "pmc fetch rc=$rc"; stop_on_crash $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 $B > gpurun_out/pmc_write.log 2>&1
rc=$?; echo "pmc write rc=$rc"; stop_on_crash $rc
python3 tools/pmc_summary.py gpurun_out/pmc_fetch gpurun_out/pmc_write "k_dense_vec<0, 1," 67108864 gpurun_out/pmc_push_traffic.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; stop_on_crash $rc
exit 0
