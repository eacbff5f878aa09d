#!/bin/bash
# GPU pass 21 (final evidence of the session): default bench line (with the CPU baseline) and its
# rocprof kernel stats, 256M and f16 1B lines, and the shared-GPU N=2 bench line.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
step() { local t=$1; shift; timeout -k 10 $t "$@"; local rc=$?; stop_on_crash $rc; return $rc; }
step 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { cat gpurun_out/bench.err | tail; exit 1; }
cat gpurun_out/bench.json
step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof64.json 2>&1 || exit 1
step 300 python3 bench.py --keys 268435456 --no-cpu-baseline > gpurun_out/bench_256M.json 2>/dev/null || exit 1
cat gpurun_out/bench_256M.json
step 300 python3 bench.py --workload dense-f16 --no-cpu-baseline > gpurun_out/bench_f16.json 2>/dev/null || exit 1
cat gpurun_out/bench_f16.json
PSG_BENCH_SHARE_GPU=1 step 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/bench_share2.json 2> gpurun_out/bench_share2.err || { tail gpurun_out/bench_share2.err; exit 1; }
grep '^{' gpurun_out/bench_share2.json
exit 0
