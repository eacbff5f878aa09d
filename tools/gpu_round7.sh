#!/bin/bash
# GPU pass 7: tests (incl. multi-process xGMI exchange), the N>1 bench path on
# one GPU (shared-GPU test mode, xGMI exchange), bench N=1.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
timeout -k 10 900 python3 -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log; stop_on_crash $rc
PSG_BENCH_SHARE_GPU=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 10 --warmup 2 > gpurun_out/bench_share2.json 2> gpurun_out/bench_share2.err
rc=$?; echo "bench shared-GPU N=2 rc=$rc"; cat gpurun_out/bench_share2.json; tail -5 gpurun_out/bench_share2.err; stop_on_crash $rc
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; stop_on_crash $rc
exit 0
