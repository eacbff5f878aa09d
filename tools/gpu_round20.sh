#!/bin/bash
# GPU pass 20: f16 1B launch sweep (Push with Pull pinned to its default; then Pull alone).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export SWEEP_ARGS="--workload dense-f16"
PSG_DENSE_PULL_UNROLL=1 PSG_DENSE_PULL_NT=3 PSG_DENSE_PULL_BPC=4 timeout -k 10 900 python3 tools/sweep_dense.py 1073741824 1,2,4 1,3 2,4,8 > gpurun_out/sweep_f16_push.log 2>&1 || { tail gpurun_out/sweep_f16_push.log; exit 1; }
tail -1 gpurun_out/sweep_f16_push.log
timeout -k 10 900 python3 tools/sweep_dense.py 1073741824 1,2,4 1,2,3 2,4,8 pull > gpurun_out/sweep_f16_pull.log 2>&1 || { tail gpurun_out/sweep_f16_pull.log; exit 1; }
tail -1 gpurun_out/sweep_f16_pull.log
exit 0
