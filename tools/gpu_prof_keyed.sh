#!/bin/bash
# rocprofv3 kernel stats of the keyed bench (fused SORTED resolve+apply).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_keyed -o run --output-format csv -- python3 bench.py --workload keyed --no-cpu-baseline --steps 20 > gpurun_out/prof_keyed.json 2> gpurun_out/prof_keyed.err
rc=$?; echo "rc=$rc"; cat gpurun_out/prof_keyed.json
f=$(find gpurun_out/prof_keyed -name "*kernel_stats.csv" | head -1); echo "$f"; cut -c1-220 "$f" | head -20
