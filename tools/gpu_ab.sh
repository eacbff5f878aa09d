#!/bin/bash
# A/B: bench.py (2 events per step) vs bench_prev.py (3 events per step), interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3; do for b in bench_prev.py bench.py; do
  timeout -k 10 120 python3 $b --no-cpu-baseline --check 0 > gpurun_out/ab.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$b', d['value'], d['ms_per_step'], d['push_ms'], d['pull_ms'])"
done; done
