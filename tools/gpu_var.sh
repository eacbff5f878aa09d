#!/bin/bash
# Variance check: the 256M bench repeated with Pull U=1 (default) and U=2 interleaved.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for i in 1 2 3; do
  for u in 1 2; do
    PSG_DENSE_PULL_UNROLL=$u timeout -k 10 120 python3 bench.py --keys 268435456 --no-cpu-baseline --check 0 --steps 50 > gpurun_out/v.json 2>/dev/null || exit $?
    python3 -c "import json;d=json.load(open('gpurun_out/v.json'));print('U=$u', d['value'], d['roofline']['frac'], d['pull_roofline_frac'])"
  done
done
