#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE) over bench.py --workload keyed under an
# env variant, summarised for the Push's two kernels by tools/pmc_summary.py.
# usage: tools/r5_pmc_keyed.sh OUTDIR NAME "ENV..." KERNELS
set -e
out=$1; name=$2; vars=$3; kernels=$4
R=$GRAFT_REPO_ROOT
mkdir -p "$R/$out"
cd /tmp && export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  env $vars timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d "$R/$out/$name.$c" -- python3 "$R/bench.py" --workload keyed --steps 10 --warmup 3 --no-cpu-baseline --no-probe256 > /dev/null
done
python3 "$R/tools/pmc_summary.py" "$R/$out/$name.FETCH_SIZE" "$R/$out/$name.WRITE_SIZE" "$kernels" 10000000 "$R/$out/$name.json" 28
