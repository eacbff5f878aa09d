#!/bin/bash
# rocprofv3 kernel stats of bench.py --workload keyed under env variants (one
# directory per variant) plus the bench line's keyed_paths.
# usage: tools/r5_keyed_prof_env.sh OUTDIR variant...
out=$1; shift
R=$GRAFT_REPO_ROOT
mkdir -p "$R/$out"
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/v$i" -- python3 "$R/bench.py" --workload keyed --steps 20 --warmup 3 --no-cpu-baseline --no-probe256 > "$R/$out/v$i.json" 2>"$R/$out/v$i.err" || exit 1
  echo "v$i: $v" >> "$R/$out/variants.txt"
done
