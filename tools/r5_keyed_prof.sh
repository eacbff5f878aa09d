#!/bin/bash
# rocprofv3 kernel stats of bench.py --workload keyed under env variants.
# usage: tools/r5_keyed_prof.sh OUTDIR "VAR=..." ...
out=$1; shift
mkdir -p "$out"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
i=0
for v in "$@"; do
  i=$((i+1))
  env $v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/v$i" -- python3 "$R/bench.py" --workload keyed --steps 20 --warmup 3 --no-cpu-baseline --no-probe256 > "$R/$out/v$i.json" 2>"$R/$out/v$i.err" || exit 1
  echo "[$v]" >> "$R/$out/summary.txt"
  python3 - "$R/$out/v$i" >> "$R/$out/summary.txt" <<'PY'
import csv, glob, sys
for f in glob.glob(sys.argv[1] + "/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if any(k in n for k in ("k_validate", "k_resolve_apply", "k_tile_apply", "k_ident", "k_dense_vec")):
            print(f"  {n[:90]:90s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:8.2f} us")
PY
done
