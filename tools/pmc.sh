#!/bin/bash
# HBM traffic of one kernel family by PMC (MI355X_MICROARCH.md's recipe): two
# rocprofv3 passes of the same command, FETCH_SIZE then WRITE_SIZE (one
# counter set a pass: FETCH_SIZE takes 3 TCC slots, WRITE_SIZE 2), each under
# its own SIGKILL time limit, summarised per launch against the algorithmic
# bytes by tools/pmc_summary.py (gfx950 factors: profiles/r5_pmc_calibration.json).
# usage (on the box):
#   bash tools/pmc.sh OUTDIR NAME 'KERNEL_REGEX' UNITS BYTES_PER_UNIT COMMAND...
# e.g. the strided run's passes of the drop-in line at N = 4:
#   bash tools/pmc.sh gpurun_out/pmc dropin4 'k_run_pass' 40000000 28 tests/_bin/kv_bench_dropin -ns 4 -nw 4 10000000 10 3 0
# Env assignments before the command (VAR=x ...) apply to both passes.
# `pmccalib` in tools/gpu_run.sh runs the calibration probe's passes.
set -e
out=$1; name=$2; kernels=$3; units=$4; per=$5
shift 5
envs=()
while [ $# -gt 0 ] && [ "${1#*=}" != "$1" ] && [ "${1#-}" = "$1" ]; do envs+=("$1"); shift; done
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p "$R/$out"
cmd=("$@")
case "${cmd[0]}" in /*) ;; *) [ -e "$R/${cmd[0]}" ] && cmd[0]="$R/${cmd[0]}" ;; esac
cd "$R" && export TMPDIR=/tmp  # (from the repo root: relative paths in COMMAND stay valid)
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf "$R/$out/$name.$c"
  env "${envs[@]}" timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d "$R/$out/$name.$c" -- "${cmd[@]}" > "$R/$out/$name.$c.log" 2>&1
done
python3 "$R/tools/pmc_summary.py" "$R/$out/$name.FETCH_SIZE" "$R/$out/$name.WRITE_SIZE" "$kernels" "$units" "$R/$out/$name.json" "$per"
