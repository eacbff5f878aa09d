#!/bin/bash
# The one A/B runner: a command under env variants, interleaved over rounds,
# every line of output tagged with its variant.  Replaces round 4-5's one-off
# scripts (r5_*.sh, ab_*.sh): each was this loop with a fixed command.
#
# usage (on the box):
#   bash tools/ab.sh OUT ROUNDS 'COMMAND' VARIANT...
#     OUT      output file (a directory for `prof:`), under gpurun_out/
#     ROUNDS   how many times the variant list is run, interleaved
#     COMMAND  run with `env VARIANT`; a leading `prof:` runs it under
#              rocprofv3 --kernel-trace --stats into OUT/rROUND.vINDEX/;
#              `grep:PATTERN:` keeps only the output lines matching PATTERN
#     VARIANT  an env assignment list ("" = defaults); -procs / -ns N in a
#              variant are appended to the command instead
# examples (the round-5 one-offs):
#   keyed lines            bash tools/ab.sh gpurun_out/k.txt 2 'grep:^{:python3 bench.py --workload keyed --steps 30 --warmup 5 --no-cpu-baseline --no-probe256' "" "PSG_RA_MIDENT=0"
#   drop-in line, N = 1    bash tools/ab.sh gpurun_out/d.txt 2 'grep:rank:tests/_bin/kv_bench_dropin -ns 1 -nw 1 10000000 30 5 0' "" "-procs"
#   configs[0] stages      bash tools/ab.sh gpurun_out/s.txt 2 'PS_STAGE_TIMES=1 tests/_dropin/test_kv_app_benchmark -ns 1 -nw 1' "" "-procs PS_SHM_ARENA_MB=0"
#   kernel stats           bash tools/ab.sh gpurun_out/p 1 'prof:python3 tools/pmc_targets.py frames8 10' "PSG_FRAMES_BPC=2" "PSG_FRAMES_BPC=8"
# Every run has its own time limit (AB_TIMEOUT, default 300 s); a crash or a
# time-out ends the script (no later GPU step runs).
set -u
out=$1
rounds=$2
cmd=$3
shift 3
[ $# -eq 0 ] && set -- ""
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
limit=${AB_TIMEOUT:-300}
prof=0
pat=""
if [ "${cmd#prof:}" != "$cmd" ]; then prof=1; cmd=${cmd#prof:}; mkdir -p "$out"; else : > "$out"; fi
if [ "${cmd#grep:}" != "$cmd" ]; then rest=${cmd#grep:}; pat=${rest%%:*}; cmd=${rest#*:}; fi
for r in $(seq 1 "$rounds"); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    envs=()
    args=()
    for w in $v; do
      case "$w" in
        -procs) args+=("$w") ;;
        *=*) envs+=("$w") ;;
        *) args+=("$w") ;;
      esac
    done
    if [ $prof = 1 ]; then
      d="$out/r$r.v$i"
      env "${envs[@]}" TMPDIR=/tmp timeout -k 10 "$limit" rocprofv3 --kernel-trace --stats --output-format csv -d "$d" -o run -- $cmd "${args[@]}" > "$d.log" 2>&1
      rc=$?
      echo "[$v] round $r -> $d (rc $rc)" >> "$out/index.txt"
    else
      res=$(env "${envs[@]}" timeout -k 10 "$limit" $cmd "${args[@]}" 2>&1)
      rc=$?
      if [ -n "$pat" ]; then res=$(printf '%s\n' "$res" | grep -E "$pat"); fi
      printf '%s\n' "$res" | sed "s|^|[$v] r$r |" >> "$out"
    fi
    case $rc in 124|134|137|139) echo "[$v] round $r: crashed or timed out ($rc); stopping" >&2; exit $rc ;; esac
  done
done
