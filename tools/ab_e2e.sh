#!/bin/bash
# Interleaved A/B of the C++ API end to end (tests/_bin/kv_cluster_device, 10 M keys,
# 1 server + 1 worker) under environment settings, thread and process mode.
#   bash tools/ab_e2e.sh ROUNDS "VAR=a" "VAR=b" ...
# E2E_ARGS: the harness's positional arguments (default "10000000 20"; "... 1" = key cache)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$1; shift
for r in $(seq 1 "$R"); do
  for e in "$@"; do
    for mode in "" "-procs"; do
      env $e timeout -k 10 120 tests/_bin/kv_cluster_device -ns 1 -nw 1 $mode ${E2E_ARGS:-10000000 20} > gpurun_out/ab_e2e.log 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "$e $mode rc=$rc"; tail -3 gpurun_out/ab_e2e.log; exit $rc; fi
      printf "%-22s %-7s %s\n" "$e" "${mode:-thr}" "$(grep '^{' gpurun_out/ab_e2e.log | head -1 | cut -c40-240)"
    done
  done
done
