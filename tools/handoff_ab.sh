#!/bin/bash
# A/B of the reply hand-off (tests/harness/unit/handoff_stress.cpp): each mode
# and size under each wait mechanism, one process at a time, each under its own
# time limit.  Stops at the first status that is neither 0 (nothing stale) nor
# 3 (stale replies seen).  Output: gpurun_out/handoff_ab.txt
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
OUT=gpurun_out/handoff_ab.txt
: > "$OUT"
ITERS=${ITERS:-2000}
for envs in "${@:-default}"; do
  for m in ${MODES:-lr dense stretch keyed}; do
    for n in ${SIZES:-200000 4000000}; do
      if [ "$envs" = default ]; then
        timeout -k 10 90 tests/_bin/handoff_stress $m $n $ITERS ${THREADS:-1} >> "$OUT" 2>&1
      else
        env $envs timeout -k 10 90 tests/_bin/handoff_stress $m $n $ITERS ${THREADS:-1} >> "$OUT" 2>&1
      fi
      rc=$?
      echo "  [$envs] rc=$rc" >> "$OUT"
      if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then
        echo "stopping: status $rc" >> "$OUT"
        cat "$OUT"
        exit $rc
      fi
    done
  done
done
cat "$OUT"
