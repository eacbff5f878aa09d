#!/bin/bash
# Round-4 measurement batch (one gpurun call): parity of what changed first,
# then the measurements.  Each GPU step has its own limit; a crash or time-out
# ends the call.  Outputs under gpurun_out/.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
stop() { case "$1" in 124|134|137|139) echo "step crashed/timed out ($1): stopping"; exit "$1";; esac; }
PYT="python3 -u -m pytest -v --timeout 150 --timeout-method thread"
for st in "$@"; do
  case "$st" in
    parity) timeout -k 10 600 $PYT tests -m gpu -k "lr or dense or handoff or sparse or configs" > gpurun_out/r4_parity.log 2>&1; rc=$?; stop $rc
            echo "parity rc=$rc"; grep -E "passed|failed" gpurun_out/r4_parity.log | tail -2 ;;
    lr) timeout -k 10 300 python3 tools/bench_lr.py 10000000 67108864 > gpurun_out/r4_bench_lr.jsonl 2>&1; rc=$?; stop $rc
        echo "bench_lr rc=$rc"; cat gpurun_out/r4_bench_lr.jsonl ;;
    shapes) for n in 10000000 67108864 268435456; do timeout -k 10 200 tools/_bin/probe_push_small $n 4; rc=$?; stop $rc; done > gpurun_out/r4_probe_push_shapes.txt 2>&1
            cat gpurun_out/r4_probe_push_shapes.txt ;;
    keyedgen) timeout -k 10 900 bash tools/run_keyed_general.sh > gpurun_out/r4_keyed_general.txt 2>&1; rc=$?; stop $rc
              echo "keyed general rc=$rc"; grep -E '"frac"|traffic|hbm_bytes|ratio' gpurun_out/r4_keyed_general.txt | cut -c1-300 | head -20 ;;
    *) bash tools/gpu_run.sh "$st"; rc=$?; stop $rc ;;
  esac
done
