#!/bin/bash
# Interleaved A/B of the LR apply (tools/bench_lr.py) under environment settings.
#   bash tools/ab_lr.sh ROUNDS N_FEATURES "VAR=a" "VAR=b" ...
# Prints, per run, the [ng=1, ng=4] fractions of 8 TB/s for SGD and Adam.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=$1; N=$2; shift 2
for r in $(seq 1 "$R"); do
  for e in "$@"; do
    env $e timeout -k 10 200 python3 tools/bench_lr.py "$N" > gpurun_out/ab_lr.jsonl 2> gpurun_out/ab_lr.err
    rc=$?
    if [ $rc -ne 0 ]; then echo "$e rc=$rc"; tail -3 gpurun_out/ab_lr.err; exit $rc; fi
    python3 - "$e" <<'PY'
import json, sys
rows = [json.loads(l) for l in open("gpurun_out/ab_lr.jsonl") if l.startswith("{")]
sgd = [r["frac"] for r in rows if r["update"] == "sgd"]
adam = [r["frac"] for r in rows if r["update"] == "adam"]
print(f"{sys.argv[1]:28s} sgd {sgd} adam {adam}")
PY
  done
done
