#!/bin/bash
# A/B of the keyed Push's launch knobs: each line one fresh bench process.
# usage (on the box): bash tools/ab_keyed.sh "ENV1" "ENV2" ...   (ENV like "PSG_LB_GRID=1024")
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for cfg in "$@"; do
  env $cfg timeout -k 10 120 python3 bench.py --workload keyed --no-cpu-baseline --steps 30 > gpurun_out/ab_tmp.json 2> gpurun_out/ab_tmp.err
  rc=$?
  python3 -c "
import json,sys
d=json.load(open('gpurun_out/ab_tmp.json'))
print('%-40s value %8.1f push_ms %.4f pull_ms %.4f frac %.4f' % (sys.argv[1], d['value'], d['push_ms'], d['pull_ms'], d['roofline']['frac']))
" "$cfg" || { echo "$cfg rc=$rc"; tail -3 gpurun_out/ab_tmp.err; }
  case $rc in 124|134|137|139) exit $rc;; esac
done
