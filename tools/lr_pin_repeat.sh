#!/bin/bash
# The LR pin case that caught a wrong model (3 workers, 200,000 features, SGD,
# BSP, dyadic gradients), run R times in a row; stops at the first failure and
# keeps its full diagnosis (gpurun_out/lr_pin_repeat.log).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
R=${1:-8}
: > gpurun_out/lr_pin_repeat.log
for i in $(seq 1 "$R"); do
  timeout -k 10 200 python3 -u -m pytest -q --timeout 150 --timeout-method thread tests/test_lr_ref_pin.py -m gpu \
    -k "3-200000" > gpurun_out/lr_pin_try.log 2>&1
  rc=$?
  echo "try $i rc=$rc" | tee -a gpurun_out/lr_pin_repeat.log
  case $rc in 124|134|137|139) echo "crash/timeout: stopping"; exit $rc;; esac
  if [ $rc -ne 0 ]; then cat gpurun_out/lr_pin_try.log >> gpurun_out/lr_pin_repeat.log; grep -E "differ|feature" gpurun_out/lr_pin_try.log | cut -c1-3000; exit 1; fi
done
