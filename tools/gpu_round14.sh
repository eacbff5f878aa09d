#!/bin/bash
# GPU pass 14: fused SORTED resolve+apply — parity suite, then keyed bench A/B (fused vs two-pass).
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_dropin_gpu.py > gpurun_out/pytest_p14.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_p14.log; stop_on_crash $rc
[ $rc -ne 0 ] && exit $rc
for i in 1 2; do for f in 0 1; do export PSG_SORTED_FUSED=$f;
  timeout -k 10 200 python3 bench.py --workload keyed --no-cpu-baseline > gpurun_out/k.json 2>gpurun_out/k.err || { cat gpurun_out/k.err | tail; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/k.json'));print('fused=$f', d['value'], d['push_ms'], d['pull_ms'], d['roofline']['frac'], d['parity_check'])"
done; done
cp gpurun_out/k.json gpurun_out/bench_keyed.json
exit 0
