#!/bin/bash
# A/B of the keyed bench over library variants in abtmp/ (interleaved), then
# the GPU parity suite on the in-tree library.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -2 gpurun_out/ab_pytest.log
for i in 1 2 3; do for v in ${VARIANTS:-old new6 glds}; do
  PSG_LIB=abtmp/libpsgpu_$v.so timeout -k 10 120 python3 bench.py --workload keyed --no-cpu-baseline --check 0 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$v', d['value'], d['ms_per_step'], d['push_ms'], d['pull_ms'], d['roofline']['frac'])"
done; done
