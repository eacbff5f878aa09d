#!/bin/bash
# A/B of the keyed bench over PSG_RA_BLOCK values (interleaved), then
# rocprof kernel stats of the in-tree library; the GPU parity suite first.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_pytest.log 2>&1 || { tail -30 gpurun_out/ab_pytest.log; exit 1; }
tail -2 gpurun_out/ab_pytest.log
for i in 1 2 3; do for v in ${VARIANTS:-512 1024}; do
  PSG_RA_BLOCK=$v timeout -k 10 120 python3 bench.py --workload keyed --no-cpu-baseline --check 0 > gpurun_out/ab.json 2>gpurun_out/ab.err || { tail gpurun_out/ab.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/ab.json'));print('$v', d['value'], d['ms_per_step'], d['push_ms'], d['pull_ms'], d['roofline']['frac'])"
done; done
rm -rf gpurun_out/prof_keyed
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_keyed -o run --output-format csv -- python3 bench.py --workload keyed --no-cpu-baseline --steps 20 > gpurun_out/prof_keyed.json 2> gpurun_out/prof_keyed.err || exit 1
f=$(find gpurun_out/prof_keyed -name "*kernel_stats.csv" | head -1); cut -c1-60 "$f" | head -4; rev "$f" | cut -d, -f1-7 | rev | head -4
