#!/bin/bash
# GPU pass 4: tests (incl. forced RCCL collectives on one rank), torch-first
# runtime ordering, bench f32/f16/256M, rocprof kernel stats.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
timeout -k 10 900 python3 -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/pytest_gpu.log; stop_on_crash $rc
timeout -k 10 300 python3 -c "import torch; import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_torch_first.log 2>&1
rc=$?; echo "smoke torch-first rc=$rc"; tail -2 gpurun_out/smoke_torch_first.log; stop_on_crash $rc
timeout -k 10 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; stop_on_crash $rc
timeout -k 10 300 python3 bench.py --workload dense-f16 --no-cpu-baseline > gpurun_out/bench_f16.json 2> gpurun_out/bench_f16.err
rc=$?; echo "bench f16 rc=$rc"; cat gpurun_out/bench_f16.json; stop_on_crash $rc
timeout -k 10 300 python3 bench.py --keys 268435456 --no-cpu-baseline --steps 20 > gpurun_out/bench_256m.json 2> gpurun_out/bench_256m.err
rc=$?; echo "bench 256M rc=$rc"; cat gpurun_out/bench_256m.json; stop_on_crash $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/prof.log 2>&1
rc=$?; echo "rocprof rc=$rc"; stop_on_crash $rc
exit 0
