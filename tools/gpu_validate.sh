# The round-end GPU validation: the GPU tests, smoke(), the default bench line
# and the keyed lines (the store's own list; a random 90 % subset).  Each step
# under its own time limit; the first failure ends the script.
set -e
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r5_pytest_gpu_final.txt 2>&1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_smoke_final.txt 2>&1
timeout -k 10 300 python -u bench.py > gpurun_out/r5_bench_default_final.txt 2>&1
timeout -k 10 300 python -u bench.py --workload keyed > gpurun_out/r5_bench_keyed_final.txt 2>&1
PSG_BENCH_SUBSET=0.9 timeout -k 10 300 python -u bench.py --workload keyed > gpurun_out/r5_bench_keyed_subset09_final.txt 2>&1
