# The round-end GPU validation, in two parts (one gpurun call each):
#   bash tools/gpu_validate.sh tests   the GPU tests and smoke()
#   bash tools/gpu_validate.sh lines   the default bench line, the keyed lines
#                                      (the store's own list; a random 90 %
#                                      subset), the LR line and the drop-in
#                                      lines at N = 1, 4, 8
# Outputs go to gpurun_out/${ROUND:-r6}_*.  Each step runs under its own time
# limit; the first failure ends the script.
set -e
R=${ROUND:-r6}
case "${1:-tests}" in
  tests)
    timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/${R}_pytest_gpu_final.txt 2>&1
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${R}_smoke_final.txt 2>&1
    ;;
  lines)
    timeout -k 10 300 python -u bench.py > gpurun_out/${R}_bench_default_final.txt 2>&1
    timeout -k 10 300 python -u bench.py --workload keyed > gpurun_out/${R}_bench_keyed_final.txt 2>&1
    PSG_BENCH_SUBSET=0.9 timeout -k 10 300 python -u bench.py --workload keyed > gpurun_out/${R}_bench_keyed_subset09_final.txt 2>&1
    timeout -k 10 300 python -u bench.py --workload lr --no-cpu-baseline > gpurun_out/${R}_bench_lr_final.txt 2>&1
    for spec in 1:threads 1:procs 4:threads 4:procs 8:threads; do
      n=${spec%%:*}; m=${spec#*:}
      timeout -k 10 300 python -u bench.py --workload dropin --gpus "$n" --dropin-mode "$m" \
        --no-cpu-baseline > gpurun_out/${R}_bench_dropin_n${n}_${m}_final.txt 2>&1
    done
    ;;
esac
