set -o pipefail
bash tools/gpu_run.sh "t:sorted or async or semantics or cluster or dropin or keyed or pull" || exit 1
for L in 1 0 1 0; do
  for n in 1000 10000000; do
    PSG_PULL_LAND=$L timeout -k 10 100 tests/_bin/kv_cluster_device -ns 1 -nw 1 $n 50 > gpurun_out/e.log 2>&1 || exit 1; echo "land=$L threads $(head -1 gpurun_out/e.log | cut -c1-150)"
    PSG_PULL_LAND=$L timeout -k 10 100 tests/_bin/kv_cluster_device -ns 1 -nw 1 -procs $n 50 > gpurun_out/e.log 2>&1 || exit 1; echo "land=$L procs $(head -1 gpurun_out/e.log | cut -c1-150)"
  done
done
bash tools/ab_keyed.sh "PSG_PULL_LAND=1" "PSG_PULL_LAND=0"
