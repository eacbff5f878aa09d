set -o pipefail
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 150 --timeout-method thread tests -m gpu -k "dropin or cluster or semantics or procs or process" > gpurun_out/pt.log 2>&1; rc=$?; tail -2 gpurun_out/pt.log; [ $rc -eq 0 ] || exit 1
for r in 1 2 3; do
  for n in 1000 10000000; do
    timeout -k 10 100 tests/_bin/kv_cluster_device -ns 1 -nw 1 -procs $n 50 > gpurun_out/e.log 2>&1 || exit 1; echo "procs $(head -1 gpurun_out/e.log | cut -c1-150)"
  done
done
for n in 1000 10000000; do
  timeout -k 10 100 tests/_bin/kv_cluster_device -ns 1 -nw 1 $n 50 > gpurun_out/e.log 2>&1 || exit 1; echo "threads $(head -1 gpurun_out/e.log | cut -c1-150)"
done
