#!/bin/bash
# The general keyed path (validation + resolve-and-apply) measured two ways:
# on the configs[3] list with identity requests off (PSG_RA_IDENT=0: the store
# is exactly the list), and on a store with one extra key between each pair of
# the list's keys (PSG_BENCH_STORE_EXTRA=1: the list is every other store key),
# each with the PMC traffic of its Push (FETCH_SIZE and WRITE_SIZE passes).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for tag in general sparse; do
  if [ $tag = general ]; then envs="PSG_RA_IDENT=0"; else envs="PSG_BENCH_STORE_EXTRA=1"; fi
  env $envs timeout -k 10 300 python3 bench.py --workload keyed --no-cpu-baseline > gpurun_out/bench_keyed_$tag.json 2> gpurun_out/bench_keyed_$tag.err || exit $?
  cut -c1-900 gpurun_out/bench_keyed_$tag.json
  rm -rf gpurun_out/pmc_f_$tag gpurun_out/pmc_w_$tag
  env $envs timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f_$tag -- python3 bench.py --workload keyed --no-cpu-baseline --steps 10 --warmup 2 --check 0 > gpurun_out/pmc_f_$tag.log 2>&1 || exit $?
  env $envs timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w_$tag -- python3 bench.py --workload keyed --no-cpu-baseline --steps 10 --warmup 2 --check 0 > gpurun_out/pmc_w_$tag.log 2>&1 || exit $?
  python3 tools/pmc_summary.py gpurun_out/pmc_f_$tag gpurun_out/pmc_w_$tag "k_validate_windows|k_resolve_apply<0, 1," 10000000 gpurun_out/pmc_keyed_push_$tag.json 28
  cat gpurun_out/pmc_keyed_push_$tag.json
done
