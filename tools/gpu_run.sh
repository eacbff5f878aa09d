#!/bin/bash
# The one GPU runner: tools/gpu_run.sh STAGE [STAGE ...], run on the box by
#   gpurun --timeout T -- 'bash tools/gpu_run.sh tests bench prof'
# Every step has its own time limit; a crash, abort or time-out ends the call
# (no later GPU step runs).  Outputs land in gpurun_out/.
#   tests    the whole -m gpu suite            smoke  __graft_entry__.smoke()
#   bench    default bench line (configs[1])   prof   rocprof kernel stats of it
#   keyed    keyed bench lines (configs[3]:    proffk / profkc  rocprof kernel stats of
#            uncached and key-cached)                  keyed / keyed-cached
#   f16      1 G f16 bench line (configs[4])   e2e    C++ API end to end, 10 M keys
#   t:EXPR   pytest -m gpu -k EXPR             pmck / pmckc / pmckp  PMC traffic of the keyed /
#                                                      key-cached Push, keyed Pull (two passes each)
#   trace    kernel trace of the keyed bench: durations and the idle gaps between
#            launches (tools/trace_gaps.py)
#   pmcki / pmckip  PMC traffic of the identity keyed Push (check + apply) / Pull
#   pmcks    PMC traffic of the key-cached Push on a stretch of slots (k_dense_vec, 12 B/key)
#   lr       LR apply roofline (tools/bench_lr.py, 10 M and 64 M features) + its rocprof stats
#   lrb      the bench line of the LR BSP round (bench.py --workload lr) + its rocprof stats
#   dropin:N:MODE:LAYOUT  the drop-in API line at ns = nw = N (MODE threads|procs,
#            LAYOUT 0 the benchmark's interleaved keys, 1 one shared list)
#   strided  kernel stats of strided runs alone (4 / 8 requests, Push / Pull)
#   pmcstrided  PMC traffic of the 4-request strided Push and Pull passes
#   pmccalib the gfx950 PMC calibration passes (tools/_bin/probe_pmc_shapes)
#   pmcdropin:N:MODE  HBM traffic per step of the drop-in line (two step counts, differenced)
#   pmcpull / pmcadam  PMC traffic of the 256 M Pull / the 64 M-feature Adam apply
#            (tools/pmc_targets.py, two passes each)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_on_crash() { case "$1" in 124|134|137|139) echo "GPU step crashed/timed out ($1); stopping"; exit "$1";; esac; }
step() { local t=$1; shift; timeout -k 10 "$t" "$@"; local rc=$?; stop_on_crash $rc; return $rc; }
PYT="python3 -u -m pytest -v --timeout 150 --timeout-method thread"
for st in "$@"; do
  case "$st" in
    tests) step 1100 $PYT tests -m gpu > gpurun_out/pytest_gpu.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/pytest_gpu.log ;;
    t:*) step 900 $PYT tests -m gpu -k "${st#t:}" > gpurun_out/pytest_k.log 2>&1; echo "tests[${st#t:}] rc=$?"; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_k.log | tail -30 ;;
    smoke) step 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; echo "smoke rc=$?"; tail -1 gpurun_out/smoke.log ;;
    bench) step 300 python3 bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; echo "bench rc=$?"; cat gpurun_out/bench.json; tail -3 gpurun_out/bench.err ;;
    prof) rm -rf gpurun_out/prof64
          step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof64 -o run --output-format csv -- python3 bench.py --no-cpu-baseline > gpurun_out/prof64.json 2>&1; echo "prof rc=$?"
          f=$(find gpurun_out/prof64 -name "*kernel_stats.csv" | head -1); cut -c1-200 "$f" | head -12 ;;
    keyed) step 300 python3 bench.py --workload keyed --no-cpu-baseline > gpurun_out/bench_keyed.json 2> gpurun_out/bench_keyed.err; echo "keyed rc=$?"; cat gpurun_out/bench_keyed.json; tail -3 gpurun_out/bench_keyed.err
           step 300 python3 bench.py --workload keyed-cached --no-cpu-baseline > gpurun_out/bench_keyed_cached.json 2> gpurun_out/bench_keyed_cached.err; echo "keyed-cached rc=$?"; cat gpurun_out/bench_keyed_cached.json; tail -3 gpurun_out/bench_keyed_cached.err ;;
    proffk) rm -rf gpurun_out/prof_keyed
          step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_keyed -o run --output-format csv -- python3 bench.py --workload keyed --no-cpu-baseline --steps 20 > gpurun_out/prof_keyed.json 2>&1; echo "proffk rc=$?"
          f=$(find gpurun_out/prof_keyed -name "*kernel_stats.csv" | head -1); cut -c1-200 "$f" | head -12 ;;
    profkc) rm -rf gpurun_out/prof_keyed_cached
          step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_keyed_cached -o run --output-format csv -- python3 bench.py --workload keyed-cached --no-cpu-baseline --steps 20 > gpurun_out/prof_keyed_cached.json 2>&1; echo "profkc rc=$?"
          f=$(find gpurun_out/prof_keyed_cached -name "*kernel_stats.csv" | head -1); cut -c1-160 "$f" | head -8 ;;
    pmck|pmckc|pmckp|pmcki|pmckip|pmcks)
          if [ "$st" = pmck ]; then wl=keyed; ks="k_validate_windows|k_resolve_apply<0, 1,"; per=28; out=pmc_keyed_push_traffic.json
          elif [ "$st" = pmcki ]; then wl=keyed; ks="k_ident_check|k_ident_apply<0, 1>"; per=28; out=pmc_keyed_ident_push_traffic.json
          elif [ "$st" = pmckip ]; then wl=keyed; ks="k_ident_apply<0, 2>"; per=24; out=pmc_keyed_ident_pull_traffic.json
          elif [ "$st" = pmckp ]; then wl=keyed; ks="k_resolve_apply<0, 2,"; per=24; out=pmc_keyed_pull_traffic.json
          elif [ "$st" = pmcks ]; then wl=keyed-cached; ks="k_dense_vec<0, 1,"; per=12; out=pmc_keyed_stretch_push_traffic.json
          else wl=keyed-cached; ks="k_slots_vec<0, 1,"; per=16; out=pmc_keyed_cached_push_traffic.json; fi
          rm -rf gpurun_out/pmc_f_$st gpurun_out/pmc_w_$st
          step 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f_$st -- python3 bench.py --workload $wl --no-cpu-baseline --steps 10 --warmup 2 --check 0 > gpurun_out/pmc_f_$st.log 2>&1; echo "$st fetch rc=$?"
          step 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w_$st -- python3 bench.py --workload $wl --no-cpu-baseline --steps 10 --warmup 2 --check 0 > gpurun_out/pmc_w_$st.log 2>&1; echo "$st write rc=$?"
          python3 tools/pmc_summary.py gpurun_out/pmc_f_$st gpurun_out/pmc_w_$st "$ks" 10000000 gpurun_out/$out $per ;;
    lrb)  step 300 python3 bench.py --workload lr > gpurun_out/bench_lr_line.json 2> gpurun_out/bench_lr_line.err; echo "lrb rc=$?"; cat gpurun_out/bench_lr_line.json; tail -3 gpurun_out/bench_lr_line.err
          rm -rf gpurun_out/prof_lrb
          step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lrb -o run --output-format csv -- python3 bench.py --workload lr --no-cpu-baseline > gpurun_out/prof_lrb.log 2>&1; echo "proflrb rc=$?"
          cut -c1-160 gpurun_out/prof_lrb/run_kernel_stats.csv | head -4 ;;
    lr)   step 300 python3 tools/bench_lr.py 10000000 67108864 > gpurun_out/bench_lr.jsonl 2> gpurun_out/bench_lr.err; echo "lr rc=$?"; cat gpurun_out/bench_lr.jsonl
          rm -rf gpurun_out/prof_lr
          step 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_lr -o run --output-format csv -- python3 tools/bench_lr.py 67108864 > gpurun_out/prof_lr.log 2>&1; echo "proflr rc=$?"
          cut -c1-160 gpurun_out/prof_lr/run_kernel_stats.csv | head -8 ;;
    pmcpull|pmcadam)
          if [ "$st" = pmcpull ]; then tg=pull256; ks="k_dense_vec<0, 2,"; keys=268435456; per=8; out=pmc_pull256_traffic.json
          else tg=adam64; ks="k_lr_apply_sum<true"; keys=67108864; per=56; out=pmc_lr_adam64_traffic.json; fi
          rm -rf gpurun_out/pmc_f_$st gpurun_out/pmc_w_$st
          step 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_f_$st -- python3 tools/pmc_targets.py $tg > gpurun_out/pmc_f_$st.log 2>&1; echo "$st fetch rc=$?"
          step 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_w_$st -- python3 tools/pmc_targets.py $tg > gpurun_out/pmc_w_$st.log 2>&1; echo "$st write rc=$?"
          python3 tools/pmc_summary.py gpurun_out/pmc_f_$st gpurun_out/pmc_w_$st "$ks" $keys gpurun_out/$out $per; cat gpurun_out/$out ;;
    trace) rm -rf gpurun_out/trace_keyed
          step 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_keyed -o run -- python3 bench.py --workload keyed --no-cpu-baseline --no-probe256 --steps 10 --warmup 2 > gpurun_out/trace_keyed.json 2>&1; echo "trace rc=$?"
          python3 tools/trace_gaps.py gpurun_out/trace_keyed/run_kernel_trace.csv 8 ;;
    f16) step 300 python3 bench.py --workload dense-f16 --no-cpu-baseline > gpurun_out/bench_f16.json 2> gpurun_out/bench_f16.err; echo "f16 rc=$?"; cat gpurun_out/bench_f16.json ;;
    e2e) step 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 10000000 20 > gpurun_out/e2e_threads_10M.log 2>&1; echo "e2e threads rc=$?"; head -3 gpurun_out/e2e_threads_10M.log
         step 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 -procs 10000000 20 > gpurun_out/e2e_procs_10M.log 2>&1; echo "e2e procs rc=$?"; head -3 gpurun_out/e2e_procs_10M.log
         step 300 tests/_bin/kv_cluster_device -ns 1 -nw 1 10000000 20 1 > gpurun_out/e2e_threads_10M_keycache.log 2>&1; echo "e2e threads key-cache rc=$?"; head -3 gpurun_out/e2e_threads_10M_keycache.log ;;
    shared2|shared8)
          nr=${st#shared}; port=$((29500 + RANDOM % 1000))
          PSG_BENCH_SHARE_GPU=1 step 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $nr --master-addr 127.0.0.1 --master-port $port bench.py --gpus $nr > gpurun_out/bench_shared_n$nr.json 2> gpurun_out/bench_shared_n$nr.err; echo "$st rc=$?"; grep "^{" gpurun_out/bench_shared_n$nr.json | cut -c1-600 ;;
    dropin:*)
          # dropin:N:mode:layout — the drop-in API line (bench.py --workload dropin)
          IFS=: read -r _ dn dm dl <<< "$st"; tag="n${dn}_${dm}_l${dl}"
          step 300 python3 bench.py --workload dropin --gpus "$dn" --dropin-mode "$dm" --dropin-layout "$dl" --no-cpu-baseline > gpurun_out/bench_dropin_$tag.json 2> gpurun_out/bench_dropin_$tag.err; echo "$st rc=$?"; cut -c1-900 gpurun_out/bench_dropin_$tag.json; tail -3 gpurun_out/bench_dropin_$tag.err ;;
    dtrace:*)
          # dtrace:N:mode:layout — kv_bench_dropin with the servers' request trace:
          # run sizes per server (PS_TRACE_REQUESTS) and the store counters
          IFS=: read -r _ dn dm dl <<< "$st"; tag="n${dn}_${dm}_l${dl}"; rm -f gpurun_out/dtrace_$tag.txt gpurun_out/dgather_$tag.txt
          md=""; [ "$dm" = procs ] && md="-procs"
          PS_TRACE_GATHER=$PWD/gpurun_out/dgather_$tag.txt PS_TRACE_REQUESTS=$PWD/gpurun_out/dtrace_$tag.txt step 200 tests/_bin/kv_bench_dropin -ns "$dn" -nw "$dn" $md 10000000 30 5 "$dl" > gpurun_out/dtrace_$tag.log 2>&1; echo "$st rc=$?"; grep "^{" gpurun_out/dtrace_$tag.log | cut -c1-300
          python3 tools/run_sizes.py gpurun_out/dtrace_$tag.txt ;;
    dprof:*)
          # dprof:N:mode:layout — rocprof kernel stats + trace of kv_bench_dropin
          IFS=: read -r _ dn dm dl <<< "$st"; tag="n${dn}_${dm}_l${dl}"; rm -rf gpurun_out/dprof_$tag
          md=""; [ "$dm" = procs ] && md="-procs"
          step 240 rocprofv3 --kernel-trace --stats -d gpurun_out/dprof_$tag -o run --output-format csv -- tests/_bin/kv_bench_dropin -ns "$dn" -nw "$dn" $md 10000000 30 5 "$dl" > gpurun_out/dprof_$tag.log 2>&1; echo "$st rc=$?"; grep '"rank": 0' gpurun_out/dprof_$tag.log | cut -c1-300
          f=$(find gpurun_out/dprof_$tag -name "*kernel_stats.csv" | head -1); cut -c1-180 "$f" | head -12 ;;
    strided)
          # the strided run's kernels alone (tools/pmc_targets.py): kernel stats
          # and PMC traffic of a 4- and an 8-request run, Push and Pull
          for t in ${STRIDED_TARGETS:-strided4push strided4pull strided8push strided8pull}; do
            rm -rf gpurun_out/prof_$t
            step 120 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$t -o run --output-format csv -- python3 tools/pmc_targets.py $t 20 > gpurun_out/prof_$t.log 2>&1; echo "$t rc=$?"
            python3 - "$t" <<'PY'
import csv, sys
t = sys.argv[1]
for r in csv.DictReader(open(f"gpurun_out/prof_{t}/run_kernel_stats.csv")):
    n = r["Name"]
    if "k_run" in n:
        avg = float(r["AverageNs"]) / 1e3
        per = 16 if "k_run_pass<0, 0" in n else (12 if "k_run_pass<0, 1" in n else (24 if "k_run_pass<0, 2" in n else 0))
        frac = (per * 10e6 / (avg * 1e-6) / 8e12) if per else 0
        print(f"  {n[:60]:60s} calls {r['Calls']:>4} avg {avg:8.1f} us  {per} B/key -> {frac:.3f} of 8 TB/s")
PY
          done ;;
    pmcstrided)
          bash tools/pmc.sh gpurun_out/pmc_strided s4push 'k_run_pass<0, 0|k_run_pass<0, 1' 10000000 28 python3 tools/pmc_targets.py strided4push 10 && cat gpurun_out/pmc_strided/s4push.json
          bash tools/pmc.sh gpurun_out/pmc_strided s4pull 'k_run_pass<0, 2' 10000000 24 python3 tools/pmc_targets.py strided4pull 10 && cat gpurun_out/pmc_strided/s4pull.json
          bash tools/pmc.sh gpurun_out/pmc_strided s8push 'k_run_pass<0, 0|k_run_pass<0, 1' 10000000 28 python3 tools/pmc_targets.py strided8push 10 && cat gpurun_out/pmc_strided/s8push.json
          bash tools/pmc.sh gpurun_out/pmc_strided s8pull 'k_run_pass<0, 2' 10000000 24 python3 tools/pmc_targets.py strided8pull 10 && cat gpurun_out/pmc_strided/s8pull.json ;;
    pmccalib)
          # the gfx950 FETCH/WRITE calibration per access shape:
          # four counter passes and a trace over tools/_bin/probe_pmc_shapes
          out=gpurun_out/pmc_calib; rm -rf "$out"; mkdir -p "$out"; R=$PWD
          ( cd /tmp && export TMPDIR=/tmp &&
            timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$out/fetch" -- "$R/tools/_bin/probe_pmc_shapes" 3 &&
            timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$out/write" -- "$R/tools/_bin/probe_pmc_shapes" 3 &&
            timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum --output-format csv -d "$R/$out/rdreq" -- "$R/tools/_bin/probe_pmc_shapes" 3 &&
            timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d "$R/$out/wrreq" -- "$R/tools/_bin/probe_pmc_shapes" 3 &&
            timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/trace" -- "$R/tools/_bin/probe_pmc_shapes" 3 ) > "$out.log" 2>&1
          rc=$?; echo "pmccalib rc=$rc"; stop_on_crash $rc
          python3 tools/pmc_calib.py "$out" "$out/calibration.json" ;;
    dstage:*)
          # dstage:N:mode:layout:gather — kv_bench_dropin with the host stage times
          # (PS_STAGE_TIMES=1), summarised per stage (tools/stage_summary.py)
          IFS=: read -r _ dn dm dl dg <<< "$st"; tag="n${dn}_${dm}_l${dl}_g${dg:-0}"
          md=""; [ "$dm" = procs ] && md="-procs"
          PS_RUN_GATHER_US=${dg:-0} PS_STAGE_TIMES=1 step 200 tests/_bin/kv_bench_dropin -ns "$dn" -nw "$dn" $md 10000000 30 5 "$dl" > gpurun_out/dstage_$tag.log 2>&1; echo "$st rc=$?"; grep '"rank": 0' gpurun_out/dstage_$tag.log | cut -c1-300
          python3 tools/stage_summary.py gpurun_out/dstage_$tag.log 40 ;;
    pmcdropin:*)
          # pmcdropin:N:mode — HBM traffic per step of the drop-in line (layout 0,
          # the default gather window): FETCH / WRITE passes of kv_bench_dropin at
          # 10 and 40 timed steps, differenced (tools/pmc_total.py)
          # (PMC_GATHER_US: the servers' gather window for these passes — under
          # counter collection every dispatch is serialized, so the requests of a
          # step reach a server spread out and, with the default window, fewer
          # runs form than in the unprofiled line)
          IFS=: read -r _ dn dm <<< "$st"; tag="n${dn}_${dm}"; o=gpurun_out/pmc_dropin_$tag; rm -rf "$o"; mkdir -p "$o"
          export PS_RUN_GATHER_US=${PMC_GATHER_US:-120} PS_RUN_GATHER_ORD_US=${PMC_GATHER_ORD_US:-1000}
          md=""; [ "$dm" = procs ] && md="-procs"
          for sN in 10 40; do for c in FETCH_SIZE WRITE_SIZE; do
            step 240 rocprofv3 --pmc $c --output-format csv -d "$o/$c.$sN" -- tests/_bin/kv_bench_dropin -ns "$dn" -nw "$dn" $md 10000000 $sN 5 0 > "$o/$c.$sN.log" 2>&1 || { echo "pmcdropin pass $c $sN failed"; exit 1; }
          done; done
          python3 tools/pmc_total.py "$o/FETCH_SIZE.10" "$o/WRITE_SIZE.10" "$o/FETCH_SIZE.40" "$o/WRITE_SIZE.40" 10 40 $((52 * 10000000 * dn)) "$o/traffic.json" "kv_bench_dropin -ns $dn -nw $dn $md, 10 M keys per worker, layout 0, gather window $PS_RUN_GATHER_US us; alg bytes per step: (28 + 24) B x 10 M keys x $dn workers"; unset PS_RUN_GATHER_US ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
