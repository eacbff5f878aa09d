#!/bin/bash
# Four rocprofv3 counter passes over tools/probe_pmc_shapes (one counter set a
# pass: FETCH_SIZE needs 3 TCC slots, WRITE_SIZE 2).  Output under $1.
set -e
out=${1:-gpurun_out/r5_pmc_calib}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$out/fetch" -- "$R/tools/probe_pmc_shapes" 3
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$out/write" -- "$R/tools/probe_pmc_shapes" 3
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum --output-format csv -d "$R/$out/rdreq" -- "$R/tools/probe_pmc_shapes" 3
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum --output-format csv -d "$R/$out/wrreq" -- "$R/tools/probe_pmc_shapes" 3
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/trace" -- "$R/tools/probe_pmc_shapes" 3
