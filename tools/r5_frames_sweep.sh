#!/bin/bash
# k_frames_apply kernel times (rocprofv3 --stats) of tools/pmc_targets.py
# frames8 / frames_cached8 under PSG_FRAMES_BPC variants.
out=${1:-gpurun_out/r5_frames_sweep}
R=$GRAFT_REPO_ROOT
mkdir -p "$R/$out"
cd /tmp && export TMPDIR=/tmp
for t in frames8 frames_cached8; do
  for b in 2 4 8 16; do
    PSG_FRAMES_BPC=$b timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/$t.b$b" -- python3 "$R/tools/pmc_targets.py" $t 10 > /dev/null 2>&1 || exit 1
  done
done
