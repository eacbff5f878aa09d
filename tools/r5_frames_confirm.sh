#!/bin/bash
# k_frames_apply on 64 M floats, k = 8 (tools/pmc_targets.py frames8): the
# size-based default grid against PSG_FRAMES_BPC=8, interleaved rounds.
out=${1:-gpurun_out/r5_frames_confirm}
R=$GRAFT_REPO_ROOT
mkdir -p "$R/$out"
cd /tmp && export TMPDIR=/tmp
for r in 1 2 3; do
  for v in "" "PSG_FRAMES_BPC=8"; do
    env $v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/r$r${v:+.b8}" -- python3 "$R/tools/pmc_targets.py" frames8 10 > /dev/null 2>&1 || exit 1
  done
done
