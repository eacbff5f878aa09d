#!/bin/bash
# PMC (FETCH_SIZE, WRITE_SIZE passes) and kernel stats of the run kernels
# (tools/pmc_targets.py frames*), summarised by tools/pmc_summary.py.
set -e
out=${1:-gpurun_out/r5_pmc_frames}
R=$GRAFT_REPO_ROOT
mkdir -p "$R/$out"
cd /tmp && export TMPDIR=/tmp
for t in frames8 frames_keyed8 frames_cached8; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$out/$t.fetch" -- python3 "$R/tools/pmc_targets.py" $t 5 > /dev/null
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$out/$t.write" -- python3 "$R/tools/pmc_targets.py" $t 5 > /dev/null
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$out/$t.trace" -- python3 "$R/tools/pmc_targets.py" $t 10 > /dev/null
done
python3 "$R/tools/pmc_summary.py" "$R/$out/frames8.fetch" "$R/$out/frames8.write" "k_frames_apply" 67108864 "$R/$out/frames8.json" 40
python3 "$R/tools/pmc_summary.py" "$R/$out/frames_keyed8.fetch" "$R/$out/frames_keyed8.write" "k_frames_base|k_frames_check|k_frames_apply" 10000000 "$R/$out/frames_keyed8.json" 112
python3 "$R/tools/pmc_summary.py" "$R/$out/frames_cached8.fetch" "$R/$out/frames_cached8.write" "k_frames_apply" 10000000 "$R/$out/frames_cached8.json" 40
