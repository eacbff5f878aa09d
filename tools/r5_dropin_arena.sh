#!/bin/bash
# configs[0]'s harness (test_kv_app_benchmark) in process mode with and
# without the pre-faulted shared-memory frame arena, and in thread mode, two
# runs each, with the runtime's stage times (tools/r5_dropin_variants.sh).
out=${1:-gpurun_out/r5_dropin_arena.txt}
tools/r5_dropin_variants.sh "$out" "" "-procs PS_SHM_ARENA_MB=0" "-procs" "-procs PS_SHM_ARENA_MB=512"
