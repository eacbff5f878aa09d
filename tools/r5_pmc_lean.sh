#!/bin/bash
# PMC traffic of the lean keyed Push (k_validate_code + k_tile_apply_db) on the
# store layouts DESIGN §5.1 quotes, for bench.py's roofline.traffic.
set -e
R=$GRAFT_REPO_ROOT
for spec in "subset09:PSG_BENCH_SUBSET=0.9:subset0.9" "subset075:PSG_BENCH_SUBSET=0.75:subset0.75" \
            "stretch16:PSG_BENCH_STRETCHES=16:stretch16" "general:PSG_RA_IDENT=0:general"; do
  IFS=: read -r name vars layout <<< "$spec"
  bash "$R/tools/r5_pmc_keyed.sh" gpurun_out/r5_pmc_lean "$name" "$vars" "k_validate_code|k_tile_apply_db"
  python3 - "$R/gpurun_out/r5_pmc_lean/$name.json" "$layout" <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); d["store_layout"] = sys.argv[2]
json.dump(d, open(sys.argv[1], "w"), indent=1)
PY
done
