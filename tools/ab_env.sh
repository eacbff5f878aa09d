# Interleaved A/B of bench.py under two environment settings.
#   bash tools/ab_env.sh "VAR=a" "VAR=b" ROUNDS [bench.py args...]
# Prints value / push_ms / pull_ms / push256 fracs per run (gpurun_out/ab_env_*.json).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
A=$1; B=$2; R=$3; shift 3
for r in $(seq 1 "$R"); do
  for e in "$A" "$B"; do
    out=gpurun_out/ab_env_${r}_$(echo "$e" | tr -c 'A-Za-z0-9' _).json
    env $e timeout -k 10 200 python3 bench.py --no-cpu-baseline "$@" > "$out" 2> "$out.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "$e rc=$rc"; tail -3 "$out.err"; exit $rc; fi
    python3 - "$out" "$e" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
p = d.get("push256_roofline") or {}
print(f"{sys.argv[2]:28s} value {d['value']:9.1f} push {d.get('push_ms')} pull {d.get('pull_ms')} "
      f"ok {d.get('parity_check')} p256 push {p.get('push_frac')} pull {p.get('pull_frac')}")
PY
  done
done
