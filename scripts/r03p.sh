#!/bin/bash
# Round 3: k_scan_l2's drain split by ablation (SYDELTA_ABLATE, measurement only: the
# match results are wrong): bit 3 no verification, bit 4 no fat-table lookups (so no
# weak hits), bit 0 no drains, bit 1 no level-2 loads (bits 0/1: phase-timing build only).
set -u
TAG=${1:-r03p}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
for ab in 0 8 16; do
  SYDELTA_ABLATE=$ab timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive \
    > "$OUT/ab$ab.json" 2> "$OUT/ab$ab.err" || { tail -20 "$OUT/ab$ab.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/ab$ab.json').read().strip().splitlines()[-1]);print('ablate $ab', d['kernels']['k_scan_l2']['avg_ms'])"
done
for ab in 0 8 16 1 3; do
  SYDELTA_ABLATE=$ab SYDELTA_PHASE_TIMING=1 timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline \
    --no-host-inclusive > "$OUT/ab${ab}_phase.json" 2> "$OUT/ab${ab}_phase.err" || { tail -20 "$OUT/ab${ab}_phase.err"; exit 1; }
  python3 - "$OUT/ab${ab}_phase.json" "$ab" "$OUT/ab${ab}_phase.err" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ph = [l for l in open(sys.argv[3]) if "phase" in l]
print("timing ablate", sys.argv[2], d["kernels"]["k_scan_l2"]["avg_ms"], "ms |", ph[-1].split("]")[-1].strip() if ph else "")
PY
done
echo "== done"
