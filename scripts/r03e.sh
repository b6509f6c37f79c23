#!/bin/bash
# Round 3: where k_scan_l1's time goes, by ablation (SYDELTA_ABLATE, measurement only:
# the match results are wrong): bit 0 no drains, bit 1 no level-2 loads, bit 2 no window
# phase.  C3 kernel time and phase cycles per variant.
set -u
TAG=${1:-r03e}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
for ab in 0 1 2 3 4 7; do
  SYDELTA_ABLATE=$ab timeout -k 10 200 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-host-inclusive \
    > "$OUT/ab$ab.json" 2> "$OUT/ab$ab.err" || { tail -20 "$OUT/ab$ab.err"; exit 1; }
  SYDELTA_ABLATE=$ab SYDELTA_PHASE_TIMING=1 timeout -k 10 200 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline \
    --no-host-inclusive > "$OUT/ab${ab}_phase.json" 2> "$OUT/ab${ab}_phase.err" || { tail -20 "$OUT/ab${ab}_phase.err"; exit 1; }
  python3 - "$OUT/ab$ab.json" "$ab" "$OUT/ab${ab}_phase.err" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ph = [l for l in open(sys.argv[3]) if "phase" in l]
print("ablate", sys.argv[2], "k_scan_l1", d["kernels"]["k_scan_l1"]["avg_ms"], "ms |", ph[-1].split("]")[-1].strip() if ph else "")
PY
done
echo "== done"
