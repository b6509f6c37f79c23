#!/bin/bash
# Round 3: index allocations reused (kept per device): C3, C5 and C4 (10 callers) legs
# with the library's host timing of the C3 step.
set -u
TAG=${1:-r03ap}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
SYDELTA_HOST_TIMING=1 timeout -k 10 200 python3 scripts/r03_step_host.py > "$OUT/step_host.log" 2>&1 || { tail -20 "$OUT/step_host.log"; exit 1; }
grep rep "$OUT/step_host.log"
for w in c3 c5; do
  timeout -k 10 300 python3 -u bench.py --workload $w --steps 20 --warmup 3 --no-cpu-baseline --no-host-inclusive \
    > "$OUT/$w.json" 2> "$OUT/$w.err" || { tail -20 "$OUT/$w.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/$w.json').read().strip().splitlines()[-1]);print('$w', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 python3 -u bench.py --workload c4 --callers 10 --no-cpu-baseline > "$OUT/c4c10.json" 2> "$OUT/c4c10.err" || { tail -20 "$OUT/c4c10.err"; exit 1; }
python3 -c "import json;d=json.loads(open('$OUT/c4c10.json').read().strip().splitlines()[-1]);print('c4 callers 10', d['value'], d['ms_per_step'])"
echo "== done"
