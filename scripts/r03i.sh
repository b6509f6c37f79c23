#!/bin/bash
# Round 3: k_scan_l2 with level-1 misses masked out of the level-2 loads
# (SYDELTA_SCAN_MASK=1) against out-of-range offsets, and the TA counters of both.
set -u
TAG=${1:-r03i}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp SYDELTA_SCAN_L1=4
cd "$R"
SYDELTA_SCAN_MASK=1 SYDELTA_TEST_SCANNERS=l2 timeout -k 10 600 python3 -u -m pytest tests/test_gpu_scan_large.py -x -q \
  --timeout 300 --timeout-method thread -p no:cacheprovider > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; exit 1; }
tail -1 "$OUT/pytest.log"
for mk in 1 0; do
  SYDELTA_SCAN_MASK=$mk timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-host-inclusive \
    > "$OUT/mask$mk.json" 2> "$OUT/mask$mk.err" || { tail -20 "$OUT/mask$mk.err"; exit 1; }
  python3 -c "import json;d=json.loads(open('$OUT/mask$mk.json').read().strip().splitlines()[-1]);print('mask $mk', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in d['kernels'].items()})"
done
cd /tmp
for mk in 0 1; do
  SYDELTA_SCAN_MASK=$mk timeout -s KILL 90 rocprofv3 --pmc TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum --kernel-trace \
    -d "$OUT/ta$mk" -o run --output-format csv -- python3 "$R/bench.py" --steps 1 --warmup 0 --no-cpu-baseline \
    --no-host-inclusive > "$OUT/ta$mk.log" 2>&1 || { tail -5 "$OUT/ta$mk.log"; break; }
  python3 - "$OUT/ta$mk/run_counter_collection.csv" $mk <<'PY'
import csv, sys, collections
agg = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if 'k_scan' in r['Kernel_Name']:
        agg[r['Counter_Name']].append(float(r['Counter_Value']))
print('mask', sys.argv[2], {k: sum(v) / len(v) for k, v in agg.items()})
PY
done
echo "== done"
