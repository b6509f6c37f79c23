#!/bin/bash
# C3 scan ablations (SYDELTA_ABLATE, measurement only: the results are wrong on purpose)
# for both level-1 layouts: bit 0 = no drains, bit 1 = no level-2 loads (so no passes).
set -u
TAG=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$R"
for l1 in ribbon bloom; do
  for ab in 0 1 3; do
    SYDELTA_L1=$l1 SYDELTA_ABLATE=$ab timeout -k 10 200 python3 -u bench.py --workload c3 --steps 8 --warmup 2 --no-cpu-baseline --no-host-inclusive > "$OUT/${l1}_ab$ab.json" 2> "$OUT/${l1}_ab$ab.err" || { tail -20 "$OUT/${l1}_ab$ab.err"; exit 1; }
    python3 -c "import json;d=json.loads(open('$OUT/${l1}_ab$ab.json').read().strip().splitlines()[-1]);print('$l1 ablate $ab', d['ms_per_step'], d['kernels']['k_scan_r'])"
  done
done
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum --kernel-trace -d "$OUT/tcc" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-host-inclusive --steps 2 --warmup 1 > "$OUT/tcc.log" 2>&1 || { tail "$OUT/tcc.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --kernel-trace -d "$OUT/sq" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-host-inclusive --steps 2 --warmup 1 > "$OUT/sq.log" 2>&1 || { tail "$OUT/sq.log"; exit 1; }
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH --kernel-trace -d "$OUT/sq2" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline --no-host-inclusive --steps 2 --warmup 1 > "$OUT/sq2.log" 2>&1 || { tail "$OUT/sq2.log"; exit 1; }
cd "$R"
python3 - "$OUT" <<'PY'
import csv, collections, glob, sys, json
out = {}
for f in sorted(glob.glob(sys.argv[1] + '/*/run_counter_collection.csv')):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'k_scan_r' in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
    for k, v in agg.items():
        out[k] = sum(v) / len(v)
print(json.dumps(out, indent=1))
json.dump(out, open(sys.argv[1] + '/k_scan_r_counters.json', 'w'), indent=1)
PY
rm -rf "$OUT/tcc" "$OUT/sq" "$OUT/sq2"
echo "== done"
