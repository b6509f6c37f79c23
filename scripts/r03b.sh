#!/bin/bash
# Round 3, second hardware call: the full-size C4/C5 tests, the SQ counters and phase
# cycles of k_scan_l1 at the C3 size, then the bench legs the verdict asked to measure
# (C5 and C4 with the host and the device walk, C4 with 10 callers, the path API at
# 4 GiB, and production block size 65536 on 4 GiB pairs).  Each step under its own
# limit; stops at the first failure.
# Usage (from the repo root on the box): bash scripts/r03b.sh [tag] [legs...]
set -u
TAG=${1:-r03b}; shift || true
LEGS=${*:-tests sq wide legs}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
step() { local t=$1; shift; echo "== $* (limit ${t}s)" >&2; timeout -k 10 "$t" "$@"; local rc=$?; echo "== rc=$rc" >&2; return $rc; }
summ() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(sys.argv[2], d["value"], d["unit"], d["ms_per_step"], "ms/step", r.get("kernel"), r.get("frac"),
      {k: (v["avg_ms"], v["launches"]) for k, v in (d.get("kernels") or {}).items()},
      "cpu", (d.get("cpu_baseline") or {}).get("value"), d.get("match_stats"))
PY
}
leg() { local name=$1; shift; step 400 python3 -u bench.py "$@" > "$OUT/bench_$name.json" 2> "$OUT/bench_$name.err" \
  || { tail -20 "$OUT/bench_$name.err"; return 1; }; summ "$OUT/bench_$name.json" "$name"; }
for L in $LEGS; do
case $L in
tests)
  step 900 python3 -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 600 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_fullsize.log" 2>&1 || { tail -40 "$OUT/pytest_fullsize.log"; exit 1; }
  tail -4 "$OUT/pytest_fullsize.log" ;;
sq)
  SYDELTA_PHASE_TIMING=1 step 200 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-host-inclusive \
    > "$OUT/phase.json" 2> "$OUT/phase.err" || { tail -20 "$OUT/phase.err"; exit 1; }
  grep "phase" "$OUT/phase.err" | tail -1
  cd /tmp
  B="$R/bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-host-inclusive"
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
    SQ_ACTIVE_INST_VALU SQ_INSTS_LDS --kernel-trace -d "$OUT/sq1" -o run --output-format csv -- python3 $B \
    > "$OUT/sq1.log" 2>&1 || { tail "$OUT/sq1.log"; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
    SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE --kernel-trace -d "$OUT/sq2" -o run \
    --output-format csv -- python3 $B > "$OUT/sq2.log" 2>&1 || { tail "$OUT/sq2.log"; exit 1; }
  cd "$R"
  python3 - "$OUT" <<'PY'
import csv, collections, glob, json, sys
out = {}
for f in sorted(glob.glob(sys.argv[1] + '/sq*/run_counter_collection.csv')):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'k_scan_l1' in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
    for k, v in agg.items():
        out[k] = sum(v) / len(v)
json.dump(out, open(sys.argv[1] + '/sq_k_scan_l1.json', 'w'), indent=1)
print(json.dumps(out))
PY
  ;;
wide)
  # first hardware run of k_scan_w: a parity failure (rc 1) keeps the legs on the old
  # kernel (SYDELTA_SCAN_WIDE=0); anything else (fault, timeout) ends the call
  step 600 python3 -u -m pytest tests/test_gpu_scan_wide.py -x -v --timeout 300 --timeout-method thread \
    -p no:cacheprovider > "$OUT/pytest_wide.log" 2>&1
  rc=$?
  tail -6 "$OUT/pytest_wide.log"
  if [ $rc -eq 1 ]; then export SYDELTA_SCAN_WIDE=0; echo "== k_scan_w parity failed: legs on k_scan" >&2;
  elif [ $rc -ne 0 ]; then exit 1; fi ;;
legs)
  # the old wide kernel, for the A/B
  SYDELTA_SCAN_WIDE=0 leg c3_bs64k_kscan --block-size 65536 --steps 2 --warmup 1 --no-cpu-baseline --no-host-inclusive || exit 1
  leg c5_host --workload c5 --steps 10 --warmup 3 --no-cpu-baseline || exit 1
  leg c5_dev --workload c5 --steps 10 --warmup 3 --no-cpu-baseline --device-walk || exit 1
  leg c4_host --workload c4 --steps 5 --warmup 2 --no-cpu-baseline || exit 1
  leg c4_callers10 --workload c4 --steps 5 --warmup 2 --no-cpu-baseline --callers 10 || exit 1
  leg c3_bs64k --block-size 65536 --steps 3 --warmup 1 --no-cpu-baseline --no-host-inclusive || exit 1
  leg c5_bs64k_4g --workload c5 --block-size 65536 --size-gib 4 --steps 5 --warmup 2 --no-cpu-baseline || exit 1
  leg path_4g --workload path --size-gib 4 --steps 3 --warmup 1 || exit 1
  ;;
esac
done
echo "== done"
