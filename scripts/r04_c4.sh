#!/bin/bash
# Round 4: where C4's step goes -- host timing of one caller, the phase probe on/off,
# k_scan_r's small mode against k_scan_lds (SYDELTA_SCAN_SMALL=0), 1 and 10 callers.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-r04i_c4}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
leg() {  # name env... -- bench args
  name=$1; shift
  envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 300 python3 -u bench.py --workload c4 --no-cpu-baseline --steps 5 --warmup 2 "$@" \
    > "$OUT/$name.json" 2> "$OUT/$name.err" || { tail -20 "$OUT/$name.err"; exit 1; }
  python3 -c "
import json;d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1])
print('$name', d['ms_per_step'], {k: round(v['avg_ms']*v['launches']/5, 2) for k, v in d.get('kernels', {}).items()})"
}
leg c1_timing SYDELTA_HOST_TIMING=1 -- --callers 1
leg c1_phase SYDELTA_PHASE_PROBE=1 -- --callers 1
leg c1_lds SYDELTA_SCAN_SMALL=0 -- --callers 1
leg c10 X=1 -- --callers 10
leg c10_phase SYDELTA_PHASE_PROBE=1 -- --callers 10
leg c10_lds SYDELTA_SCAN_SMALL=0 -- --callers 10
leg c10_phase_timing SYDELTA_PHASE_PROBE=1 SYDELTA_HOST_TIMING=1 -- --callers 10 --steps 1 --warmup 1
echo "== done"
