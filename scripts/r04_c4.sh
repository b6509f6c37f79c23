#!/bin/bash
# Round 4: bench legs with env variants, one JSON line each plus the kernel times per step.
# Usage: bash scripts/r04_c4.sh TAG "name|ENV=V ...|bench args" ...
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
for spec in "$@"; do
  name=${spec%%|*}; rest=${spec#*|}; envs=${rest%%|*}; args=${rest#*|}
  env $envs timeout -k 10 300 python3 -u bench.py --no-cpu-baseline $args > "$OUT/$name.json" 2> "$OUT/$name.err" \
    || { tail -20 "$OUT/$name.err"; exit 1; }
  python3 -c "
import json;d=json.loads(open('$OUT/$name.json').read().strip().splitlines()[-1])
st=d['steps'];print('$name', d['value'], d['ms_per_step'], {k: round(v['avg_ms']*v['launches']/st, 2) for k, v in d.get('kernels', {}).items()})"
done
echo "== done"
