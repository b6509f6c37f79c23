#!/bin/bash
# Several bench.py lines in one GPU call, each under its own time limit; stops at the first
# failure.  Each run is "label;ENV=V ENV2=V2;bench args" (env may be empty); the JSON line goes
# to gpurun_out/<tag>/<label>.json, stderr to <label>.err, a one-line summary to stdout.
# Usage (repo root, on the box): bash scripts/runs.sh <tag> "c4_1250;SYDELTA_HOST_THREADS=2;--workload c4 --files 1250" ...
set -u
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
cd "$R"
for spec in "$@"; do
  IFS=';' read -r label envs args <<< "$spec"
  echo "== $label: env [$envs] args [$args]" >&2
  env $envs timeout -k 10 400 python -u bench.py $args > "$OUT/$label.json" 2> "$OUT/$label.err"
  rc=$?
  if [ $rc -ne 0 ]; then echo "== $label rc=$rc" >&2; tail -20 "$OUT/$label.err"; exit 1; fi
  python - "$OUT/$label.json" "$label" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(sys.argv[2], d["value"], d["unit"], d["ms_per_step"], "ms/step", r.get("kernel"), r.get("frac"),
      {k: v["avg_ms"] for k, v in (d.get("kernels") or {}).items()},
      {k: (d[k]["ms_per_step"], d[k]["value"]) for k in ("c4", "c5") if k in d})
PY
done
echo "== done"
