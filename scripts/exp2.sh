set -e
cd $GRAFT_REPO_ROOT
SYDELTA_PHASE_TIMING=1 timeout -k 10 300 python bench.py --workload c4 --files 2000 --steps 1 --warmup 0 --no-cpu-baseline 2>&1 | grep -E "phase" | head -2
SYDELTA_PHASE_TIMING=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-host-inclusive --basis-mib 32 2>&1 | grep -E "phase" | head -1
SYDELTA_PHASE_TIMING=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-host-inclusive 2>&1 | grep -E "phase" | head -1
