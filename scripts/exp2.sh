set -e
cd $GRAFT_REPO_ROOT
SYDELTA_PHASE_TIMING=1 timeout -k 10 300 python bench.py --steps 1 --warmup 0 --no-cpu-baseline --basis-mib 32 2>&1 | grep -v amdgpu.ids | cut -c1-300
