#!/bin/bash
# Round 5: fill size of an L2 miss (k_cal_pair) and the calibration kernels' EA requests.
set -uo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 "$R/tools/micro_fetch_cal.hip" -o /tmp/micro_fetch_cal || exit 1
timeout -k 10 120 /tmp/micro_fetch_cal > "$out/counts.txt" 2>&1 || exit 1
P="TCC_EA0_RDREQ_sum TCC_REQ_sum TCC_MISS_sum TCC_HIT_sum"
timeout -k 10 120 rocprofv3 --pmc $P --kernel-trace -d "$out/cal_ea" -o run --output-format csv -- /tmp/micro_fetch_cal \
    > "$out/cal_ea.log" 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$out/pmc_fetch" -o run --output-format csv -- /tmp/micro_fetch_cal \
    > "$out/pmc_fetch.log" 2>&1 || exit 1
echo done
