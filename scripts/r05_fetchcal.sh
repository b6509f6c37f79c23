#!/bin/bash
# Round 5: FETCH_SIZE calibration for 4-byte gathers and 16-byte reads (tools/micro_fetch_cal.hip).
set -uo pipefail
tag=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
out=$R/gpurun_out/$tag
mkdir -p "$out"
export TMPDIR=/tmp
cd /tmp
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 "$R/tools/micro_fetch_cal.hip" -o /tmp/micro_fetch_cal || exit 1
timeout -k 10 60 rocprofv3 -L > "$out/counters_list.txt" 2>&1 || true
timeout -k 10 120 /tmp/micro_fetch_cal > "$out/counts.txt" 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$out/pmc_fetch" -o run --output-format csv -- \
    /tmp/micro_fetch_cal > "$out/pmc_fetch.log" 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-trace -d "$out/pmc_ea" -o run \
    --output-format csv -- /tmp/micro_fetch_cal > "$out/pmc_ea.log" 2>&1 || true
timeout -k 10 120 rocprofv3 --pmc TCC_REQ_sum TCC_MISS_sum TCC_HIT_sum --kernel-trace -d "$out/pmc_tcc" -o run \
    --output-format csv -- /tmp/micro_fetch_cal > "$out/pmc_tcc.log" 2>&1 || true
echo done
