#!/bin/bash
# SQ counters of the C2 signature kernel (variant from SYDELTA_SIG_VARIANT).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
R=$(pwd)
mkdir -p gpurun_out/pmc_sig
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY --kernel-trace -d $R/gpurun_out/pmc_sig/sq -o run --output-format csv -- python3 $R/bench.py --workload c2 --steps 3 --warmup 1 > $R/gpurun_out/pmc_sig/log 2>&1 || { tail $R/gpurun_out/pmc_sig/log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_MISC --kernel-trace -d $R/gpurun_out/pmc_sig/sq2 -o run --output-format csv -- python3 $R/bench.py --workload c2 --steps 3 --warmup 1 >> $R/gpurun_out/pmc_sig/log 2>&1 || { tail $R/gpurun_out/pmc_sig/log; exit 1; }
python3 - <<'PY'
import csv, collections, glob
for f in glob.glob('/root/repo/gpurun_out/pmc_sig/*/run_counter_collection.csv') + glob.glob('gpurun_out/pmc_sig/*/run_counter_collection.csv'):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if 'k_sig' in r['Kernel_Name']:
            agg[r['Counter_Name']].append(float(r['Counter_Value']))
    for k, v in agg.items():
        print(f, k, sum(v) / len(v))
PY
