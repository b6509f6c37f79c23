set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s7
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_ACTIVE_INST_VALU --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/s7/sq -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --basis-mib 32 > $GRAFT_REPO_ROOT/gpurun_out/s7/log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_BRANCH SQ_WAVES --kernel-trace -d $GRAFT_REPO_ROOT/gpurun_out/s7/sq2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 0 --no-cpu-baseline --basis-mib 32 >> $GRAFT_REPO_ROOT/gpurun_out/s7/log 2>&1
echo ok
