# PMC counters of the batched-decode step (bench.py --batch 32, eager), one counter group per pass
set -u
cd $GRAFT_REPO_ROOT
ROOT=$PWD
mkdir -p gpurun_out/pmc
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d $ROOT/gpurun_out/pmc/p$i -o run --output-format csv -- \
    python3 $ROOT/bench.py --batch 32 --steps 4 --warmup 1 --no-graph --no-secondary > $ROOT/gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $ROOT/gpurun_out/pmc/p$i.log; exit 1; }
  echo "pass $i ok"
done
cd $ROOT && python3 tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc_summary.txt && head -60 gpurun_out/pmc_summary.txt
