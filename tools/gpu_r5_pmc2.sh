#!/bin/bash
# round 5: PMC anatomy of the prefill-GEMM probe variants (gate/up M=2048)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
run() {  # name counters...
  local n=$1; shift
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc2/$n -o $n --output-format csv -- python3 tools/bench_gemm.py --pf-probe --shapes gate_up --ms 2048 --no-torch > gpurun_out/pmc2/$n.log 2>&1
}
run a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS && \
run b SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INSTS_MFMA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT && \
run c SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_VMEM SQ_WAVES
echo rc=$?
