#!/bin/bash
# round 5: memory-path counters of the prefill GEMM probes (gate/up M=2048), with and without DMA
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc3
export TMPDIR=/tmp
run() {
  local n=$1; shift
  timeout -s KILL 180 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc3/$n -o $n --output-format csv -- python3 tools/bench_gemm.py --pf-probe --shapes gate_up --ms 2048 --no-torch > gpurun_out/pmc3/$n.log 2>&1
}
run a TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TCP_PENDING_STALL_CYCLES TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_TA_TCP_STATE_READ && \
run b SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS && \
run c TCC_HIT TCC_MISS GRBM_GUI_ACTIVE TA_DATA_STALLED_BY_TC_CYCLES TCP_LFIFO_STALL_CYCLES TCP_RFIFO_STALL_CYCLES TCP_READ_TAGCONFLICT_STALL_CYCLES
echo rc=$?
