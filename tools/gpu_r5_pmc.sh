#!/bin/bash
# round 5: PMC counters of one prefill-GEMM shape (gate/up M=2048 by default)
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
SHAPE=${SHAPE:-gate_up}; MS=${MS:-2048}
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters.txt 2>&1 || true
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS -d gpurun_out/pmc/p1 -o p1 --output-format csv -- python3 tools/bench_gemm.py --shapes $SHAPE --ms $MS --no-torch > gpurun_out/pmc/p1.log 2>&1
echo "pmc1 rc=$?"
