#!/bin/bash
# MFMA busy fraction and LDS bank conflicts of the prefill kernels (Mistral-7B Q4_K_M, 512- and 2048-token
# prefill): one --pmc pass with --kernel-trace (counters only, no sys/runtime trace)
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/pmc6"
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES --kernel-trace \
  -d "$R/gpurun_out/pmc6" -o run --output-format csv -- python3 "$R/tools/bench_prefill.py" --lens 512,2048 > "$R/gpurun_out/pmc6/run.log" 2>&1 || { tail -20 "$R/gpurun_out/pmc6/run.log"; exit 1; }
c=$(find "$R/gpurun_out/pmc6" -name '*counter_collection.csv' | head -n 1)
t=$(find "$R/gpurun_out/pmc6" -name '*kernel_trace.csv' | head -n 1)
python3 "$R/tools/pmc_mfma.py" "$c" "$t" | tee "$R/gpurun_out/pmc6/summary.txt"
