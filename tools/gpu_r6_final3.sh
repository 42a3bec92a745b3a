#!/bin/bash
# round-6 end validation, part 2: the full bench.py line (all secondaries)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1100 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -30 gpurun_out/bench_final.err; exit 1; }
cat gpurun_out/bench_final.json
