#!/bin/bash
# sampler: numerics / distribution tests, then the service decode profile and goal -> plan / gRPC numbers
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_runtime_gpu.py -x -q --timeout 300 --timeout-method thread -k "sample or sampl" > gpurun_out/samp_tests.log 2>&1 || { tail -40 gpurun_out/samp_tests.log; exit 1; }
tail -n 1 gpurun_out/samp_tests.log
bash tools/gpu_r6_m.sh || exit 1
timeout -k 10 300 python tools/bench_goal_plan.py > gpurun_out/gp.json 2> gpurun_out/gp.err || { tail -20 gpurun_out/gp.err; exit 1; }
head -c 600 gpurun_out/gp.json; echo
