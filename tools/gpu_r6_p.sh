#!/bin/bash
# sampler rewrite: tests, sampler probe, goal -> plan and the BF16 gRPC stream
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_runtime_gpu.py -x -q --timeout 300 --timeout-method thread -k "sample or sampl or pipelin" > gpurun_out/samp_tests.log 2>&1 || { tail -40 gpurun_out/samp_tests.log; exit 1; }
tail -n 1 gpurun_out/samp_tests.log
timeout -k 10 300 python tools/sample_probe.py > gpurun_out/sprobe.jsonl 2>&1 || { tail -20 gpurun_out/sprobe.jsonl; exit 1; }
cut -c1-70 gpurun_out/sprobe.jsonl
timeout -k 10 300 python tools/bench_goal_plan.py > gpurun_out/gp.json 2> gpurun_out/gp.err || { tail -20 gpurun_out/gp.err; exit 1; }
head -c 700 gpurun_out/gp.json; echo
timeout -k 10 300 python tools/bench_grpc.py > gpurun_out/grpc.json 2> gpurun_out/grpc.err || { tail -20 gpurun_out/grpc.err; exit 1; }
cat gpurun_out/grpc.json | head -c 900; echo
