#!/bin/bash
# round-5 secondaries: BASELINE configs 2 (gRPC operational tier) and 4 (co-resident), goal->plan burst
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python tools/bench_grpc.py > gpurun_out/grpc.json 2> gpurun_out/grpc.err || { tail -20 gpurun_out/grpc.err; exit 1; }
cat gpurun_out/grpc.json
timeout -k 10 300 python tools/bench_coresident.py --steps 256 > gpurun_out/cores.json 2> gpurun_out/cores.err || { tail -20 gpurun_out/cores.err; exit 1; }
cat gpurun_out/cores.json
timeout -k 10 400 python tools/bench_goal_plan.py --goals 16 --burst 3 --burst-plan-tokens 300 > gpurun_out/gp.json 2> gpurun_out/gp.err || { tail -20 gpurun_out/gp.err; exit 1; }
cat gpurun_out/gp.json
