#!/bin/bash
# BF16 engine slot/ring sweep, co-resident CU-split sweep, masked-tier numerics
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 300 $T tests/test_coresident_gpu.py > gpurun_out/t_cores.log 2>&1 || { tail -40 gpurun_out/t_cores.log; exit 1; }
tail -2 gpurun_out/t_cores.log
timeout -k 10 300 $T tests/test_kernels_gpu.py -k "bf16_engine" > gpurun_out/t_bf16.log 2>&1 || { tail -40 gpurun_out/t_bf16.log; exit 1; }
tail -2 gpurun_out/t_bf16.log
for c in 23 24 14 16 23; do
  AIOS_LB_CFG=$c timeout -k 10 200 python bench.py --steps 256 --warmup 16 --no-secondary --model tinyllama-1.1b --recipe BF16 > gpurun_out/lb_$c.json 2>gpurun_out/lb.err || { tail -20 gpurun_out/lb.err; exit 1; }
  echo "LB_CFG=$c $(grep -o '"value": [0-9.]*' gpurun_out/lb_$c.json)"
done
for s in 0 64 96 128; do
  timeout -k 10 300 python tools/bench_coresident.py --steps 512 --cu-split $s > gpurun_out/cores_$s.json 2>gpurun_out/cores.err || { tail -20 gpurun_out/cores.err; exit 1; }
  echo "split $s: $(cat gpurun_out/cores_$s.json)"
done
