#!/bin/bash
# fp8 KV numerics + long context, BF16 engine slot/ring sweep, co-resident CU-split sweep
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 400 $T tests/test_kernels_gpu.py -k "fp8_kv or attention_decode or attention_prefill or bf16_engine" > gpurun_out/t_k.log 2>&1 || { tail -40 gpurun_out/t_k.log; exit 1; }
tail -2 gpurun_out/t_k.log
timeout -k 10 400 $T tests/test_engine_gpu.py -k "fp8 or greedy or prefill_logits or paged" > gpurun_out/t_e.log 2>&1 || { tail -40 gpurun_out/t_e.log; exit 1; }
tail -2 gpurun_out/t_e.log
timeout -k 10 300 $T tests/test_coresident_gpu.py > gpurun_out/t_cores.log 2>&1 || { tail -40 gpurun_out/t_cores.log; exit 1; }
tail -2 gpurun_out/t_cores.log
for kv in bf16 fp8_e4m3; do for p in 4000 16000 32000; do
  timeout -k 10 300 python bench.py --steps 128 --warmup 8 --no-secondary --prompt $p --kv-dtype $kv > gpurun_out/lc_${kv}_$p.json 2> gpurun_out/lc.err || { tail -20 gpurun_out/lc.err; exit 1; }
  echo "kv $kv prompt $p: $(grep -o '"value": [0-9.]*' gpurun_out/lc_${kv}_$p.json) $(grep -o '"kv_gb": [0-9.]*' gpurun_out/lc_${kv}_$p.json)"
done; done
timeout -k 10 200 python bench.py --steps 128 --warmup 8 --no-secondary --kv-dtype fp8_e4m3 > gpurun_out/fp8_128.json 2>gpurun_out/lc.err || { tail -20 gpurun_out/lc.err; exit 1; }
echo "kv fp8 prompt 128: $(grep -o '"value": [0-9.]*' gpurun_out/fp8_128.json)"
for c in 23 24 14 16; do
  AIOS_LB_CFG=$c timeout -k 10 200 python bench.py --steps 256 --warmup 16 --no-secondary --model tinyllama-1.1b --recipe BF16 > gpurun_out/lb_$c.json 2>gpurun_out/lb.err || { tail -20 gpurun_out/lb.err; exit 1; }
  echo "LB_CFG=$c $(grep -o '"value": [0-9.]*' gpurun_out/lb_$c.json)"
done
for s in 0 64 96 128; do
  timeout -k 10 300 python tools/bench_coresident.py --steps 512 --cu-split $s > gpurun_out/cores_$s.json 2>gpurun_out/cores.err || { tail -20 gpurun_out/cores.err; exit 1; }
  echo "split $s: $(cat gpurun_out/cores_$s.json)"
done
