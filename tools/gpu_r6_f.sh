#!/bin/bash
# fp8 long-context attention workgroups per CU; Q5_K_M / Q8_0 prefill (fallback GEMM); the full bench.py
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for w in 2 4; do for p in 16000 32000; do
  AIOS_ATTN_WG_PER_CU=$w timeout -k 10 300 python bench.py --steps 128 --warmup 8 --no-secondary --prompt $p --kv-dtype fp8_e4m3 > gpurun_out/wpc.json 2> gpurun_out/lc.err || { tail -20 gpurun_out/lc.err; exit 1; }
  echo "fp8 wg_per_cu $w prompt $p: $(grep -o '"value": [0-9.]*' gpurun_out/wpc.json)"
  AIOS_ATTN_WG_PER_CU=$w timeout -k 10 300 python bench.py --steps 128 --warmup 8 --no-secondary --prompt $p > gpurun_out/wpc.json 2> gpurun_out/lc.err || { tail -20 gpurun_out/lc.err; exit 1; }
  echo "bf16 wg_per_cu $w prompt $p: $(grep -o '"value": [0-9.]*' gpurun_out/wpc.json)"
done; done
for r in Q5_K_M Q8_0; do
  timeout -k 10 300 python tools/bench_prefill.py --recipe $r --lens 512,2048 > gpurun_out/pf_$r.jsonl 2> gpurun_out/pf.err || { tail -20 gpurun_out/pf.err; exit 1; }
  cat gpurun_out/pf_$r.jsonl
done
timeout -k 10 900 python bench.py > gpurun_out/bench_full.json 2> gpurun_out/bench_full.err || { tail -30 gpurun_out/bench_full.err; exit 1; }
cat gpurun_out/bench_full.json
