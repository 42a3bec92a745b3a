#!/bin/bash
# fp8 KV attention with 16 dims per lane (hd 128): numerics + long context; co-resident priority streams
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
T="python -u -m pytest -x -q --timeout 240 --timeout-method thread"
timeout -k 10 600 $T tests/test_kernels_gpu.py -k "fp8_kv or attention_decode or rmsnorm or tail_split_ragged or production_shapes or stream_k or gemm_pf" > gpurun_out/t_k.log 2>&1 || { tail -40 gpurun_out/t_k.log; exit 1; }
tail -2 gpurun_out/t_k.log
timeout -k 10 400 $T tests/test_engine_gpu.py -k "fp8" > gpurun_out/t_e.log 2>&1 || { tail -40 gpurun_out/t_e.log; exit 1; }
tail -2 gpurun_out/t_e.log
timeout -k 10 300 python tools/bench_prefill.py --lens 128,512,2048 > gpurun_out/pf.jsonl 2> gpurun_out/pf.err || { tail -20 gpurun_out/pf.err; exit 1; }
cat gpurun_out/pf.jsonl
AIOS_GEMM_PF_SK=0 timeout -k 10 300 python tools/bench_prefill.py --lens 512 > gpurun_out/pf_nosk.jsonl 2> gpurun_out/pf.err || { tail -20 gpurun_out/pf.err; exit 1; }
cat gpurun_out/pf_nosk.jsonl
for kv in fp8_e4m3 bf16; do for p in 4000 16000 32000; do
  timeout -k 10 300 python bench.py --steps 128 --warmup 8 --no-secondary --prompt $p --kv-dtype $kv > gpurun_out/lc_${kv}_$p.json 2> gpurun_out/lc.err || { tail -20 gpurun_out/lc.err; exit 1; }
  echo "kv $kv prompt $p: $(grep -o '"value": [0-9.]*' gpurun_out/lc_${kv}_$p.json)"
done; done
BENCH_ARGS="--prompt 32000 --kv-dtype fp8_e4m3" timeout -k 10 700 bash tools/prof_decode.sh > /dev/null 2>&1 || { tail -20 gpurun_out/prof.log; exit 1; }
cp gpurun_out/prof_summary.txt gpurun_out/prof_mistral_32k_fp8.txt
head -14 gpurun_out/prof_mistral_32k_fp8.txt
for pr in mistral tinyllama; do
  timeout -k 10 300 python tools/bench_coresident.py --steps 512 --priority $pr > gpurun_out/cores_p_$pr.json 2>gpurun_out/cores.err || { tail -20 gpurun_out/cores.err; exit 1; }
  echo "priority $pr: $(cat gpurun_out/cores_p_$pr.json)"
done
