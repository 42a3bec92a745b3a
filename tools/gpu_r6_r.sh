#!/bin/bash
# prefill QKV epilogue auto mode: engine prefill tests, then prefill A/B (auto vs off)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -k "prefill" > gpurun_out/eng_pf.log 2>&1 || { tail -40 gpurun_out/eng_pf.log; exit 1; }
tail -n 1 gpurun_out/eng_pf.log
for m in 2 0 2 0; do
  AIOS_PREFILL_QKV_EPI=$m timeout -k 10 300 python tools/bench_prefill.py --lens 128,512,2048 > gpurun_out/pfq.jsonl 2> gpurun_out/pfq.err || { tail -20 gpurun_out/pfq.err; exit 1; }
  echo "qkv_epi=$m: $(grep -o '"prompt_tokens": [0-9]*, "ms": [0-9.]*' gpurun_out/pfq.jsonl | tr '\n' ' ')"
done
