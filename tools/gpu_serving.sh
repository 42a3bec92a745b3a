#!/bin/bash
# serving record: 2 / 3 / 4 / 8 concurrent JSON-mode Mistral streams, 3k prompts sharing a 2k prefix
# (the autonomy loop's pattern); one JSON line each into gpurun_out/serving.jsonl
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
: > gpurun_out/serving.jsonl
for n in 2 3 4 8; do
  timeout -k 10 400 python tools/bench_serving.py --streams $n --json gpurun_out/serving$n.json > gpurun_out/serve$n.log 2>&1 || { tail -30 gpurun_out/serve$n.log; exit 1; }
  cat gpurun_out/serving$n.json >> gpurun_out/serving.jsonl; echo >> gpurun_out/serving.jsonl
  python -c "import json;d=json.load(open('gpurun_out/serving$n.json'));print($n, {k:d[k] for k in d if 'itl' in k or 'step' in k or 'ttft' in k or 'tok_s' in k})"
done
