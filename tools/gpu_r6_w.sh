#!/bin/bash
# Infinity Cache probe, memory-tier latency bench, and the batch-1 decode weight-prefetch A/B
# (AIOS_DECODE_PF mask: 1 next QKV, 2 this O, 4 next O, 8 this gate/up head)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
hipcc --offload-arch=gfx950 -O3 -o /tmp/mall_probe tools/mall_probe.hip || exit 1
timeout -k 10 180 /tmp/mall_probe > gpurun_out/mall_probe.txt 2>&1 || { cat gpurun_out/mall_probe.txt; exit 1; }
cat gpurun_out/mall_probe.txt
timeout -k 10 400 python tools/bench_memory.py --calls 300 --entries 2000 --json gpurun_out/memory_tiers.json > gpurun_out/bench_memory.log 2>&1 || { tail -20 gpurun_out/bench_memory.log; exit 1; }
echo "memory bench done"
for rep in 1 2; do for v in "X=0" "AIOS_DECODE_PF=1" "AIOS_DECODE_PF=3" "AIOS_DECODE_PF=5" "AIOS_DECODE_PF=8"; do
  env $v timeout -k 10 300 python bench.py --steps 256 --warmup 16 --no-secondary > gpurun_out/pf.json 2> gpurun_out/pf.err || { tail -20 gpurun_out/pf.err; exit 1; }
  echo "$v: $(grep -o '"value": [0-9.]*' gpurun_out/pf.json | head -1)"
done; done
