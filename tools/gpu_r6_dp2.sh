#!/bin/bash
# the driver's multi-GPU bench invocation at N = 2 (both ranks on this box's one GPU: ranks_share_gpu)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 64 --warmup 8 > gpurun_out/dp2.json 2> gpurun_out/dp2.err || { tail -30 gpurun_out/dp2.err; exit 1; }
grep '"metric"' gpurun_out/dp2.json | head -n 1 | cut -c1-600
