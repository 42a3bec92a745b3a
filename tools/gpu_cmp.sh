#!/bin/bash
# same-box A/B of two builds: the tree's .so vs a snapshot in $1 (a copy of aios_amd/ + bench.py)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
CMP=$1; shift
ARGS=${*:-"--steps 128 --warmup 8 --no-secondary"}
j() { grep '^{"metric"' | tail -1 | grep -o '"value": [0-9.]*'; }
for r in 0 1; do
  echo "base $(cd $CMP && timeout -k 10 300 python bench.py $ARGS 2>/dev/null | j)" || exit 1
  echo "new  $(timeout -k 10 300 python bench.py $ARGS 2>/dev/null | j)" || exit 1
done
