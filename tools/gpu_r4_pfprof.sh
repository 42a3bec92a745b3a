#!/usr/bin/env bash
# rocprofv3 kernel stats of 8-token prompt prefills, short-chunk fusions off vs on
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
for f in 0 1; do
  AIOS_PREFILL_SHORT_FUSE=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/pfprof_$f" -o run \
    --output-format csv -- python3 "$ROOT/tools/bench_prefill.py" --lens 8 > "$ROOT/gpurun_out/pfprof_$f.log" 2>&1 \
    || { tail -20 "$ROOT/gpurun_out/pfprof_$f.log"; exit 1; }
  echo "== AIOS_PREFILL_SHORT_FUSE=$f"
  grep -v amdgpu.ids "$ROOT/gpurun_out/pfprof_$f.log" | grep prompt_tokens | cut -c1-140
  head -14 "$ROOT/gpurun_out/pfprof_$f/run_kernel_stats.csv" | cut -d, -f1-4 | cut -c1-150
done
