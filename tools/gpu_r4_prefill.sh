#!/usr/bin/env bash
# round-4: hipBLASLt prefill (numerics + speed arms) and TinyLlama per-kernel profiles, round-3 tree vs
# this one.  Every GPU step under its own limit; stop at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests -k "prefill" \
  > gpurun_out/t_prefill.log 2>&1 || { tail -40 gpurun_out/t_prefill.log; exit 1; }
tail -1 gpurun_out/t_prefill.log
for b in 0 1; do
  echo "AIOS_PREFILL_BLAS=$b"
  AIOS_PREFILL_BLAS=$b timeout -k 10 300 python tools/bench_prefill.py --lens 128,256,512,1024,2048 > gpurun_out/pf_$b.log 2>&1 \
    || { tail -20 gpurun_out/pf_$b.log; exit 1; }
  grep -v amdgpu.ids gpurun_out/pf_$b.log | cut -c1-200
done
(cd cmp_r3 && MODEL=tinyllama-1.1b timeout -k 10 700 bash tools/prof_decode.sh > /dev/null 2>&1) || { echo "r3 prof failed"; exit 1; }
cp cmp_r3/gpurun_out/prof_summary.txt gpurun_out/prof_tl_r3.txt
MODEL=tinyllama-1.1b timeout -k 10 700 bash tools/prof_decode.sh > /dev/null 2>&1 || { echo "prof failed"; tail -20 gpurun_out/prof.log; exit 1; }
cp gpurun_out/prof_summary.txt gpurun_out/prof_tl_r4.txt
head -14 gpurun_out/prof_tl_r3.txt; head -14 gpurun_out/prof_tl_r4.txt
