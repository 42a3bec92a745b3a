# batched decode B=2/4/8: skinny MFMA GEMM path (default) vs int8 GEMV path
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bab
export HSA_ENABLE_IPC_MODE_LEGACY=0
for b in 2 4 8; do
  for minb in 2 9; do
    AIOS_DECODE_GEMM_MIN_B=$minb timeout -k 10 200 python bench.py --batch $b --steps 64 --warmup 8 --no-secondary > gpurun_out/bab/b${b}_m${minb}.log 2>&1 || { echo "b=$b minb=$minb failed"; tail -5 gpurun_out/bab/b${b}_m${minb}.log; exit 1; }
    echo "B=$b min_b=$minb $(grep '^{' gpurun_out/bab/b${b}_m${minb}.log | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"
  done
done
