# batched-decode path threshold: int8 GEMV vs skinny MFMA GEMM at B = 2 / 3 (same box)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -1 | cut -c1-160; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -30 gpurun_out/$name.log; exit 1; }; }
for B in 2 3; do
  AIOS_DECODE_GEMM_MIN_B=4 run mb_gemv_b$B 300 python bench.py --batch $B --steps 64 --warmup 8
  AIOS_DECODE_GEMM_MIN_B=2 run mb_gemm_b$B 300 python bench.py --batch $B --steps 64 --warmup 8
done
AIOS_DECODE_GEMM_MIN_B=4 run mb_gemv2_b2 300 python bench.py --batch 2 --steps 64 --warmup 8
