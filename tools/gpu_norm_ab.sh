# Split-RMSNorm fusion in the batched-decode GEMMs: correctness tests, then a same-box A/B of
# AIOS_GEMM_NORM_FUSE on the Mistral-7B Q4_K_M batched decode bench (B = 4, 16, 32)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -1 | cut -c1-300; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -30 gpurun_out/$name.log; exit 1; }; }
run nrm_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py -k "batched or graph or greedy"
for B in 16 32 4; do
  AIOS_GEMM_NORM_FUSE=0 run nrm_off_b$B 300 python bench.py --batch $B --steps 32 --warmup 4
  AIOS_GEMM_NORM_FUSE=1 run nrm_on_b$B 300 python bench.py --batch $B --steps 32 --warmup 4
done
AIOS_GEMM_NORM_FUSE=0 run nrm_off2_b16 300 python bench.py --batch 16 --steps 32 --warmup 4
AIOS_GEMM_NORM_FUSE=1 run nrm_on2_b16 300 python bench.py --batch 16 --steps 32 --warmup 4
