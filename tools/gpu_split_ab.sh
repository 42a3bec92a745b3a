# Skinny GEMM split-K choice: round-aware split (AIOS_SKINNY_SPLIT_MODE=1, up to 16 slices) vs the
# old fill-the-chip rule (=0); kernel + engine tests, then a same-box A/B on bench.py --batch B
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -1 | cut -c1-200; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -30 gpurun_out/$name.log; exit 1; }; }
run sp_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "batched or gemm or skinny"
for B in 32 16 4; do
  AIOS_SKINNY_SPLIT_MODE=0 run sp_old_b$B 300 python bench.py --batch $B --steps 32 --warmup 4
  AIOS_SKINNY_SPLIT_MODE=1 run sp_new_b$B 300 python bench.py --batch $B --steps 32 --warmup 4
  AIOS_SKINNY_SPLIT_MODE=1 AIOS_SKINNY_SMAX=8 run sp_new8_b$B 300 python bench.py --batch $B --steps 32 --warmup 4
done
