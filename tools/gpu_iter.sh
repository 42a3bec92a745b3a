# one GPU iteration (used through gpurun): engine tests, batched decode with / without BLAS
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-2}; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -40 gpurun_out/$name.log; exit 1; }; }
run t_eng 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py
for b in 8 16 32 64; do
  TAILN=1 run b$b 200 python bench.py --batch $b --steps 64 --warmup 8 --no-secondary
  AIOS_BLAS_DECODE_MIN_B=8 TAILN=1 run b${b}x 200 python bench.py --batch $b --steps 64 --warmup 8 --no-secondary
done
