# B=2/4 decode with the new GEMV/GEMM threshold; 4k-context decode with 1 vs 2 attention WGs per CU
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab2
export HSA_ENABLE_IPC_MODE_LEGACY=0
r() { local n=$1; shift; timeout -k 10 300 "$@" > gpurun_out/ab2/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab2/$n.log; exit 1; }; echo "$n $(grep '^{' gpurun_out/ab2/$n.log | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"; }
run_tests() { timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py -m gpu -k "attn or batched or decode" > gpurun_out/ab2/t.log 2>&1 || { echo tests failed; tail -30 gpurun_out/ab2/t.log; exit 1; }; tail -1 gpurun_out/ab2/t.log; }
run_tests
r b8 python bench.py --batch 8 --steps 64 --warmup 8 --no-secondary
r b2 python bench.py --batch 2 --steps 64 --warmup 8 --no-secondary
r b3 python bench.py --batch 3 --steps 64 --warmup 8 --no-secondary
r b4 python bench.py --batch 4 --steps 64 --warmup 8 --no-secondary
r k4_p1 python bench.py --steps 64 --warmup 8 --prompt 4000 --no-secondary
AIOS_ATTN_WG_PER_CU=2 r k4_p2 python bench.py --steps 64 --warmup 8 --prompt 4000 --no-secondary
r k4_p1b python bench.py --steps 64 --warmup 8 --prompt 4000 --no-secondary
