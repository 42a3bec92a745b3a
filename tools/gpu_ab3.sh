# batched decode with the QKV-epilogue skinny GEMM: numerics + B=4/8/16 bench
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab3
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_runtime_gpu.py tests/test_kernels_gpu.py tests/test_tp.py -m gpu > gpurun_out/ab3/t.log 2>&1 || { echo tests failed; tail -30 gpurun_out/ab3/t.log; exit 1; }
tail -1 gpurun_out/ab3/t.log
r() { local n=$1; shift; timeout -k 10 300 "$@" > gpurun_out/ab3/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab3/$n.log; exit 1; }; echo "$n $(grep '^{' gpurun_out/ab3/$n.log | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"; }
r b4 python bench.py --batch 4 --steps 64 --warmup 8 --no-secondary
r b8 python bench.py --batch 8 --steps 64 --warmup 8 --no-secondary
r b16 python bench.py --batch 16 --steps 64 --warmup 8 --no-secondary
r b32 python bench.py --batch 32 --steps 64 --warmup 8 --no-secondary
