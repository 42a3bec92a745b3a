# decode attention: numerics tests, probe, B=1 decode bench at 128 / 4000-token prompts
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-2}; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -40 gpurun_out/$name.log; exit 1; }; }
run t_attn 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attn or attention" tests/test_attn_block_gpu.py tests/test_engine_gpu.py
TAILN=30 run probe 300 python tools/attn_probe.py
TAILN=1 run bench 300 python bench.py --steps 128 --warmup 8
TAILN=1 run bench4k 300 python bench.py --steps 64 --warmup 8 --prompt 4000 --no-secondary
