# fused attention block: correctness vs the three-launch path, then the B=1 decode bench per mode
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-2}; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -40 gpurun_out/$name.log; exit 1; }; }
run t_fuse 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_attn_block_gpu.py
run t_eng 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_runtime_gpu.py
for m in 0 1 2; do TAILN=1 AIOS_FUSE_ATTN=$m run bench_f$m 300 python bench.py --steps 128 --warmup 8; done
for m in 0 1 2; do TAILN=1 AIOS_FUSE_ATTN=$m run bench4k_f$m 300 python bench.py --steps 64 --warmup 8 --prompt 4000 --no-secondary; done
