# one GPU iteration (used through gpurun): new-kernel tests, engine tests, prefill + decode bench, profile
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; tail -4 gpurun_out/$name.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -40 gpurun_out/$name.log; exit 1; }; }
run t_new 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemm or prefill or attention"
run t_eng 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py
run prefill 300 python tools/bench_prefill.py --gemv --lens 128,512,2048
run bench 300 python bench.py --steps 128 --warmup 16
