# prefill numerics + 2k-token prefill bench
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-2} | cut -c1-400; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -40 gpurun_out/$name.log; exit 1; }; }
run t_pf 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_runtime_gpu.py tests/test_tp.py -m gpu
TAILN=3 run pf 300 python tools/bench_prefill.py
