# decode-graph pre-capture: engine/runtime tests, then the 8 / 16-stream serving bench
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -1 | cut -c1-300; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -30 gpurun_out/$name.log; exit 1; }; }
run g_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_runtime_gpu.py tests/test_coresident_gpu.py
run serve8 400 python tools/bench_serving.py --streams 8 --json gpurun_out/serving8.json
run serve16 400 python tools/bench_serving.py --streams 16 --json gpurun_out/serving16.json
