# GPU iteration for the LDS-DMA decode GEMV: GEMV kernel tests, phase probe, engine tests, bench
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-2}; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -40 gpurun_out/$name.log; exit 1; }; }
run t_gemv 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemv"
TAILN=8 run probe 400 python tools/gemv_cu_probe.py --json gpurun_out/cu_probe.json ${PROBE_ARGS:-}
run t_eng 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py
TAILN=1 run bench 300 python bench.py ${BENCH_ARGS:-}
[ -n "${NOPROF:-}" ] || bash tools/prof_decode.sh > /dev/null
