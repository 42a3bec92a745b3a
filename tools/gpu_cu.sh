# one GPU iteration for the CU-balanced decode GEMV (through gpurun): GEMV kernel tests, engine tests,
# B=1 bench with the new kernel and with the row-pair kernel, decode-step profile
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-2}; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -40 gpurun_out/$name.log; exit 1; }; }
run t_gemv 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "gemv"
run t_eng 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py
TAILN=1 run bench 300 python bench.py ${BENCH_ARGS:-}
AIOS_GEMV_CU=0 TAILN=1 run bench_rows 300 python bench.py --no-secondary
AIOS_GEMV_CU=4 TAILN=1 run bench_d4 300 python bench.py --no-secondary
[ -n "${NOPROF:-}" ] || bash tools/prof_decode.sh > /dev/null
