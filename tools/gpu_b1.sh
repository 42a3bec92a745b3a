# one GPU iteration (used through gpurun): kernel + engine tests, B=1 headline bench, decode profile
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-2}; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -40 gpurun_out/$name.log; exit 1; }; }
run t_kern 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py
run t_eng 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py
TAILN=1 run bench 300 python bench.py ${BENCH_ARGS:-}
[ -n "${NOPROF:-}" ] || bash tools/prof_decode.sh > /dev/null
