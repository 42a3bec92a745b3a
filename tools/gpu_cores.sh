# co-resident tiers: isolation test + concurrent decode bench
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-2} | cut -c1-600; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -40 gpurun_out/$name.log; exit 1; }; }
run t_cores 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_coresident_gpu.py
TAILN=1 run cores 300 python tools/bench_coresident.py
