# round validation: every GPU test, smoke(), the B=1 bench, the goal->plan latency bench
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-2} | cut -c1-400; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -40 gpurun_out/$name.log; exit 1; }; }
run t_all 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 run bench 300 python bench.py
TAILN=1 run goal_plan 600 python tools/bench_goal_plan.py
