set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-2}; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -30 gpurun_out/$name.log; exit 1; }; }
run b8 200 python bench.py --batch 8 --steps 64 --warmup 8 --no-secondary
run b4 200 python bench.py --batch 4 --steps 64 --warmup 8 --no-secondary
run b2 200 python bench.py --batch 2 --steps 64 --warmup 8 --no-secondary
run goalplan 400 python tools/bench_goal_plan.py
TAILN=4 run prefill_tl 200 python tools/bench_prefill.py --model tinyllama-1.1b --lens 128,512,2048
