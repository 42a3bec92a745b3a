# refresh the serving / co-resident records: 8 and 16 concurrent JSON-mode Mistral streams with
# 3k prompts sharing a 2k prefix, and the co-resident TinyLlama + Mistral bench
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -${TAILN:-1} | cut -c1-600; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -30 gpurun_out/$name.log; exit 1; }; }
run serve8 400 python tools/bench_serving.py --streams 8 --json gpurun_out/serving8.json
run serve16 400 python tools/bench_serving.py --streams 16 --json gpurun_out/serving16.json
run cores 300 python tools/bench_coresident.py
