# skinny GEMM register budget for 3 workgroups per CU (Q4_K, M <= 16) vs the previous build
# (ab_old/: same tree with the default budget), same box, bench.py --batch B
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -1 | cut -c1-160; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -30 gpurun_out/$name.log; exit 1; }; }


for B in 16 8 4; do
  run oc_old_b$B 300 python tools/bench_ab_old.py --batch $B --steps 32 --warmup 4
  run oc_new_b$B 300 python bench.py --batch $B --steps 32 --warmup 4
done
run oc_old2_b16 300 python tools/bench_ab_old.py --batch 16 --steps 32 --warmup 4
run oc_new2_b16 300 python bench.py --batch 16 --steps 32 --warmup 4
