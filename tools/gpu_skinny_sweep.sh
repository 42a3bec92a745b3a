# Skinny GEMM knob sweep on the batched decode bench (same box): split cap, waves per workgroup;
# then a rocprofv3 kernel trace of the B=32 step
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -1 | cut -c1-200; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -30 gpurun_out/$name.log; exit 1; }; }
for B in 32 16 8; do
  run sw_def_b$B 300 python bench.py --batch $B --steps 32 --warmup 4
  AIOS_SKINNY_SMAX=4 run sw_s4_b$B 300 python bench.py --batch $B --steps 32 --warmup 4
  AIOS_SKINNY_SMAX=6 run sw_s6_b$B 300 python bench.py --batch $B --steps 32 --warmup 4
  AIOS_SKINNY_RB=4 run sw_rb4_b$B 300 python bench.py --batch $B --steps 32 --warmup 4
done
BENCH_ARGS="--batch 32" bash tools/prof_decode.sh > /dev/null 2>&1 && head -12 gpurun_out/prof_summary.txt
