# grouped decode attention at B = 16 / 32: long-mode workgroups per CU (AIOS_ATTN_WG_PER_CU 1 vs 2)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -1 | cut -c1-160; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -30 gpurun_out/$name.log; exit 1; }; }
for P in 128 1024; do
  for B in 32 16; do
    AIOS_ATTN_WG_PER_CU=1 run aw1_b${B}_p$P 300 python bench.py --batch $B --prompt $P --steps 32 --warmup 4
    AIOS_ATTN_WG_PER_CU=2 run aw2_b${B}_p$P 300 python bench.py --batch $B --prompt $P --steps 32 --warmup 4
  done
done
