# grouped decode attention head-set size: 4 (default) vs 2 (AIOS_ATTN_GL=2), tests + same-box A/B
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -1 | cut -c1-160; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -30 gpurun_out/$name.log; exit 1; }; }
# (the AIOS_ATTN_GL=2 prototype was removed after this A/B: profiles/attn_headset_ab_r2s3.txt)
for P in 128 1024; do
  for B in 32 16; do
    run gl4_b${B}_p$P 300 python bench.py --batch $B --prompt $P --steps 32 --warmup 4
    AIOS_ATTN_GL=2 run gl2_b${B}_p$P 300 python bench.py --batch $B --prompt $P --steps 32 --warmup 4
  done
done
