# batch-1 decode attention knobs on the bench (same box): passes per workgroup at 4k context,
# per-head split at 128-token prompts
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -1 | cut -c1-160; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -30 gpurun_out/$name.log; exit 1; }; }
AIOS_ATTN_PPW=1 run ab_ppw1_4k 300 python bench.py --prompt 4000 --steps 64 --warmup 8 --no-secondary
AIOS_ATTN_PPW=2 run ab_ppw2_4k 300 python bench.py --prompt 4000 --steps 64 --warmup 8 --no-secondary
AIOS_ATTN_WG_PER_CU=2 run ab_wg2_4k 300 python bench.py --prompt 4000 --steps 64 --warmup 8 --no-secondary
AIOS_ATTN_SHORT_P=1 run ab_sp1_128 300 python bench.py --steps 128 --warmup 8 --no-secondary
AIOS_ATTN_SHORT_P=2 run ab_sp2_128 300 python bench.py --steps 128 --warmup 8 --no-secondary
