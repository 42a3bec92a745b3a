# B=32 regression hunt: the round's reference config (32 steps, 4 warmup) with each new fusion toggled
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab5
export HSA_ENABLE_IPC_MODE_LEGACY=0
r() { local n=$1; shift; timeout -k 10 300 "$@" > gpurun_out/ab5/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab5/$n.log; exit 1; }; echo "$n $(grep '^{' gpurun_out/ab5/$n.log | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"; }
r b32_new python bench.py --batch 32 --steps 32 --warmup 4 --no-secondary
AIOS_ATTN_OUT16=0 r b32_noout16 python bench.py --batch 32 --steps 32 --warmup 4 --no-secondary
AIOS_ATTN_OUT16=0 AIOS_GEMM_QKV_EPI_MAX_B=0 r b32_old python bench.py --batch 32 --steps 32 --warmup 4 --no-secondary
r b16_new python bench.py --batch 16 --steps 32 --warmup 4 --no-secondary
AIOS_ATTN_OUT16=0 AIOS_GEMM_QKV_EPI_MAX_B=0 r b16_old python bench.py --batch 16 --steps 32 --warmup 4 --no-secondary
