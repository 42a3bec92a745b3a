# QKV epilogue vs qkv_post launch at B=8/16/32 and the prior B=32 reference
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab4
export HSA_ENABLE_IPC_MODE_LEGACY=0
r() { local n=$1; shift; timeout -k 10 300 "$@" > gpurun_out/ab4/$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab4/$n.log; exit 1; }; echo "$n $(grep '^{' gpurun_out/ab4/$n.log | python3 -c 'import json,sys; j=json.loads(sys.stdin.read()); print(j["value"], j["ms_per_step"])')"; }
for b in 8 16 32; do
  r b${b}_epi python bench.py --batch $b --steps 64 --warmup 8 --no-secondary
  AIOS_GEMM_QKV_EPI_MAX_B=0 r b${b}_post python bench.py --batch $b --steps 64 --warmup 8 --no-secondary
done
