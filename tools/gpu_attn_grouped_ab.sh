# Batched decode attention: per-query-head split vs grouped (one K/V read per KV head) mode --
# kernel tests, then a same-box A/B of AIOS_ATTN_GROUPED_MIN on bench.py --batch B
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -1 | cut -c1-200; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -30 gpurun_out/$name.log; exit 1; }; }
run ag_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention_decode"
for B in 32 16 8 4; do
  AIOS_ATTN_GROUPED_MIN=0 run ag_off_b$B 300 python bench.py --batch $B --steps 32 --warmup 4
  AIOS_ATTN_GROUPED_MIN=1 run ag_on_b$B 300 python bench.py --batch $B --steps 32 --warmup 4
done
AIOS_ATTN_GROUPED_MIN=0 run ag_off_b32_p1k 300 python bench.py --batch 32 --prompt 1024 --steps 32 --warmup 4
AIOS_ATTN_GROUPED_MIN=1 run ag_on_b32_p1k 300 python bench.py --batch 32 --prompt 1024 --steps 32 --warmup 4
AIOS_ATTN_GROUPED_MIN=0 run ag_off_b1 300 python bench.py --steps 64 --warmup 8
AIOS_ATTN_GROUPED_MIN=1 run ag_on_b1 300 python bench.py --steps 64 --warmup 8
