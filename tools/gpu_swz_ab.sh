# Skinny GEMM X staging: XOR-swizzled rows (default) vs the padded rows (AIOS_SKINNY_XPAD=1) --
# tests, same-box A/B on bench.py --batch B, and one PMC pass for LDS bank conflicts at B = 32
set -u
cd $GRAFT_REPO_ROOT
ROOT=$PWD
mkdir -p gpurun_out/pmcs
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -1 | cut -c1-200; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -30 gpurun_out/$name.log; exit 1; }; }
run sw_tests 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "batched or gemm or skinny"
for B in 32 16 8 4; do
  AIOS_SKINNY_XPAD=1 run sz_pad_b$B 300 python bench.py --batch $B --steps 32 --warmup 4
  run sz_swz_b$B 300 python bench.py --batch $B --steps 32 --warmup 4
done
AIOS_SKINNY_XPAD=1 run sz_pad2_b32 300 python bench.py --batch 32 --steps 32 --warmup 4
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_MFMA SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_WAVES --kernel-trace -d $ROOT/gpurun_out/pmcs/p1 -o run --output-format csv -- \
    python3 $ROOT/bench.py --batch 32 --steps 4 --warmup 1 --no-graph --no-secondary > $ROOT/gpurun_out/pmcs/p1.log 2>&1 || { echo "pmc failed"; exit 1; }
cd $ROOT && python3 tools/pmc_summary.py gpurun_out/pmcs > gpurun_out/pmcs_summary.txt && grep -A7 "skinny" gpurun_out/pmcs_summary.txt | head -60
