# A/B of runtime environment knobs on the B=1 decode bench (same box, back to back)
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/$name.log | tail -1 | cut -c1-200; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -20 gpurun_out/$name.log; exit 1; }; }
run ab_base 300 python bench.py --steps 128 --warmup 8
HIP_FORCE_DEV_KERNARG=1 run ab_devkarg 300 python bench.py --steps 128 --warmup 8
HIP_FORCE_DEV_KERNARG=0 run ab_hostkarg 300 python bench.py --steps 128 --warmup 8
run ab_base2 300 python bench.py --steps 128 --warmup 8
