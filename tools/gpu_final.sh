# round-end validation: every GPU test, smoke(), bench (driver defaults), rocprofv3 decode profile
set -u
cd $GRAFT_REPO_ROOT
ROOT=$PWD
mkdir -p gpurun_out/final
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() { local name=$1 t=$2; shift 2; timeout -k 10 $t "$@" > gpurun_out/final/$name.log 2>&1; local rc=$?; grep -v amdgpu.ids gpurun_out/final/$name.log | tail -${TAILN:-2} | cut -c1-400; [ $rc -eq 0 ] || { echo "[$name] rc=$rc"; tail -40 gpurun_out/final/$name.log; exit 1; }; }
run t_all 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests -m gpu
run smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
TAILN=1 run bench 300 python bench.py
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/final/prof -o run --output-format csv -- \
  python3 $ROOT/bench.py --steps 32 --warmup 4 --no-secondary > $ROOT/gpurun_out/final/prof.log 2>&1 || { echo prof failed; exit 1; }
cd $ROOT
python3 tools/prof_step.py gpurun_out/final/prof/run_kernel_trace.csv > gpurun_out/final/prof_summary.txt
head -14 gpurun_out/final/prof_summary.txt
