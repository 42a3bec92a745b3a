# prefill kernel-time profile (no counters) + balanced co-resident bench
set -u
cd $GRAFT_REPO_ROOT
ROOT=$PWD
mkdir -p gpurun_out/pf
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 300 python tools/bench_coresident.py > gpurun_out/cores2.log 2>&1 || { echo cores failed; tail -5 gpurun_out/cores2.log; exit 1; }
grep '^{' gpurun_out/cores2.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/gpurun_out/pf -o run --output-format csv -- \
  python3 $ROOT/tools/bench_prefill.py --lens 2048 > $ROOT/gpurun_out/pf/log 2>&1 || { echo prof failed; tail -5 $ROOT/gpurun_out/pf/log; exit 1; }
grep '^{' $ROOT/gpurun_out/pf/log | tail -1
