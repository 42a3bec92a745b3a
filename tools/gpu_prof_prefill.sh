#!/bin/bash
# kernel-time profile of one prefill length: LEN=512 bash tools/gpu_prof_prefill.sh
set -o pipefail
ROOT=$PWD
LEN=${LEN:-512}
OUT=gpurun_out/pf$LEN
mkdir -p $OUT
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $ROOT/$OUT -o run --output-format csv -- \
  python3 $ROOT/tools/bench_prefill.py --lens $LEN > $ROOT/$OUT/log 2>&1 || { echo prof failed; tail -5 $ROOT/$OUT/log; exit 1; }
grep '^{' $ROOT/$OUT/log
cd $ROOT && python3 tools/prof_prefill_table.py $OUT/run_kernel_trace.csv --tokens $LEN | tee $OUT/table.txt
