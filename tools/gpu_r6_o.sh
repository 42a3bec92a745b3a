#!/bin/bash
# PMC of the filtered (top-k / top-p) device sampler
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
ROOT=$PWD
cd /tmp && export TMPDIR=/tmp
export SAMPLE_ONLY="temp0.7 k40 p0.95"
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace -d $ROOT/gpurun_out/pmcs/p$i -o run --output-format csv -- \
    python3 $ROOT/tools/sample_probe.py > $ROOT/gpurun_out/pmcs_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $ROOT/gpurun_out/pmcs_p$i.log; exit 1; }
done
cd $ROOT
python3 - <<'PY'
import csv
from collections import defaultdict
for i in (1, 2):
    acc = defaultdict(float); n = set()
    for r in csv.DictReader(open(f"gpurun_out/pmcs/p{i}/run_counter_collection.csv")):
        if "sample_kernel" not in r["Kernel_Name"]: continue
        acc[r["Counter_Name"]] += float(r["Counter_Value"]); n.add(r["Dispatch_Id"])
    print({k: round(v / len(n)) for k, v in acc.items()})
PY
rm -rf gpurun_out/pmcs
