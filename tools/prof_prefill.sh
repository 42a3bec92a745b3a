#!/usr/bin/env bash
# rocprofv3 kernel trace of Mistral prefill (tools/bench_prefill.py); per-kernel totals of ONE prefill
# -> gpurun_out/pf_summary.txt.   BENCH_ARGS="--lens 2048" by default.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out/pf
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/pf" -o run --output-format csv -- \
  python3 "$ROOT/tools/bench_prefill.py" ${BENCH_ARGS:---lens 2048} > "$ROOT/gpurun_out/pf/log" 2>&1
cd "$ROOT"
grep '^{' gpurun_out/pf/log | tail -1
python3 - <<'PY' > gpurun_out/pf_summary.txt
import csv
from collections import defaultdict
rows = sorted(csv.DictReader(open("gpurun_out/pf/run_kernel_trace.csv")), key=lambda r: int(r["Start_Timestamp"]))
# the bench runs 1 warm + 3 timed prefills: count kernel time per name over all of them / 4
agg = defaultdict(lambda: [0, 0])
for r in rows:
    n = r["Kernel_Name"].split("(")[0][:80]
    if "fill_random" in n or "repack" in n:
        continue
    agg[n][0] += 1
    agg[n][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
tot = sum(v[1] for v in agg.values())
print(f"kernel time per prefill (1 warm + 3 timed runs averaged): {tot / 4 / 1e6:.2f} ms")
for k, v in sorted(agg.items(), key=lambda x: -x[1][1])[:20]:
    print(f"{v[1] / 4 / 1e3:9.1f} us {v[0] // 4:5d}x  avg {v[1] / max(v[0], 1) / 1e3:8.2f}  {k}")
PY
cat gpurun_out/pf_summary.txt
