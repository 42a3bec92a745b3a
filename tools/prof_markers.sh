#!/usr/bin/env bash
# rocprofv3 marker (roctx) + kernel trace of a prefill + decode run; summary of the engine's
# host-side phases -> gpurun_out/markers_summary.txt
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --stats -d "$ROOT/gpurun_out/mprof" -o run --output-format csv -- \
  python3 "$ROOT/bench.py" --steps 16 --warmup 2 --no-secondary --prompt 512 > "$ROOT/gpurun_out/mprof.log" 2>&1
cd "$ROOT"
python3 - <<'PY' > gpurun_out/markers_summary.txt
import csv, glob, collections
f = glob.glob("gpurun_out/mprof/*marker_api_trace.csv")
rows = list(csv.DictReader(open(f[0]))) if f else []
agg = collections.defaultdict(list)
for r in rows:
    try:
        agg[r.get("Message") or r.get("Function")].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    except Exception:
        pass
print(f"{'range':34s} {'calls':>6s} {'mean_us':>10s} {'total_us':>10s}")
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{str(k)[:34]:34s} {len(v):6d} {sum(v) / len(v):10.1f} {sum(v):10.1f}")
PY
cat gpurun_out/markers_summary.txt
