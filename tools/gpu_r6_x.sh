#!/bin/bash
# one-launch streaming-read speed of light at the Mistral-7B decode matrices' sizes (MiB: O 9.0, QKV 13.5,
# Q6_K down 45.9, gate/up 63.0, Q6_K lm_head 102.5), cold caches, kernel-trace timed
set -o pipefail
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out"
hipcc --offload-arch=gfx950 -O3 -o /tmp/mall_probe "$R/tools/mall_probe.hip" || exit 1
cd /tmp && export TMPDIR=/tmp
SIZES="9.0 13.5 45.9 63.0 102.5"
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/sol" -- /tmp/mall_probe --sol $SIZES > "$R/gpurun_out/sol_run.txt" 2>&1 || { tail -20 "$R/gpurun_out/sol_run.txt"; exit 1; }
f=$(find "$R/gpurun_out/sol" -name '*kernel_trace.csv' | head -n 1)
python "$R/tools/sol_trace.py" "$f" $SIZES | tee "$R/gpurun_out/sol.txt"
