#!/bin/bash
# round-6 validation: every GPU test, smoke(), the full bench.py line (all secondaries)
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 1500 python -u -m pytest -x -q --timeout 900 --timeout-method thread -m gpu tests > gpurun_out/t_final.log 2>&1 || { tail -40 gpurun_out/t_final.log; exit 1; }
tail -n 1 gpurun_out/t_final.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -n 1 gpurun_out/smoke.log
timeout -k 10 1100 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err || { tail -30 gpurun_out/bench_final.err; exit 1; }
cat gpurun_out/bench_final.json
