# one GPU iteration (used through gpurun): attention tests + probe, engine tests, bench, rocprof summary
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k attention > gpurun_out/t_attn.log 2>&1 || { tail -30 gpurun_out/t_attn.log; exit 1; }
tail -2 gpurun_out/t_attn.log
timeout -k 10 200 python tools/attn_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_engine_gpu.py > gpurun_out/t_eng.log 2>&1 || { tail -30 gpurun_out/t_eng.log; exit 1; }
tail -2 gpurun_out/t_eng.log
timeout -k 10 300 python bench.py --steps 128 --warmup 16 > gpurun_out/bench.log 2>&1 || { tail gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
timeout -k 10 400 bash tools/prof_decode.sh > /dev/null 2>&1 || exit 1
head -12 gpurun_out/prof_summary.txt
