#!/usr/bin/env bash
# round 4: TP tests with the fused O / down epilogue (world 2 / 4 / 8 sharing this GPU), then the TP=2
# step with fused vs separate collectives (AIOS_TP_FUSE=1 / 0) and rank 0's kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_tp.py \
  > gpurun_out/t_tp.log 2>&1 || { tail -60 gpurun_out/t_tp.log; exit 1; }
grep -E "PASS|FAIL" gpurun_out/t_tp.log | tail -12
export MASTER_ADDR=127.0.0.1 WORLD_SIZE=2 LOCAL_RANK=0
for f in 0 1; do
  port=$((29640 + f))
  AIOS_TP_FUSE=$f MASTER_PORT=$port RANK=1 timeout -k 10 400 python3 tools/bench_tp.py --model mistral-7b --steps 64 \
    --warmup 8 > gpurun_out/tpf${f}_r1.log 2>&1 &
  p1=$!
  AIOS_TP_FUSE=$f MASTER_PORT=$port RANK=0 timeout -k 10 400 python3 tools/bench_tp.py --model mistral-7b --steps 64 \
    --warmup 8 > gpurun_out/tpf${f}.log 2>&1
  rc=$?; wait $p1; rc1=$?
  [ $rc -eq 0 ] && [ $rc1 -eq 0 ] || { echo "fuse=$f rc=$rc/$rc1"; tail -20 gpurun_out/tpf${f}.log; exit 1; }
  echo -n "AIOS_TP_FUSE=$f: "; grep -v amdgpu.ids gpurun_out/tpf${f}.log | tail -1 | cut -c1-160
done
AIOS_TP_FUSE=1 MASTER_PORT=29650 RANK=1 timeout -k 10 400 python3 "$ROOT/tools/bench_tp.py" --model mistral-7b --steps 64 \
  --warmup 8 > gpurun_out/tpfp_r1.log 2>&1 &
p1=$!
(cd /tmp && TMPDIR=/tmp AIOS_TP_FUSE=1 MASTER_PORT=29650 RANK=0 timeout -k 10 400 rocprofv3 --kernel-trace --stats \
  -d "$ROOT/gpurun_out/tpfprof" -o run --output-format csv -- python3 "$ROOT/tools/bench_tp.py" --model mistral-7b \
  --steps 64 --warmup 8 > "$ROOT/gpurun_out/tpfp.log" 2>&1)
rc=$?; wait $p1; rc1=$?
[ $rc -eq 0 ] && [ $rc1 -eq 0 ] || { echo "prof rc=$rc/$rc1"; tail -20 gpurun_out/tpfp.log; exit 1; }
python3 tools/prof_step.py gpurun_out/tpfprof/run_kernel_trace.csv > gpurun_out/tpfprof.txt
head -16 gpurun_out/tpfprof.txt
