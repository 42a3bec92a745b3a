#!/usr/bin/env bash
# TP=2 with both ranks sharing the one GPU of a gpurun box: step time (B=1, 4), and rank 0's kernel
# trace (rocprofv3 on rank 0 only; rank 1 runs unprofiled) -> GEMV / attention kernel time vs
# all-reduce kernel time (its spin-wait for the peer included) vs wall.  TP=1 of the same model for
# reference.  Ranks are started from this shell (no launcher re-exec under the profiler).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 MASTER_ADDR=127.0.0.1 WORLD_SIZE=2 LOCAL_RANK=0
M=${MODEL:-mistral-7b}
pair() {  # $1 = port, $2 = batch, $3 = tag, rest = rank-0 command prefix (empty or rocprofv3 ...)
  local port=$1 b=$2 tag=$3; shift 3
  MASTER_PORT=$port RANK=1 timeout -k 10 400 python3 "$ROOT/tools/bench_tp.py" --model $M --steps 64 --warmup 8 \
    --batch $b > "$ROOT/gpurun_out/tp2_${tag}_r1.log" 2>&1 &
  local p1=$!
  (cd /tmp && TMPDIR=/tmp MASTER_PORT=$port RANK=0 timeout -k 10 400 "$@" python3 "$ROOT/tools/bench_tp.py" --model $M \
    --steps 64 --warmup 8 --batch $b > "$ROOT/gpurun_out/tp2_${tag}.log" 2>&1)
  local rc=$?
  wait $p1
  local rc1=$?
  [ $rc -eq 0 ] && [ $rc1 -eq 0 ] || { echo "[$tag] rc=$rc/$rc1"; tail -20 "$ROOT/gpurun_out/tp2_${tag}.log"; exit 1; }
  grep -v amdgpu.ids "$ROOT/gpurun_out/tp2_${tag}.log" | tail -1 | cut -c1-240
}
for b in 1 4; do
  WORLD_SIZE=1 RANK=0 timeout -k 10 400 python3 tools/bench_tp.py --model $M --steps 64 --warmup 8 --batch $b \
    > gpurun_out/tp1_b$b.log 2>&1 || { tail -20 gpurun_out/tp1_b$b.log; exit 1; }
  echo -n "TP=1 B=$b: "; grep -v amdgpu.ids gpurun_out/tp1_b$b.log | tail -1 | cut -c1-200
  pair $((29610 + b)) $b b$b
  pair $((29620 + b)) $b prof_b$b rocprofv3 --kernel-trace --stats -d "$ROOT/gpurun_out/tp2prof_b$b" -o run --output-format csv --
  python3 tools/prof_step.py gpurun_out/tp2prof_b$b/run_kernel_trace.csv > gpurun_out/tp2prof_b$b.txt
  head -16 gpurun_out/tp2prof_b$b.txt
done
