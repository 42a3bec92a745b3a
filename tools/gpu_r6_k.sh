#!/bin/bash
# fp8 long-mode attention: LDS-DMA ring (nt) vs register buffers, interleaved
set -o pipefail
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do for p in 32000 16000; do for nb in 1 0; do
  AIOS_ATTN_NB=$nb timeout -k 10 300 python bench.py --steps 128 --warmup 8 --no-secondary --prompt $p --kv-dtype fp8_e4m3 > gpurun_out/nb.json 2> gpurun_out/nb.err || { tail -20 gpurun_out/nb.err; exit 1; }
  echo "fp8 nb $nb prompt $p: $(grep -o '"value": [0-9.]*' gpurun_out/nb.json)"
done; done; done
# PMC: the fp8 32k decode attention (register-buffer schedule): VALU vs memory vs waits
cd /tmp && export TMPDIR=/tmp
ROOT=$GRAFT_REPO_ROOT
i=0
for grp in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU" \
           "SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  AIOS_ATTN_NB=0 timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace -d $ROOT/gpurun_out/pmca/p$i -o run --output-format csv -- \
    python3 $ROOT/bench.py --prompt 32000 --kv-dtype fp8_e4m3 --steps 4 --warmup 1 --no-graph --no-secondary > $ROOT/gpurun_out/pmca_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $ROOT/gpurun_out/pmca_p$i.log; exit 1; }
  echo "pass $i ok"
done
cd $ROOT && python3 tools/pmc_summary.py gpurun_out/pmca > gpurun_out/pmca_summary.txt && grep -A3 -i "attn_decode\|kernel" gpurun_out/pmca_summary.txt | head -40
