// Host-visible argument block for the fused decode GEMV (kernels/gemv.hip).
#pragma once
#include "common.h"
#include "qweight.h"

namespace aios {

constexpr int GEMV_MAX_SEGS = 3;

enum GemvEpilogue : int {
  EPI_STORE = 0,   // y[b][n]  = acc
  EPI_RESID = 1,   // y[b][n] += acc        (residual stream update)
  EPI_SWIGLU = 2,  // y[b][n/2] = silu(acc[2i]) * acc[2i+1]   (rows interleaved gate/up)
  EPI_QKV = 3,     // (+bias) RoPE on Q/K, Q -> y, K/V -> bf16 KV cache at pos[b]
  EPI_TP_RESID = 4,  // TP row-parallel O / down at batch 1: y[n] += sum over ranks of acc (the one-shot
                     //   all-reduce in the row-pair kernel's epilogue, GemvArgs::tp, gemv_q8.h)
};

struct ArDevCtx;  // comm.h

struct GemvArgs {
  QWeight seg[GEMV_MAX_SEGS];   // row-range segments (e.g. Q,K in Q4_K + V in Q6_K)
  int seg_row0[GEMV_MAX_SEGS];  // first global row of each segment (multiples of 8)
  int nseg;
  int N, K, B;
  int row_base;                 // global row of local row 0 (epilogue indexing)
  int kt_max;                   // K tile held in LDS (set by launch_gemv)
  int force_v1;                 // testing: bypass the persistent kernel
  int act_q8;                   // int8-quantised activations (v_dot4) for quantised weights
  int tune_grid;                // blocks per CU override for the persistent kernels (0 = auto)
  int tune_u;                   // chunks per lane per work item override (0 = auto; 1, 2, 4)
  int tune_ksplit;              // -1 disables the K-split decomposition (testing / tuning)
  int tune_dbg;                 // microbenchmarks only: bit0 skip x staging, bit1 skip dot compute
  int kernel_sel;               // testing / probes: 0 = launcher's choice, 1 = row-pair int8 kernel,
                                //   2 = CU register-streaming kernel, 3 = LDS-DMA engine
  unsigned long long* dbg_ts;   // probes: per-workgroup phase timestamps (s_memrealtime) or null
  const float* x;               // [B][ldx] fp32 input (residual stream if norm_w != null)
  int ldx;
  const bf16_t* x16;            // int8-activation kernels only: bf16 input [B][ldx] read instead of x
                                //   (the SwiGLU output handed from gate/up to down at half the bytes)
  const float* norm_w;          // RMSNorm weight [K] or null
  float eps;
  float* y;                     // output, see epilogue
  int ldy;
  bf16_t* y16;                  // EPI_SWIGLU: bf16 output [B][ldy] written instead of y (or null)
  int epi;
  // QKV epilogue
  const float* bias;            // [N] or null
  int head_dim, q_dim, kv_dim, n_kv_heads, max_ctx;
  int rope_neox;
  float rope_base;
  const float2* rope_cs;         // [max_ctx][head_dim/2] (cos, sin) table or null
  const int* pos;               // [B] position of the token being written
  const int* slot;              // [B] KV-cache slot (null -> b)
  bf16_t* k_cache;              // layer base of the paged pool [blocks][n_kv][KV_BLOCK][hd]
  const int* block_table;       // [slots][max_ctx / KV_BLOCK] or null (identity)
  bf16_t* v_cache;
  int kv_fp8;                   // KV pool in fp8 e4m3: stores code = value * kv_inv_{k,v}
  float kv_inv_k, kv_inv_v;
  // batch-1 decode: {pos, physical KV block} and the RoPE (cos, sin) row of this step's position,
  // prepared by the step's embedding launch (StepPrep, ops.h) -- no pos -> block table / rope chain
  // in the QKV kernel (null: looked up from pos / slot / block_table)
  const int* step_kv;
  const float2* step_rope;
  const ArDevCtx* tp;           // EPI_TP_RESID: the XgmiComm device context (XgmiComm::fuse_ctx)
  int grid_cap;                 // EPI_TP_RESID row kernel: workgroups at most (0: no cap; ranks sharing a GPU)
  int dry;                      // EPI_TP_RESID (launch_gemv_tp_fused): only report whether it would launch
};

void launch_gemv(const GemvArgs& a, hipStream_t st);
bool gemv_engine_fits(const GemvArgs& a);  // the B-row LDS-DMA engine serves a (gemv_dispatch.hip)
bool gemv_bf16_engine_fits(const GemvArgs& a);  // the BF16 LDS-DMA engine serves a (gemv_lds16.h)
// EPI_TP_RESID through the row-pair kernel; false = nothing launched (gemv_dispatch.hip)
bool launch_gemv_tp_fused(const GemvArgs& a, hipStream_t st);

}  // namespace aios
