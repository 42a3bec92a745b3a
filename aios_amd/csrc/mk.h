// Host-visible argument blocks of the persistent batch-1 decode kernel (kernels/decode_mk.hip).
//
// One launch runs a whole decode step (every layer's QKV -> attention -> O -> gate/up -> down and
// the lm_head) on exactly one 1024-thread workgroup per CU.  The step is a list of stages; every
// CU owns an equal slice of every projection's rows, streams that slice's weight bytes HBM -> LDS
// with LDS-DMA in one uninterrupted ring across all stages (the loader never waits for an
// activation, only for a free ring slot), and stage boundaries are all-to-all hand-offs through
// write-through (sc1) stores + per-XCD sharded arrival counters instead of kernel boundaries.
#pragma once
#include "common.h"
#include "qweight.h"

#include <vector>

namespace aios {

enum MkKind : int { MK_QKV = 0, MK_ATT = 1, MK_O = 2, MK_GU = 3, MK_DOWN = 4, MK_LM = 5 };

struct MkStage {
  int kind;
  int nseg;
  int K;                 // input width of the projection
  int layer;
  QWeight seg[3];        // row segments (QKV: q, k, v -- each split over the CUs on its own)
  int seg_row0[3];       // global output row of each segment's row 0
  int pad_;
  const float* norm_w;   // RMSNorm weight of the input (QKV, GU, LM) or null
  bf16_t* k_cache;       // QKV / ATT: this layer's paged K / V pools
  bf16_t* v_cache;
};

struct MkArgs {
  const MkStage* stages;
  int nstages;
  int d, q_dim, kv_dim, n_heads, n_kv_heads, head_dim, d_ff, vocab;
  float eps, attn_scale;
  const float2* rope_cs;  // [max_ctx][head_dim/2]
  int max_ctx;
  const int* pos;         // [1] position of the token being decoded
  const int* seq_len;     // [1] keys after this step's K/V row is written (pos + 1)
  const int* slot;        // [1]
  const int* block_table; // [slots][max_ctx / KV_BLOCK] (slot-indexed)
  float* x;               // [d] residual stream (row slices owned by their CU; read by all via sc1)
  float* q;               // [n_heads * head_dim]
  float* attn;            // [n_heads * head_dim]
  float* ffb;             // [d_ff] SwiGLU output
  float* logits;          // [vocab]
  float* o_part;          // [n_heads][MK_MAXU][head_dim] attention partials
  float* ml;              // [n_heads][MK_MAXU][2]
  int* cnt;               // [nstages][8 shards] arrival counters, 32 ints apart
  int* tick;              // [n_layers * n_kv_heads] attention tickets, 32 ints apart
  int* done;              // [1] workgroups finished (the last one re-arms every counter)
  int* err;               // [1] a bounded wait gave up (outputs garbage; host raises)
  int n_layers;
  int racc_n;             // LDS row accumulators per CU (most rows any CU owns in a stage)
  int scratch_off;        // LDS byte offset of the staging / attention scratch
  int lds_bytes;
  int timeout_us;         // per wait
  unsigned long long* ts; // probes only: [grid][nstages][8] s_memrealtime stamps (null: off)
  int dbg;                // probes only: bit0 consumers skip the slot dot products, bit1 loaders
                          // issue no DMA (outputs garbage; tools/mk_probe.py --dbg)
};

constexpr int MK_MAXU = 32;  // attention pieces per KV head

// total device bytes of the counter block (cnt + tick + done + err) for a model
inline size_t mk_counter_ints(int nstages, int n_layers, int n_kv_heads) {
  return (size_t)nstages * 8 * 32 + (size_t)n_layers * n_kv_heads * 32 + 64;
}

// true when the persistent kernel serves this model shape (LDS budget, formats, head layout);
// fills a.racc_n / a.scratch_off / a.lds_bytes
bool mk_plan(MkArgs& a, const std::vector<MkStage>& stages_host, int cus);
void launch_decode_mk(const MkArgs& a, int grid, hipStream_t st);
bool mk_format_ok(int qt);

}  // namespace aios
