// Host launchers for every device op of the engine (one header so the engine, the bindings and
// the tests see the same signatures).  All launchers are stream-ordered and capture-safe: no
// allocation, no synchronisation (CDNA guide §6 Guideline 9), so the decode step can be captured
// into a hipGraph.
#pragma once
#include "common.h"
#include <vector>
#include "gemv.h"
#include "qweight.h"

namespace aios {

// ---- weights -------------------------------------------------------------------------------
void launch_repack(int qt, const void* raw, size_t nblocks, const QWeight& w, hipStream_t st);
void launch_get_rows(const QWeight& w, const int* rows, int nrows, float* out, int ldo, float scale,
                     hipStream_t st);
// Per-step lookups the batch-1 QKV epilogue needs, done by the step's first (embedding) launch while
// it gathers the rows: kv[b] = {pos[b], physical KV block of (slot[b], pos[b])}, rope[b][:] = the
// (cos, sin) row of pos[b].  Every layer's QKV GEMV then loads them with no dependent round trip.
struct StepPrep {
  const int* pos;          // [B]
  const int* slot;         // [B] or null (row b)
  const int* block_table;  // [slots][maxb] or null (identity)
  int maxb;
  const float2* rope_cs;   // [max_ctx][half] or null (no rope rows)
  int half;
  int* kv;                 // out [B][2]
  float2* rope;            // out [B][half]
};
void launch_get_rows_step(const QWeight& w, const int* rows, int nrows, float* out, int ldo, float scale,
                          const StepPrep& prep, hipStream_t st);
void launch_dequant_bf16(const QWeight& w, void* out, hipStream_t st);
void launch_legacy_to_bf16(int qt, const void* raw, size_t n, void* out, hipStream_t st);
void fill_random_weight(const QWeight& w, uint64_t seed, float amp, hipStream_t st);
void fill_random_f32(float* p, size_t n, uint64_t seed, float base, float amp, hipStream_t st);
bool gemv_supports(int qt0, int qt1);

// ---- elementwise / norms ---------------------------------------------------------------------
// y[b] = x[b] * rsqrt(mean(x^2)+eps) * w     (rows of length n, row strides ldx/ldy)
void launch_rmsnorm(const float* x, int ldx, const float* w, float* y, int ldy, int rows, int n, float eps,
                    hipStream_t st);
// same, bf16 output (GEMM A operand)
void launch_rmsnorm_bf16(const float* x, int ldx, const float* w, bf16_t* y, int ldy, int rows, int n, float eps,
                         hipStream_t st);
void launch_f32_to_bf16(const float* x, bf16_t* y, size_t n, hipStream_t st);
void launch_add(float* y, const float* x, size_t n, hipStream_t st);

// Producer side of the split RMSNorm after a TP all-reduce (the skinny GEMM's nrm_in contract,
// GemmQArgs below): out16[m][:] = bf16(x_new[m][:] * g) and part[m * parts + j] = sum of x_new^2 over
// the j-th 1024-column block of row m (parts = round_up(d / 1024, 4) <= 64, the tail parts zero).
constexpr int RNORM_COLS = 1024;
struct ResidNorm {
  const float* g;   // [d] RMSNorm weight of the consumer
  bf16_t* out16;    // [rows][ld16]
  int ld16;
  float* part;      // [rows][parts]
  int parts;
};
inline int resid_norm_parts(int d) { return d % RNORM_COLS ? 0 : ((d / RNORM_COLS + 3) & ~3); }
// residual[m][:] += data[m][:] (data may be null: residual already holds the sum), then the outputs above
void launch_add_norm(float* residual, const float* data, int rows, int d, const ResidNorm& nm, hipStream_t st);

// out[b][i] = silu(gu[b][2i]) * gu[b][2i+1]
void launch_swiglu_interleaved(const float* gu, int ldg, float* out, int ldo, int rows, int n, hipStream_t st);
void launch_swiglu_interleaved_bf16(const float* gu, int ldg, bf16_t* out, int ldo, int rows, int n, hipStream_t st);

// Per-head: optional RMSNorm(q/k heads) + RoPE + Q store + K/V cache write, from a packed
// qkv row [B][q_dim + 2 kv_dim] (used for Qwen3 QK-norm and the prefill GEMM path).
struct QkvPostArgs {
  const float* qkv;  // [T][ldqkv]
  int ldqkv;
  int T;
  int n_heads, n_kv_heads, head_dim;
  const float* bias = nullptr;  // [q_dim + 2 kv_dim] or null (added before norm / RoPE)
  const float* q_norm;  // [head_dim] or null
  const float* k_norm;
  float eps;
  int rope_neox;
  float rope_base;
  const float2* rope_cs;  // [max_ctx][head_dim/2] table or null
  const int* pos;    // [T]
  const int* slot;   // [T] or null (0)
  float* q_out;      // [T][n_heads*head_dim]
  bf16_t* k_cache;   // layer base of the paged pool [blocks][n_kv][KV_BLOCK][hd]
  bf16_t* v_cache;
  int max_ctx;
  const int* block_table = nullptr;  // [slots][max_ctx / KV_BLOCK] or null (identity)
  int kv_fp8 = 0;    // fp8 e4m3 pool: code = value * kv_inv_{k,v}
  float kv_inv_k = 1.f, kv_inv_v = 1.f;
};
void launch_qkv_post(const QkvPostArgs& a, hipStream_t st);

// ---- attention ---------------------------------------------------------------------------------
struct AttnDecodeArgs {
  const float* q;          // [B][n_heads][head_dim]
  const bf16_t* k_cache;   // layer base of the paged pool [blocks][n_kv][KV_BLOCK][hd]
  const bf16_t* v_cache;
  const int* block_table = nullptr;  // [slots][max_ctx / KV_BLOCK] or null (identity)
  int bt_rows = 0;         // block_table indexed by row b instead of slot[b]
  const int* seq_len;      // [B] number of valid keys (pos+1)
  const int* slot;         // [B] or null
  int B, n_heads, n_kv_heads, head_dim, max_ctx;
  int n_chunks;            // grid chunks (>= ceil(max_len / ATTN_CHUNK))
  int split;               // keys per workgroup (multiple of ATTN_CHUNK); 0 -> chosen by the launcher
  float scale;
  float* o_part;           // [B][n_heads][n_chunks][hd]
  float* ml;               // [B][n_heads][n_chunks][2]
  float* out;              // [B][n_heads*hd]
  bf16_t* out16 = nullptr; // if set: the output as bf16 instead (the batched-decode GEMM's A operand)
  int short_len = -1;      // contexts up to this many keys split by query head (-1: launcher decides)
  int* counters;           // [B][n_kv_heads] arrival tickets, zero-initialised, self re-arming
  unsigned long long* ts = nullptr;  // probes: [grid][8] s_memrealtime phase stamps (tools/attn_probe.py --stamps)
  int kv_nt = -1;          // long mode: K/V loads with the streaming (nt) policy (-1: AIOS_ATTN_NT, default 1)
  int kv_tail = -1;        // last partial block: loads only for live keys (-1: AIOS_ATTN_TAIL, default 1)
  int combine_trips = 0;   // split-K combine: 0 = launcher (AIOS_ATTN_COMBINE, default one round trip), 2 = two
  int out_wt = 0;          // fp32 out with write-through (agent-scope) stores
  int kv_fp8 = 0;          // fp8 e4m3 pool: value = code * kv_scale_{k,v}
  float kv_scale_k = 1.f, kv_scale_v = 1.f;
};
constexpr int ATTN_CHUNK = 64;
void launch_attn_decode(const AttnDecodeArgs& a, hipStream_t st);
struct GemvArgs;
int attn_decode_split(int max_ctx, int B, int n_kv_heads);

// causal flash attention for a prefill chunk of T tokens at positions [start, start+T) of one
// slot, over the cached keys [0, start+T) (MFMA; kernels/attention_prefill.hip)
struct AttnPrefillArgs {
  const float* q;          // [T][n_heads][head_dim] (RoPE applied)
  const bf16_t* k_cache;   // layer base of the paged pool [blocks][n_kv][KV_BLOCK][hd]
  const bf16_t* v_cache;
  const int* block_table = nullptr;  // [slots][max_ctx / KV_BLOCK] or null (identity)
  int slot, start, T;
  int n_heads, n_kv_heads, head_dim, max_ctx;
  float scale;
  bf16_t* out;             // [T][ldo] bf16
  int ldo;
  int kv_fp8 = 0;          // fp8 e4m3 pool: value = code * kv_scale_{k,v}
  float kv_scale_k = 1.f, kv_scale_v = 1.f;
};
void launch_attn_prefill(const AttnPrefillArgs& a, hipStream_t st);
bool attn_prefill_supports(int n_heads, int n_kv_heads, int head_dim);  // keys per workgroup the launcher picks

// ---- sampling ---------------------------------------------------------------------------------
// per row b: token[b] = argmax(logits[b])   (temperature[b] > 0 -> Gumbel-max sample from
// softmax(logits / T) restricted to the top-k (top_k[b] > 0, <= 256) and the nucleus top_p[b]
// (< 1; over the top-256 when top-k is off)); then pos[b] += 1, seq_len[b] = pos[b] + 1,
// history[b][step] = token.
struct SampleArgs {
  const float* logits;
  int ldl;
  int B, V;
  const float* temperature;  // [B] or null (greedy)
  const int* top_k;          // [B] or null
  uint64_t seed;             // RNG key = (seed, row, pos[row])
  const uint64_t* seed_dev;  // if non-null, the seed is read from device memory (graph-replay safe)
  const uint64_t* seeds;     // [B] per-row seeds or null: RNG key = (seeds[b], pos[b]) -- a request's
                             // samples then depend on its seed and positions only, not its batch row
  int* tokens;               // [B] out
  int* pos;                  // [B] in/out (incremented when advance != 0)
  int* seq_len;              // [B] out (pos+1) or null
  int* history;              // [B][hist_stride] or null
  int hist_stride;
  int advance;
  const uint8_t* mask;       // [B][ceil(V/8)] allowed-token bitmask or null
  const float* top_p;        // [B] nucleus mass (>= 1: off) or null
  void* ws;                  // sample_ws_bytes(B, V) scratch (slice partials + candidates)
  size_t ws_bytes;
  int* counters;             // [B] arrival tickets, zero-initialised, self re-arming
  long long* ts;             // probe stamps [B][slices][16] (tools/sample_probe.py --stamps) or null
};
void launch_sample(const SampleArgs& a, hipStream_t st);
size_t sample_ws_bytes(int B, int V);

// ---- MFMA GEMM (prefill) ----------------------------------------------------------------------
// C[M][N] (fp32, epilogue) = A[M][K] (bf16) x W[N][K]^T (quantized, dequantized tile-wise in LDS)
struct GemmArgs {
  const bf16_t* A;
  int lda;
  QWeight w;
  int M, N, K;
  float* C;
  int ldc;
  int accumulate;  // C += result
  float* ws = nullptr;  // split-K workspace of the skinny (M <= 64) kernel, see GemmQArgs
  size_t ws_bytes = 0;
  int* cnt = nullptr;
  int cnt_len = 0;
};
void launch_gemm(const GemmArgs& a, hipStream_t st);
bool gemm_supports(int qt);

// multi-segment GEMM with fused epilogues (the prefill path): C = A x [W0; W1; W2]^T
enum GemmEpi { GEPI_STORE = 0, GEPI_ACCUM = 1, GEPI_SWIGLU_BF16 = 2, GEPI_QKV = 3, GEPI_ACCUM_NORM = 4 };
struct GemmQArgs {
  const bf16_t* A;   // [M][lda] bf16
  int lda;
  QWeight seg[3];    // weight segments stacked along N (rows of each a multiple of 64)
  int seg_n0[3];     // first output column of each segment
  int nseg;
  int M, N, K;
  float* C;          // [M][ldc] fp32 (STORE / ACCUM)
  bf16_t* C16;       // [M][ldc] bf16 (SWIGLU_BF16: column n/2 = silu(col n) * col n+1)
  int ldc;
  int epi;
  int ksplit;        // K split over workgroups: 0 = auto, 1 = off
  // skinny (M <= 64) split-K: fp32 partial slabs [S][tiles][16*Mt][rows] + per-tile arrival
  // tickets (zero-initialised, re-armed by each tile's last arriver).  Null -> no split.
  float* ws;
  size_t ws_bytes;
  int* cnt;
  int cnt_len;
  // GEPI_QKV (skinny kernel, batched decode; non-NeoX RoPE, no QK-norm / bias): global column
  // col0 + n of the packed [q | k | v] product -> RoPE'd q to q_out[M][q_dim], RoPE'd k / v as bf16
  // into the paged KV cache at (slot[m], pos[m]) -- the qkv_post launch folded into the epilogue
  int col0;
  int head_dim, q_dim, kv_dim, n_kv_heads, max_ctx;
  const float2* rope_cs;  // [max_ctx][head_dim / 2] (cos, sin)
  const int* pos;
  const int* slot;
  const int* block_table;
  float* q_out;
  bf16_t* k_cache;
  bf16_t* v_cache;
  int kv_fp8;        // fp8 e4m3 pool: code = value * kv_inv_{k,v}
  float kv_inv_k, kv_inv_v;
  // RMSNorm split across two skinny GEMMs (batched decode: no normalisation launch).
  //  producer (GEPI_ACCUM_NORM = residual add): also writes bf16(x_new * nrm_g) to nrm_out16
  //    [M][ldc] and, per output tile t, sum_n x_new[m][n]^2 to nrm_part[m * nrm_parts + t]
  //    (nrm_parts = gemm_skinny_ntile(producer args); fixed-order reductions, no atomics)
  //  consumer (any epilogue, nrm_in set): A is that bf16(x * g); output row m is scaled by
  //    rsqrt(sum_t nrm_in[m * nrm_parts + t] / K + nrm_eps) before the epilogue
  const float* nrm_g;
  bf16_t* nrm_out16;
  float* nrm_part;
  const float* nrm_in;
  int nrm_parts;
  float nrm_eps;
  unsigned long long* dbg_ts;  // probes (skinny kernel): [grid][8] s_memrealtime phase stamps or null
};
// bytes of split-K workspace / ticket count the skinny GEMM may use for an M x N output
size_t gemm_skinny_ws_bytes(int M, int N);
int gemm_skinny_cnt_len(int N);
// output tiles of the skinny kernel for these args (0: not served by the skinny kernel)
int gemm_skinny_ntile(const GemmQArgs& a);
void launch_gemm_q(const GemmQArgs& a, hipStream_t st);
// the prefill GEMM (kernels/gemm_pf.hip): true if it took the launch; its tile / split plan for a shape
bool launch_gemm_pf(const GemmQArgs& a, hipStream_t st);
bool gemm_pf_serves(const GemmQArgs& a);  // launch_gemm_pf would take a (gemm_pf.hip)
void gemm_pf_plan(const GemmQArgs& a, int& bm, int& bn, int& s);
bool gemm_pf_probe(const GemmQArgs& a, int probe, hipStream_t st);  // timing anatomy (tools only)
// time every prefill-GEMM plan for these args (buffers overwritten) and keep the fastest for their M
// bucket; returns the number of plans timed
int gemm_pf_autotune(const GemmQArgs& a, hipStream_t st);
std::vector<int> gemm_pf_export();              // the process's tuned prefill plans (flat ints)
void gemm_pf_import(const std::vector<int>& v);  // ... installed (TP: the leader's; persisted sets)

}  // namespace aios
