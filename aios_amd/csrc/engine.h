// In-process inference engine for Llama-family GGUF models on one MI355X (gfx950).
//
// Replaces the reference's per-model llama-server child process
// (`runtime/src/model_manager.rs:185-204`, HTTP at `runtime/src/inference.rs:94-186`):
// weights live in HBM in the repacked GEMV layout, the KV cache is a bf16 slab
// [layer][slot][kv_head][max_ctx][head_dim], and the whole decode step (embed -> L x {QKV+RoPE+KV,
// attention, O+residual, gate/up+SwiGLU, down+residual} -> norm+lm_head -> sample) is one
// stream-ordered sequence of launches that is captured once per batch size into a hipGraph and
// replayed (SURVEY.md §2.7 fusion targets, §7.6 hard part 2).  Sampled tokens are fed back on
// device, so N decode steps need no host round trip.
#pragma once
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "common.h"
#include "ops.h"

namespace aios {

struct EngineConfig {
  std::string name = "model";
  int vocab_size = 32000;
  int d_model = 2048;
  int n_layers = 22;
  int n_heads = 32;
  int n_kv_heads = 4;
  int head_dim = 64;
  int d_ff = 5632;
  float rope_theta = 10000.f;
  int rope_neox = 0;
  float norm_eps = 1e-5f;
  int max_ctx = 2048;
  int max_slots = 4;
  int max_batch = 8;
  int tie_embeddings = 0;
  int qk_norm = 0;
  int qkv_bias = 0;
  int act_q8 = 1;  // int8 activations (v_dot4) in the quantised GEMVs, as llama.cpp's q8_1 path
  // tensor parallel (the engine holds this rank's shard; collectives via the comm hook)
  int tp_rank = 0;
  int tp_size = 1;
  // vocab-parallel lm_head under TP: output.weight holds rows [rank*V/tp, (rank+1)*V/tp) and the
  // logits are completed by the all-gather hook (ignored for tp_size 1 / tied embeddings)
  int vocab_parallel = 0;
  int device = 0;
  // KV cache element type: 0 = bf16, 1 = fp8 e4m3 (OCP) with a per-layer K / V scale (value = code x
  // scale, Engine::set_kv_scales; 1.0 until set) -- half the cache bytes and the decode attention's
  // K / V reads (bf16 or fp8 on MI355X)
  int kv_fp8 = 0;
  // CU mask of the engine's stream (hipExtStreamCreateWithCUMask; 32 CUs per word, empty = every CU):
  // co-resident tiers each get their own CUs, and the engine sizes its grids to the mask's CU count
  std::vector<uint32_t> cu_mask;
  // stream priority (co-resident tiers, unmasked streams): 0 = normal, < 0 = higher (the range of
  // hipDeviceGetStreamPriorityRange; the hardware queue's dispatcher serves it first)
  int stream_priority = 0;
};

// device matrix in repacked layout (owns its buffer)
struct QMat {
  QWeight w{};
  void* buf = nullptr;
  size_t bytes = 0;
  bool valid() const { return buf != nullptr; }
};

struct LayerW {
  float* attn_norm = nullptr;
  float* ffn_norm = nullptr;
  float* q_norm = nullptr;
  float* k_norm = nullptr;
  float* bqkv = nullptr;  // [q_dim + 2 kv_dim]
  QMat wq, wk, wv, wo, wgu, wdown;
};

// all-reduce hook (TP): sum `n` floats of `data` over the TP ranks on `stream` and add the
// total into `residual` (or into `data` when residual is null); installed by aios_amd/parallel.
using AllReduceFn = void (*)(void* ctx, float* data, size_t n, float* residual, hipStream_t stream);
// all-gather hook (vocab-parallel lm_head): rank r owns columns [r*slice, (r+1)*slice) of the
// rows x ld fp32 matrix `data`; afterwards every rank holds all of them
using AllGatherFn = void (*)(void* ctx, float* data, int rows, int slice, int ld, hipStream_t stream);
// fused all-reduce + split-RMSNorm producer hook (batched TP decode, C1 / C2): residual ([rows][d]) +=
// sum of partials, then the ResidNorm outputs (ops.h) the next skinny GEMM consumes -- no RMSNorm launch
using AllReduceNormFn = void (*)(void* ctx, float* data, int rows, int d, float* residual, const ResidNorm& nm,
                                 hipStream_t stream);

class Engine {
 public:
  explicit Engine(const EngineConfig& cfg);
  ~Engine();

  const EngineConfig& config() const { return cfg_; }

  // --- weights -------------------------------------------------------------------------------
  // raw GGUF bytes (host pointer) of a named tensor; names follow GGUF ("blk.3.attn_q.weight").
  void set_tensor(const std::string& name, int ggml_type, int rows, int cols, const void* host, size_t nbytes);
  // random-init synthetic weights generated in HBM (recipe: "Q4_K_M", "Q4_0", "Q8_0", "BF16", ...)
  void init_random(const std::string& recipe, uint64_t seed);
  void finalize();  // checks completeness, allocates KV cache + workspace
  bool ready() const { return finalized_; }
  size_t weight_bytes() const { return weight_bytes_; }
  size_t kv_bytes() const { return kv_bytes_; }
  size_t workspace_bytes() const { return ws_bytes_; }
  std::vector<std::string> missing_tensors() const;
  std::string weight_type_summary() const;

  // --- inference -----------------------------------------------------------------------------
  // Prefill `tokens` into `slot` starting at position `start_pos`.  Returns logits of the last
  // token (host copy) if want_logits, and leaves the slot ready to decode.
  std::vector<float> prefill(int slot, const std::vector<int>& tokens, int start_pos, bool want_logits);
  // One decode step for B sequences: input token ids at positions pos[b] in slots[b].  Samples
  // with per-row temperature/top_k (0 = greedy) and optional grammar bitmasks; returns tokens.
  std::vector<int> decode(const std::vector<int>& slots, const std::vector<int>& tokens, const std::vector<int>& pos,
                          const std::vector<float>& temperature, const std::vector<int>& top_k, uint64_t seed,
                          const std::vector<uint8_t>& mask, const std::vector<float>& top_p = {},
                          const std::vector<uint64_t>& seeds = {});
  // sample the token after a prefill from its last logits (logits_ row 0) on the device, with the
  // same sampler and RNG stream (seed, pos) as the decode steps -- pos: the prompt's last position
  int sample_first(int pos, float temperature, int top_k, float top_p, uint64_t seed, const std::vector<uint8_t>& mask);
  // re-sample the last step's logits (no state advance), e.g. with a grammar mask
  std::vector<int> resample(int B, const std::vector<float>& temperature, const std::vector<int>& top_k, uint64_t seed,
                            const std::vector<uint8_t>& mask, const std::vector<float>& top_p = {});
  // logits of the last decode (B x V) -- host copy
  std::vector<float> last_logits(int B);

  // Pipelined decode (the serving scheduler's fast path): decode() split so that the forward of step
  // t+1 is enqueued before the host has seen step t's token -- the rows' tokens are the ones step t's
  // sampler left on the device -- and only the sampler waits for the host's grammar mask:
  //   decode_submit(..., tokens = {})   forward graph of the next step (tokens from the device)
  //   decode_sample(mask)               mask upload + sampler + token copy, one event
  //   decode_collect()                  waits for that event: the sampled tokens
  // The stream holds sample(t), forward(t+1) while the host turns token t into mask t+1.
  // decode_submit with tokens: the host's tokens (a batch's first step).
  void decode_submit(const std::vector<int>& slots, const std::vector<int>& tokens, const std::vector<int>& pos,
                     const std::vector<float>& temperature, const std::vector<int>& top_k, uint64_t seed,
                     const std::vector<float>& top_p = {}, const std::vector<uint64_t>& seeds = {});
  void decode_sample(const std::vector<uint8_t>& mask);
  std::vector<int> decode_collect();

  // Device-resident greedy generation for benchmarking: runs n_steps decode steps for B
  // sequences without host synchronisation (tokens fed back on device, graph replay when
  // use_graph).  Sequences must already be prefilled to positions pos[b].
  void decode_loop_prepare(const std::vector<int>& slots, const std::vector<int>& tokens, const std::vector<int>& pos);
  void decode_loop_run(int B, int n_steps, bool use_graph);
  std::vector<int> decode_loop_history(int B, int from_pos, int n);

  void synchronize();
  uintptr_t stream_handle() const { return (uintptr_t)stream_; }
  void set_allreduce(AllReduceFn fn, void* ctx) { allreduce_ = fn; allreduce_ctx_ = ctx; }
  void set_allgather(AllGatherFn fn, void* ctx) { allgather_ = fn; allgather_ctx_ = ctx; }
  void set_allreduce_norm(AllReduceNormFn fn, void* ctx) { allreduce_norm_ = fn; allreduce_norm_ctx_ = ctx; }
  // TP: the O / down all-reduces fused into the B <= 4 GEMV engine's epilogue (EPI_TP_RESID);
  // ctx null = separate all-reduce launches; grid = engine workgroups per launch (0: one per CU)
  void set_tp_fuse(const ArDevCtx* ctx, int grid) { tp_fuse_ = ctx; tp_fuse_grid_ = grid; }
  bool tp_fused() const { return tp_fuse_ != nullptr; }
  // TP init: for every layer's O and down projection at batch 1, whether the fused all-reduce
  // epilogue would launch on THIS rank (row kernel stage fit under the co-residency cap, which
  // depends on the device's CU count); the ranks all-gather it and turn fusion off everywhere unless
  // every rank fits every shape (a rank falling back alone would leave its peers waiting on flags)
  std::vector<int> tp_fuse_fits();
  void disable_tp_fuse() { tp_fuse_ = nullptr; }
  // fp8 KV: the per-layer (K, V) scales, 2 x n_layers values (value = code x scale; captured decode
  // graphs are dropped, they hold the old ones).  1.0 until set: e4m3 spans 2^-9 .. 448, the range of
  // post-RoPE keys and values, as serving stacks' uncalibrated fp8 KV caches do; a calibrated model
  // (per-layer K / V absolute maxima / 448) sets them here
  void set_kv_scales(const std::vector<float>& s);
  std::vector<float> kv_scales() const { return kv_scale_; }
  int kv_fp8() const { return cfg_.kv_fp8; }
  bool vocab_parallel() const { return cfg_.vocab_parallel != 0; }
  void reset_graphs();
  int capture_graphs(int max_b);  // pre-capture the decode-step graphs of B = 1..max_b (masked + unmasked)
  // ---- paged KV (block table per slot; see kv_offset in common.h) --------------------------------
  // prefix sharing: dst's positions [0, n) become src's -- full blocks shared (refcounted, never
  // written again by either slot: writes un-share first), the partial last block copied
  void copy_slot(int src, int dst, int n_tokens);
  void release_slot(int slot);         // drop every block reference of the slot
  int kv_blocks_free() const { return (int)free_blocks_.size(); }
  int kv_blocks_total() const { return kv_nblocks_; }
  int norm_fused_parts() const { return nrm_parts_; }  // 0: batched-decode RMSNorm not split into the GEMMs
  std::vector<int> block_table(int slot) const;

  // raw device pointers for tests / custom kernels
  uintptr_t kv_cache_k() const { return (uintptr_t)k_cache_; }
  uintptr_t kv_cache_v() const { return (uintptr_t)v_cache_; }

 private:
  void enqueue_decode_step(int B);       // uses device arrays d_tokens_/d_pos_/d_seqlen_/d_slot_
  void enqueue_decode_forward(int B);    // ... up to the logits (no sampler)
  void enqueue_sample(int B);            // the step's sampler (sample_mask_: with d_mask_)
  hipGraphExec_t forward_graph(int B);
  int cus_ = 0;                          // CUs of the stream's mask (0: the whole device)
  int kv_es_ = 2;                        // bytes per KV element (2 bf16, 1 fp8)
  std::vector<float> kv_scale_;          // [n_layers][K, V] fp8 scales (value = code * scale)
  bf16_t* kv_layer(bf16_t* base, int l) const {  // layer l's pool (element indices as bf16, bytes as kv_es_)
    return (bf16_t*)((char*)base + (size_t)l * layer_kv_elems_ * kv_es_);
  }
  template <typename T>
  void kv_write_args(T& a, int l) const {
    a.kv_fp8 = cfg_.kv_fp8;
    a.kv_inv_k = 1.f / kv_scale_[2 * l];
    a.kv_inv_v = 1.f / kv_scale_[2 * l + 1];
  }
  template <typename T>
  void kv_read_args(T& a, int l) const {
    a.kv_fp8 = cfg_.kv_fp8;
    a.kv_scale_k = kv_scale_[2 * l];
    a.kv_scale_v = kv_scale_[2 * l + 1];
  }
  int pipe_B_ = 0;                       // rows of the submitted, not yet sampled step
  int par_buf_ = 0;                      // which half of the double-buffered pinned parameter block
  uint8_t* h_mask_ = nullptr;            // pinned staging of the pipelined sampler's masks
  hipEvent_t pipe_ev_ = nullptr;         // the pipelined sampler's token copy
  bool gemm_prefill_ok(int T) const;
  void prefill_gemm(int slot, const std::vector<int>& tokens, int start_pos, bool want_logits);
  void layer_decode(int l, int B);
  void gemv(const std::vector<const QMat*>& segs, int N, int K, int B, const float* x, int ldx, const float* norm_w,
            float* y, int ldy, int epi, int layer);
  GemvArgs gemv_args(const std::vector<const QMat*>& segs, int N, int K, int B, const float* x, int ldx,
                     const float* norm_w, float* y, int ldy, int epi, int layer);
  QMat alloc_qmat(int qt, int rows, int cols);
  QMat upload_qmat(int qt, int rows, int cols, const void* host, size_t nbytes);
  // load-time staging: two device buffers (tensor i repacks while i+1 uploads) fed through two
  // pinned 64 MB host chunks
  void stage_upload(const void* host, size_t nbytes, void*& dev_staging);
  void stage_done();
  void stage_release();
  void* stage_dev_[2] = {nullptr, nullptr};
  size_t stage_dev_bytes_[2] = {0, 0};
  hipEvent_t stage_ev_[2] = {nullptr, nullptr};
  void* stage_host_[2] = {nullptr, nullptr};
  hipEvent_t stage_host_ev_[2] = {nullptr, nullptr};
  int stage_next_ = 0, stage_host_next_ = 0, stage_cur_ = 0;
  float* upload_f32(const void* host, size_t n, int qt);
  QMat interleave_rows(const QMat& a, const QMat& b);
  void* dmalloc(size_t bytes);
  void tune_prefill_gemm();  // measured prefill-GEMM plans for this model's projection shapes
  void allreduce(float* p, size_t n, float* residual);
  void lm_head(int B, const float* x, int ldx);  // logits_[B][V] (vocab-parallel aware)

  EngineConfig cfg_;
  hipStream_t stream_ = nullptr;

  bool finalized_ = false;
  std::vector<void*> allocs_;
  size_t weight_bytes_ = 0, kv_bytes_ = 0, ws_bytes_ = 0;

  QMat tok_embd_, output_;
  float* out_norm_ = nullptr;
  std::vector<LayerW> layers_;
  std::map<std::string, QMat> pending_;  // gate/up waiting for their partner

  bf16_t* k_cache_ = nullptr;
  bf16_t* v_cache_ = nullptr;
  size_t layer_kv_elems_ = 0;

  // workspace
  float *x_ = nullptr, *q_ = nullptr, *attn_ = nullptr, *ff_ = nullptr, *qkv_ = nullptr;
  // the GEMV path's SwiGLU hand-off in bf16 (gate/up epilogue -> down staging: half the bytes every
  // down workgroup re-reads; AIOS_FF16=0 keeps fp32), [max_batch][d_ff]
  bf16_t* gv_ff16_ = nullptr;
  float *opart_ = nullptr, *ml_ = nullptr, *logits_ = nullptr;
  int *d_tokens_ = nullptr, *d_pos_ = nullptr, *d_seqlen_ = nullptr, *d_slot_ = nullptr, *d_history_ = nullptr;
  int *d_topk_ = nullptr, *d_step_ = nullptr;
  float* d_temp_ = nullptr;
  float* d_topp_ = nullptr;
  char* d_par_ = nullptr;          // per-step parameter block (seed, slot, token, pos, seq_len, top_k, T, top_p | masks)
  char* h_par_ = nullptr;          // pinned mirror
  int* h_tok_out_ = nullptr;       // pinned sampled tokens
  size_t par_bytes_ = 0, par_mask_off_ = 0;
  void* sample_ws_ = nullptr;
  size_t sample_ws_bytes_ = 0;
  int* sample_cnt_ = nullptr;
  uint64_t* d_seed_ = nullptr;
  uint64_t* d_seeds_ = nullptr;    // [max_batch] per-row sampling seeds (in the parameter block)
  int* d_fpos_ = nullptr;          // sample_first's RNG position
  // StepPrep outputs of the decode step's embedding launch: [max_batch][2] {pos, KV block} and
  // [max_batch][head_dim / 2] rope rows, read by the batch-1 QKV epilogue while step_prep_on_
  int* d_step_kv_ = nullptr;
  float2* d_step_rope_ = nullptr;
  bool step_prep_on_ = false;
  void fill_row_seeds(uint64_t* host_seeds, int B, uint64_t seed, const std::vector<uint64_t>& seeds);
  uint8_t* d_mask_ = nullptr;
  int n_chunks_ = 0;
  int* attn_cnt_ = nullptr;  // [max(prefill_rows, max_batch)][n_kv_heads] combine tickets
  float2* rope_cs_ = nullptr;  // [max_ctx][head_dim/2] cos/sin computed in double on the host
  int prefill_rows_ = 64;  // rows of the prefill workspace
  float *pf_x_ = nullptr, *pf_q_ = nullptr, *pf_attn_ = nullptr, *pf_ff_ = nullptr, *pf_qkv_ = nullptr;
  float *pf_opart_ = nullptr, *pf_ml_ = nullptr;
  bf16_t* pf_a16_ = nullptr;
  // GEMM prefill workspace (chunks of gm_rows_ tokens through MFMA GEMMs + flash attention)
  int gm_rows_ = 512;
  // prompts shorter than this take the GEMV path, whose batched LDS-DMA engine serves up to 4 rows
  // (tools/bench_prefill.py, round 3: 2 / 3 / 4 tokens 1.85 / 2.02 / 2.29 ms there vs 3.25 ms for 4 through
  // the skinny GEMM; from 5 rows the GEMV falls back to the row kernels, 8.5 ms, the GEMM 3.25)
  int gm_min_rows_ = 5;
  bool gm_ok_ = false;    // every layer's weights / head shape supported
  float *gm_x_ = nullptr, *gm_qkv_ = nullptr, *gm_q_ = nullptr, *gm_part_ = nullptr;
  bf16_t *gm_a16_ = nullptr, *gm_ff16_ = nullptr, *gm_attn16_ = nullptr;
  int *gm_tokens_ = nullptr, *gm_pos_ = nullptr, *gm_slot_ = nullptr;
  // chunks of <= 64 rows: the residual GEMMs' bf16(x * g_next) + per-tile sums (split RMSNorm)
  bf16_t* gm_xn16_ = nullptr;
  float* gm_npart_ = nullptr;
  int gm_nparts_ = 0;
  const ArDevCtx* tp_fuse_ = nullptr;
  int tp_fuse_grid_ = 0;
  bool tp_fuse_gemv(GemvArgs a);  // EPI_TP_RESID launch when the engine serves the shape (else false)
  // batched decode through the skinny MFMA GEMM (B >= dec_gemm_min_b_): bf16 activation buffers
  // (MI355X, Mistral-7B Q4_K_M, tools/gpu_batch_ab.sh: B=2 GEMV 2.41 ms vs GEMM 3.25 ms, B=4 3.31 vs 3.26,
  // B=8 5.80 vs 3.37 -- the skinny GEMM's per-step dequant floor lost below 4 rows; after the split
  // RMSNorm / mixed-QKV / split-K work, tools/gpu_minb_ab.sh: B=3 GEMV 956 vs GEMM 1065 tok/s, B=2 829 vs 712)
  // round 3: the LDS-DMA GEMV engine serves B = 2..4 from one weight stream (gemv_lds.h):
  // B = 2 / 3 / 4 1.82 / 2.29 / 2.45 ms vs the skinny GEMM's 3.25 / 2.83 / 2.84 (profiles/lds_batched_r3.txt)
  int dec_gemm_min_b_ = 5;
  bf16_t *dec_a16_ = nullptr, *dec_ff16_ = nullptr;
  // split-K slabs + arrival tickets of the skinny GEMM (shared by every decode GEMM of a step)
  float* gk_ws_ = nullptr;
  size_t gk_ws_bytes_ = 0;
  int* gk_cnt_ = nullptr;
  int gk_cnt_len_ = 0;
  void gemm(GemmQArgs& g);  // launch_gemm_q with the engine's split-K workspace
  // RMSNorm split across the skinny GEMMs (AIOS_GEMM_NORM_FUSE, default on): the residual GEMMs
  // (O, down) also write bf16(x * g_next) to dec_xn16_ and per-tile row sums of squares to
  // nrm_part_; the next GEMM (gate/up, next layer's QKV, lm_head) scales its rows by the inverse
  // RMS in the epilogue -- two normalisation launches per layer less
  bf16_t* dec_xn16_ = nullptr;
  float* nrm_part_ = nullptr;
  int nrm_fuse_ = 1;
  int nrm_parts_ = 0;  // tiles of the d_model-wide producer GEMM (0: fusion unavailable)
  bool nrm_on(int B) const;
  bool tpn_on(int B) const;  // batched TP decode: C1 / C2 fused with the next RMSNorm
 private:
  void layer_decode_gemm(int l, int B);
  hipGraphExec_t step_graph(int B);
  bool nrm_lm_ = false;  // the last layer's down GEMM prepared dec_xn16_ / nrm_part_ for lm_head(x_)
  int *pf_tokens_ = nullptr, *pf_pos_ = nullptr, *pf_seqlen_ = nullptr, *pf_slot_ = nullptr;

  // paged KV state: host tables are the truth, device copies uploaded (stream idle) when dirty
  int kv_maxb_ = 0;                // blocks per slot = max_ctx / KV_BLOCK
  int kv_nblocks_ = 0;             // allocatable blocks per layer pool (+1 null block at the end)
  std::vector<int> bt_;            // [max_slots][kv_maxb_], -1 = unmapped
  std::vector<int> refcnt_;        // [kv_nblocks_]
  std::vector<int> free_blocks_;
  std::vector<int> row_bt_host_;   // [max_batch][kv_maxb_] as last uploaded
  int* d_bt_ = nullptr;            // [max_slots][kv_maxb_] slot-indexed (unmapped -> null block)
  int* d_row_bt_ = nullptr;        // [max_batch][kv_maxb_] rows of the decode batch
  bool bt_dirty_ = false;
  std::vector<int> row_slots_, row_pos_;  // decode rows: slot and host-tracked next position
  const int* attn_bt_ = nullptr;   // table the decode attention reads (rows / slot indexed)
  int attn_bt_rows_ = 1;
  int kv_alloc();
  void kv_unref(int blk);
  void kv_copy_block(int src, int dst);
  void kv_prepare_write(int slot, int from, int to);  // map + un-share the blocks of [from, to)
  void kv_sync(int B);                                 // upload dirty tables (rows 0..B-1)

  std::map<int, hipGraphExec_t> graphs_;
  AllReduceFn allreduce_ = nullptr;
  void* allreduce_ctx_ = nullptr;
  AllGatherFn allgather_ = nullptr;
  AllReduceNormFn allreduce_norm_ = nullptr;
  void* allreduce_norm_ctx_ = nullptr;
  // batched TP decode: the fused all-reduce's split-norm partials [max_batch][tpn_parts_] (0: off)
  int tpn_parts_ = 0;
  float* tpn_part_ = nullptr;
  // the split-norm partials the lm_head consumes when nrm_lm_ is set (nrm_part_ or tpn_part_)
  const float* lm_nrm_in_ = nullptr;
  int lm_nrm_parts_ = 0;
  void* allgather_ctx_ = nullptr;
  // sampling config for the enqueued step
  bool sample_temp_ = false;
  bool sample_mask_ = false;
  uint64_t sample_seed_ = 0;
};

}  // namespace aios
