// Tensor-parallel collectives for one MI355X node over IPC-mapped peer buffers: every GPU reads
// its <= 7 peers directly over the point-to-point xGMI links.
//
//  * one-shot all-reduce (decode-size messages, 16-256 KB): stage my partial, flag, pull every
//    peer's partial and sum -- ~one xGMI round trip, all 7 links in parallel; fp32 payload;
//  * two-shot all-reduce = reduce-scatter + all-gather (prefill-size messages, MBs): each rank
//    reduces only its 1/world sub-shard of every workgroup chunk (pulling 7 peers' staged
//    partials, optionally bf16 to halve the link bytes), publishes it, and all ranks gather the
//    reduced sub-shards: 2(W-1)/W of the message crosses each GPU's links instead of (W-1)x,
//    a mesh (all links at once), not a per-link-bound ring;
//  * all-gather of per-rank column slices of a [rows][ld] fp32 matrix (the vocab-parallel
//    lm_head: each rank computes V/world logits, every rank needs all of them for the identical
//    on-device sampler and the JSON-grammar mask).
// All three are fused with their consumer where it is an elementwise op (residual add).
//  * C1 / C2 of the batch-1 TP decode step fused into the PRODUCER instead (round 4): the O / down row
//    GEMV's workgroups publish their rows' partials to per-workgroup stage slots behind the one-shot
//    region and exchange per-slot flags (EPI_TP_RESID, gemv_q8.h) -- no all-reduce launch.  Stage and
//    flags are uncached, so a retired store is visible to every peer without a system-scope fence.
//
// Why not a ring: a ring pays 2(W-1) latency hops and is bound by one link.
//
// Protocol (per workgroup g; epoch e = this WG's call counter, identical on every rank because
// every rank issues the same sequence of collectives with the same sizes):
//   1. copy my part of chunk g into my stage buffer half e & 1
//   2. release fence (system scope), store e into flag[phase][g][my_rank] of every peer
//   3. wait until my own flag[phase][g][p] >= e for every peer (bounded spin -> error flag)
//   4. consume the peers' half e & 1 (two-shot: reduce, publish result, flag phase 2, wait, gather)
// Buffer position j is always owned by workgroup j / AR_CHUNK in every kernel (each call moves
// at most AR_MAX_WG * AR_CHUNK elements; larger messages are split into several calls), so the
// per-workgroup epochs stay consistent across calls of different sizes and kinds.  Double
// buffering is safe: a rank reuses half e&1 at epoch e+2, which needs every peer's epoch-(e+1)
// phase-1 flag, which a peer sets only after it finished all its reads of epoch e.
// Flags / buffers are uncached device memory (hipDeviceMallocUncached), so remote stores and
// loads bypass the caches of both GPUs; works across GPUs (xGMI) and between processes that share
// one GPU (how the TP path is tested on a single-GPU box).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include "ops.h"
#include <string>
#include <vector>

namespace aios {

constexpr int AR_MAX_RANKS = 8;
constexpr int AR_MAX_WG = 512;
constexpr int AR_THREADS = 256;
constexpr int AR_CHUNK = AR_THREADS * 4;              // elements per workgroup per call
constexpr size_t AR_MAX_CALL = (size_t)AR_MAX_WG * AR_CHUNK;  // elements per kernel call
// C1 / C2 fused into the batch-1 row GEMV epilogue (EPI_TP_RESID, gemv_q8.h): per GEMV
// workgroup ("slot") a private double-buffered stage of up to TPF_CAP partial outputs behind the
// one-shot region, and one flag per (slot, rank) behind the collectives' flags
constexpr int TPF_SLOTS = 256;
constexpr int TPF_CAP = 1024;

struct ArDevCtx {
  float* buf[AR_MAX_RANKS];         // rank r's shared region: stage f32 [2][cap] | result f32 [2][cap] | stage bf16 [2][cap]
  uint32_t* flags[AR_MAX_RANKS];    // rank r's flags: [2 phases][AR_MAX_WG][AR_MAX_RANKS]
  uint32_t* epoch;                  // my per-WG epoch counters [AR_MAX_WG] (local)
  uint32_t* error;                  // set to 1 when a wait timed out (device view of pinned host memory)
  int rank, world;
  size_t cap;                       // elements per half-buffer (<= AR_MAX_CALL)
  uint32_t* fepoch;                 // my per-slot epochs of the fused GEMV epilogue [TPF_SLOTS] (local)
};
// the fused epilogue's regions of rank p (same offsets on every rank)
__host__ __device__ inline float* tpf_stage(const ArDevCtx* c, int p) { return c->buf[p] + 5 * c->cap; }
__host__ __device__ inline uint32_t* tpf_flags(const ArDevCtx* c, int p) {
  return c->flags[p] + 2 * AR_MAX_WG * AR_MAX_RANKS;
}

class XgmiComm {
 public:
  XgmiComm(int rank, int world, int device, size_t cap_floats);
  ~XgmiComm();
  // opaque IPC handles of my shared region + flag buffer (hipIpcMemHandle_t x 2)
  std::string ipc_handle() const;
  // map every peer's buffers (handles indexed by rank; my own entry is ignored)
  void connect(const std::vector<std::string>& handles);
  bool connected() const { return connected_; }
  // sum `n` floats of `data` over all ranks; result into `data`, or added into `residual`
  // (data left as my partial) when residual != nullptr.  Stream-ordered, graph-capturable.
  // Messages above two_shot_min() floats use reduce-scatter + all-gather; messages above the
  // capacity are split into several calls.
  void allreduce(float* data, size_t n, float* residual, hipStream_t st);
  // allreduce into `residual` ([rows][d]) plus the split-RMSNorm producer outputs of the consumer
  // GEMM (ResidNorm, ops.h): one launch when the message is a one-shot call (decode sizes, d a
  // multiple of RNORM_COLS), else the all-reduce followed by launch_add_norm
  void allreduce_norm(float* data, int rows, int d, float* residual, const ResidNorm& nm, hipStream_t st);
  // every rank owns columns [r*slice, (r+1)*slice) of the rows x ld fp32 matrix `data`;
  // afterwards every rank holds all columns
  void allgather_cols(float* data, int rows, int slice, int ld, hipStream_t st);
  bool error() const;
  void reset_error();
  int rank() const { return h_.rank; }
  int world() const { return h_.world; }
  size_t capacity() const { return h_.cap; }
  size_t two_shot_min() const { return two_shot_min_; }
  // workgroups per collective launch (elements per call = wg * AR_CHUNK, larger messages split):
  // AR_MAX_WG by default; ranks that SHARE one GPU (the single-GPU test setting) must fit all their
  // spinning workgroups on it at once, so tp.create_comm lowers it to 1024 / ranks-per-GPU.  Every
  // rank must use the same value (the per-workgroup epochs follow the call sequence).
  int call_wg() const { return (int)(call_cap_ / AR_CHUNK); }
  void set_call_wg(int wg);
  void set_two_shot_min(size_t n) { two_shot_min_ = n; }
  // the fused O / down epilogue (EPI_TP_RESID): device context for GemvArgs::tp (null when off:
  // world 1 or AIOS_TP_FUSE=0) and the engine-workgroup cap that lets every rank's grid be resident
  // at once when ranks share a GPU (0: one workgroup per CU)
  const ArDevCtx* fuse_ctx() const { return fuse_on_ && uncached_ && h_.world > 1 ? d_ : nullptr; }
  // this rank's eligibility for the fused epilogue; create_comm all-gathers it and turns the path off
  // everywhere unless EVERY rank is eligible (a rank on the fused path spins on flags that a rank
  // running separate all-reduces never raises)
  bool fuse_eligible() const { return fuse_on_ && uncached_; }
  void disable_fuse() { fuse_on_ = false; }
  bool uncached() const { return uncached_; }
  int fuse_grid() const { return fuse_grid_; }
  void set_ranks_per_gpu(int n);
  bool bf16_payload() const { return bf16_; }
  void set_bf16_payload(bool on) { bf16_ = on; }
  // Engine hooks (AllReduceFn / AllGatherFn-compatible trampolines)
  static void hook(void* self, float* data, size_t n, float* residual, hipStream_t st);
  static void gather_hook(void* self, float* data, int rows, int slice, int ld, hipStream_t st);
  static void norm_hook(void* self, float* data, int rows, int d, float* residual, const ResidNorm& nm,
                        hipStream_t st);

 private:
  ArDevCtx h_{};
  ArDevCtx* d_ = nullptr;        // device copy of h_
  float* mybuf_ = nullptr;
  uint32_t* myflags_ = nullptr;
  // the give-up flag lives in pinned, device-mapped host memory: the kernels set it with
  // system-scope stores and error() is a plain host load -- no per-call hipMemcpy (which
  // serialised every leader call behind the device, verdict r2)
  volatile uint32_t* host_error_ = nullptr;
  std::vector<void*> opened_;
  int device_ = 0;
  bool connected_ = false;
  size_t two_shot_min_ = 64 * 1024;  // floats (256 KB)
  size_t call_cap_ = AR_MAX_CALL;    // elements per launch (see set_call_wg)
  bool bf16_ = true;                 // bf16 staging for the two-shot (prefill) path
  bool fuse_on_ = true;              // AIOS_TP_FUSE (default 1)
  bool uncached_ = false;            // shared regions got uncached memory (required by the fused path)
  int fuse_grid_ = 0;
};

void launch_allreduce(const ArDevCtx* ctx, int world, float* data, size_t n, float* residual, hipStream_t st);

}  // namespace aios
