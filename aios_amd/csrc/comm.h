// Tensor-parallel collectives for one MI355X node: a one-shot all-reduce over IPC-mapped peer
// buffers (each GPU reads its <=7 peers directly over the point-to-point xGMI links), used for the
// row-parallel o_proj / down_proj partial sums of the TP "strategic" tier.
//
// Why not a ring: a decode all-reduce is 16-64 KB; a ring pays 2(N-1) latency hops and is
// bound by one link, while the one-shot pull reads all peers in parallel across the 7 links and
// finishes in ~one xGMI round trip.  Prefill chunks (<= 64 rows x d) fit the same buffers.
//
// Protocol (per workgroup g, epoch e = this WG's launch counter, identical on every rank because
// every rank issues the same sequence of collectives):
//   1. copy my chunk of the input into my IPC buffer half  e & 1
//   2. release fence (system scope), then store e into flag[g][my_rank] of every peer
//   3. wait until my own flag[g][p] >= e for every peer p (bounded spin -> error flag, never hangs)
//   4. out = sum over ranks of buf_p[e & 1][chunk]   (+ residual when fused)
// Double buffering is safe: a rank can only reuse half e&1 at epoch e+2, which needs every peer's
// epoch-(e+1) flag, which a peer sets only after it finished reading epoch e.
// Flags / buffers are uncached device memory (hipDeviceMallocUncached), so remote stores and
// loads bypass the caches of both GPUs; works both across GPUs (xGMI) and between processes that
// share one GPU (how the TP path is tested on a single-GPU box).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace aios {

constexpr int AR_MAX_RANKS = 8;
constexpr int AR_MAX_WG = 512;

struct ArDevCtx {
  float* buf[AR_MAX_RANKS];         // rank r's data buffer (mapped into this process): [2][cap]
  uint32_t* flags[AR_MAX_RANKS];    // rank r's flag array: [AR_MAX_WG][AR_MAX_RANKS]
  uint32_t* epoch;                  // my per-WG epoch counters [AR_MAX_WG] (local)
  uint32_t* error;                  // set to 1 when a wait timed out
  int rank, world;
  size_t cap;                       // floats per half-buffer
};

class XgmiComm {
 public:
  XgmiComm(int rank, int world, int device, size_t cap_floats);
  ~XgmiComm();
  // opaque IPC handles of my data + flag buffers (hipIpcMemHandle_t x 2)
  std::string ipc_handle() const;
  // map every peer's buffers (handles indexed by rank; my own entry is ignored)
  void connect(const std::vector<std::string>& handles);
  bool connected() const { return connected_; }
  // sum `n` floats of `data` over all ranks; result into `data`, or added into `residual`
  // (data left as my partial) when residual != nullptr.  Stream-ordered, graph-capturable.
  void allreduce(float* data, size_t n, float* residual, hipStream_t st);
  bool error() const;
  void reset_error();
  int rank() const { return h_.rank; }
  int world() const { return h_.world; }
  size_t capacity() const { return h_.cap; }
  // Engine hook (AllReduceFn-compatible trampoline)
  static void hook(void* self, float* data, size_t n, float* residual, hipStream_t st);

 private:
  ArDevCtx h_{};
  ArDevCtx* d_ = nullptr;        // device copy of h_
  float* mybuf_ = nullptr;
  uint32_t* myflags_ = nullptr;
  std::vector<void*> opened_;
  int device_ = 0;
  bool connected_ = false;
};

void launch_allreduce(const ArDevCtx* ctx, int world, float* data, size_t n, float* residual, hipStream_t st);

}  // namespace aios
