// RCCL collectives for the tensor-parallel engine: the library path next to the hand-written xGMI
// one-shot / two-shot kernels of comm.h (verdict r2: the north star names
// "RCCL all-reduce over xGMI").
//
// Role: comparator and fallback.  The decode-size all-reduces (16-256 KB per layer edge) are
// latency-bound and the one-shot IPC kernel pulls all 7 peers in one xGMI round trip, fused with
// the residual add; RCCL's ring / tree kernels are the reference point for prefill-size messages
// (MBs, where link bandwidth rules) and the path that needs no IPC-mappable memory (containers
// without dmabuf IPC).  Selected per TP tier by AIOS_TP_COMM=rccl (aios_amd/parallel/tp.py).
//
// librccl is dlopen'd at first use (no link-time dependency: the engine still loads on a node
// without RCCL, and the process may already hold torch's copy).  Every call is stream-ordered and
// graph-capturable (RCCL supports hipStreamBeginCapture), so the collectives sit inside the
// engine's captured decode step exactly where the xGMI kernels do.  One GPU per rank: RCCL
// refuses two ranks of a communicator on one device (the single-GPU TP tests use XgmiComm).
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <string>

#include "ops.h"

namespace aios {

class RcclComm {
 public:
  // 128-byte ncclUniqueId; rank 0 creates it, every rank passes the same bytes to the constructor
  static std::string unique_id();
  static bool available();  // librccl could be loaded and resolved
  RcclComm(int rank, int world, int device, const std::string& id);
  ~RcclComm();
  RcclComm(const RcclComm&) = delete;
  RcclComm& operator=(const RcclComm&) = delete;

  // sum n floats of `data` over the ranks (in place); with `residual`, the sum is then added into
  // it (the engine's C1/C2 contract: residual += sum of partials)
  void allreduce(float* data, size_t n, float* residual, hipStream_t st);
  // the same into `residual` ([rows][d]) with the split-RMSNorm producer outputs (ResidNorm, ops.h)
  // written by the residual-add kernel that follows the library all-reduce
  void allreduce_norm(float* data, int rows, int d, float* residual, const ResidNorm& nm, hipStream_t st);
  // every rank owns columns [r*slice, (r+1)*slice) of the rows x ld fp32 matrix `data`; afterwards
  // every rank holds all columns (in-place ncclAllGather per row, grouped)
  void allgather_cols(float* data, int rows, int slice, int ld, hipStream_t st);
  bool error() const;  // an asynchronous communicator error was reported
  void reset_error() {}
  int rank() const { return rank_; }
  int world() const { return world_; }

  static void hook(void* self, float* data, size_t n, float* residual, hipStream_t st);
  static void gather_hook(void* self, float* data, int rows, int slice, int ld, hipStream_t st);
  static void norm_hook(void* self, float* data, int rows, int d, float* residual, const ResidNorm& nm,
                        hipStream_t st);

 private:
  int rank_ = 0, world_ = 1, device_ = 0;
  void* comm_ = nullptr;  // ncclComm_t
};

}  // namespace aios
