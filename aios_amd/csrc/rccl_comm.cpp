// RCCL communicator (see rccl_comm.h): librccl resolved with dlopen/dlsym at first use.
#include "rccl_comm.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <stdexcept>

#include "common.h"
#include "ops.h"

namespace aios {

namespace {

struct RcclApi {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  bool ok = false;
  std::string why;
};

const RcclApi& api() {
  static RcclApi a;
  static std::once_flag once;
  std::call_once(once, [] {
    void* h = nullptr;
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      h = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (h) break;
    }
    if (!h) {
      a.why = std::string("dlopen(librccl) failed: ") + (dlerror() ? dlerror() : "?");
      return;
    }
    auto sym = [&](const char* s) {
      void* p = dlsym(h, s);
      if (!p && a.why.empty()) a.why = std::string("librccl lacks ") + s;
      return p;
    };
    a.GetUniqueId = (decltype(a.GetUniqueId))sym("ncclGetUniqueId");
    a.CommInitRank = (decltype(a.CommInitRank))sym("ncclCommInitRank");
    a.CommDestroy = (decltype(a.CommDestroy))sym("ncclCommDestroy");
    a.CommGetAsyncError = (decltype(a.CommGetAsyncError))sym("ncclCommGetAsyncError");
    a.AllReduce = (decltype(a.AllReduce))sym("ncclAllReduce");
    a.AllGather = (decltype(a.AllGather))sym("ncclAllGather");
    a.GroupStart = (decltype(a.GroupStart))sym("ncclGroupStart");
    a.GroupEnd = (decltype(a.GroupEnd))sym("ncclGroupEnd");
    a.GetErrorString = (decltype(a.GetErrorString))sym("ncclGetErrorString");
    a.ok = a.why.empty();
  });
  return a;
}

const RcclApi& need() {
  const RcclApi& a = api();
  if (!a.ok) throw std::runtime_error("RCCL unavailable: " + a.why);
  return a;
}

void check(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    const RcclApi& a = api();
    throw std::runtime_error(std::string("RCCL ") + what + ": " + (a.GetErrorString ? a.GetErrorString(r) : "error"));
  }
}

}  // namespace

bool RcclComm::available() { return api().ok; }

std::string RcclComm::unique_id() {
  const RcclApi& a = need();
  ncclUniqueId id;
  check(a.GetUniqueId(&id), "ncclGetUniqueId");
  return std::string(id.internal, sizeof(id.internal));
}

RcclComm::RcclComm(int rank, int world, int device, const std::string& id)
    : rank_(rank), world_(world), device_(device) {
  if (world < 1 || rank < 0 || rank >= world) throw std::invalid_argument("RcclComm: bad rank/world");
  if (id.size() != NCCL_UNIQUE_ID_BYTES) throw std::invalid_argument("RcclComm: unique id must be 128 bytes");
  const RcclApi& a = need();
  HIP_CHECK(hipSetDevice(device));
  ncclUniqueId uid;
  std::memcpy(uid.internal, id.data(), sizeof(uid.internal));
  ncclComm_t c = nullptr;
  check(a.CommInitRank(&c, world, uid, rank), "ncclCommInitRank");
  comm_ = c;
}

RcclComm::~RcclComm() {
  if (comm_) {
    const RcclApi& a = api();
    if (a.ok) a.CommDestroy((ncclComm_t)comm_);
  }
}

void RcclComm::allreduce(float* data, size_t n, float* residual, hipStream_t st) {
  if (world_ > 1) check(need().AllReduce(data, data, n, ncclFloat32, ncclSum, (ncclComm_t)comm_, st), "ncclAllReduce");
  if (residual) launch_add(residual, data, n, st);
}

void RcclComm::allreduce_norm(float* data, int rows, int d, float* residual, const ResidNorm& nm, hipStream_t st) {
  const size_t n = (size_t)rows * d;
  if (world_ > 1) check(need().AllReduce(data, data, n, ncclFloat32, ncclSum, (ncclComm_t)comm_, st), "ncclAllReduce");
  launch_add_norm(residual, data, rows, d, nm, st);
}

void RcclComm::allgather_cols(float* data, int rows, int slice, int ld, hipStream_t st) {
  if (world_ == 1) return;
  if (slice * world_ > ld) throw std::invalid_argument("RcclComm::allgather_cols: slice * world > ld");
  const RcclApi& a = need();
  // in place: the send buffer of row r is recvbuff + rank * slice, as ncclAllGather requires
  check(a.GroupStart(), "ncclGroupStart");
  for (int r = 0; r < rows; ++r) {
    float* row = data + (size_t)r * ld;
    check(a.AllGather(row + (size_t)rank_ * slice, row, (size_t)slice, ncclFloat32, (ncclComm_t)comm_, st),
          "ncclAllGather");
  }
  check(a.GroupEnd(), "ncclGroupEnd");
}

bool RcclComm::error() const {
  if (!comm_) return false;
  ncclResult_t r = ncclSuccess;
  if (need().CommGetAsyncError((ncclComm_t)comm_, &r) != ncclSuccess) return true;
  return r != ncclSuccess && r != ncclInProgress;
}

void RcclComm::hook(void* self, float* data, size_t n, float* residual, hipStream_t st) {
  static_cast<RcclComm*>(self)->allreduce(data, n, residual, st);
}

void RcclComm::norm_hook(void* self, float* data, int rows, int d, float* residual, const ResidNorm& nm,
                         hipStream_t st) {
  static_cast<RcclComm*>(self)->allreduce_norm(data, rows, d, residual, nm, st);
}

void RcclComm::gather_hook(void* self, float* data, int rows, int slice, int ld, hipStream_t st) {
  static_cast<RcclComm*>(self)->allgather_cols(data, rows, slice, ld, st);
}

}  // namespace aios
