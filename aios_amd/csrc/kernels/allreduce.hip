// One-shot xGMI all-reduce for tensor parallelism (protocol in comm.h).
#include <cstring>
#include <stdexcept>

#include "../comm.h"
#include "../common.h"
#include "../ops.h"

namespace aios {

namespace {

constexpr int AR_THREADS = 256;
constexpr int AR_CHUNK = AR_THREADS * 4;                    // floats per WG iteration
constexpr uint64_t AR_TIMEOUT_TICKS = 100ull * 1000 * 1000 * 3;  // 3 s of the 100 MHz wall clock

__device__ __forceinline__ float4 ld_peer(const float* p) {
  float4 v;
  v.x = __builtin_nontemporal_load(p + 0);
  v.y = __builtin_nontemporal_load(p + 1);
  v.z = __builtin_nontemporal_load(p + 2);
  v.w = __builtin_nontemporal_load(p + 3);
  return v;
}

__global__ __launch_bounds__(AR_THREADS) void allreduce_oneshot(const ArDevCtx* __restrict__ c, float* __restrict__ data,
                                                                 size_t n, float* __restrict__ residual) {
  const int g = blockIdx.x, G = gridDim.x, t = threadIdx.x;
  const int rank = c->rank, world = c->world;
  __shared__ uint32_t s_e;
  if (t == 0) {
    const uint32_t e = c->epoch[g] + 1;  // only this WG touches epoch[g]
    c->epoch[g] = e;
    s_e = e;
  }
  __syncthreads();
  const uint32_t e = s_e;
  const size_t half = (size_t)(e & 1u) * c->cap;
  float* mine = c->buf[rank] + half;
  const size_t stride = (size_t)G * AR_CHUNK;
  // 1. stage my partial into my IPC buffer
  for (size_t i = ((size_t)g * AR_THREADS + t) * 4; i < n; i += stride) {
    if (i + 4 <= n) {
      *(float4*)(mine + i) = *(const float4*)(data + i);
    } else {
      for (size_t k = i; k < n; ++k) mine[k] = data[k];
    }
  }
  // 2. publish: every thread's stores are ordered before the flags
  __threadfence_system();
  __syncthreads();
  if (t < world && t != rank)
    __hip_atomic_store(c->flags[t] + g * AR_MAX_RANKS + rank, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  // 3. wait for every peer's epoch-e flag (bounded: an exit every wave reaches)
  if (t < world && t != rank) {
    uint32_t* f = c->flags[rank] + g * AR_MAX_RANKS + t;
    const uint64_t t0 = wall_clock64();
    while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (wall_clock64() - t0 > AR_TIMEOUT_TICKS) {
        __hip_atomic_store(c->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
  __threadfence_system();
  // 4. reduce: my partial (local) + every peer's staged partial (remote, over xGMI)
  for (size_t i = ((size_t)g * AR_THREADS + t) * 4; i < n; i += stride) {
    if (i + 4 <= n) {
      float4 acc = *(const float4*)(data + i);
#pragma unroll
      for (int p = 0; p < AR_MAX_RANKS; ++p) {
        if (p < world && p != rank) {
          const float4 v = ld_peer(c->buf[p] + half + i);
          acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
      }
      if (residual) {
        float4 r = *(float4*)(residual + i);
        r.x += acc.x; r.y += acc.y; r.z += acc.z; r.w += acc.w;
        *(float4*)(residual + i) = r;
      } else {
        *(float4*)(data + i) = acc;
      }
    } else {
      for (size_t k = i; k < n; ++k) {
        float acc = data[k];
        for (int p = 0; p < world; ++p)
          if (p != rank) acc += __builtin_nontemporal_load(c->buf[p] + half + k);
        if (residual) residual[k] += acc; else data[k] = acc;
      }
    }
  }
}

void* alloc_shared(size_t bytes) {
  // uncached device memory: remote stores / loads bypass both GPUs' caches
  void* p = nullptr;
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) == hipSuccess) return p;
  (void)hipGetLastError();
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained) == hipSuccess) return p;
  (void)hipGetLastError();
  HIP_CHECK(hipMalloc(&p, bytes));
  return p;
}

}  // namespace

void launch_allreduce(const ArDevCtx* ctx, int world, float* data, size_t n, float* residual, hipStream_t st) {
  (void)world;
  if (n == 0) return;
  const size_t chunks = (n + AR_CHUNK - 1) / AR_CHUNK;
  const int grid = (int)std::min<size_t>(chunks, AR_MAX_WG);
  hipLaunchKernelGGL(allreduce_oneshot, dim3(grid), dim3(AR_THREADS), 0, st, ctx, data, n, residual);
}

XgmiComm::XgmiComm(int rank, int world, int device, size_t cap_floats) : device_(device) {
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world) throw std::runtime_error("bad TP rank/world");
  HIP_CHECK(hipSetDevice(device));
  h_.rank = rank;
  h_.world = world;
  h_.cap = (cap_floats + 3) & ~size_t(3);
  mybuf_ = (float*)alloc_shared(2 * h_.cap * sizeof(float));
  myflags_ = (uint32_t*)alloc_shared(AR_MAX_WG * AR_MAX_RANKS * sizeof(uint32_t));
  HIP_CHECK(hipMemset(myflags_, 0, AR_MAX_WG * AR_MAX_RANKS * sizeof(uint32_t)));
  HIP_CHECK(hipMalloc(&h_.epoch, AR_MAX_WG * sizeof(uint32_t)));
  HIP_CHECK(hipMemset(h_.epoch, 0, AR_MAX_WG * sizeof(uint32_t)));
  h_.error = (uint32_t*)alloc_shared(64);
  HIP_CHECK(hipMemset(h_.error, 0, 64));
  h_.buf[rank] = mybuf_;
  h_.flags[rank] = myflags_;
  HIP_CHECK(hipMalloc(&d_, sizeof(ArDevCtx)));
  HIP_CHECK(hipMemcpy(d_, &h_, sizeof(ArDevCtx), hipMemcpyHostToDevice));
  HIP_CHECK(hipDeviceSynchronize());
  if (world == 1) connected_ = true;
}

XgmiComm::~XgmiComm() {
  hipSetDevice(device_);
  hipDeviceSynchronize();
  for (void* p : opened_) hipIpcCloseMemHandle(p);
  hipFree(d_);
  hipFree(h_.epoch);
  hipFree(h_.error);
  hipFree(mybuf_);
  hipFree(myflags_);
}

std::string XgmiComm::ipc_handle() const {
  hipIpcMemHandle_t a, b;
  HIP_CHECK(hipIpcGetMemHandle(&a, mybuf_));
  HIP_CHECK(hipIpcGetMemHandle(&b, myflags_));
  std::string s(sizeof(a) + sizeof(b), '\0');
  std::memcpy(&s[0], &a, sizeof(a));
  std::memcpy(&s[sizeof(a)], &b, sizeof(b));
  return s;
}

void XgmiComm::connect(const std::vector<std::string>& handles) {
  if ((int)handles.size() != h_.world) throw std::runtime_error("connect: need one handle per rank");
  HIP_CHECK(hipSetDevice(device_));
  for (int p = 0; p < h_.world; ++p) {
    if (p == h_.rank) continue;
    const std::string& s = handles[p];
    hipIpcMemHandle_t a, b;
    if (s.size() != sizeof(a) + sizeof(b)) throw std::runtime_error("connect: bad IPC handle size");
    std::memcpy(&a, s.data(), sizeof(a));
    std::memcpy(&b, s.data() + sizeof(a), sizeof(b));
    void *pa = nullptr, *pb = nullptr;
    HIP_CHECK(hipIpcOpenMemHandle(&pa, a, hipIpcMemLazyEnablePeerAccess));
    opened_.push_back(pa);
    HIP_CHECK(hipIpcOpenMemHandle(&pb, b, hipIpcMemLazyEnablePeerAccess));
    opened_.push_back(pb);
    h_.buf[p] = (float*)pa;
    h_.flags[p] = (uint32_t*)pb;
  }
  HIP_CHECK(hipMemcpy(d_, &h_, sizeof(ArDevCtx), hipMemcpyHostToDevice));
  HIP_CHECK(hipDeviceSynchronize());
  connected_ = true;
}

void XgmiComm::allreduce(float* data, size_t n, float* residual, hipStream_t st) {
  if (!connected_) throw std::runtime_error("XgmiComm: allreduce before connect()");
  if (n > h_.cap) throw std::runtime_error("XgmiComm: message of " + std::to_string(n) + " floats exceeds capacity " +
                                           std::to_string(h_.cap));
  if (h_.world == 1) {
    if (residual) launch_add(residual, data, n, st);
    return;
  }
  launch_allreduce(d_, h_.world, data, n, residual, st);
}

bool XgmiComm::error() const {
  uint32_t e = 0;
  HIP_CHECK(hipMemcpy(&e, h_.error, sizeof(e), hipMemcpyDeviceToHost));
  return e != 0;
}

void XgmiComm::reset_error() { HIP_CHECK(hipMemset(h_.error, 0, 4)); }

void XgmiComm::hook(void* self, float* data, size_t n, float* residual, hipStream_t st) {
  static_cast<XgmiComm*>(self)->allreduce(data, n, residual, st);
}

}  // namespace aios
