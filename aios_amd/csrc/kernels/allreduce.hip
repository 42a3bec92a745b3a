// xGMI collectives for tensor parallelism: one-shot and two-shot (reduce-scatter + all-gather)
// all-reduce, column all-gather.  Protocol and buffer ownership in comm.h.
#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "../comm.h"
#include "../common.h"
#include "../ops.h"

namespace aios {

namespace {

constexpr uint64_t AR_TIMEOUT_TICKS = 100ull * 1000 * 1000 * 3;  // 3 s of the 100 MHz wall clock

__device__ __forceinline__ float4 ld_peer(const float* p) {
  float4 v;
  v.x = __builtin_nontemporal_load(p + 0);
  v.y = __builtin_nontemporal_load(p + 1);
  v.z = __builtin_nontemporal_load(p + 2);
  v.w = __builtin_nontemporal_load(p + 3);
  return v;
}

__device__ __forceinline__ uint32_t flag_idx(int phase, int g, int r) {
  return ((uint32_t)phase * AR_MAX_WG + g) * AR_MAX_RANKS + r;
}

// this WG's epoch (one increment per call), broadcast through LDS
__device__ __forceinline__ uint32_t next_epoch(const ArDevCtx* c, int g, uint32_t* s_e) {
  if (threadIdx.x == 0) {
    const uint32_t e = c->epoch[g] + 1;  // only this WG touches epoch[g]
    c->epoch[g] = e;
    *s_e = e;
  }
  __syncthreads();
  return *s_e;
}

// every thread's stores are ordered before the flags; one lane per peer raises its flag
__device__ __forceinline__ void publish(const ArDevCtx* c, int phase, int g, uint32_t e) {
  __threadfence_system();
  __syncthreads();
  const int t = threadIdx.x;
  if (t < c->world && t != c->rank)
    __hip_atomic_store(c->flags[t] + flag_idx(phase, g, c->rank), e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// wait for every peer's epoch-e flag of `phase` (bounded: an exit every wave reaches)
__device__ __forceinline__ void wait_peers(const ArDevCtx* c, int phase, int g, uint32_t e) {
  const int t = threadIdx.x;
  if (t < c->world && t != c->rank) {
    uint32_t* f = c->flags[c->rank] + flag_idx(phase, g, t);
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
}

__device__ __forceinline__ void put(float* data, float* residual, size_t i, float4 v) {
  if (residual) {
    float4 r = *(float4*)(residual + i);
    r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
    *(float4*)(residual + i) = r;
  } else {
    *(float4*)(data + i) = v;
  }
}

// ---- split-RMSNorm producer (ResidNorm, ops.h) for one RNORM_COLS-column block j of row m: r holds
// this thread's 4 new residual values at column j * RNORM_COLS + 4 t.  The block's sum of squares is
// reduced in a fixed order, so every TP rank (same residual bits) writes the same parts.  Every
// thread of the workgroup calls it.
static_assert(AR_CHUNK == RNORM_COLS, "one all-reduce workgroup = one norm column block");
__device__ __forceinline__ void norm_block(const ResidNorm& nm, int m, int j, int ncb, int t, float4 r) {
  __shared__ float s_red[AR_THREADS / 64];
  const int col = j * RNORM_COLS + 4 * t;
  const float4 g = *(const float4*)(nm.g + col);
  *(uint2*)(nm.out16 + (size_t)m * nm.ld16 + col) =
      make_uint2((uint32_t)f32_to_bf16(r.x * g.x) | ((uint32_t)f32_to_bf16(r.y * g.y) << 16),
                 (uint32_t)f32_to_bf16(r.z * g.z) | ((uint32_t)f32_to_bf16(r.w * g.w) << 16));
  float s = r.x * r.x + r.y * r.y + r.z * r.z + r.w * r.w;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((t & 63) == 0) s_red[t >> 6] = s;
  __syncthreads();
  if (t == 0) {
    float tot = 0.f;
#pragma unroll
    for (int w = 0; w < AR_THREADS / 64; ++w) tot += s_red[w];
    nm.part[(size_t)m * nm.parts + j] = tot;
  }
  if (j == 0 && t >= ncb && t < nm.parts) nm.part[(size_t)m * nm.parts + t] = 0.f;  // padding parts
}

// residual += data (data null: residual already holds the sum), then the norm outputs
__global__ __launch_bounds__(AR_THREADS) void add_norm_kernel(float* __restrict__ residual, const float* __restrict__ data,
                                                              int d, ResidNorm nm) {
  const int j = blockIdx.x, m = blockIdx.y, t = threadIdx.x;
  const size_t i = (size_t)m * d + (size_t)j * RNORM_COLS + 4 * t;
  float4 r = *(const float4*)(residual + i);
  if (data) {
    const float4 v = *(const float4*)(data + i);
    r.x += v.x; r.y += v.y; r.z += v.z; r.w += v.w;
    *(float4*)(residual + i) = r;
  }
  norm_block(nm, m, j, d / RNORM_COLS, t, r);
}

// ---- one-shot: every rank pulls every peer's whole partial (decode-size messages).  The sum runs
// in rank order on every rank (own partial at its rank's position), so all ranks produce the
// bit-identical result and their on-device samplers stay in lock step.  NORM (C1 / C2 of the
// batched TP decode): residual required, n = rows * d with d % RNORM_COLS == 0, and the workgroup
// also writes the split-RMSNorm outputs of its column block (no separate RMSNorm launch).
template <bool NORM>
__global__ __launch_bounds__(AR_THREADS) void allreduce_oneshot(const ArDevCtx* __restrict__ c, float* __restrict__ data,
                                                                 size_t n, float* __restrict__ residual, int d,
                                                                 ResidNorm nm) {
  __shared__ uint32_t s_e;
  const int g = blockIdx.x, t = threadIdx.x;
  const int rank = c->rank, world = c->world;
  const uint32_t e = next_epoch(c, g, &s_e);
  const size_t half = (size_t)(e & 1u) * c->cap;
  float* mine = c->buf[rank] + half;
  const size_t i = (size_t)g * AR_CHUNK + 4 * t;
  const bool full = i + 4 <= n;
  if (full) *(float4*)(mine + i) = *(const float4*)(data + i);
  else for (size_t k = i; k < n; ++k) mine[k] = data[k];
  publish(c, 0, g, e);
  wait_peers(c, 0, g, e);
  if (full) {
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
    for (int p = 0; p < AR_MAX_RANKS; ++p) {
      if (p < world) {
        const float4 v = p == rank ? *(const float4*)(data + i) : ld_peer(c->buf[p] + half + i);
        acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
      }
    }
    if constexpr (NORM) {
      float4 r = *(const float4*)(residual + i);
      r.x += acc.x; r.y += acc.y; r.z += acc.z; r.w += acc.w;
      *(float4*)(residual + i) = r;
      const size_t e0 = (size_t)g * AR_CHUNK;  // the workgroup's first element: one row, one column block
      norm_block(nm, (int)(e0 / d), (int)(e0 % d) / RNORM_COLS, d / RNORM_COLS, t, r);
      return;
    }
    put(data, residual, i, acc);
  } else {
    for (size_t k = i; k < n; ++k) {
      float acc = 0.f;
      for (int p = 0; p < world; ++p) acc += p == rank ? data[k] : __builtin_nontemporal_load(c->buf[p] + half + k);
      if (residual) residual[k] += acc; else data[k] = acc;
    }
  }
}

// ---- two-shot: reduce-scatter (each rank sums its 1/world sub-shard of the chunk, pulling the
// peers' staged partials -- bf16 when BF16, halving the link bytes) then all-gather of the reduced
// sub-shards.  Each element is reduced once, by its owner, so every rank gets identical bits.
// The host launches it only for n % 4 == 0.
template <bool BF16>
__global__ __launch_bounds__(AR_THREADS) void allreduce_twoshot(const ArDevCtx* __restrict__ c, float* __restrict__ data,
                                                                 size_t n, float* __restrict__ residual) {
  __shared__ uint32_t s_e;
  const int g = blockIdx.x, t = threadIdx.x;
  const int rank = c->rank, world = c->world;
  const uint32_t e = next_epoch(c, g, &s_e);
  const size_t half = (size_t)(e & 1u) * c->cap;
  const size_t base = (size_t)g * AR_CHUNK;
  // 1. stage my partial of the chunk (bf16: rounded once here, summed in fp32 by the owner)
  {
    const size_t i = base + 4 * t;
    if (i + 4 <= n) {
      const float4 v = *(const float4*)(data + i);
      if constexpr (BF16) {
        uint16_t* s16 = (uint16_t*)(c->buf[rank] + 4 * c->cap);
        *(uint2*)(s16 + half + i) = make_uint2((uint32_t)f32_to_bf16(v.x) | ((uint32_t)f32_to_bf16(v.y) << 16),
                                               (uint32_t)f32_to_bf16(v.z) | ((uint32_t)f32_to_bf16(v.w) << 16));
      } else {
        *(float4*)(c->buf[rank] + half + i) = v;
      }
    }
  }
  publish(c, 0, g, e);
  wait_peers(c, 0, g, e);
  // 2. reduce-scatter: float4 groups [lo, hi) of the chunk belong to this rank
  const int nq = AR_CHUNK / 4;
  const int lo = rank * nq / world, hi = (rank + 1) * nq / world;
  for (int f = lo + t; f < hi; f += AR_THREADS) {
    const size_t i = base + 4 * (size_t)f;
    if (i + 4 > n) continue;
    float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
    for (int p = 0; p < world; ++p) {
      float4 v;
      if (p == rank) {
        v = *(const float4*)(data + i);
      } else if constexpr (BF16) {
        const uint16_t* s16 = (const uint16_t*)(c->buf[p] + 4 * c->cap);
        typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
        const u32x2_t u = __builtin_nontemporal_load((const u32x2_t*)(s16 + half + i));
        v = make_float4(bf16_to_f32(u.x & 0xffff), bf16_to_f32(u.x >> 16), bf16_to_f32(u.y & 0xffff),
                        bf16_to_f32(u.y >> 16));
      } else {
        v = ld_peer(c->buf[p] + half + i);
      }
      acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
    }
    *(float4*)(c->buf[rank] + 2 * c->cap + half + i) = acc;  // my reduced sub-shard
    put(data, residual, i, acc);
  }
  publish(c, 1, g, e);
  wait_peers(c, 1, g, e);
  // 3. all-gather the other ranks' reduced sub-shards
  for (int p = 0; p < world; ++p) {
    if (p == rank) continue;
    const int plo = p * nq / world, phi = (p + 1) * nq / world;
    for (int f = plo + t; f < phi; f += AR_THREADS) {
      const size_t i = base + 4 * (size_t)f;
      if (i + 4 > n) continue;
      put(data, residual, i, ld_peer(c->buf[p] + 2 * c->cap + half + i));
    }
  }
}

// ---- column all-gather: position j = r*rows*slice + b*slice + col is owned by rank r
__global__ __launch_bounds__(AR_THREADS) void allgather_cols_kernel(const ArDevCtx* __restrict__ c,
                                                                    float* __restrict__ data, int rows, int slice,
                                                                    int ld) {
  __shared__ uint32_t s_e;
  const int g = blockIdx.x, t = threadIdx.x;
  const int rank = c->rank;
  const uint32_t e = next_epoch(c, g, &s_e);
  const size_t half = (size_t)(e & 1u) * c->cap;
  const size_t per = (size_t)rows * slice, total = per * c->world;
  float* mine = c->buf[rank] + half;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const size_t j = (size_t)g * AR_CHUNK + k * AR_THREADS + t;
    if (j < total && (int)(j / per) == rank) {
      const size_t w = j % per;
      mine[j] = data[(w / slice) * (size_t)ld + (size_t)rank * slice + w % slice];
    }
  }
  publish(c, 0, g, e);
  wait_peers(c, 0, g, e);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const size_t j = (size_t)g * AR_CHUNK + k * AR_THREADS + t;
    const int r = (int)(j / per);
    if (j < total && r != rank) {
      const size_t w = j % per;
      data[(w / slice) * (size_t)ld + (size_t)r * slice + w % slice] = __builtin_nontemporal_load(c->buf[r] + half + j);
    }
  }
}

void* alloc_shared(size_t bytes, bool* uncached = nullptr) {
  // uncached device memory: remote stores / loads bypass both GPUs' caches
  void* p = nullptr;
  if (uncached) *uncached = true;
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) == hipSuccess) return p;
  if (uncached) *uncached = false;
  (void)hipGetLastError();
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocFinegrained) == hipSuccess) return p;
  (void)hipGetLastError();
  HIP_CHECK(hipMalloc(&p, bytes));
  return p;
}

int grid_for(size_t n) { return (int)std::max<size_t>(1, (n + AR_CHUNK - 1) / AR_CHUNK); }

}  // namespace

void launch_allreduce(const ArDevCtx* ctx, int world, float* data, size_t n, float* residual, hipStream_t st) {
  (void)world;
  if (n == 0) return;
  if (n > AR_MAX_CALL) throw std::runtime_error("launch_allreduce: call above AR_MAX_CALL elements");
  hipLaunchKernelGGL((allreduce_oneshot<false>), dim3(grid_for(n)), dim3(AR_THREADS), 0, st, ctx, data, n, residual, 0,
                     ResidNorm{});
}

void launch_add_norm(float* residual, const float* data, int rows, int d, const ResidNorm& nm, hipStream_t st) {
  if (rows <= 0) return;
  if (d % RNORM_COLS || nm.parts < d / RNORM_COLS || nm.parts > 64 || nm.parts % 4)
    throw std::runtime_error("launch_add_norm: d must be a multiple of 1024 and parts = resid_norm_parts(d)");
  hipLaunchKernelGGL(add_norm_kernel, dim3(d / RNORM_COLS, rows), dim3(AR_THREADS), 0, st, residual, data, d, nm);
}

XgmiComm::XgmiComm(int rank, int world, int device, size_t cap_floats) : device_(device) {
  if (world < 1 || world > AR_MAX_RANKS || rank < 0 || rank >= world) throw std::runtime_error("bad TP rank/world");
  HIP_CHECK(hipSetDevice(device));
  h_.rank = rank;
  h_.world = world;
  // every call moves at most AR_MAX_CALL elements (larger messages are split), so the buffers
  // are sized for that regardless of the requested capacity: 5 x 2 MB per rank
  (void)cap_floats;
  h_.cap = AR_MAX_CALL;
  // + the fused GEMV epilogue's stage [TPF_SLOTS][2][TPF_CAP] and flags [TPF_SLOTS][ranks]
  bool unc0 = false, unc1 = false;
  mybuf_ = (float*)alloc_shared((5 * h_.cap + (size_t)2 * TPF_SLOTS * TPF_CAP) * sizeof(float), &unc0);
  const size_t nflags = (size_t)(2 * AR_MAX_WG + TPF_SLOTS) * AR_MAX_RANKS;
  myflags_ = (uint32_t*)alloc_shared(nflags * sizeof(uint32_t), &unc1);
  // the fused epilogue's fence-free hand-off relies on uncached stage / flags (lg_tp_fuse)
  uncached_ = unc0 && unc1;
  HIP_CHECK(hipMemset(myflags_, 0, nflags * sizeof(uint32_t)));
  HIP_CHECK(hipMalloc(&h_.epoch, AR_MAX_WG * sizeof(uint32_t)));
  HIP_CHECK(hipMemset(h_.epoch, 0, AR_MAX_WG * sizeof(uint32_t)));
  HIP_CHECK(hipMalloc(&h_.fepoch, TPF_SLOTS * sizeof(uint32_t)));
  HIP_CHECK(hipMemset(h_.fepoch, 0, TPF_SLOTS * sizeof(uint32_t)));
  if (const char* e = std::getenv("AIOS_TP_FUSE")) fuse_on_ = std::atoi(e) != 0;
  {
    void* hp = nullptr;
    HIP_CHECK(hipHostMalloc(&hp, 64, hipHostMallocMapped));
    std::memset(hp, 0, 64);
    host_error_ = (volatile uint32_t*)hp;
    void* dp = nullptr;
    HIP_CHECK(hipHostGetDevicePointer(&dp, hp, 0));
    h_.error = (uint32_t*)dp;
  }
  h_.buf[rank] = mybuf_;
  h_.flags[rank] = myflags_;
  HIP_CHECK(hipMalloc(&d_, sizeof(ArDevCtx)));
  HIP_CHECK(hipMemcpy(d_, &h_, sizeof(ArDevCtx), hipMemcpyHostToDevice));
  HIP_CHECK(hipDeviceSynchronize());
  if (const char* e = std::getenv("AIOS_TP_TWO_SHOT_MIN")) two_shot_min_ = (size_t)std::atoll(e);
  if (const char* e = std::getenv("AIOS_TP_BF16")) bf16_ = std::atoi(e) != 0;
  if (world == 1) connected_ = true;
}

XgmiComm::~XgmiComm() {
  hipSetDevice(device_);
  hipDeviceSynchronize();
  for (void* p : opened_) hipIpcCloseMemHandle(p);
  hipFree(d_);
  hipFree(h_.epoch);
  hipFree(h_.fepoch);
  hipHostFree((void*)host_error_);
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

void XgmiComm::set_ranks_per_gpu(int n) {
  fuse_grid_ = n > 1 ? std::max(1, device_cu_count() / n) : 0;
}

void XgmiComm::set_call_wg(int wg) {
  call_cap_ = (size_t)std::max(1, std::min(AR_MAX_WG, wg)) * AR_CHUNK;
}

void XgmiComm::allreduce(float* data, size_t n, float* residual, hipStream_t st) {
  if (!connected_) throw std::runtime_error("XgmiComm: allreduce before connect()");
  if (h_.world == 1) {
    if (residual) launch_add(residual, data, n, st);
    return;
  }
  for (size_t off = 0; off < n; off += call_cap_) {
    const size_t m = std::min(call_cap_, n - off);
    float* d = data + off;
    float* r = residual ? residual + off : nullptr;
    if (m >= two_shot_min_ && m % 4 == 0) {
      if (bf16_)
        hipLaunchKernelGGL((allreduce_twoshot<true>), dim3(grid_for(m)), dim3(AR_THREADS), 0, st, d_, d, m, r);
      else
        hipLaunchKernelGGL((allreduce_twoshot<false>), dim3(grid_for(m)), dim3(AR_THREADS), 0, st, d_, d, m, r);
    } else {
      launch_allreduce(d_, h_.world, d, m, r, st);
    }
  }
}

void XgmiComm::allreduce_norm(float* data, int rows, int d, float* residual, const ResidNorm& nm, hipStream_t st) {
  if (!connected_) throw std::runtime_error("XgmiComm: allreduce before connect()");
  const size_t n = (size_t)rows * d;
  if (h_.world == 1) {
    launch_add_norm(residual, data, rows, d, nm, st);
  } else if (d % RNORM_COLS == 0 && n <= call_cap_ && n < two_shot_min_) {
    if (nm.parts < d / RNORM_COLS || nm.parts > 64 || nm.parts % 4)
      throw std::runtime_error("XgmiComm::allreduce_norm: parts must be resid_norm_parts(d)");
    hipLaunchKernelGGL((allreduce_oneshot<true>), dim3(grid_for(n)), dim3(AR_THREADS), 0, st, d_, data, n, residual, d,
                       nm);
  } else {
    allreduce(data, n, residual, st);
    launch_add_norm(residual, nullptr, rows, d, nm, st);
  }
}

void XgmiComm::allgather_cols(float* data, int rows, int slice, int ld, hipStream_t st) {
  if (!connected_) throw std::runtime_error("XgmiComm: allgather before connect()");
  if (h_.world == 1 || rows <= 0) return;
  if ((size_t)h_.world * slice > call_cap_) throw std::runtime_error("XgmiComm: all-gather slice above capacity");
  const int rows_per = (int)std::max<size_t>(1, call_cap_ / ((size_t)h_.world * slice));
  for (int r0 = 0; r0 < rows; r0 += rows_per) {
    const int nr = std::min(rows_per, rows - r0);
    const size_t total = (size_t)h_.world * nr * slice;
    hipLaunchKernelGGL(allgather_cols_kernel, dim3(grid_for(total)), dim3(AR_THREADS), 0, st, d_,
                       data + (size_t)r0 * ld, nr, slice, ld);
  }
}

// a host load of the mapped flag: reports give-ups of work that has COMPLETED (callers that need
// the verdict of a step check after their synchronisation point)
bool XgmiComm::error() const { return host_error_[0] != 0; }

void XgmiComm::reset_error() { host_error_[0] = 0; }

void XgmiComm::hook(void* self, float* data, size_t n, float* residual, hipStream_t st) {
  static_cast<XgmiComm*>(self)->allreduce(data, n, residual, st);
}

void XgmiComm::norm_hook(void* self, float* data, int rows, int d, float* residual, const ResidNorm& nm,
                         hipStream_t st) {
  static_cast<XgmiComm*>(self)->allreduce_norm(data, rows, d, residual, nm, st);
}

void XgmiComm::gather_hook(void* self, float* data, int rows, int slice, int ld, hipStream_t st) {
  static_cast<XgmiComm*>(self)->allgather_cols(data, rows, slice, ld, st);
}

}  // namespace aios
