// Common device/host definitions for the aiOS-MI355X inference engine (gfx950 / CDNA4).
//
// Everything here is written for wave64 CDNA4: lane = threadIdx.x & 63, 64-bit ballots,
// cross-lane reductions over 64 lanes with __shfl_xor.
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_fp16.h>
#include <stdint.h>
#include <cstring>
#include <type_traits>

#include <stdexcept>
#include <string>

#define AIOS_WAVE 64

#define HIP_CHECK(expr)                                                                   \
  do {                                                                                    \
    hipError_t _e = (expr);                                                               \
    if (_e != hipSuccess) {                                                               \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + " at " + \
                               __FILE__ + ":" + std::to_string(__LINE__) + " : " #expr);  \
    }                                                                                     \
  } while (0)

namespace aios {

// ggml type ids (GGUF on-disk ids)
enum QType : int {
  QT_F32 = 0,
  QT_F16 = 1,
  QT_Q4_0 = 2,
  QT_Q4_1 = 3,
  QT_Q5_0 = 6,
  QT_Q5_1 = 7,
  QT_Q8_0 = 8,
  QT_Q2_K = 10,  // load-time only: expanded to bf16 (kernels/quant_pack.hip legacy_to_bf16)
  QT_Q3_K = 11,
  QT_Q4_K = 12,
  QT_Q5_K = 13,
  QT_Q6_K = 14,
  QT_IQ4_NL = 20,  // load-time only, like Q2_K / Q3_K
  QT_IQ4_XS = 23,
  QT_BF16 = 30,
};

typedef uint16_t bf16_t;

__device__ __forceinline__ float bf16_to_f32(uint32_t h) { return __uint_as_float(h << 16); }

// ---- paged KV cache ------------------------------------------------------------------------------
// One layer's K (and V) pool is [n_blocks][n_kv_heads][KV_BLOCK][head_dim] bf16.  Row `slot` of a
// block table [slots][max_blocks] maps position / KV_BLOCK to a physical block, so slots share the
// full blocks of a common prompt prefix (refcounted, copy-on-write on the host: engine.hip).  A
// null table is the identity map block = slot * max_blocks + position / KV_BLOCK.  KV_BLOCK is
// the decode attention's pass length, so one pass reads one contiguous 32 KB block per KV head.
constexpr int KV_BLOCK = 128;
__host__ __device__ __forceinline__ int kv_block(const int* bt, int max_blocks, int slot, int pos) {
  const int j = pos / KV_BLOCK;
  return bt ? bt[slot * max_blocks + j] : slot * max_blocks + j;
}
__host__ __device__ __forceinline__ size_t kv_offset(const int* bt, int max_blocks, int slot, int n_kv_heads,
                                                     int kvh, int pos, int hd) {
  return (((size_t)kv_block(bt, max_blocks, slot, pos) * n_kv_heads + kvh) * KV_BLOCK + (pos % KV_BLOCK)) * hd;
}
__device__ __forceinline__ uint16_t f32_to_bf16(float f) {
  // round-to-nearest-even; NaN stays NaN
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}
__device__ __forceinline__ float h2f(uint16_t h) { return __half2float(__ushort_as_half(h)); }

// ---- KV cache element formats: bf16, or OCP fp8 e4m3 (gfx950's e4m3fn, max 448) with a per-layer
// K / V scale (EngineConfig::kv_fp8; value = code * scale).  Element indices are the same for both;
// an fp8 pool is addressed in bytes.
__device__ __forceinline__ uint32_t f32x2_to_fp8x2(float a, float b) {
  a = fminf(fmaxf(a, -448.f), 448.f);  // (saturate: e4m3fn has no infinity, an overflow is NaN)
  b = fminf(fmaxf(b, -448.f), 448.f);
  return (uint32_t)__builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false) & 0xffffu;
}
// K or V pair (v0 -> element i0, v1 -> element i1) of one token: one 4-B (bf16) / 2-B (fp8) store when
// adjacent; inv = 1 / the layer's scale (fp8 only)
__device__ __forceinline__ void kv_store_pair(bf16_t* cache, size_t i0, size_t i1, float v0, float v1, int fp8,
                                              float inv) {
  if (fp8) {
    uint8_t* c = (uint8_t*)cache;
    const uint32_t p = f32x2_to_fp8x2(v0 * inv, v1 * inv);
    if (i1 == i0 + 1 && !(i0 & 1)) {
      *(uint16_t*)(c + i0) = (uint16_t)p;
    } else {
      c[i0] = (uint8_t)(p & 0xff);
      c[i1] = (uint8_t)(p >> 8);
    }
  } else if (i1 == i0 + 1 && !(i0 & 1)) {
    *(uint32_t*)(cache + i0) = (uint32_t)f32_to_bf16(v0) | ((uint32_t)f32_to_bf16(v1) << 16);
  } else {
    cache[i0] = f32_to_bf16(v0);
    cache[i1] = f32_to_bf16(v1);
  }
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum over blockDim.x threads (multiple of 64, <= 1024). `red` has >= 16 floats.
__device__ __forceinline__ float block_sum(float v, float* red) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  float t = 0.f;
  for (int i = 0; i < nw; ++i) t += red[i];
  return t;
}

// 6-bit (scale, min) of sub-block j (0..7) of a Q4_K/Q5_K super-block.
__device__ __forceinline__ void kq_scale_min(int j, const uint8_t* q, int& sc, int& m) {
  if (j < 4) {
    sc = q[j] & 63;
    m = q[j + 4] & 63;
  } else {
    sc = (q[j + 4] & 0xF) | ((q[j - 4] >> 6) << 4);
    m = (q[j + 4] >> 4) | ((q[j] >> 6) << 4);
  }
}

// compile-time loop: f(std::integral_constant<int, I>{}) for I in [0, N) -- register arrays
// indexed by I stay in VGPRs even where the unroller would keep a runtime loop (and put the
// array in scratch)
template <int N, int I = 0, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<N, I + 1>(f);
  }
}

// Touch every 64-byte line of the kernel's argument block (BYTES of explicit arguments + the
// hidden-argument line after them) in ONE scalar-load clause, waited for once.  Left to itself the
// compiler loads kernarg fields where they are first used, and each s_waitcnt behind a scalar-cache
// miss costs an L2 round trip: the batch-1 row GEMV spent 0.67 us between its first instruction and
// its first weight load in four such waits (tools/gemv_cu_probe.py stamps, round 4).  After this the
// real field loads hit the scalar cache.
template <int BYTES>
__device__ __forceinline__ void kernarg_warm() {
  using kp_t = const __attribute__((address_space(4))) uint32_t*;
  const auto* kp = (const __attribute__((address_space(4))) uint8_t*)__builtin_amdgcn_kernarg_segment_ptr();
  uint32_t acc = 0;
  static_for<(BYTES + 63) / 64 + 1>([&](auto i) {
    constexpr int off = decltype(i)::value * 64;
    acc ^= *(kp_t)(kp + off);
  });
  asm volatile("" ::"s"(acc));
}

// per-lane choice between two kernel-argument pointers (K vs V cache of a QKV epilogue).  A plain
// `c ? a.p : a.q` lets LLVM turn it into a load through a selected address, i.e. an alloca copy of
// the two fields indexed per lane -- scratch in every kernel using it (round 4: 24 B in each
// batched LDS GEMV).  Pinning both values in SGPRs first keeps it a register select.
template <typename T>
__device__ __forceinline__ T* pick_ptr(bool first, T* p, T* q) {
  asm("" : "+s"(p), "+s"(q));
  return first ? p : q;
}

// roctx ranges around the engine's host-side phases (load, prefill chunk, decode step / graph
// replay, sampling): visible with `rocprofv3 --marker-trace` next to the kernel trace; ~free
// when no profiler is attached.  AIOS_TRACE=0 turns them off.
struct TraceRange {
  explicit TraceRange(const char* name);
  ~TraceRange();
  bool on;
};

// Per-thread CU budget: an engine whose stream is CU-masked (co-resident tiers, EngineConfig::cu_mask)
// sizes its one-workgroup-per-CU grids to its mask while it enqueues (CuScope); 0 = the whole device
inline int& cu_budget() {
  static thread_local int v = 0;
  return v;
}
struct CuScope {
  int saved;
  explicit CuScope(int n) : saved(cu_budget()) {
    if (n > 0) cu_budget() = n;
  }
  ~CuScope() { cu_budget() = saved; }
};

// CUs of the current device (host; cached per process), or the enqueuing engine's CU budget
inline int device_cu_count() {
  if (cu_budget() > 0) return cu_budget();
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  }
  return cus;
}

}  // namespace aios
