// In-launch hand-offs between the workgroup roles of a fused decode launch (attn_block.hip:
// QKV GEMV -> attention -> O GEMV in ONE launch).
//
// MI355X rules (cdna_hip_programming.md Guideline 16, MI355X_MICROARCH.md 'inter-workgroup
// visibility'): per-XCD L2s are not coherent and a CU's L1 is never refreshed by another CU's
// stores, so every handed-off byte is stored write-through (sc1: relaxed agent-scope atomic
// stores), every storing wave drains its stores (s_waitcnt vmcnt(0)) before ONE lane of the
// workgroup adds to the edge's counter (agent-scope atomic), and the consumer polls the counter
// with sc1 loads and reads the handed-off bytes with sc1 loads -- bytes the consuming XCD never
// touched earlier in the launch, so no stale line can sit in its L2.
//
// Producers are always dispatched before their consumers (lower blockIdx; the dispatcher deals
// workgroups in index order) and never wait on them, so a waiting consumer cannot starve its
// producer of a CU slot.  Every wait is still bounded (~50 ms of s_memrealtime): a wait that gives
// up sets *err and lets the workgroup finish (its outputs are garbage, the host throws), so a
// broken hand-off can never hang the GPU.
#pragma once
#include "../common.h"

namespace aios {

struct FuseEdge {
  const int* wait = nullptr;  // counter this workgroup waits on (null: no wait)
  int target = 0;             // ... until it reaches this value
  int* sig = nullptr;         // counter this workgroup adds to once its outputs are written
  int* err = nullptr;         // set to 1 when a wait gives up
};

__device__ __forceinline__ uint64_t ld_sc1_8(const void* p) {
  return __hip_atomic_load((uint64_t*)const_cast<void*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// 16 bytes as two 8-byte sc1 loads (there is no 16-byte atomic load)
__device__ __forceinline__ uint4 ld_sc1_16(const void* p) {
  const uint64_t lo = ld_sc1_8(p), hi = ld_sc1_8((const uint8_t*)p + 8);
  return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}
__device__ __forceinline__ float4 ld_sc1_f4(const float* p) {
  const uint4 u = ld_sc1_16(p);
  return make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
}
__device__ __forceinline__ void st_sc1_f32(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_u32(void* p, uint32_t v) {
  __hip_atomic_store((uint32_t*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_sc1_f2(float* p, float v0, float v1) {
  const uint64_t u = (uint64_t)__float_as_uint(v0) | ((uint64_t)__float_as_uint(v1) << 32);
  __hip_atomic_store((uint64_t*)p, u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// whole workgroup: thread 0 polls until *e.wait >= e.target (bounded), then a barrier
__device__ __forceinline__ void fuse_wait(const FuseEdge& e) {
  if (threadIdx.x == 0 && e.wait) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz
    while (__hip_atomic_load(const_cast<int*>(e.wait), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < e.target) {
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 5000000ull) {  // 50 ms: give up, never hang
        if (e.err) __hip_atomic_store(e.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
    }
  }
  __syncthreads();
}

// whole workgroup: every wave drains its (write-through) stores, then one lane publishes n
__device__ __forceinline__ void fuse_signal(const FuseEdge& e, int n) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0 && e.sig) __hip_atomic_fetch_add(e.sig, n, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

}  // namespace aios
