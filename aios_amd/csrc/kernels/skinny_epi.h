// Output stage shared by the batched-decode MFMA GEMMs (gemm_skinny.hip: weights streamed into
// registers; gemm_ring.hip: weights streamed through an LDS-DMA ring): one 16 x (16 MT) block of
// D[n][m] per wave (lane: D[n0 + 16 wave + 4 q + j][16 mt + rr], j = 0..3) goes through the epilogue
// (store / residual add / SwiGLU bf16 / RoPE + KV-cache write / residual + split-RMSNorm producer),
// directly for S == 1, else through write-through fp32 slabs reduced by the tile's last-arriving
// workgroup (relaxed agent ticket + one agent acquire; CDNA guide §5 "in-launch split-K reduction").
#pragma once
#include "gemm_common.h"

namespace aios {

constexpr int SK_SB = 8;  // slices summed per batch of loads in the last arriver

// Returns false for a split-K workgroup that was not its tile's last arriver (nothing written).
// red: >= RB * 16 * MT floats of workgroup-shared scratch (free after the main loop);
// last_flag: a __shared__ int of the caller.  NTB: threads of the workgroup, which ALL call this
// (waves past the RB MFMA waves -- the ring GEMM's loaders -- hold no outputs but take part in
// the barriers and the split-K reduction).
template <int RB, int MT, int EPI, int NTB = RB * 64>
__device__ __forceinline__ bool sk_epilogue(const GemmQArgs& a, gf32x4 (&acc)[MT], int n0, int rg, int sp, int S,
                                            int ntile, const float* inv_s, bool nrm, float* red, int& last_flag) {
  constexpr int NT = NTB, ROWS = 16 * RB, MP = 16 * MT;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool active = wave < RB;  // holds D values
  const int rr = lane & 15, q = lane >> 4;
  // ---- epilogue.  lane holds D[n = 4q + j][m = 16 mt + rr], j = 0..3
  const int nl = 16 * wave + 4 * q;  // tile-local first row of this lane's 4 outputs
  // returns the sum of squares of the new residual row slice (GEPI_ACCUM_NORM), else 0
  auto finish = [&](int m, int n, gf32x4 v) __attribute__((always_inline)) -> float {
    if (m >= a.M) return 0.f;
    if (nrm) v *= inv_s[m];
    if constexpr (EPI == GEPI_SWIGLU_BF16) {
      const uint32_t pk = pk_bf16(v[0] / (1.f + __expf(-v[0])) * v[1], v[2] / (1.f + __expf(-v[2])) * v[3]);
      *(uint32_t*)(a.C16 + (size_t)m * a.ldc + (n >> 1)) = pk;
    } else if constexpr (EPI == GEPI_QKV) {
      // the lane's 4 consecutive columns are two RoPE pairs (2i, 2i + 1)
      const int hd = a.head_dim, pos = a.pos[m], slot = a.slot ? a.slot[m] : 0;
#pragma unroll
      for (int j = 0; j < 4; j += 2) {
        const int c = a.col0 + n + j;
        float v0 = v[j], v1 = v[j + 1];
        const int part = c < a.q_dim ? 0 : (c < a.q_dim + a.kv_dim ? 1 : 2);
        const int r = c - (part == 0 ? 0 : (part == 1 ? a.q_dim : a.q_dim + a.kv_dim));
        const int head = r / hd, lr = r - head * hd;
        if (part < 2) {
          const float2 t = a.rope_cs[(size_t)pos * (hd >> 1) + (lr >> 1)];
          const float o0 = v0 * t.x - v1 * t.y, o1 = v0 * t.y + v1 * t.x;
          v0 = o0;
          v1 = o1;
        }
        if (part == 0) {
          *(float2*)(a.q_out + (size_t)m * a.q_dim + c) = make_float2(v0, v1);
        } else {
          bf16_t* cache = part == 1 ? a.k_cache : a.v_cache;
          const size_t base = kv_offset(a.block_table, a.max_ctx / KV_BLOCK, slot, a.n_kv_heads, head, pos, hd);
          if (a.kv_fp8) kv_store_pair(cache, base + lr, base + lr + 1, v0, v1, 1, part == 1 ? a.kv_inv_k : a.kv_inv_v);
          else *(uint32_t*)(cache + base + lr) = pk_bf16(v0, v1);
        }
      }
    } else {
      float4* c = (float4*)(a.C + (size_t)m * a.ldc + n);
      if constexpr (EPI == GEPI_ACCUM_NORM) {
        const float4 o = *c;
        const float4 x = make_float4(o.x + v[0], o.y + v[1], o.z + v[2], o.w + v[3]);
        *c = x;
        const float4 g = *(const float4*)(a.nrm_g + n);
        *(uint2*)(a.nrm_out16 + (size_t)m * a.ldc + n) = make_uint2(pk_bf16(x.x * g.x, x.y * g.y),
                                                                      pk_bf16(x.z * g.z, x.w * g.w));
        return (x.x * x.x + x.y * x.y) + (x.z * x.z + x.w * x.w);
      } else if constexpr (EPI == GEPI_ACCUM) {
        const float4 o = *c;
        *c = make_float4(o.x + v[0], o.y + v[1], o.z + v[2], o.w + v[3]);
      } else {
        *c = make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    return 0.f;
  };
  if (S == 1) {
    float ss[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) ss[mt] = active ? finish(16 * mt + rr, n0 + nl, acc[mt]) : 0.f;
    if constexpr (EPI == GEPI_ACCUM_NORM) {
      // tile partial per row: the 4 q lanes of a wave (shuffles), then the RB waves (LDS, in
      // wave order); Xs is free after the main loop's last barrier
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        float s = ss[mt];
        s += __shfl_xor(s, 16, 64);
        s += __shfl_xor(s, 32, 64);
        if (q == 0 && active) red[wave * MP + 16 * mt + rr] = s;
      }
      __syncthreads();
      if (tid < a.M) {
        float s = red[tid];
        for (int w = 1; w < RB; ++w) s += red[w * MP + tid];
        a.nrm_part[(size_t)tid * a.nrm_parts + rg] = s;
      }
    }
    return true;
  }
  // split-K: slab [sp][rg][MP][ROWS] written through (sc1: no release fence needed), then the
  // last arriver of the tile (relaxed agent ticket) acquires and reduces (CDNA guide §5 item 2)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)a.ws, (short)0, 0x7fffffff, 0x00020000);
  const int sbase = (int)(((size_t)sp * ntile + rg) * MP * ROWS * 4);
#pragma unroll
  for (int mt = 0; mt < MT; ++mt)
    if (active) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(gu32x4, acc[mt]), rs,
                                           sbase + ((16 * mt + rr) * ROWS + nl) * 4, 0, 16 /* sc1 */);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its slab stores
  __syncthreads();
  if (tid == 0) {
    const int t = __hip_atomic_fetch_add(a.cnt + rg, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = t == S - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __hip_atomic_store(a.cnt + rg, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    }
    last_flag = last;
  }
  __syncthreads();
  if (!last_flag) return false;
  const size_t sstride = (size_t)ntile * MP * ROWS;
  const float* base = a.ws + (size_t)rg * MP * ROWS;
  for (int u = tid; u < MP * ROWS / 4; u += NT) {
    const int m = u / (ROWS / 4), n4 = 4 * (u % (ROWS / 4));
    // SK_SB slices' loads in flight at once (clamped re-reads weighted by zero), in fixed order
    gf32x4 v = gf32x4{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < S; k0 += SK_SB) {
      gf32x4 part[SK_SB];
#pragma unroll
      for (int k = 0; k < SK_SB; ++k)
        part[k] = *(const gf32x4*)(base + min(k0 + k, S - 1) * sstride + (size_t)m * ROWS + n4);
#pragma unroll
      for (int k = 0; k < SK_SB; ++k)
        if (k0 + k < S) v += part[k];
    }
    float s = finish(m, n0 + n4, v);
    if constexpr (EPI == GEPI_ACCUM_NORM) {
      // a row's ROWS / 4 units sit on consecutive lanes of one wave
#pragma unroll
      for (int o = 1; o < ROWS / 4; o <<= 1) s += __shfl_xor(s, o, 64);
      if (n4 == 0 && m < a.M) a.nrm_part[(size_t)m * a.nrm_parts + rg] = s;
    }
  }
  return true;
}

}  // namespace aios
