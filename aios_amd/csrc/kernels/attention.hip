// Split-K flash-decode GQA attention over the bf16 KV cache (decode shape),
// with the log-sum-exp combine fused in (last-arriving workgroup per (row, kv-head)).
//
// grid = (roles, 1, B), 512 threads (8 waves); every workgroup picks its role from seq_len (see
// attn_decode_kernel).  The context is cut into 128-key passes (16 keys per wave); every
// workgroup owns two passes at a time with ALL of their K and V loads issued up front (buffers A
// and B), so up to 256 keys cost one memory round trip: P = ceil(passes / 2) workgroups per
// (row, head set), capped by the grid (workgroups then loop, the next pass's loads issued while
// the current one is scored).  At a 153-key context this is one workgroup per query head with
// no combine; at 4k keys up to 32 workgroups per KV head.  (Round 1 walked up to three 64-key
// passes serially in one 4-wave workgroup: 7.8 us per layer at 153 keys.)
//
// Inside a pass every lane loads 16 B = 8 dims of a key (LPK = hd/8 lanes per key).  Each WAVE
// keeps its own online-softmax state (m, l, o) for the G = H/Hkv query heads of the group --
// scores are reduced over the LPK lanes of a key with DPP (no LDS), and no workgroup barrier is
// needed until the eight waves merge their states in LDS at the end.
//
// Combine: with more than one active workgroup each writes its partial (o, m, l) with
// write-through (sc1, agent scope) stores, drains them (s_waitcnt vmcnt(0)), and after a
// workgroup barrier one lane takes an agent-scope ticket for (row, kv head).  The last arriver
// reads every partial's (m, l) in one parallel sweep (one lane per partial), then each thread
// sums its outputs over the partials with independent loads -- the write-through hand-off of
// CDNA guide §6 Guideline 16 / split-K item 2 -- and re-arms the counter.
#include "../common.h"
#include "../ops.h"

namespace aios {

__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void bf16x8_to_f32(const uint4& v, float f[8]) {
  f[0] = bf16_to_f32(v.x & 0xffff); f[1] = bf16_to_f32(v.x >> 16);
  f[2] = bf16_to_f32(v.y & 0xffff); f[3] = bf16_to_f32(v.y >> 16);
  f[4] = bf16_to_f32(v.z & 0xffff); f[5] = bf16_to_f32(v.z >> 16);
  f[6] = bf16_to_f32(v.w & 0xffff); f[7] = bf16_to_f32(v.w >> 16);
}

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
// sum over aligned groups of N lanes (N = 8 or 16), result in every lane of the group
template <int N>
__device__ __forceinline__ float group_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror: lane i <-> 7-i within 8
  if constexpr (N == 16) v += dpp<0x140>(v);  // row_mirror: lane i <-> 15-i within 16
  return v;
}
// value of lane ^ OFF (OFF = 8, 16, 32) without the LDS crossbar: DPP row rotate for 8, the
// gfx950 v_permlane16/32_swap VALU exchanges for 16 / 32
template <int OFF>
__device__ __forceinline__ float xlane(float v) {
  const int lane = threadIdx.x & 63;
  if constexpr (OFF == 8) {
    return dpp<0x128>(v);  // row_ror:8 within 16 lanes = lane ^ 8
  } else if constexpr (OFF == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float((lane & 16) ? r[0] : r[1]);
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float((lane & 32) ? r[0] : r[1]);
  }
}
// max / sum over the lanes that share (lane % LPK), i.e. across the 64/LPK key groups of a wave
template <int LPK>
__device__ __forceinline__ float keys_max(float v) {
  if constexpr (LPK <= 8) v = fmaxf(v, xlane<8>(v));
  if constexpr (LPK <= 16) v = fmaxf(v, xlane<16>(v));
  return fmaxf(v, xlane<32>(v));
}
template <int LPK>
__device__ __forceinline__ float keys_sum(float v) {
  if constexpr (LPK <= 8) v += xlane<8>(v);
  if constexpr (LPK <= 16) v += xlane<16>(v);
  return v + xlane<32>(v);
}

constexpr float kLog2e = 1.4426950408889634f;

// One workgroup's share: heads [h0, h0 + G) of KV head kvh, keys of the passes sp, sp + P, ...
// (P active workgroups per (row, head set); counters indexed by `ci`).
template <int HD, int G>
__device__ __forceinline__ void attn_core(const AttnDecodeArgs& a, int sp, int kvh, int h0, int ci, int P_max) {
  constexpr int NW = 8;                // waves per workgroup
  constexpr int LPK = HD / 8;          // lanes per key (8 dims per lane)
  constexpr int KPS = 64 / LPK;        // keys per wave-instruction
  constexpr int CH = 128;              // keys per workgroup pass
  constexpr int KPW = CH / NW;         // keys per wave per pass
  constexpr int STEPS = KPW / KPS;     // loads per lane per pass (each of K and V)
  constexpr int NT = NW * 64;
  __shared__ float s_o[NW][G][HD];
  __shared__ float s_m[NW][G], s_l[NW][G];
  __shared__ int s_last;

  const int b = blockIdx.z;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ksub = lane / LPK, dsl = lane % LPK;
  const int slot = a.slot ? a.slot[b] : b;
  const size_t kv_base = (((size_t)slot * a.n_kv_heads + kvh) * a.max_ctx) * HD;
  const bf16_t* kc = a.k_cache + kv_base + dsl * 8;
  const bf16_t* vc = a.v_cache + kv_base + dsl * 8;
  const int koff = wave * KPW + ksub;  // this lane's key within a pass (+ s * KPS)
  const int cmax = a.max_ctx / CH - 1; // last chunk with valid memory

  // two passes in flight per workgroup: buffers A and B (static, so they stay in VGPRs)
  uint4 kA[STEPS], vA[STEPS], kB[STEPS], vB[STEPS];
  auto issue = [&](uint4 (&kr)[STEPS], uint4 (&vr)[STEPS], int chunk) __attribute__((always_inline)) {
    const int k0 = min(chunk, cmax) * CH + koff;  // clamped: always valid memory
#pragma unroll
    for (int s = 0; s < STEPS; ++s) kr[s] = *(const uint4*)(kc + (size_t)(k0 + s * KPS) * HD);
#pragma unroll
    for (int s = 0; s < STEPS; ++s) vr[s] = *(const uint4*)(vc + (size_t)(k0 + s * KPS) * HD);
  };
  const int len = a.seq_len[b];
  const int nchunk = (len + CH - 1) / CH;
  // active workgroups: two passes per workgroup, all of their loads in flight at once (one
  // memory round trip for up to 256 keys); beyond 2 x gridDim.x chunks workgroups loop
  const int P = max(1, min((nchunk + 1) / 2, P_max));
  if (sp >= P) return;  // uniform: this workgroup has no chunk, issues no K/V traffic
  issue(kA, vA, sp);
  if (sp + P < nchunk) issue(kB, vB, sp + P);
  const float qs = a.scale * kLog2e;  // scores in the log2 domain: exp2 below
  float q[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float* qp = a.q + ((size_t)b * a.n_heads + h0 + g) * HD + dsl * 8;
    const float4 q0 = *(const float4*)qp, q1 = *(const float4*)(qp + 4);
    q[g][0] = q0.x * qs; q[g][1] = q0.y * qs; q[g][2] = q0.z * qs; q[g][3] = q0.w * qs;
    q[g][4] = q1.x * qs; q[g][5] = q1.y * qs; q[g][6] = q1.z * qs; q[g][7] = q1.w * qs;
  }
  float m[G], l[G], o[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[g][i] = 0.f;
  }
  auto pass = [&](const uint4 (&kr)[STEPS], const uint4 (&vr)[STEPS], int c) __attribute__((always_inline)) {
    // ---- scores of this lane's STEPS keys for the G heads (reduced over the key's LPK lanes)
    float sc[STEPS][G];
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      float kf[8];
      bf16x8_to_f32(kr[s], kf);
      const bool valid = c * CH + koff + s * KPS < len;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) d = fmaf(q[g][i], kf[i], d);
        d = group_sum<LPK>(d);
        sc[s][g] = valid ? d : -INFINITY;
      }
    }
    // ---- per-wave online softmax over this pass's KPW keys
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float mx = sc[0][g];
#pragma unroll
      for (int s = 1; s < STEPS; ++s) mx = fmaxf(mx, sc[s][g]);
      mx = keys_max<LPK>(mx);
      const float mn = fmaxf(m[g], mx);
      const float alpha = (mn == -INFINITY) ? 1.f : exp2f(m[g] - mn);
      float ps = 0.f;
#pragma unroll
      for (int s = 0; s < STEPS; ++s) {
        const float p = (sc[s][g] == -INFINITY) ? 0.f : exp2f(sc[s][g] - mn);
        sc[s][g] = p;
        ps += p;
      }
      l[g] = l[g] * alpha + keys_sum<LPK>(ps);
      m[g] = mn;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[g][i] *= alpha;
    }
    // ---- P.V (lane-local over its keys; merged across key groups and waves at the end)
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      float vf[8];
      bf16x8_to_f32(vr[s], vf);
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 8; ++i) o[g][i] = fmaf(sc[s][g], vf[i], o[g][i]);
    }
  };
  for (int c = sp; c < nchunk; c += 2 * P) {
    pass(kA, vA, c);
    if (c + 2 * P < nchunk) issue(kA, vA, c + 2 * P);
    if (c + P < nchunk) {
      pass(kB, vB, c + P);
      if (c + 3 * P < nchunk) issue(kB, vB, c + 3 * P);
    }
  }
  // ---- merge the key groups of a wave (shuffles), then the 8 waves in LDS (one barrier)
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int i = 0; i < 8; ++i) o[g][i] = keys_sum<LPK>(o[g][i]);
  if (ksub == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int i = 0; i < 8; ++i) s_o[wave][g][dsl * 8 + i] = o[g][i];
  }
  if (lane < G) {
    // m/l are wave-uniform after keys_max/keys_sum; lane g publishes head g
    float mv = m[0], lv = l[0];
#pragma unroll
    for (int g = 1; g < G; ++g)
      if (lane == g) { mv = m[g]; lv = l[g]; }
    s_m[wave][lane] = mv;
    s_l[wave][lane] = lv;
  }
  __syncthreads();
  const int nact = P;  // workgroups that arrive
  for (int idx = threadIdx.x; idx < G * HD; idx += NT) {
    const int g = idx / HD, d = idx - g * HD;
    float M = s_m[0][g];
#pragma unroll
    for (int w = 1; w < NW; ++w) M = fmaxf(M, s_m[w][g]);
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float sw = (s_m[w][g] == -INFINITY) ? 0.f : exp2f(s_m[w][g] - M);
      L += sw * s_l[w][g];
      acc += sw * s_o[w][g][d];
    }
    const int h = h0 + g;
    if (nact == 1) {
      a.out[((size_t)b * a.n_heads + h) * HD + d] = acc / L;
    } else {
      st_wt(a.o_part + (((size_t)b * a.n_heads + h) * a.n_chunks + sp) * HD + d, acc);
      if (d == 0) {
        float* ml = a.ml + (((size_t)b * a.n_heads + h) * a.n_chunks + sp) * 2;
        st_wt(ml, M);
        st_wt(ml + 1, L);
      }
    }
  }
  if (nact == 1) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  int* cnt = a.counters + (size_t)b * a.n_heads + ci;
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == nact - 1);
  }
  __syncthreads();
  if (!s_last) return;
  // ---- last arriver: each output sums its partials; m, l and o of 8 partials are loaded
  //      together (one memory round trip per 8 partials, online rescale across blocks)
  for (int idx = threadIdx.x; idx < G * HD; idx += NT) {
    const int g = idx / HD, d = idx - g * HD;
    const int h = h0 + g;
    const float* mlp = a.ml + ((size_t)b * a.n_heads + h) * a.n_chunks * 2;
    const float* op = a.o_part + ((size_t)b * a.n_heads + h) * a.n_chunks * HD + d;
    float M = -INFINITY, L = 0.f, acc = 0.f;
    for (int c = 0; c < nact; c += 8) {
      float mv[8], lv[8], ov[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int cc = min(c + j, nact - 1);
        mv[j] = ld_wt(mlp + 2 * cc);
        lv[j] = ld_wt(mlp + 2 * cc + 1);
        ov[j] = ld_wt(op + (size_t)cc * HD);
      }
      float mb = M;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (c + j < nact) mb = fmaxf(mb, mv[j]);
      const float al = (M == -INFINITY) ? 0.f : exp2f(M - mb);
      L *= al;
      acc *= al;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (c + j < nact) {
          const float w = exp2f(mv[j] - mb);
          L = fmaf(w, lv[j], L);
          acc = fmaf(w, ov[j], acc);
        }
      }
      M = mb;
    }
    a.out[((size_t)b * a.n_heads + h) * HD + d] = acc / L;
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
}

// Up to ATTN_SPLIT_LEN keys the G query heads of a KV head are split over G workgroups (one head
// each; the K/V re-reads hit L2): 4x less dot / softmax / P.V work per workgroup on the latency-
// bound short contexts of agent turns.  Beyond that one workgroup set per KV head computes all G
// heads (the KV stream, not the arithmetic, dominates).  The grid is flat (one x-slot per role of
// the larger mode) and each workgroup derives its role from seq_len, so a hipGraph-captured launch
// sized for max_ctx carries at most n_heads * ATTN_SHORT_P idle workgroups, never Pmax * n_heads
// (round-2 probe: 384 idle 512-thread workgroups cost 4 us at a 256-key context).
constexpr int ATTN_SPLIT_LEN = 512;
constexpr int ATTN_SHORT_P = 2;  // (512 / 128 + 1) / 2 workgroups per head in the short mode
template <int HD, int G>
__global__ void __launch_bounds__(512) attn_decode_kernel(AttnDecodeArgs a, int p_max) {
  const int wg = blockIdx.x;
  const int len = a.seq_len[blockIdx.z];
  if (G > 1 && len <= ATTN_SPLIT_LEN) {
    const int h = wg / ATTN_SHORT_P, sp = wg % ATTN_SHORT_P;
    if (h >= a.n_heads) return;
    attn_core<HD, 1>(a, sp, h / G, h, h, ATTN_SHORT_P);
  } else {
    const int kvh = wg / p_max, sp = wg % p_max;
    if (kvh >= a.n_kv_heads) return;
    attn_core<HD, G>(a, sp, kvh, kvh * G, kvh * G, p_max);
  }
}

template <int HD>
static void launch_hd(const AttnDecodeArgs& a, int G, hipStream_t st) {
  const int nch = std::max(1, a.max_ctx / 128);  // 128-key passes
  const int P = std::max(1, std::min(nch, a.split / ATTN_CHUNK));  // workgroups per (row, kv head)
  if (P > a.n_chunks || P > 64 || ATTN_SHORT_P > a.n_chunks)
    throw std::runtime_error("attn_decode: more splits than partial buffers / 64");
  const int nwg = std::max(a.n_kv_heads * P, G > 1 ? a.n_heads * ATTN_SHORT_P : 0);
  dim3 grid(nwg, 1, a.B);
  switch (G) {
    case 1: hipLaunchKernelGGL((attn_decode_kernel<HD, 1>), grid, dim3(512), 0, st, a, P); break;
    case 2: hipLaunchKernelGGL((attn_decode_kernel<HD, 2>), grid, dim3(512), 0, st, a, P); break;
    case 4: hipLaunchKernelGGL((attn_decode_kernel<HD, 4>), grid, dim3(512), 0, st, a, P); break;
    case 5: hipLaunchKernelGGL((attn_decode_kernel<HD, 5>), grid, dim3(512), 0, st, a, P); break;
    case 8: hipLaunchKernelGGL((attn_decode_kernel<HD, 8>), grid, dim3(512), 0, st, a, P); break;
    default: throw std::runtime_error("attn_decode: unsupported GQA group size " + std::to_string(G));
  }
}

// `split` (kept in the args for the API) now encodes P * ATTN_CHUNK: the number of workgroups
// per (row, kv head) in the long-context mode.  Target one workgroup per CU for the whole grid
// (a 512-thread workgroup of this kernel fills a CU's register file), 1..64 per head, each
// owning at least one 128-key pass of a max_ctx context.
int attn_decode_split(int max_ctx, int B, int n_kv_heads) {
  const int nch = std::max(1, max_ctx / 128);
  const int P = std::max(1, std::min({64, nch, 256 / std::max(1, B * n_kv_heads)}));
  return P * ATTN_CHUNK;
}

void launch_attn_decode(const AttnDecodeArgs& a, hipStream_t st) {
  if (a.n_heads % a.n_kv_heads) throw std::runtime_error("attn_decode: n_heads % n_kv_heads != 0");
  if (!a.counters) throw std::runtime_error("attn_decode: counters buffer required ([B][n_heads])");
  if (a.max_ctx % 128) throw std::runtime_error("attn_decode: max_ctx must be a multiple of 128");
  const int G = a.n_heads / a.n_kv_heads;
  AttnDecodeArgs b = a;
  if (b.split <= 0) b.split = attn_decode_split(a.max_ctx, a.B, a.n_kv_heads);
  if (b.split % ATTN_CHUNK) throw std::runtime_error("attn_decode: split must be a multiple of ATTN_CHUNK");
  if (a.head_dim == 128) launch_hd<128>(b, G, st);
  else if (a.head_dim == 64) launch_hd<64>(b, G, st);
  else throw std::runtime_error("attn_decode: head_dim must be 64 or 128");
}

}  // namespace aios
