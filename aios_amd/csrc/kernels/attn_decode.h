// Split-K flash-decode attention core (device code of attention.hip's decode kernel).  See
// attention.hip for the design.
#pragma once
#include "../common.h"
#include "../ops.h"
#include "gemm_common.h"

#include <algorithm>
#include <cstdlib>

#ifndef AIOS_ATTN_PROBES
#define AIOS_ATTN_PROBES 0
#endif

namespace aios {

__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
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
// op(v[lane], v[lane ^ OFF]) for OFF = 8, 16, 32 without the LDS crossbar: DPP row rotate for 8;
// for 16 / 32 the gfx950 v_permlane16/32_swap of v with itself returns the lower and the upper
// row of every pair in r[0] / r[1] on all lanes, so op(r[0], r[1]) needs no lane select
template <int OFF, typename Op>
__device__ __forceinline__ float xlane_op(float v, Op op) {
  if constexpr (OFF == 8) {
    return op(v, dpp<0x128>(v));  // row_ror:8 within 16 lanes = lane ^ 8
  } else if constexpr (OFF == 16) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return op(__uint_as_float(r[0]), __uint_as_float(r[1]));
  } else {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return op(__uint_as_float(r[0]), __uint_as_float(r[1]));
  }
}
struct OpMax { __device__ float operator()(float a, float b) const { return fmaxf(a, b); } };
struct OpAdd { __device__ float operator()(float a, float b) const { return a + b; } };
// max / sum over the lanes that share (lane % LPK), i.e. across the 64/LPK key groups of a wave
template <int LPK>
__device__ __forceinline__ float keys_max(float v) {
  if constexpr (LPK <= 8) v = xlane_op<8>(v, OpMax{});
  if constexpr (LPK <= 16) v = xlane_op<16>(v, OpMax{});
  return xlane_op<32>(v, OpMax{});
}
template <int LPK>
__device__ __forceinline__ float keys_sum(float v) {
  if constexpr (LPK <= 8) v = xlane_op<8>(v, OpAdd{});
  if constexpr (LPK <= 16) v = xlane_op<16>(v, OpAdd{});
  return xlane_op<32>(v, OpAdd{});
}

constexpr float kLog2e = 1.4426950408889634f;
// masked-key score / empty-state max: finite, so exp2(kNeg - m) underflows to 0 and
// exp2(kNeg - kNeg) = 1 without -inf compares on the hot path
constexpr float kNeg = -1e30f;
// raw v_exp_f32 (denormal results flush to 0, which is all a softmax weight needs); ocml's exp2f
// adds a range-scaling compare + 2 selects per call
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

__device__ __forceinline__ uint4 ld_nt16(const bf16_t* p) {
  const gu32x4 v = __builtin_nontemporal_load((const gu32x4*)p);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

__device__ __forceinline__ float dot2_bf16(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(gbf16x2, a), __builtin_bit_cast(gbf16x2, b), c, false);
}

typedef unsigned int gu32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint2 ld_nt8(const uint8_t* p) {
  const gu32x2 v = __builtin_nontemporal_load((const gu32x2*)p);
  return make_uint2(v[0], v[1]);
}
// fp8 KV (OCP e4m3): 2 codes (bytes 2*hi, 2*hi+1 of w) -> a bf16 pair (one v_cvt_scalef32_pk_bf16_fp8)
template <bool HI>
__device__ __forceinline__ uint32_t fp8x2_bf16x2(uint32_t w) {
  return __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w, 1.f, HI));
}
// ... -> an fp32 pair (v_cvt_pk_f32_fp8)
template <bool HI>
__device__ __forceinline__ gf32x2 fp8x2_f32x2(uint32_t w) {
  return __builtin_amdgcn_cvt_pk_f32_fp8((int)w, HI);
}

// One workgroup's share: heads [h0, h0 + G) of KV head kvh, keys of the passes sp, sp + P, ...
// (P active workgroups per (row, head set); counters indexed by `ci`).  `ppw` = passes per
// workgroup the split aims for (1: more workgroups, each one 128-key pass; 2: both buffers).
//
// VALU diet (the kernel is VALU-bound per CU once its loads are in flight): q . k runs on
// v_dot2_f32_bf16 against q pre-rounded to bf16 pairs (4 instructions per 8 dims and head, as the
// MFMA prefill path rounds q), P . V on packed v_pk_fma_f32 with the probabilities in fp32.
// F8: the pool holds fp8 e4m3 codes (EngineConfig::kv_fp8): K converted to bf16 pairs for the same
// v_dot2 (the layer's K scale folded into q), V to fp32 pairs for the P.V FMAs (its V scale applied to
// the output).  At head_dim 128 a lane takes 16 dims (16 bytes: the bf16 path's load width -- with 8
// dims per lane the fp8 kernel issued as many load instructions for half the bytes and measured only
// 3 % faster than bf16 at 32k keys, latency- not byte-bound); head_dim 64 keeps 8 dims (8 bytes).
#ifndef AIOS_ATTN_RESCALE_SKIP
#define AIOS_ATTN_RESCALE_SKIP 1
#endif
template <int HD, int G, bool F8 = false>
__device__ __forceinline__ void attn_core(const AttnDecodeArgs& a, int sp, int kvh, int h0, int ci, int P_max,
                                          int ppw, bool nt = false) {
  constexpr int DPL = (F8 && HD == 128) ? 16 : 8;  // dims per lane
  using KVT = typename std::conditional<F8 && DPL == 8, uint2, uint4>::type;
  constexpr int ES = F8 ? 1 : 2;  // bytes per cached element
  constexpr int NP = DPL / 2;     // bf16 / fp32 pairs per lane
  constexpr int NW = 8;                // waves per workgroup
  constexpr int LPK = HD / DPL;        // lanes per key
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
  // probe stamps (a.ts, null in production: one scalar compare per site): 0 entry, 1 seq_len known,
  // 2 first pass computed (its K/V landed), 3 waves merged, 4 partial published + ticket, 5 (m, l)
  // weights ready (last arriver), 6 done
  // (probe builds only, -DAIOS_ATTN_PROBES=1 / AIOS_BUILD_PROBES=1: a branch per stamp site in the
  // pass loop costs production launches, as the GEMVs' probe branches did)
  auto stamp = [&](int k) __attribute__((always_inline)) {
    if (AIOS_ATTN_PROBES && a.ts && threadIdx.x == 0)
      a.ts[((size_t)blockIdx.z * gridDim.x + blockIdx.x) * 8 + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  static_assert(CH == KV_BLOCK, "one decode pass = one paged KV block");
  const int slot = a.slot ? a.slot[b] : b;
  // paged KV: pass c reads physical block bt[c]; a row-indexed table (bt_rows) is looked up
  // without waiting for slot[b], so its load overlaps the seq_len / slot loads
  const int maxb = a.max_ctx / KV_BLOCK;
  const int* btr = a.block_table ? a.block_table + (size_t)(a.bt_rows ? b : slot) * maxb : nullptr;
  const size_t blk_stride = (size_t)a.n_kv_heads * KV_BLOCK * HD;
  const int koff = wave * KPW + ksub;  // this lane's key within a pass (+ s * KPS)
  const uint8_t* kc = (const uint8_t*)a.k_cache + ((size_t)kvh * KV_BLOCK * HD + (size_t)koff * HD + dsl * DPL) * ES;
  const uint8_t* vc = (const uint8_t*)a.v_cache + ((size_t)kvh * KV_BLOCK * HD + (size_t)koff * HD + dsl * DPL) * ES;
  const int cmax = maxb - 1;           // last chunk with valid memory

  const int len = a.seq_len[b];
  const int nchunk = (len + CH - 1) / CH;
  const int P = max(1, min((nchunk + ppw - 1) / ppw, P_max));
  if (sp >= P) return;  // uniform: this workgroup has no chunk, issues no K/V traffic
  stamp(1);

  // two passes in flight per workgroup: buffers A and B (static, so they stay in VGPRs)
  KVT kA[STEPS], vA[STEPS], kB[STEPS], vB[STEPS];
  const bool tail = a.kv_tail != 0;
  auto ld = [&](const uint8_t* p) __attribute__((always_inline)) { return *(const KVT*)p; };
  auto ld_nt = [&](const uint8_t* p) __attribute__((always_inline)) {
    if constexpr (F8 && DPL == 8) return ld_nt8(p);
    else return ld_nt16((const bf16_t*)p);
  };
  auto issue = [&](KVT (&kr)[STEPS], KVT (&vr)[STEPS], int chunk) __attribute__((always_inline)) {
    const int c = min(chunk, cmax);  // clamped: always a mapped block
    const size_t base = (size_t)(btr ? btr[c] : slot * maxb + c) * blk_stride * ES;  // (bytes)
    if (tail && (chunk + 1) * CH > len) {
      // the context's last, partly filled block: only the lanes of live keys load (a 153-key context
      // fetched 2 x 64 KB for 25 keys of its second block); dead keys hold zeros (scores masked, V x 0)
      const int k0 = chunk * CH + koff;
#pragma unroll
      for (int s = 0; s < STEPS; ++s) {
        kr[s] = KVT{};
        vr[s] = KVT{};
        if (k0 + s * KPS < len) {
          kr[s] = ld(kc + base + (size_t)s * KPS * HD * ES);
          vr[s] = ld(vc + base + (size_t)s * KPS * HD * ES);
        }
      }
    } else if (nt) {  // streaming (nt) policy: K/V lines read once per launch (long mode)
#pragma unroll
      for (int s = 0; s < STEPS; ++s) kr[s] = ld_nt(kc + base + (size_t)s * KPS * HD * ES);
#pragma unroll
      for (int s = 0; s < STEPS; ++s) vr[s] = ld_nt(vc + base + (size_t)s * KPS * HD * ES);
    } else {
#pragma unroll
      for (int s = 0; s < STEPS; ++s) kr[s] = ld(kc + base + (size_t)s * KPS * HD * ES);
#pragma unroll
      for (int s = 0; s < STEPS; ++s) vr[s] = ld(vc + base + (size_t)s * KPS * HD * ES);
    }
  };
  issue(kA, vA, sp);
  if (sp + P < nchunk) issue(kB, vB, sp + P);
  const float qs = a.scale * kLog2e * (F8 ? a.kv_scale_k : 1.f);  // scores in the log2 domain: exp2 below
  const float vs = F8 ? a.kv_scale_v : 1.f;                         // (fp8: V's scale, on the output)
  uint32_t q2[G][NP];                 // q * scale as bf16 pairs
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float* qp = a.q + ((size_t)b * a.n_heads + h0 + g) * HD + dsl * DPL;
#pragma unroll
    for (int j = 0; j < DPL / 4; ++j) {
      const float4 q0 = *(const float4*)(qp + 4 * j);
      q2[g][2 * j] = pk_bf16(q0.x * qs, q0.y * qs);
      q2[g][2 * j + 1] = pk_bf16(q0.z * qs, q0.w * qs);
    }
  }
  float m[G], l[G];
  gf32x2 o[G][NP];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = kNeg;
    l[g] = 0.f;
#pragma unroll
    for (int i = 0; i < NP; ++i) o[g][i] = gf32x2{0.f, 0.f};
  }
  auto pass = [&](const KVT (&kr)[STEPS], const KVT (&vr)[STEPS], int c) __attribute__((always_inline)) {
    // ---- scores of this lane's STEPS keys for the G heads (reduced over the key's LPK lanes)
    float sc[STEPS][G];
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      const bool valid = c * CH + koff + s * KPS < len;
      uint32_t kb[NP];
      if constexpr (F8 && DPL == 16) {
        const uint32_t w4[4] = {kr[s].x, kr[s].y, kr[s].z, kr[s].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) { kb[2 * i] = fp8x2_bf16x2<false>(w4[i]); kb[2 * i + 1] = fp8x2_bf16x2<true>(w4[i]); }
      } else if constexpr (F8) {
        kb[0] = fp8x2_bf16x2<false>(kr[s].x); kb[1] = fp8x2_bf16x2<true>(kr[s].x);
        kb[2] = fp8x2_bf16x2<false>(kr[s].y); kb[3] = fp8x2_bf16x2<true>(kr[s].y);
      } else {
        kb[0] = kr[s].x; kb[1] = kr[s].y; kb[2] = kr[s].z; kb[3] = kr[s].w;
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float d = dot2_bf16(kb[0], q2[g][0], 0.f);
#pragma unroll
        for (int i = 1; i < NP; ++i) d = dot2_bf16(kb[i], q2[g][i], d);
        d = group_sum<LPK>(d);
        sc[s][g] = valid ? d : kNeg;
      }
    }
    // ---- online softmax over this lane's keys (round 6: per key group -- the LPK lanes of a key share
    // its score, so (m, l) are uniform over them; the cross-key-group max / sum, two 3-stage lane
    // reductions per head and pass, move to the end of the pass loop: the fp8 long mode's passes are
    // bound by their own VALU chain, profiles/long_context_r6.txt)
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float mx = sc[0][g];
#pragma unroll
      for (int s = 1; s < STEPS; ++s) mx = fmaxf(mx, sc[s][g]);
      const float mn = fmaxf(m[g], mx);
      float ps = 0.f;
#pragma unroll
      for (int s = 0; s < STEPS; ++s) {
        const float p = fast_exp2(sc[s][g] - mn);
        sc[s][g] = p;
        ps += p;
      }
      // rescale only when some lane's max grew (a wave-uniform branch: past the first passes of a long
      // context the running max rarely moves, and the NP packed multiplies + exp2 per head were per pass)
      if (AIOS_ATTN_RESCALE_SKIP == 0 || __builtin_amdgcn_ballot_w64(mn > m[g])) {
        const float alpha = fast_exp2(m[g] - mn);
        l[g] *= alpha;
#pragma unroll
        for (int i = 0; i < NP; ++i) o[g][i] *= alpha;
      }
      l[g] += ps;
      m[g] = mn;
    }
    // ---- P.V (lane-local over its keys; merged across key groups and waves at the end)
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      gf32x2 vf[NP];
      if constexpr (F8 && DPL == 16) {
        const uint32_t w4[4] = {vr[s].x, vr[s].y, vr[s].z, vr[s].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) { vf[2 * i] = fp8x2_f32x2<false>(w4[i]); vf[2 * i + 1] = fp8x2_f32x2<true>(w4[i]); }
      } else if constexpr (F8) {
        vf[0] = fp8x2_f32x2<false>(vr[s].x); vf[1] = fp8x2_f32x2<true>(vr[s].x);
        vf[2] = fp8x2_f32x2<false>(vr[s].y); vf[3] = fp8x2_f32x2<true>(vr[s].y);
      } else {
        const uint32_t w[4] = {vr[s].x, vr[s].y, vr[s].z, vr[s].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) vf[i] = gf32x2{__uint_as_float(w[i] << 16), __uint_as_float(w[i] & 0xffff0000u)};
      }
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const gf32x2 pp = gf32x2{sc[s][g], sc[s][g]};
#pragma unroll
        for (int i = 0; i < NP; ++i) o[g][i] = __builtin_elementwise_fma(pp, vf[i], o[g][i]);
      }
    }
  };
  for (int c = sp; c < nchunk; c += 2 * P) {
    pass(kA, vA, c);
    if (c == sp) stamp(2);
    if (c + 2 * P < nchunk) issue(kA, vA, c + 2 * P);
    if (c + P < nchunk) {
      pass(kB, vB, c + P);
      if (c + 3 * P < nchunk) issue(kB, vB, c + 3 * P);
    }
  }
  // ---- merge the key groups of a wave (shuffles: their (m, l, o) rescaled to the wave's max), then the 8
  // waves in LDS (one barrier)
  float of[G][DPL];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float M = keys_max<LPK>(m[g]);
    const float w = fast_exp2(m[g] - M);
    l[g] = keys_sum<LPK>(l[g] * w);
    m[g] = M;
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      of[g][2 * i] = keys_sum<LPK>(o[g][i].x * w);
      of[g][2 * i + 1] = keys_sum<LPK>(o[g][i].y * w);
    }
  }
  if (ksub == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float4* dst = (float4*)&s_o[wave][g][dsl * DPL];
#pragma unroll
      for (int j = 0; j < DPL / 4; ++j) dst[j] = make_float4(of[g][4 * j], of[g][4 * j + 1], of[g][4 * j + 2], of[g][4 * j + 3]);
    }
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
  stamp(3);
  const int nact = P;  // workgroups that arrive
  for (int idx = threadIdx.x; idx < G * HD; idx += NT) {
    const int g = idx / HD, d = idx - g * HD;
    float M = s_m[0][g];
#pragma unroll
    for (int w = 1; w < NW; ++w) M = fmaxf(M, s_m[w][g]);
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const float sw = fast_exp2(s_m[w][g] - M);
      L += sw * s_l[w][g];
      acc += sw * s_o[w][g][d];
    }
    const int h = h0 + g;
    if (F8) acc *= vs;
    if (nact == 1) {
      if (a.out16) a.out16[((size_t)b * a.n_heads + h) * HD + d] = f32_to_bf16(acc / L);
      else if (a.out_wt) st_wt(a.out + ((size_t)b * a.n_heads + h) * HD + d, acc / L);
      else a.out[((size_t)b * a.n_heads + h) * HD + d] = acc / L;
    } else {
      st_wt(a.o_part + (((size_t)b * a.n_heads + h) * a.n_chunks + sp) * HD + d, acc);
      if (d == 0) {
        float* ml = a.ml + (((size_t)b * a.n_heads + h) * a.n_chunks + sp) * 2;
        st_wt(ml, M);
        st_wt(ml + 1, L);
      }
    }
  }
  if (nact == 1) {
    stamp(6);
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  int* cnt = a.counters + (size_t)b * a.n_heads + ci;
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == nact - 1);
  }
  __syncthreads();
  stamp(4);
  if (!s_last) return;
  // ---- last arriver.  (1) one thread per (head, partial) loads that partial's (m, l);
  //      (measured: one batch of (m, l) + o loads per output thread -- one round trip but 2x the
  //      loads, the (m, l) ones redundant across a head's 128 threads -- was 1.3 us SLOWER at 1000
  //      keys, 10.09 vs 8.73 us; hoisting the block-table loads above the seq_len test, or
  //      issuing pass 0's K/V before seq_len is read, did not help either: 4.32-4.40 vs 4.18 us
  //      at 153 keys, tools/attn_probe.py -- the short-context launch is the 1.7 us launch chain
  //      plus one K/V round trip plus the merge, not the table lookups)
  //      (2) wave g reduces head g's max M and total L and turns them into normalised weights
  //      w_p = exp2(m_p - M) / L in LDS; (3) every output sums w_p * o_p with 16 loads in flight.
  //      Two memory round trips for up to 64 partials (was one per 8 partials).
  __shared__ float s_pm[G][64], s_pl[G][64];
  // one memory round trip (round 4): when every output has one thread and the partials fit one
  // register batch, each thread issues its output's nact partial loads TOGETHER with the (m, l)
  // sweep and folds them after the weights are ready -- same order of sums as the two-trip path
  auto one_trip = [&](auto ob) __attribute__((always_inline)) {
    constexpr int OB = decltype(ob)::value;
    const int idx = threadIdx.x;
    const bool act = idx < G * HD;
    const int g = act ? idx / HD : 0, d = act ? idx - g * HD : 0;
    const float* op = a.o_part + ((size_t)b * a.n_heads + h0 + g) * a.n_chunks * HD + d;
    float ov[OB];
#pragma unroll
    for (int j = 0; j < OB; ++j) ov[j] = ld_wt(op + (size_t)min(j, nact - 1) * HD);  // clamped: in bounds
    for (int i = threadIdx.x; i < G * nact; i += NT) {
      const int gg = i / nact, p = i - gg * nact;
      const float* mlp = a.ml + (((size_t)b * a.n_heads + h0 + gg) * a.n_chunks + p) * 2;
      s_pm[gg][p] = ld_wt(mlp);
      s_pl[gg][p] = ld_wt(mlp + 1);
    }
    __syncthreads();
    if (wave < G) {
      const float mv = lane < nact ? s_pm[wave][lane] : kNeg;
      const float lv = lane < nact ? s_pl[wave][lane] : 0.f;
      float M = mv;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) M = fmaxf(M, __shfl_xor(M, o));
      const float e = fast_exp2(mv - M);
      float L = e * lv;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) L += __shfl_xor(L, o);
      if (lane < nact) s_pm[wave][lane] = e / L;
    }
    __syncthreads();
    stamp(5);
    if (act) {
      float acc = 0.f;
#pragma unroll
      for (int j = 0; j < OB; ++j)
        if (j < nact) acc = fmaf(s_pm[g][j], ov[j], acc);
      const int h = h0 + g;
      if (a.out16) a.out16[((size_t)b * a.n_heads + h) * HD + d] = f32_to_bf16(acc);
      else if (a.out_wt) st_wt(a.out + ((size_t)b * a.n_heads + h) * HD + d, acc);
      else a.out[((size_t)b * a.n_heads + h) * HD + d] = acc;
    }
  };
  if (G * HD <= NT && nact <= 32 && a.combine_trips != 2) {
    if (nact <= 8) one_trip(std::integral_constant<int, 8>{});
    else if (nact <= 16) one_trip(std::integral_constant<int, 16>{});
    else one_trip(std::integral_constant<int, 32>{});
    if (threadIdx.x == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
    stamp(6);
    return;
  }
  for (int i = threadIdx.x; i < G * nact; i += NT) {
    const int g = i / nact, p = i - g * nact;
    const float* mlp = a.ml + (((size_t)b * a.n_heads + h0 + g) * a.n_chunks + p) * 2;
    s_pm[g][p] = ld_wt(mlp);
    s_pl[g][p] = ld_wt(mlp + 1);
  }
  __syncthreads();
  if (wave < G) {
    const int g = wave;
    const float mv = lane < nact ? s_pm[g][lane] : kNeg;
    const float lv = lane < nact ? s_pl[g][lane] : 0.f;
    float M = mv;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) M = fmaxf(M, __shfl_xor(M, o));
    const float e = fast_exp2(mv - M);
    float L = e * lv;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) L += __shfl_xor(L, o);
    if (lane < nact) s_pm[g][lane] = e / L;
  }
  __syncthreads();
  stamp(5);
  for (int idx = threadIdx.x; idx < G * HD; idx += NT) {
    const int g = idx / HD, d = idx - g * HD;
    const int h = h0 + g;
    const float* op = a.o_part + ((size_t)b * a.n_heads + h) * a.n_chunks * HD + d;
    float acc = 0.f;
    for (int c = 0; c < nact; c += 16) {
      float ov[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) ov[j] = ld_wt(op + (size_t)min(c + j, nact - 1) * HD);
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if (c + j < nact) acc = fmaf(s_pm[g][c + j], ov[j], acc);
    }
    if (a.out16) a.out16[((size_t)b * a.n_heads + h) * HD + d] = f32_to_bf16(acc);
    else if (a.out_wt) st_wt(a.out + ((size_t)b * a.n_heads + h) * HD + d, acc);
      else a.out[((size_t)b * a.n_heads + h) * HD + d] = acc;
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  stamp(6);
}

// Up to ATTN_SPLIT_LEN keys the G query heads of a KV head are split over G workgroups (one head
// each; the K/V re-reads hit L2): 4x less dot / softmax / P.V work per workgroup on the latency-
// bound short contexts of agent turns.  Beyond that one workgroup set per (KV head, head set of
// GL <= 4 query heads) computes its heads (the KV stream, not the arithmetic, dominates; GL = 4
// keeps G = 8 groups in registers).  The grid is flat (one x-slot per role of the larger mode)
// and each workgroup derives its role from seq_len, so a hipGraph-captured launch sized for
// max_ctx carries no idle head-split grid (round-2 probe: 384 idle 512-thread workgroups cost
// 4 us at a 256-key context).
constexpr int ATTN_SPLIT_LEN = 512;
template <int G>
struct AttnGL { static constexpr int value = (G % 4 == 0) ? 4 : G; };

struct AttnSplit {
  int p_long;   // workgroups per (row, head set) in the long mode
  int p_short;  // workgroups per (row, head) in the short mode
  int ppw;      // passes per workgroup the split aims for
  int n_attn;   // attention workgroups of the flat grid
  int xcd;      // short mode: the G query heads of a KV head on one XCD (attention.hip)
};


// workgroup wg's role in the flat grid (see attn_decode_kernel, attention.hip); returns with the
// whole workgroup (every early exit inside is workgroup-uniform)
template <int HD, int G, bool F8 = false>
__device__ __forceinline__ void attn_role(const AttnDecodeArgs& a, const AttnSplit& sp_, int wg) {
  const int len = a.seq_len[blockIdx.z];
  if (G > 1 && len <= a.short_len) {
    // XCD-aware roles: workgroups are dealt round-robin over the 8 XCDs (blockIdx % 8), so
    // workgroup wg takes query head (wg % 8) * (H / 8) + (wg / 8) / P -- the G query heads of a KV
    // head then run on one XCD and read its K/V from that XCD's L2 after the first miss (the plain
    // mapping put them on G different XCDs: G MALL/HBM reads of every K/V line)
    int h, sp;
    if ((a.n_heads & 7) == 0 && sp_.xcd) {
      if (wg >= a.n_heads * sp_.p_short) return;
      const int j = wg >> 3;
      h = (wg & 7) * (a.n_heads >> 3) + j / sp_.p_short;
      sp = j % sp_.p_short;
    } else {
      h = wg / sp_.p_short;
      sp = wg % sp_.p_short;
    }
    if (h >= a.n_heads) return;
    attn_core<HD, 1, F8>(a, sp, h / G, h, h, sp_.p_short, sp_.ppw);
  } else {
    constexpr int GL = AttnGL<G>::value;
    const int hsi = wg / sp_.p_long, sp = wg % sp_.p_long;
    if (hsi >= a.n_kv_heads * (G / GL)) return;
    const int kvh = hsi / (G / GL), h0 = kvh * G + (hsi % (G / GL)) * GL;
    // long mode: every K/V line is read by exactly one workgroup -> streaming loads (round 4,
    // same box: --prompt 4000 546.9 -> 567.0 tok/s, 16000 467.6 -> 487.3)
    attn_core<HD, GL, F8>(a, sp, kvh, h0, h0, sp_.p_long, sp_.ppw, a.kv_nt != 0);
  }
}

inline int attn_env_int(const char* k, int dflt) {
  const char* e = std::getenv(k);
  return e ? std::atoi(e) : dflt;
}

int attn_decode_split(int max_ctx, int B, int n_kv_heads);
// the launcher's defaults filled in (split, combine, K/V load policy, short-mode length)
inline AttnDecodeArgs attn_resolve(const AttnDecodeArgs& a) {
  AttnDecodeArgs b = a;
  if (b.split <= 0) b.split = attn_decode_split(a.max_ctx, a.B, a.n_kv_heads);
  if (b.combine_trips == 0) b.combine_trips = attn_env_int("AIOS_ATTN_COMBINE", 1);
  if (b.kv_nt < 0) b.kv_nt = attn_env_int("AIOS_ATTN_NT", 1);
  if (b.kv_tail < 0) b.kv_tail = attn_env_int("AIOS_ATTN_TAIL", 1);
  // Batched decode fills the chip with (row, KV head) workgroups on its own: from
  // AIOS_ATTN_GROUPED_MIN such workgroups up, every context length takes the grouped mode (one
  // K/V read for the G query heads of a KV head) instead of the per-query-head split that buys
  // batch-1 latency with G x the K/V reads and workgroups
  if (b.short_len < 0) {
    const int grouped_min = attn_env_int("AIOS_ATTN_GROUPED_MIN", 128);
    b.short_len = (grouped_min > 0 && a.B * a.n_kv_heads >= grouped_min) ? 0 : ATTN_SPLIT_LEN;
  }
  return b;
}

// the launch shape for AttnDecodeArgs a (split already resolved): fills the split and returns the
// flat workgroup count (one x-slot per role of the larger mode)
inline int attn_plan(const AttnDecodeArgs& a, int G, AttnSplit& sp) {
  const int nch = std::max(1, a.max_ctx / 128);  // 128-key passes
  sp.p_long = std::max(1, std::min(nch, a.split / ATTN_CHUNK));
  // short mode: one workgroup per query head walks all (<= 4) passes -- the probe's best at
  // <= 256 keys (a combine costs more than the second pass it would spread)
  sp.p_short = std::max(1, std::min(4, attn_env_int("AIOS_ATTN_SHORT_P", 1)));
  sp.ppw = std::max(1, std::min(2, attn_env_int("AIOS_ATTN_PPW", 1)));
  if (sp.p_long > a.n_chunks || sp.p_long > 64 || sp.p_short > a.n_chunks)
    throw std::runtime_error("attn_decode: more splits than partial buffers / 64");
  const int GL = (G % 4 == 0) ? 4 : G;
  sp.n_attn = std::max(a.n_kv_heads * (G / GL) * sp.p_long, G > 1 && a.short_len != 0 ? a.n_heads * sp.p_short : 0);
  return std::max(a.n_kv_heads * (G / GL) * sp.p_long, G > 1 && a.short_len != 0 ? a.n_heads * sp.p_short : 0);
}
}  // namespace aios
