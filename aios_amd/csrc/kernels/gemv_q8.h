// int8-activation GEMV path (included by gemv_impl.h after the shared helpers).
//
// The llama.cpp "q8_1 x" trick, done per workgroup in LDS: x is quantised to int8 per 32-element
// block (dx = amax/127) while it is staged, and every 16-B weight chunk is multiplied with
// v_dot4_i32_i8 (4 MACs per VALU op) directly on the 4-/5-/6-bit codes.  Per 16-run r of a chunk:
//     contrib = sc_r * dx_r * isum_r - of_r * sx_r,    sx_r = dx_r * sum(xq over the run)
// (the K-quant "min" and the Q4_0 / Q6_K code bias fold into of_r).
//
// Block quantisation is scale-invariant, so x*w is quantised un-normalised and 1/rms is applied
// to the finished dot product in the epilogue (y = inv_rms * W (x*w)) -- the RMSNorm statistic
// and the int8 staging come from ONE read of x.
//
// Measured on MI355X (tools/gemv_probe.py): with 256-thread workgroups x 4 per CU the per-WG
// staging cost 1.5-4 us of a 6-20 us GEMV; this version stages once per 512-thread workgroup
// with every thread quantising one octet (DPP quad reductions), streams weights with
// non-temporal loads, and sizes the per-lane chunk count U so a row pair's whole K slice is in
// flight at once.  Q4_K / Q5_K / Q6_K share one chunk order (qweight.h), so a mixed Q4_K_M QKV
// segment list stages x once.
#pragma once
// (included inside namespace aios by gemv_impl.h)

template <int QT>
struct QDot;
template <>
struct QDot<QT_Q4_K> {
  __device__ static void isums(const RawChunk& r, int c, const int (&x)[8], int* is) {
    int s0 = 0, s1 = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t wv = u4_word(r.a, i);
      s0 = __builtin_amdgcn_sdot4((int)(wv & 0x0f0f0f0fu), x[i], s0, false);
      s1 = __builtin_amdgcn_sdot4((int)((wv >> 4) & 0x0f0f0f0fu), x[4 + i], s1, false);
    }
    is[0] = s0;
    is[1] = s1;
  }
};
template <>
struct QDot<QT_Q4_0> {
  __device__ static void isums(const RawChunk& r, int c, const int (&x)[8], int* is) {
    QDot<QT_Q4_K>::isums(r, c, x, is);
  }
};
template <>
struct QDot<QT_Q5_K> {
  __device__ static void isums(const RawChunk& r, int c, const int (&x)[8], int* is) {
    const int g = (c & 7) >> 1;
    int s0 = 0, s1 = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t wv = u4_word(r.a, i), hv = u4_word(r.c, i);
      const uint32_t lo = (wv & 0x0f0f0f0fu) | (((hv >> (2 * g)) & 0x01010101u) << 4);
      const uint32_t hi = ((wv >> 4) & 0x0f0f0f0fu) | (((hv >> (2 * g + 1)) & 0x01010101u) << 4);
      s0 = __builtin_amdgcn_sdot4((int)lo, x[i], s0, false);
      s1 = __builtin_amdgcn_sdot4((int)hi, x[4 + i], s1, false);
    }
    is[0] = s0;
    is[1] = s1;
  }
};
template <>
struct QDot<QT_Q6_K> {
  __device__ static void isums(const RawChunk& r, int c, const int (&x)[8], int* is) {
    int s0 = 0, s1 = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      s0 = __builtin_amdgcn_sdot4((int)QFmt<QT_Q6_K>::code_lo(r, i), x[i], s0, false);
      s1 = __builtin_amdgcn_sdot4((int)QFmt<QT_Q6_K>::code_hi(r, i), x[4 + i], s1, false);
    }
    is[0] = s0;
    is[1] = s1;
  }
};
template <>
struct QDot<QT_Q8_0> {
  __device__ static void isums(const RawChunk& r, int c, const int (&x)[8], int* is) {
    int s = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) s = __builtin_amdgcn_sdot4((int)u4_word(r.a, i), x[i], s, false);
    is[0] = s;
  }
};

template <int QT>
__device__ __forceinline__ void q8_scales(const RawChunk& r, int c, float* sc, float* of) {
  if constexpr (QT == QT_Q8_0) {
    sc[0] = __half2float(__ushort_as_half((uint16_t)r.d));
    of[0] = 0.f;  // signed codes, no bias
  } else {
    QStream<QT>::scales(r, c, sc, of);
  }
}

// ---------------------------------------------------------------------------------------------
// weight loads: non-temporal (each weight byte is read exactly once per decode step; keeping it
// out of L2/MALL leaves those for x, the KV cache and the residual stream)
// ---------------------------------------------------------------------------------------------
typedef unsigned int q8_u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int q8_u32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 ldnt16(const uint8_t* p) {
  const q8_u32x4 v = __builtin_nontemporal_load((const q8_u32x4*)p);
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint2 ldnt8(const uint8_t* p) {
  const q8_u32x2 v = __builtin_nontemporal_load((const q8_u32x2*)p);
  return make_uint2(v.x, v.y);
}
__device__ __forceinline__ uint32_t ldnt2(const uint8_t* p) {
  return (uint32_t)__builtin_nontemporal_load((const uint16_t*)p);
}

// One wave-uniform weight segment as buffer descriptors: every weight load is a
// buffer_load with the row's byte offset in an SGPR (soffset) and only the lane's chunk offset in
// a VGPR -- no 64-bit address arithmetic per load, and (p made uniform with readfirstlane) no
// per-item reload of the segment table from the kernarg segment.
struct SegRs {
  __amdgpu_buffer_rsrc_t r0, r1, r2, r3;
  int cols;
};
__device__ __forceinline__ __amdgpu_buffer_rsrc_t mk_rsrc(const uint8_t* p) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, 0x7fffffff, 0x00020000);
}
// Wave-uniform copy of a kernarg pointer.  Reading every segment's fields into SGPRs first and
// selecting VALUES (not addresses into the kernarg struct) keeps the struct out of scratch.
__device__ __forceinline__ const uint8_t* sgpr_ptr(const uint8_t* p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const uint8_t*)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ const uint8_t* sel3(int s, const uint8_t* a, const uint8_t* b, const uint8_t* c) {
  a = sgpr_ptr(a);
  b = sgpr_ptr(b);
  c = sgpr_ptr(c);
  return s == 0 ? a : (s == 1 ? b : c);
}
__device__ __forceinline__ SegRs seg_rsrc(const GemvArgs& a, int s) {
  const uint8_t* p0 = sel3(s, a.seg[0].p0, a.seg[1].p0, a.seg[2].p0);
  const uint8_t* p1 = sel3(s, a.seg[0].p1, a.seg[1].p1, a.seg[2].p1);
  const uint8_t* p2 = sel3(s, a.seg[0].p2, a.seg[1].p2, a.seg[2].p2);
  const uint8_t* p3 = sel3(s, a.seg[0].p3, a.seg[1].p3, a.seg[2].p3);
  const int c0 = __builtin_amdgcn_readfirstlane(a.seg[0].cols), c1 = __builtin_amdgcn_readfirstlane(a.seg[1].cols),
            c2 = __builtin_amdgcn_readfirstlane(a.seg[2].cols);
  int cols = s == 0 ? c0 : (s == 1 ? c1 : c2);
  SegRs r;
  r.r0 = mk_rsrc(p0);
  r.r1 = mk_rsrc(p1);
  r.r2 = mk_rsrc(p2);
  r.r3 = mk_rsrc(p3);
  r.cols = cols;
  return r;
}
constexpr int LD_NT = 2;  // cache policy: non-temporal (each weight byte is read once per step)
__device__ __forceinline__ uint4 bl16(__amdgpu_buffer_rsrc_t r, int voff, int soff) {
  const auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, LD_NT);
  return make_uint4(v[0], v[1], v[2], v[3]);
}

// chunk c (lane-varying) of local row `row` (wave-uniform) of a segment
template <int QT>
__device__ __forceinline__ void q8_load(const SegRs& w, int row, int c, RawChunk& r) {
  if constexpr (QT == QT_Q4_K || QT == QT_Q5_K || QT == QT_Q6_K) {
    const int nb = w.cols >> 8;
    const int blk0 = row * nb;  // first block of the row
    r.a = bl16(w.r0, c * 16, blk0 * 128);
    if constexpr (QT == QT_Q6_K) {
      const auto h = __builtin_amdgcn_raw_buffer_load_b64(w.r1, c * 8, blk0 * 64, LD_NT);
      r.b.x = h[0];
      r.b.y = h[1];
      r.c.x = __builtin_amdgcn_raw_buffer_load_b16(w.r2, c * 2, blk0 * 16, LD_NT);  // chunk's scale pair
      r.d = __builtin_amdgcn_raw_buffer_load_b16(w.r3, (c >> 3) * 2, blk0 * 2, LD_NT);
    } else {
      r.b = bl16(w.r1, (c >> 3) * 16, blk0 * 16);
      if constexpr (QT == QT_Q5_K) r.c = bl16(w.r2, (c >> 3) * 32 + 16 * (c & 1), blk0 * 32);
    }
  } else if constexpr (QT == QT_Q4_0) {
    const int blk0 = row * (w.cols >> 5);
    r.a = bl16(w.r0, c * 16, blk0 * 16);
    r.d = __builtin_amdgcn_raw_buffer_load_b16(w.r1, c * 2, blk0 * 2, LD_NT);
  } else {  // Q8_0
    r.a = bl16(w.r0, c * 16, row * w.cols);
    r.d = __builtin_amdgcn_raw_buffer_load_b16(w.r1, (c >> 1) * 2, row * (w.cols >> 5) * 2, LD_NT);
  }
}

// all U chunks of work item `it` for both rows; lanes past the row end re-load the last chunk
// (cheap, in-bounds) and are zeroed in q8_compute instead of branching
template <int QT, int U>
__device__ __forceinline__ void q8_load_item(const SegRs& w, int lrow, int it, int nch, RawChunk (&r)[U][GEMV_ROWS]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = min((it * U + u) * 64 + lane, nch - 1);
#pragma unroll
    for (int rr = 0; rr < GEMV_ROWS; ++rr) q8_load<QT>(w, lrow + rr, c, r[u][rr]);
  }
}

__device__ __forceinline__ float dpp_xor1(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));  // quad_perm 1,0,3,2
}
__device__ __forceinline__ float dpp_xor2(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0x4E, 0xF, 0xF, false));  // quad_perm 2,3,0,1
}
__device__ __forceinline__ int dpp_xor1_i(int v) { return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false); }

// ---------------------------------------------------------------------------------------------
// Prologue: every thread quantises one 8-element octet of x (times the RMSNorm weight, NOT
// normalised) per pass; the 4 lanes of a 32-block share amax through DPP quad permutes and the
// two octets of a 16-run their code sums.  Writes int8 codes in QT's chunk order and per run
// {dx, dx*sum(codes)}; per-wave partial sums of squares go to red[wave][b].
// ---------------------------------------------------------------------------------------------
// x passes loaded ahead of the weights: NPF = ceil(B*K/8 / 512) for the shapes a kernel serves
// (1 for K <= 4096 at B = 1; 4 for the long-K down projection, K <= 16384)
template <int NPF>
struct StagePre {
  float4 x0[NPF], x1[NPF], g0[NPF], g1[NPF];
};
// tid / nthr: the staging threads (default: the whole workgroup)
__device__ __forceinline__ float4 ldx4(const float* p) { return *(const float4*)p; }
template <int NPF>
__device__ __forceinline__ void q8_stage_prefetch(const GemvArgs& a, StagePre<NPF>& pf, int tid = -1, int nthr = 0) {
  if (tid < 0) { tid = threadIdx.x; nthr = blockDim.x; }
  const int noct = a.K >> 3, total = a.B * noct;
#pragma unroll
  for (int i = 0; i < NPF; ++i) {
    const int t = tid + i * nthr;
    // past the end: re-read octet 0 (in bounds, unused) -- no branch around the load
    const int tt = t < total ? t : 0;
    const int b = tt / noct, o = tt - b * noct;
    const float* src = a.x + (size_t)b * a.ldx + 8 * o;
    // both registers are written on both paths: a member left unwritten on one side of the branch
    // sends the whole StagePre to scratch (measured: 80 B/lane in the B=1 engine, -15 % decode)
    float4 r0, r1;
    if (a.x16) {  // 8 bf16 in one 16-B load, widened in q8_stage (no wait here)
      const uint4 u = *(const uint4*)(a.x16 + (size_t)b * a.ldx + 8 * o);
      r0 = make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w));
      r1 = r0;
    } else {
      r0 = ldx4(src);
      r1 = ldx4(src + 4);
    }
    pf.x0[i] = r0;
    pf.x1[i] = r1;
    // the norm weights of every prefetched pass too: a load issued after the weight stream would
    // make its wait cover every weight load in flight
    const float* g = a.norm_w ? a.norm_w + 8 * o : src;
    pf.g0[i] = *(const float4*)g;
    pf.g1[i] = *(const float4*)(g + 4);
  }
}

// 8 bf16 (as the 4 raw words of a float4) -> two float4
__device__ __forceinline__ void bf16x8_widen(float4 raw, float4& f0, float4& f1) {
  const uint32_t w0 = __float_as_uint(raw.x), w1 = __float_as_uint(raw.y), w2 = __float_as_uint(raw.z),
                 w3 = __float_as_uint(raw.w);
  f0 = make_float4(__uint_as_float(w0 << 16), __uint_as_float(w0 & 0xffff0000u), __uint_as_float(w1 << 16),
                   __uint_as_float(w1 & 0xffff0000u));
  f1 = make_float4(__uint_as_float(w2 << 16), __uint_as_float(w2 & 0xffff0000u), __uint_as_float(w3 << 16),
                   __uint_as_float(w3 & 0xffff0000u));
}

// quantise one octet (t -> row b, octet o) of x (times the norm weight) into the staging layout
template <int QT, int B>
__device__ __forceinline__ void q8_octet(const GemvArgs& a, int b, int o, float4 f0, float4 f1, float4 g0, float4 g1,
                                         int8_t* xq, float2* ms, float (&ssq)[B]) {
  using F_ = QFmt<QT>;
  constexpr int W = F_::W, R = F_::RUNS;
  const int nch = a.K / W;
  float v[8] = {f0.x, f0.y, f0.z, f0.w, f1.x, f1.y, f1.z, f1.w};
  float s2 = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) s2 = fmaf(v[i], v[i], s2);
#pragma unroll
  for (int bb = 0; bb < B; ++bb)
    if (bb == b) ssq[bb] += s2;
  if (a.norm_w) {
    v[0] *= g0.x; v[1] *= g0.y; v[2] *= g0.z; v[3] *= g0.w;
    v[4] *= g1.x; v[5] *= g1.y; v[6] *= g1.z; v[7] *= g1.w;
  }
  float am = 0.f;
#pragma unroll
  for (int i = 0; i < 8; ++i) am = fmaxf(am, fabsf(v[i]));
  am = fmaxf(am, dpp_xor1(am));
  am = fmaxf(am, dpp_xor2(am));
  const float dx = am * (1.f / 127.f);
  const float inv = am > 0.f ? 127.f / am : 0.f;
  uint32_t wq[2];
  int isum = 0;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    uint32_t wv = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int q = (int)rintf(v[4 * j + e] * inv);
      isum += q;
      wv |= ((uint32_t)(q & 0xff)) << (8 * e);
    }
    wq[j] = wv;
  }
  isum += dpp_xor1_i(isum);  // the other octet of this 16-run
  const int quarter = o & 3;
  int c, s0;
  F_::run_pos(2 * (o >> 2) + (quarter >> 1), c, s0);
  int piece = s0 >> 4;
  if (W == 32) piece = (piece + (c >> 3)) & 1;
  *(uint2*)(xq + ((size_t)b * nch + c) * W + 16 * piece + 8 * (quarter & 1)) = make_uint2(wq[0], wq[1]);
  if (!(quarter & 1)) ms[((size_t)b * nch + c) * R + (s0 >> 4)] = make_float2(dx, dx * (float)isum);
}

template <int QT, int B, int NPF>
__device__ __forceinline__ void q8_stage(const GemvArgs& a, int8_t* xq, float2* ms, float* red,
                                         const StagePre<NPF>& pf, int tid = -1, int nthr = 0) {
  if (tid < 0) { tid = threadIdx.x; nthr = blockDim.x; }
  const int noct = a.K >> 3, total = a.B * noct;
  float ssq[B];
#pragma unroll
  for (int b = 0; b < B; ++b) ssq[b] = 0.f;
  // the prefetched passes, fully unrolled so the prefetch registers never become an indexed array
#pragma unroll
  for (int i = 0; i < NPF; ++i) {
    const int t = tid + i * nthr;
    if (t < total) {
      const int b = t / noct, o = t - b * noct;
      float4 f0 = pf.x0[i], f1 = pf.x1[i];
      if (a.x16) bf16x8_widen(pf.x0[i], f0, f1);
      q8_octet<QT, B>(a, b, o, f0, f1, pf.g0[i], pf.g1[i], xq, ms, ssq);
    }
  }
  for (int t = tid + NPF * nthr; t < total; t += nthr) {
    const int b = t / noct, o = t - b * noct;
    const float* src = a.x + (size_t)b * a.ldx + 8 * o;
    float4 f0, f1;
    if (a.x16) {
      const uint4 u = *(const uint4*)(a.x16 + (size_t)b * a.ldx + 8 * o);
      bf16x8_widen(make_float4(__uint_as_float(u.x), __uint_as_float(u.y), __uint_as_float(u.z), __uint_as_float(u.w)),
                   f0, f1);
    } else {
      f0 = ldx4(src);
      f1 = ldx4(src + 4);
    }
    float4 g0 = f0, g1 = f1;
    if (a.norm_w) {
      g0 = *(const float4*)(a.norm_w + 8 * o);
      g1 = *(const float4*)(a.norm_w + 8 * o + 4);
    }
    q8_octet<QT, B>(a, b, o, f0, f1, g0, g1, xq, ms, ssq);
  }
  if (a.norm_w) {
    const int wave = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int b = 0; b < B; ++b) {
      const float s = wave_sum(ssq[b]);
      if (lane == 0) red[wave * B + b] = s;
    }
  }
}

// Q4_K/Q5_K scale/min decode for the chunk's sub-block pair (g = (c&7)>>1): one funnel shift of
// the repacked meta (qweight.h kq_field), four bit-field extracts
__device__ __forceinline__ void kq_scales_bf(const RawChunk& r, int c, float* sc, float* of) {
  const int g = (c & 7) >> 1;
  const uint32_t dd = r.b.x;
  const float d = __half2float(__ushort_as_half((uint16_t)(dd & 0xffff)));
  const float dmin = __half2float(__ushort_as_half((uint16_t)(dd >> 16)));
  const uint32_t f = kq_field(r.b.y, r.b.z, r.b.w, g);
  sc[0] = d * (float)(f & 63);
  sc[1] = d * (float)((f >> 6) & 63);
  of[0] = dmin * (float)((f >> 12) & 63);
  of[1] = dmin * (float)((f >> 18) & 63);
}

template <int QT>
__device__ __forceinline__ void q8_scales_bf(const RawChunk& r, int c, float* sc, float* of) {
  if constexpr (QT == QT_Q4_K || QT == QT_Q5_K) kq_scales_bf(r, c, sc, of);
  else q8_scales<QT>(r, c, sc, of);
}

// Microbenchmark bits of tune_dbg inside the dot loop (2: no dot work, 4: no x LDS reads, 8: no
// scale decode) exist only in probe builds (-DAIOS_GEMV_PROBES=1): as runtime branches they cut the
// loop body into basic blocks, and every x LDS read was then waited for right where it was issued
// (the ring GEMM's hot loop measured the same effect, profiles/ring_gemm_r4.txt)
#ifndef AIOS_GEMV_PROBES
#define AIOS_GEMV_PROBES 0
#endif

template <int QT, int B, int U>
__device__ __forceinline__ void q8_compute(const RawChunk (&raw)[U][GEMV_ROWS], int it, int nch, const int8_t* xq,
                                           const float2* ms, float (&acc)[GEMV_ROWS][B], int dbg = 0) {
  using F_ = QFmt<QT>;
  constexpr int W = F_::W, R = F_::RUNS;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c0 = (it * U + u) * 64 + lane;
    const bool valid = c0 < nch;
    const int c = valid ? c0 : nch - 1;
    float sc[GEMV_ROWS][R], of[GEMV_ROWS][R];
#pragma unroll
    for (int r = 0; r < GEMV_ROWS; ++r) {
      if (AIOS_GEMV_PROBES && (dbg & 8)) {  // microbenchmark: scale decode skipped
#pragma unroll
        for (int rr = 0; rr < R; ++rr) { sc[r][rr] = __int_as_float(raw[u][r].b.y | 0x3f000000); of[r][rr] = 0.5f; }
      } else {
        q8_scales_bf<QT>(raw[u][r], c, sc[r], of[r]);
      }
    }
#pragma unroll
    for (int b = 0; b < B; ++b) {
      int xv[8];
      const int8_t* xc = xq + ((size_t)b * nch + c) * W;
      if (AIOS_GEMV_PROBES && (dbg & 4)) {  // microbenchmark: x LDS reads skipped
#pragma unroll
        for (int i = 0; i < 8; ++i) xv[i] = c * 0x01010101 + i;
      } else if constexpr (W == 32) {
        const int rot = (c >> 3) & 1;
        const uint4 p0 = *(const uint4*)(xc + 16 * rot);
        const uint4 p1 = *(const uint4*)(xc + 16 * (rot ^ 1));
        xv[0] = p0.x; xv[1] = p0.y; xv[2] = p0.z; xv[3] = p0.w;
        xv[4] = p1.x; xv[5] = p1.y; xv[6] = p1.z; xv[7] = p1.w;
      } else {
        const uint4 p0 = *(const uint4*)xc;
        xv[0] = p0.x; xv[1] = p0.y; xv[2] = p0.z; xv[3] = p0.w;
        xv[4] = xv[5] = xv[6] = xv[7] = 0;
      }
      float2 m[R];
      const float2* mp = ms + ((size_t)b * nch + c) * R;
#pragma unroll
      for (int rr = 0; rr < R; ++rr) {
        m[rr] = (AIOS_GEMV_PROBES && (dbg & 4)) ? make_float2(1.f, (float)c) : mp[rr];
        if (!valid) m[rr] = make_float2(0.f, 0.f);
      }
#pragma unroll
      for (int r = 0; r < GEMV_ROWS; ++r) {
        int is[R];
        QDot<QT>::isums(raw[u][r], c, xv, is);
#pragma unroll
        for (int rr = 0; rr < R; ++rr) acc[r][b] += sc[r][rr] * m[rr].x * (float)is[rr] - of[r][rr] * m[rr].y;
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// a zero the compiler cannot see through: keeps a uniform load on the vector path (vmcnt-ordered)
__device__ __forceinline__ int opaque_zero() {
  int z;
  asm volatile("v_mov_b32 %0, 0" : "=v"(z));
  return z;
}

// B = 1 epilogue that issues no global LOAD: vmcnt drains in issue order, so a load here would
// wait for the next item's whole weight prefetch.  The residual add is a no-return atomic add
// (each element has exactly one writer, so the result is deterministic); the RoPE (cos, sin) of
// the pair, pos and the KV block were loaded behind the first weight loads (q8_rows_body).  Only
// the rare QKV-bias models load in the epilogue.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ void qkv_part(const GemvArgs& a, int grow, int& part, int& head, int& lr) {
  const int hd = a.head_dim, qd = a.q_dim, kvd = a.kv_dim;
  int r;
  if (grow < qd) { part = 0; r = grow; }
  else if (grow < qd + kvd) { part = 1; r = grow - qd; }
  else { part = 2; r = grow - qd - kvd; }
  head = r / hd;
  lr = r - head * hd;
}
// rope: (cos, sin) of this pair at pos0 (QKV; ignored for V rows and the other epilogues)
__device__ __forceinline__ void gemv_epilogue1(const GemvArgs& a, int grow, float v0, float v1, float2 rope = {1.f, 0.f},
                                               int pos0 = 0, int kv_blk0 = 0) {
  const int nrow = a.row_base + a.N;
  switch (a.epi) {
    case EPI_STORE:
      a.y[grow] = v0;
      if (grow + 1 < nrow) a.y[grow + 1] = v1;
      break;
    case EPI_RESID:
      unsafeAtomicAdd(a.y + grow, v0);
      if (grow + 1 < nrow) unsafeAtomicAdd(a.y + grow + 1, v1);
      break;
    case EPI_SWIGLU: {
      const float h = v0 / (1.f + __expf(-v0)) * v1;
      if (a.y16) a.y16[grow >> 1] = f32_to_bf16(h);
      else a.y[grow >> 1] = h;
    } break;
    case EPI_QKV: {
      if (a.bias) {
        v0 += a.bias[grow];
        v1 += a.bias[grow + 1];
      }
      const int hd = a.head_dim;
      int part, head, lr;
      qkv_part(a, grow, part, head, lr);
      const int pp = lr >> 1;
      int da, db;
      if (part == 2) { da = lr; db = lr + 1; }
      else if (a.rope_neox) { da = pp; db = pp + (hd >> 1); }
      else { da = 2 * pp; db = 2 * pp + 1; }
      if (part < 2) {
        const float o0 = v0 * rope.x - v1 * rope.y, o1 = v0 * rope.y + v1 * rope.x;
        v0 = o0;
        v1 = o1;
      }
      if (part == 0) {
        float* q = a.y + head * hd;
        q[da] = v0;
        q[db] = v1;
      } else {
        bf16_t* cache = pick_ptr(part == 1, a.k_cache, a.v_cache);
        // kv_blk0: the physical block of (slot, pos), looked up once behind the first weight loads
        const size_t base = (((size_t)kv_blk0 * a.n_kv_heads + head) * KV_BLOCK + (pos0 % KV_BLOCK)) * hd;
        // (adjacent pair -- V rows, non-NeoX RoPE: one store)
        kv_store_pair(cache, base + da, base + db, v0, v1, a.kv_fp8, part == 1 ? a.kv_inv_k : a.kv_inv_v);
      }
    } break;
    default:
      __builtin_trap();  // an epilogue this kernel does not do (EPI_TP_RESID runs in the tpf path)
  }
}

// sum of two per-lane values over the wave with 7 cross-lane steps instead of 12:
// returns (row-0 total, row-1 total) in every lane
__device__ __forceinline__ float2 wave_sum_pair(float a0, float a1) {
  const int lane = threadIdx.x & 63;
  float keep = (lane & 32) ? a1 : a0;
  const float send = (lane & 32) ? a0 : a1;
  keep += __shfl_xor(send, 32, 64);
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) keep += __shfl_xor(keep, o, 64);
  const float other = __shfl_xor(keep, 32, 64);
  return (lane & 32) ? make_float2(other, keep) : make_float2(keep, other);
}

// ---------------------------------------------------------------------------------------------
// One wave owns a row pair; a workgroup of nw waves (blockDim / 64: Q8_WAVES, or at batch 1 as
// many as make every CU's wave count equal its pair count, see launch_q8_rows) stages x once and
// walks row pairs grid-stride.  U = 16-B chunks per lane per work item (U*64*W weights of K); host picks U so one
// item spans all of K where it fits (the row pair's whole weight slice in flight at once).
// PIPE = 2 double-buffers across items/pairs (short K), 1 = single buffer (large U).
// ---------------------------------------------------------------------------------------------
constexpr int Q8_WAVES = 8;
// up to 16 waves per workgroup for the register-light variants (U <= 2 single-buffered: the batch-1
// QKV / O shapes).  The double-buffered ones keep 8: at 16 waves (128 VGPRs) they spilled 12-230 B
// per lane to scratch (tools/kernel_resources.py)
template <int U, int PIPE>
constexpr int q8_max_threads() { return U <= 2 && PIPE == 1 ? 1024 : Q8_WAVES * 64; }

template <int QT>
struct FmtTag {
  static constexpr int value = QT;
};

template <int QT0, int QT1, int B, int U, int PIPE>
__global__ void __launch_bounds__((q8_max_threads<U, PIPE>())) gemv_q8_rows(GemvArgs a) {
  static_assert(same_xlayout<QT0, QT1>, "mixed segments must share the activation layout");
  kernarg_warm<sizeof(GemvArgs)>();
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr bool MIXED = QT0 != QT1;
  constexpr int W = QFmt<QT0>::W, R = QFmt<QT0>::RUNS;
  const int nch = a.K / W;
  float* red = smem;                                   // [nw][B] (nw * B <= 64)
  float2* ms = (float2*)(smem + 64);                   // [B][nch][R]
  int8_t* xq = (int8_t*)(ms + (size_t)B * nch * R);    // [B][nch][W]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int nw = __builtin_amdgcn_readfirstlane(blockDim.x >> 6);
  const int npairs = a.N >> 1;
  // pairs [0, np0) use QT0, [np0, npairs) the last segment's QT1: one loop per format, so every
  // loop issues a fixed load sequence and the compiler's vmcnt waits stay exact
  const int srow1 = __builtin_amdgcn_readfirstlane(a.seg_row0[1]);
  const int srow2 = __builtin_amdgcn_readfirstlane(a.seg_row0[2]);
  const int np0 = (MIXED && a.nseg > 1) ? (a.nseg == 2 ? srow1 : srow2) >> 1 : npairs;
  const int nit = (nch + 64 * U - 1) / (64 * U);
  const int stride = gridDim.x * nw;
  const int wid = __builtin_amdgcn_readfirstlane(blockIdx.x * nw + wave);  // wave-uniform -> SGPR
  // probes (tools/gemv_cu_probe.py): phase stamps of the first and last wave of every workgroup --
  // 0 start, 1 first weight loads issued, 2 x staged, 3 barrier passed, 4 first pair computed, 5 done
  // (probe launches only: a wave-uniform branch on the kernarg; each stamp is stored when taken --
  // an array held to the end kept 16 SGPRs live through the kernel and the row GEMVs spilled SGPRs)
  const bool stamps = AIOS_GEMV_PROBES && a.dbg_ts != nullptr;  // (probe builds only)
  bool stamped4 = false;
  auto stamp = [&](int i) __attribute__((always_inline)) {
    if (stamps && lane == 0 && (wave == 0 || wave == nw - 1))
      a.dbg_ts[((size_t)blockIdx.x * 2 + (wave != 0)) * 8 + i] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  // EPI_TP_RESID (batch 1, single format): C1 / C2 of the TP decode step in the epilogue.  Every
  // workgroup ("slot") writes its rows' partials to its private double-buffered stage slot (half
  // e & 1; fine-grained uncached memory mapped by every peer, comm.h), one lane per peer raises that
  // peer's flag [slot][my rank], one lane per peer waits for the peer's flag (bounded, XgmiComm's
  // error flag on a give-up), then each output is summed over the ranks IN RANK ORDER (bit-identical
  // on every rank: the on-device samplers stay in lock step) and added to the residual with a
  // no-return atomic (one writer per element).  A rank reuses half e & 1 at epoch e + 2 only after
  // every peer's epoch-(e + 1) flag of the slot, which the peer raises after its epoch-e reads; every
  // rank runs the same launch shape, so slot s covers the same rows everywhere.  The wave's j-th pair
  // goes to stage position j * nw + wave; the slot's epoch is read here (ordered before use by the
  // x-staging barrier) and written back at the end.  Removes the two all-reduce launches per layer.
  __shared__ uint32_t s_tpe;
  const bool tpf = B == 1 && !MIXED && a.epi == EPI_TP_RESID;
  if (tpf && threadIdx.x == 0) s_tpe = a.tp->fepoch[blockIdx.x] + 1;
  int tpj = 0;          // pairs this wave has finished
  float* tp_mine = nullptr;
  size_t tp_half = 0;

  auto seg_idx = [&](int p, int& lrow) -> int {
    const int row = 2 * p;
    int s = 0;
#pragma unroll
    for (int k = 1; k < GEMV_MAX_SEGS; ++k)
      if (k < a.nseg && row >= a.seg_row0[k]) s = k;
    lrow = row - (s == 0 ? 0 : (s == 1 ? a.seg_row0[1] : a.seg_row0[2]));
    return s;
  };
  // Loads are issued unconditionally: past the range end they read x (L2-resident, in bounds for
  // every stream's small offsets) instead of branching -- a conditional load makes the
  // outstanding-load count path dependent and the compiler then drains with vmcnt(0).
  auto load = [&](auto tag, int p, int pend, int it, RawChunk (&r)[U][GEMV_ROWS]) __attribute__((always_inline)) {
    constexpr int QT = decltype(tag)::value;
    const bool live = p < pend;
    int lrow;
    const int s = seg_idx(live ? p : pend - 1, lrow);
    SegRs w = seg_rsrc(a, s);
    if (!live) {
      const __amdgpu_buffer_rsrc_t rx = mk_rsrc((const uint8_t*)a.x);
      w.r0 = w.r1 = w.r2 = w.r3 = rx;
      lrow = 0;
    }
    q8_load_item<QT, U>(w, lrow, it, nch, r);
  };

  // Batch-1 QKV: pos, the KV block and the pair's RoPE (cos, sin) are looked up AFTER the x and
  // first weight loads are issued and x is staged (a dependent pos -> block table / rope chain in
  // front of them held every weight byte back by two memory round trips,
  // profiles/qkv_prologue_r4.txt); the values are waited for only in the epilogue.
  int pos0 = 0, kv_blk0 = 0, rope_p = -1;
  float2 rope_w = make_float2(1.f, 0.f);
  // decode steps: the step's embedding launch prepared pos / KV block / rope row (StepPrep) -- loads
  // with no dependency, issued here, waited for only in the epilogue
  // (vector loads through an opaque zero offset: a scalar load's lgkmcnt wait would also gate every
  // LDS access of the compute until it returned)
  const bool prepped = B == 1 && a.epi == EPI_QKV && a.step_kv;
  auto rope_of = [&](int p) __attribute__((always_inline)) -> float2 {
    int part, head, lr;
    qkv_part(a, a.row_base + 2 * p, part, head, lr);
    const int pp = lr >> 1;
    if (prepped) return a.step_rope[(part < 2 ? pp : 0) + opaque_zero()];
    if (a.rope_cs) return a.rope_cs[(size_t)pos0 * (a.head_dim >> 1) + (part < 2 ? pp : 0)];
    float sn, cs;
    sincosf((float)pos0 * powf(a.rope_base, -2.f * (float)pp / (float)a.head_dim), &sn, &cs);
    return make_float2(cs, sn);
  };
  auto qkv_lookup = [&](int p_first) __attribute__((always_inline)) {
    if constexpr (B == 1) {
      if (prepped) {
        const int2 kv = *(const int2*)(a.step_kv + opaque_zero());
        pos0 = kv.x;
        kv_blk0 = kv.y;
        if (p_first < npairs) {
          rope_w = rope_of(p_first);
          rope_p = p_first;
        }
      } else if (a.epi == EPI_QKV && !prepped && !(a.tune_dbg & 0x20000)) {  // (probe bit: timing only)
        pos0 = a.pos[0];
        kv_blk0 = kv_block(a.block_table, a.max_ctx / KV_BLOCK, a.slot ? a.slot[0] : 0, pos0);
        if (p_first < npairs) {
          rope_w = rope_of(p_first);
          rope_p = p_first;
        }
      }
    }
  };

  float acc[GEMV_ROWS][B];
#pragma unroll
  for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
    for (int b = 0; b < B; ++b) acc[r][b] = 0.f;
  auto compute = [&](auto tag, int it, const RawChunk (&cur)[U][GEMV_ROWS]) __attribute__((always_inline)) {
    constexpr int QT = decltype(tag)::value;
    if (AIOS_GEMV_PROBES && (a.tune_dbg & 2)) {
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int r = 0; r < GEMV_ROWS; ++r) {
          const RawChunk& q = cur[u][r];
          acc[r][0] += (float)((q.a.x ^ q.a.y ^ q.a.z ^ q.a.w ^ q.b.x ^ q.b.y ^ q.b.z ^ q.b.w ^ q.c.x ^ q.c.w ^ q.d) & 0xff);
        }
      return;
    }
    q8_compute<QT, B, U>(cur, it, nch, xq, ms, acc, a.tune_dbg);
  };
  auto finish = [&](int p) __attribute__((always_inline)) {
    float s[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      s[b] = 1.f;
      if (a.norm_w) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < nw; ++w) t += red[w * B + b];
        s[b] = rsqrtf(t / (float)a.K + a.eps);
      }
    }
    if (stamps && !stamped4) {
      stamp(4);
      stamped4 = true;
    }
    if constexpr (B == 1) {
      const float2 v = wave_sum_pair(acc[0][0], acc[1][0]);
      float2 rope = rope_w;
      if (a.epi == EPI_QKV && p != rope_p) rope = rope_of(p);  // a grid-stride pair after the first
      if (tpf) {
        if (!tp_mine) {  // first pair: the epoch is in LDS (written before the staging barrier)
          const uint32_t e = s_tpe;
          tp_half = ((size_t)blockIdx.x * 2 + (e & 1u)) * TPF_CAP;
          tp_mine = tpf_stage(a.tp, a.tp->rank) + tp_half;
        }
        if (lane == 0) *(float2*)(tp_mine + 2 * (tpj * nw + wave)) = make_float2(v.x * s[0], v.y * s[0]);
        ++tpj;
      } else if (lane == 0) {
        gemv_epilogue1(a, a.row_base + 2 * p, v.x * s[0], v.y * s[0], rope, pos0, kv_blk0);
      }
    } else {
#pragma unroll
      for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
        for (int b = 0; b < B; ++b) acc[r][b] = wave_sum(acc[r][b]);
      if (lane < a.B) {
        float v0 = 0.f, v1 = 0.f, sc = 1.f;
#pragma unroll
        for (int b = 0; b < B; ++b)
          if (lane == b) { v0 = acc[0][b]; v1 = acc[1][b]; sc = s[b]; }
        gemv_epilogue(a, a.row_base + 2 * p, lane, v0 * sc, v1 * sc);
      }
    }
#pragma unroll
    for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
      for (int b = 0; b < B; ++b) acc[r][b] = 0.f;
  };

  RawChunk buf[PIPE][U][GEMV_ROWS];
  auto& bufA = buf[0];
  // walk pairs [p, pend) grid-stride; B[0] already holds item (p, 0).  The register buffer is a
  // parameter so the two formats of a mixed launch each get their own (one shared array written
  // through two different load sequences defeats SROA and lands in scratch)
  auto run = [&](auto tag, int p, int pend, int stride, RawChunk (&buf)[PIPE][U][GEMV_ROWS]) __attribute__((always_inline)) {
    auto& bufA = buf[0];
    if (p >= pend) return;
    if constexpr (PIPE >= 2) {
      // PIPE register buffers in rotation, each reloaded right after it was consumed with the item
      // PIPE-1 ahead of the one computing next: PIPE-1 items stay in flight during every compute
      int pk[PIPE], ik[PIPE];
      pk[0] = p;
      ik[0] = 0;
      int tp = p, ti = 0;  // most recently scheduled item
#pragma unroll
      for (int k = 1; k < PIPE; ++k) {
        if (++ti >= nit) { ti = 0; tp += stride; }
        pk[k] = tp;
        ik[k] = ti;
        load(tag, tp, pend, ti, buf[k]);
      }
      bool done = false;
      while (!done) {
#pragma unroll
        for (int k = 0; k < PIPE; ++k) {
          if (!done) {
            if (pk[k] >= pend) {
              done = true;
            } else {
              compute(tag, ik[k], buf[k]);
              if (ik[k] == nit - 1) finish(pk[k]);
              if (++ti >= nit) { ti = 0; tp += stride; }
              pk[k] = tp;
              ik[k] = ti;
              load(tag, tp, pend, ti, buf[k]);
            }
          }
        }
      }
    } else {
      int it = 0;
      while (true) {
        compute(tag, it, bufA);
        if (++it >= nit) {
          finish(p);
          it = 0;
          p += stride;
          if (p >= pend) break;
        }
        load(tag, p, pend, it, bufA);
      }
    }
  };

  constexpr int NPF = (B == 1 && U >= 3) ? 4 : 1;
  StagePre<NPF> pf{};
  q8_stage_prefetch(a, pf);  // x first: its wait then does not cover the weights
  if constexpr (!MIXED) {
    load(FmtTag<QT0>{}, wid, npairs, 0, bufA);  // weight loads in flight during the prologue
    stamp(1);
    if (!(a.tune_dbg & 1)) q8_stage<QT0, B, NPF>(a, xq, ms, red, pf);
    qkv_lookup(wid);
    stamp(2);
    __syncthreads();
    stamp(3);
    run(FmtTag<QT0>{}, wid, npairs, stride, buf);
    if (tpf) {
      // every wave's stage stores, then one flag per peer (wave 0), the bounded wait, and the
      // rank-ordered sum of each of this wave's pairs into the residual
      const ArDevCtx* c = a.tp;
      const int rank = c->rank, world = c->world;
      const uint32_t e = s_tpe;
      const size_t half = ((size_t)blockIdx.x * 2 + (e & 1u)) * TPF_CAP;
      // (uncached stage / flags: retired stores are visible to the peers -- no system-scope fence,
      // which writes back the whole L2 and, from every wave, cost ~80 us per launch)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (wave == 0) {
        constexpr uint64_t TIMEOUT = 100ull * 1000 * 1000 * 3;  // 3 s of the 100 MHz wall clock
        if (lane < world && lane != rank)
          __hip_atomic_store(tpf_flags(c, lane) + blockIdx.x * AR_MAX_RANKS + rank, e, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_SYSTEM);
        if (lane < world && lane != rank) {
          uint32_t* f = tpf_flags(c, rank) + blockIdx.x * AR_MAX_RANKS + lane;
          const uint64_t t0 = wall_clock64();
          while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
            __builtin_amdgcn_s_sleep(2);
            if (wall_clock64() - t0 > TIMEOUT) {
              __hip_atomic_store(c->error, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
              break;
            }
          }
        }
      }
      __syncthreads();
      int j = 0;
      for (int p = wid; p < npairs; p += stride, ++j) {
        if (lane < 2) {  // lane 0: the pair's first row, lane 1: its second
          const size_t o = half + 2 * (j * nw + wave) + lane;
          float acc = 0.f;
          for (int q = 0; q < world; ++q) acc += __builtin_nontemporal_load(tpf_stage(c, q) + o);
          unsafeAtomicAdd(a.y + a.row_base + 2 * p + lane, acc);
        }
      }
      if (threadIdx.x == 0) c->fepoch[blockIdx.x] = e;
    }
  } else {
    // Mixed formats (Q4_K q/k + Q6_K v of a Q4_K_M QKV): the waves of EVERY workgroup are split
    // in proportion to the pair counts (Mistral: 10 Q4_K + 2 Q6_K pairs per 12-wave workgroup), so
    // each CU streams the same bytes -- a split by whole workgroups left the Q6_K CUs 1.46x the
    // bytes of the others (QKV 8.25 us vs 7.09 with V in Q4_K, profiles/qkv_prologue_r4.txt) -- and
    // both formats stream concurrently (a Q6_K phase after the Q4_K one added a full memory round
    // trip: 11.6 vs 8.3 us).  Each branch runs the same x staging and exactly one workgroup barrier
    // (s_barrier counts waves, not call sites); the x staging is the same for both formats
    // (same_xlayout).
    const int W = stride;
    int nw0 = (int)(((long)nw * np0 + npairs / 2) / npairs);
    nw0 = max(1, min(nw - 1, nw0));
    const int nw1 = nw - nw0;
    if (W < 16) {  // tiny grid: the sequential schedule
      load(FmtTag<QT0>{}, wid, np0, 0, bufA);
      stamp(1);
      if (!(a.tune_dbg & 1)) q8_stage<QT0, B, NPF>(a, xq, ms, red, pf);
      qkv_lookup(wid < np0 ? wid : npairs);
      stamp(2);
      __syncthreads();
      stamp(3);
      run(FmtTag<QT0>{}, wid, np0, stride, buf);
      // the second format gets its own register buffer: one array written through two different
      // load sequences defeats SROA and lands in scratch
      RawChunk bufT[PIPE][U][GEMV_ROWS];
      load(FmtTag<QT1>{}, np0 + wid, npairs, 0, bufT[0]);
      stamp(1);
      run(FmtTag<QT1>{}, np0 + wid, npairs, stride, bufT);
    } else if (wave < nw0) {
      const int p0 = __builtin_amdgcn_readfirstlane(blockIdx.x * nw0 + wave);
      load(FmtTag<QT0>{}, p0, np0, 0, bufA);
      stamp(1);
      if (!(a.tune_dbg & 1)) q8_stage<QT0, B, NPF>(a, xq, ms, red, pf);
      qkv_lookup(p0 < np0 ? p0 : npairs);
      stamp(2);
      __syncthreads();
      stamp(3);
      run(FmtTag<QT0>{}, p0, np0, (int)gridDim.x * nw0, buf);
    } else {
      const int p1 = __builtin_amdgcn_readfirstlane(np0 + blockIdx.x * nw1 + (wave - nw0));
      RawChunk buf1[PIPE][U][GEMV_ROWS];
      load(FmtTag<QT1>{}, p1, npairs, 0, buf1[0]);
      stamp(1);
      if (!(a.tune_dbg & 1)) q8_stage<QT0, B, NPF>(a, xq, ms, red, pf);
      qkv_lookup(p1);
      stamp(2);
      __syncthreads();
      stamp(3);
      run(FmtTag<QT1>{}, p1, npairs, (int)gridDim.x * nw1, buf1);
    }
  }
  stamp(5);
}

template <int QT0, int QT1, int B>
inline size_t q8_lds_bytes(int K) {
  constexpr int W = QFmt<QT0>::W, R = QFmt<QT0>::RUNS;
  return 64 * 4 + (size_t)B * (K / W) * R * 8 + (size_t)B * K + 2048 + 16;
}

// false (nothing launched): an EPI_TP_RESID launch whose rows do not fit the fused stage within the
// co-residency cap -- the caller takes the separate all-reduce instead
template <int QT0, int QT1, int B, int U, int PIPE>
bool launch_q8_rows(const GemvArgs& a, size_t lds, hipStream_t st) {
  static int occ = -1;
  if (occ < 0) {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, gemv_q8_rows<QT0, QT1, B, U, PIPE>, Q8_WAVES * 64, lds) !=
            hipSuccess || o <= 0)
      o = 1;
    occ = o;
  }
  int per_cu = std::min(occ, 2);
  if (a.tune_grid > 0) per_cu = a.tune_grid;
  const int npairs = a.N / 2;
  const int cus = device_cu_count();
  // Batch 1, one pair per wave: 8-wave workgroups leave CUs unequal whenever npairs / 8 is not a
  // multiple of the CU count (Mistral QKV: 3072 pairs = 384 workgroups on 256 CUs -> half the CUs
  // stream 16 pairs, half 8).  Instead size the workgroup to ceil(npairs / CUs) waves (<= 16) and
  // launch one per CU: every CU streams the same bytes (AIOS_Q8_BALANCE=0: the 8-wave grid).
  static const int balance = [] {
    const char* e = std::getenv("AIOS_Q8_BALANCE");
    return e ? std::atoi(e) : 1;
  }();
  int nw = Q8_WAVES;
  int blocks = 0;
  if (B == 1 && balance && a.tune_grid <= 0 && npairs >= 2 * cus) {
    // round 4: also for the register-heavy U >= 3 variants (<= 8 waves) and for shapes with more
    // pairs than waves (ppw pairs per wave, one workgroup per CU): TinyLlama's down (1024 pairs,
    // U = 3) ran 128 8-wave workgroups on half the chip, its gate/up (5632 pairs) 512 workgroups with
    // 1 or 2 pairs per wave
    const int maxw = q8_max_threads<U, PIPE>() / 64;
    const int ppw = (npairs + cus * maxw - 1) / (cus * maxw);
    int want = (npairs + cus * ppw - 1) / (cus * ppw);
    bool mixed = false;
    int np0 = 0;
    if (QT0 != QT1 && a.nseg > 1 && ppw == 1) {
      // mixed formats: whole waves per format in every workgroup (the kernel splits nw by pair
      // counts), e.g. TinyLlama's QKV 1152 Q4_K + 128 Q6_K pairs -> 5 + 1 waves, not 4 + 1
      np0 = a.seg_row0[a.nseg - 1] / 2;
      want = (np0 + cus - 1) / cus + (npairs - np0 + cus - 1) / cus;
      mixed = true;
    }
    // several pairs per wave only for the long-K (U >= 3) shapes: TinyLlama's 5632-pair gate/up at
    // U = 1 went 6.96 -> 9.15 us as 3 pairs per wave on one 8-wave workgroup per CU
    // (profiles/decode_tinyllama_rocprof_r4.txt)
    if (want >= 2 && want <= maxw && (ppw == 1 || U >= 3)) {
      nw = want;
      blocks = std::min(cus, (npairs + nw - 1) / nw);
      if (mixed) {
        // the grid must cover each format's pairs with ITS waves (the kernel's split below):
        // 214 blocks x 5 Q4_K waves left 82 of TinyLlama's 1152 Q|K pairs to a second pass (9.5 us)
        int nw0 = (int)(((long)nw * np0 + npairs / 2) / npairs);
        nw0 = std::max(1, std::min(nw - 1, nw0));
        const int nw1 = nw - nw0;
        blocks = std::min(cus, std::max((np0 + nw0 - 1) / nw0, (npairs - np0 + nw1 - 1) / nw1));
      }
    }
  }
  if (!blocks) blocks = std::min((npairs + nw - 1) / nw, cus * per_cu);
  if (a.epi == EPI_TP_RESID) {
    // fused all-reduce: at most grid_cap workgroups (every rank sharing a GPU resident at once --
    // spinning workgroups past it could wait on peers that cannot be scheduled), at most
    // TPF_SLOTS, and each workgroup's pairs inside its stage slot (TPF_CAP values)
    const int cap = a.grid_cap > 0 ? std::min(a.grid_cap, TPF_SLOTS) : TPF_SLOTS;
    blocks = std::min(blocks, cap);
    auto per_wg = [&](int g) { return 2 * nw * ((npairs + g * nw - 1) / (g * nw)); };
    while (per_wg(blocks) > TPF_CAP && blocks < cap) ++blocks;
    if (per_wg(blocks) > TPF_CAP) return false;
    if (a.dry) return true;  // (TP init: every rank's fit for this shape is all-gathered first)
  }
  hipLaunchKernelGGL((gemv_q8_rows<QT0, QT1, B, U, PIPE>), dim3(blocks), dim3(nw * 64), lds, st, a);
  return true;
}

template <int QT0, int QT1, int B>
bool launch_gemv_q8(GemvArgs a, hipStream_t st) {
  if constexpr (!same_xlayout<QT0, QT1>) {
    return false;
  } else {
    const size_t lds = q8_lds_bytes<QT0, QT1, B>(a.K);
    if (lds > 128 * 1024) return false;
    a.kt_max = a.K;
    if constexpr (B == 1) {
      const int nch = a.K / QFmt<QT0>::W;
      int u = a.tune_u;
      if (u <= 0 || (u > 8 && u != 11 && u != 12 && u != 13 && u != 14 && u != 21 && u != 22 && u != 31)) {
        // MI355X sweep (tools/gemv_probe.py --sweep): one chunk per lane per item for short K,
        // except the mid-sized Q4_K/Q5_K projections; the whole K slice in flight for long K
        // (U = 1 for the small/huge-N shapes won in the eager sweep but lost 2-3 % inside the
        // captured decode step, so the whole-K-slice rule stays)
        // (re-swept in the captured step, tools/gemv_knob_sweep.sh: U = 1 for K = 4096 gate/up
        // +1.8 %, QKV +1 %, O / lm_head neutral)
        u = nch <= 128 ? 1 : (nch <= 512 ? (nch + 63) / 64 : 2);
        // Round 4 (tools/gemv_cu_probe.py row-kernel stamps): when the balanced launch gives every
        // wave exactly ONE row pair, the double-buffered U = 1 pipeline issued the pair's second K
        // half only after the x-staging barrier -- a second memory round trip on the critical path
        // (O: barrier 1.9 us, pair computed 3.6 us).  The pair's whole K slice in one single-buffered
        // item instead: QKV 8.27 -> 7.36 us, O 5.71 -> 5.05 (profiles/qkv_prologue_r4.txt).
        const int npairs = a.N / 2;
        static const int balance = [] {
          const char* e = std::getenv("AIOS_Q8_BALANCE");
          return e ? std::atoi(e) : 1;
        }();
        if (balance && a.tune_grid <= 0 && npairs <= 16 * device_cu_count() && nch <= 128)
          u = nch <= 64 ? 11 : 12;
      }
      switch (u) {
        case 11: return launch_q8_rows<QT0, QT1, 1, 1, 1>(a, lds, st);  // one pair per wave: the K slice in
        case 12: return launch_q8_rows<QT0, QT1, 1, 2, 1>(a, lds, st);  // one single-buffered item
        case 13: return launch_q8_rows<QT0, QT1, 1, 3, 2>(a, lds, st);  // tuning: U = 3/4 double-buffered
        case 14: return launch_q8_rows<QT0, QT1, 1, 4, 2>(a, lds, st);
        case 21: return launch_q8_rows<QT0, QT1, 1, 1, 3>(a, lds, st);  // tuning: triple / quad buffers
        case 22: return launch_q8_rows<QT0, QT1, 1, 2, 3>(a, lds, st);
        case 31: return launch_q8_rows<QT0, QT1, 1, 1, 4>(a, lds, st);
        case 1: return launch_q8_rows<QT0, QT1, 1, 1, 2>(a, lds, st);
        case 2: return launch_q8_rows<QT0, QT1, 1, 2, 2>(a, lds, st);
        case 3: return launch_q8_rows<QT0, QT1, 1, 3, 1>(a, lds, st);
        case 4: return launch_q8_rows<QT0, QT1, 1, 4, 1>(a, lds, st);
        case 5: return launch_q8_rows<QT0, QT1, 1, 5, 1>(a, lds, st);
        case 6: return launch_q8_rows<QT0, QT1, 1, 6, 1>(a, lds, st);
        case 7: return launch_q8_rows<QT0, QT1, 1, 7, 1>(a, lds, st);
        default: return launch_q8_rows<QT0, QT1, 1, 8, 1>(a, lds, st);
      }
    } else if constexpr (B == 8) {
      return launch_q8_rows<QT0, QT1, 8, 1, 2>(a, lds, st);
    } else {
      return launch_q8_rows<QT0, QT1, B, 2, 2>(a, lds, st);
    }
    return true;
  }
}
