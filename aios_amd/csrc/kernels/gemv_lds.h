// Loader / consumer batch-1 decode GEMV (int8 activations) with an LDS-DMA weight ring; included by
// gemv_impl.h after gemv_cu.h.
//
// Measured on MI355X (tools/gemv_cu_probe.py, in-kernel s_memrealtime stamps): in a GEMV whose waves
// both load weights into registers and compute, the weight stream STALLS while x is staged -- the
// registers hold the first loads, no more can be issued until x (the previous kernel's output, ~1-2
// us away) is quantised into LDS and the workgroup barrier passes, and x's own loads queue behind
// the CU's weight loads.  gate_up: barrier at 6.5 us of a 19 us kernel whose bytes need 10.7 us.
//
// Here the roles are split, the MI355X batch-1 engine shape (MI355X_MICROARCH.md price list rows
// 'ldsdma-fill', 'engine-vs-launches'): per CU one 1024-thread workgroup, waves 14-15 only move
// weight bytes HBM -> LDS with LDS-DMA (global_load_lds_dwordx4 nt, no VGPR round trip) into a ring
// of R slots (5-8), waves 0-13 stage x and then each computes one 64-chunk group per slot.  The loaders
// never wait for compute: a slot is refilled one step after it was consumed, R-1 slots (95-112 KB)
// stay in flight, so the x staging latency is covered by the ring instead of idling the stream.
// Steps are lock-stepped with raw s_barrier (no fence: a __syncthreads would drain every in-flight
// DMA, cdna_hip_programming.md 'Pipelining across barriers'); the loaders' counted vmcnt waits are
// inline asm with immediates fixed by the format's DMA count per slot.
//
// Each slot holds NG = 14 groups (one per consumer wave); a group is 64 chunks of one row (so
// nch % 64 == 0 is required), and every weight plane of the format is copied per slot as its own
// contiguous region (group k of plane P at P_off + k * bytes_per_group(P)); a DMA lane computes its
// own source address, so a slot may span segments (Q|K) and rows freely.
#pragma once
// (included inside namespace aios by gemv_impl.h)

constexpr int LG_NG = 14;               // consumer waves
constexpr int LG_NL = 2;                // loader waves
constexpr int LG_THREADS = (LG_NG + LG_NL) * 64;
// tune_dbg bit (probes only): the consumers skip the slot reads and the dot work -- the bare
// DMA ring + barrier cadence of the engine (tools/gemv_cu_probe.py 'ring' column)
constexpr int LG_DBG_RING = 0x10000;
// B0 (x loads queued ahead of the first weight DMA): measured slower -- the loaders' first slots
// then start ~1.6 us late while x is an L2/MALL hit either way
#ifndef LG_B0
#define LG_B0 0
#endif

// planes of a format: bytes per 64-chunk group and the LDS-DMA width used to copy it
template <int QT>
struct LgPlanes;
template <>
struct LgPlanes<QT_Q4_K> {
  static constexpr int n = 2;
  static constexpr int bpg[4] = {1024, 128, 0, 0};
  static constexpr int dsz[4] = {16, 16, 0, 0};
};
template <>
struct LgPlanes<QT_Q5_K> {
  static constexpr int n = 3;
  static constexpr int bpg[4] = {1024, 128, 256, 0};
  static constexpr int dsz[4] = {16, 16, 16, 0};
};
template <>
struct LgPlanes<QT_Q6_K> {
  static constexpr int n = 4;
  static constexpr int bpg[4] = {1024, 512, 128, 16};
  static constexpr int dsz[4] = {16, 16, 16, 4};
};
template <>
struct LgPlanes<QT_Q4_0> {
  static constexpr int n = 2;
  static constexpr int bpg[4] = {1024, 128, 0, 0};
  static constexpr int dsz[4] = {16, 16, 0, 0};
};
template <>
struct LgPlanes<QT_Q8_0> {
  static constexpr int n = 2;
  static constexpr int bpg[4] = {1024, 64, 0, 0};
  static constexpr int dsz[4] = {16, 16, 0, 0};
};

template <int QT, int RSUB = 0>
struct LgLayout {
  using P = LgPlanes<QT>;
  // groups per consumer wave per step: 2 for the 4.5-bit formats (the pair shares one row sum and
  // gives each wave two independent chains per step), 1 where a slot would not fit R >= 5 in LDS
  static constexpr int GPW = (QT == QT_Q6_K || QT == QT_Q5_K) ? 1 : 2;
  static constexpr int NGS = LG_NG * GPW;  // groups per slot
  // DMA instructions (one wave each) for plane p of a slot, and its padded LDS region
  static constexpr int ninst(int p) { return (NGS * P::bpg[p] + 64 * P::dsz[p] - 1) / (64 * P::dsz[p]); }
  static constexpr int region(int p) { return p < P::n ? ninst(p) * 64 * P::dsz[p] : 0; }
  static constexpr int off(int p) { return p == 0 ? 0 : off(p - 1) + region(p - 1); }
  static constexpr int slot_bytes = off(4);
  static constexpr int total_inst = (P::n > 0 ? ninst(0) : 0) + (P::n > 1 ? ninst(1) : 0) + (P::n > 2 ? ninst(2) : 0) +
                                    (P::n > 3 ? ninst(3) : 0);
  // instructions per slot issued by one loader wave (instruction i goes to loader i % LG_NL); the
  // loaders' vmcnt immediates assume every slot issues exactly this many
  static constexpr int per_loader = (total_inst + LG_NL - 1) / LG_NL;
  // ring slots: R - 1 slots in flight must cover HBM latency x the CU's share of the bandwidth
  // (~2-3 us x 24 GB/s under full load): 3 x 32 KB for the 4.5-bit formats, 4 x 24 KB for Q6_K
  // (RSUB: one slot fewer for the batched launches, whose B staged x vectors take the LDS)
  static constexpr int R = (slot_bytes > 28 * 1024 ? 4 : (slot_bytes <= 20 * 1024 ? 6 : 5)) - RSUB;
  static_assert(R >= 2 && (R - 2) * per_loader <= 63, "ring depth / vmcnt immediate");
};

__device__ __forceinline__ const uint8_t* lg_plane_ptr(const QWeight& w, int p) {
  return p == 0 ? w.p0 : (p == 1 ? w.p1 : (p == 2 ? w.p2 : w.p3));
}

// raw workgroup barrier (no fence: in-flight LDS-DMA survives it), a compiler memory barrier on
// both sides so no LDS access moves across it
__device__ __forceinline__ void lg_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int N>
__device__ __forceinline__ void lg_vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt immediate");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// Copy slot s (groups [s*NGS, s*NGS+NGS) of this workgroup) into ring buffer `dst`.
//
// A 64-chunk group is 64 chunks of one row, so in every plane the group with global index
// G = row * nit + it sits at plane_base(seg) + (G - first_group(seg)) * bytes_per_group: within a
// segment a plane is LINEAR in the group index and one slot's plane region is one contiguous byte
// range.  Fast path (the slot inside one segment, no tail clamp): buffer_load ... lds with the
// segment's plane as the resource, the slot offset in an SGPR and lane * width as the only VGPR --
// one SALU add per 1 KB instruction (a per-lane address version spent ~25-65 instructions per DMA
// and the loaders' issue rate, not HBM, set the step time).  General path (a slot crossing Q|K, or
// the last slot): per-lane segment select and clamp.  Loader wave lw issues instructions lw,
// lw + NL, ...; every loader issues exactly per_loader instructions per slot (exact counted waits).
template <int QT>
__device__ __forceinline__ void lg_dma_slot(const GemvArgs& a, uint8_t* dst, int s, int lw, int r0, int nit,
                                            int ngroups) {
  using L = LgLayout<QT>;  // (slot geometry only: identical for every RSUB)
  using P = LgPlanes<QT>;
  constexpr int NGS = L::NGS;
  const int lane = threadIdx.x & 63;
  const int g0 = r0 * nit + s * NGS;            // global group index of the slot's first group
  const int glast = r0 * nit + ngroups - 1;     // last group of the workgroup
  const int G1 = a.nseg > 1 ? a.seg_row0[1] * nit : 0x7fffffff;
  const int G2 = a.nseg > 2 ? a.seg_row0[2] * nit : 0x7fffffff;
  const int gend = g0 + NGS - 1;
  const int sg0 = g0 >= G2 ? 2 : (g0 >= G1 ? 1 : 0);
  const int Gs = sg0 == 0 ? 0 : (sg0 == 1 ? G1 : G2);
  const int Gn = sg0 == 0 ? G1 : (sg0 == 1 ? G2 : 0x7fffffff);
  const bool fast = gend <= glast && gend < Gn;
  int issued = 0;
  int idx = 0;  // running instruction index over the planes
  static_for<4>([&](auto pc) {
    constexpr int p = decltype(pc)::value;
    if constexpr (p < P::n) {
      constexpr int S = P::dsz[p], BPG = P::bpg[p];
      constexpr int NI = L::ninst(p);
      const uint8_t* pb0 = sgpr_ptr(lg_plane_ptr(a.seg[0], p));
      const uint8_t* pb1 = sgpr_ptr(lg_plane_ptr(a.seg[1], p));
      const uint8_t* pb2 = sgpr_ptr(lg_plane_ptr(a.seg[2], p));
      if (fast) {
        const __amdgpu_buffer_rsrc_t rs = mk_rsrc(sg0 == 0 ? pb0 : (sg0 == 1 ? pb1 : pb2));
        const int soff0 = (g0 - Gs) * BPG;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          if ((idx + i) % LG_NL != lw) continue;
          auto* ldst = (__attribute__((address_space(3))) void*)(dst + L::off(p) + i * 64 * S);
          // (default policy instead of nt: +6-7 % on gate_up / down / lm_head, tools/gemv_cu_probe.py)
          if constexpr (S == 16) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, ldst, 16, lane * 16, soff0 + i * 1024, 0, 2);
          else __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, ldst, 4, lane * 4, soff0 + i * 256, 0, 2 /* nt */);
          ++issued;
        }
      } else {
        // per-segment base shifted so that (group * BPG) indexes it directly
        const uint64_t b0 = (uint64_t)pb0;
        const uint64_t b1 = (uint64_t)pb1 - (uint64_t)(a.nseg > 1 ? G1 : 0) * BPG;
        const uint64_t b2 = (uint64_t)pb2 - (uint64_t)(a.nseg > 2 ? G2 : 0) * BPG;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          if ((idx + i) % LG_NL != lw) continue;
          const int b = i * 64 * S + lane * S;  // byte within the plane's slot region
          int g = g0 + b / BPG;                 // BPG is a power of two: a shift
          const int o = b & (BPG - 1);
          g = min(g, glast);                    // the last slot's tail and the padding lanes
          const uint64_t base = g >= G2 ? b2 : (g >= G1 ? b1 : b0);
          const uint8_t* src = (const uint8_t*)(base + (uint64_t)g * BPG + o);
          auto* ldst = (__attribute__((address_space(3))) void*)(dst + L::off(p) + i * 64 * S);
          if constexpr (S == 16) __builtin_amdgcn_global_load_lds((const void*)src, ldst, 16, 0, 2 /* nt */);
          else __builtin_amdgcn_global_load_lds((const void*)src, ldst, 4, 0, 2 /* nt */);
          ++issued;
        }
      }
      idx += NI;
    }
  });
  // pad to per_loader instructions (re-issue the slot's first piece of plane 0 into its own place)
  if (issued < L::per_loader) {
    const int g = min(g0, glast);
    const uint64_t b0 = (uint64_t)sgpr_ptr(a.seg[0].p0);
    const uint64_t b1 = (uint64_t)sgpr_ptr(a.seg[1].p0) - (uint64_t)(a.nseg > 1 ? G1 : 0) * 1024;
    const uint64_t b2 = (uint64_t)sgpr_ptr(a.seg[2].p0) - (uint64_t)(a.nseg > 2 ? G2 : 0) * 1024;
    const uint64_t base = g >= G2 ? b2 : (g >= G1 ? b1 : b0);
    const uint8_t* src = (const uint8_t*)(base + (uint64_t)g * 1024 + lane * 16);
    for (; issued < L::per_loader; ++issued)
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 2);
  }
}

// consumer: the raw chunk of lane `lane` of group k from a ring slot
template <int QT>
__device__ __forceinline__ void lg_read(const uint8_t* slot, int k, int lane, RawChunk& r) {
  using L = LgLayout<QT>;
  const uint8_t* A = slot + L::off(0) + k * 1024;
  r.a = *(const uint4*)(A + lane * 16);
  if constexpr (QT == QT_Q4_K || QT == QT_Q5_K) {
    r.b = *(const uint4*)(slot + L::off(1) + k * 128 + (lane >> 3) * 16);
    if constexpr (QT == QT_Q5_K) r.c = *(const uint4*)(slot + L::off(2) + k * 256 + (lane >> 3) * 32 + 16 * (lane & 1));
  } else if constexpr (QT == QT_Q6_K) {
    const uint2 h = *(const uint2*)(slot + L::off(1) + k * 512 + lane * 8);
    r.b.x = h.x;
    r.b.y = h.y;
    r.c.x = *(const uint16_t*)(slot + L::off(2) + k * 128 + lane * 2);
    r.d = *(const uint16_t*)(slot + L::off(3) + k * 16 + (lane >> 3) * 2);
  } else if constexpr (QT == QT_Q4_0) {
    r.d = *(const uint16_t*)(slot + L::off(1) + k * 128 + lane * 2);
  } else {  // Q8_0
    r.d = *(const uint16_t*)(slot + L::off(1) + k * 64 + (lane >> 1) * 2);
  }
}

// ---- batched consumers (B = 2..4 rows of x, one weight read): the weight decode is shared, the
// integer dot products and the float scaling run per row
template <int B>
__device__ __forceinline__ void q4p_dot_b(const uint4& a0, const uint4& a1, const uint4& mt, int g,
                                          const Q4PairX (&X)[B], float (&out)[B]) {
  const float d = __half2float(__ushort_as_half((uint16_t)(mt.x & 0xffff)));
  const float dmin = __half2float(__ushort_as_half((uint16_t)(mt.x >> 16)));
  const uint32_t f = kq_field(mt.y, mt.z, mt.w, g);
  int s0[B], s1[B];
#pragma unroll
  for (int b = 0; b < B; ++b) s0[b] = s1[b] = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t w = u4_word(i < 4 ? a0 : a1, i & 3);
    const int lo = (int)(w & 0x0f0f0f0fu), hi = (int)((w >> 4) & 0x0f0f0f0fu);
#pragma unroll
    for (int b = 0; b < B; ++b) {
      s0[b] = __builtin_amdgcn_sdot4(lo, X[b].x0[i], s0[b], false);
      s1[b] = __builtin_amdgcn_sdot4(hi, X[b].x1[i], s1[b], false);
    }
  }
  const float c0 = (float)(f & 63), c1 = (float)((f >> 6) & 63);
  const float m0 = (float)((f >> 12) & 63), m1 = (float)((f >> 18) & 63);
#pragma unroll
  for (int b = 0; b < B; ++b)
    out[b] = d * (c0 * X[b].dx0 * (float)s0[b] + c1 * X[b].dx1 * (float)s1[b]) - dmin * (m0 * X[b].sx0 + m1 * X[b].sx1);
}

// B row sums over each 32-lane half at the cost of ~one: a butterfly first halves the value set per
// lane (xor 1: lanes keep rows {0,1} / {2,3}; xor 2: one row each), then the rows' classes reduce
// with row rotations by 4 and 8 and the 16-lane swap.  Returns, in every lane, the half's total of row
// lg_half_row<B>(p) (p = lane & 31): rows 0..B-1 end up in lanes 0..3 of each half (B = 3: the
// fourth value is 0 and its lane idle).  ~13 VALU for B = 4 instead of 4 x cu_half_sum's ~7.
template <int B>
__device__ __forceinline__ int lg_half_row(int p) {
  return B > 2 ? 2 * (p & 1) + ((p >> 1) & 1) : (p & 1);
}
template <int B>
__device__ __forceinline__ float lg_half_sum_rows(const float (&v)[B], int p) {
  static_assert(B >= 2 && B <= 4, "rows");
  const bool b0 = p & 1;
  float u;
  if constexpr (B == 2) {
    const float send = b0 ? v[0] : v[1], keep = b0 ? v[1] : v[0];
    u = keep + cu_dpp<0xB1>(send);          // quad_perm [1,0,3,2]: lane ^ 1
    u += cu_dpp<0x4E>(u);                   // lane ^ 2 (same row class)
  } else {
    const float v3 = B == 4 ? v[B - 1] : 0.f;
    const float s0 = b0 ? v[0] : v[2], s1 = b0 ? v[1] : v3;
    const float k0 = b0 ? v[2] : v[0], k1 = b0 ? v3 : v[1];
    const float u0 = k0 + cu_dpp<0xB1>(s0), u1 = k1 + cu_dpp<0xB1>(s1);
    const bool b1 = (p >> 1) & 1;
    const float send = b1 ? u0 : u1, keep = b1 ? u1 : u0;
    u = keep + cu_dpp<0x4E>(send);          // lane ^ 2
  }
  u += cu_dpp<0x124>(u);                    // row_ror:4 within 16 lanes (keeps lane & 3)
  u += cu_dpp<0x128>(u);                    // row_ror:8
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(u), __float_as_uint(u), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// the int8 weight codes of a Q6_K / Q5_K chunk (run 0 words, run 1 words) -- QDot::isums without the dots
template <int QT>
__device__ __forceinline__ void lg_codes(const RawChunk& r, int c, int (&lo)[4], int (&hi)[4]) {
  if constexpr (QT == QT_Q6_K) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo[i] = (int)QFmt<QT_Q6_K>::code_lo(r, i);
      hi[i] = (int)QFmt<QT_Q6_K>::code_hi(r, i);
    }
  } else {
    static_assert(QT == QT_Q5_K, "Q6_K / Q5_K only");
    const int g = (c & 7) >> 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t wv = u4_word(r.a, i), hv = u4_word(r.c, i);
      lo[i] = (int)((wv & 0x0f0f0f0fu) | (((hv >> (2 * g)) & 0x01010101u) << 4));
      hi[i] = (int)(((wv >> 4) & 0x0f0f0f0fu) | (((hv >> (2 * g + 1)) & 0x01010101u) << 4));
    }
  }
}

// one 64-chunk group of a row against B staged x rows (x read from LDS)
template <int QT, int B>
__device__ __forceinline__ void lg_compute_b(const RawChunk& raw, int it, int nch, const int8_t* xq, const float2* ms,
                                             float (&acc)[B]) {
  using F_ = QFmt<QT>;
  constexpr int W = F_::W, R = F_::RUNS;
  const int lane = threadIdx.x & 63;
  const int c0 = it * 64 + lane;
  const bool valid = c0 < nch;
  const int c = valid ? c0 : nch - 1;
  float sc[R], of[R];
  q8_scales_bf<QT>(raw, c, sc, of);
#pragma unroll
  for (int b = 0; b < B; ++b) {
    int xv[8];
    const int8_t* xc = xq + ((size_t)b * nch + c) * W;
    if constexpr (W == 32) {
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
    int is[R];
    QDot<QT>::isums(raw, c, xv, is);
#pragma unroll
    for (int rr = 0; rr < R; ++rr) {
      float2 m = ms[((size_t)b * nch + c) * R + rr];
      if (!valid) m = make_float2(0.f, 0.f);
      acc[b] += sc[rr] * m.x * (float)is[rr] - of[rr] * m.y;
    }
  }
}

// B = 1: the batch-1 decode engine; B = 2..4 (RSUB = 1: one ring slot fewer, the B staged x rows
// take its LDS): the same weight stream serves B rows -- the small-batch decode of the agent OS
// (<= 3 concurrent reasoning loops + agents) at close to the batch-1 step time
template <int QT0, int QT1, int B = 1, int RSUB = 0>
__global__ void __launch_bounds__(LG_THREADS) gemv_lds_b1(GemvArgs a, CuPlan pl) {
  static_assert(same_xlayout<QT0, QT1>, "mixed segments must share the activation layout");
  kernarg_warm<sizeof(GemvArgs) + sizeof(CuPlan)>();
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr bool MIXED = QT0 != QT1;
  constexpr int W = QFmt<QT0>::W, R = QFmt<QT0>::RUNS;
  const int nch = a.K / W;
  const int nit = nch >> 6;
  const int npairs = a.N >> 1;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool loader = wave >= LG_NG;
  unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  CU_STAMP(0);

  // ---- this workgroup's pair range (as gemv_cu_b1)
  const int g = blockIdx.x;
  const bool fmt1 = MIXED && g >= pl.g0;
  int pb, pe;
  if (!fmt1) {
    const int np = MIXED ? pl.np0 : npairs, G = MIXED ? pl.g0 : (int)gridDim.x;
    pb = (int)((long)g * np / G);
    pe = (int)((long)(g + 1) * np / G);
  } else {
    const int np = npairs - pl.np0, G = (int)gridDim.x - pl.g0, gg = g - pl.g0;
    pb = pl.np0 + (int)((long)gg * np / G);
    pe = pl.np0 + (int)((long)(gg + 1) * np / G);
  }
  if (pb >= pe) return;  // whole workgroup, before any barrier
  const int r0 = 2 * pb, nrows = 2 * (pe - pb);
  const int ngroups = nrows * nit;

  // ---- LDS: red[64] | rowacc[B][racc_n] | ms [B][nch][R] | xq [B][nch][W] | ring [LG_R][slot]
  float* red = smem;
  float* rowacc = smem + 64;
  float2* ms = (float2*)(rowacc + B * pl.racc_n);
  int8_t* xq = (int8_t*)(ms + (size_t)B * nch * R);
  // (offset arithmetic on the __shared__ base: a pointer cast through uintptr_t loses the LDS
  // address space and every ring read became a flat load waited with vmcnt)
  const int ring_off = (int)(((const uint8_t*)(xq + (size_t)B * a.K) - (const uint8_t*)smem + 255) & ~255);
  uint8_t* ring = (uint8_t*)smem + ring_off;
  for (int i = threadIdx.x; i < B * pl.racc_n; i += LG_THREADS) rowacc[i] = 0.f;
  if (threadIdx.x < 64) red[threadIdx.x] = 0.f;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ordered before B0

  // Loader and consumer paths are separate (no register merge between them: a phi of the
  // consumers' in-flight x registers made the compiler wait for them before the first barrier,
  // holding the loaders back).  Both execute the same T + 3 barriers.
  auto loader_path = [&](auto tag) __attribute__((always_inline)) {
    constexpr int QT = decltype(tag)::value;
    using L = LgLayout<QT, RSUB>;
    constexpr int PL = L::per_loader;
    constexpr int LG_R = L::R;
    const int T = (ngroups + L::NGS - 1) / L::NGS;
    const int lw = wave - LG_NG;
    // (an L2 prefetch of the slots past the ring -- one 4-B LDS-DMA per 128-B line, default
    // policy -- measured 25-30 % SLOWER on every shape, at any distance incl. the DMA'd slot
    // itself: the per-line requests double the CU's TA / L2 request count)
    if (LG_B0) lg_barrier();  // B0: the consumers' x loads are queued ahead of any weight byte
    const int npro = min(T, LG_R - 1);
    for (int s = 0; s < npro; ++s) lg_dma_slot<QT>(a, ring + (size_t)s * L::slot_bytes, s, lw, r0, nit, ngroups);
    if (npro == LG_R - 1) lg_vmcnt<(LG_R - 2) * PL>();
    else lg_vmcnt<0>();
    lg_barrier();  // B1: slot 0 landed, x staged
    for (int t = 0; t < T; ++t) {
      if (t + LG_R - 1 < T) {
        lg_dma_slot<QT>(a, ring + (size_t)((t + LG_R - 1) % LG_R) * L::slot_bytes, t + LG_R - 1, lw, r0, nit,
                        ngroups);
        lg_vmcnt<(LG_R - 2) * PL>();  // slot t + 1 landed
      } else {
        lg_vmcnt<0>();
      }
      lg_barrier();
    }
    lg_barrier();  // final
  };
  auto consumer_path = [&](auto tag, float2& rope, int& pos0, int& kv_blk0) __attribute__((always_inline)) {
    constexpr int QT = decltype(tag)::value;
    using L = LgLayout<QT, RSUB>;
    constexpr int LG_R = L::R;
    constexpr int GPW = L::GPW;
    const int T = (ngroups + L::NGS - 1) / L::NGS;
    constexpr int NPF = 2;
    StagePre<NPF> pf{};
    q8_stage_prefetch(a, pf, threadIdx.x, LG_NG * 64);
    if (LG_B0) lg_barrier();  // B0
    CU_STAMP(1);
    q8_stage<QT0, B, NPF>(a, xq, ms, red, pf, threadIdx.x, LG_NG * 64);
    // RoPE (cos, sin) of the epilogue lane's pair: issued now, waited for in the epilogue (the
    // consumers issue no other global load until then)
    if (B == 1 && a.epi == EPI_QKV && wave == 0) {
      // pos and the KV block too: a lookup after the final barrier put two dependent round trips
      // on the epilogue's path
      pos0 = a.pos[0];
      kv_blk0 = kv_block(a.block_table, a.max_ctx / KV_BLOCK, a.slot ? a.slot[0] : 0, pos0);
      if (a.rope_cs) {
        int part, head, lrr;
        qkv_part(a, a.row_base + r0 + 2 * lane, part, head, lrr);
        rope = a.rope_cs[(size_t)pos0 * (a.head_dim >> 1) + (part < 2 ? (lrr >> 1) : 0)];
      }
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    CU_STAMP(2);
    lg_barrier();  // B1
    CU_STAMP(3);
    if constexpr (B > 1) {
      if constexpr (QT == QT_Q4_K) {
        if (L::NGS % nit == 0) {
          // chunk pairs with B x-operand sets in registers (as the B = 1 path below)
          const int half = lane >> 5, p = lane & 31;
          const int kk = wave * GPW + half;
          Q4PairX X[B];
#pragma unroll
          for (int b = 0; b < B; ++b) q4p_load_x(xq + (size_t)b * a.K, ms + (size_t)b * nch * R, (kk % nit) * 64 + 2 * p, X[b]);
          const int rps = L::NGS / nit, rk = kk / nit;
          for (int t = 0; t < T; ++t) {
            if (t * L::NGS + wave * GPW < ngroups) {
              const uint8_t* slot = ring + (size_t)(t % LG_R) * L::slot_bytes;
              const uint4 a0 = *(const uint4*)(slot + L::off(0) + kk * 1024 + p * 32);
              const uint4 a1 = *(const uint4*)(slot + L::off(0) + kk * 1024 + p * 32 + 16);
              const uint4 mt = *(const uint4*)(slot + L::off(1) + kk * 128 + (p >> 2) * 16);
              const bool ok = t * L::NGS + kk < ngroups;
              float v[B];
              q4p_dot_b<B>(a0, a1, mt, p & 3, X, v);
              if (!ok) {
#pragma unroll
                for (int b = 0; b < B; ++b) v[b] = 0.f;
              }
              const float r = lg_half_sum_rows<B>(v, p);
              const int rb = lg_half_row<B>(p);
              if (p < (B > 2 ? 4 : 2) && rb < B && ok)  // one LDS atomic instruction for all B rows
                __hip_atomic_fetch_add(&rowacc[rb * pl.racc_n + t * rps + rk], r, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            lg_barrier();
          }
          CU_STAMP(4);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          lg_barrier();  // final
          CU_STAMP(5);
          return;
        }
      } else if constexpr (GPW == 1 && QFmt<QT>::W == 32) {
        if (L::NGS % nit == 0) {
          // Q6_K / Q5_K (the Q4_K_M down projection and lm_head): one group per wave per slot, the same K
          // columns in every slot, so the B rows' x stay in registers (as the B = 1 path below); the
          // scale decode is shared, the rows' partials fold with one butterfly + a 32-lane swap
          const int c = (wave % nit) * 64 + lane;
          int xv[B][8];
          float4 m[B];
#pragma unroll
          for (int b = 0; b < B; ++b) {
            const int8_t* xc = xq + ((size_t)b * nch + c) * 32;
            const int rot = (c >> 3) & 1;
            const uint4 p0 = *(const uint4*)(xc + 16 * rot), p1 = *(const uint4*)(xc + 16 * (rot ^ 1));
            xv[b][0] = p0.x; xv[b][1] = p0.y; xv[b][2] = p0.z; xv[b][3] = p0.w;
            xv[b][4] = p1.x; xv[b][5] = p1.y; xv[b][6] = p1.z; xv[b][7] = p1.w;
            m[b] = *(const float4*)(ms + ((size_t)b * nch + c) * 2);
          }
          const int rps = L::NGS / nit, rk = wave / nit;
          for (int t = 0; t < T; ++t) {
            if (t * L::NGS + wave < ngroups) {
              const uint8_t* slot = ring + (size_t)(t % LG_R) * L::slot_bytes;
              RawChunk raw;
              lg_read<QT>(slot, wave, lane, raw);
              float sc[2], of[2];
              q8_scales_bf<QT>(raw, c, sc, of);
              // the weight codes once, then the B rows' integer dots (isums per row would decode them B times)
              int lo[4], hi[4];
              lg_codes<QT>(raw, c, lo, hi);
              float v[B];
#pragma unroll
              for (int b = 0; b < B; ++b) {
                int s0 = 0, s1 = 0;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                  s0 = __builtin_amdgcn_sdot4(lo[i], xv[b][i], s0, false);
                  s1 = __builtin_amdgcn_sdot4(hi[i], xv[b][4 + i], s1, false);
                }
                v[b] = sc[0] * m[b].x * (float)s0 - of[0] * m[b].y + sc[1] * m[b].z * (float)s1 - of[1] * m[b].w;
              }
              float r = lg_half_sum_rows<B>(v, lane & 31);
              const auto h = __builtin_amdgcn_permlane32_swap(__float_as_uint(r), __float_as_uint(r), false, false);
              r = __uint_as_float(h[0]) + __uint_as_float(h[1]);  // both 32-lane halves
              const int rb = lg_half_row<B>(lane & 31);
              if (lane < (B > 2 ? 4 : 2) && rb < B)
                __hip_atomic_fetch_add(&rowacc[rb * pl.racc_n + t * rps + rk], r, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
            }
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            lg_barrier();
          }
          CU_STAMP(4);
          lg_barrier();  // final
          CU_STAMP(5);
          return;
        }
      }
      for (int t = 0; t < T; ++t) {
        const int gb = t * L::NGS + wave * GPW;
        if (gb < ngroups) {
          const uint8_t* slot = ring + (size_t)(t % LG_R) * L::slot_bytes;
          RawChunk raw[GPW];
          static_for<GPW>([&](auto j) { lg_read<QT>(slot, wave * GPW + j, lane, raw[j]); });
          int row = gb / nit, it = gb - row * nit;
          float acc[B];
#pragma unroll
          for (int b = 0; b < B; ++b) acc[b] = 0.f;
          static_for<GPW>([&](auto j) {
            const int gg = gb + j;
            if (gg < ngroups) {
              lg_compute_b<QT, B>(raw[j], it, nch, xq, ms, acc);
              if (it == nit - 1 || j == GPW - 1 || gg == ngroups - 1) {
#pragma unroll
                for (int b = 0; b < B; ++b) {
                  const float v = cu_wave_sum(acc[b]);
                  if (lane == 0) atomicAdd(&rowacc[b * pl.racc_n + row], v);
                  acc[b] = 0.f;
                }
              }
            }
            if (++it == nit) { it = 0; ++row; }
          });
        }
        lg_barrier();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      lg_barrier();  // final
      return;
    }
    if constexpr (QT == QT_Q4_K) {
      if (L::NGS % nit == 0) {
        // chunk pairs, x in registers (gemv_cu.h Q4PairX): lanes 0-31 take group 2w's 32 pairs,
        // lanes 32-63 group 2w+1's; every slot holds NGS / nit whole rows
        const int half = lane >> 5, p = lane & 31;
        const int kk = wave * GPW + half;
        Q4PairX X;
        q4p_load_x(xq, ms, (kk % nit) * 64 + 2 * p, X);
        const int rps = L::NGS / nit, rk = kk / nit;
        for (int t = 0; t < T; ++t) {
          if (t * L::NGS + wave * GPW < ngroups) {
            const uint8_t* slot = ring + (size_t)(t % LG_R) * L::slot_bytes;
            if (AIOS_GEMV_PROBES && (a.tune_dbg & LG_DBG_RING)) { lg_barrier(); continue; }  // probe builds only
            const uint4 a0 = *(const uint4*)(slot + L::off(0) + kk * 1024 + p * 32);
            const uint4 a1 = *(const uint4*)(slot + L::off(0) + kk * 1024 + p * 32 + 16);
            const uint4 mt = *(const uint4*)(slot + L::off(1) + kk * 128 + (p >> 2) * 16);
            const bool ok = t * L::NGS + kk < ngroups;
            const float v = cu_half_sum(ok ? q4p_dot(a0, a1, mt, p & 3, X) : 0.f);
            if (p == 0 && ok)
              __hip_atomic_fetch_add(&rowacc[t * rps + rk], v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          lg_barrier();
        }
        CU_STAMP(4);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        lg_barrier();  // final
        CU_STAMP(5);
        return;
      }
    } else if constexpr (GPW == 1 && QFmt<QT>::W == 32) {
      if (L::NGS % nit == 0) {
        // one group per wave per slot, the same K columns in every slot: x in registers
        const int c = (wave % nit) * 64 + lane;
        int xv[8];
        const int8_t* xc = xq + (size_t)c * 32;
        const int rot = (c >> 3) & 1;
        const uint4 p0 = *(const uint4*)(xc + 16 * rot), p1 = *(const uint4*)(xc + 16 * (rot ^ 1));
        xv[0] = p0.x; xv[1] = p0.y; xv[2] = p0.z; xv[3] = p0.w;
        xv[4] = p1.x; xv[5] = p1.y; xv[6] = p1.z; xv[7] = p1.w;
        const float4 m = *(const float4*)(ms + (size_t)c * 2);
        const int rps = L::NGS / nit, rk = wave / nit;
        for (int t = 0; t < T; ++t) {
          if (t * L::NGS + wave < ngroups) {
            const uint8_t* slot = ring + (size_t)(t % LG_R) * L::slot_bytes;
            RawChunk raw;
            lg_read<QT>(slot, wave, lane, raw);
            float sc[2], of[2];
            q8_scales_bf<QT>(raw, c, sc, of);
            int is[2];
            QDot<QT>::isums(raw, c, xv, is);
            const float v = cu_wave_sum(sc[0] * m.x * (float)is[0] - of[0] * m.y + sc[1] * m.z * (float)is[1] - of[1] * m.w);
            if (lane == 0) atomicAdd(&rowacc[t * rps + rk], v);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          lg_barrier();
        }
        CU_STAMP(4);
        lg_barrier();  // final
        CU_STAMP(5);
        return;
      }
    }
    for (int t = 0; t < T; ++t) {
      const int gb = t * L::NGS + wave * GPW;  // this wave's first group of the slot
      if (gb < ngroups) {
        const uint8_t* slot = ring + (size_t)(t % LG_R) * L::slot_bytes;
        RawChunk raw[GPW];
        static_for<GPW>([&](auto j) { lg_read<QT>(slot, wave * GPW + j, lane, raw[j]); });
        int row = gb / nit, it = gb - row * nit;
        float acc = 0.f;
        static_for<GPW>([&](auto j) {
          const int gg = gb + j;
          if (gg < ngroups) {
            cu_compute<QT>(raw[j], it, nch, xq, ms, acc);
            // one row sum per row this wave finished or leaves in this step
            if (it == nit - 1 || j == GPW - 1 || gg == ngroups - 1) {
              const float v = cu_wave_sum(acc);
              if (lane == 0) atomicAdd(&rowacc[row], v);
              acc = 0.f;
            }
          }
          if (++it == nit) { it = 0; ++row; }
        });
      }
      lg_barrier();
    }
    CU_STAMP(4);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    lg_barrier();  // final: every row sum is in rowacc
    CU_STAMP(5);
  };
  float2 rope = make_float2(1.f, 0.f);
  int pos0 = 0, kv_blk0 = 0;
  if (loader) {
    if (!fmt1) loader_path(FmtTag<QT0>{});
    else loader_path(FmtTag<QT1>{});
    return;
  }
  if (!fmt1) consumer_path(FmtTag<QT0>{}, rope, pos0, kv_blk0);
  else consumer_path(FmtTag<QT1>{}, rope, pos0, kv_blk0);
  auto flush_ts = [&]() {
    if (a.dbg_ts && lane == 0 && (wave == 0 || wave == LG_NG - 1))
      for (int i = 0; i < 8; ++i) a.dbg_ts[((size_t)blockIdx.x * 2 + (wave != 0)) * 8 + i] = ts[i];
  };
  if (wave != 0) {
    flush_ts();
    return;
  }

  if constexpr (B > 1) {
    // ---- batched epilogues: wave 0, one lane per (row b, pair)
    float sb[B];
#pragma unroll
    for (int b = 0; b < B; ++b) {
      sb[b] = 1.f;
      if (a.norm_w) {
        float t = 0.f;
#pragma unroll
        for (int w = 0; w < LG_NG; ++w) t += red[w * B + b];
        sb[b] = rsqrtf(t / (float)a.K + a.eps);
      }
    }
    const int npl = nrows >> 1;
    for (int i = lane; i < a.B * npl; i += 64) {
      const int b = i / npl, p = i - b * npl;
      float s_ = sb[0];
#pragma unroll
      for (int bb = 1; bb < B; ++bb)
        if (b == bb) s_ = sb[bb];
      gemv_epilogue(a, a.row_base + r0 + 2 * p, b, rowacc[b * pl.racc_n + 2 * p] * s_,
                    rowacc[b * pl.racc_n + 2 * p + 1] * s_);
    }
    CU_STAMP(6);
    flush_ts();
    return;
  }
  // ---- pair epilogues: wave 0, one lane per pair
  float s = 1.f;
  if (a.norm_w) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < LG_NG; ++w) t += red[w];
    s = rsqrtf(t / (float)a.K + a.eps);
  }
  for (int p = lane; 2 * p < nrows; p += 64) {
    const int grow = a.row_base + r0 + 2 * p;
    const float v0 = rowacc[2 * p] * s, v1 = rowacc[2 * p + 1] * s;
    if (a.epi == EPI_QKV) {
      float2 t = rope;
      if (p >= 64 || !a.rope_cs) {
        int part, head, lrr;
        qkv_part(a, grow, part, head, lrr);
        const int pp = lrr >> 1;
        if (a.rope_cs) {
          t = a.rope_cs[(size_t)pos0 * (a.head_dim >> 1) + pp];
        } else {
          float sn, cs;
          sincosf((float)pos0 * powf(a.rope_base, -2.f * (float)pp / (float)a.head_dim), &sn, &cs);
          t = make_float2(cs, sn);
        }
      }
      cu_qkv_epilogue(a, grow, v0, v1, t, pos0, kv_blk0);
    } else {
      gemv_epilogue1(a, grow, v0, v1);
    }
  }
  CU_STAMP(6);
  flush_ts();
}

template <int QT>
constexpr bool lg_supported() {
  return QT == QT_Q4_K || QT == QT_Q5_K || QT == QT_Q6_K || QT == QT_Q4_0 || QT == QT_Q8_0;
}

// returns false when the shape does not fit (then the register kernels run)
template <int QT0, int QT1, int B, int RSUB>
size_t lg_lds_bytes(const GemvArgs& a, const CuPlan& pl) {
  constexpr int W = QFmt<QT0>::W, R = QFmt<QT0>::RUNS;
  const int nch = a.K / W;
  const size_t head = (64 + (size_t)B * pl.racc_n) * 4 + (size_t)B * nch * R * 8 + (size_t)B * a.K;
  const size_t ringb = std::max(LgLayout<QT0, RSUB>::R * LgLayout<QT0, RSUB>::slot_bytes,
                                LgLayout<QT1, RSUB>::R * LgLayout<QT1, RSUB>::slot_bytes);
  return (head + 255) / 256 * 256 + ringb;
}

// dry = true: only whether the engine WOULD serve these args (the engine's per-B path choice)
template <int QT0, int QT1>
bool launch_gemv_lds(const GemvArgs& a, hipStream_t st, bool dry = false) {
  if constexpr (!same_xlayout<QT0, QT1> || !lg_supported<QT0>() || !lg_supported<QT1>()) {
    return false;
  } else {
    // AIOS_GEMV_LDS: 0 = off, 1 = projections >= 96 KB per CU (default), 2 = every shape
    static const int mode = [] {
      const char* e = std::getenv("AIOS_GEMV_LDS");
      return e ? std::atoi(e) : 1;
    }();
    // AIOS_GEMV_LDS_MAXB: batch rows the engine serves (1..4, default 4; whether B = 3 / 4 decode takes this path or the skinny MFMA GEMM is the
    // engine's dec_gemm_min_b_, profiles/lds_batched_r3.txt)
    static const int maxb = [] {
      const char* e = std::getenv("AIOS_GEMV_LDS_MAXB");
      return e ? std::max(1, std::min(4, std::atoi(e))) : 4;
    }();
    // (tune_dbg LG_DBG_RING: the probe's ring-only mode; every other microbenchmark bit -> row kernels)
    if (!mode || a.B < 1 || a.B > (a.kernel_sel == 3 ? 4 : maxb) || (a.tune_dbg & ~LG_DBG_RING) ||
        (a.kernel_sel != 0 && a.kernel_sel != 3))
      return false;
    constexpr int W = QFmt<QT0>::W, R = QFmt<QT0>::RUNS;
    const int nch = a.K / W;
    if (nch % 64) return false;
    const int npairs = a.N / 2;
    const int G = std::min(a.tune_grid > 0 ? a.tune_grid : device_cu_count(), npairs);
    auto rup = [](int n, int g) { return (n + g - 1) / g; };
    CuPlan pl{G, npairs, (2 * rup(npairs, G) + 3) & ~3};
    if (QT0 != QT1 && a.nseg > 1) {
      const int np0 = a.seg_row0[a.nseg - 1] / 2;
      if (G < 2 || np0 < 1 || np0 >= npairs) return false;
      const double b0 = (double)np0 * cu_fmt_bytes_per_256(QT0), b1 = (double)(npairs - np0) * cu_fmt_bytes_per_256(QT1);
      int g0 = (int)(G * b0 / (b0 + b1) + 0.5);
      g0 = std::max(1, std::min(G - 1, g0));
      const int most = std::max(rup(np0, g0), rup(npairs - np0, G - g0));
      pl = CuPlan{g0, np0, (2 * most + 3) & ~3};
    }
    // small projections (O: <= ~40 KB per CU) stay on the row-pair kernel: the engine's fixed
    // start-up (first slot lands ~3-4 us after issue, behind the CU's whole prologue burst) and its
    // barrier steps cost more than the row kernel's x-staging stall there (tools/gemv_cu_probe.py:
    // O 6.96 vs 5.60 us, QKV 8.73 vs 8.38; gate_up 17.35 vs 19.39, down 13.8 vs 15.2, lm_head 24.8
    // vs 25.9).  AIOS_GEMV_LDS=2 forces the engine for every shape.
    // batched launches (B >= 2) take the engine for every shape: the row-pair kernels re-read the
    // B x vectors per wave and measured 2-3x slower there (B = 2 QKV 26 us vs 9.6 at B = 1)
    if (mode != 2 && a.kernel_sel != 3 && a.B == 1) {
      // AIOS_GEMV_LDS_MIN_KB: per-CU weight bytes from which the engine serves a shape.  Round 5
      // (same box, tools/ab.sh): 40 instead of 96 -- the Mistral QKV (59 KB per CU) and the
      // TinyLlama gate/up (50 KB) move to the engine: Mistral 668.2 / 668.1 -> 672.6 / 671.5 tok/s,
      // TinyLlama 1500.7 / 1500.5 -> 1530.8 / 1535.3 (O, 37 KB, stays on the row kernel)
      static const double min_kb = [] {
        const char* e = std::getenv("AIOS_GEMV_LDS_MIN_KB");
        return e ? std::atof(e) : 40.0;
      }();
      double bytes = 0;
      for (int sg = 0; sg < a.nseg; ++sg)
        bytes += (double)a.seg[sg].rows * a.K / 256.0 * cu_fmt_bytes_per_256(a.seg[sg].qtype);
      if (bytes / G < min_kb * 1024) return false;
    }
    constexpr size_t LDS_MAX = 160 * 1024;
    size_t lds = 0;
    if (a.B == 1) {
      // AIOS_LDS_B1_RSUB (default 1): ring slots fewer than LgLayout's depth at batch 1.  A smaller
      // prologue burst (~64 instead of ~96 KB per CU, 16 MB chip-wide) lands the first slot sooner,
      // and R - 1 slots in flight still cover the stream's latency: 649.4 -> 662.9 tok/s same box
      // (tools/gpu_r4_ab5.sh, profiles/decode_mistral_rocprof_r4_final.txt)
      static const int rsub_all = [] {
        const char* e = std::getenv("AIOS_LDS_B1_RSUB");
        return e ? std::atoi(e) : 1;
      }();
      // AIOS_LDS_B1_RSUB_Q6: Q6_K matrices' own value (default 2: their 23.5 KB slots cover the latency with
      // one slot fewer still -- Mistral B=1 670.7 / 670.9 -> 672.6 / 672.0 tok/s, profiles/decode_b1_experiments_r6.txt)
      static const int rsub_q6 = [] {
        const char* e = std::getenv("AIOS_LDS_B1_RSUB_Q6");
        return e ? std::atoi(e) : 2;
      }();
      const int rsub = (QT0 == QT_Q6_K && rsub_q6 >= 0) ? rsub_q6 : rsub_all;
      if (rsub == 1 || rsub == 2) {
        if (rsub == 1) lds = lg_lds_bytes<QT0, QT1, 1, 1>(a, pl);
        else lds = lg_lds_bytes<QT0, QT1, 1, 2>(a, pl);
        if (lds > LDS_MAX) return false;
        if (dry) return true;
        if (rsub == 1) hipLaunchKernelGGL((gemv_lds_b1<QT0, QT1, 1, 1>), dim3(G), dim3(LG_THREADS), lds, st, a, pl);
        else hipLaunchKernelGGL((gemv_lds_b1<QT0, QT1, 1, 2>), dim3(G), dim3(LG_THREADS), lds, st, a, pl);
        return true;
      }
      lds = lg_lds_bytes<QT0, QT1, 1, 0>(a, pl);
      if (lds > LDS_MAX) return false;
      if (dry) return true;
      hipLaunchKernelGGL((gemv_lds_b1<QT0, QT1, 1, 0>), dim3(G), dim3(LG_THREADS), lds, st, a, pl);
    } else if (a.B == 2) {
      lds = lg_lds_bytes<QT0, QT1, 2, 1>(a, pl);
      if (lds > LDS_MAX) return false;
      if (dry) return true;
      hipLaunchKernelGGL((gemv_lds_b1<QT0, QT1, 2, 1>), dim3(G), dim3(LG_THREADS), lds, st, a, pl);
    } else if (a.B == 3) {  // its own instantiation: no idle fourth row in the dot work / staging
      if ((lds = lg_lds_bytes<QT0, QT1, 3, 1>(a, pl)) <= LDS_MAX) {
        if (dry) return true;
        hipLaunchKernelGGL((gemv_lds_b1<QT0, QT1, 3, 1>), dim3(G), dim3(LG_THREADS), lds, st, a, pl);
      } else {
        lds = lg_lds_bytes<QT0, QT1, 3, 2>(a, pl);
        if (lds > LDS_MAX) return false;
        if (dry) return true;
        hipLaunchKernelGGL((gemv_lds_b1<QT0, QT1, 3, 2>), dim3(G), dim3(LG_THREADS), lds, st, a, pl);
      }
    } else if ((lds = lg_lds_bytes<QT0, QT1, 4, 1>(a, pl)) <= LDS_MAX) {
      if (dry) return true;
      hipLaunchKernelGGL((gemv_lds_b1<QT0, QT1, 4, 1>), dim3(G), dim3(LG_THREADS), lds, st, a, pl);
    } else {
      // long K (the d_ff-wide down projection): four staged x rows leave room for a shallower ring
      lds = lg_lds_bytes<QT0, QT1, 4, 2>(a, pl);
      if (lds > LDS_MAX) return false;
      if (dry) return true;
      hipLaunchKernelGGL((gemv_lds_b1<QT0, QT1, 4, 2>), dim3(G), dim3(LG_THREADS), lds, st, a, pl);
    }
    return true;
  }
}
