// CU-balanced batch-1 decode GEMV (int8 activations), included by gemv_impl.h after gemv_q8.h.
//
// Why a second B = 1 kernel: a decode projection is 9-108 MB streamed once, and on MI355X one CU
// moves at most ~24 GB/s (MI355X_MICROARCH.md, 'global_load_dwordx4 (HBM-bound) ~10 B/cyc/CU'), so
// the chip reaches its ~6.2 TB/s only when all 256 CUs carry the SAME byte count.  gemv_q8_rows
// deals row pairs to waves grid-stride, which leaves whole CUs with 2x the bytes of others on the
// small projections (QKV: 384 workgroups over 256 CUs) -- measured 1.3-1.7 TB/s on QKV / O against
// a 3.8 TB/s streaming-read floor for the same bytes (profiles/stream_floor_r2.txt).
//
// Decomposition: exactly one 1024-thread workgroup per CU (LDS sized so a second cannot fit), each
// owning a contiguous range of row pairs; the 16 waves split that range's (row, 64-chunk item) list
// evenly, so every CU streams the same bytes and every wave the same number of 1 KB loads.  A mixed
// Q4_K_M QKV (V in Q6_K) gives each format a share of the CUs proportional to its bytes.
// A wave issues all loads of up to DMAX items at once (the small projections: every byte of the
// CU's share in flight from the start, x staged meanwhile); each chunk is a static case so the
// compiler's counted vmcnt waits are exact (cu_body).  Row partials are wave-reduced with
// DPP / permlane swaps and summed into an LDS row accumulator (ds_add_f32: rows may straddle two
// waves); after one barrier a single wave runs the pair epilogues (store / residual / SwiGLU /
// RoPE + KV write) with no global load left on the path (the RoPE (cos, sin) of each epilogue lane
// is fetched right behind the first weight loads).
#pragma once
// (included inside namespace aios by gemv_impl.h)

constexpr int CU_WAVES = 16;
constexpr int CU_THREADS = CU_WAVES * 64;

struct CuPlan {
  int g0;      // workgroups serving format-0 pairs [0, np0)
  int np0;     // pairs of format 0; pairs [np0, N/2) use the last segment's format
  int racc_n;  // LDS row accumulators: 2 x the most pairs any workgroup owns, rounded to 4
};

template <int CTRL>
__device__ __forceinline__ float cu_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
// sum over the 64 lanes, result in every lane: quad / half-row / row DPP, then permlane swaps
__device__ __forceinline__ float cu_wave_sum(float v) {
  v += cu_dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += cu_dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += cu_dpp<0x141>(v);  // row_half_mirror
  v += cu_dpp<0x140>(v);  // row_mirror
  {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  }
  return v;
}

// sum over each 32-lane half (lanes 0-31 / 32-63), result in every lane of the half
__device__ __forceinline__ float cu_half_sum(float v) {
  v += cu_dpp<0xB1>(v);
  v += cu_dpp<0x4E>(v);
  v += cu_dpp<0x141>(v);
  v += cu_dpp<0x140>(v);
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// ---------------------------------------------------------------------------------------------
// Q4_K chunk PAIRS with the activation operand in registers (batch-1 ring consumers).
//
// Chunks 2p and 2p+1 of a row hold the two 16-halves of one sub-block pair g = p & 3 of
// superblock p >> 2: they share the scale/min decode, and run r of both is ONE 32-element int8 x
// block (one dx), so both chunks' integer dot products add before the float scaling.  A lane
// that takes a pair spends ~64 VALU per 64 weights against ~75 per 32 for one chunk with its x
// read from LDS (measured issue-bound: gate_up's 8 ring slots per CU computed in 11 us of a 17 us
// kernel, tools/mk_probe.py --dbg 2).  When every slot holds whole rows (NGS % groups-per-row
// == 0) a wave's lanes see the same K columns in every slot, so x is loaded once per GEMV.
// ---------------------------------------------------------------------------------------------
struct Q4PairX {
  int x0[8], x1[8];          // run 0 / run 1 codes: chunk 2p's 4 words, then chunk 2p+1's
  float dx0, dx1, sx0, sx1;  // block scales; dx * code sums over both chunks' runs
};

// c0: the pair's first chunk (even) within the row, staged by q8_stage (x in QT_Q4_K order)
__device__ __forceinline__ void q4p_load_x(const int8_t* xq, const float2* ms, int c0, Q4PairX& X) {
  const int rot = (c0 >> 3) & 1;  // the staging swizzle (q8_octet): run r at 16 * (r ^ rot)
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int8_t* xc = xq + (size_t)(c0 + h) * 32;
    const uint4 p0 = *(const uint4*)(xc + 16 * rot);
    const uint4 p1 = *(const uint4*)(xc + 16 * (rot ^ 1));
    X.x0[4 * h + 0] = p0.x; X.x0[4 * h + 1] = p0.y; X.x0[4 * h + 2] = p0.z; X.x0[4 * h + 3] = p0.w;
    X.x1[4 * h + 0] = p1.x; X.x1[4 * h + 1] = p1.y; X.x1[4 * h + 2] = p1.z; X.x1[4 * h + 3] = p1.w;
  }
  const float4 m0 = *(const float4*)(ms + (size_t)c0 * 2);      // (dx, sx) of runs 0, 1 of chunk 2p
  const float4 m1 = *(const float4*)(ms + (size_t)c0 * 2 + 2);  // ... of chunk 2p+1
  X.dx0 = m0.x;
  X.dx1 = m0.z;
  X.sx0 = m0.y + m1.y;
  X.sx1 = m0.w + m1.w;
}

// a0 / a1: the pair's two 16-B code chunks, mt: its superblock's repacked meta, g = p & 3
__device__ __forceinline__ float q4p_dot(const uint4& a0, const uint4& a1, const uint4& mt, int g, const Q4PairX& X) {
  const float d = __half2float(__ushort_as_half((uint16_t)(mt.x & 0xffff)));
  const float dmin = __half2float(__ushort_as_half((uint16_t)(mt.x >> 16)));
  const uint32_t f = kq_field(mt.y, mt.z, mt.w, g);
  int s0 = 0, s1 = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t w = u4_word(a0, i);
    s0 = __builtin_amdgcn_sdot4((int)(w & 0x0f0f0f0fu), X.x0[i], s0, false);
    s1 = __builtin_amdgcn_sdot4((int)((w >> 4) & 0x0f0f0f0fu), X.x1[i], s1, false);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const uint32_t w = u4_word(a1, i);
    s0 = __builtin_amdgcn_sdot4((int)(w & 0x0f0f0f0fu), X.x0[4 + i], s0, false);
    s1 = __builtin_amdgcn_sdot4((int)((w >> 4) & 0x0f0f0f0fu), X.x1[4 + i], s1, false);
  }
  const float u = (float)(f & 63) * X.dx0 * (float)s0 + (float)((f >> 6) & 63) * X.dx1 * (float)s1;
  const float o = (float)((f >> 12) & 63) * X.sx0 + (float)((f >> 18) & 63) * X.sx1;
  return d * u - dmin * o;
}

// one 64-chunk item (chunk c = it * 64 + lane) of a row against the staged int8 x
template <int QT>
__device__ __forceinline__ void cu_compute(const RawChunk& raw, int it, int nch, const int8_t* xq,
                                           const float2* ms, float& acc) {
  using F_ = QFmt<QT>;
  constexpr int W = F_::W, R = F_::RUNS;
  const int lane = threadIdx.x & 63;
  const int c0 = it * 64 + lane;
  const bool valid = c0 < nch;
  const int c = valid ? c0 : nch - 1;
  float sc[R], of[R];
  q8_scales_bf<QT>(raw, c, sc, of);
  int xv[8];
  const int8_t* xc = xq + (size_t)c * W;
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
  float2 m[R];
#pragma unroll
  for (int rr = 0; rr < R; ++rr) {
    const float2 t = ms[(size_t)c * R + rr];  // unconditional LDS read, then a select (no branch)
    m[rr] = valid ? t : make_float2(0.f, 0.f);
  }
  int is[R];
  QDot<QT>::isums(raw, c, xv, is);
#pragma unroll
  for (int rr = 0; rr < R; ++rr) acc += sc[rr] * m[rr].x * (float)is[rr] - of[rr] * m[rr].y;
}

// (+bias) RoPE on a Q/K pair with its (cos, sin) = t, Q -> y, K/V -> the bf16 paged KV cache
__device__ __forceinline__ void cu_qkv_epilogue(const GemvArgs& a, int grow, float v0, float v1, float2 t, int pos0,
                                                int kv_blk0) {
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
    const float o0 = v0 * t.x - v1 * t.y, o1 = v0 * t.y + v1 * t.x;
    v0 = o0;
    v1 = o1;
  }
  if (part == 0) {
    float* q = a.y + head * hd;
    q[da] = v0;
    q[db] = v1;
  } else {
    bf16_t* cache = pick_ptr(part == 1, a.k_cache, a.v_cache);
    const size_t base = (((size_t)kv_blk0 * a.n_kv_heads + head) * KV_BLOCK + (pos0 % KV_BLOCK)) * hd;
    kv_store_pair(cache, base + da, base + db, v0, v1, a.kv_fp8, part == 1 ? a.kv_inv_k : a.kv_inv_v);
  }
}

// probes (tools/gemv_cu_probe.py): phase timestamps of waves 0 and 15 of every workgroup, held in
// `ts` and flushed at the end (the engine has SGPRs to spare: stamps stored as taken -- what the row
// GEMV now does -- measured 0.2-0.6 us slower per engine launch, profiles/decode_tinyllama_rocprof_r4.txt)
#define CU_STAMP(i)                                                   \
  do {                                                                \
    if (AIOS_GEMV_PROBES && a.dbg_ts) ts[i] = __builtin_amdgcn_s_memrealtime();  \
  } while (0)

// f(integral_constant<I>) for the run-time n in [0, N]: every case is a fully static body
template <int N, int I = 0, typename F>
__device__ __forceinline__ void cu_dispatch(int n, F&& f) {
  if constexpr (I <= N) {
    if (n == I) f(std::integral_constant<int, I>{});
    else cu_dispatch<N, I + 1>(n, f);
  }
}

// Per-workgroup body for one weight format QT (the activation layout is QTX's); every thread of
// the workgroup runs it.  A wave's items are taken in chunks of at most DMAX; each chunk is one
// static case (its item count a compile-time constant) that issues exactly its own loads and
// computes them, so the compiler's counted vmcnt waits are exact and no load is ever issued for an
// item that does not exist (out-of-range buffer loads still cost TA cycles: measured 1.5-2x slower
// decode with a fixed-depth ring padded by such loads).  The first chunk also stages x between
// issuing its loads and computing them.  Row sums land in rowacc.
template <int QT, int QTX, int DMAX>
__device__ __forceinline__ void cu_body(const GemvArgs& a, int r0, int j0, int j1, int nit, int nch, float* red,
                                        float* rowacc, float2* ms, int8_t* xq, float2& rope,
                                        unsigned long long* ts) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  auto load_item = [&](int row, int it, RawChunk& r) __attribute__((always_inline)) {
    int s = 0;
#pragma unroll
    for (int k = 1; k < GEMV_MAX_SEGS; ++k)
      if (k < a.nseg && row >= a.seg_row0[k]) s = k;
    const int lrow = row - (s == 0 ? 0 : (s == 1 ? a.seg_row0[1] : a.seg_row0[2]));
    q8_load<QT>(seg_rsrc(a, s), lrow, min(it * 64 + lane, nch - 1), r);
  };
  float acc = 0.f;
  auto chunk = [&](auto NC, auto FIRST, int jb) __attribute__((always_inline)) {
    constexpr int N = decltype(NC)::value;
    constexpr bool first = decltype(FIRST)::value;
    constexpr int NPF = 2;  // x octets prefetched per thread: K <= 16384 at 1024 threads
    StagePre<NPF> pf{};
    if constexpr (first) q8_stage_prefetch(a, pf);  // x first: its wait does not cover the weights
    RawChunk ring[N > 0 ? N : 1];
    const int row0 = r0 + jb / nit, it0 = jb - (row0 - r0) * nit;
    {
      int lr = row0, li = it0;
      static_for<N>([&](auto k) {
        load_item(lr, li, ring[k]);
        if (++li == nit) { li = 0; ++lr; }
      });
    }
    if constexpr (first) CU_STAMP(1);
    if constexpr (first) {
      // RoPE (cos, sin) of the epilogue lane's pair (wave 0): behind the first weight loads,
      // waited for only in the epilogue
      if (a.epi == EPI_QKV && wave == 0) {
        const int pos0 = a.pos[0];
        const int p = r0 / 2 + lane;
        int part, head, lrr;
        qkv_part(a, a.row_base + 2 * p, part, head, lrr);
        const int pp = lrr >> 1;
        if (a.rope_cs && part < 2) rope = a.rope_cs[(size_t)pos0 * (a.head_dim >> 1) + pp];
      }
      q8_stage<QTX, 1, NPF>(a, xq, ms, red, pf);
      CU_STAMP(2);
      __syncthreads();
      CU_STAMP(3);
    }
    int cr = row0, ci = it0;
    static_for<N>([&](auto k) {
      cu_compute<QT>(ring[k], ci, nch, xq, ms, acc);
      if (ci == nit - 1 || jb + (int)k == j1 - 1) {
        const float v = cu_wave_sum(acc);
        if (lane == 0) atomicAdd(&rowacc[cr - r0], v);
        acc = 0.f;
      }
      if (++ci == nit) { ci = 0; ++cr; }
    });
  };
  cu_dispatch<DMAX>(min(DMAX, j1 - j0), [&](auto NC) { chunk(NC, std::true_type{}, j0); });
  for (int jb = j0 + DMAX; jb < j1; jb += DMAX)
    cu_dispatch<DMAX>(min(DMAX, j1 - jb), [&](auto NC) { chunk(NC, std::false_type{}, jb); });
  CU_STAMP(4);
}

template <int QT0, int QT1, int D>
__global__ void __launch_bounds__(CU_THREADS) gemv_cu_b1(GemvArgs a, CuPlan pl) {
  static_assert(same_xlayout<QT0, QT1>, "mixed segments must share the activation layout");
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr bool MIXED = QT0 != QT1;
  constexpr int W = QFmt<QT0>::W, R = QFmt<QT0>::RUNS;
  const int nch = a.K / W;
  const int nit = (nch + 63) >> 6;
  const int npairs = a.N >> 1;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  unsigned long long ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  CU_STAMP(0);
  auto flush_ts = [&]() {
    if (a.dbg_ts && lane == 0 && (wave == 0 || wave == CU_WAVES - 1))
      for (int i = 0; i < 8; ++i) a.dbg_ts[((size_t)blockIdx.x * 2 + (wave != 0)) * 8 + i] = ts[i];
  };

  // ---- this workgroup's pair range
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
  const int items = nrows * nit;
  const int ipw = (items + CU_WAVES - 1) / CU_WAVES;
  const int j0 = __builtin_amdgcn_readfirstlane(min(items, wave * ipw));
  const int j1 = __builtin_amdgcn_readfirstlane(min(items, j0 + ipw));

  // ---- LDS: red[64] | rowacc[racc_n] | ms [nch][R] | xq [nch][W]
  float* red = smem;
  float* rowacc = smem + 64;
  const int racc_n = pl.racc_n;
  float2* ms = (float2*)(rowacc + racc_n);
  int8_t* xq = (int8_t*)(ms + (size_t)nch * R);
  for (int i = threadIdx.x; i < nrows; i += CU_THREADS) rowacc[i] = 0.f;  // ordered by q8_stage's barrier

  float2 rope = make_float2(1.f, 0.f);
  if (!fmt1) cu_body<QT0, QT0, D>(a, r0, j0, j1, nit, nch, red, rowacc, ms, xq, rope, ts);
  else cu_body<QT1, QT0, D>(a, r0, j0, j1, nit, nch, red, rowacc, ms, xq, rope, ts);
  __syncthreads();
  CU_STAMP(5);

  // ---- pair epilogues: wave 0, one lane per pair (a second pass for > 64 pairs)
  if (wave != 0) {
    flush_ts();
    return;
  }
  float s = 1.f;
  if (a.norm_w) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < CU_WAVES; ++w) t += red[w];
    s = rsqrtf(t / (float)a.K + a.eps);
  }
  int pos0 = 0, kv_blk0 = 0;
  if (a.epi == EPI_QKV) {
    pos0 = a.pos[0];
    kv_blk0 = kv_block(a.block_table, a.max_ctx / KV_BLOCK, a.slot ? a.slot[0] : 0, pos0);
  }
  for (int p = lane; 2 * p < nrows; p += 64) {
    const int grow = a.row_base + r0 + 2 * p;
    const float v0 = rowacc[2 * p] * s, v1 = rowacc[2 * p + 1] * s;
    if (a.epi == EPI_QKV) {
      float2 t = rope;
      if (p >= 64 || !a.rope_cs) {  // the lane's prefetched pair covers p < 64 from the table
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

template <int QT0, int QT1>
inline size_t cu_lds_bytes(const GemvArgs& a, int racc_n) {
  constexpr int W = QFmt<QT0>::W, R = QFmt<QT0>::RUNS;
  return (64 + (size_t)racc_n) * 4 + (size_t)(a.K / W) * R * 8 + (size_t)a.K + 16;
}

inline int cu_fmt_bytes_per_256(int qt) {
  switch (qt) {
    case QT_Q4_K: return 144;
    case QT_Q5_K: return 176;
    case QT_Q6_K: return 210;
    case QT_Q4_0: return 144;
    case QT_Q8_0: return 272;
  }
  return 256;
}

// returns false when the shape does not fit (then the row-pair kernel runs)
template <int QT0, int QT1>
bool launch_gemv_cu(const GemvArgs& a, hipStream_t st) {
  if constexpr (!same_xlayout<QT0, QT1>) {
    return false;
  } else {
    // register-streaming variant, kept for probes (kernel_sel 2 / AIOS_GEMV_CU=4|8): slower than the
    // LDS-DMA engine (gemv_lds.h) because its weight stream stalls during the x staging
    static const int env = [] {
      const char* e = std::getenv("AIOS_GEMV_CU");
      return e ? std::atoi(e) : 0;
    }();
    const int mode = a.kernel_sel == 2 ? 8 : (a.kernel_sel == 0 ? env : 0);
    if (!mode || a.B != 1 || a.tune_dbg) return false;
    const int npairs = a.N / 2;
    const int cus = device_cu_count();
    // tune_grid > 0: that many workgroups (tests: ragged splits, > 64 pairs per workgroup)
    const int G = std::min(a.tune_grid > 0 ? a.tune_grid : cus, npairs);
    auto rup = [](int n, int g) { return (n + g - 1) / g; };
    CuPlan pl{G, npairs, (2 * rup(npairs, G) + 3) & ~3};
    if (QT0 != QT1 && a.nseg > 1) {
      const int np0 = a.seg_row0[a.nseg - 1] / 2;
      const double b0 = (double)np0 * cu_fmt_bytes_per_256(QT0), b1 = (double)(npairs - np0) * cu_fmt_bytes_per_256(QT1);
      int g0 = (int)(G * b0 / (b0 + b1) + 0.5);
      g0 = std::max(1, std::min(G - 1, g0));
      if (G < 2 || np0 < 1 || np0 >= npairs) return false;
      const int most = std::max(rup(np0, g0), rup(npairs - np0, G - g0));
      pl = CuPlan{g0, np0, (2 * most + 3) & ~3};
    }
    size_t lds = cu_lds_bytes<QT0, QT1>(a, pl.racc_n);
    if (lds > 160 * 1024) return false;
    lds = std::max(lds, (size_t)(81 * 1024));  // one workgroup per CU
    if (mode <= 4)
      hipLaunchKernelGGL((gemv_cu_b1<QT0, QT1, 4>), dim3(G), dim3(CU_THREADS), lds, st, a, pl);
    else
      hipLaunchKernelGGL((gemv_cu_b1<QT0, QT1, 8>), dim3(G), dim3(CU_THREADS), lds, st, a, pl);
    return true;
  }
}
