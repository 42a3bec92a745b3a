// Batched-decode GEMM (M <= 64 rows of activations): C[M][N] = X[M][K] (bf16) x W[N][K]^T with
// W streamed from its repacked quantised layout straight into MFMA operand registers.
//
// SURVEY.md §2.7 K3 decode column at B > 1 (llama.cpp's mul_mat_q / mmvq for small batches inside
// llama-server, /root/reference/runtime/src/model_manager.rs:187-204): the weights are the only
// large operand, read once per step, so the kernel is shaped like a GEMV that happens to finish
// on the matrix cores:
//   * transposed product D[n][m] = W[n][:] . X[m][:] on v_mfma_f32_16x16x32_bf16 with the weight
//     rows as the A operand: lane (n = l & 15, q = l >> 4) loads one 16-B quant chunk (32 weights)
//     per step, dequantises it in registers into four 8-weight fragments and never touches LDS
//     with weight data (CDNA guide §5 "GEMV / M <= 16 decode weights": straight to VGPRs);
//   * the k-slots of a fragment are whatever k the chunk holds -- the activation fragment of lane
//     (m, q) is read from the same k set, so no weight repack for MFMA is needed;
//   * X (bf16, the small operand) is staged through LDS in 4-step chunks, double-buffered and
//     register-prefetched one chunk ahead, so its loads are always OLDER than the weight loads in
//     flight and no vmcnt wait ever drains the weight ring;
//   * weights are ring-buffered NL = 4 steps ahead per lane (the whole 16-row x 512-k slice of a
//     wave in flight for Q4_K), 8 (or 4) waves per workgroup each on their own 16 rows;
//   * K is split over S workgroups when the row tiles alone do not fill the chip; partial tiles
//     go to write-through (sc1) fp32 slabs and the LAST arriving workgroup of a tile (relaxed
//     agent ticket, one agent-scope acquire; CDNA guide §5 "In-launch split-K reduction") sums
//     them and runs the epilogue -- no float atomics, deterministic result, one launch.
// The B = 1 step keeps the int8-activation GEMV (gemv_q8.h, 4 MACs per VALU op); from B = 2 the
// dequant-once MFMA form is cheaper than B passes of v_dot4.
#include "skinny_epi.h"

namespace aios {

constexpr int SK_NL = 4;    // weight ring depth = steps per X chunk
constexpr int SK_SMAX = 16;  // K splits at most (slab workspace: gemm_skinny_ws_bytes)

template <int QT>
struct SkFmt {
  static constexpr int W = QFmt<QT>::W;   // weights per 16-B chunk
  static constexpr int NP = W / 8;         // 8-weight MFMA k-slots per chunk
  static constexpr int STEPK = 4 * W;      // k covered by one load step (4 lanes per row)
  static constexpr int KC = SK_NL * STEPK; // k per staged X chunk
  // first k of part i of chunk c
  __device__ static int part_k(int c, int i) {
    if constexpr (NP == 4) return QFmt<QT>::chunk_k0(c, i >> 1) + 8 * (i & 1);
    else if constexpr (NP == 2) return QFmt<QT>::chunk_k0(c, 0) + 8 * i;
    else return QFmt<QT>::chunk_k0(c, 0);
  }
};

// the workgroup body for weight format QT (the kernel below picks it per tile); X chunks live in
// the launch's dynamic LDS (two buffers of MP x XROW bf16, sized for the larger format)
template <int QT, int RB, int MT, int EPI>
__device__ __forceinline__ void sk_body(const GemmQArgs& a, int S) {
  using F = SkFmt<QT>;
  constexpr int NT = RB * 64, ROWS = 16 * RB, MP = 16 * MT;
  // X rows are KC bf16 (a multiple of 256 B) with the 16-B units of row m XOR-swizzled by
  // h(m) = (m ^ 2m) & 15: the MFMA B-operand ds_read_b128 of lane (rr, q) then hits 16 distinct
  // 4-bank slots in each of the instruction's four 16-lane groups ({0-3,12-15,20-27}, ... --
  // MI355X_MICROARCH.md §LDS) for every format's chunk -> k map (Q4_K q offsets 0/2/8/10 units,
  // Q6_K 0/2/4/6, Q4_0/Q8_0 0/4/8/12, F16/BF16 0/1/2/3).  The padded row (+16 B) left 2 lanes of
  // every group sharing banks: SQ_LDS_BANK_CONFLICT = 4 cycles per read (tools/gpu_pmc_skinny.sh)
  constexpr int KC = F::KC, XROW = KC;
  // (same-box A/B against the padded rows, profiles/skinny_swizzle_ab_r2s3.txt: conflicts 4 cycles
  // per read -> 0, step time unchanged within 0.3 % -- the kernel is load-latency bound)
  constexpr int xpitch = XROW;
  auto xsw = [](int m, int kl) __attribute__((always_inline)) { return m * XROW + (kl ^ (((m ^ (m << 1)) & 15) << 3)); };
  constexpr int XU = MP * KC / 8;           // 16-B units of one X chunk
  constexpr int XPT = (XU + NT - 1) / NT;   // per thread
  extern __shared__ __attribute__((aligned(16))) bf16_t sk_xs[];
  __shared__ int last_flag;
  // probes (tools/skinny_probe.py): 0 start, 1 prologue loads issued, 2 first X chunk staged,
  // 3 main loop done, 4 done (a slice that handed its slab to the tile's last arriver), 5 done
  // (the epilogue written)
  // (stored as taken, probe launches only: no stamp state live through the kernel)
  auto stamp = [&](int i) __attribute__((always_inline)) {
    if (a.dbg_ts && threadIdx.x == 0) a.dbg_ts[(size_t)blockIdx.x * 8 + i] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int rr = lane & 15, q = lane >> 4;
  const int ntile = a.N / ROWS, total = ntile * S;
  const int L = xcd_remap(blockIdx.x, total);
  const int rg = L / S, sp = L % S;  // a tile's slices are consecutive: one XCD, same-L2 slabs
  const int n0 = rg * ROWS;
  int s = 0;
  if (a.nseg > 1 && n0 >= a.seg_n0[1]) s = 1;
  if (a.nseg > 2 && n0 >= a.seg_n0[2]) s = 2;
  QWeight w;
  w.qtype = QT;
  w.rows = s == 0 ? a.seg[0].rows : (s == 1 ? a.seg[1].rows : a.seg[2].rows);
  w.cols = a.K;
  w.pad_ = 0;
  w.p0 = s == 0 ? a.seg[0].p0 : (s == 1 ? a.seg[1].p0 : a.seg[2].p0);
  w.p1 = s == 0 ? a.seg[0].p1 : (s == 1 ? a.seg[1].p1 : a.seg[2].p1);
  w.p2 = s == 0 ? a.seg[0].p2 : (s == 1 ? a.seg[1].p2 : a.seg[2].p2);
  w.p3 = s == 0 ? a.seg[0].p3 : (s == 1 ? a.seg[1].p3 : a.seg[2].p3);
  const int lrow = n0 - (s == 0 ? a.seg_n0[0] : (s == 1 ? a.seg_n0[1] : a.seg_n0[2])) + 16 * wave + rr;
  const int nch = a.K / F::W;                       // chunks per weight row
  const int nsteps = (nch + 3) / 4;                 // load steps per row
  const int nchunk = (nsteps + SK_NL - 1) / SK_NL;  // X chunks over K
  const int c0 = (int)((long)sp * nchunk / S), c1 = (int)((long)(sp + 1) * nchunk / S);
  const int tb = c0 * SK_NL, te = min(c1 * SK_NL, nsteps);  // this workgroup's steps [tb, te)

  // ---- X chunk staging (register prefetch one chunk ahead, zero past M / K)
  gu32x4 xr[XPT];
  auto x_load = [&](int c) __attribute__((always_inline)) {
    const int kc0 = c * KC;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int u = tid + NT * i;
      const int m = u / (KC / 8), k = kc0 + 8 * (u % (KC / 8));
      const int mm = min(m, a.M - 1), kk = min(k, a.K - 8);
      xr[i] = *(const gu32x4*)(a.A + (size_t)mm * a.lda + kk);  // unconditional (clamped) load
    }
  };
  auto x_store = [&](int buf, int c) __attribute__((always_inline)) {
    const int kc0 = c * KC;
#pragma unroll
    for (int i = 0; i < XPT; ++i) {
      const int u = tid + NT * i;
      if (XU % NT == 0 || u < XU) {
        const int m = u / (KC / 8), kl = 8 * (u % (KC / 8));
        gu32x4 v = xr[i];
        if (m >= a.M || kc0 + kl >= a.K) v = gu32x4{0u, 0u, 0u, 0u};
        *(gu32x4*)&sk_xs[buf * (MP * xpitch) + xsw(m, kl)] = v;
      }
    }
  };

  // ---- weight ring: step t -> chunk 4t + q of this lane's row (clamped in-bounds load).  Q4_K /
  // Q5_K keep one 16-B scale/min record per 256-block = per two steps: only even steps load it
  // and the odd step re-uses it (meta_cur), halving the load instructions.
  constexpr bool MB = QT == QT_Q4_K || QT == QT_Q5_K;
  RawChunk ring[SK_NL];
  uint4 meta_cur = make_uint4(0, 0, 0, 0);
  const int nbk = a.K >> 8;
  auto w_load = [&](int t, RawChunk& r, bool with_meta) __attribute__((always_inline)) {
    const int c = min(4 * min(t, te - 1) + q, nch - 1);
    if constexpr (MB) {
      r.a = *(const uint4*)(w.p0 + ((size_t)lrow * nbk * 8 + c) * 16);
      if (with_meta) r.b = *(const uint4*)(w.p1 + ((size_t)lrow * nbk + (c >> 3)) * 16);
      if constexpr (QT == QT_Q5_K) r.c = *(const uint4*)(w.p2 + ((size_t)lrow * nbk + (c >> 3)) * 32 + 16 * (c & 1));
    } else {
      QFmt<QT>::load(w, lrow, c, r);
    }
  };

  gf32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = gf32x4{0.f, 0.f, 0.f, 0.f};

  constexpr bool BYTES = QT != QT_F16 && QT != QT_BF16;
  auto compute = [&](const RawChunk& r, const uint4& meta, int t, int buf, int kc0) __attribute__((always_inline)) {
    const int c = 4 * t + q;
    const bool valid = c < nch;
    float sc[2], of[2];
    if constexpr (MB) {
      RawChunk rm = r;
      rm.b = meta;
      QStream<QT>::scales(rm, c, sc, of);
    } else {
      QStream<QT>::scales(r, c, sc, of);
    }
    if (!valid) sc[0] = sc[1] = of[0] = of[1] = 0.f;
    if constexpr (QFmt<QT>::RUNS == 1) { sc[1] = sc[0]; of[1] = of[0]; }
#pragma unroll
    for (int i = 0; i < F::NP; ++i) {
      float qv[8];
      if constexpr (BYTES) {
        // raw codes as byte words made opaque, so every byte converts with one v_cvt_f32_ubyteN
        uint32_t w0 = QStream<QT>::word(r, c, 2 * i), w1 = QStream<QT>::word(r, c, 2 * i + 1);
        asm volatile("" : "+v"(w0), "+v"(w1));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          qv[e] = (float)((w0 >> (8 * e)) & 0xff);
          qv[4 + e] = (float)((w1 >> (8 * e)) & 0xff);
        }
      } else {
        QStream<QT>::quad(r, c, 2 * i, qv);
        QStream<QT>::quad(r, c, 2 * i + 1, qv + 4);
      }
      const int run = F::NP == 4 ? (i >> 1) : 0;
      const float s_ = sc[run], o_ = of[run];
      uint32_t p[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) p[e] = pk_bf16(fmaf(s_, qv[2 * e], -o_), fmaf(s_, qv[2 * e + 1], -o_));
      gbf16x8 wf;
      __builtin_memcpy(&wf, p, 16);
      const int kl = F::part_k(c, i) - kc0;
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const uint4 xv = *(const uint4*)&sk_xs[buf * (MP * xpitch) + xsw(16 * mt + rr, kl)];
        gbf16x8 xf;
        __builtin_memcpy(&xf, &xv, 16);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, xf, acc[mt], 0, 0, 0);
      }
    }
  };

  // ---- fused RMSNorm (consumer): the producer's per-tile sums of squares, nG <= 16 lanes per row
  // (power of two >= parts / 4, one float4 each), loaded before everything else and reduced in a
  // fixed order once the first X chunk has landed -> inv_s[m]
  constexpr int NR = (MP * 16 + NT - 1) / NT;
  __shared__ float inv_s[MP];
  const bool nrm = a.nrm_in != nullptr;
  int nlg = 0;
  gf32x4 nv[NR];
  if (nrm) {
    const int p4 = a.nrm_parts >> 2;
    while ((1 << nlg) < p4) ++nlg;
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int u = tid + NT * r, m = u >> nlg, j = u & ((1 << nlg) - 1);
      nv[r] = gf32x4{0.f, 0.f, 0.f, 0.f};
      if (m < a.M && j < p4) nv[r] = *(const gf32x4*)(a.nrm_in + (size_t)m * a.nrm_parts + 4 * j);
    }
  }
  // prologue: X chunk c0 first (oldest loads), then the weight ring, then X chunk c0+1
  x_load(c0);
#pragma unroll
  for (int u = 0; u < SK_NL; ++u) w_load(tb + u, ring[u], !MB || (u & 1) == 0);
  stamp(1);
  x_store(0, c0);
  if (nrm) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int u = tid + NT * r, m = u >> nlg;
      float s = (nv[r][0] + nv[r][1]) + (nv[r][2] + nv[r][3]);
      for (int o = 1; o < (1 << nlg); o <<= 1) s += __shfl_xor(s, o, 64);
      if ((u & ((1 << nlg) - 1)) == 0 && m < MP) inv_s[m] = rsqrtf(s / (float)a.K + a.nrm_eps);
    }
  }
  x_load(min(c0 + 1, c1 - 1));
  __syncthreads();
  stamp(2);
  for (int c = c0; c < c1; ++c) {
    const int buf = (c - c0) & 1, kc0 = c * KC;
#pragma unroll
    for (int u = 0; u < SK_NL; ++u) {
      const int t = c * SK_NL + u;
      if (t < te) compute(ring[u], (u & 1) ? meta_cur : ring[u].b, t, buf, kc0);
      if (MB && (u & 1) == 0) meta_cur = ring[u].b;
      w_load(t + SK_NL, ring[u], !MB || (u & 1) == 0);
    }
    if (c + 1 < c1) x_store(buf ^ 1, c + 1);
    x_load(min(c + 2, c1 - 1));
    __syncthreads();
  }

  stamp(3);
  const bool wrote = sk_epilogue<RB, MT, EPI>(a, acc, n0, rg, sp, S, ntile, inv_s, nrm, (float*)&sk_xs[0], last_flag);
  if (wrote) stamp(5); else stamp(4);  // 4: a split-K slice that was not its tile's last arriver
}

// One launch for every tile: with mixed formats (Q4_K_M: Q|K Q4_K, V Q6_K) the tiles of the last
// segment run the QT1 body -- the V rows then share the launch (and the chip) with Q|K instead of
// following as a 64-workgroup launch of their own
template <int QT0, int QT1, int RB, int MT, int EPI>
__global__ void __launch_bounds__(RB * 64) gemm_skinny_kernel(GemmQArgs a, int S) {
  if constexpr (QT0 != QT1) {
    const int L = xcd_remap(blockIdx.x, (a.N / (16 * RB)) * S);
    if ((L / S) * 16 * RB >= a.seg_n0[a.nseg - 1]) {
      sk_body<QT1, RB, MT, EPI>(a, S);
      return;
    }
  }
  sk_body<QT0, RB, MT, EPI>(a, S);
}

int gemm_skinny_cnt_len(int N) { return N / 64 + 1; }

static int sk_env(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}
// slab bytes for the largest split the launcher can pick: AIOS_SKINNY_SMAX (default 8) or an
// explicit AIOS_SKINNY_S, never above SK_SMAX (sizing for SK_SMAX left half unused)
size_t gemm_skinny_ws_bytes(int M, int N) {
  const int smax = std::min(SK_SMAX, std::max(sk_env("AIOS_SKINNY_SMAX", 8), sk_env("AIOS_SKINNY_S", 0)));
  return (size_t)smax * 16 * ((M + 15) / 16) * N * 4;
}

template <int QT0, int QT1, int RB, int MT>
static void sk_launch(const GemmQArgs& a, int S, hipStream_t st) {
  const int grid = (a.N / (16 * RB)) * S;
  const int lds = 2 * 16 * MT * (std::max(SkFmt<QT0>::KC, SkFmt<QT1>::KC) + 8) * 2;
#define SK_GO(E) hipLaunchKernelGGL((gemm_skinny_kernel<QT0, QT1, RB, MT, E>), dim3(grid), dim3(RB * 64), lds, st, a, S)
  if constexpr (QT0 != QT1) {  // mixed formats: the packed QKV projection only
    if (a.epi == GEPI_QKV) SK_GO(GEPI_QKV);
    else SK_GO(GEPI_STORE);
  } else {
    switch (a.epi) {
      case GEPI_STORE: SK_GO(GEPI_STORE); break;
      case GEPI_QKV: SK_GO(GEPI_QKV); break;
      case GEPI_ACCUM: SK_GO(GEPI_ACCUM); break;
      case GEPI_ACCUM_NORM: SK_GO(GEPI_ACCUM_NORM); break;
      default: SK_GO(GEPI_SWIGLU_BF16); break;
    }
  }
#undef SK_GO
}

template <int QT0, int QT1, int RB>
static void sk_mt(const GemmQArgs& a, int S, hipStream_t st) {
  if (a.M <= 16) sk_launch<QT0, QT1, RB, 1>(a, S, st);
  else if (a.M <= 32) sk_launch<QT0, QT1, RB, 2>(a, S, st);
  else sk_launch<QT0, QT1, RB, 4>(a, S, st);
}

// waves (16-row groups) per workgroup: 8 when every segment splits into 128-row tiles
static int sk_rb(const GemmQArgs& a) {
  bool rows128 = a.N % 128 == 0;
  for (int s = 0; s < a.nseg; ++s)
    if (a.seg_n0[s] % 128 || a.seg[s].rows % 128) rows128 = false;
  const int force_rb = sk_env("AIOS_SKINNY_RB", 0);
  return force_rb == 4 ? 4 : (rows128 ? 8 : 4);
}

static bool sk_fits(const GemmQArgs& a) {
  if (a.M > 64 || a.N % 64) return false;
  if (a.epi == GEPI_SWIGLU_BF16 && a.ldc % 2) return false;
  if ((a.epi != GEPI_SWIGLU_BF16 && a.ldc % 4) || a.lda % 8) return false;
  if (a.nrm_in && (a.nrm_parts % 4 || a.nrm_parts > 64)) return false;
  if (a.epi == GEPI_ACCUM_NORM && (!a.nrm_g || !a.nrm_out16 || !a.nrm_part || a.N / (16 * sk_rb(a)) != a.nrm_parts))
    return false;
  switch (a.seg[0].qtype) {
    case QT_Q4_K: case QT_Q5_K: case QT_Q6_K: case QT_Q4_0: case QT_Q8_0: case QT_F16: case QT_BF16: return true;
    default: return false;
  }
}

int gemm_skinny_ntile(const GemmQArgs& a) { return a.M <= 64 && a.N % 64 == 0 ? a.N / (16 * sk_rb(a)) : 0; }

template <int QT0, int QT1>
static bool sk_qt(const GemmQArgs& a, hipStream_t st) {
  using F0 = SkFmt<QT0>;
  using F1 = SkFmt<QT1>;
  const int RB = sk_rb(a);
  const int ntile = a.N / (16 * RB);
  auto nchunk_of = [&](int W) { return ((a.K / W + 3) / 4 + SK_NL - 1) / SK_NL; };
  const int nchunk = std::min(nchunk_of(F0::W), nchunk_of(F1::W));
  const int MP = 16 * (a.M <= 16 ? 1 : (a.M <= 32 ? 2 : 4));
  // LDS per workgroup: two X chunks; resident workgroups per CU bounded by LDS and by 2048 threads
  const int lds = 2 * MP * (std::max(F0::KC, F1::KC) + 8) * 2;
  const int per_cu = std::max(1, std::min(163840 / lds, 2048 / (RB * 64)));
  int S = a.ksplit > 0 ? a.ksplit : sk_env("AIOS_SKINNY_S", 0);
  if (S <= 0) {
    // resident workgroups: LDS / threads allow per_cu, the ~100-VGPR bodies 2 of 8 waves
    const int cap = device_cu_count() * std::min(per_cu, sk_env("AIOS_SKINNY_WGCU", 2));
    if (sk_env("AIOS_SKINNY_SPLIT_MODE", 1) == 0) {
      S = ntile >= cap ? 1 : (cap + ntile - 1) / ntile;
    } else {
      // fewest dispatch rounds per unit of K work: a partial second round of workgroups costs a
      // whole round (224 gate/up tiles: S = 2 in one round, not S = 3 in 1.3).  At most 8 slices
      // by default (AIOS_SKINNY_SMAX; tools/gpu_split_ab.sh, Mistral B = 32: 16 slices for the
      // d_model-wide projections 8333 tok/s, 8 slices 8867, the old fill rule 8038)
      double best = 1e30;
      const int smax = std::min({nchunk, SK_SMAX, sk_env("AIOS_SKINNY_SMAX", 8)});
      for (int s = 1; s <= smax; ++s) {
        const double cost = (double)((ntile * s + cap - 1) / cap) / s;
        if (cost < best - 1e-9) { best = cost; S = s; }
      }
    }
  }
  S = std::max(1, std::min({S, nchunk, SK_SMAX}));
  // split-K needs the slab workspace and tickets; without them, one workgroup per tile
  if (S > 1 && (!a.ws || !a.cnt || a.cnt_len < ntile || a.ws_bytes < (size_t)S * MP * a.N * 4)) S = 1;
  if (RB == 8) sk_mt<QT0, QT1, 8>(a, S, st);
  else sk_mt<QT0, QT1, 4>(a, S, st);
  return true;
}

// the mixed-format launch (AIOS_SKINNY_MIXED, default on): leading segments Q4_K, last Q6_K (the
// Q4_K_M QKV stack), the QKV / store epilogues
bool gemm_skinny_mixed_ok(const GemmQArgs& a) {
  if (a.nseg < 2 || !sk_env("AIOS_SKINNY_MIXED", 1)) return false;
  const int q1 = a.seg[a.nseg - 1].qtype;
  for (int s = 0; s + 1 < a.nseg; ++s)
    if (a.seg[s].qtype != QT_Q4_K) return false;
  return q1 == QT_Q6_K && (a.epi == GEPI_QKV || a.epi == GEPI_STORE);
}

bool launch_gemm_skinny(const GemmQArgs& a, hipStream_t st) {
  if (!sk_fits(a)) return false;
  bool same = true;
  for (int s = 1; s < a.nseg; ++s) same &= a.seg[s].qtype == a.seg[0].qtype;
  if (!same) return gemm_skinny_mixed_ok(a) && sk_qt<QT_Q4_K, QT_Q6_K>(a, st);
  switch (a.seg[0].qtype) {
    case QT_Q4_K: return sk_qt<QT_Q4_K, QT_Q4_K>(a, st);
    case QT_Q5_K: return sk_qt<QT_Q5_K, QT_Q5_K>(a, st);
    case QT_Q6_K: return sk_qt<QT_Q6_K, QT_Q6_K>(a, st);
    case QT_Q4_0: return sk_qt<QT_Q4_0, QT_Q4_0>(a, st);
    case QT_Q8_0: return sk_qt<QT_Q8_0, QT_Q8_0>(a, st);
    case QT_F16: return sk_qt<QT_F16, QT_F16>(a, st);
    case QT_BF16: return sk_qt<QT_BF16, QT_BF16>(a, st);
    default: return false;
  }
}

}  // namespace aios
