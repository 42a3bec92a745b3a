// int8-activation GEMV path (included by gemv_impl.h after the shared helpers).
//
// The llama.cpp "q8_1 x" trick, done per workgroup in LDS: x is quantised to int8 per 32-element
// block (dx = amax/127) while it is staged, and every 16-B weight chunk is multiplied with
// v_dot4_i32_i8 (4 MACs per VALU op) directly on the 4-/5-/6-bit codes -- ~5x fewer VALU ops per
// weight than the fp32 path and 4x fewer LDS bytes.  Per 16-run r of a chunk:
//     contrib = sc_r * dx_r * isum_r - of_r * sx_r,    sx_r = dx_r * sum(xq over the run)
// (the K-quant "min" and the Q4_0 / Q6_K code bias fold into of_r).
//
// Single-pass prologue: the RMSNorm statistic and the int8 staging come from ONE global read of
// x.  Block quantisation is scale-invariant, so x*w is quantised un-normalised and 1/rms is
// applied to the finished dot product in the epilogue (y = inv_rms * W (x*w)).
//
// Two work decompositions:
//  * gemv_q8_rows  : one wave owns a row-pair (grid-stride, 2-deep register pipeline) -- for
//                    short K where a pair is 1-2 work items;
//  * gemv_q8_ksplit: the 4 waves of a workgroup split the K items of the same row-pair and
//                    combine through LDS every G pairs -- for long K (down-proj), where one
//                    wave per pair would be a 4-7 item dependent chain.
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
    const int hs = 2 * ((c & 3) >> 1);
    int s0 = 0, s1 = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t wv = u4_word(r.a, i), hv = u4_word(r.b, i);
      const uint32_t lo = (wv & 0x0f0f0f0fu) | (((hv >> hs) & 0x03030303u) << 4);
      const uint32_t hi = ((wv >> 4) & 0x0f0f0f0fu) | (((hv >> (hs + 4)) & 0x03030303u) << 4);
      s0 = __builtin_amdgcn_sdot4((int)lo, x[i], s0, false);
      s1 = __builtin_amdgcn_sdot4((int)hi, x[4 + i], s1, false);
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

// Stage B rows of x (times the RMSNorm weight when nw != null, NOT normalised) as int8 per
// 32-block in QT's chunk order; returns per-thread partial sum of squares of x in ssq[b].
template <int QT, int B>
__device__ __forceinline__ void stage_q8(const float* __restrict__ x, int ldx, int nb, int K,
                                         const float* __restrict__ nw, int8_t* xq, float2* ms, float (&ssq)[B]) {
  using F_ = QFmt<QT>;
  constexpr int W = F_::W, R = F_::RUNS;
  const int nch = K / W, nblk = K / 32;
#pragma unroll
  for (int b = 0; b < B; ++b) ssq[b] = 0.f;
  for (int t = threadIdx.x; t < nb * nblk; t += blockDim.x) {
    const int b = t / nblk, blk = t - b * nblk;
    const float* src = x + (size_t)b * ldx + blk * 32;
    float v[32];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float4 f = *(const float4*)(src + 4 * i);
      v[4 * i] = f.x; v[4 * i + 1] = f.y; v[4 * i + 2] = f.z; v[4 * i + 3] = f.w;
    }
    float s2 = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) s2 = fmaf(v[i], v[i], s2);
#pragma unroll
    for (int bb = 0; bb < B; ++bb)
      if (bb == b) ssq[bb] += s2;
    if (nw) {
      const float* wp = nw + blk * 32;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float4 g = *(const float4*)(wp + 4 * i);
        v[4 * i] *= g.x; v[4 * i + 1] *= g.y; v[4 * i + 2] *= g.z; v[4 * i + 3] *= g.w;
      }
    }
    float amax = 0.f;
#pragma unroll
    for (int i = 0; i < 32; ++i) amax = fmaxf(amax, fabsf(v[i]));
    const float dx = amax / 127.f;
    const float inv = amax > 0.f ? 127.f / amax : 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      uint32_t wq[4];
      int isum = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        uint32_t w = 0;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int q = (int)rintf(v[16 * h + 4 * j + e] * inv);
          isum += q;
          w |= ((uint32_t)(q & 0xff)) << (8 * e);
        }
        wq[j] = w;
      }
      int c, s0;
      F_::run_pos(blk * 2 + h, c, s0);
      int piece = s0 >> 4;
      if (W == 32) piece = (piece + (c >> 3)) & 1;
      *(uint4*)(xq + ((size_t)b * nch + c) * W + 16 * piece) = make_uint4(wq[0], wq[1], wq[2], wq[3]);
      ms[((size_t)b * nch + c) * R + (s0 >> 4)] = make_float2(dx, dx * (float)isum);
    }
  }
}

template <int QT, int B, int U>
__device__ __forceinline__ void q8_compute(const RawChunk (&raw)[U][GEMV_ROWS], int it, int nch, const int8_t* xq,
                                           const float2* ms, float (&acc)[GEMV_ROWS][B]) {
  using F_ = QFmt<QT>;
  constexpr int W = F_::W, R = F_::RUNS;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = (it * U + u) * 64 + lane;
    if (c < nch) {
      float sc[GEMV_ROWS][R], of[GEMV_ROWS][R];
#pragma unroll
      for (int r = 0; r < GEMV_ROWS; ++r) q8_scales<QT>(raw[u][r], c, sc[r], of[r]);
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
        float2 m[R];
        const float2* mp = ms + ((size_t)b * nch + c) * R;
#pragma unroll
        for (int rr = 0; rr < R; ++rr) m[rr] = mp[rr];
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
}

// shared prologue: issue nothing, stage x for one or two layouts, produce inv_rms[b] in LDS
template <int QT0, int QT1, int B>
__device__ __forceinline__ void q8_prologue(const GemvArgs& a, float* red, float* inv_rms, int8_t* xq0, float2* ms0,
                                            int8_t* xq1, float2* ms1) {
  float ssq[B];
  stage_q8<QT0, B>(a.x, a.ldx, a.B, a.K, a.norm_w, xq0, ms0, ssq);
  if (QT0 != QT1) {
    float dummy[B];
    stage_q8<QT1, B>(a.x, a.ldx, a.B, a.K, a.norm_w, xq1, ms1, dummy);
  }
  if (a.norm_w) {
#pragma unroll
    for (int b = 0; b < B; ++b) {
      if (b < a.B) {
        const float s = block_sum(ssq[b], red);
        if (threadIdx.x == 0) inv_rms[b] = rsqrtf(s / (float)a.K + a.eps);
      }
    }
  }
  __syncthreads();
}

template <int QT0, int QT1, int B>
struct Q8Lds {
  float* red;
  float* inv_rms;
  float2* ms0;
  int8_t* xq0;
  float2* ms1;
  int8_t* xq1;
  float* part;  // k-split partials
  __device__ Q8Lds(float* smem, int K) {
    constexpr int W0 = QFmt<QT0>::W, W1 = QFmt<QT1>::W, R0 = QFmt<QT0>::RUNS, R1 = QFmt<QT1>::RUNS;
    red = smem;
    inv_rms = smem + 16;
    part = smem + 64;                       // 512 floats
    ms0 = (float2*)(smem + 64 + 512);
    xq0 = (int8_t*)(ms0 + (size_t)B * (K / W0) * R0);
    ms1 = (QT0 != QT1) ? (float2*)(xq0 + (size_t)B * K) : ms0;
    xq1 = (QT0 != QT1) ? (int8_t*)(ms1 + (size_t)B * (K / W1) * R1) : xq0;
  }
  static size_t bytes(int K) {
    constexpr int W0 = QFmt<QT0>::W, W1 = QFmt<QT1>::W, R0 = QFmt<QT0>::RUNS, R1 = QFmt<QT1>::RUNS;
    size_t b = (64 + 512) * 4 + (size_t)B * K + (size_t)B * (K / W0) * R0 * 8;
    if (QT0 != QT1) b += (size_t)B * K + (size_t)B * (K / W1) * R1 * 8;
    return b + 64;
  }
};

__device__ __forceinline__ float q8_rms_scale(const GemvArgs& a, const float* inv_rms, int b) {
  return a.norm_w ? inv_rms[b] : 1.f;
}

// ---------------------------------------------------------------------------------------------
// one wave per row-pair
// ---------------------------------------------------------------------------------------------
template <int QT0, int QT1, int B, int U>
__global__ void __launch_bounds__(GP_THREADS) gemv_q8_rows(GemvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr bool MIXED = QT0 != QT1;
  constexpr int W0 = QFmt<QT0>::W, W1 = QFmt<QT1>::W;
  Q8Lds<QT0, QT1, B> L(smem, a.K);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int npairs = a.N >> 1;
  const int nch0 = a.K / W0, nch1 = a.K / W1;
  const int nit0 = (nch0 + 64 * U - 1) / (64 * U), nit1 = (nch1 + 64 * U - 1) / (64 * U);
  const int stride = gridDim.x * GP_WAVES;

  auto info = [&](int p, int& lrow, bool& t1, const QWeight*& w) {
    const int row = 2 * p;
    int s = 0;
#pragma unroll
    for (int k = 1; k < GEMV_MAX_SEGS; ++k)
      if (k < a.nseg && row >= a.seg_row0[k]) s = k;
    lrow = row - a.seg_row0[s];
    t1 = MIXED && (s == a.nseg - 1) && a.nseg > 1;
    w = &a.seg[s];
  };
  auto load = [&](int p, int it, RawChunk (&r)[U][GEMV_ROWS]) {
    int lrow;
    bool t1;
    const QWeight* w;
    info(p, lrow, t1, w);
    if (MIXED && t1) gp_load<QT1, U>(*w, lrow, it, nch1, r);
    else gp_load<QT0, U>(*w, lrow, it, nch0, r);
  };

  int p = blockIdx.x * GP_WAVES + wave;
  int it = 0;
  RawChunk bufA[U][GEMV_ROWS], bufB[U][GEMV_ROWS];
  if (p < npairs) load(p, 0, bufA);  // weight loads in flight during the prologue
  q8_prologue<QT0, QT1, B>(a, L.red, L.inv_rms, L.xq0, L.ms0, L.xq1, L.ms1);

  float acc[GEMV_ROWS][B];
#pragma unroll
  for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
    for (int b = 0; b < B; ++b) acc[r][b] = 0.f;

  auto step = [&](RawChunk (&cur)[U][GEMV_ROWS], RawChunk (&nxt)[U][GEMV_ROWS]) -> bool {
    int lrow;
    bool t1;
    const QWeight* w;
    info(p, lrow, t1, w);
    const int nit = (MIXED && t1) ? nit1 : nit0;
    int pn = p, itn = it + 1;
    if (itn >= nit) { pn = p + stride; itn = 0; }
    if (pn < npairs) load(pn, itn, nxt);
    if (MIXED && t1) q8_compute<QT1, B, U>(cur, it, nch1, L.xq1, L.ms1, acc);
    else q8_compute<QT0, B, U>(cur, it, nch0, L.xq0, L.ms0, acc);
    if (itn == 0) {
#pragma unroll
      for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
        for (int b = 0; b < B; ++b) acc[r][b] = wave_sum(acc[r][b]);
      if (lane < a.B) {
        float v0 = 0.f, v1 = 0.f;
#pragma unroll
        for (int b = 0; b < B; ++b)
          if (lane == b) { v0 = acc[0][b]; v1 = acc[1][b]; }
        const float s = q8_rms_scale(a, L.inv_rms, lane);
        gemv_epilogue(a, a.row_base + 2 * p, lane, v0 * s, v1 * s);
      }
#pragma unroll
      for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
        for (int b = 0; b < B; ++b) acc[r][b] = 0.f;
    }
    p = pn;
    it = itn;
    return p < npairs;
  };
  while (p < npairs) {
    if (!step(bufA, bufB)) break;
    if (!step(bufB, bufA)) break;
  }
}

// ---------------------------------------------------------------------------------------------
// K split over the 4 waves of a workgroup (single format).  Pair j of the workgroup is
// p = blockIdx.x + j*gridDim.x; wave w handles items it = w, w+4, ... of every pair; partials go
// to LDS part[g][w][2][B] and every KS_G pairs one barrier + a 4-way sum runs the epilogues.
// ---------------------------------------------------------------------------------------------
constexpr int KS_G = 8;

template <int QT, int B, int U>
__global__ void __launch_bounds__(GP_THREADS) gemv_q8_ksplit(GemvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int W = QFmt<QT>::W;
  Q8Lds<QT, QT, B> L(smem, a.K);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int npairs = a.N >> 1;
  const int nch = a.K / W;
  const int nit = (nch + 64 * U - 1) / (64 * U);
  const QWeight& w = a.seg[0];
  const int npb = blockIdx.x < npairs ? (npairs - 1 - blockIdx.x) / gridDim.x + 1 : 0;  // pairs of this WG
  const int ni = wave < nit ? (nit - wave + GP_WAVES - 1) / GP_WAVES : 0;                // items per pair
  const int total = npb * ni;

  auto load_f = [&](int f, RawChunk (&r)[U][GEMV_ROWS]) {
    const int j = f / ni, i = f - j * ni;
    const int p = blockIdx.x + j * gridDim.x;
    gp_load<QT, U>(w, 2 * p, wave + GP_WAVES * i, nch, r);
  };
  RawChunk bufA[U][GEMV_ROWS], bufB[U][GEMV_ROWS];
  if (total > 0) load_f(0, bufA);
  q8_prologue<QT, QT, B>(a, L.red, L.inv_rms, L.xq0, L.ms0, L.xq0, L.ms0);

  float acc[GEMV_ROWS][B];
#pragma unroll
  for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
    for (int b = 0; b < B; ++b) acc[r][b] = 0.f;

  int f = 0;  // this wave's flattened item cursor
  for (int j0 = 0; j0 < npb; j0 += KS_G) {
    const int jn = min(j0 + KS_G, npb);
    for (int j = j0; j < jn; ++j) {
      for (int i = 0; i < ni; ++i) {
        if (f + 1 < total) load_f(f + 1, bufB);  // next item in flight while this one computes
        q8_compute<QT, B, U>(bufA, wave + GP_WAVES * i, nch, L.xq0, L.ms0, acc);
        ++f;
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int r = 0; r < GEMV_ROWS; ++r) bufA[u][r] = bufB[u][r];
      }
      // this wave's partial of pair j -> LDS
#pragma unroll
      for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
        for (int b = 0; b < B; ++b) {
          const float v = wave_sum(acc[r][b]);
          if (lane == 0) L.part[(((j - j0) * GP_WAVES + wave) * GEMV_ROWS + r) * B + b] = v;
          acc[r][b] = 0.f;
        }
    }
    __syncthreads();
    for (int t = threadIdx.x; t < (jn - j0) * B; t += GP_THREADS) {
      const int g = t / B, b = t - g * B;
      if (b < a.B) {
        float v[GEMV_ROWS] = {0.f, 0.f};
#pragma unroll
        for (int ww = 0; ww < GP_WAVES; ++ww)
#pragma unroll
          for (int r = 0; r < GEMV_ROWS; ++r) v[r] += L.part[((g * GP_WAVES + ww) * GEMV_ROWS + r) * B + b];
        const float s = q8_rms_scale(a, L.inv_rms, b);
        const int p = blockIdx.x + (j0 + g) * gridDim.x;
        gemv_epilogue(a, a.row_base + 2 * p, b, v[0] * s, v[1] * s);
      }
    }
    __syncthreads();
  }
}

template <int QT0, int QT1, int B, int U>
bool launch_gemv_q8(GemvArgs a, hipStream_t st) {
  const size_t lds = Q8Lds<QT0, QT1, B>::bytes(a.K);
  if (lds > 96 * 1024) return false;
  constexpr int W0 = QFmt<QT0>::W;
  const int nit = (a.K / W0 + 64 * U - 1) / (64 * U);
  const int npairs = a.N / 2;
  // K-split measured slower than row pairs on MI355X (down-proj 15.6 vs 13.6 us): opt-in only
  const bool ksplit = (QT0 == QT1) && nit >= 3 && a.tune_ksplit > 0;
  a.kt_max = a.K;
  if (ksplit) {
    static int occ = -1;
    if (occ < 0) {
      int o = 0;
      if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, gemv_q8_ksplit<QT0, B, U>, GP_THREADS, lds) != hipSuccess ||
          o <= 0)
        o = 1;
      occ = o;
    }
    int per_cu = std::max(1, std::min(occ, (int)((160 * 1024) / lds)));
    if (a.tune_grid > 0) per_cu = a.tune_grid;
    const int blocks = std::min(npairs, device_cu_count() * per_cu);
    hipLaunchKernelGGL((gemv_q8_ksplit<QT0, B, U>), dim3(blocks), dim3(GP_THREADS), lds, st, a);
    return true;
  }
  static int occ = -1;
  if (occ < 0) {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, gemv_q8_rows<QT0, QT1, B, U>, GP_THREADS, lds) !=
            hipSuccess || o <= 0)
      o = 1;
    occ = o;
  }
  int per_cu = std::max(1, std::min(occ, (int)((160 * 1024) / lds)));
  if (a.tune_grid > 0) per_cu = a.tune_grid;
  const int groups = (npairs + GP_WAVES - 1) / GP_WAVES;
  const int blocks = std::min(groups, device_cu_count() * per_cu);
  hipLaunchKernelGGL((gemv_q8_rows<QT0, QT1, B, U>), dim3(blocks), dim3(GP_THREADS), lds, st, a);
  return true;
}
