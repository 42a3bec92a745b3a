// Prefill GEMM: C[M][N] (+)= A[M][K] (bf16) x W[N][K]^T with W in any repacked quant format,
// dequantised tile-by-tile into LDS as bf16 and multiplied on the CDNA4 matrix cores
// (v_mfma_f32_32x32x16_bf16).  SURVEY.md §2.7 K3 prefill column: "MFMA GEMM (mul_mat_q)" with
// "Q4_K/Q5_K/Q8_0 dequant fused into MFMA matmul" (BASELINE.json north star).
//
// Tile 64(M) x 64(N) x 64(K), 4 waves as 2x2, one 32x32 accumulator per wave.  BK = 64 is one
// Q4_K/Q5_K 64-weight group (one qs group + its two 6-bit sub-block scales) and a quarter of a
// Q6_K super-block, so each thread dequantises 16 contiguous weights of one row per K step.
// LDS tiles are [64 rows][64 bf16] with a 16-B-chunk XOR swizzle (chunk ^ (row & 7)): the
// fragment reads (32 rows x one 16-B chunk per half-wave) are then bank-conflict free.
// Double-buffered: the next tile's global loads are issued before the current tile's MFMAs.
#include "../common.h"
#include "../ops.h"

namespace aios {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));  // register arrays (see below)

constexpr int GM = 64, GN = 64, GK = 64;

__device__ __forceinline__ int swz(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }  // in 16-B units

__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
  return (uint32_t)f32_to_bf16(a) | ((uint32_t)f32_to_bf16(b) << 16);
}

// 16 contiguous weights W[row][k0 .. k0+15] (k0 % 16 == 0) -> 8 packed bf16 pairs (one phase;
// the tiled GEMM below uses the split raw-load / convert form so the loads of K-step kt+1 are in
// flight during the MFMAs of K-step kt)
__device__ __forceinline__ void dequant16(const QWeight& w, int row, int k0, uint32_t out[8]) {
  float v[16];
  switch (w.qtype) {
    case QT_Q4_K:
    case QT_Q5_K: {
      const int nb = w.cols >> 8, b = k0 >> 8, kk = k0 & 255, g = kk >> 6, hi = (kk >> 5) & 1, i0 = kk & 31;
      const size_t blk = (size_t)row * nb + b;
      const uint4 meta = *(const uint4*)(w.p1 + blk * 16);
      const float d = __half2float(__ushort_as_half((uint16_t)(meta.x & 0xffff)));
      const float dmin = __half2float(__ushort_as_half((uint16_t)(meta.x >> 16)));
      const uint32_t f = kq_field(meta.y, meta.z, meta.w, g);
      const int sc = (f >> (6 * hi)) & 63, m = (f >> (12 + 6 * hi)) & 63;
      const float ds = d * sc, dm = dmin * m;
      const uint4 q = *(const uint4*)(w.p0 + blk * 128 + 32 * g + i0);
      uint4 qh = make_uint4(0, 0, 0, 0);
      if (w.qtype == QT_Q5_K) qh = *(const uint4*)(w.p2 + blk * 32 + i0);
      const int hb = 2 * g + hi;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t wv = u4_word(q, j);
        const uint32_t nib = hi ? ((wv >> 4) & 0x0f0f0f0fu) : (wv & 0x0f0f0f0fu);
        const uint32_t h5 = (w.qtype == QT_Q5_K) ? (((u4_word(qh, j) >> hb) & 0x01010101u) << 4) : 0u;
        const uint32_t qq = nib | h5;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * j + e] = ds * (float)((qq >> (8 * e)) & 0xff) - dm;
      }
    } break;
    case QT_Q6_K: {  // Q4_K-order repack (qweight.h)
      const int nb = w.cols >> 8, b = k0 >> 8, kk = k0 & 255, g = kk >> 6, hi = (kk >> 5) & 1, i0 = kk & 31;
      const size_t blk = (size_t)row * nb + b;
      const int l = 2 * g + (i0 >> 4);
      const uint4 q = *(const uint4*)(w.p0 + blk * 128 + 32 * g + i0);
      const uint32_t hv = *(const uint32_t*)(w.p1 + blk * 64 + l * 8 + 4 * hi);
      const int8_t s = *(const int8_t*)(w.p2 + blk * 16 + 2 * l + hi);
      const float d = __half2float(__ushort_as_half(*(const uint16_t*)(w.p3 + blk * 2))) * (float)s;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t wv = u4_word(q, j);
        const uint32_t nib = hi ? ((wv >> 4) & 0x0f0f0f0fu) : (wv & 0x0f0f0f0fu);
        const uint32_t qq = nib | (((hv >> (2 * j)) & 0x03030303u) << 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * j + e] = d * (float)((int)((qq >> (8 * e)) & 0xff) - 32);
      }
    } break;
    case QT_Q4_0: {
      const int nb = w.cols >> 5, b = k0 >> 5, h = (k0 >> 4) & 1;
      const size_t blk = (size_t)row * nb + b;
      const float d = __half2float(__ushort_as_half(*(const uint16_t*)(w.p1 + blk * 2)));
      const uint4 q = *(const uint4*)(w.p0 + blk * 16);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t wv = u4_word(q, j);
        const uint32_t nib = h ? ((wv >> 4) & 0x0f0f0f0fu) : (wv & 0x0f0f0f0fu);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * j + e] = d * (float)((int)((nib >> (8 * e)) & 0xff) - 8);
      }
    } break;
    case QT_Q8_0: {
      const int nb = w.cols >> 5;
      const float d = __half2float(__ushort_as_half(*(const uint16_t*)(w.p1 + ((size_t)row * nb + (k0 >> 5)) * 2)));
      const uint4 q = *(const uint4*)(w.p0 + (size_t)row * w.cols + k0);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t wv = u4_word(q, j);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * j + e] = d * (float)(int8_t)((wv >> (8 * e)) & 0xff);
      }
    } break;
    case QT_BF16: {
      const uint4* p = (const uint4*)(w.p0 + ((size_t)row * w.cols + k0) * 2);
      const uint4 a = p[0], bq = p[1];
      out[0] = a.x; out[1] = a.y; out[2] = a.z; out[3] = a.w;
      out[4] = bq.x; out[5] = bq.y; out[6] = bq.z; out[7] = bq.w;
      return;
    }
    default: {  // F16
      const uint4* p = (const uint4*)(w.p0 + ((size_t)row * w.cols + k0) * 2);
      const uint4 a = p[0], bq = p[1];
      const uint32_t u[8] = {a.x, a.y, a.z, a.w, bq.x, bq.y, bq.z, bq.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[2 * j] = __half2float(__ushort_as_half((uint16_t)(u[j] & 0xffff)));
        v[2 * j + 1] = __half2float(__ushort_as_half((uint16_t)(u[j] >> 16)));
      }
    } break;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = pack_bf16(v[2 * j], v[2 * j + 1]);
}


// ---------------------------------------------------------------------------------------------
// Raw bytes of 16 contiguous weights (k0 % 16 == 0) and their conversion to 8 packed bf16 pairs.
// Layouts are the engine's repacked ones (qweight.h): K-quants keep 128 B of codes per 256-block
// in p0 (Q4_K order for Q6_K too), 16 B of scale/min meta per block in p1 (Q4_K/Q5_K), the Q5_K
// high bits in p2; Q6_K high bits / int8 sub-scales / f16 d in p1 / p2 / p3.
// ---------------------------------------------------------------------------------------------
struct RawB {
  uint4 q;   // codes (or the first 8 bf16/f16 values)
  uint4 m;   // K-quant meta (or the next 8 bf16/f16 values)
  uint4 h;   // Q5_K high bits
  uint32_t x, y;
};

template <int QT>
__device__ __forceinline__ void load_raw16(const QWeight& w, int row, int k0, RawB& r) {
  r.m = r.h = make_uint4(0, 0, 0, 0);
  r.x = r.y = 0;
  switch (QT) {
    case QT_Q4_K:
    case QT_Q5_K: {
      const int nb = w.cols >> 8, b = k0 >> 8, kk = k0 & 255, g = kk >> 6, i0 = kk & 31;
      const size_t blk = (size_t)row * nb + b;
      r.m = *(const uint4*)(w.p1 + blk * 16);
      r.q = *(const uint4*)(w.p0 + blk * 128 + 32 * g + i0);
      if constexpr (QT == QT_Q5_K) r.h = *(const uint4*)(w.p2 + blk * 32 + i0);
    } break;
    case QT_Q6_K: {
      const int nb = w.cols >> 8, b = k0 >> 8, kk = k0 & 255, g = kk >> 6, hi = (kk >> 5) & 1, i0 = kk & 31;
      const size_t blk = (size_t)row * nb + b;
      const int l = 2 * g + (i0 >> 4);
      r.q = *(const uint4*)(w.p0 + blk * 128 + 32 * g + i0);
      r.x = *(const uint32_t*)(w.p1 + blk * 64 + l * 8 + 4 * hi);
      r.y = (uint32_t)(*(const uint8_t*)(w.p2 + blk * 16 + 2 * l + hi)) |
            ((uint32_t)(*(const uint16_t*)(w.p3 + blk * 2)) << 16);
    } break;
    case QT_Q4_0: {
      const int nb = w.cols >> 5, b = k0 >> 5;
      const size_t blk = (size_t)row * nb + b;
      r.x = *(const uint16_t*)(w.p1 + blk * 2);
      r.q = *(const uint4*)(w.p0 + blk * 16);
    } break;
    case QT_Q8_0: {
      const int nb = w.cols >> 5;
      r.x = *(const uint16_t*)(w.p1 + ((size_t)row * nb + (k0 >> 5)) * 2);
      r.q = *(const uint4*)(w.p0 + (size_t)row * w.cols + k0);
    } break;
    default: {  // BF16 / F16
      const uint4* p = (const uint4*)(w.p0 + ((size_t)row * w.cols + k0) * 2);
      r.q = p[0];
      r.m = p[1];
    } break;
  }
}

template <int QT>
__device__ __forceinline__ void convert16(const RawB& r, int k0, uint32_t out[8]) {
  constexpr int qt = QT;
  float v[16];
  switch (qt) {
    case QT_Q4_K:
    case QT_Q5_K: {
      const int kk = k0 & 255, g = kk >> 6, hi = (kk >> 5) & 1, i0 = kk & 31;
      const float d = __half2float(__ushort_as_half((uint16_t)(r.m.x & 0xffff)));
      const float dmin = __half2float(__ushort_as_half((uint16_t)(r.m.x >> 16)));
      const uint32_t f = kq_field(r.m.y, r.m.z, r.m.w, g);
      const int sc = (f >> (6 * hi)) & 63, mn = (f >> (12 + 6 * hi)) & 63;
      const float ds = d * sc, dm = dmin * mn;
      const int hb = 2 * g + hi;
      (void)i0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t wv = u4_word(r.q, j);
        const uint32_t nib = hi ? ((wv >> 4) & 0x0f0f0f0fu) : (wv & 0x0f0f0f0fu);
        const uint32_t h5 = (qt == QT_Q5_K) ? (((u4_word(r.h, j) >> hb) & 0x01010101u) << 4) : 0u;
        const uint32_t qq = nib | h5;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * j + e] = ds * (float)((qq >> (8 * e)) & 0xff) - dm;
      }
    } break;
    case QT_Q6_K: {
      const int hi = ((k0 & 255) >> 5) & 1;
      const float d = __half2float(__ushort_as_half((uint16_t)(r.y >> 16))) * (float)(int8_t)(r.y & 0xff);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t wv = u4_word(r.q, j);
        const uint32_t nib = hi ? ((wv >> 4) & 0x0f0f0f0fu) : (wv & 0x0f0f0f0fu);
        const uint32_t qq = nib | (((r.x >> (2 * j)) & 0x03030303u) << 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * j + e] = d * (float)((int)((qq >> (8 * e)) & 0xff) - 32);
      }
    } break;
    case QT_Q4_0: {
      const int h = (k0 >> 4) & 1;
      const float d = __half2float(__ushort_as_half((uint16_t)r.x));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t wv = u4_word(r.q, j);
        const uint32_t nib = h ? ((wv >> 4) & 0x0f0f0f0fu) : (wv & 0x0f0f0f0fu);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * j + e] = d * (float)((int)((nib >> (8 * e)) & 0xff) - 8);
      }
    } break;
    case QT_Q8_0: {
      const float d = __half2float(__ushort_as_half((uint16_t)r.x));
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t wv = u4_word(r.q, j);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * j + e] = d * (float)(int8_t)((wv >> (8 * e)) & 0xff);
      }
    } break;
    case QT_BF16:
      out[0] = r.q.x; out[1] = r.q.y; out[2] = r.q.z; out[3] = r.q.w;
      out[4] = r.m.x; out[5] = r.m.y; out[6] = r.m.z; out[7] = r.m.w;
      return;
    default: {  // F16
      const uint32_t u[8] = {r.q.x, r.q.y, r.q.z, r.q.w, r.m.x, r.m.y, r.m.z, r.m.w};
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[2 * j] = __half2float(__ushort_as_half((uint16_t)(u[j] & 0xffff)));
        v[2 * j + 1] = __half2float(__ushort_as_half((uint16_t)(u[j] >> 16)));
      }
    } break;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = pack_bf16(v[2 * j], v[2 * j + 1]);
}

// ---------------------------------------------------------------------------------------------
// Tiled MFMA GEMM with fused weight dequant.  Workgroup tile BM x BN x 64, 4 waves as 2 x 2, wave
// tile (BM/2) x (BN/2) of 32x32 v_mfma_f32_32x32x16_bf16 accumulators.  Per K-step: the A tile
// (bf16 activations) and the raw weight bytes of step kt+1 are loaded into registers while the
// MFMAs of step kt run; the weights are then dequantised to bf16 and both tiles written to the
// other LDS buffer (16-B chunk XOR swizzle: conflict-free fragment reads), one barrier per step.
// Up to 3 weight segments (e.g. Q/K/V with their own formats) share the A tile stream: each
// BN-column tile lies inside one segment.  Tiles are mapped XCD-aware: the 8 XCDs each take a
// contiguous range of (m-tile, n-tile) pairs, n fastest, so an XCD keeps its A rows in its L2.
// ---------------------------------------------------------------------------------------------
template <int QT, int BM, int BN, int EPI>
__global__ void __launch_bounds__(256) gemm_q_kernel(GemmQArgs a) {
  constexpr int WM = BM / 2, WN = BN / 2, TM = WM / 32, TN = WN / 32;
  constexpr int AU = BM * 8 / 256;   // 16-B A chunks per thread per K-step
  constexpr int BU = BN * 4 / 256;   // 16-weight B units per thread per K-step
  __shared__ __attribute__((aligned(16))) uint4 sA[2][BM * 8];
  __shared__ __attribute__((aligned(16))) uint4 sB[2][BN * 8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  // XCD-aware tile order
  const int nN = a.N / BN, nM = (a.M + BM - 1) / BM, total = nN * nM;
  int L = blockIdx.x;
  if ((total & 7) == 0) L = (L & 7) * (total >> 3) + (L >> 3);
  const int tn = L % nN, tm = L / nN;
  const int m0 = tm * BM, n0 = tn * BN;
  int s = 0;
  if (a.nseg > 1 && n0 >= a.seg_n0[1]) s = 1;
  if (a.nseg > 2 && n0 >= a.seg_n0[2]) s = 2;
  QWeight w;  // field-wise uniform selects (a dynamically indexed struct copy goes to scratch)
  w.qtype = QT;
  w.rows = s == 0 ? a.seg[0].rows : (s == 1 ? a.seg[1].rows : a.seg[2].rows);
  w.cols = a.K;
  w.pad_ = 0;
  w.p0 = s == 0 ? a.seg[0].p0 : (s == 1 ? a.seg[1].p0 : a.seg[2].p0);
  w.p1 = s == 0 ? a.seg[0].p1 : (s == 1 ? a.seg[1].p1 : a.seg[2].p1);
  w.p2 = s == 0 ? a.seg[0].p2 : (s == 1 ? a.seg[1].p2 : a.seg[2].p2);
  w.p3 = s == 0 ? a.seg[0].p3 : (s == 1 ? a.seg[1].p3 : a.seg[2].p3);
  const int wrow0 = n0 - (s == 0 ? a.seg_n0[0] : (s == 1 ? a.seg_n0[1] : a.seg_n0[2]));
  // split-K (blockIdx.y of gridDim.y): this workgroup's K-steps [kt0, kt1); partial sums are
  // added atomically (the launcher zeroes C first for STORE)
  const int nk_all = a.K / 64, S = gridDim.y;
  const int kt0 = (int)((long)blockIdx.y * nk_all / S), kt1 = (int)((long)(blockIdx.y + 1) * nk_all / S);

  // three register stages of raw tiles: tile t lives in stage (t - kt0) % 3 and is converted into
  // LDS two K-steps after its loads were issued (one K-step of MFMAs hides too little latency at
  // decode-sized M: each step then waited a full memory round trip)
  u32x4 ra0[AU], ra1[AU], ra2[AU];  // native vectors: arrays of HIP's uint4 struct end up in scratch
  RawB rb0[BU], rb1[BU], rb2[BU];
#define GEMM_LOAD(kt_, RA, RB)                                                          \
  {                                                                                     \
    _Pragma("unroll") for (int i = 0; i < AU; ++i) {                                    \
      const int idx = tid + 256 * i, r = idx >> 3, c = idx & 7;                         \
      const int m = min(m0 + r, a.M - 1); /* rows past M re-read the last row */        \
      RA[i] = *(const u32x4*)(a.A + (size_t)m * a.lda + (kt_) * 64 + c * 8);            \
    }                                                                                   \
    _Pragma("unroll") for (int i = 0; i < BU; ++i) {                                    \
      const int idx = tid + 256 * i, r = idx >> 2, p = idx & 3;                         \
      load_raw16<QT>(w, wrow0 + r, (kt_) * 64 + 16 * p, RB[i]);                        \
    }                                                                                   \
  }
#define GEMM_STORE(buf_, kt_, RA, RB)                                                   \
  {                                                                                     \
    _Pragma("unroll") for (int i = 0; i < AU; ++i) {                                    \
      const int idx = tid + 256 * i, r = idx >> 3, c = idx & 7;                         \
      *(u32x4*)&sA[buf_][r * 8 + (c ^ (r & 7))] = RA[i];                                \
    }                                                                                   \
    _Pragma("unroll") for (int i = 0; i < BU; ++i) {                                    \
      const int idx = tid + 256 * i, r = idx >> 2, p = idx & 3;                         \
      uint32_t o[8];                                                                    \
      convert16<QT>(RB[i], (kt_) * 64 + 16 * p, o);                                     \
      sB[buf_][r * 8 + ((2 * p) ^ (r & 7))] = make_uint4(o[0], o[1], o[2], o[3]);       \
      sB[buf_][r * 8 + ((2 * p + 1) ^ (r & 7))] = make_uint4(o[4], o[5], o[6], o[7]);   \
    }                                                                                   \
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int half = lane >> 5, l32 = lane & 31;
  auto mfma_step = [&](int cur) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * WM + i * 32 + l32;
        const uint4 v = sA[cur][r * 8 + ((2 * ks + half) ^ (r & 7))];
        __builtin_memcpy(&af[i], &v, 16);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * WN + j * 32 + l32;
        const uint4 v = sB[cur][r * 8 + ((2 * ks + half) ^ (r & 7))];
        __builtin_memcpy(&bfr[j], &v, 16);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  // Loads are issued unconditionally (tile index clamped into [kt0, kt1): a re-read of the last
  // tile instead of a branch) -- a conditional load makes the outstanding-load count path
  // dependent and the compiler then drains everything with vmcnt(0) before each conversion,
  // which serialised every K-step on a full memory round trip (measured: 1.6 us per step).
  const int klast = kt1 - 1;
  GEMM_LOAD(kt0, ra0, rb0);
  GEMM_LOAD(min(kt0 + 1, klast), ra1, rb1);
  GEMM_LOAD(min(kt0 + 2, klast), ra2, rb2);
  GEMM_STORE(0, kt0, ra0, rb0);
  __syncthreads();
  // one K-step: MFMAs on the LDS tile k, convert tile k+1 (stage RC) into the other LDS buffer,
  // then reuse tile k's stage (RL) for the loads of tile k+3
#define GEMM_STEP(k_, RC_A, RC_B, RL_A, RL_B)                                           \
  {                                                                                     \
    const int cur = ((k_) - kt0) & 1;                                                   \
    mfma_step(cur);                                                                     \
    if ((k_) + 1 < kt1) GEMM_STORE(cur ^ 1, (k_) + 1, RC_A, RC_B);                      \
    GEMM_LOAD(min((k_) + 3, klast), RL_A, RL_B);                                        \
    __syncthreads();                                                                    \
  }
  int kt = kt0;
  for (; kt + 3 <= kt1; kt += 3) {
    GEMM_STEP(kt, ra1, rb1, ra0, rb0);
    GEMM_STEP(kt + 1, ra2, rb2, ra1, rb1);
    GEMM_STEP(kt + 2, ra0, rb0, ra2, rb2);
  }
  if (kt < kt1) GEMM_STEP(kt, ra1, rb1, ra0, rb0);
  if (kt + 1 < kt1) GEMM_STEP(kt + 1, ra2, rb2, ra1, rb1);
#undef GEMM_STEP
  // C/D map of the 32x32 accumulator: col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * WN + j * 32 + l32;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        const float v = acc[i][j][r];
        if constexpr (EPI == GEPI_SWIGLU_BF16) {
          // interleaved gate/up columns: even lane = gate, odd lane = its up partner
          const float up = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), 0xB1, 0xF, 0xF, false));
          if (m < a.M && !(l32 & 1)) a.C16[(size_t)m * a.ldc + (n >> 1)] = f32_to_bf16(v / (1.f + __expf(-v)) * up);
        } else if (m < a.M) {
          float* c = a.C + (size_t)m * a.ldc + n;
          if (S > 1) unsafeAtomicAdd(c, v);
          else if constexpr (EPI == GEPI_ACCUM) *c += v;
          else *c = v;
        }
      }
    }
  }
}

#undef GEMM_LOAD
#undef GEMM_STORE

bool gemm_supports(int qt) {
  return qt == QT_Q4_K || qt == QT_Q5_K || qt == QT_Q6_K || qt == QT_Q4_0 || qt == QT_Q8_0 || qt == QT_F16 ||
         qt == QT_BF16;
}

template <int QT, int BM, int BN>
static void launch_tiles(const GemmQArgs& a, hipStream_t st) {
  const int tiles = (a.N / BN) * ((a.M + BM - 1) / BM);
  // split-K for grids below ~2 workgroups per CU (decode-sized M, short prefill chunks)
  int S = a.ksplit;
  if (S <= 0) {
    const int cus = device_cu_count(), nk = a.K / 64;
    // up to ~4 workgroups per CU (one wave per SIMD leaves every LDS / MFMA / VALU latency
    // exposed at decode-sized M), >= 4 K-steps per workgroup
    S = tiles >= 2 * cus ? 1 : std::max(1, std::min(nk / 4, (4 * cus + tiles - 1) / tiles));
  }
  if (a.epi == GEPI_SWIGLU_BF16) S = 1;  // nonlinear epilogue needs the full sum
  S = std::max(1, std::min(S, a.K / 64));
  if (S > 1 && a.epi == GEPI_STORE)
    HIP_CHECK(hipMemset2DAsync(a.C, (size_t)a.ldc * 4, 0, (size_t)a.N * 4, a.M, st));
  const dim3 grid(tiles, S);
  switch (a.epi) {
    case GEPI_STORE: hipLaunchKernelGGL((gemm_q_kernel<QT, BM, BN, GEPI_STORE>), grid, dim3(256), 0, st, a); break;
    case GEPI_ACCUM: hipLaunchKernelGGL((gemm_q_kernel<QT, BM, BN, GEPI_ACCUM>), grid, dim3(256), 0, st, a); break;
    case GEPI_SWIGLU_BF16:
      hipLaunchKernelGGL((gemm_q_kernel<QT, BM, BN, GEPI_SWIGLU_BF16>), grid, dim3(256), 0, st, a);
      break;
    default: throw std::runtime_error("gemm: bad epilogue");
  }
}

template <int QT>
static void launch_qt(const GemmQArgs& a, hipStream_t st) {
  bool ok128 = a.N % 128 == 0;
  for (int s = 0; s < a.nseg; ++s)
    if (a.seg_n0[s] % 128 || a.seg[s].rows % 128) ok128 = false;
  // largest tile that still gives >= ~one workgroup per CU
  const int cus = device_cu_count();
  const int mt128 = (a.M + 127) / 128, mt64 = (a.M + 63) / 64;
  if (ok128 && (a.N / 128) * mt128 >= cus) launch_tiles<QT, 128, 128>(a, st);
  else if (ok128 && (a.N / 128) * mt64 >= cus / 2) launch_tiles<QT, 64, 128>(a, st);
  else launch_tiles<QT, 64, 64>(a, st);
}

static void launch_one(const GemmQArgs& a, hipStream_t st) {
  switch (a.seg[0].qtype) {
    case QT_Q4_K: launch_qt<QT_Q4_K>(a, st); break;
    case QT_Q5_K: launch_qt<QT_Q5_K>(a, st); break;
    case QT_Q6_K: launch_qt<QT_Q6_K>(a, st); break;
    case QT_Q4_0: launch_qt<QT_Q4_0>(a, st); break;
    case QT_Q8_0: launch_qt<QT_Q8_0>(a, st); break;
    case QT_F16: launch_qt<QT_F16>(a, st); break;
    case QT_BF16: launch_qt<QT_BF16>(a, st); break;
    default: throw std::runtime_error("gemm: unsupported weight format");
  }
}

// Segments sharing a format go in one launch; a format change starts a new launch whose C
// pointer is shifted to the segment's first column (e.g. Q4_K Q/K + Q6_K V in Q4_K_M layers).
void launch_gemm_q(const GemmQArgs& a, hipStream_t st) {
  if (a.K % 64) throw std::runtime_error("gemm: K must be a multiple of 64");
  if (a.nseg < 1 || a.nseg > 3) throw std::runtime_error("gemm: 1..3 weight segments");
  for (int s = 0; s < a.nseg; ++s) {
    if (!gemm_supports(a.seg[s].qtype)) throw std::runtime_error("gemm: unsupported weight format");
    if (a.seg[s].cols != a.K) throw std::runtime_error("gemm: weight cols != K");
    if (a.seg[s].rows % 64 || a.seg_n0[s] % 64) throw std::runtime_error("gemm: segment sizes must be multiples of 64");
  }
  if (a.N % 64) throw std::runtime_error("gemm: N must be a multiple of 64");
  int s0 = 0;
  while (s0 < a.nseg) {
    int s1 = s0 + 1;
    while (s1 < a.nseg && a.seg[s1].qtype == a.seg[s0].qtype) ++s1;
    GemmQArgs b = a;
    b.nseg = s1 - s0;
    const int c0 = a.seg_n0[s0];
    for (int s = 0; s < b.nseg; ++s) {
      b.seg[s] = a.seg[s0 + s];
      b.seg_n0[s] = a.seg_n0[s0 + s] - c0;
    }
    b.N = (s1 < a.nseg ? a.seg_n0[s1] : a.N) - c0;
    if (a.epi == GEPI_SWIGLU_BF16) {
      if (c0 % 2) throw std::runtime_error("gemm: odd swiglu segment start");
      b.C16 = a.C16 + c0 / 2;
    } else {
      b.C = a.C + c0;
    }
    launch_one(b, st);
    s0 = s1;
  }
}

// single-segment form kept for the bindings / tests
void launch_gemm(const GemmArgs& g, hipStream_t st) {
  GemmQArgs a;
  std::memset(&a, 0, sizeof(a));
  a.A = g.A; a.lda = g.lda; a.nseg = 1; a.seg[0] = g.w; a.seg_n0[0] = 0;
  a.M = g.M; a.N = g.N; a.K = g.K; a.C = g.C; a.ldc = g.ldc;
  a.epi = g.accumulate ? GEPI_ACCUM : GEPI_STORE;
  if (g.N % 64 == 0) {
    launch_gemm_q(a, st);
    return;
  }
  throw std::runtime_error("gemm: N must be a multiple of 64");
}

}  // namespace aios
