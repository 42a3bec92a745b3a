// Device helpers shared by the two matrix-core GEMMs (gemm.hip: M > 64 prefill tiles,
// gemm_skinny.hip: M <= 64 batched decode).  Both dequantise the engine's repacked weight streams
// (qweight.h) on the fly into bf16 MFMA operands -- there is no resident bf16 copy of any weight.
#pragma once
#include "../common.h"
#include "../ops.h"

namespace aios {

typedef __bf16 gbf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 gbf16x2 __attribute__((ext_vector_type(2)));
typedef float gf32x2 __attribute__((ext_vector_type(2)));
typedef float gf32x4 __attribute__((ext_vector_type(4)));
typedef float gf32x16 __attribute__((ext_vector_type(16)));
typedef unsigned int gu32x4 __attribute__((ext_vector_type(4)));

// two floats -> packed bf16 pair, round-to-nearest-even in hardware (v_cvt_pk_bf16_f32)
__device__ __forceinline__ uint32_t pk_bf16(float a, float b) {
  const gf32x2 v = {a, b};
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, gbf16x2));
}

// 8 dequantised weights w = sc * q - of (q raw unsigned codes) -> one bf16x8 MFMA fragment
__device__ __forceinline__ gbf16x8 dq8_frag(const float (&q)[8], float sc, float of) {
  gbf16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = (__bf16)fmaf(sc, q[e], -of);
  return r;
}

// ---------------------------------------------------------------------------------------------
// Raw bytes of 16 contiguous weights W[row][k0 .. k0+15] (k0 % 16 == 0) and their conversion to
// 8 packed bf16 pairs.  K-quants keep 128 B of codes per 256-block in p0 (Q4_K order for Q6_K
// too), 16 B of scale/min meta per block in p1 (Q4_K/Q5_K), the Q5_K high bits in p2; Q6_K high
// bits / int8 sub-scales / f16 d in p1 / p2 / p3 (qweight.h).
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
      const int kk = k0 & 255, g = kk >> 6, hi = (kk >> 5) & 1;
      const float d = __half2float(__ushort_as_half((uint16_t)(r.m.x & 0xffff)));
      const float dmin = __half2float(__ushort_as_half((uint16_t)(r.m.x >> 16)));
      const uint32_t f = kq_field(r.m.y, r.m.z, r.m.w, g);
      const int sc = (f >> (6 * hi)) & 63, mn = (f >> (12 + 6 * hi)) & 63;
      const float ds = d * sc, dm = dmin * mn;
      const int hb = 2 * g + hi;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t wv = u4_word(r.q, j);
        const uint32_t nib = hi ? ((wv >> 4) & 0x0f0f0f0fu) : (wv & 0x0f0f0f0fu);
        const uint32_t h5 = (qt == QT_Q5_K) ? (((u4_word(r.h, j) >> hb) & 0x01010101u) << 4) : 0u;
        const uint32_t qq = nib | h5;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * j + e] = fmaf(ds, (float)((qq >> (8 * e)) & 0xff), -dm);
      }
    } break;
    case QT_Q6_K: {
      const int hi = ((k0 & 255) >> 5) & 1;
      const float d = __half2float(__ushort_as_half((uint16_t)(r.y >> 16))) * (float)(int8_t)(r.y & 0xff);
      const float dm = 32.f * d;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t wv = u4_word(r.q, j);
        const uint32_t nib = hi ? ((wv >> 4) & 0x0f0f0f0fu) : (wv & 0x0f0f0f0fu);
        const uint32_t qq = nib | (((r.x >> (2 * j)) & 0x03030303u) << 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * j + e] = fmaf(d, (float)((qq >> (8 * e)) & 0xff), -dm);
      }
    } break;
    case QT_Q4_0: {
      const int h = (k0 >> 4) & 1;
      const float d = __half2float(__ushort_as_half((uint16_t)r.x));
      const float dm = 8.f * d;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint32_t wv = u4_word(r.q, j);
        const uint32_t nib = h ? ((wv >> 4) & 0x0f0f0f0fu) : (wv & 0x0f0f0f0fu);
#pragma unroll
        for (int e = 0; e < 4; ++e) v[4 * j + e] = fmaf(d, (float)((nib >> (8 * e)) & 0xff), -dm);
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
  for (int j = 0; j < 8; ++j) out[j] = pk_bf16(v[2 * j], v[2 * j + 1]);
}

// Bijective XCD-aware block remap (CDNA guide §5 "XCD swizzle must be bijective"): consecutive
// logical tiles land on one XCD (blocks b, b+8, ... share an XCD under round-robin dispatch), so
// tiles that share an operand panel share that XCD's L2.  Speed only, never correctness.
__device__ __forceinline__ int xcd_remap(int L, int nwg) {
  if (nwg <= 8) return L;
  const int xcd = L & 7, q = nwg >> 3, r = nwg & 7;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (L >> 3);
}

}  // namespace aios
