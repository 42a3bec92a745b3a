// Device-side quantized weight descriptor + per-format chunk decoders (gfx950).
//
// Weights are repacked at load time (quant_pack.hip) from the GGUF array-of-blocks layout into
// a structure-of-arrays layout per row, so that one lane loads exactly one aligned 16-byte
// "chunk" of quant bits per global_load_dwordx4 and the per-block metadata sits in a separate,
// separately-aligned stream:
//
//   Q4_K : p0 = qs   [rows][nb*128]    p1 = meta [rows][nb*16] = {f16 d, f16 dmin, u8 scales[12]}
//   Q5_K : p0 = qs   [rows][nb*128]    p1 = meta [rows][nb*16]   p2 = qh [rows][nb*32]
//   Q6_K : p0 = lo4  [rows][nb*128]    p1 = hi2  [rows][nb*64]   p2 = sc [rows][nb*16] (int8)
//          p3 = d    [rows][nb] (f16)         (re-ordered into the Q4_K chunk order, see below)
//   Q4_0 : p0 = qs   [rows][nb*16]     p1 = d    [rows][nb] (f16)             (nb = K/32)
//   Q8_0 : p0 = qs   [rows][nb*32]     p1 = d    [rows][nb] (f16)             (nb = K/32)
//   F16 / BF16 : p0 = [rows][K]
//
// A chunk covers W weights (32 for Q4_K/Q5_K/Q6_K/Q4_0, 16 for Q8_0, 8 for F16/BF16) made of
// RUNS contiguous 16-weight runs (K index ranges).  `chunk_k0(c, run)` gives the first K index
// of each run; the GEMV prologue lays x out in LDS in chunk order so a lane reads its W x-values
// with W/4 conflict-free ds_read_b128.
#pragma once
#include "common.h"

namespace aios {

struct QWeight {
  int qtype;
  int rows;
  int cols;
  int pad_;
  const uint8_t* p0;
  const uint8_t* p1;
  const uint8_t* p2;
  const uint8_t* p3;
};

struct RawChunk {
  uint4 a;      // main quant bits
  uint4 b;      // meta / qh
  uint4 c;      // qh / scales
  uint32_t d;   // f16 scale (Q6_K / Q4_0 / Q8_0)
};

template <int QT>
struct QFmt;

// formats whose chunk -> k mapping is identical share one staged activation layout
__host__ __device__ constexpr bool kq_layout(int q) { return q == QT_Q4_K || q == QT_Q5_K || q == QT_Q6_K; }
template <int A, int B>
constexpr bool same_xlayout = A == B || (kq_layout(A) && kq_layout(B));

// Q4_K / Q5_K repacked block meta (16 B): word0 = {f16 d, f16 dmin}; words 1..3 hold a 96-bit
// string of four 24-bit fields, field g = sc[2g] | sc[2g+1] << 6 | m[2g] << 12 | m[2g+1] << 18
// (the 6-bit sub-block scales / mins of the 64-weight group g).  One funnel shift extracts the
// four values a chunk needs -- the GGUF 12-byte packing needs a g-dependent bit shuffle instead.
__device__ __forceinline__ uint32_t kq_field(uint32_t w1, uint32_t w2, uint32_t w3, int g) {
  const uint32_t lo = g < 2 ? w1 : (g == 2 ? w2 : w3);
  const uint32_t hi = g < 2 ? w2 : w3;
  return __builtin_amdgcn_alignbit(hi, lo, (24 * g) & 31);
}

__device__ __forceinline__ uint32_t u4_word(const uint4& v, int i) {
  return i == 0 ? v.x : (i == 1 ? v.y : (i == 2 ? v.z : v.w));
}

// ------------------------------------------------------------------------------------ Q4_K
template <>
struct QFmt<QT_Q4_K> {
  static constexpr int W = 32, RUNS = 2, CHUNKS_PER_BLOCK = 8, BLOCK = 256;
  __device__ static int chunk_k0(int c, int run) {
    const int b = c >> 3, l = c & 7, g = l >> 1, h = l & 1;
    return b * 256 + 64 * g + 16 * h + 32 * run;
  }
  // run r (16 contiguous k) -> (chunk, slot0)
  __device__ static void run_pos(int r, int& c, int& s0) {
    const int b = r >> 4, rr = r & 15, g = rr >> 2, hi = (rr >> 1) & 1, h = rr & 1;
    c = b * 8 + 2 * g + h;
    s0 = 16 * hi;
  }
  __device__ static void load(const QWeight& w, int row, int c, RawChunk& r) {
    const int nb = w.cols >> 8;
    r.a = *(const uint4*)(w.p0 + ((size_t)row * nb * 8 + c) * 16);
    r.b = *(const uint4*)(w.p1 + ((size_t)row * nb + (c >> 3)) * 16);
  }
  // q[] as raw unsigned values, run scale/offset: contribution = sc*dot(q,x) - of*sum(x)
  __device__ static void decode(const RawChunk& r, int c, float q[32], float sc[2], float of[2]) {
    const int l = c & 7, g = l >> 1;
    const uint32_t dd = r.b.x;
    const float d = __half2float(__ushort_as_half((uint16_t)(dd & 0xffff)));
    const float dmin = __half2float(__ushort_as_half((uint16_t)(dd >> 16)));
    const uint32_t f = kq_field(r.b.y, r.b.z, r.b.w, g);
    const uint32_t scp = (f & 63) | (((f >> 6) & 63) << 8), mp = ((f >> 12) & 63) | (((f >> 18) & 63) << 8);
    sc[0] = d * (float)(scp & 0xff);
    sc[1] = d * (float)(scp >> 8);
    of[0] = dmin * (float)(mp & 0xff);
    of[1] = dmin * (float)(mp >> 8);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t wv = u4_word(r.a, i);
      const uint32_t lo = wv & 0x0f0f0f0fu, hi = (wv >> 4) & 0x0f0f0f0fu;
      q[4 * i + 0] = (float)(lo & 0xff);
      q[4 * i + 1] = (float)((lo >> 8) & 0xff);
      q[4 * i + 2] = (float)((lo >> 16) & 0xff);
      q[4 * i + 3] = (float)(lo >> 24);
      q[16 + 4 * i + 0] = (float)(hi & 0xff);
      q[16 + 4 * i + 1] = (float)((hi >> 8) & 0xff);
      q[16 + 4 * i + 2] = (float)((hi >> 16) & 0xff);
      q[16 + 4 * i + 3] = (float)(hi >> 24);
    }
  }
};

// ------------------------------------------------------------------------------------ Q5_K
template <>
struct QFmt<QT_Q5_K> {
  static constexpr int W = 32, RUNS = 2, CHUNKS_PER_BLOCK = 8, BLOCK = 256;
  __device__ static int chunk_k0(int c, int run) { return QFmt<QT_Q4_K>::chunk_k0(c, run); }
  __device__ static void run_pos(int r, int& c, int& s0) { QFmt<QT_Q4_K>::run_pos(r, c, s0); }
  __device__ static void load(const QWeight& w, int row, int c, RawChunk& r) {
    const int nb = w.cols >> 8;
    r.a = *(const uint4*)(w.p0 + ((size_t)row * nb * 8 + c) * 16);
    r.b = *(const uint4*)(w.p1 + ((size_t)row * nb + (c >> 3)) * 16);
    // qh bytes [16*h, 16*h+16) of the block's 32
    r.c = *(const uint4*)(w.p2 + ((size_t)row * nb + (c >> 3)) * 32 + 16 * (c & 1));
  }
  __device__ static void decode(const RawChunk& r, int c, float q[32], float sc[2], float of[2]) {
    QFmt<QT_Q4_K>::decode(r, c, q, sc, of);
    const int g = (c & 7) >> 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t hv = u4_word(r.c, i);
      const uint32_t h0 = (hv >> (2 * g)) & 0x01010101u, h1 = (hv >> (2 * g + 1)) & 0x01010101u;
      q[4 * i + 0] += (float)((h0 & 0xff) << 4);
      q[4 * i + 1] += (float)(((h0 >> 8) & 0xff) << 4);
      q[4 * i + 2] += (float)(((h0 >> 16) & 0xff) << 4);
      q[4 * i + 3] += (float)((h0 >> 24) << 4);
      q[16 + 4 * i + 0] += (float)((h1 & 0xff) << 4);
      q[16 + 4 * i + 1] += (float)(((h1 >> 8) & 0xff) << 4);
      q[16 + 4 * i + 2] += (float)(((h1 >> 16) & 0xff) << 4);
      q[16 + 4 * i + 3] += (float)((h1 >> 24) << 4);
    }
  }
};

// ------------------------------------------------------------------------------------ Q6_K
// Repacked into the Q4_K chunk order (quant_pack.hip), so x staging is shared with Q4_K/Q5_K and a
// mixed Q4_K_M QKV segment list (V in Q6_K) needs ONE activation layout:
//   p0 = low nibbles exactly where Q4_K keeps its 4-bit codes,
//   p1 = 8 B per chunk {h0, h1}: bits (8e + 2j)..+1 of h_run = high 2 bits of weight 4j+e of the run,
//   p2 = the 16 int8 scales re-ordered so chunk l's pair is bytes (2l, 2l+1),  p3 = f16 d.
template <>
struct QFmt<QT_Q6_K> {
  static constexpr int W = 32, RUNS = 2, CHUNKS_PER_BLOCK = 8, BLOCK = 256;
  __device__ static int chunk_k0(int c, int run) { return QFmt<QT_Q4_K>::chunk_k0(c, run); }
  __device__ static void run_pos(int r, int& c, int& s0) { QFmt<QT_Q4_K>::run_pos(r, c, s0); }
  __device__ static void load(const QWeight& w, int row, int c, RawChunk& r) {
    const int nb = w.cols >> 8;
    const size_t blk = (size_t)row * nb + (c >> 3);
    const size_t ch = (size_t)row * nb * 8 + c;
    r.a = *(const uint4*)(w.p0 + ch * 16);
    const uint2 h = *(const uint2*)(w.p1 + ch * 8);
    r.b.x = h.x;
    r.b.y = h.y;
    r.c.x = *(const uint16_t*)(w.p2 + ch * 2);  // this chunk's (run 0, run 1) int8 scale pair
    r.d = *(const uint16_t*)(w.p3 + blk * 2);
  }
  __device__ static float sc_lo(const RawChunk& r) { return (float)(int8_t)(r.c.x & 0xff); }
  __device__ static float sc_hi(const RawChunk& r) { return (float)(int8_t)((r.c.x >> 8) & 0xff); }
  __device__ static uint32_t code_lo(const RawChunk& r, int i) {
    return (u4_word(r.a, i) & 0x0f0f0f0fu) | (((r.b.x >> (2 * i)) & 0x03030303u) << 4);
  }
  __device__ static uint32_t code_hi(const RawChunk& r, int i) {
    return ((u4_word(r.a, i) >> 4) & 0x0f0f0f0fu) | (((r.b.y >> (2 * i)) & 0x03030303u) << 4);
  }
  __device__ static void decode(const RawChunk& r, int c, float q[32], float sc[2], float of[2]) {
    const float d = __half2float(__ushort_as_half((uint16_t)r.d));
    sc[0] = d * sc_lo(r);
    sc[1] = d * sc_hi(r);
    of[0] = 32.f * sc[0];  // q - 32 folded as -32*sc*sum(x)
    of[1] = 32.f * sc[1];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t lo = code_lo(r, i), hi = code_hi(r, i);
      q[4 * i + 0] = (float)(lo & 0xff);
      q[4 * i + 1] = (float)((lo >> 8) & 0xff);
      q[4 * i + 2] = (float)((lo >> 16) & 0xff);
      q[4 * i + 3] = (float)(lo >> 24);
      q[16 + 4 * i + 0] = (float)(hi & 0xff);
      q[16 + 4 * i + 1] = (float)((hi >> 8) & 0xff);
      q[16 + 4 * i + 2] = (float)((hi >> 16) & 0xff);
      q[16 + 4 * i + 3] = (float)(hi >> 24);
    }
  }
};

// ------------------------------------------------------------------------------------ Q4_0
template <>
struct QFmt<QT_Q4_0> {
  static constexpr int W = 32, RUNS = 2, CHUNKS_PER_BLOCK = 1, BLOCK = 32;
  __device__ static int chunk_k0(int c, int run) { return c * 32 + 16 * run; }
  __device__ static void run_pos(int r, int& c, int& s0) {
    c = r >> 1;
    s0 = 16 * (r & 1);
  }
  __device__ static void load(const QWeight& w, int row, int c, RawChunk& r) {
    const int nb = w.cols >> 5;
    r.a = *(const uint4*)(w.p0 + ((size_t)row * nb + c) * 16);
    r.d = *(const uint16_t*)(w.p1 + ((size_t)row * nb + c) * 2);
  }
  __device__ static void decode(const RawChunk& r, int c, float q[32], float sc[2], float of[2]) {
    const float d = __half2float(__ushort_as_half((uint16_t)r.d));
    sc[0] = sc[1] = d;
    of[0] = of[1] = 8.f * d;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t wv = u4_word(r.a, i);
      const uint32_t lo = wv & 0x0f0f0f0fu, hi = (wv >> 4) & 0x0f0f0f0fu;
      q[4 * i + 0] = (float)(lo & 0xff);
      q[4 * i + 1] = (float)((lo >> 8) & 0xff);
      q[4 * i + 2] = (float)((lo >> 16) & 0xff);
      q[4 * i + 3] = (float)(lo >> 24);
      q[16 + 4 * i + 0] = (float)(hi & 0xff);
      q[16 + 4 * i + 1] = (float)((hi >> 8) & 0xff);
      q[16 + 4 * i + 2] = (float)((hi >> 16) & 0xff);
      q[16 + 4 * i + 3] = (float)(hi >> 24);
    }
  }
};

// ------------------------------------------------------------------------------------ Q8_0
template <>
struct QFmt<QT_Q8_0> {
  static constexpr int W = 16, RUNS = 1, CHUNKS_PER_BLOCK = 2, BLOCK = 32;
  __device__ static int chunk_k0(int c, int run) { return c * 16; }
  __device__ static void run_pos(int r, int& c, int& s0) {
    c = r;
    s0 = 0;
  }
  __device__ static void load(const QWeight& w, int row, int c, RawChunk& r) {
    const int nb = w.cols >> 5;
    r.a = *(const uint4*)(w.p0 + (size_t)row * w.cols + c * 16);
    r.d = *(const uint16_t*)(w.p1 + ((size_t)row * nb + (c >> 1)) * 2);
  }
  __device__ static void decode(const RawChunk& r, int c, float q[16], float sc[1], float of[1]) {
    const float d = __half2float(__ushort_as_half((uint16_t)r.d));
    sc[0] = d;
    of[0] = 128.f * d;  // bytes re-biased to unsigned
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t u = u4_word(r.a, i) ^ 0x80808080u;
      q[4 * i + 0] = (float)(u & 0xff);
      q[4 * i + 1] = (float)((u >> 8) & 0xff);
      q[4 * i + 2] = (float)((u >> 16) & 0xff);
      q[4 * i + 3] = (float)(u >> 24);
    }
  }
};

// ------------------------------------------------------------------------------------ F16
template <>
struct QFmt<QT_F16> {
  static constexpr int W = 8, RUNS = 1, CHUNKS_PER_BLOCK = 1, BLOCK = 8;
  __device__ static int chunk_k0(int c, int run) { return c * 8; }
  __device__ static void load(const QWeight& w, int row, int c, RawChunk& r) {
    r.a = *(const uint4*)(w.p0 + ((size_t)row * w.cols + c * 8) * 2);
  }
  __device__ static void decode(const RawChunk& r, int c, float q[8], float sc[1], float of[1]) {
    sc[0] = 1.f;
    of[0] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t u = u4_word(r.a, i);
      q[2 * i] = __half2float(__ushort_as_half((uint16_t)(u & 0xffff)));
      q[2 * i + 1] = __half2float(__ushort_as_half((uint16_t)(u >> 16)));
    }
  }
};

// ------------------------------------------------------------------------------------ BF16
template <>
struct QFmt<QT_BF16> {
  static constexpr int W = 8, RUNS = 1, CHUNKS_PER_BLOCK = 1, BLOCK = 8;
  __device__ static int chunk_k0(int c, int run) { return c * 8; }
  __device__ static void load(const QWeight& w, int row, int c, RawChunk& r) {
    r.a = *(const uint4*)(w.p0 + ((size_t)row * w.cols + c * 8) * 2);
  }
  __device__ static void decode(const RawChunk& r, int c, float q[8], float sc[1], float of[1]) {
    sc[0] = 1.f;
    of[0] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint32_t u = u4_word(r.a, i);
      q[2 * i] = __uint_as_float(u << 16);
      q[2 * i + 1] = __uint_as_float(u & 0xffff0000u);
    }
  }
};


// ------------------------------------------------------------------------------------------
// Streaming decode interface used by the GEMV: per chunk scales, then 4 weights at a time
// (j = float4 index inside the chunk's W weights) so decoded values stay transient.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void ubytes4(uint32_t v, float q[4]) {
  q[0] = (float)(v & 0xff);
  q[1] = (float)((v >> 8) & 0xff);
  q[2] = (float)((v >> 16) & 0xff);
  q[3] = (float)(v >> 24);
}

template <int QT>
struct QStream;

template <>
struct QStream<QT_Q4_K> {
  __device__ static void scales(const RawChunk& r, int c, float* sc, float* of) {
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
  // j in 0..7: j<4 -> low nibbles of word j (run 0), j>=4 -> high nibbles of word j-4 (run 1)
  __device__ static void quad(const RawChunk& r, int c, int j, float q[4]) {
    const uint32_t wv = u4_word(r.a, j & 3);
    ubytes4(j < 4 ? (wv & 0x0f0f0f0fu) : ((wv >> 4) & 0x0f0f0f0fu), q);
  }
  // the 4 raw codes of quad j as the 4 bytes of one word
  __device__ static uint32_t word(const RawChunk& r, int c, int j) {
    const uint32_t wv = u4_word(r.a, j & 3);
    return j < 4 ? (wv & 0x0f0f0f0fu) : ((wv >> 4) & 0x0f0f0f0fu);
  }
};

template <>
struct QStream<QT_Q5_K> {
  __device__ static void scales(const RawChunk& r, int c, float* sc, float* of) {
    QStream<QT_Q4_K>::scales(r, c, sc, of);
  }
  __device__ static void quad(const RawChunk& r, int c, int j, float q[4]) {
    const int g = (c & 7) >> 1;
    const uint32_t wv = u4_word(r.a, j & 3), hv = u4_word(r.c, j & 3);
    const uint32_t nib = j < 4 ? (wv & 0x0f0f0f0fu) : ((wv >> 4) & 0x0f0f0f0fu);
    const uint32_t hb = (hv >> (2 * g + (j >= 4 ? 1 : 0))) & 0x01010101u;
    ubytes4(nib | (hb << 4), q);
  }
  __device__ static uint32_t word(const RawChunk& r, int c, int j) {
    const int g = (c & 7) >> 1;
    const uint32_t wv = u4_word(r.a, j & 3), hv = u4_word(r.c, j & 3);
    const uint32_t nib = j < 4 ? (wv & 0x0f0f0f0fu) : ((wv >> 4) & 0x0f0f0f0fu);
    return nib | (((hv >> (2 * g + (j >= 4 ? 1 : 0))) & 0x01010101u) << 4);
  }
};

template <>
struct QStream<QT_Q6_K> {
  __device__ static void scales(const RawChunk& r, int c, float* sc, float* of) {
    const float d = __half2float(__ushort_as_half((uint16_t)r.d));
    sc[0] = d * QFmt<QT_Q6_K>::sc_lo(r);
    sc[1] = d * QFmt<QT_Q6_K>::sc_hi(r);
    of[0] = 32.f * sc[0];
    of[1] = 32.f * sc[1];
  }
  __device__ static void quad(const RawChunk& r, int c, int j, float q[4]) {
    ubytes4(j < 4 ? QFmt<QT_Q6_K>::code_lo(r, j) : QFmt<QT_Q6_K>::code_hi(r, j & 3), q);
  }
  __device__ static uint32_t word(const RawChunk& r, int c, int j) {
    return j < 4 ? QFmt<QT_Q6_K>::code_lo(r, j) : QFmt<QT_Q6_K>::code_hi(r, j & 3);
  }
};

template <>
struct QStream<QT_Q4_0> {
  __device__ static void scales(const RawChunk& r, int c, float* sc, float* of) {
    const float d = __half2float(__ushort_as_half((uint16_t)r.d));
    sc[0] = sc[1] = d;
    of[0] = of[1] = 8.f * d;
  }
  __device__ static void quad(const RawChunk& r, int c, int j, float q[4]) {
    const uint32_t wv = u4_word(r.a, j & 3);
    ubytes4(j < 4 ? (wv & 0x0f0f0f0fu) : ((wv >> 4) & 0x0f0f0f0fu), q);
  }
  __device__ static uint32_t word(const RawChunk& r, int c, int j) {
    const uint32_t wv = u4_word(r.a, j & 3);
    return j < 4 ? (wv & 0x0f0f0f0fu) : ((wv >> 4) & 0x0f0f0f0fu);
  }
};

template <>
struct QStream<QT_Q8_0> {
  __device__ static void scales(const RawChunk& r, int c, float* sc, float* of) {
    const float d = __half2float(__ushort_as_half((uint16_t)r.d));
    sc[0] = d;
    of[0] = 128.f * d;
  }
  __device__ static void quad(const RawChunk& r, int c, int j, float q[4]) {
    ubytes4(u4_word(r.a, j) ^ 0x80808080u, q);
  }
  __device__ static uint32_t word(const RawChunk& r, int c, int j) { return u4_word(r.a, j) ^ 0x80808080u; }
};

template <>
struct QStream<QT_F16> {
  __device__ static void scales(const RawChunk& r, int c, float* sc, float* of) { sc[0] = 1.f; of[0] = 0.f; }
  __device__ static void quad(const RawChunk& r, int c, int j, float q[4]) {
    const uint32_t u0 = u4_word(r.a, 2 * j), u1 = u4_word(r.a, 2 * j + 1);
    q[0] = __half2float(__ushort_as_half((uint16_t)(u0 & 0xffff)));
    q[1] = __half2float(__ushort_as_half((uint16_t)(u0 >> 16)));
    q[2] = __half2float(__ushort_as_half((uint16_t)(u1 & 0xffff)));
    q[3] = __half2float(__ushort_as_half((uint16_t)(u1 >> 16)));
  }
};

template <>
struct QStream<QT_BF16> {
  __device__ static void scales(const RawChunk& r, int c, float* sc, float* of) { sc[0] = 1.f; of[0] = 0.f; }
  __device__ static void quad(const RawChunk& r, int c, int j, float q[4]) {
    const uint32_t u0 = u4_word(r.a, 2 * j), u1 = u4_word(r.a, 2 * j + 1);
    q[0] = __uint_as_float(u0 << 16);
    q[1] = __uint_as_float(u0 & 0xffff0000u);
    q[2] = __uint_as_float(u1 << 16);
    q[3] = __uint_as_float(u1 & 0xffff0000u);
  }
};

}  // namespace aios
