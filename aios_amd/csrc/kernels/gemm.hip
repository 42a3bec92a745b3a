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

constexpr int GM = 64, GN = 64, GK = 64;

__device__ __forceinline__ int swz(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }  // in 16-B units

__device__ __forceinline__ uint32_t pack_bf16(float a, float b) {
  return (uint32_t)f32_to_bf16(a) | ((uint32_t)f32_to_bf16(b) << 16);
}

// 16 contiguous weights W[row][k0 .. k0+15] (k0 % 16 == 0) -> 8 packed bf16 pairs
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

__global__ void __launch_bounds__(256) gemm_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) uint4 sA[2][GM * 8];
  __shared__ __attribute__((aligned(16))) uint4 sB[2][GN * 8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int m0 = blockIdx.y * GM, n0 = blockIdx.x * GN;
  const int lr = tid >> 2, lp = tid & 3;  // loader: row, 16-element part
  const int nk = a.K / GK;

  uint32_t ra[8], rb[8];
  auto load_tiles = [&](int kt) {
    const int k0 = kt * GK + 16 * lp;
    const int m = m0 + lr;
    if (m < a.M) {
      const uint4* src = (const uint4*)(a.A + (size_t)m * a.lda + k0);
      const uint4 x0 = src[0], x1 = src[1];
      ra[0] = x0.x; ra[1] = x0.y; ra[2] = x0.z; ra[3] = x0.w; ra[4] = x1.x; ra[5] = x1.y; ra[6] = x1.z; ra[7] = x1.w;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) ra[j] = 0;
    }
    const int n = n0 + lr;
    if (n < a.N) dequant16(a.w, n, k0, rb);
    else {
#pragma unroll
      for (int j = 0; j < 8; ++j) rb[j] = 0;
    }
  };
  auto store_tiles = [&](int buf) {
    sA[buf][swz(lr, 2 * lp)] = make_uint4(ra[0], ra[1], ra[2], ra[3]);
    sA[buf][swz(lr, 2 * lp + 1)] = make_uint4(ra[4], ra[5], ra[6], ra[7]);
    sB[buf][swz(lr, 2 * lp)] = make_uint4(rb[0], rb[1], rb[2], rb[3]);
    sB[buf][swz(lr, 2 * lp + 1)] = make_uint4(rb[4], rb[5], rb[6], rb[7]);
  };

  f32x16 acc;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;

  load_tiles(0);
  store_tiles(0);
  __syncthreads();
  const int arow = wm * 32 + (lane & 31), brow = wn * 32 + (lane & 31), half = lane >> 5;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tiles(kt + 1);  // global loads in flight during the MFMAs
#pragma unroll
    for (int ks = 0; ks < GK / 16; ++ks) {
      const uint4 av = sA[cur][swz(arow, 2 * ks + half)];
      const uint4 bv = sB[cur][swz(brow, 2 * ks + half)];
      bf16x8 af, bfv;
      __builtin_memcpy(&af, &av, 16);
      __builtin_memcpy(&bfv, &bv, 16);
      acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfv, acc, 0, 0, 0);
    }
    if (kt + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }
  // C/D map: col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
  const int n = n0 + wn * 32 + (lane & 31);
  if (n >= a.N) return;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
    if (m < a.M) {
      float* c = a.C + (size_t)m * a.ldc + n;
      if (a.accumulate) *c += acc[r];
      else *c = acc[r];
    }
  }
}

bool gemm_supports(int qt) {
  return qt == QT_Q4_K || qt == QT_Q5_K || qt == QT_Q6_K || qt == QT_Q4_0 || qt == QT_Q8_0 || qt == QT_F16 ||
         qt == QT_BF16;
}

void launch_gemm(const GemmArgs& a, hipStream_t st) {
  if (a.K % GK) throw std::runtime_error("gemm: K must be a multiple of 64");
  if (!gemm_supports(a.w.qtype)) throw std::runtime_error("gemm: unsupported weight format");
  dim3 grid((a.N + GN - 1) / GN, (a.M + GM - 1) / GM);
  hipLaunchKernelGGL(gemm_kernel, grid, dim3(256), 0, st, a);
}

}  // namespace aios
