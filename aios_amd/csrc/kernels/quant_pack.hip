// Load-time weight repack (GGUF array-of-blocks -> per-row structure-of-arrays, see qweight.h)
// and element dequantizers (embedding rows, bf16 expansion for formats the GEMV does not
// stream natively, test oracles).  SURVEY.md §2.7 K12: "maps tensors to device memory, where
// the Q4_K/Q6_K blocks may be repacked into MFMA-friendly tiles".
#include "../common.h"
#include "../qweight.h"
#include "../ops.h"

namespace aios {

// GGUF Q4_K/Q5_K {d, dmin, scales[12]} -> repacked meta (qweight.h kq_field)
__device__ void write_kq_meta(const uint8_t* s, uint8_t* out) {
  uint32_t f[4];
  for (int g = 0; g < 4; ++g) {
    int sc0, m0, sc1, m1;
    kq_scale_min(2 * g, s + 4, sc0, m0);
    kq_scale_min(2 * g + 1, s + 4, sc1, m1);
    f[g] = (uint32_t)sc0 | ((uint32_t)sc1 << 6) | ((uint32_t)m0 << 12) | ((uint32_t)m1 << 18);
  }
  const uint32_t w[4] = {(uint32_t)s[0] | ((uint32_t)s[1] << 8) | ((uint32_t)s[2] << 16) | ((uint32_t)s[3] << 24),
                         f[0] | (f[1] << 24), (f[1] >> 8) | (f[2] << 16), (f[2] >> 16) | (f[3] << 8)};
  for (int k = 0; k < 16; ++k) out[k] = (uint8_t)(w[k >> 2] >> (8 * (k & 3)));
}

// one thread per block; byte-wise copies (load time only)
__global__ void repack_kernel(int qt, const uint8_t* __restrict__ raw, size_t nblocks, uint8_t* p0, uint8_t* p1,
                              uint8_t* p2, uint8_t* p3) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= nblocks) return;
  switch (qt) {
    case QT_Q4_K:
    case QT_Q5_K: {
      const bool q5 = qt == QT_Q5_K;
      const uint8_t* s = raw + i * (q5 ? 176 : 144);
      write_kq_meta(s, p1 + i * 16);
      if (q5)
        for (int k = 0; k < 32; ++k) p2[i * 32 + k] = s[16 + k];
      for (int k = 0; k < 128; ++k) p0[i * 128 + k] = s[(q5 ? 48 : 16) + k];
    } break;
    case QT_Q6_K: {
      // re-ordered into the Q4_K chunk order (see qweight.h): 6-bit code q[k] -> low nibble in
      // the Q4_K qs position of k, high 2 bits in a per-chunk {h0, h1} word pair.
      const uint8_t* s = raw + i * 210;
      const uint8_t* ql = s;
      const uint8_t* qh = s + 128;
      uint8_t q[256];
      for (int k = 0; k < 256; ++k) {
        const int n = k >> 7, r = k & 127, q4 = r >> 5, l = r & 31;
        const uint8_t lb = ql[64 * n + 32 * (q4 & 1) + l];
        const int nib = (q4 >> 1) ? (lb >> 4) : (lb & 0xF);
        q[k] = (uint8_t)(nib | (((qh[32 * n + l] >> (2 * q4)) & 3) << 4));
      }
      for (int j = 0; j < 128; ++j) {
        const int g = j >> 5, t = j & 31;
        p0[i * 128 + j] = (uint8_t)((q[64 * g + t] & 0xF) | ((q[64 * g + 32 + t] & 0xF) << 4));
      }
      for (int l = 0; l < 8; ++l) {
        const int k0 = 64 * (l >> 1) + 16 * (l & 1);
        for (int half = 0; half < 2; ++half) {
          uint32_t hw = 0;
          for (int j = 0; j < 4; ++j)
            for (int e = 0; e < 4; ++e) hw |= (uint32_t)((q[k0 + 32 * half + 4 * j + e] >> 4) & 3) << (8 * e + 2 * j);
          for (int bb = 0; bb < 4; ++bb) p1[i * 64 + l * 8 + 4 * half + bb] = (uint8_t)(hw >> (8 * bb));
        }
      }
      for (int l = 0; l < 8; ++l) {  // chunk l = 2g+h: (run 0, run 1) scales = sc[4g+h], sc[4g+2+h]
        const int g = l >> 1, h = l & 1;
        p2[i * 16 + 2 * l] = s[192 + 4 * g + h];
        p2[i * 16 + 2 * l + 1] = s[192 + 4 * g + 2 + h];
      }
      p3[i * 2] = s[208];
      p3[i * 2 + 1] = s[209];
    } break;
    case QT_Q4_0: {
      const uint8_t* s = raw + i * 18;
      p1[i * 2] = s[0];
      p1[i * 2 + 1] = s[1];
      for (int k = 0; k < 16; ++k) p0[i * 16 + k] = s[2 + k];
    } break;
    case QT_Q8_0: {
      const uint8_t* s = raw + i * 34;
      p1[i * 2] = s[0];
      p1[i * 2 + 1] = s[1];
      for (int k = 0; k < 32; ++k) p0[i * 32 + k] = s[2 + k];
    } break;
    default:
      break;
  }
}

void launch_repack(int qt, const void* raw, size_t nblocks, const QWeight& w, hipStream_t st) {
  const int T = 256;
  const int G = (int)((nblocks + T - 1) / T);
  hipLaunchKernelGGL(repack_kernel, dim3(G), dim3(T), 0, st, qt, (const uint8_t*)raw, nblocks, (uint8_t*)w.p0,
                     (uint8_t*)w.p1, (uint8_t*)w.p2, (uint8_t*)w.p3);
}

// ---------------------------------------------------------------------------------------------
// element dequant from the repacked layout
// ---------------------------------------------------------------------------------------------
__device__ float dq_elem(const QWeight& w, int row, int k) {
  switch (w.qtype) {
    case QT_Q4_K:
    case QT_Q5_K: {
      const int nb = w.cols >> 8, b = k >> 8, kk = k & 255, g = kk >> 6, hi = (kk >> 5) & 1, i = kk & 31;
      const size_t blk = (size_t)row * nb + b;
      const uint8_t* meta = w.p1 + blk * 16;
      const float d = h2f(*(const uint16_t*)meta), dmin = h2f(*(const uint16_t*)(meta + 2));
      const uint32_t* mw = (const uint32_t*)meta;
      const uint32_t f = kq_field(mw[1], mw[2], mw[3], g);
      const int sc = (f >> (6 * hi)) & 63, m = (f >> (12 + 6 * hi)) & 63;
      const uint8_t byte = w.p0[blk * 128 + 32 * g + i];
      int q = hi ? (byte >> 4) : (byte & 0xF);
      if (w.qtype == QT_Q5_K) q += ((w.p2[blk * 32 + i] >> (2 * g + hi)) & 1) << 4;
      return d * sc * q - dmin * m;
    }
    case QT_Q6_K: {
      const int nb = w.cols >> 8, b = k >> 8, kk = k & 255, g = kk >> 6, hi = (kk >> 5) & 1, i = kk & 31;
      const size_t blk = (size_t)row * nb + b;
      const uint8_t byte = w.p0[blk * 128 + 32 * g + i];
      const int nib = hi ? (byte >> 4) : (byte & 0xF);
      const int l = 2 * g + (i >> 4), j = (i & 15) >> 2, e = i & 3;
      const uint8_t* hp = w.p1 + blk * 64 + l * 8 + 4 * hi;
      const uint32_t hw = hp[0] | (hp[1] << 8) | (hp[2] << 16) | ((uint32_t)hp[3] << 24);
      const int q = (nib | (((hw >> (8 * e + 2 * j)) & 3) << 4)) - 32;
      const float d = h2f(*(const uint16_t*)(w.p3 + blk * 2));
      return d * (float)((const int8_t*)(w.p2 + blk * 16))[2 * l + hi] * q;
    }
    case QT_Q4_0: {
      const int nb = w.cols >> 5, b = k >> 5, j = k & 31;
      const size_t blk = (size_t)row * nb + b;
      const float d = h2f(*(const uint16_t*)(w.p1 + blk * 2));
      const uint8_t byte = w.p0[blk * 16 + (j & 15)];
      return d * ((j < 16 ? (byte & 0xF) : (byte >> 4)) - 8);
    }
    case QT_Q8_0: {
      const int nb = w.cols >> 5;
      const float d = h2f(*(const uint16_t*)(w.p1 + ((size_t)row * nb + (k >> 5)) * 2));
      return d * (float)(int8_t)w.p0[(size_t)row * w.cols + k];
    }
    case QT_F16:
      return h2f(((const uint16_t*)w.p0)[(size_t)row * w.cols + k]);
    case QT_BF16:
      return bf16_to_f32(((const uint16_t*)w.p0)[(size_t)row * w.cols + k]);
    case QT_F32:
      return ((const float*)w.p0)[(size_t)row * w.cols + k];
  }
  return 0.f;
}

// out[i][k] = W[rows[i]][k]   (rows == null -> row i);   optional scale
__global__ void get_rows_kernel(QWeight w, const int* __restrict__ rows, int nrows, float* __restrict__ out, int ldo,
                                float scale) {
  const int i = blockIdx.y;
  if (i >= nrows) return;
  const int r = rows ? rows[i] : i;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < w.cols; k += gridDim.x * blockDim.x)
    out[(size_t)i * ldo + k] = dq_elem(w, r, k) * scale;
}

// the same gather; workgroup (0, i) also prepares row i's StepPrep outputs
__global__ void get_rows_step_kernel(QWeight w, const int* __restrict__ rows, int nrows, float* __restrict__ out,
                                     int ldo, float scale, StepPrep sp) {
  const int i = blockIdx.y;
  if (i >= nrows) return;
  if (blockIdx.x == 0) {
    const int pos = sp.pos[i];
    if (threadIdx.x == 0) {
      const int slot = sp.slot ? sp.slot[i] : i;
      sp.kv[2 * i] = pos;
      sp.kv[2 * i + 1] = kv_block(sp.block_table, sp.maxb, slot, pos);
    }
    if (sp.rope_cs)
      for (int t = threadIdx.x; t < sp.half; t += blockDim.x)
        sp.rope[(size_t)i * sp.half + t] = sp.rope_cs[(size_t)pos * sp.half + t];
  }
  const int r = rows ? rows[i] : i;
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < w.cols; k += gridDim.x * blockDim.x)
    out[(size_t)i * ldo + k] = dq_elem(w, r, k) * scale;
}

void launch_get_rows_step(const QWeight& w, const int* rows, int nrows, float* out, int ldo, float scale,
                          const StepPrep& prep, hipStream_t st) {
  const int T = 256;
  const int gx = std::min(64, (w.cols + T - 1) / T);
  hipLaunchKernelGGL(get_rows_step_kernel, dim3(gx, nrows), dim3(T), 0, st, w, rows, nrows, out, ldo, scale, prep);
}

void launch_get_rows(const QWeight& w, const int* rows, int nrows, float* out, int ldo, float scale, hipStream_t st) {
  const int T = 256;
  const int gx = std::min(64, (w.cols + T - 1) / T);
  hipLaunchKernelGGL(get_rows_kernel, dim3(gx, nrows), dim3(T), 0, st, w, rows, nrows, out, ldo, scale);
}

__global__ void dequant_bf16_kernel(QWeight w, bf16_t* __restrict__ out) {
  const size_t n = (size_t)w.rows * w.cols;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int r = (int)(i / w.cols), k = (int)(i % w.cols);
    out[i] = f32_to_bf16(dq_elem(w, r, k));
  }
}

void launch_dequant_bf16(const QWeight& w, void* out, hipStream_t st) {
  hipLaunchKernelGGL(dequant_bf16_kernel, dim3(2048), dim3(256), 0, st, w, (bf16_t*)out);
}

// Raw (not repacked) formats -> bf16 at load time: the legacy 32-blocks (Q4_1 / Q5_0 / Q5_1), F32, and the
// 2- / 3-bit K-quants (Q2_K / Q3_K: Q2_K / Q3_K_M GGUFs run on the bf16 engines); none is on a hot path of
// the named models.  Q2_K / Q3_K element j of a 256-block: its 2-bit field is at bits 2 ((j >> 5) & 3) of
// quant byte 32 (j >> 7) + (j & 31), its scale is sub-block j >> 4, and (Q3_K) its high bit is bit j >> 5
// of byte j & 31 (aios_amd/gguf/quants.py dequant_q2_k / dequant_q3_k are the host references).
// IQ4_NL / IQ4_XS: 4-bit indices into these 16 levels, scaled by the block (IQ4_NL) or sub-block (IQ4_XS:
// d x (6-bit scale - 32), low 4 bits in nibble ib & 1 of byte 4 + ib / 2, top 2 at bits 2 ib of the u16 at
// byte 2) scale; the nibble order of a 32-element run is Q4_0's (quants.py dequant_iq4_nl / _xs)
__constant__ int8_t kIq4Levels[16] = {-127, -104, -83, -65, -49, -35, -22, -10, 1, 13, 25, 38, 53, 69, 89, 113};

__global__ void legacy_to_bf16_kernel(int qt, const uint8_t* __restrict__ raw, size_t n, bf16_t* __restrict__ out) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const size_t b = i >> 5;
    const int j = (int)(i & 31);
    float v = 0.f;
    if (qt == QT_IQ4_NL) {
      const uint8_t* s = raw + b * 18;
      const uint8_t byte = s[2 + (j & 15)];
      v = h2f(*(const uint16_t*)s) * (float)kIq4Levels[j < 16 ? (byte & 0xF) : (byte >> 4)];
    } else if (qt == QT_IQ4_XS) {
      const uint8_t* s = raw + (i >> 8) * 136;
      const int e = (int)(i & 255), ib = e >> 5, t = e & 31;
      const int ls = ((s[4 + (ib >> 1)] >> (4 * (ib & 1))) & 0xF) | (((*(const uint16_t*)(s + 2) >> (2 * ib)) & 3) << 4);
      const uint8_t byte = s[8 + 16 * ib + (t & 15)];
      v = h2f(*(const uint16_t*)s) * (float)(ls - 32) * (float)kIq4Levels[t < 16 ? (byte & 0xF) : (byte >> 4)];
    } else if (qt == QT_Q2_K || qt == QT_Q3_K) {
      const int e = (int)(i & 255), sub = e >> 4;
      const int q2 = (int)((qt == QT_Q2_K ? raw + (i >> 8) * 84 + 16 : raw + (i >> 8) * 110 + 32)[32 * (e >> 7) + (e & 31)] >>
                           (2 * ((e >> 5) & 3))) & 3;
      if (qt == QT_Q2_K) {
        const uint8_t* s = raw + (i >> 8) * 84;
        const float d = h2f(*(const uint16_t*)(s + 80)), dmin = h2f(*(const uint16_t*)(s + 82));
        v = d * (float)(s[sub] & 0xF) * (float)q2 - dmin * (float)(s[sub] >> 4);
      } else {
        const uint8_t* s = raw + (i >> 8) * 110;
        const int g = sub >> 2, k = sub & 3;
        const int lo4 = (s[96 + ((g & 1) ? 4 : 0) + k] >> ((g & 2) ? 4 : 0)) & 0xF;
        const int sc = (lo4 | (((s[104 + k] >> (2 * g)) & 3) << 4)) - 32;
        const int hb = (s[e & 31] >> (e >> 5)) & 1;
        v = h2f(*(const uint16_t*)(s + 108)) * (float)sc * (float)(q2 - (hb ? 0 : 4));
      }
    } else if (qt == QT_F32) {
      v = ((const float*)raw)[i];
    } else if (qt == QT_Q4_1) {
      const uint8_t* s = raw + b * 20;
      const float d = h2f(*(const uint16_t*)s), m = h2f(*(const uint16_t*)(s + 2));
      const uint8_t byte = s[4 + (j & 15)];
      v = d * (j < 16 ? (byte & 0xF) : (byte >> 4)) + m;
    } else if (qt == QT_Q5_0 || qt == QT_Q5_1) {
      const int hdr = qt == QT_Q5_0 ? 2 : 4;
      const uint8_t* s = raw + b * (qt == QT_Q5_0 ? 22 : 24);
      const float d = h2f(*(const uint16_t*)s);
      const uint32_t qh = s[hdr] | (s[hdr + 1] << 8) | (s[hdr + 2] << 16) | ((uint32_t)s[hdr + 3] << 24);
      const uint8_t byte = s[hdr + 4 + (j & 15)];
      int q;
      if (j < 16) q = (byte & 0xF) | (((qh >> j) << 4) & 0x10);
      else q = (byte >> 4) | ((qh >> (j - 16 + 12)) & 0x10);
      if (qt == QT_Q5_0) v = d * (q - 16);
      else v = d * q + h2f(*(const uint16_t*)(s + 2));
    }
    out[i] = f32_to_bf16(v);
  }
}

void launch_legacy_to_bf16(int qt, const void* raw, size_t n, void* out, hipStream_t st) {
  hipLaunchKernelGGL(legacy_to_bf16_kernel, dim3(2048), dim3(256), 0, st, qt, (const uint8_t*)raw, n, (bf16_t*)out);
}

// ---------------------------------------------------------------------------------------------
// Synthetic random-init weights generated directly in HBM (benchmarks: no 4 GB host round trip).
// Writes valid blocks of the repacked layout with bounded scales.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t hash32(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}

__global__ void fill_random_bytes_kernel(uint8_t* p, size_t n, uint64_t seed) {
  for (size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += (size_t)gridDim.x * blockDim.x * 4) {
    const uint32_t h = hash32(seed * 0x9E3779B97F4A7C15ULL + i);
    if (i + 4 <= n) *(uint32_t*)(p + i) = h;
    else for (size_t k = i; k < n; ++k) p[k] = (uint8_t)(h >> (8 * (k - i)));
  }
}

// f16 scales: value = amp * (0.5 + u) with u uniform in [0,1)
__global__ void fill_random_f16_kernel(uint16_t* p, size_t n, uint64_t seed, float amp, int stride_bytes, int offset) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float u = (hash32(seed + i * 7919) & 0xffffff) / 16777216.f;
    uint16_t* q = (uint16_t*)((uint8_t*)p + i * stride_bytes + offset);
    *q = __half_as_ushort(__float2half(amp * (0.5f + u)));
  }
}

// symmetric uniform [-amp, amp) as f16 (bf16=0) or bf16 (bf16=1)
__global__ void fill_random_sym16_kernel(uint16_t* p, size_t n, uint64_t seed, float amp, int bf16) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float u = (hash32(seed * 31 + i) & 0xffffff) / 16777216.f;
    const float v = amp * (2.f * u - 1.f);
    p[i] = bf16 ? f32_to_bf16(v) : __half_as_ushort(__float2half(v));
  }
}

// f32 vector (norm weights): 1 + amp*(2u-1)
__global__ void fill_random_f32_kernel(float* p, size_t n, uint64_t seed, float base, float amp) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float u = (hash32(seed * 131 + i) & 0xffffff) / 16777216.f;
    p[i] = base + amp * (2.f * u - 1.f);
  }
}

void fill_random_f32(float* p, size_t n, uint64_t seed, float base, float amp, hipStream_t st) {
  hipLaunchKernelGGL(fill_random_f32_kernel, dim3(256), dim3(256), 0, st, p, n, seed, base, amp);
}

void fill_random_weight(const QWeight& w, uint64_t seed, float amp, hipStream_t st) {
  const int nb = w.cols / (w.qtype == QT_Q4_K || w.qtype == QT_Q5_K || w.qtype == QT_Q6_K ? 256 : 32);
  const size_t nblk = (size_t)w.rows * nb;
  auto bytes = [&](const uint8_t* p, size_t n, uint64_t s) {
    hipLaunchKernelGGL(fill_random_bytes_kernel, dim3(4096), dim3(256), 0, st, (uint8_t*)p, n, s);
  };
  auto f16s = [&](const uint8_t* p, size_t n, float a, int stride, int off, uint64_t s) {
    hipLaunchKernelGGL(fill_random_f16_kernel, dim3(2048), dim3(256), 0, st, (uint16_t*)p, n, s, a, stride, off);
  };
  switch (w.qtype) {
    case QT_Q4_K:
      bytes(w.p0, nblk * 128, seed);
      bytes(w.p1, nblk * 16, seed + 1);
      f16s(w.p1, nblk, amp / 32.f, 16, 0, seed + 2);   // d
      f16s(w.p1, nblk, amp / 64.f, 16, 2, seed + 3);   // dmin
      break;
    case QT_Q5_K:
      bytes(w.p0, nblk * 128, seed);
      bytes(w.p1, nblk * 16, seed + 1);
      bytes(w.p2, nblk * 32, seed + 4);
      f16s(w.p1, nblk, amp / 64.f, 16, 0, seed + 2);
      f16s(w.p1, nblk, amp / 64.f, 16, 2, seed + 3);
      break;
    case QT_Q6_K:
      bytes(w.p0, nblk * 128, seed);
      bytes(w.p1, nblk * 64, seed + 1);
      bytes(w.p2, nblk * 16, seed + 2);
      f16s(w.p3, nblk, amp / 4096.f, 2, 0, seed + 3);
      break;
    case QT_Q4_0:
      bytes(w.p0, nblk * 16, seed);
      f16s(w.p1, nblk, amp / 8.f, 2, 0, seed + 1);
      break;
    case QT_Q8_0:
      bytes(w.p0, nblk * 32, seed);
      f16s(w.p1, nblk, amp / 128.f, 2, 0, seed + 1);
      break;
    case QT_F16:
    case QT_BF16:
      hipLaunchKernelGGL(fill_random_sym16_kernel, dim3(4096), dim3(256), 0, st, (uint16_t*)w.p0,
                         (size_t)w.rows * w.cols, seed, amp, w.qtype == QT_BF16 ? 1 : 0);
      break;
  }
}

}  // namespace aios
