// Batched-decode GEMM on an LDS-DMA weight ring (M = 5..32 rows of bf16 activations):
//   C[M][N] = X[M][K] x W[N][K]^T,  W in the repacked Q4_K / Q6_K planes (qweight.h).
//
// Why (round 4, tools/skinny_probe.py at B = 8): the register-streamed skinny GEMM keeps one X
// chunk (4 load steps = 64 B per lane) of weights in flight, so its main loop runs at ~12 GB/s per
// CU (Mistral down: 16 us for 48 MB) and its 384 / 448-workgroup QKV / gate-up grids take two
// dispatch rounds: 1.5-2.2 TB/s where the batch-1 LDS-DMA engine streams 5.8.  Here the weight
// stream is the batch-1 engine's (gemv_lds.h): per CU one workgroup, two loader waves move every
// weight byte HBM -> LDS by buffer_load ... lds into a ring of R slots, R - 1 in flight, never
// waiting for compute; eight MFMA waves dequantise the slot in registers and multiply it with the
// X rows staged in the same slot (skinny's dequant-to-bf16 + v_mfma_f32_16x16x32_bf16 body, the
// weight rows as the A operand, no weight repack).
//
// Geometry: a workgroup owns one 128-row tile (8 waves x 16 rows) and a contiguous range of its
// 256-k superblocks (split-K when the tiles alone do not cover the CUs: one dispatch round, slices
// reduced in-launch by the tile's last arriver, skinny_epi.h).  One ring slot = one superblock of
// the tile: 128 rows x 128 B of codes (16-B units XOR-swizzled by row so the 16 lanes of a
// ds_read_b128 group hit distinct banks), the per-row scale records, Q6_K's high bits / f16 d, and
// the MP x 256 bf16 X rows of those k (skinny's xsw swizzle).  Steps are lock-stepped with raw
// s_barrier (in-flight LDS-DMA survives it) exactly as in the batch-1 engine.
#include "skinny_epi.h"

namespace aios {

constexpr int RG_RB = 8;  // MFMA waves: 128-row tiles
constexpr int RG_NL = 2;  // loader waves
constexpr int RG_SMAX = 8;  // K slices at most (the engine sizes its split-K slabs for 8: gemm_skinny_ws_bytes)
constexpr int RG_THREADS = (RG_RB + RG_NL) * 64;

// XR (M <= 8): the workgroup's X slice (8 rows x <= 4096 k, bf16, row stride + 16 B against bank
// conflicts) is staged ONCE into LDS ahead of the ring instead of riding in every slot -- at B = 8 the
// per-slot X made each CU move 1.4x the weight bytes and the bare ring (no compute) took 16.7 us for
// gate/up against the batch-1 engine's 13.5 (tools/gpu_r4_ringprobe.sh, profiles/lds_batched_r3.txt)
constexpr int RG_XR_ROWS = 8, RG_XR_KMAX = 4096;
#ifndef RG_RSUB
#define RG_RSUB 1
#endif
constexpr int RG_XR_BYTES = (RG_XR_ROWS * (RG_XR_KMAX + 8) * 2 + 255) / 256 * 256;

template <int QT, int MT, bool XR = false>
struct RgLayout {
  static constexpr bool Q6 = QT == QT_Q6_K;
  static constexpr int MP = 16 * MT;
  static constexpr int CODES = 128 * 128;           // 8 chunks x 16 B per row
  static constexpr int HI = Q6 ? 128 * 64 : 0;      // Q6_K: 8 B of high bits per chunk
  static constexpr int META = 128 * 16;             // Q4_K: scale/min record; Q6_K: 8 int8 scale pairs
  static constexpr int DQ = Q6 ? 512 : 0;           // Q6_K: the aligned dword holding the row's f16 d
  static constexpr int XB = XR ? 0 : MP * 256 * 2;  // X rows, bf16 (XR: resident, not in the slot)
  static constexpr int OFF_HI = CODES, OFF_META = OFF_HI + HI, OFF_D = OFF_META + META, OFF_X = OFF_D + DQ;
  static constexpr int SLOT = (OFF_X + XB + 255) / 256 * 256;
  // DMA instructions per slot: 1 KB each, Q6_K d as 4-byte pieces (256 B per instruction: a narrow
  // LDS-DMA lands lane i at base + 4 i whatever its width -- measured, a 2-byte one zero-fills)
  static constexpr int NI_CODES = 16, NI_HI = HI / 1024, NI_META = 2, NI_D = Q6 ? 2 : 0, NI_X = XB / 1024;
  static constexpr int TI = NI_CODES + NI_HI + NI_META + NI_D + NI_X;
  static constexpr int PL = (TI + RG_NL - 1) / RG_NL;  // per loader (exact: the vmcnt immediates)
  // (one slot below what fits: a smaller chip-wide prologue burst lands the first slot sooner, as
  // measured for the batch-1 engine, profiles/decode_mistral_rocprof_r4_final.txt)
  static constexpr int RFIT = std::min(6, (150 * 1024 - (XR ? RG_XR_BYTES : 0)) / SLOT);
  static constexpr int R = RFIT >= 4 ? RFIT - RG_RSUB : RFIT;
  static_assert(R >= 3 && (R - 2) * PL <= 63, "ring depth / vmcnt immediate");
};

__device__ __forceinline__ void rg_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
template <int N>
__device__ __forceinline__ void rg_vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt immediate");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// X unit swizzle of skinny (h(m) = (m ^ 2m) & 15 on 16-B units of a 512-B row)
__device__ __forceinline__ int rg_xh(int m) { return (m ^ (m << 1)) & 15; }

// Loader wave lw issues its PL instructions of slot s (superblock sb) into dst.
template <int QT, int MT, bool XR>
__device__ __forceinline__ void rg_dma_slot(const GemmQArgs& a, const QWeight& w, int row0, int nbk, int sb,
                                            uint8_t* dst, int lw) {
  using L = RgLayout<QT, MT, XR>;
  const int lane = threadIdx.x & 63;
  int issued = 0;
#pragma unroll
  for (int i = 0; i < L::TI; ++i) {
    if (i % RG_NL != lw) continue;
    const uint8_t* src;
    int region, width = 16;
    int j = i;
    if (j < L::NI_CODES) {  // codes: 8 rows per instruction, dest unit du of row r holds chunk du ^ (r & 7)
      const int r = 8 * j + (lane >> 3), du = lane & 7;
      src = w.p0 + (((size_t)(row0 + r) * nbk + sb) * 8 + (du ^ (r & 7))) * 16;
      region = j * 1024;
    } else if ((j -= L::NI_CODES) < L::NI_HI) {  // Q6_K high bits: 16 rows x 64 B, units swizzled by r & 3
      const int r = 16 * j + (lane >> 2), v = lane & 3;
      src = w.p1 + (((size_t)(row0 + r) * nbk + sb) * 8) * 8 + (v ^ (r & 3)) * 16;
      region = L::OFF_HI + j * 1024;
    } else if ((j -= L::NI_HI) < L::NI_META) {  // one 16-B record per row
      const int r = 64 * j + lane;
      if constexpr (L::Q6) src = w.p2 + (((size_t)(row0 + r) * nbk + sb) * 8) * 2;
      else src = w.p1 + ((size_t)(row0 + r) * nbk + sb) * 16;
      region = L::OFF_META + j * 1024;
    } else if ((j -= L::NI_META) < L::NI_D) {  // Q6_K f16 d: the 4-B aligned word holding it, per row
      const int r = 64 * j + lane;
      src = w.p3 + ((((size_t)(row0 + r) * nbk + sb) * 2) & ~(size_t)3);
      region = L::OFF_D + j * 256;
      width = 4;
    } else {  // X: dest unit u = (m, ud) holds k units ud ^ h(m) of row m (rows past M re-read row M-1)
      j -= L::NI_D;
      const int u = 64 * j + lane, m = u >> 5, ud = u & 31;
      const int mm = min(m, a.M - 1);
      src = (const uint8_t*)(a.A + (size_t)mm * a.lda + sb * 256 + 8 * (ud ^ rg_xh(m)));
      region = L::OFF_X + j * 1024;
    }
    auto* ldst = (__attribute__((address_space(3))) void*)(dst + region);
    if (region >= L::OFF_X) __builtin_amdgcn_global_load_lds((const void*)src, ldst, 16, 0, 0);  // X: L2-shared
    else if (width == 16) __builtin_amdgcn_global_load_lds((const void*)src, ldst, 16, 0, 2 /* nt */);
    else __builtin_amdgcn_global_load_lds((const void*)src, ldst, 4, 0, 2);
    ++issued;
  }
  // pad to PL (re-issue this wave's first codes piece into its own place)
  if (issued < L::PL) {
    const int r = 8 * lw + (lane >> 3), du = lane & 7;
    const uint8_t* src = w.p0 + (((size_t)(row0 + r) * nbk + sb) * 8 + (du ^ (r & 7))) * 16;
    for (; issued < L::PL; ++issued)
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)(dst + lw * 1024),
                                       16, 0, 2);
  }
}

// one MFMA wave: the 2 chunk steps of slot s (chunks q, q + 4 of its rows) into acc.
// (Measured alternatives, profiles/ring_gemm_r4.txt: every LDS read of the slot issued up front and
// waited for once -- neutral at B = 5 / 8, 2-3 % slower at B = 16 / 32; probe branches in the slot
// loop -- even one around this call -- cost up to ~3 us of gate/up, so the anatomy knobs are gone.)
// XR: X from the resident slice xr (row stride xst bf16, this superblock at k offset xk)
template <int QT, int MT, bool XR>
__device__ __forceinline__ void rg_compute_slot(const uint8_t* slot, int sb, int row0, int nbk, gf32x4 (&acc)[MT],
                                                const bf16_t* xr, int xst, int xk) {
  using L = RgLayout<QT, MT, XR>;
  constexpr bool MB = QT == QT_Q4_K;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int rr = lane & 15, q = lane >> 4;
  const int r = 16 * wave + rr;  // tile row
  const bf16_t* xs = (const bf16_t*)(slot + L::OFF_X);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int cc = q + 4 * u;  // chunk within the superblock
    RawChunk raw;
    raw.a = *(const uint4*)(slot + r * 128 + ((cc ^ (r & 7)) << 4));
    if constexpr (MB) {
      raw.b = *(const uint4*)(slot + L::OFF_META + r * 16);
    } else {
      const uint2 h = *(const uint2*)(slot + L::OFF_HI + r * 64 + (((cc >> 1) ^ (r & 3)) << 4) + 8 * (cc & 1));
      raw.b.x = h.x;
      raw.b.y = h.y;
      raw.c.x = *(const uint16_t*)(slot + L::OFF_META + r * 16 + 2 * cc);
      const uint32_t dw = *(const uint32_t*)(slot + L::OFF_D + 4 * r);
      raw.d = (dw >> (16 * (int)(((size_t)(row0 + r) * nbk + sb) & 1))) & 0xffffu;
    }
    const int c = sb * 8 + cc;
    float sc[2], of[2];
    QStream<QT>::scales(raw, c, sc, of);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t w0 = QStream<QT>::word(raw, c, 2 * i), w1 = QStream<QT>::word(raw, c, 2 * i + 1);
      asm volatile("" : "+v"(w0), "+v"(w1));  // one v_cvt_f32_ubyteN per byte
      float qv[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        qv[e] = (float)((w0 >> (8 * e)) & 0xff);
        qv[4 + e] = (float)((w1 >> (8 * e)) & 0xff);
      }
      const int run = i >> 1;
      uint32_t p[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) p[e] = pk_bf16(fmaf(sc[run], qv[2 * e], -of[run]), fmaf(sc[run], qv[2 * e + 1], -of[run]));
      gbf16x8 wf;
      __builtin_memcpy(&wf, p, 16);
      const int kl = QFmt<QT>::chunk_k0(cc, i >> 1) + 8 * (i & 1);  // k of this fragment within the superblock
#pragma unroll
      for (int mt = 0; mt < MT; ++mt) {
        const int m = 16 * mt + rr;
        uint4 xv;
        if constexpr (XR) xv = *(const uint4*)(xr + (rr & 7) * xst + xk + kl);  // lanes 8-15: duplicate columns
        else xv = *(const uint4*)(xs + m * 256 + (kl ^ (rg_xh(m) << 3)));
        gbf16x8 xf;
        __builtin_memcpy(&xf, &xv, 16);
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf, xf, acc[mt], 0, 0, 0);
      }
    }
  }
}

template <int QT, int MT, int EPI, bool XR>
__device__ __forceinline__ void rg_body(const GemmQArgs& a, int S, int rg, int sp, float* inv_s) {
  using L = RgLayout<QT, MT, XR>;
  extern __shared__ __attribute__((aligned(16))) uint8_t rg_smem[];
  __shared__ int last_flag;
  const int tid = threadIdx.x, wave = tid >> 6;
  const int ntile = a.N / 128;
  const int n0 = rg * 128;
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
  const int row0 = n0 - (s == 0 ? a.seg_n0[0] : (s == 1 ? a.seg_n0[1] : a.seg_n0[2]));
  const int nbk = a.K >> 8;
  const int sb0 = (int)((long)sp * nbk / S), sb1 = (int)((long)(sp + 1) * nbk / S);
  const int T = sb1 - sb0;  // ring steps (>= 1: S <= nbk)
  uint8_t* ring = rg_smem + (XR ? RG_XR_BYTES : 0);
  bf16_t* xr = (bf16_t*)rg_smem;
  const int xst = T * 256 + 8;  // XR: resident row stride (bf16)
  gf32x4 acc[MT];
#pragma unroll
  for (int mt = 0; mt < MT; ++mt) acc[mt] = gf32x4{0.f, 0.f, 0.f, 0.f};

  if (wave >= RG_RB) {
    // ---- loaders: R - 1 slots in flight, a slot refilled one step after it was consumed
    const int lw = wave - RG_RB;
    const int npro = min(T, L::R - 1);
    for (int t = 0; t < npro; ++t) rg_dma_slot<QT, MT, XR>(a, w, row0, nbk, sb0 + t, ring + (size_t)t * L::SLOT, lw);
    if (npro == L::R - 1) rg_vmcnt<(L::R - 2) * L::PL>();
    else rg_vmcnt<0>();
    rg_barrier();  // B1: slot 0 landed
    for (int t = 0; t < T; ++t) {
      if (t + L::R - 1 < T) {
        rg_dma_slot<QT, MT, XR>(a, w, row0, nbk, sb0 + t + L::R - 1, ring + (size_t)((t + L::R - 1) % L::R) * L::SLOT,
                                lw);
        rg_vmcnt<(L::R - 2) * L::PL>();  // slot t + 1 landed
      } else {
        rg_vmcnt<0>();
      }
      rg_barrier();
    }
  } else {
    if constexpr (XR) {
      // the MFMA waves stage the X slice (rows past M re-read row M - 1) while the loaders' prologue
      // slots are in flight: 8 x 16-B loads per thread per batch, then their LDS stores
      const int nu = RG_XR_ROWS * T * 32;  // 16-B units
      for (int u0 = tid; u0 < nu; u0 += 8 * RG_RB * 64) {
        uint4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int u = min(u0 + j * RG_RB * 64, nu - 1), m = u / (T * 32), k8 = u - m * (T * 32);
          v[j] = *(const uint4*)(a.A + (size_t)min(m, a.M - 1) * a.lda + sb0 * 256 + 8 * k8);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int u = u0 + j * RG_RB * 64;
          if (u < nu) {
            const int m = u / (T * 32), k8 = u - m * (T * 32);
            *(uint4*)(xr + m * xst + 8 * k8) = v[j];
          }
        }
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the slice in LDS before B1
    }
    rg_barrier();  // B1
    for (int t = 0; t < T; ++t) {
      rg_compute_slot<QT, MT, XR>(ring + (size_t)(t % L::R) * L::SLOT, sb0 + t, row0, nbk, acc, xr, xst, t * 256);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this slot's LDS reads done before it is refilled
      rg_barrier();
    }
  }
  rg_barrier();  // every wave past the ring: the LDS is scratch for the epilogue
  sk_epilogue<RG_RB, MT, EPI, RG_THREADS>(a, acc, n0, rg, sp, S, ntile, inv_s, inv_s != nullptr,
                                          (float*)rg_smem, last_flag);
}

// one launch for every tile; mixed formats (Q4_K_M QKV: Q|K Q4_K, V Q6_K): the last segment's
// tiles run the QT1 body
template <int QT0, int QT1, int MT, int EPI, bool XR>
__global__ void __launch_bounds__(RG_THREADS) gemm_ring_kernel(GemmQArgs a, int S) {
  kernarg_warm<sizeof(GemmQArgs) + sizeof(int)>();
  constexpr int MP = 16 * MT;
  const int ntile = a.N / 128, total = ntile * S;
  const int L = xcd_remap(blockIdx.x, total);
  const int rg = L / S, sp = L % S;
  // fused RMSNorm consumer: inv_s[m] from the producer's per-tile sums of squares (fixed order)
  __shared__ float inv_s[MP];
  const bool nrm = a.nrm_in != nullptr;
  if (nrm) {
    // all of a row's (<= 64, multiple-of-4) partial sums requested at once: a dependent load per
    // part held wave 0 -- a loader wave -- ~3 us before its first weight request
    for (int m = threadIdx.x; m < MP; m += RG_THREADS) {
      float t = 0.f;
      if (m < a.M) {
        const float4* p = (const float4*)(a.nrm_in + (size_t)m * a.nrm_parts);
        const int n4 = a.nrm_parts >> 2;
#pragma unroll
        for (int h = 0; h < 16; h += 8) {
          float4 v[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) v[j] = h + j < n4 ? p[h + j] : make_float4(0.f, 0.f, 0.f, 0.f);
#pragma unroll
          for (int j = 0; j < 8; ++j) t += (v[j].x + v[j].y) + (v[j].z + v[j].w);
        }
      }
      inv_s[m] = rsqrtf(t / (float)a.K + a.nrm_eps);
    }
    // ordered before the epilogue by the ring's barriers
  }
  float* is = nrm ? inv_s : nullptr;
  if constexpr (QT0 != QT1) {
    if (rg * 128 >= a.seg_n0[a.nseg - 1]) {
      rg_body<QT1, MT, EPI, XR>(a, S, rg, sp, is);
      return;
    }
  }
  rg_body<QT0, MT, EPI, XR>(a, S, rg, sp, is);
}

static int rg_env(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

template <int QT0, int QT1, int MT, bool XR>
static bool rg_launch(const GemmQArgs& a, hipStream_t st) {
  const int ntile = a.N / 128;
  const int nbk = a.K / 256;
  const int cus = device_cu_count();
  // one dispatch round: tiles x slices <= CUs (one 640-thread workgroup per CU, LDS-bound)
  int S = a.ksplit > 0 ? a.ksplit : std::max(1, cus / ntile);
  S = std::max(1, std::min({S, nbk, RG_SMAX}));
  if (S > 1 && (!a.ws || !a.cnt || a.cnt_len < ntile || a.ws_bytes < (size_t)S * 16 * MT * a.N * 4)) S = 1;
  if (XR && ((nbk + S - 1) / S) * 256 > RG_XR_KMAX) return false;  // the resident slice must fit
  const size_t lds = (size_t)(XR ? RG_XR_BYTES : 0) +
                     (size_t)std::max(RgLayout<QT0, MT, XR>::R * RgLayout<QT0, MT, XR>::SLOT,
                                      RgLayout<QT1, MT, XR>::R * RgLayout<QT1, MT, XR>::SLOT);
  const dim3 grid(ntile * S), block(RG_THREADS);
#define RG_GO(E) hipLaunchKernelGGL((gemm_ring_kernel<QT0, QT1, MT, E, XR>), grid, block, lds, st, a, S)
  switch (a.epi) {
    case GEPI_STORE: RG_GO(GEPI_STORE); break;
    case GEPI_QKV: RG_GO(GEPI_QKV); break;
    case GEPI_ACCUM: RG_GO(GEPI_ACCUM); break;
    case GEPI_ACCUM_NORM: RG_GO(GEPI_ACCUM_NORM); break;
    default: RG_GO(GEPI_SWIGLU_BF16); break;
  }
#undef RG_GO
  return true;
}

// AIOS_GEMM_RING: 1 (default) = the ring GEMM serves the batched-decode shapes it supports
// (M 5..32, Q4_K / Q6_K / mixed Q4_K|Q6_K, 128-row tiles, K % 256 == 0); 0 = skinny only
bool launch_gemm_ring(const GemmQArgs& a, hipStream_t st) {
  static const int on = rg_env("AIOS_GEMM_RING", 1);
  static const int min_m = rg_env("AIOS_GEMM_RING_MIN_M", 2);
  if (!on || a.M < min_m || a.M > 32 || a.N % 128 || a.K % 256 || a.lda % 8) return false;
  if (a.nrm_in && (a.nrm_parts <= 0 || a.nrm_parts > 64 || a.nrm_parts % 4)) return false;
  if (a.epi == GEPI_SWIGLU_BF16 && a.ldc % 2) return false;
  if (a.epi != GEPI_SWIGLU_BF16 && a.ldc % 4) return false;
  for (int s = 0; s < a.nseg; ++s)
    if (a.seg_n0[s] % 128 || a.seg[s].rows % 128) return false;
  // the split-RMSNorm producer's per-tile partials follow the skinny kernel's 128-row tiles too
  if (a.epi == GEPI_ACCUM_NORM && (!a.nrm_g || !a.nrm_out16 || !a.nrm_part || a.N / 128 != a.nrm_parts)) return false;
  const int qt0 = a.seg[0].qtype, qt1 = a.seg[a.nseg - 1].qtype;
  for (int s = 0; s + 1 < a.nseg; ++s)
    if (a.seg[s].qtype != qt0) return false;
  auto go = [&](auto mt, auto xr) {
    constexpr int MT = decltype(mt)::value;
    constexpr bool XR = decltype(xr)::value;
    if (qt0 == QT_Q4_K && qt1 == QT_Q4_K) return rg_launch<QT_Q4_K, QT_Q4_K, MT, XR>(a, st);
    if (qt0 == QT_Q6_K && qt1 == QT_Q6_K) return rg_launch<QT_Q6_K, QT_Q6_K, MT, XR>(a, st);
    if (qt0 == QT_Q4_K && qt1 == QT_Q6_K && (a.epi == GEPI_QKV || a.epi == GEPI_STORE))
      return rg_launch<QT_Q4_K, QT_Q6_K, MT, XR>(a, st);
    return false;
  };
  // AIOS_RING_XR (default 1): M <= 8 with the X slice resident in LDS (falls back when it does not fit)
  static const int xr_on = rg_env("AIOS_RING_XR", 1);
  if (a.M <= RG_XR_ROWS && xr_on && go(std::integral_constant<int, 1>{}, std::true_type{})) return true;
  if (a.M <= 16) return go(std::integral_constant<int, 1>{}, std::false_type{});
  return go(std::integral_constant<int, 2>{}, std::false_type{});
}

}  // namespace aios
