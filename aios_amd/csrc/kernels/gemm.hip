// Prefill GEMM (M > 64): C[M][N] (+)= A[M][K] (bf16) x W[N][K]^T with W in any repacked quant
// format, dequantised tile-by-tile into LDS as bf16 and multiplied on the CDNA4 matrix cores
// (v_mfma_f32_32x32x16_bf16).  SURVEY.md §2.7 K3 prefill column ("MFMA GEMM", the reference's
// llama.cpp mul_mat_q inside llama-server, /root/reference/runtime/src/model_manager.rs:187-204)
// with the dequant fused into the matmul (BASELINE.json north star).  No resident bf16 copy of
// any weight exists: every weight byte is decoded in the workgroup that multiplies it.
//
// Workgroup tile BM x 128 x 64 (BM = 256 with 8 waves, 128 with 4 waves); each wave owns a 64x64
// output tile = 2x2 32x32 MFMA accumulators.  BK = 64 is one Q4_K/Q5_K 64-weight group (one qs
// group + its two 6-bit sub-block scales) and a quarter of a Q6_K super-block.  Per K-step every
// thread moves four 16-B chunks of A and dequantises 16 (BM=256) or 32 (BM=128) weights; with the
// large M tile the decode work per weight is amortised over 256 rows, so the VALU conversion
// (cvt_f32_ubyte + pk_fma + cvt_pk_bf16) runs beside the MFMAs instead of ahead of them.
//
// Pipeline: three register stages of raw (A, W) bytes -- the loads of K-step k+3 are issued at
// the top of step k, two MFMA phases before they are consumed -- and two LDS buffers, one
// barrier per K-step.  LDS images are [row][64 bf16] with the 16-B chunk of logical column c of
// row r at slot c ^ ((r >> 1) & 7): the 32x32x16 fragment reads (ds_read_b128, lane groups of 16
// rows) are then bank-conflict free (two 128-B rows per 256-B bank row).
// Tiles are mapped XCD-aware (bijective remap) with n fastest so one XCD keeps an A panel in L2.
#include "gemm_common.h"

namespace aios {

__device__ __forceinline__ int lds_slot(int row, int c) { return row * 8 + (c ^ ((row >> 1) & 7)); }

template <int QT, int BM, int BN, int EPI>
__global__ void __launch_bounds__(BM * BN / 64) gemm_big_kernel(GemmQArgs a) {
  constexpr int WN_ = BN / 64, NT = BM * BN / 64;  // waves along N; threads (one wave per 64x64)
  constexpr int AU = BM * 8 / NT;   // 16-B A chunks per thread per K-step
  constexpr int BU = BN * 4 / NT;   // 16-weight units per thread per K-step
  __shared__ __attribute__((aligned(16))) uint4 sA[2][BM * 8];
  __shared__ __attribute__((aligned(16))) uint4 sB[2][BN * 8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN_, wn = wave % WN_;
  const int nN = a.N / BN, nM = (a.M + BM - 1) / BM, total = nN * nM;
  const int L = xcd_remap(blockIdx.x, total);
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
  // split-K (gridDim.y > 1, only when the tile grid is below one workgroup per CU): K-steps
  // [kt0, kt1) of this workgroup, partial sums added atomically (the launcher zeroes C for STORE)
  const int nk_all = a.K / 64, S = gridDim.y;
  const int kt0 = (int)((long)blockIdx.y * nk_all / S), kt1 = (int)((long)(blockIdx.y + 1) * nk_all / S);

  gu32x4 ra0[AU], ra1[AU], ra2[AU];  // native vectors: arrays of HIP's uint4 struct land in scratch
  RawB rb0[BU], rb1[BU], rb2[BU];
#define GB_LOAD(kt_, RA, RB)                                                            \
  {                                                                                     \
    _Pragma("unroll") for (int i = 0; i < AU; ++i) {                                    \
      const int idx = tid + NT * i, r = idx >> 3, c = idx & 7;                          \
      const int m = min(m0 + r, a.M - 1); /* rows past M re-read the last row */        \
      RA[i] = *(const gu32x4*)(a.A + (size_t)m * a.lda + (kt_) * 64 + c * 8);           \
    }                                                                                   \
    _Pragma("unroll") for (int i = 0; i < BU; ++i) {                                    \
      const int idx = tid + NT * i, r = idx >> 2, p = idx & 3;                          \
      load_raw16<QT>(w, wrow0 + r, (kt_) * 64 + 16 * p, RB[i]);                        \
    }                                                                                   \
  }
#define GB_STORE(buf_, kt_, RA, RB)                                                     \
  {                                                                                     \
    _Pragma("unroll") for (int i = 0; i < AU; ++i) {                                    \
      const int idx = tid + NT * i, r = idx >> 3, c = idx & 7;                          \
      *(gu32x4*)&sA[buf_][lds_slot(r, c)] = RA[i];                                      \
    }                                                                                   \
    _Pragma("unroll") for (int i = 0; i < BU; ++i) {                                    \
      const int idx = tid + NT * i, r = idx >> 2, p = idx & 3;                          \
      uint32_t o[8];                                                                    \
      convert16<QT>(RB[i], (kt_) * 64 + 16 * p, o);                                     \
      sB[buf_][lds_slot(r, 2 * p)] = make_uint4(o[0], o[1], o[2], o[3]);                \
      sB[buf_][lds_slot(r, 2 * p + 1)] = make_uint4(o[4], o[5], o[6], o[7]);            \
    }                                                                                   \
  }

  gf32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][j][e] = 0.f;

  const int half = lane >> 5, l32 = lane & 31;
  auto mfma_step = [&](int cur) __attribute__((always_inline)) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      gbf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int r = wm * 64 + i * 32 + l32;
        const uint4 v = sA[cur][lds_slot(r, 2 * ks + half)];
        __builtin_memcpy(&af[i], &v, 16);
      }
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int r = wn * 64 + j * 32 + l32;
        const uint4 v = sB[cur][lds_slot(r, 2 * ks + half)];
        __builtin_memcpy(&bfr[j], &v, 16);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };
  // Loads are issued unconditionally (tile index clamped into [kt0, kt1): a re-read of the last
  // tile instead of a branch): a conditional load makes the outstanding-load count path dependent
  // and the compiler then drains with vmcnt(0) before each conversion.
  const int klast = kt1 - 1;
  GB_LOAD(kt0, ra0, rb0);
  GB_LOAD(min(kt0 + 1, klast), ra1, rb1);
  GB_LOAD(min(kt0 + 2, klast), ra2, rb2);
  GB_STORE(0, kt0, ra0, rb0);
  __syncthreads();
  // one K-step: reload the stage freed by the previous step with tile k+3, MFMAs on LDS tile k,
  // convert tile k+1 (stage RC) into the other LDS buffer, one barrier
#define GB_STEP(k_, RC_A, RC_B, RL_A, RL_B)                                             \
  {                                                                                     \
    const int cur = ((k_) - kt0) & 1;                                                   \
    GB_LOAD(min((k_) + 3, klast), RL_A, RL_B);                                          \
    mfma_step(cur);                                                                     \
    if ((k_) + 1 < kt1) GB_STORE(cur ^ 1, (k_) + 1, RC_A, RC_B);                        \
    __syncthreads();                                                                    \
  }
  int kt = kt0;
  for (; kt + 3 <= kt1; kt += 3) {
    GB_STEP(kt, ra1, rb1, ra0, rb0);
    GB_STEP(kt + 1, ra2, rb2, ra1, rb1);
    GB_STEP(kt + 2, ra0, rb0, ra2, rb2);
  }
  if (kt < kt1) GB_STEP(kt, ra1, rb1, ra0, rb0);
  if (kt + 1 < kt1) GB_STEP(kt + 1, ra2, rb2, ra1, rb1);
#undef GB_STEP
  // C/D map of the 32x32 accumulator: col = lane & 31, row = (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int n = n0 + wn * 64 + j * 32 + l32;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
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

#undef GB_LOAD
#undef GB_STORE

bool gemm_supports(int qt) {
  return qt == QT_Q4_K || qt == QT_Q5_K || qt == QT_Q6_K || qt == QT_Q4_0 || qt == QT_Q8_0 || qt == QT_F16 ||
         qt == QT_BF16;
}

static int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

template <int QT, int BM, int BN>
static void launch_big_tiles(const GemmQArgs& a, hipStream_t st) {
  constexpr int NT = BM * BN / 64;
  const int tiles = (a.N / BN) * ((a.M + BM - 1) / BM);
  const int cus = device_cu_count();
  // split-K only when the tile grid leaves most CUs idle (short prefill chunks)
  int S = a.ksplit;
  if (S <= 0) {
    const int per_cu = std::max(1, 163840 / ((BM + BN) * 256));  // LDS-resident workgroups per CU
    S = tiles >= cus * per_cu / 2 ? 1 : std::max(1, std::min(a.K / 64 / 8, (cus * per_cu) / tiles));
  }
  if (a.epi == GEPI_SWIGLU_BF16) S = 1;  // nonlinear epilogue needs the full sum
  S = std::max(1, std::min(S, a.K / 64));
  if (S > 1 && a.epi == GEPI_STORE)
    HIP_CHECK(hipMemset2DAsync(a.C, (size_t)a.ldc * 4, 0, (size_t)a.N * 4, a.M, st));
  const dim3 grid(tiles, S);
  switch (a.epi) {
    case GEPI_STORE: hipLaunchKernelGGL((gemm_big_kernel<QT, BM, BN, GEPI_STORE>), grid, dim3(NT), 0, st, a); break;
    case GEPI_ACCUM: hipLaunchKernelGGL((gemm_big_kernel<QT, BM, BN, GEPI_ACCUM>), grid, dim3(NT), 0, st, a); break;
    case GEPI_SWIGLU_BF16:
      hipLaunchKernelGGL((gemm_big_kernel<QT, BM, BN, GEPI_SWIGLU_BF16>), grid, dim3(NT), 0, st, a);
      break;
    default: throw std::runtime_error("gemm: bad epilogue");
  }
}

template <int QT>
static void launch_big(const GemmQArgs& a, hipStream_t st) {
  // 256-row tiles once the grid still covers the chip (dequant amortised over twice the rows),
  // 128-row tiles below that (AIOS_GEMM_BM forces one)
  static const int force_bm = env_int("AIOS_GEMM_BM", 0);
  const int cus = device_cu_count();
  bool n128 = a.N % 128 == 0;
  for (int s = 0; s < a.nseg; ++s)
    if (a.seg_n0[s] % 128 || a.seg[s].rows % 128) n128 = false;
  const int bn = n128 ? 128 : 64;
  const int t256 = (a.N / bn) * ((a.M + 255) / 256);
  const bool big = force_bm ? force_bm == 256 : t256 >= cus * 3 / 4;
  if (n128) {
    if (big) launch_big_tiles<QT, 256, 128>(a, st);
    else launch_big_tiles<QT, 128, 128>(a, st);
  } else {
    if (big) launch_big_tiles<QT, 256, 64>(a, st);
    else launch_big_tiles<QT, 128, 64>(a, st);
  }
}

// M <= 64: the skinny kernel (gemm_skinny.hip) streams the quantised weights straight into MFMA
// operand registers; returns false when the shape / workspace does not fit it
bool launch_gemm_skinny(const GemmQArgs& a, hipStream_t st);
bool gemm_skinny_mixed_ok(const GemmQArgs& a);
// M <= 32, Q4_K / Q6_K: the LDS-DMA ring GEMM (gemm_ring.hip); false when it does not serve the shape
bool launch_gemm_ring(const GemmQArgs& a, hipStream_t st);
// M >= 33, Q4_K / Q6_K / mixed / bf16 stacks: the LDS-DMA prefill GEMM (gemm_pf.hip)
bool launch_gemm_pf(const GemmQArgs& a, hipStream_t st);

static void launch_one(const GemmQArgs& a, hipStream_t st) {
  static const int skinny_max = env_int("AIOS_GEMM_SKINNY_MAX_M", 64);
  if (launch_gemm_ring(a, st)) return;
  if (a.M <= skinny_max && launch_gemm_skinny(a, st)) return;
  if (a.epi == GEPI_QKV || a.epi == GEPI_ACCUM_NORM || a.nrm_in)
    throw std::runtime_error("gemm: the QKV / fused-RMSNorm epilogues need the skinny (M <= 64) kernel");
  switch (a.seg[0].qtype) {
    case QT_Q4_K: launch_big<QT_Q4_K>(a, st); break;
    case QT_Q5_K: launch_big<QT_Q5_K>(a, st); break;
    case QT_Q6_K: launch_big<QT_Q6_K>(a, st); break;
    case QT_Q4_0: launch_big<QT_Q4_0>(a, st); break;
    case QT_Q8_0: launch_big<QT_Q8_0>(a, st); break;
    case QT_F16: launch_big<QT_F16>(a, st); break;
    case QT_BF16: launch_big<QT_BF16>(a, st); break;
    default: throw std::runtime_error("gemm: unsupported weight format");
  }
}

// Segments sharing a format go in one launch; a format change starts a new launch whose C
// pointer is shifted to the segment's first column (e.g. Q4_K Q/K + Q6_K V in Q4_K_M layers).
void launch_gemm_q(const GemmQArgs& a, hipStream_t st) {
  if (a.K % 64) throw std::runtime_error("gemm: K must be a multiple of 64");
  if (a.nseg < 1 || a.nseg > 3) throw std::runtime_error("gemm: 1..3 weight segments");
  if (a.M < 1) return;
  for (int s = 0; s < a.nseg; ++s) {
    if (!gemm_supports(a.seg[s].qtype)) throw std::runtime_error("gemm: unsupported weight format");
    if (a.seg[s].cols != a.K) throw std::runtime_error("gemm: weight cols != K");
    if (a.seg[s].rows % 64 || a.seg_n0[s] % 64) throw std::runtime_error("gemm: segment sizes must be multiples of 64");
  }
  if (a.N % 64) throw std::runtime_error("gemm: N must be a multiple of 64");
  // mixed formats in ONE skinny launch where supported (the Q4_K_M QKV stack)
  static const int skinny_max = env_int("AIOS_GEMM_SKINNY_MAX_M", 64);
  if (launch_gemm_ring(a, st)) return;  // the mixed Q4_K_M QKV stack in one ring launch
  if (launch_gemm_pf(a, st)) return;    // prefill chunks: the mixed stack in one launch too
  if (a.M <= skinny_max && gemm_skinny_mixed_ok(a) && launch_gemm_skinny(a, st)) return;
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
    b.col0 = a.col0 + c0;  // global column of the launch's first column (GEPI_QKV)
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
  a.ws = g.ws; a.ws_bytes = g.ws_bytes; a.cnt = g.cnt; a.cnt_len = g.cnt_len;
  launch_gemm_q(a, st);
}

}  // namespace aios
