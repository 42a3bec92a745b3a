// Causal flash attention for prefill (prefill column: "[T,H,hd]^2 causal
// flash-attention (MFMA)"), reading K/V from the bf16 KV cache the QKV epilogue just wrote, so a
// chunk of T new tokens attends over every cached position [0, start + T) of its slot.
//
// GQA packing: a workgroup owns one KV head and BQ = 128 / G query positions x all G query heads
// of that group = 128 query rows, so every K/V tile staged in LDS is used by 4x32 rows.  Wave w
// owns rows [32w, 32w + 32) (row = position * G + head).  Per 64-key tile:
//   S^T[key][row] = K Q^T   -- v_mfma_f32_32x32x16_bf16, K rows straight from LDS (A operand),
//                              Q^T from registers (B operand, loaded once, pre-scaled by
//                              scale*log2 e): the lane then holds one query row's 32 keys, so
//                              the row max / sum need one cross-half shuffle, not a 32-lane tree.
//   O^T[dim][row] += V^T P^T -- P^T is taken straight from the S^T accumulator registers: the key
//                              order of the k-dimension is permuted (rho below) to match the
//                              accumulator layout; V is staged ROW-major (16-byte stores) and the
//                              V^T fragment is two gfx950 transposed LDS reads (ds_read_b64_tr_b16:
//                              4 keys x 16 dims per 16-lane group, delivered column-major) at rho.
//                              (Round 2 staged V transposed with 2-byte stores: 32 ds_write_b16
//                              per thread per tile and the kernel's worst bank conflicts.)
// Online softmax per row in the log2 domain; fully masked rows cannot occur (key 0 <= pos).
// Output: bf16 [T][n_heads * hd] (the O-projection GEMM's A operand).
//
// VALU diet (rocprofv3 PMC at 2048 tokens: ~12 VALU instructions per MFMA, 129 TF/s): bf16 packing
// in hardware (v_cvt_pk_bf16_f32, not a software RNE with a NaN test), raw v_exp_f32 (ocml's
// exp2f adds range scaling), and the O rescale skipped when no row max of the wave moved.
#include "../common.h"
#include "../ops.h"
#include "gemm_common.h"

namespace aios {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x16_t __attribute__((ext_vector_type(16)));
// native vector type for register arrays (HIP's uint4 is a struct; arrays of it copied with
// memcpy defeat SROA and land in scratch)
typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));
typedef short v4i16_t __attribute__((ext_vector_type(4)));
typedef short v8i16_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float raw_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

constexpr int FP_KT = 64;  // keys per tile

typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));

// F8: the pool holds fp8 e4m3 codes (EngineConfig::kv_fp8): the tile loads move half the bytes and
// staging converts the codes to bf16 (exact; v_cvt_scalef32_pk_bf16_fp8 at scale 1 -- its scale
// operand is applied as a power of two, so the layer's K scale is folded into q and its V scale into
// the output instead) -- the LDS tiles and the MFMA math are the bf16 kernel's
template <int HD, int G, bool F8 = false>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) attn_prefill_kernel(AttnPrefillArgs a) {
  constexpr int BQ = 128 / G;          // query positions per workgroup
  constexpr int KS = HD / 16;          // k-steps of the S MFMA
  constexpr int OT = HD / 32;          // O^T accumulator tiles (32 dims each)
  constexpr int KROW = HD + 8;         // padded LDS row (bf16) of the K tile
  // padded LDS row (bf16) of the row-major V tile: a 16-lane transposed read takes 4 rows x 4
  // 8-byte column chunks and its 32-lane half two such groups 16 dims apart; rows HD + 32 elements
  // apart put the 4 rows 16 banks apart (mod 64) and the two groups 8 banks apart: conflict-free
  constexpr int VROW = HD + 32;
  // two LDS tile buffers (dynamic: 2 x 37 KB for HD 128), K then V in each
  constexpr int TILE_ELEMS = FP_KT * (KROW + VROW);
  extern __shared__ __attribute__((aligned(16))) bf16_t fp_smem[];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l32 = lane & 31, half = lane >> 5;
  // Causal balance: workgroup L (dispatch order, x fastest) and L + W/2 share a CU once the grid
  // fills every CU twice (the second pass lands on the CUs in the same order), so the first half
  // takes query blocks heaviest-first and the second half lightest-first: every CU gets blocks qb and
  // nx-1-qb, nx + 1 key tiles in all.  (Before, both of a CU's workgroups had the same qb: at 2k
  // tokens one CU did 64 tiles while the average was 33.)  Odd KV-head counts keep heaviest-first.
  const int nx = gridDim.x, ny = gridDim.y;
  int qb, kvh;
  if ((ny & 1) == 0) {
    const int L = blockIdx.y * nx + blockIdx.x, W2 = nx * ny / 2;
    if (L < W2) {
      qb = nx - 1 - L % nx;
      kvh = L / nx;
    } else {
      qb = (L - W2) % nx;
      kvh = ny / 2 + (L - W2) / nx;
    }
  } else {
    qb = nx - 1 - blockIdx.x;
    kvh = blockIdx.y;
  }
  const int T = a.T, start = a.start;
  const int t0 = qb * BQ;
  // this lane's query row (column of S^T / O^T)
  const int row = wave * 32 + l32;
  const int tq = t0 + row / G, g = row % G;
  const bool qvalid = tq < T;
  const int tql = qvalid ? tq : T - 1;
  const int qpos = start + tql;  // absolute position: keys <= qpos are visible
  const int h = kvh * G + g;

  // Q^T fragments (B operand): lane holds Q[row][16s + 8*half + 0..7] for s = 0..KS-1
  bf16x8_t qf[KS];
  {
    const float* qp = a.q + ((size_t)tql * a.n_heads + h) * HD + 8 * half;
    const float sc = a.scale * 1.4426950408889634f * (F8 ? a.kv_scale_k : 1.f);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const float4 x0 = *(const float4*)(qp + 16 * s), x1 = *(const float4*)(qp + 16 * s + 4);
      const uint4 u = make_uint4(pk_bf16(x0.x * sc, x0.y * sc), pk_bf16(x0.z * sc, x0.w * sc),
                                 pk_bf16(x1.x * sc, x1.y * sc), pk_bf16(x1.z * sc, x1.w * sc));
      __builtin_memcpy(&qf[s], &u, 16);
    }
  }

  f32x16_t o[OT];
#pragma unroll
  for (int i = 0; i < OT; ++i)
#pragma unroll
    for (int e = 0; e < 16; ++e) o[i][e] = 0.f;
  float m_run = -INFINITY, l_run = 0.f;

  // paged KV: 64-key tile kt lives in block bt[kt / 2] at key offset (kt % 2) * 64
  static_assert(KV_BLOCK == 2 * FP_KT, "two prefill key tiles per paged KV block");
  const int maxb = a.max_ctx / KV_BLOCK;
  const size_t blk_stride = (size_t)a.n_kv_heads * KV_BLOCK * HD;
  constexpr int ES = F8 ? 1 : 2;  // bytes per cached element
  const uint8_t* kc = (const uint8_t*)a.k_cache + (size_t)kvh * KV_BLOCK * HD * ES;
  const uint8_t* vc = (const uint8_t*)a.v_cache + (size_t)kvh * KV_BLOCK * HD * ES;
  const int last_pos = start + min(T, t0 + BQ) - 1;  // highest query position of the block
  const int ntiles = last_pos / FP_KT + 1;

  // tile loader: 64 keys x HD dims of K and of V, 16 B per piece, into register buffer r (2 of
  // them: tile kt + 2 is requested while tile kt is computed, so two tiles of math cover the
  // memory latency); stage() writes one buffer to an LDS tile buffer
  constexpr int PIECES = FP_KT * HD / 8;  // 16-B pieces per tensor per tile
  constexpr int PPT = PIECES / 256;        // per thread
  using PT = typename std::conditional<F8, u32x2_t, u32x4_t>::type;  // one 8-element piece
  struct Regs {
    PT k[PPT], v[PPT];
  };
  const int nt_last = ntiles - 1;
  auto load = [&](Regs& r, int kt) {
    kt = min(kt, nt_last);  // (clamped: the pipeline's tail requests are re-reads, never unmapped blocks)
    const size_t tbase = (size_t)kv_block(a.block_table, maxb, a.slot, kt * FP_KT) * blk_stride +
                         (size_t)(kt & 1) * FP_KT * HD;
    static_for<PPT>([&](auto I) {
      constexpr int i = decltype(I)::value;
      const int idx = tid + 256 * i, key = idx / (HD / 8), c = idx % (HD / 8);
      const size_t off = (tbase + (size_t)key * HD + c * 8) * ES;
      r.k[i] = *(const PT*)(kc + off);
      r.v[i] = *(const PT*)(vc + off);
    });
  };
  auto stage = [&](const Regs& r, bf16_t* buf) {
    bf16_t* sK = buf;
    bf16_t* sV = buf + FP_KT * KROW;
    static_for<PPT>([&](auto I) {
      constexpr int i = decltype(I)::value;
      const int idx = tid + 256 * i, key = idx / (HD / 8), c = idx % (HD / 8);
      if constexpr (F8) {
        auto cv = [](u32x2_t w) {
          u32x4_t o;
          o[0] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[0], 1.f, false));
          o[1] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[0], 1.f, true));
          o[2] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[1], 1.f, false));
          o[3] = __builtin_bit_cast(uint32_t, __builtin_amdgcn_cvt_scalef32_pk_bf16_fp8(w[1], 1.f, true));
          return o;
        };
        *(u32x4_t*)(sK + key * KROW + c * 8) = cv(r.k[i]);
        *(u32x4_t*)(sV + key * VROW + c * 8) = cv(r.v[i]);
      } else {
        *(u32x4_t*)(sK + key * KROW + c * 8) = r.k[i];
        *(u32x4_t*)(sV + key * VROW + c * 8) = r.v[i];
      }
    });
  };
  // one 64-key tile of math on LDS buffer buf (a tile past the last one -- the odd count's pad --
  // is fully masked: p = 0, alpha = 1)
  auto math = [&](const bf16_t* buf, int kt) {
    const bf16_t* sK = buf;
    const bf16_t* sV = buf + FP_KT * KROW;
    // ---- S^T = K Q^T for the tile's two 32-key halves
    f32x16_t st[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
#pragma unroll
      for (int e = 0; e < 16; ++e) st[t][e] = 0.f;
      const bf16_t* kr = sK + (t * 32 + l32) * KROW + 8 * half;
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const uint4 u = *(const uint4*)(kr + 16 * s);
        bf16x8_t kf;
        __builtin_memcpy(&kf, &u, 16);
        st[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(kf, qf[s], st[t], 0, 0, 0);
      }
    }
    // ---- causal mask + online softmax for this lane's row (32 of the 64 keys; partner lane^32)
    const int kbase = kt * FP_KT;
    const bool full = kbase + FP_KT - 1 <= qpos;
    float mx = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kbase + t * 32 + (r & 3) + 8 * (r >> 2) + 4 * half;
        if (!full && key > qpos) st[t][r] = -INFINITY;
        mx = fmaxf(mx, st[t][r]);
      }
    mx = fmaxf(mx, __shfl_xor(mx, 32, 64));
    const float mn = fmaxf(m_run, mx);  // finite: key 0 of tile 0 is always visible
    const float alpha = raw_exp2(m_run - mn);  // exp2(-inf) = 0 on the first tile
    float ps = 0.f;
    uint32_t pb[2][8];  // P^T as packed bf16 pairs, accumulator order
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        const float p0 = raw_exp2(st[t][r] - mn), p1 = raw_exp2(st[t][r + 1] - mn);
        ps += p0 + p1;
        pb[t][r >> 1] = pk_bf16(p0, p1);
      }
    ps += __shfl_xor(ps, 32, 64);
    l_run = l_run * alpha + ps;
    // the O rescale only when some row max of this wave moved (alpha == 1 on every lane otherwise)
    if (__any(mn != m_run)) {
#pragma unroll
      for (int i = 0; i < OT; ++i)
#pragma unroll
        for (int e = 0; e < 16; ++e) o[i][e] *= alpha;
    }
    m_run = mn;
    // ---- O^T += V^T P^T over 4 k-steps of 16 keys: step s uses accumulator half t = s/2,
    //      registers 8*(s%2) .. +7, i.e. keys rho = 16s + 4*half + {0..3} and 16s + 8 + 4*half + {0..3}
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int t = s >> 1, rb = (s & 1) * 4;
      const uint4 pu = make_uint4(pb[t][rb], pb[t][rb + 1], pb[t][rb + 2], pb[t][rb + 3]);
      bf16x8_t pf;
      __builtin_memcpy(&pf, &pu, 16);
#pragma unroll
      for (int i = 0; i < OT; ++i) {
        // lane 4q+p of each 16-lane group addresses key row (16s + 4 half + q), dims
        // 32 i + 16 (group & 1) + 4p .. +3; lane l32 receives dim 32 i + l32 of those 4 keys
        const bf16_t* va = sV + (16 * s + 4 * half + ((lane & 15) >> 2)) * VROW + i * 32 + 16 * ((lane >> 4) & 1) +
                           4 * (lane & 3);
        const v4i16_t x0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16_t*)va);
        const v4i16_t x1 =
            __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) v4i16_t*)(va + 8 * VROW));
        const v8i16_t xv = __builtin_shufflevector(x0, x1, 0, 1, 2, 3, 4, 5, 6, 7);
        bf16x8_t vf;
        __builtin_memcpy(&vf, &xv, 16);
        o[i] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(vf, pf, o[i], 0, 0, 0);
      }
    }
  };

  // Pipeline (round 5; was: one register buffer, stage + two barriers per tile, 130-150 us per
  // 2k-token layer): two register buffers A / B and two LDS tile buffers L0 / L1, ONE barrier per
  // tile.  Iteration kt computes tile kt from L[kt & 1] while tile kt + 2 is requested into the
  // register buffer just staged, then stages tile kt + 1 into the other LDS buffer (last read two
  // iterations ago, before the previous barrier) and barriers.  Branch-free: tiles run in pairs, an
  // odd count computes one fully masked pad tile.
  bf16_t* L0 = fp_smem;
  bf16_t* L1 = fp_smem + TILE_ELEMS;
  Regs A, B;
  load(A, 0);
  load(B, 1);
  stage(A, L0);
  __syncthreads();
  for (int kt = 0; kt < ntiles; kt += 2) {
    load(A, kt + 2);
    math(L0, kt);
    stage(B, L1);
    __syncthreads();
    load(B, kt + 3);
    math(L1, kt + 1);
    stage(A, L0);
    __syncthreads();
  }
  // ---- normalise and store bf16: O^T[dim][row], dim = 32 i + (r&3) + 8 (r>>2) + 4 half
  if (qvalid) {
    const float inv = (F8 ? a.kv_scale_v : 1.f) / l_run;
    bf16_t* op = a.out + (size_t)tq * a.ldo + (size_t)h * HD;
#pragma unroll
    for (int i = 0; i < OT; ++i)
#pragma unroll
      for (int r = 0; r < 16; r += 4) {
        const int d = i * 32 + 8 * (r >> 2) + 4 * half;
        const uint2 u = make_uint2(pk_bf16(o[i][r] * inv, o[i][r + 1] * inv), pk_bf16(o[i][r + 2] * inv, o[i][r + 3] * inv));
        *(uint2*)(op + d) = u;
      }
  }
}

bool attn_prefill_supports(int n_heads, int n_kv_heads, int head_dim) {
  if (n_kv_heads <= 0 || n_heads % n_kv_heads) return false;
  const int G = n_heads / n_kv_heads;
  return (head_dim == 64 || head_dim == 128) && (G == 1 || G == 2 || G == 4 || G == 8);
}

template <int HD, bool F8>
static void prefill_hd(const AttnPrefillArgs& a, int G, hipStream_t st) {
  const int BQ = 128 / G;
  dim3 grid((a.T + BQ - 1) / BQ, a.n_kv_heads);
  const size_t lds = (size_t)2 * FP_KT * ((HD + 8) + (HD + 32)) * sizeof(bf16_t);  // two K|V tile buffers
  switch (G) {
    case 1: hipLaunchKernelGGL((attn_prefill_kernel<HD, 1, F8>), grid, dim3(256), lds, st, a); break;
    case 2: hipLaunchKernelGGL((attn_prefill_kernel<HD, 2, F8>), grid, dim3(256), lds, st, a); break;
    case 4: hipLaunchKernelGGL((attn_prefill_kernel<HD, 4, F8>), grid, dim3(256), lds, st, a); break;
    case 8: hipLaunchKernelGGL((attn_prefill_kernel<HD, 8, F8>), grid, dim3(256), lds, st, a); break;
    default: throw std::runtime_error("attn_prefill: unsupported GQA group size");
  }
}

void launch_attn_prefill(const AttnPrefillArgs& a, hipStream_t st) {
  if (!attn_prefill_supports(a.n_heads, a.n_kv_heads, a.head_dim))
    throw std::runtime_error("attn_prefill: unsupported head configuration");
  if (a.T <= 0) return;
  if (a.start + a.T > a.max_ctx) throw std::runtime_error("attn_prefill: context overflow");
  const int G = a.n_heads / a.n_kv_heads;
  if (a.head_dim == 128) {
    if (a.kv_fp8) prefill_hd<128, true>(a, G, st);
    else prefill_hd<128, false>(a, G, st);
  } else {
    if (a.kv_fp8) prefill_hd<64, true>(a, G, st);
    else prefill_hd<64, false>(a, G, st);
  }
}

}  // namespace aios
