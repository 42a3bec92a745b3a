// Fused dequant-GEMV for decode (M = batch <= 8): y[b][n] = sum_k W[n][k] * xn[b][k]
// (SURVEY.md §2.7 K3 "mul_mat_vec_q", fused with K2 RMSNorm prologue, K4/K5 RoPE + KV write,
//  K7 SwiGLU and K8 residual epilogues).
//
// Design (gfx950, wave64):
//  * 256-thread workgroup = 4 waves; each wave owns ROWS=2 adjacent output rows (a RoPE pair,
//    or an interleaved (gate_i, up_i) pair) and streams them with 16-B lane chunks straight to
//    VGPRs (decode weights are read once: the 'GEMV / M <= 16' row of the CDNA guide -- no LDS
//    round trip for weights).  U chunks x ROWS rows of loads are issued before any decode.
//  * x (optionally RMS-normalised) is staged once per workgroup in LDS in *chunk order* with a
//    float4 rotation swizzle, so each lane reads its W x-values with conflict-free ds_read_b128,
//    plus per-16-run sums of x (for the K-quant min/bias terms).  The x reads are shared by the
//    2 rows of a wave and the B batch columns reuse the decoded weights.
//  * One kernel per (format0, format1) pair: segment 0 (e.g. Q and K rows) and segment 1 (e.g.
//    V rows in Q6_K) can differ, so a mixed Q4_K_M QKV projection is still one launch.
//  * Epilogues: store / residual-add / SwiGLU / QKV(+bias, RoPE, bf16 KV-cache write).
#pragma once
#include <algorithm>

#include "../comm.h"
#include "../common.h"
#include "../gemv.h"
#include "../qweight.h"

namespace aios {

// Segment `s` of a kernel argument by VALUE, selected field by field: indexing a.seg[s] with a
// run-time s takes the address of the by-value kernarg struct and copies all of it to scratch
// (352 B of private segment per launch of the fp32 GEMV before this).
__device__ __forceinline__ QWeight seg_at(const GemvArgs& a, int s) {
  QWeight w;
  w.qtype = s == 0 ? a.seg[0].qtype : (s == 1 ? a.seg[1].qtype : a.seg[2].qtype);
  w.rows = s == 0 ? a.seg[0].rows : (s == 1 ? a.seg[1].rows : a.seg[2].rows);
  w.cols = s == 0 ? a.seg[0].cols : (s == 1 ? a.seg[1].cols : a.seg[2].cols);
  w.pad_ = 0;
  w.p0 = s == 0 ? a.seg[0].p0 : (s == 1 ? a.seg[1].p0 : a.seg[2].p0);
  w.p1 = s == 0 ? a.seg[0].p1 : (s == 1 ? a.seg[1].p1 : a.seg[2].p1);
  w.p2 = s == 0 ? a.seg[0].p2 : (s == 1 ? a.seg[1].p2 : a.seg[2].p2);
  w.p3 = s == 0 ? a.seg[0].p3 : (s == 1 ? a.seg[1].p3 : a.seg[2].p3);
  return w;
}
__device__ __forceinline__ int seg_row0_at(const GemvArgs& a, int s) {
  return s == 0 ? a.seg_row0[0] : (s == 1 ? a.seg_row0[1] : a.seg_row0[2]);
}


constexpr int GEMV_THREADS = 256;
constexpr int GEMV_WAVES = GEMV_THREADS / 64;
constexpr int GEMV_ROWS = 2;  // rows per wave
constexpr int GEMV_ROWS_PER_BLOCK = GEMV_WAVES * GEMV_ROWS;
constexpr int GEMV_LDS_FLOATS = 16384;  // 64 KiB of x per K tile

__device__ __forceinline__ int swz_pos(int c, int j, int F, int S) { return (j + (c >> S)) & (F - 1); }

template <int QT>
__device__ __forceinline__ void stage_x_tile(const float* __restrict__ x, int ldx, int B, int k0, int kt,
                                             const float* __restrict__ inv_rms, const float* __restrict__ nw,
                                             float* xl, float* xs) {
  using F_ = QFmt<QT>;
  constexpr int W = F_::W, F = W / 4, S = (F == 8 ? 1 : (F == 4 ? 2 : 3));
  const int tile_chunks = kt / W;
  if constexpr (W >= 16) {
    const int runs = kt / 16;  // one thread per 16-wide run
    for (int t = threadIdx.x; t < B * runs; t += blockDim.x) {
      const int b = t / runs, r = t - b * runs;
      int c, s0;
      F_::run_pos(r, c, s0);
      const float* src = x + (size_t)b * ldx + k0 + r * 16;
      float v[16];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float4 f = *(const float4*)(src + 4 * i);
        v[4 * i] = f.x; v[4 * i + 1] = f.y; v[4 * i + 2] = f.z; v[4 * i + 3] = f.w;
      }
      if (nw) {
        const float ir = inv_rms[b];
        const float* wp = nw + k0 + r * 16;
#pragma unroll
        for (int i = 0; i < 16; ++i) v[i] = v[i] * ir * wp[i];
      }
      float s = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) s += v[i];
      float* dst = xl + ((size_t)b * tile_chunks + c) * W;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int jj = s0 / 4 + j;
        *(float4*)(dst + 4 * swz_pos(c, jj, F, S)) = make_float4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
      }
      xs[(size_t)b * tile_chunks * F_::RUNS + c * F_::RUNS + (s0 >> 4)] = s;
    }
  } else {
    for (int t = threadIdx.x; t < B * tile_chunks; t += blockDim.x) {
      const int b = t / tile_chunks, c = t - b * tile_chunks;
      const float* src = x + (size_t)b * ldx + k0 + c * W;
      float v[W];
#pragma unroll
      for (int i = 0; i < W / 4; ++i) {
        float4 f = *(const float4*)(src + 4 * i);
        v[4 * i] = f.x; v[4 * i + 1] = f.y; v[4 * i + 2] = f.z; v[4 * i + 3] = f.w;
      }
      if (nw) {
        const float ir = inv_rms[b];
        const float* wp = nw + k0 + c * W;
#pragma unroll
        for (int i = 0; i < W; ++i) v[i] = v[i] * ir * wp[i];
      }
      float* dst = xl + ((size_t)b * tile_chunks + c) * W;
#pragma unroll
      for (int j = 0; j < F; ++j)
        *(float4*)(dst + 4 * swz_pos(c, j, F, S)) = make_float4(v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]);
    }
  }
}

// rows (row0, row0+1) of w over the K-tile [k0, k0+kt)
template <int QT, int B, int U>
__device__ __forceinline__ void gemv_tile(const QWeight& w, int row0, int k0, int kt, const float* xl,
                                          const float* xs, float (&acc)[GEMV_ROWS][B]) {
  using F_ = QFmt<QT>;
  using S_ = QStream<QT>;
  constexpr int W = F_::W, F = W / 4, S = (F == 8 ? 1 : (F == 4 ? 2 : 3)), R = F_::RUNS;
  const int lane = threadIdx.x & 63;
  const int c_base = k0 / W;
  const int tile_chunks = kt / W;
  for (int it = 0; it < tile_chunks; it += 64 * U) {
    RawChunk raw[U][GEMV_ROWS];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = it + u * 64 + lane;
      if (c < tile_chunks) {
#pragma unroll
        for (int r = 0; r < GEMV_ROWS; ++r) F_::load(w, row0 + r, c_base + c, raw[u][r]);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int c = it + u * 64 + lane;
      if (c < tile_chunks) {
        const int cg = c_base + c;
        float sc[GEMV_ROWS][R], of[GEMV_ROWS][R];
#pragma unroll
        for (int r = 0; r < GEMV_ROWS; ++r) S_::scales(raw[u][r], cg, sc[r], of[r]);
#pragma unroll
        for (int b = 0; b < B; ++b) {
          const float* xc = xl + ((size_t)b * tile_chunks + c) * W;
          float part[GEMV_ROWS][R];
#pragma unroll
          for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
            for (int rr = 0; rr < R; ++rr) part[r][rr] = 0.f;
#pragma unroll
          for (int j = 0; j < F; ++j) {
            const float4 xv = *(const float4*)(xc + 4 * swz_pos(c, j, F, S));
            constexpr int JPR = 16 / 4;  // float4s per 16-run
            const int rr = (R == 1) ? 0 : (j / JPR);
#pragma unroll
            for (int r = 0; r < GEMV_ROWS; ++r) {
              float q[4];
              S_::quad(raw[u][r], cg, j, q);
              part[r][rr] = fmaf(q[0], xv.x, part[r][rr]);
              part[r][rr] = fmaf(q[1], xv.y, part[r][rr]);
              part[r][rr] = fmaf(q[2], xv.z, part[r][rr]);
              part[r][rr] = fmaf(q[3], xv.w, part[r][rr]);
            }
          }
          if constexpr (W >= 16) {
            const float* xsc = xs + (size_t)b * tile_chunks * R + c * R;
            float xsv[R];
#pragma unroll
            for (int rr = 0; rr < R; ++rr) xsv[rr] = xsc[rr];
#pragma unroll
            for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
              for (int rr = 0; rr < R; ++rr) acc[r][b] += sc[r][rr] * part[r][rr] - of[r][rr] * xsv[rr];
          } else {
#pragma unroll
            for (int r = 0; r < GEMV_ROWS; ++r) acc[r][b] += part[r][0];
          }
        }
      }
    }
  }
}

__device__ __forceinline__ void gemv_epilogue(const GemvArgs& a, int grow, int b, float v0, float v1) {
  const int nrow = a.row_base + a.N;
  switch (a.epi) {
    case EPI_STORE: {
      float* y = a.y + (size_t)b * a.ldy;
      y[grow] = v0;
      if (grow + 1 < nrow) y[grow + 1] = v1;
    } break;
    case EPI_RESID: {
      float* y = a.y + (size_t)b * a.ldy;
      y[grow] += v0;
      if (grow + 1 < nrow) y[grow + 1] += v1;
    } break;
    case EPI_SWIGLU: {
      const float g = v0, u = v1;  // rows (2i, 2i+1) = (gate_i, up_i)
      const float h = g / (1.f + __expf(-g)) * u;
      if (a.y16) a.y16[(size_t)b * a.ldy + (grow >> 1)] = f32_to_bf16(h);
      else a.y[(size_t)b * a.ldy + (grow >> 1)] = h;
    } break;
    case EPI_QKV: {
      if (a.bias) { v0 += a.bias[grow]; v1 += a.bias[grow + 1]; }
      const int hd = a.head_dim, qd = a.q_dim, kvd = a.kv_dim;
      const int pos = a.pos[b];
      const int slot = a.slot ? a.slot[b] : b;
      int part, r;
      if (grow < qd) { part = 0; r = grow; }
      else if (grow < qd + kvd) { part = 1; r = grow - qd; }
      else { part = 2; r = grow - qd - kvd; }
      const int head = r / hd, lr = r - head * hd, p = lr >> 1;
      int da, db;
      if (part == 2) { da = lr; db = lr + 1; }
      else if (a.rope_neox) { da = p; db = p + (hd >> 1); }
      else { da = 2 * p; db = 2 * p + 1; }
      if (part < 2) {
        float sn, cs;
        if (a.rope_cs) {
          const float2 t = a.rope_cs[(size_t)pos * (hd >> 1) + p];
          cs = t.x; sn = t.y;
        } else {
          const float theta = (float)pos * powf(a.rope_base, -2.f * (float)p / (float)hd);
          sincosf(theta, &sn, &cs);
        }
        const float o0 = v0 * cs - v1 * sn, o1 = v0 * sn + v1 * cs;
        v0 = o0; v1 = o1;
      }
      if (part == 0) {
        float* q = a.y + (size_t)b * a.ldy + head * hd;
        q[da] = v0; q[db] = v1;
      } else {
        bf16_t* cache = pick_ptr(part == 1, a.k_cache, a.v_cache);
        const size_t base = kv_offset(a.block_table, a.max_ctx / KV_BLOCK, slot, a.n_kv_heads, head, pos, hd);
        kv_store_pair(cache, base + da, base + db, v0, v1, a.kv_fp8, part == 1 ? a.kv_inv_k : a.kv_inv_v);
      }
    } break;
    default:
      __builtin_trap();  // an epilogue these kernels do not do (EPI_TP_RESID: row-pair kernel only)
  }
}

template <int QT, int B, int U>
__device__ __forceinline__ void gemv_seg(const GemvArgs& a, const QWeight& w, int local_row, bool active,
                                         const float* inv_rms, float* xl, float* xs, float (&acc)[GEMV_ROWS][B]) {
  const int K = a.K, kt_max = a.kt_max;
  for (int k0 = 0; k0 < K; k0 += kt_max) {
    const int kt = min(kt_max, K - k0);
    if (k0 > 0) __syncthreads();
    stage_x_tile<QT>(a.x, a.ldx, a.B, k0, kt, inv_rms, a.norm_w, xl, xs);
    __syncthreads();
    if (active) gemv_tile<QT, B, U>(w, local_row, k0, kt, xl, xs, acc);
  }
}

template <int QT0, int QT1, int B, int U>
__global__ void __launch_bounds__(GEMV_THREADS) gemv_kernel(GemvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* red = smem;  // 64 floats: block-reduction scratch + inv_rms[16..]
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int row_blk = blockIdx.x * GEMV_ROWS_PER_BLOCK;
  // segments are row ranges (multiples of 8 rows) so a workgroup never straddles two
  int sidx = 0;
#pragma unroll
  for (int s = 1; s < GEMV_MAX_SEGS; ++s)
    if (s < a.nseg && row_blk >= a.seg_row0[s]) sidx = s;
  const int seg_row0 = seg_row0_at(a, sidx);
  const int K = a.K;
  const int nb_act = a.B;  // real batch (<= B; padding columns are never stored)

  float* inv_rms = red + 16;
  if (a.norm_w) {
    for (int b = 0; b < nb_act; ++b) {
      float s = 0.f;
      const float* xb = a.x + (size_t)b * a.ldx;
      for (int k = threadIdx.x * 4; k < K; k += GEMV_THREADS * 4) {
        const float4 v = *(const float4*)(xb + k);
        s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
      }
      s = block_sum(s, red);
      if (threadIdx.x == 0) inv_rms[b] = rsqrtf(s / (float)K + a.eps);
      __syncthreads();
    }
  }

  float acc[GEMV_ROWS][B];
#pragma unroll
  for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
    for (int b = 0; b < B; ++b) acc[r][b] = 0.f;
  float* xl = smem + 64;
  float* xs = xl + B * a.kt_max;
  const int local_row = row_blk - seg_row0 + wave * GEMV_ROWS;
  const bool active = (row_blk + wave * GEMV_ROWS) < a.N;
  // the type-0 segment(s) come first; type-1 is only ever the last segment
  if (QT0 == QT1 || sidx < a.nseg - 1 || a.nseg == 1)
    gemv_seg<QT0, B, U>(a, seg_at(a, sidx), local_row, active, inv_rms, xl, xs, acc);
  else
    gemv_seg<QT1, B, U>(a, seg_at(a, sidx), local_row, active, inv_rms, xl, xs, acc);
  if (!active) return;

#pragma unroll
  for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
    for (int b = 0; b < B; ++b) acc[r][b] = wave_sum(acc[r][b]);
  if (lane >= nb_act) return;
  float v0 = 0.f, v1 = 0.f;  // lane b handles batch column b
#pragma unroll
  for (int b = 0; b < B; ++b)
    if (lane == b) { v0 = acc[0][b]; v1 = acc[1][b]; }
  gemv_epilogue(a, a.row_base + row_blk + wave * GEMV_ROWS, lane, v0, v1);
}


// =============================================================================================
// Persistent, software-pipelined GEMV (v2).
//
// The v1 kernel above gives every 8-row workgroup its own RMSNorm + x-staging prologue; for the
// Mistral gate/up projection that is 7168 prologues re-reading 32 KB each (more L2 traffic than
// the 132 MB of weights) and each workgroup's weight loads only start after it.  Here:
//  * grid = min(row groups, CUs x occupancy): each workgroup stages x ONCE, then walks its
//    row-pairs grid-stride (pair p = blk*WAVES + wave + i*grid*WAVES);
//  * the first pair's weight loads are issued before the prologue (they do not depend on x);
//  * work items (pair, K-iteration) are double-buffered in registers: the next item's loads are
//    in flight while the current one is decoded (hipcc's counted vmcnt waits only for the
//    older group), so each wave keeps two items (~2 x 8 KB for Q4_K) in flight at all times.
// Requires B*K floats of x (+ run sums) to fit the LDS budget; the launcher falls back to v1.
// =============================================================================================
constexpr int GP_THREADS = 256;
constexpr int GP_WAVES = GP_THREADS / 64;

template <int QT, int U>
__device__ __forceinline__ void gp_load(const QWeight& w, int lrow, int it, int nch, RawChunk (&r)[U][GEMV_ROWS]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = (it * U + u) * 64 + lane;
    if (c < nch) {
#pragma unroll
      for (int rr = 0; rr < GEMV_ROWS; ++rr) QFmt<QT>::load(w, lrow + rr, c, r[u][rr]);
    }
  }
}

template <int QT, int B, int U>
__device__ __forceinline__ void gp_compute(const RawChunk (&raw)[U][GEMV_ROWS], int it, int nch, const float* xl,
                                           const float* xs, float (&acc)[GEMV_ROWS][B]) {
  using F_ = QFmt<QT>;
  using S_ = QStream<QT>;
  constexpr int W = F_::W, F = W / 4, S = (F == 8 ? 1 : (F == 4 ? 2 : 3)), R = F_::RUNS;
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int c = (it * U + u) * 64 + lane;
    if (c < nch) {
      float sc[GEMV_ROWS][R], of[GEMV_ROWS][R];
#pragma unroll
      for (int r = 0; r < GEMV_ROWS; ++r) S_::scales(raw[u][r], c, sc[r], of[r]);
#pragma unroll
      for (int b = 0; b < B; ++b) {
        const float* xc = xl + ((size_t)b * nch + c) * W;
        float part[GEMV_ROWS][R];
#pragma unroll
        for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
          for (int rr = 0; rr < R; ++rr) part[r][rr] = 0.f;
#pragma unroll
        for (int j = 0; j < F; ++j) {
          const float4 xv = *(const float4*)(xc + 4 * swz_pos(c, j, F, S));
          const int rr = (R == 1) ? 0 : (j / 4);
#pragma unroll
          for (int r = 0; r < GEMV_ROWS; ++r) {
            float q[4];
            S_::quad(raw[u][r], c, j, q);
            part[r][rr] = fmaf(q[0], xv.x, part[r][rr]);
            part[r][rr] = fmaf(q[1], xv.y, part[r][rr]);
            part[r][rr] = fmaf(q[2], xv.z, part[r][rr]);
            part[r][rr] = fmaf(q[3], xv.w, part[r][rr]);
          }
        }
        if constexpr (W >= 16) {
          const float* xsc = xs + (size_t)b * nch * R + c * R;
          float xsv[R];
#pragma unroll
          for (int rr = 0; rr < R; ++rr) xsv[rr] = xsc[rr];
#pragma unroll
          for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
            for (int rr = 0; rr < R; ++rr) acc[r][b] += sc[r][rr] * part[r][rr] - of[r][rr] * xsv[rr];
        } else {
#pragma unroll
          for (int r = 0; r < GEMV_ROWS; ++r) acc[r][b] += part[r][0];
        }
      }
    }
  }
}

template <int QT0, int QT1, int B, int U>
__global__ void __launch_bounds__(GP_THREADS) gemv_persistent(GemvArgs a) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* red = smem;
  float* inv_rms = red + 16;
  constexpr bool MIXED = QT0 != QT1;
  constexpr int W0 = QFmt<QT0>::W, W1 = QFmt<QT1>::W;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int K = a.K;
  const int npairs = a.N >> 1;
  const int nch0 = K / W0, nch1 = K / W1;
  const int nit0 = (nch0 + 64 * U - 1) / (64 * U), nit1 = (nch1 + 64 * U - 1) / (64 * U);
  const int stride = gridDim.x * GP_WAVES;
  // LDS: [red 64][x layout 0: B*K][sums 0: B*K/16][x layout 1][sums 1]
  float* xl0 = smem + 64;
  float* xs0 = xl0 + B * K;
  constexpr bool SEP = !same_xlayout<QT0, QT1>;
  float* xl1 = SEP ? xs0 + B * K / 16 : xl0;
  float* xs1 = SEP ? xl1 + B * K : xs0;

  auto info = [&](int p, int& lrow, bool& t1, QWeight& w) {
    const int row = 2 * p;
    int s = 0;
#pragma unroll
    for (int k = 1; k < GEMV_MAX_SEGS; ++k)
      if (k < a.nseg && row >= a.seg_row0[k]) s = k;
    lrow = row - seg_row0_at(a, s);
    t1 = MIXED && (s == a.nseg - 1) && a.nseg > 1;
    w = seg_at(a, s);
  };
  auto load = [&](int p, int it, RawChunk (&r)[U][GEMV_ROWS]) {
    int lrow;
    bool t1;
    QWeight w;
    info(p, lrow, t1, w);
    if (MIXED && t1) gp_load<QT1, U>(w, lrow, it, nch1, r);
    else gp_load<QT0, U>(w, lrow, it, nch0, r);
  };

  int p = blockIdx.x * GP_WAVES + wave;
  int it = 0;
  RawChunk bufA[U][GEMV_ROWS], bufB[U][GEMV_ROWS];
  if (p < npairs) load(p, 0, bufA);  // weight loads in flight during the prologue

  // ---- prologue: RMSNorm statistics + x staging (once per workgroup)
  if (a.norm_w) {
    for (int b = 0; b < a.B; ++b) {
      float s = 0.f;
      const float* xb = a.x + (size_t)b * a.ldx;
      for (int k = threadIdx.x * 4; k < K; k += GP_THREADS * 4) {
        const float4 v = *(const float4*)(xb + k);
        s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
      }
      s = block_sum(s, red);
      if (threadIdx.x == 0) inv_rms[b] = rsqrtf(s / (float)K + a.eps);
      __syncthreads();
    }
  }
  stage_x_tile<QT0>(a.x, a.ldx, a.B, 0, K, inv_rms, a.norm_w, xl0, xs0);
  if constexpr (SEP) stage_x_tile<QT1>(a.x, a.ldx, a.B, 0, K, inv_rms, a.norm_w, xl1, xs1);
  __syncthreads();

  float acc[GEMV_ROWS][B];
#pragma unroll
  for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
    for (int b = 0; b < B; ++b) acc[r][b] = 0.f;

  // one pipelined step: prefetch the item after (p,it) into `nxt`, compute `cur`
  auto step = [&](RawChunk (&cur)[U][GEMV_ROWS], RawChunk (&nxt)[U][GEMV_ROWS]) -> bool {
    int lrow;
    bool t1;
    QWeight w;
    info(p, lrow, t1, w);
    const int nit = (MIXED && t1) ? nit1 : nit0;
    int pn = p, itn = it + 1;
    if (itn >= nit) { pn = p + stride; itn = 0; }
    if (pn < npairs) load(pn, itn, nxt);
    if (MIXED && t1) gp_compute<QT1, B, U>(cur, it, nch1, xl1, xs1, acc);
    else gp_compute<QT0, B, U>(cur, it, nch0, xl0, xs0, acc);
    if (itn == 0) {  // pair p complete
#pragma unroll
      for (int r = 0; r < GEMV_ROWS; ++r)
#pragma unroll
        for (int b = 0; b < B; ++b) acc[r][b] = wave_sum(acc[r][b]);
      if (lane < a.B) {
        float v0 = 0.f, v1 = 0.f;
#pragma unroll
        for (int b = 0; b < B; ++b)
          if (lane == b) { v0 = acc[0][b]; v1 = acc[1][b]; }
        gemv_epilogue(a, a.row_base + 2 * p, lane, v0, v1);
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


// returns false when the shape does not fit the persistent kernel's LDS budget
template <int QT0, int QT1, int B, int U>
bool launch_gemv_persistent(GemvArgs a, hipStream_t st) {
  constexpr bool SEP = !same_xlayout<QT0, QT1>;
  const size_t xfl = (size_t)B * a.K + (size_t)B * a.K / 16;
  const size_t lds = (64 + xfl * (SEP ? 2 : 1) + 4) * sizeof(float);
  if (lds > 96 * 1024) return false;
  static int occ = -1;  // resident workgroups per CU for this instantiation (VGPR + LDS limited)
  if (occ < 0) {
    int o = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&o, gemv_persistent<QT0, QT1, B, U>, GP_THREADS, lds) !=
            hipSuccess || o <= 0)
      o = 1;
    occ = o;
  }
  const int per_cu = std::max(1, std::min(occ, (int)((160 * 1024) / lds)));
  const int groups = (a.N / 2 + GP_WAVES - 1) / GP_WAVES;
  const int blocks = std::min(groups, device_cu_count() * per_cu);
  a.kt_max = a.K;
  hipLaunchKernelGGL((gemv_persistent<QT0, QT1, B, U>), dim3(blocks), dim3(GP_THREADS), lds, st, a);
  return true;
}


#include "gemv_q8.h"
#include "gemv_cu.h"
#include "gemv_lds.h"
#include "gemv_lds16.h"

inline int qtype_block(int qt) {
  return (qt == QT_Q4_K || qt == QT_Q5_K || qt == QT_Q6_K) ? 256 : (qt == QT_F16 || qt == QT_BF16 ? 8 : 32);
}

template <int QT0, int QT1, int B, int U>
void launch_gemv_t(GemvArgs a, hipStream_t st) {
  const int blocks = (a.N + GEMV_ROWS_PER_BLOCK - 1) / GEMV_ROWS_PER_BLOCK;
  int kt = (GEMV_LDS_FLOATS / B) / 256 * 256;
  if (kt >= a.K) kt = a.K;
  int blk = 8;
  for (int s = 0; s < a.nseg; ++s) blk = std::max(blk, qtype_block(a.seg[s].qtype));
  if (kt < blk) kt = blk;
  a.kt_max = kt;
  const size_t lds = (64 + (size_t)B * kt + (size_t)B * kt / 16 + 4) * sizeof(float);
  hipLaunchKernelGGL((gemv_kernel<QT0, QT1, B, U>), dim3(blocks), dim3(GEMV_THREADS), lds, st, a);
}

// the fused TP all-reduce epilogue (EPI_TP_RESID, batch 1): the row-pair kernel or nothing
template <int QT0>
bool launch_gemv_tpf(const GemvArgs& a, hipStream_t st) {
  if constexpr (QT0 == QT_F16 || QT0 == QT_BF16) {
    return false;
  } else {
    if (a.B != 1 || !a.act_q8 || a.nseg != 1 || a.epi != EPI_TP_RESID) return false;
    return launch_gemv_q8<QT0, QT0, 1>(a, st);
  }
}

template <int QT0, int QT1>
void launch_gemv_pair(const GemvArgs& a, hipStream_t st) {
  constexpr int W = QFmt<QT0>::W;
  const int chunks_per_lane = (a.K / W + 63) / 64;
  constexpr bool Q8OK = QT0 != QT_F16 && QT0 != QT_BF16;
  if constexpr (Q8OK) {
    if (!a.force_v1 && a.act_q8) {
      if (a.B <= 4 && launch_gemv_lds<QT0, QT1>(a, st)) return;  // B = 1..4: the LDS-DMA engine
      if (a.B == 1 && launch_gemv_cu<QT0, QT1>(a, st)) return;
      if (a.B == 1 && launch_gemv_q8<QT0, QT1, 1>(a, st)) return;
      if (a.B == 2 && launch_gemv_q8<QT0, QT1, 2>(a, st)) return;
      if (a.B > 2 && a.B <= 4 && launch_gemv_q8<QT0, QT1, 4>(a, st)) return;
      if (a.B > 4 && launch_gemv_q8<QT0, QT1, 8>(a, st)) return;
    }
  }
  if constexpr (QT0 == QT_BF16 && QT1 == QT_BF16) {
    if (!a.force_v1 && launch_gemv_lds16(a, st)) return;  // B = 1..4: the BF16 LDS-DMA engine
  }
  if (a.epi == EPI_TP_RESID)  // only the row-pair int8 kernel does the fused all-reduce epilogue
    throw std::runtime_error("gemv: EPI_TP_RESID launch not taken by the row-pair kernel (use launch_gemv_tp_fused)");
  if (a.x16 || a.y16) throw std::runtime_error("bf16 GEMV input / SwiGLU output: int8-activation kernels only");
  if (!a.force_v1) {
    if (a.B == 1 && launch_gemv_persistent<QT0, QT1, 1, 2>(a, st)) return;
    if (a.B == 2 && launch_gemv_persistent<QT0, QT1, 2, 2>(a, st)) return;
    if (a.B > 2 && a.B <= 4 && launch_gemv_persistent<QT0, QT1, 4, 1>(a, st)) return;
  }
  if (a.B == 1) {
    if (chunks_per_lane >= 4) launch_gemv_t<QT0, QT1, 1, 4>(a, st);
    else launch_gemv_t<QT0, QT1, 1, 2>(a, st);
  } else if (a.B == 2) {
    launch_gemv_t<QT0, QT1, 2, 2>(a, st);
  } else if (a.B <= 4) {
    launch_gemv_t<QT0, QT1, 4, 2>(a, st);
  } else {
    launch_gemv_t<QT0, QT1, 8, 1>(a, st);
  }
}

}  // namespace aios
