// Persistent batch-1 decode step: ONE launch, one 1024-thread workgroup per CU, every layer.
//
// Why (MI355X, Mistral-7B Q4_K_M, profiles/decode_mistral_rocprof_r2s3_final.txt): the step as 163
// launches spends ~52 us per layer against a ~27 us read floor.  Every GEMV launch pays the
// launch chain (~1.75 us), an x-staging ramp and a first-slot landing ~3-4 us after its start
// (its CUs' whole prologue burst queues at once), and the 5 us attention launch runs on 32 of 256
// CUs while HBM idles.  The weight stream itself does not depend on any activation, so here it
// never stops:
//
//  * Stages: per layer QKV (+RoPE, KV write) | attention | O (+residual) | gate/up (+SwiGLU) |
//    down (+residual), then the lm_head.  Every CU owns an equal row slice of every projection
//    (each QKV segment split on its own, so every CU streams the same bytes).
//  * Loader waves 14-15 stream the CU's slices of ALL stages, in order, HBM -> LDS with LDS-DMA
//    (buffer_load ... lds, nt) into a 4 x 32 KB ring, R-1 slots ahead of the consumers and across
//    stage boundaries: while a CU waits for the previous stage's outputs (or for attention) the
//    next stage's first 96 KB are already landing.  Slots are chunk-linear (a slot may straddle a
//    row), so any K with K % 256 == 0 works.
//  * Consumer waves 0-13 stage the stage's input vector (int8 per 32-block, the q8_1 GEMV path's
//    precision), dot each slot with v_dot4 and reduce rows into LDS accumulators; wave 0 runs the
//    epilogue and publishes with write-through (sc1) stores.
//  * Edges: after its stores drain (s_waitcnt vmcnt(0)) the epilogue wave adds 1 to the stage's
//    counter shard (blockIdx % 8: per-XCD shards, MI355X_MICROARCH.md 'fanin' / 'dequeue'); the
//    next stage's wave 0 polls the 8 shards with sc1 loads, a workgroup barrier releases the
//    consumers, which read the handed-off bytes with sc1 loads only (MI355X_MICROARCH.md 'Valid
//    forms' row 1: sc1 stores, drained, one signalling lane; sc1 poll; sc1 loads).
//  * Attention: units (KV head, key piece of >= 128 keys, <= MK_MAXU pieces per head) dealt over
//    the CUs; 8 waves per unit keep per-wave online-softmax state (v_dot2_f32_bf16 scores, packed
//    fp32 P.V), merge in LDS, publish a partial, and the last arriver per KV head (agent ticket)
//    combines the partials and signals the O stage.
//  * Loaders and consumers run the SAME sequence of raw s_barriers (no fences: in-flight LDS-DMA
//    survives them); the loaders' counted vmcnt waits assume every slot issues exactly MK_PL
//    DMA instructions per loader wave (padded), and the loader reads the stage table through the
//    constant address space (scalar loads), so no other vector-memory op enters its count.
//  * Every wait is bounded (a_timeout) and checks a shared abort word: a workgroup that is not
//    resident (another kernel holds its CU) makes the step fail fast and loudly, never hang.
//  * The last workgroup to finish re-arms every counter, so a captured step replays as is.
#include <vector>

#include "gemv_impl.h"
#include "attn_decode.h"
#include "../mk.h"

namespace aios {

constexpr int MK_NC = LG_NG;  // consumer waves
constexpr int MK_NL = LG_NL;  // loader waves
constexpr int MK_THREADS = LG_THREADS;
constexpr int MK_R = 4;          // ring slots
constexpr int MK_SLOT = 32768;   // ring slot stride (the Q4_K slot: 28 groups x 1152 B, padded)
constexpr int MK_PL = 16;        // DMA instructions per loader wave per slot (padded to this)
constexpr int MK_AW = 8;         // attention waves
constexpr int MK_RED = 64;       // LDS floats of the staging reduction
constexpr int MK_FLAGS = 16;     // LDS ints of flags
constexpr int MK_ATT_SHORT = 256;  // contexts up to this many keys: one attention unit per KV head

static_assert(LgLayout<QT_Q4_K>::slot_bytes <= MK_SLOT && LgLayout<QT_Q5_K>::slot_bytes <= MK_SLOT &&
                  LgLayout<QT_Q6_K>::slot_bytes <= MK_SLOT, "ring slot");
static_assert(LgLayout<QT_Q4_K>::per_loader <= MK_PL && LgLayout<QT_Q5_K>::per_loader <= MK_PL &&
                  LgLayout<QT_Q6_K>::per_loader <= MK_PL, "loader count");

// probes (tools/mk_probe.py): lane 0 of wave 0 (consumers) / wave MK_NC (loaders) stamps phase k of
// stage s; a null a.ts costs one scalar compare
#define MK_TS(s, k)                                                                                     \
  do {                                                                                                  \
    if (a.ts && (threadIdx.x & 63) == 0)                                                                \
      a.ts[((size_t)blockIdx.x * a.nstages + (s)) * 8 + (k)] = __builtin_amdgcn_s_memrealtime();        \
  } while (0)

typedef const __attribute__((address_space(4))) MkStage* CStage;

bool mk_format_ok(int qt) { return qt == QT_Q4_K || qt == QT_Q5_K || qt == QT_Q6_K; }

// chunks (16 B of 4-bit codes = 32 weights) per ring slot
__host__ __device__ constexpr int mk_cps(int qt) {
  return qt == QT_Q4_K ? LgLayout<QT_Q4_K>::NGS * 64 : (qt == QT_Q5_K ? LgLayout<QT_Q5_K>::NGS * 64 : LgLayout<QT_Q6_K>::NGS * 64);
}

// this CU's row range of a segment: pairs split evenly (RoPE / SwiGLU pairs never straddle CUs)
__device__ __forceinline__ void mk_rows(int rows, int c, int G, int& r0, int& r1) {
  const int np = rows >> 1;
  r0 = 2 * (int)((long)c * np / G);
  r1 = 2 * (int)((long)(c + 1) * np / G);
}

template <typename F>
__device__ __forceinline__ void mk_fmt(int qt, F&& f) {
  if (qt == QT_Q4_K) f(FmtTag<QT_Q4_K>{});
  else if (qt == QT_Q6_K) f(FmtTag<QT_Q6_K>{});
  else f(FmtTag<QT_Q5_K>{});
}

__device__ __forceinline__ const uint8_t* mk_plane(CStage st, int sg, int p) {
  const uint8_t* v = p == 0 ? st->seg[sg].p0 : (p == 1 ? st->seg[sg].p1 : (p == 2 ? st->seg[sg].p2 : st->seg[sg].p3));
  return sgpr_ptr(v);
}

// ---------------------------------------------------------------------------------------------
// loader: copy chunks [jb, jb + n) of segment sg (every plane) into ring slot `dst`.  Each plane's
// bytes are one contiguous range (planes are linear in the chunk index); the buffer resource is
// clamped to the range, so the fixed-count DMA of a partial slot reads zeros past its end.
// ---------------------------------------------------------------------------------------------
template <int QT>
__device__ __forceinline__ void mk_dma(CStage st, int sg, uint8_t* dst, int jb, int n, int lw) {
  using L = LgLayout<QT>;
  using P = LgPlanes<QT>;
  const int lane = threadIdx.x & 63;
  int idx = 0, issued = 0;
  static_for<4>([&](auto pc) {
    constexpr int p = decltype(pc)::value;
    if constexpr (p < P::n) {
      constexpr int S = P::dsz[p], BPG = P::bpg[p];
      constexpr int NI = L::ninst(p);
      const uint8_t* base = mk_plane(st, sg, p) + (size_t)jb * BPG / 64;
      const int nbytes = n * BPG / 64;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, nbytes, 0x00020000);
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        if ((idx + i) % MK_NL != lw) continue;
        auto* ldst = (__attribute__((address_space(3))) void*)(dst + L::off(p) + i * 64 * S);
        if constexpr (S == 16) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, ldst, 16, i * 1024 + lane * 16, 0, 0, 2 /* nt */);
        else __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, ldst, 4, i * 256 + lane * 4, 0, 0, 2 /* nt */);
        ++issued;
      }
      idx += NI;
    }
  });
  if (issued < MK_PL) {  // pad: re-copy this loader's first plane-0 piece onto itself
    const uint8_t* base = mk_plane(st, sg, 0) + (size_t)jb * 16;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, n * 16, 0x00020000);
    auto* ldst = (__attribute__((address_space(3))) void*)(dst + lw * 1024);
    for (; issued < MK_PL; ++issued) __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, ldst, 16, lw * 1024 + lane * 16, 0, 0, 2);
  }
}

// the loader's position in the slot stream: (stage, segment, slot), ATT stages skipped
struct MkCur {
  int s, sg, t, nsl, qt, cbeg, cend;
};
__device__ __forceinline__ void mk_settle(CStage stages, int ns, int c, int G, MkCur& k) {
  while (k.s < ns) {
    CStage st = stages + k.s;
    if (st->kind == MK_ATT || k.sg >= st->nseg) {
      ++k.s;
      k.sg = 0;
      k.t = 0;
      k.nsl = -1;
      continue;
    }
    if (k.nsl < 0) {
      int r0, r1;
      mk_rows(st->seg[k.sg].rows, c, G, r0, r1);
      const int nch = st->K >> 5;
      k.qt = st->seg[k.sg].qtype;
      k.cbeg = r0 * nch;
      k.cend = r1 * nch;
      const int cps = mk_cps(k.qt);
      k.nsl = (k.cend - k.cbeg + cps - 1) / cps;
    }
    if (k.t >= k.nsl) {
      ++k.sg;
      k.t = 0;
      k.nsl = -1;
      continue;
    }
    return;
  }
}

__device__ __forceinline__ void mk_issue(CStage stages, MkCur& k, uint8_t* dst, int lw) {
  CStage st = stages + k.s;
  const int cps = mk_cps(k.qt);
  const int jb = k.cbeg + k.t * cps;
  const int n = min(cps, k.cend - jb);
  mk_fmt(k.qt, [&](auto tag) { mk_dma<decltype(tag)::value>(st, k.sg, dst, jb, n, lw); });
}

// wait until ring slot `need` has landed, given `issued` slots issued so far
__device__ __forceinline__ void mk_loader_wait(int issued, int need) {
  const int allowed = issued - need - 1;
  if (allowed >= 2) lg_vmcnt<2 * MK_PL>();
  else if (allowed == 1) lg_vmcnt<MK_PL>();
  else lg_vmcnt<0>();
}

// ---------------------------------------------------------------------------------------------
// consumers
// ---------------------------------------------------------------------------------------------
template <int QT>
__device__ __forceinline__ float mk_dot(const RawChunk& raw, int c, const int8_t* xq, const float2* ms) {
  using F_ = QFmt<QT>;
  constexpr int W = F_::W, R = F_::RUNS;
  float sc[R], of[R];
  q8_scales_bf<QT>(raw, c, sc, of);
  int xv[8];
  const int8_t* xc = xq + (size_t)c * W;
  const int rot = (c >> 3) & 1;
  const uint4 p0 = *(const uint4*)(xc + 16 * rot);
  const uint4 p1 = *(const uint4*)(xc + 16 * (rot ^ 1));
  xv[0] = p0.x; xv[1] = p0.y; xv[2] = p0.z; xv[3] = p0.w;
  xv[4] = p1.x; xv[5] = p1.y; xv[6] = p1.z; xv[7] = p1.w;
  int is[R];
  QDot<QT>::isums(raw, c, xv, is);
  float acc = 0.f;
#pragma unroll
  for (int rr = 0; rr < R; ++rr) {
    const float2 m = ms[(size_t)c * R + rr];
    acc += sc[rr] * m.x * (float)is[rr] - of[rr] * m.y;
  }
  return acc;
}

// one ring slot: wave w takes groups [w*GPW, w*GPW + GPW) (64 chunks each; a group may straddle
// rows -- two at the model shapes, K >= 2048 -- ) and adds its row partials into racc (indexed
// by segment-local row - r0)
template <int QT>
__device__ __forceinline__ void mk_consume(const uint8_t* slotp, int jb, int n, int nch, int r0, float* racc,
                                           const int8_t* xq, const float2* ms, int wave, int lane) {
  constexpr int GPW = LgLayout<QT>::GPW;
  static_for<GPW>([&](auto kk) {
    const int k = wave * GPW + (int)decltype(kk)::value;
    if (k * 64 < n) {
      RawChunk raw;
      lg_read<QT>(slotp, k, lane, raw);
      const int jg = jb + k * 64;
      const int row0 = jg / nch;
      const int c0 = jg - row0 * nch;
      int c = c0 + lane, dr = 0;
      while (c >= nch) {  // at most once when nch >= 64
        c -= nch;
        ++dr;
      }
      const int nv = min(64, n - k * 64);  // valid lanes
      const float v = mk_dot<QT>(raw, c, xq, ms);
      const float vv = lane < nv ? v : 0.f;
      const int nrt = (c0 + nv - 1) / nch + 1;  // rows touched by the valid lanes
      const float s0 = cu_wave_sum(dr == 0 ? vv : 0.f);
      if (lane == 0) atomicAdd(&racc[row0 - r0], s0);
      for (int r = 1; r < nrt; ++r) {
        const float sr = cu_wave_sum(dr == r ? vv : 0.f);
        if (lane == 0) atomicAdd(&racc[row0 + r - r0], sr);
      }
    }
  });
}

// bounded wait (wave 0) until every shard of stage s's counter reached its arrival count;
// false when it gave up or another workgroup already did
__device__ __forceinline__ bool mk_wait(const MkArgs& a, int s, bool att, int G) {
  const int lane = threadIdx.x & 63;
  const int j = lane & 7;
  int target = 0;
  if (lane < 8) target = att ? (j < a.n_kv_heads ? (a.n_kv_heads - j + 7) / 8 : 0) : (j < G ? (G - j + 7) / 8 : 0);
  const int* p = a.cnt + ((size_t)s * 8 + j) * 32;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint64_t lim = (uint64_t)a.timeout_us * 100;
  while (true) {
    int v = 0x7fffffff;
    if (lane < 8) v = __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int e = __hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (__builtin_amdgcn_ballot_w64(v < target) == 0) return true;
    if (e) return false;
    if (__builtin_amdgcn_s_memrealtime() - t0 > lim) {
      if (lane == 0) __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(1);
  }
}

// wave 0: this CU's stores are drained -> one arrival on stage s's shard
__device__ __forceinline__ void mk_signal(const MkArgs& a, int s, int shard) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0)
    __hip_atomic_fetch_add(a.cnt + ((size_t)s * 8 + (shard & 7)) * 32, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// stage the input vector (written in this launch: sc1 loads) as int8 per 32-block into xq / ms;
// per-wave sums of squares into red when norm_w
__device__ __forceinline__ void mk_stage_in(const float* src, int K, const float* norm_w, int8_t* xq, float2* ms,
                                            float* red) {
  GemvArgs g;
  g.x = src;
  g.ldx = K;
  g.K = K;
  g.B = 1;
  g.norm_w = norm_w;
  StagePre<2> pf{};
  q8_stage_prefetch<2, true>(g, pf, threadIdx.x, MK_NC * 64);
  q8_stage<QT_Q4_K, 1, 2, true>(g, xq, ms, red, pf, threadIdx.x, MK_NC * 64);
}

// epilogue of a projection stage (wave 0): rows -> outputs (write-through), accumulators re-zeroed
__device__ __forceinline__ void mk_epilogue(const MkArgs& a, CStage st, int c, int G, float* rowacc, const float* red) {
  const int lane = threadIdx.x & 63;
  const int kind = st->kind;
  float s = 1.f;
  if (st->norm_w) {
    float t = 0.f;
#pragma unroll
    for (int w = 0; w < MK_NC; ++w) t += red[w];
    s = rsqrtf(t / (float)st->K + a.eps);
  }
  const int hd = a.head_dim;
  int pos = 0, kvb = 0;
  if (kind == MK_QKV) {
    pos = a.pos[0];
    kvb = kv_block(a.block_table, a.max_ctx / KV_BLOCK, a.slot[0], pos);
  }
  int roff = 0;
  for (int sg = 0; sg < st->nseg; ++sg) {
    int r0, r1;
    mk_rows(st->seg[sg].rows, c, G, r0, r1);
    const int nr = r1 - r0;
    const int row0 = st->seg_row0[sg] + r0;
    for (int p = lane; 2 * p < nr; p += 64) {
      const int lr = roff + 2 * p;
      const int grow = row0 + 2 * p;
      float v0 = rowacc[lr] * s, v1 = rowacc[lr + 1] * s;
      rowacc[lr] = 0.f;
      rowacc[lr + 1] = 0.f;
      if (kind == MK_QKV) {
        int part, r;
        if (grow < a.q_dim) { part = 0; r = grow; }
        else if (grow < a.q_dim + a.kv_dim) { part = 1; r = grow - a.q_dim; }
        else { part = 2; r = grow - a.q_dim - a.kv_dim; }
        const int head = r / hd, lrr = r - head * hd;
        if (part < 2) {
          const float2 t = a.rope_cs[(size_t)pos * (hd >> 1) + (lrr >> 1)];
          const float o0 = v0 * t.x - v1 * t.y, o1 = v0 * t.y + v1 * t.x;
          v0 = o0;
          v1 = o1;
        }
        if (part == 0) {
          st_sc1_f2(a.q + r, v0, v1);
        } else {
          bf16_t* cache = part == 1 ? st->k_cache : st->v_cache;
          const size_t off = (((size_t)kvb * a.n_kv_heads + head) * KV_BLOCK + (pos % KV_BLOCK)) * hd + lrr;
          st_sc1_u32(cache + off, (uint32_t)f32_to_bf16(v0) | ((uint32_t)f32_to_bf16(v1) << 16));
        }
      } else if (kind == MK_O || kind == MK_DOWN) {
        const uint64_t u = ld_sc1_8(a.x + grow);
        st_sc1_f2(a.x + grow, __uint_as_float((uint32_t)u) + v0, __uint_as_float((uint32_t)(u >> 32)) + v1);
      } else if (kind == MK_GU) {
        st_sc1_f32(a.ffb + (grow >> 1), v0 / (1.f + __expf(-v0)) * v1);
      } else {  // MK_LM: read after the launch
        *(float2*)(a.logits + grow) = make_float2(v0, v1);
      }
    }
    roff += nr;
  }
}

// ---------------------------------------------------------------------------------------------
// attention stage
// ---------------------------------------------------------------------------------------------
template <int HD, int G>
struct MkAtt {
  static constexpr int LPK = HD / 8;           // lanes per key (8 dims per lane)
  static constexpr int KPS = 64 / LPK;         // keys per wave-instruction
  static constexpr int ROUND = MK_AW * KPS;    // keys per round of the 8 waves
  static constexpr int HG = G > 5 ? 4 : G;     // query heads per register pass (VGPR budget: 128)
  static constexpr int U = HG >= 5 ? 2 : 4;    // rounds in flight per lane (128 keys per pass at hd 128)
};

// the unit split of the live context: pieces of >= 128 keys (a multiple of the 8-wave round),
// at most MK_MAXU per KV head
template <int HD, int G>
__device__ __forceinline__ void mk_att_split(int len, int& piece, int& P) {
  using A = MkAtt<HD, G>;
  if (len <= MK_ATT_SHORT) {  // one unit per KV head, no partials / combine round trips
    piece = len;
    P = 1;
    return;
  }
  piece = max(128, (len + MK_MAXU - 1) / MK_MAXU);
  piece = (piece + A::ROUND - 1) / A::ROUND * A::ROUND;
  P = (len + piece - 1) / piece;
}

// seq_len through the constant address space: a scalar load (the loader waves must issue no
// vector-memory op besides their counted DMAs)
__device__ __forceinline__ int mk_len(const MkArgs& a) {
  return *(const __attribute__((address_space(4))) int*)a.seq_len;
}

// per-wave partial over keys [k0, k1) of KV head kvh for query heads [hg0, hg0 + HG) of its group
template <int HD, int G>
__device__ __forceinline__ void mk_att_wave(const MkArgs& a, CStage st, int kvh, int hg0, int k0, int k1, int newest,
                                            float* s_o, float* s_m, float* s_l, int wave, int lane) {
  using A = MkAtt<HD, G>;
  constexpr int LPK = A::LPK, KPS = A::KPS, ROUND = A::ROUND, U = A::U, HG = A::HG;
  const int ksub = lane / LPK, dsl = lane % LPK;
  const int maxb = a.max_ctx / KV_BLOCK;
  // the block table through the constant address space: the KPS keys of one wave-instruction sit
  // in one 128-key block, so each lookup is a wave-uniform scalar load (K$), not a vector load the
  // K/V addresses would wait a memory round trip for
  typedef const __attribute__((address_space(4))) int* CInt;
  const CInt btr = (CInt)a.block_table + (size_t)(*(CInt)a.slot) * maxb;
  const size_t blk_stride = (size_t)a.n_kv_heads * KV_BLOCK * HD;
  const bf16_t* kc = st->k_cache + (size_t)kvh * KV_BLOCK * HD + dsl * 8;
  const bf16_t* vc = st->v_cache + (size_t)kvh * KV_BLOCK * HD + dsl * 8;
  const float qs = a.attn_scale * kLog2e;
  uint32_t q2[HG][4];
#pragma unroll
  for (int g = 0; g < HG; ++g) {
    const float* qp = a.q + (size_t)(kvh * G + hg0 + g) * HD + dsl * 8;
    const float4 f0 = ld_sc1_f4(qp), f1 = ld_sc1_f4(qp + 4);
    q2[g][0] = pk_bf16(f0.x * qs, f0.y * qs);
    q2[g][1] = pk_bf16(f0.z * qs, f0.w * qs);
    q2[g][2] = pk_bf16(f1.x * qs, f1.y * qs);
    q2[g][3] = pk_bf16(f1.z * qs, f1.w * qs);
  }
  float m[HG], l[HG];
  gf32x2 o[HG][4];
#pragma unroll
  for (int g = 0; g < HG; ++g) {
    m[g] = kNeg;
    l[g] = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[g][i] = gf32x2{0.f, 0.f};
  }
  for (int base = k0 + wave * KPS; base < k1; base += ROUND * U) {
    uint4 kr[U], vr[U];
    bool valid[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int kb = base + u * ROUND;  // wave-uniform first key of the instruction
      const int key = kb + ksub;
      valid[u] = key < k1;
      const int blk = btr[min(kb / KV_BLOCK, maxb - 1)];
      const int kk = valid[u] ? key : kb;
      const size_t off = (size_t)blk * blk_stride + (size_t)(kk % KV_BLOCK) * HD;
      if (kk == newest) {  // written in this launch by another CU
        kr[u] = ld_sc1_16(kc + off);
        vr[u] = ld_sc1_16(vc + off);
      } else {
        kr[u] = *(const uint4*)(kc + off);
        vr[u] = *(const uint4*)(vc + off);
      }
    }
    float sc[U][HG];
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int g = 0; g < HG; ++g) {
        float d = dot2_bf16(kr[u].x, q2[g][0], 0.f);
        d = dot2_bf16(kr[u].y, q2[g][1], d);
        d = dot2_bf16(kr[u].z, q2[g][2], d);
        d = dot2_bf16(kr[u].w, q2[g][3], d);
        d = group_sum<LPK>(d);
        sc[u][g] = valid[u] ? d : kNeg;
      }
#pragma unroll
    for (int g = 0; g < HG; ++g) {
      float mx = sc[0][g];
#pragma unroll
      for (int u = 1; u < U; ++u) mx = fmaxf(mx, sc[u][g]);
      mx = keys_max<LPK>(mx);
      const float mn = fmaxf(m[g], mx);
      const float alpha = fast_exp2(m[g] - mn);
      float ps = 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float p = fast_exp2(sc[u][g] - mn);
        sc[u][g] = p;
        ps += p;
      }
      l[g] = l[g] * alpha + keys_sum<LPK>(ps);
      m[g] = mn;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[g][i] *= alpha;
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint32_t w[4] = {vr[u].x, vr[u].y, vr[u].z, vr[u].w};
      gf32x2 vf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) vf[i] = gf32x2{__uint_as_float(w[i] << 16), __uint_as_float(w[i] & 0xffff0000u)};
#pragma unroll
      for (int g = 0; g < HG; ++g) {
        const gf32x2 pp = gf32x2{sc[u][g], sc[u][g]};
#pragma unroll
        for (int i = 0; i < 4; ++i) o[g][i] = __builtin_elementwise_fma(pp, vf[i], o[g][i]);
      }
    }
  }
#pragma unroll
  for (int g = 0; g < HG; ++g) {
    float of[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      of[2 * i] = keys_sum<LPK>(o[g][i].x);
      of[2 * i + 1] = keys_sum<LPK>(o[g][i].y);
    }
    const int gg = hg0 + g;
    if (ksub == 0) {
      float4* dst = (float4*)(s_o + ((size_t)wave * G + gg) * HD + dsl * 8);
      dst[0] = make_float4(of[0], of[1], of[2], of[3]);
      dst[1] = make_float4(of[4], of[5], of[6], of[7]);
    }
    if (lane == 0) {
      s_m[wave * G + gg] = m[g];
      s_l[wave * G + gg] = l[g];
    }
  }
}

// consumer side of the attention stage (barriers mirrored by mk_attention_loader)
template <int HD, int G>
__device__ __forceinline__ void mk_attention(const MkArgs& a, int s, CStage st, uint8_t* scratch, int* flags, int c,
                                             int GR, int wave, int lane) {
  using A = MkAtt<HD, G>;
  const int len = mk_len(a);
  const int newest = len - 1;
  int piece, P;
  mk_att_split<HD, G>(len, piece, P);
  const int Hkv = a.n_kv_heads;
  const int nunits = Hkv * P;
  if (c < nunits && wave == 0) mk_wait(a, s - 1, false, GR);
  if (wave == 0) MK_TS(s, 1);
  lg_barrier();
  if (wave == 0) MK_TS(s, 2);
  float* s_o = (float*)scratch;
  float* s_m = s_o + MK_AW * G * HD;
  float* s_l = s_m + MK_AW * G;
  float* s_pm = s_l + MK_AW * G;
  float* s_pl = s_pm + G * MK_MAXU;
  float* s_pw = s_pl + G * MK_MAXU;
  const bool aw = wave < MK_AW;
  const int tid = threadIdx.x;  // attention threads: 0 .. MK_AW*64-1
  for (int u = c; u < nunits; u += GR) {
    const int kvh = u / P, pi = u - kvh * P;
    const int k0 = pi * piece, k1 = min(len, k0 + piece);
    if (aw) {
      for (int hg0 = 0; hg0 < G; hg0 += A::HG)
        mk_att_wave<HD, G>(a, st, kvh, hg0, k0, k1, newest, s_o, s_m, s_l, wave, lane);
    }
    lg_barrier();  // A1: the waves' partials are in LDS
    if (P == 1) {  // short context: the merged, normalised output straight to the O stage
      if (aw) {
        for (int idx = tid; idx < G * HD; idx += MK_AW * 64) {
          const int g = idx / HD, dd = idx - g * HD;
          float M = s_m[g];
#pragma unroll
          for (int w = 1; w < MK_AW; ++w) M = fmaxf(M, s_m[w * G + g]);
          float L = 0.f, acc = 0.f;
#pragma unroll
          for (int w = 0; w < MK_AW; ++w) {
            const float sw = fast_exp2(s_m[w * G + g] - M);
            L += sw * s_l[w * G + g];
            acc += sw * s_o[((size_t)w * G + g) * HD + dd];
          }
          st_sc1_f32(a.attn + (size_t)(kvh * G + g) * HD + dd, acc / L);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      lg_barrier();  // A2: drained
      if (tid == 0)
        __hip_atomic_fetch_add(a.cnt + ((size_t)s * 8 + (kvh & 7)) * 32, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      continue;
    }
    if (aw) {
      for (int idx = tid; idx < G * HD; idx += MK_AW * 64) {
        const int g = idx / HD, dd = idx - g * HD;
        float M = s_m[g];
#pragma unroll
        for (int w = 1; w < MK_AW; ++w) M = fmaxf(M, s_m[w * G + g]);
        float L = 0.f, acc = 0.f;
#pragma unroll
        for (int w = 0; w < MK_AW; ++w) {
          const float sw = fast_exp2(s_m[w * G + g] - M);
          L += sw * s_l[w * G + g];
          acc += sw * s_o[((size_t)w * G + g) * HD + dd];
        }
        const int h = kvh * G + g;
        st_sc1_f32(a.o_part + ((size_t)h * MK_MAXU + pi) * HD + dd, acc);
        if (dd == 0) st_sc1_f2(a.ml + ((size_t)h * MK_MAXU + pi) * 2, M, L);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lg_barrier();  // A2: every storing wave drained
    if (tid == 0) {
      const int t = __hip_atomic_fetch_add(a.tick + ((size_t)st->layer * Hkv + kvh) * 32, 1, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
      flags[0] = (t == P - 1);
    }
    lg_barrier();  // A3
    // C1-C3 run for every unit (the loaders mirror a fixed barrier count and never read LDS: an
    // LDS read behind their DMAs would make the compiler drain the ring first)
    const bool last = flags[0] != 0;
    if (last && aw && tid < G * P) {
      const int g = tid / P, p = tid - g * P;
      const uint64_t v = ld_sc1_8(a.ml + ((size_t)(kvh * G + g) * MK_MAXU + p) * 2);
      s_pm[g * MK_MAXU + p] = __uint_as_float((uint32_t)v);
      s_pl[g * MK_MAXU + p] = __uint_as_float((uint32_t)(v >> 32));
    }
    lg_barrier();  // C1
    if (last && wave < G) {
      const float mv = lane < P ? s_pm[wave * MK_MAXU + lane] : kNeg;
      const float lv = lane < P ? s_pl[wave * MK_MAXU + lane] : 0.f;
      float M = mv;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) M = fmaxf(M, __shfl_xor(M, o));
      const float e = fast_exp2(mv - M);
      float L = e * lv;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) L += __shfl_xor(L, o);
      if (lane < P) s_pw[wave * MK_MAXU + lane] = e / L;
    }
    lg_barrier();  // C2
    if (last && aw) {
      for (int idx = tid; idx < G * HD; idx += MK_AW * 64) {
        const int g = idx / HD, dd = idx - g * HD;
        const int h = kvh * G + g;
        const float* op = a.o_part + (size_t)h * MK_MAXU * HD + dd;
        float acc = 0.f;
        for (int p0 = 0; p0 < P; p0 += 8) {
          float ov[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) ov[j] = ld_wt(op + (size_t)min(p0 + j, P - 1) * HD);
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (p0 + j < P) acc = fmaf(s_pw[g * MK_MAXU + p0 + j], ov[j], acc);
        }
        st_sc1_f32(a.attn + (size_t)h * HD + dd, acc);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    lg_barrier();  // C3: the output of KV head kvh is drained
    if (last && tid == 0)
      __hip_atomic_fetch_add(a.cnt + ((size_t)s * 8 + (kvh & 7)) * 32, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// the loader waves' mirror of mk_attention: the same barriers, nothing else
template <int HD, int G>
__device__ __forceinline__ void mk_attention_loader(const MkArgs& a, int c, int GR) {
  const int len = mk_len(a);
  int piece, P;
  mk_att_split<HD, G>(len, piece, P);
  const int nunits = a.n_kv_heads * P;
  lg_barrier();
  for (int u = c; u < nunits; u += GR) {
    lg_barrier();  // A1
    lg_barrier();  // A2
    if (P == 1) continue;
    lg_barrier();  // A3
    lg_barrier();  // C1
    lg_barrier();  // C2
    lg_barrier();  // C3
  }
}

// ---------------------------------------------------------------------------------------------
// the kernel: loader and consumer programs run the same barrier sequence
// ---------------------------------------------------------------------------------------------
template <int HD, int G>
__device__ __forceinline__ void mk_loader_prog(const MkArgs& a, uint8_t* ring, const int* flags, int lw, int c, int GR) {
  const int ns = a.nstages;
  CStage stages = (CStage)a.stages;
  MkCur lc{0, 0, 0, -1, 0, 0, 0};
  int issued = 0;
  mk_settle(stages, ns, c, GR, lc);
  for (int i = 0; i < MK_R - 1 && lc.s < ns; ++i) {
    mk_issue(stages, lc, ring + (size_t)(issued % MK_R) * MK_SLOT, lw);
    ++issued;
    ++lc.t;
    mk_settle(stages, ns, c, GR, lc);
  }
  int t = 0;
  for (int s = 0; s < ns; ++s) {
    CStage st = stages + s;
    if (st->kind == MK_ATT) {
      mk_attention_loader<HD, G>(a, c, GR);
      continue;
    }
    if (lw == 0) MK_TS(s, 6);
    lg_barrier();  // B_w
    if (t == 0) mk_loader_wait(issued, 0);
    lg_barrier();  // B_in
    const int nch = st->K >> 5;
    for (int sg = 0; sg < st->nseg; ++sg) {
      int r0, r1;
      mk_rows(st->seg[sg].rows, c, GR, r0, r1);
      const int cps = mk_cps(st->seg[sg].qtype);
      const int nsl = (r1 * nch - r0 * nch + cps - 1) / cps;
      for (int k = 0; k < nsl; ++k, ++t) {
        if (lc.s < ns) {
          if (!(a.dbg & 2)) mk_issue(stages, lc, ring + (size_t)(issued % MK_R) * MK_SLOT, lw);
          ++issued;
          ++lc.t;
          mk_settle(stages, ns, c, GR, lc);
        }
        mk_loader_wait(issued, t + 1);
        lg_barrier();
      }
    }
    if (lw == 0) MK_TS(s, 7);
  }
  lg_vmcnt<0>();
}

template <int HD, int G>
__device__ __forceinline__ void mk_consumer_prog(const MkArgs& a, uint8_t* ring, float* red, int* flags, float* rowacc,
                                              uint8_t* scratch, int wave, int c, int GR) {
  const int lane = threadIdx.x & 63;
  const int ns = a.nstages;
  CStage stages = (CStage)a.stages;
  int t = 0;  // slot steps so far (= next ring slot to read)
  for (int s = 0; s < ns; ++s) {
    CStage st = stages + s;
    const int kind = st->kind;
    if (wave == 0) MK_TS(s, 0);
    if (kind == MK_ATT) {
      mk_attention<HD, G>(a, s, st, scratch, flags, c, GR, wave, lane);
      if (wave == 0) MK_TS(s, 5);
      continue;
    }
    // ---- input: wait for the previous stage, stage its output vector
    if (wave == 0 && s > 0) mk_wait(a, s - 1, stages[s - 1].kind == MK_ATT, GR);
    if (wave == 0) MK_TS(s, 1);
    lg_barrier();  // B_w
    if (wave == 0) MK_TS(s, 2);
    const int K = st->K;
    const int nch = K >> 5;
    float2* ms = (float2*)scratch;
    int8_t* xq = (int8_t*)(ms + (size_t)nch * 2);
    const float* src = (kind == MK_O) ? a.attn : (kind == MK_DOWN ? a.ffb : a.x);
    mk_stage_in(src, K, st->norm_w, xq, ms, red);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    lg_barrier();  // B_in
    if (wave == 0) MK_TS(s, 3);
    // ---- slot steps
    int roff = 0;
    for (int sg = 0; sg < st->nseg; ++sg) {
      int r0, r1;
      mk_rows(st->seg[sg].rows, c, GR, r0, r1);
      const int qt = st->seg[sg].qtype;
      const int cps = mk_cps(qt);
      const int cbeg = r0 * nch, cend = r1 * nch;
      const int nsl = (cend - cbeg + cps - 1) / cps;
      constexpr int NGS4 = LgLayout<QT_Q4_K>::NGS;
      if (qt == QT_Q4_K && (nch & 63) == 0 && NGS4 % (nch >> 6) == 0 && !(a.dbg & 1)) {
        // Q4_K chunk pairs with x in registers (gemv_cu.h Q4PairX): every slot holds whole rows,
        // so a lane sees the same K columns in every slot of the segment
        const int m = nch >> 6;
        const int half = lane >> 5, p = lane & 31, kk = wave * 2 + half;
        Q4PairX X;
        q4p_load_x(xq, ms, (kk % m) * 64 + 2 * p, X);
        using L4 = LgLayout<QT_Q4_K>;
        const int rps = NGS4 / m, rk = kk / m;
        for (int k = 0; k < nsl; ++k, ++t) {
          const uint8_t* slotp = ring + (size_t)(t % MK_R) * MK_SLOT;
          const int n = min(cps, cend - cbeg - k * cps);
          if (wave * 128 < n) {
            const uint4 a0 = *(const uint4*)(slotp + L4::off(0) + kk * 1024 + p * 32);
            const uint4 a1 = *(const uint4*)(slotp + L4::off(0) + kk * 1024 + p * 32 + 16);
            const uint4 mt = *(const uint4*)(slotp + L4::off(1) + kk * 128 + (p >> 2) * 16);
            const bool ok = kk * 64 < n;
            const float v = cu_half_sum(ok ? q4p_dot(a0, a1, mt, p & 3, X) : 0.f);
            if (p == 0 && ok)
              __hip_atomic_fetch_add(rowacc + roff + k * rps + rk, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          }
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // row sums visible past the barrier
          lg_barrier();
        }
        roff += r1 - r0;
        continue;
      }
      for (int k = 0; k < nsl; ++k, ++t) {
        const uint8_t* slotp = ring + (size_t)(t % MK_R) * MK_SLOT;
        const int jb = cbeg + k * cps;
        const int n = min(cps, cend - jb);
        if (!(a.dbg & 1))
          mk_fmt(qt, [&](auto tag) {
            mk_consume<decltype(tag)::value>(slotp, jb, n, nch, r0, rowacc + roff, xq, ms, wave, lane);
          });
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        lg_barrier();
      }
      roff += r1 - r0;
    }
    // ---- epilogue + arrival
    if (wave == 0) {
      MK_TS(s, 4);
      mk_epilogue(a, st, c, GR, rowacc, red);
      if (kind != MK_LM) mk_signal(a, s, c);
      MK_TS(s, 5);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <int HD, int G>
__global__ void __launch_bounds__(MK_THREADS) decode_mk_kernel(MkArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  uint8_t* ring = smem;
  float* red = (float*)(smem + MK_R * MK_SLOT);
  int* flags = (int*)(red + MK_RED);
  float* rowacc = (float*)(flags + MK_FLAGS);
  uint8_t* scratch = smem + a.scratch_off;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int c = blockIdx.x, GR = gridDim.x;
  for (int i = threadIdx.x; i < a.racc_n; i += MK_THREADS) rowacc[i] = 0.f;
  if (wave >= MK_NC) mk_loader_prog<HD, G>(a, ring, flags, wave - MK_NC, c, GR);
  else mk_consumer_prog<HD, G>(a, ring, red, flags, rowacc, scratch, wave, c, GR);

  // ---- finish: the last workgroup re-arms every counter for the next replay
  lg_barrier();
  if (threadIdx.x == 0) {
    const int t1 = __hip_atomic_fetch_add(a.done, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flags[1] = (t1 == GR - 1);
  }
  lg_barrier();
  if (flags[1]) {
    const size_t n1 = (size_t)a.nstages * 8 * 32, n2 = (size_t)a.n_layers * a.n_kv_heads * 32;
    for (size_t i = threadIdx.x; i < n1; i += MK_THREADS) a.cnt[i] = 0;
    for (size_t i = threadIdx.x; i < n2; i += MK_THREADS) a.tick[i] = 0;
    if (threadIdx.x == 0) *a.done = 0;
  }
}

// ---------------------------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------------------------
static int mk_scratch_floats(int HD, int G) { return MK_AW * G * HD + 2 * MK_AW * G + 3 * G * MK_MAXU; }

static bool mk_shape_ok(int HD, int G) { return (HD == 128 && (G == 4 || G == 8 || G == 5 || G == 1)) || (HD == 64 && (G == 8 || G == 4)); }

bool mk_plan(MkArgs& a, const std::vector<MkStage>& st, int cus) {
  if (a.n_heads % a.n_kv_heads) return false;
  const int G = a.n_heads / a.n_kv_heads;
  if (!mk_shape_ok(a.head_dim, G)) return false;
  int racc = 0, kmax = 0;
  for (const MkStage& s : st) {
    if (s.kind == MK_ATT) continue;
    if (s.K % 256) return false;
    kmax = std::max(kmax, s.K);
    int rows = 0;
    for (int g = 0; g < s.nseg; ++g) {
      if (!mk_format_ok(s.seg[g].qtype) || s.seg[g].rows % 2 || s.seg[g].cols != s.K) return false;
      const int np = s.seg[g].rows / 2;
      rows += 2 * ((np + cus - 1) / cus);
    }
    racc = std::max(racc, rows);
  }
  a.racc_n = (racc + 3) & ~3;
  const int head = MK_R * MK_SLOT + (MK_RED + MK_FLAGS + a.racc_n) * 4;
  a.scratch_off = (head + 15) & ~15;
  const int stage_bytes = (kmax / 32) * 2 * 8 + kmax;
  const int att_bytes = mk_scratch_floats(a.head_dim, G) * 4;
  a.lds_bytes = a.scratch_off + std::max(stage_bytes, att_bytes);
  return a.lds_bytes <= 160 * 1024;
}

template <int HD, int G>
static void mk_launch_t(const MkArgs& a, int grid, hipStream_t st) {
  hipLaunchKernelGGL((decode_mk_kernel<HD, G>), dim3(grid), dim3(MK_THREADS), a.lds_bytes, st, a);
}

void launch_decode_mk(const MkArgs& a, int grid, hipStream_t st) {
  const int G = a.n_heads / a.n_kv_heads;
  if (a.head_dim == 128) {
    switch (G) {
      case 4: mk_launch_t<128, 4>(a, grid, st); return;
      case 8: mk_launch_t<128, 8>(a, grid, st); return;
      case 5: mk_launch_t<128, 5>(a, grid, st); return;
      case 1: mk_launch_t<128, 1>(a, grid, st); return;
    }
  } else if (a.head_dim == 64) {
    switch (G) {
      case 8: mk_launch_t<64, 8>(a, grid, st); return;
      case 4: mk_launch_t<64, 4>(a, grid, st); return;
    }
  }
  throw std::runtime_error("decode_mk: unsupported head layout");
}

}  // namespace aios
