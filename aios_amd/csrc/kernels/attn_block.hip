// Batch-1 decode attention block as ONE launch: QKV GEMV (RMSNorm prologue, RoPE + KV-write
// epilogue) -> split-K flash-decode attention -> O GEMV (+= residual), three workgroup roles of
// one grid wired by in-launch hand-offs (fuse.h) instead of three dependent launches.
//
// Why (profiles/decode_mistral_rocprof_r2_engine.txt): at batch 1 each of these launches is
// latency-bound -- QKV 9.4 us, attention 5.5 us, O 6.1 us for 25 MB of weights, ~8 us of
// floor -- and a dependent boundary costs 1.5-1.8 us plus the next kernel's ramp (its first
// weight bytes land ~2-4 us after it starts).  In one launch:
//   * the attention workgroups issue the K/V of every OLD position before the QKV edge, so the
//     seq_len -> block table -> K/V dependent-load chain overlaps the QKV GEMV;
//   * the O workgroups issue their first weight items before the attention edge, so the O
//     weight stream overlaps attention (the MI355X 'prefetch-credit' of a dependency edge);
//   * the two edges are single counters (<= 256 arrivals, spread over the producers' tail).
// Roles by blockIdx: [0, nq) QKV rows | [nq, nq + na) attention | [nq + na, +no) O rows --
// producers first, so a waiting consumer never holds a CU slot its producer needs.  nq = 0
// (AIOS_FUSE_ATTN=1): the QKV GEMV is its own launch and only attention -> O is fused (the idle
// attention workgroups of a short context exit at once and the O workgroups take their CUs).
//
// MEASURED (profiles/attn_block_fusion_r2.jsonl): correct, but slower than three launches --
// Mistral B=1 604 -> 561 (attention + O) / 511 (all three) tok/s, TinyLlama 1477 -> 1340 / 1157.
// Each edge (drained write-through stores + agent atomic + sc1 polling by every waiting workgroup)
// costs more than the launch boundary it removes, and the attention role's ~180 VGPRs cap the
// launch at one 512-thread workgroup per CU.  Opt-in only (AIOS_FUSE_ATTN=1/2), kept as the
// tested in-launch hand-off machinery.
//
// Restrictions (host-checked, else the three-launch path runs): B = 1, no TP, non-NeoX RoPE,
// no QK-norm, K / 32 <= 128 chunks (U = 1 row items: Mistral / Llama-3-8B / TinyLlama shapes),
// QKV in Q4_K (+ Q6_K V) or Q4_K, O in Q4_K, head_dim 64 / 128, GQA group 4 or 8.
#include "attn_decode.h"
#include "gemv_impl.h"

namespace aios {

struct AttnBlockCtl {
  int nq, na, no;   // workgroups per role
  int* cnt;         // [2]: QKV arrivals, attention heads published (zeroed before each step)
  int* err;         // hand-off give-up flag
};

template <int QQ0, int QQ1, int QO, int HD, int G>
__global__ void __launch_bounds__(512) attn_block_kernel(GemvArgs qkv, AttnDecodeArgs at, AttnSplit sp, GemvArgs o,
                                                         AttnBlockCtl c) {
  const int bx = blockIdx.x;
  if (bx < c.nq) {
    FuseEdge e;
    e.sig = c.cnt;
    e.err = c.err;
    q8_rows_body<QQ0, QQ1, 1, 1, 2, true>(qkv, bx, c.nq, e);
    return;
  }
  if (bx < c.nq + c.na) {
    FuseEdge e;
    e.wait = c.nq ? c.cnt : nullptr;  // nq = 0: the QKV GEMV ran as its own launch before this one
    e.target = c.nq;
    e.sig = c.cnt + 1;
    e.err = c.err;
    const int wg = bx - c.nq;
    const int len = at.seq_len[0];
    if (G > 1 && len <= ATTN_SPLIT_LEN) {
      const int h = wg / sp.p_short, s = wg % sp.p_short;
      if (h >= at.n_heads) return;
      attn_core<HD, 1, true>(at, s, h / G, h, h, sp.p_short, sp.ppw, e);
    } else {
      constexpr int GL = AttnGL<G>::value;
      const int hsi = wg / sp.p_long, s = wg % sp.p_long;
      if (hsi >= at.n_kv_heads * (G / GL)) return;
      const int kvh = hsi / (G / GL), h0 = kvh * G + (hsi % (G / GL)) * GL;
      attn_core<HD, GL, true>(at, s, kvh, h0, h0, sp.p_long, sp.ppw, e);
    }
    return;
  }
  FuseEdge e;
  e.wait = c.cnt + 1;
  e.target = at.n_heads;
  e.err = c.err;
  q8_rows_body<QO, QO, 1, 1, 2, true>(o, bx - c.nq - c.na, c.no, e);
}

template <int QQ0, int QQ1, int QO, int HD, int G>
static void launch_block_t(const GemvArgs& qkv, const AttnDecodeArgs& at, const AttnSplit& sp, const GemvArgs& o,
                           const AttnBlockCtl& c, size_t lds, hipStream_t st) {
  hipLaunchKernelGGL((attn_block_kernel<QQ0, QQ1, QO, HD, G>), dim3(c.nq + c.na + c.no), dim3(512), lds, st, qkv, at,
                     sp, o, c);
}

template <int HD, int G>
static bool launch_block_fmt(const GemvArgs& qkv, const AttnDecodeArgs& at, const AttnSplit& sp, const GemvArgs& o,
                             const AttnBlockCtl& c, size_t lds, hipStream_t st) {
  const int q0 = qkv.seg[0].qtype, q1 = qkv.seg[qkv.nseg - 1].qtype;
  if (o.seg[0].qtype != QT_Q4_K || q0 != QT_Q4_K) return false;
  if (q1 == QT_Q4_K) launch_block_t<QT_Q4_K, QT_Q4_K, QT_Q4_K, HD, G>(qkv, at, sp, o, c, lds, st);
  else if (q1 == QT_Q6_K) launch_block_t<QT_Q4_K, QT_Q6_K, QT_Q4_K, HD, G>(qkv, at, sp, o, c, lds, st);
  else return false;
  return true;
}

bool attn_block_supported(const GemvArgs& qkv, const AttnDecodeArgs& at, const GemvArgs& o) {
  if (qkv.B != 1 || o.B != 1 || at.B != 1 || qkv.epi != EPI_QKV || o.epi != EPI_RESID || qkv.rope_neox) return false;
  if (qkv.seg[0].qtype != QT_Q4_K || o.seg[0].qtype != QT_Q4_K || o.nseg != 1) return false;
  for (int s = 0; s + 1 < qkv.nseg; ++s)
    if (qkv.seg[s].qtype != QT_Q4_K) return false;
  const int q1 = qkv.seg[qkv.nseg - 1].qtype;
  if (q1 != QT_Q4_K && q1 != QT_Q6_K) return false;
  if (qkv.K / 32 > 128 || o.K / 32 > 128 || qkv.K % 256 || o.K % 256) return false;  // U = 1 row items
  if (qkv.N % 16 || o.N % 16) return false;
  const int G = at.n_heads / at.n_kv_heads;
  if (at.n_heads % at.n_kv_heads || (G != 4 && G != 8) || (at.head_dim != 64 && at.head_dim != 128)) return false;
  if (q8_lds_bytes<QT_Q4_K, QT_Q6_K, 1>(qkv.K) > 64 * 1024) return false;
  return true;
}

void launch_attn_block(const GemvArgs& qkv_in, const AttnDecodeArgs& at_in, const GemvArgs& o_in, int* cnt, int* err,
                       bool with_qkv, hipStream_t st) {
  if (!attn_block_supported(qkv_in, at_in, o_in)) throw std::runtime_error("attn_block: unsupported shape");
  if (!at_in.counters) throw std::runtime_error("attn_block: attention counters required");
  GemvArgs qkv = qkv_in, o = o_in;
  qkv.kt_max = qkv.K;
  o.kt_max = o.K;
  AttnDecodeArgs at = at_in;
  if (at.split <= 0) at.split = attn_decode_split(at.max_ctx, at.B, at.n_kv_heads);
  const int G = at.n_heads / at.n_kv_heads;
  AttnSplit sp;
  AttnBlockCtl c;
  c.na = attn_plan(at, G, sp);
  // the attention role's ~180 VGPRs leave room for ONE 512-thread workgroup per CU, so the GEMV
  // roles walk their rows with one workgroup per CU
  const int cus = device_cu_count();
  c.nq = with_qkv ? std::min((qkv.N / 2 + Q8_WAVES - 1) / Q8_WAVES, cus) : 0;
  c.no = std::min((o.N / 2 + Q8_WAVES - 1) / Q8_WAVES, cus);
  if (!with_qkv) launch_gemv(qkv_in, st);
  c.cnt = cnt;
  c.err = err;
  // dynamic LDS: the larger GEMV role's x staging (+ the RoPE row); attention's LDS is static
  const size_t lds = std::max(q8_lds_bytes<QT_Q4_K, QT_Q4_K, 1>(qkv.K), q8_lds_bytes<QT_Q4_K, QT_Q4_K, 1>(o.K));
  bool ok = false;
  if (at.head_dim == 128) ok = G == 4 ? launch_block_fmt<128, 4>(qkv, at, sp, o, c, lds, st)
                                      : launch_block_fmt<128, 8>(qkv, at, sp, o, c, lds, st);
  else ok = G == 4 ? launch_block_fmt<64, 4>(qkv, at, sp, o, c, lds, st) : launch_block_fmt<64, 8>(qkv, at, sp, o, c, lds, st);
  if (!ok) throw std::runtime_error("attn_block: unsupported format");
}

}  // namespace aios
