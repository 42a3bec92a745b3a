// Split-K flash-decode GQA attention over the bf16 KV cache (decode shape),
// with the log-sum-exp combine fused in (last-arriving workgroup per (row, kv-head)).
//
// grid = (roles, 1, B), 512 threads (8 waves); every workgroup picks its role from seq_len (see
// attn_decode_kernel).  The context is cut into 128-key passes (16 keys per wave); every
// workgroup owns two passes at a time with ALL of their K and V loads issued up front (buffers A
// and B), so up to 256 keys cost one memory round trip: P = ceil(passes / 2) workgroups per
// (row, head set), capped by the grid (workgroups then loop, the next pass's loads issued while
// the current one is scored).  At a 153-key context this is one workgroup per query head with
// no combine; at 4k keys up to 32 workgroups per KV head.  (Round 1 walked up to three 64-key
// passes serially in one 4-wave workgroup: 7.8 us per layer at 153 keys.)
//
// Inside a pass every lane loads 16 B = 8 dims of a key (LPK = hd/8 lanes per key).  Each WAVE
// keeps its own online-softmax state (m, l, o) for the G = H/Hkv query heads of the group --
// scores are reduced over the LPK lanes of a key with DPP (no LDS), and no workgroup barrier is
// needed until the eight waves merge their states in LDS at the end.
//
// Combine: with more than one active workgroup each writes its partial (o, m, l) with
// write-through (sc1, agent scope) stores, drains them (s_waitcnt vmcnt(0)), and after a
// workgroup barrier one lane takes an agent-scope ticket for (row, kv head).  The last arriver
// reads every partial's (m, l) in one parallel sweep (one lane per partial), then each thread
// sums its outputs over the partials with independent loads -- the write-through hand-off of
// CDNA guide §6 Guideline 16 / split-K item 2 -- and re-arms the counter.
#include "attn_decode.h"

namespace aios {

template <int HD, int G, bool F8>
__global__ void __launch_bounds__(512) attn_decode_kernel(AttnDecodeArgs a, AttnSplit sp_) {
  kernarg_warm<sizeof(AttnDecodeArgs) + sizeof(AttnSplit)>();
  attn_role<HD, G, F8>(a, sp_, blockIdx.x);
}

template <int HD, bool F8>
static void launch_hd(const AttnDecodeArgs& a, int G, hipStream_t st) {
  AttnSplit sp;
  const int nwg = attn_plan(a, G, sp);
  sp.xcd = attn_env_int("AIOS_ATTN_XCD", 1);  // XCD-aware short-mode roles (0: the plain mapping)
  sp.n_attn = nwg;
  dim3 grid(nwg, 1, a.B);
  switch (G) {
    case 1: hipLaunchKernelGGL((attn_decode_kernel<HD, 1, F8>), grid, dim3(512), 0, st, a, sp); break;
    case 2: hipLaunchKernelGGL((attn_decode_kernel<HD, 2, F8>), grid, dim3(512), 0, st, a, sp); break;
    case 4: hipLaunchKernelGGL((attn_decode_kernel<HD, 4, F8>), grid, dim3(512), 0, st, a, sp); break;
    case 5: hipLaunchKernelGGL((attn_decode_kernel<HD, 5, F8>), grid, dim3(512), 0, st, a, sp); break;
    case 8: hipLaunchKernelGGL((attn_decode_kernel<HD, 8, F8>), grid, dim3(512), 0, st, a, sp); break;
    default: throw std::runtime_error("attn_decode: unsupported GQA group size " + std::to_string(G));
  }
}

// `split` (kept in the args for the API) encodes P * ATTN_CHUNK: the number of workgroups per
// (row, head set) in the long-context mode.  Target one workgroup per CU for the whole grid (a
// 512-thread workgroup of this kernel fills a CU's register file), 1..64 per head set, each
// owning at least one 128-key pass of a max_ctx context.
int attn_decode_split(int max_ctx, int B, int n_kv_heads) {
  const int nch = std::max(1, max_ctx / 128);
  // AIOS_ATTN_WG_PER_CU (default 1): long-context workgroups per CU the split aims for
  const int per_cu = std::max(1, std::min(4, attn_env_int("AIOS_ATTN_WG_PER_CU", 1)));
  const int P = std::max(1, std::min({64, nch, 256 * per_cu / std::max(1, B * n_kv_heads)}));
  return P * ATTN_CHUNK;
}

void launch_attn_decode(const AttnDecodeArgs& a, hipStream_t st) {
  if (a.n_heads % a.n_kv_heads) throw std::runtime_error("attn_decode: n_heads % n_kv_heads != 0");
  if (!a.counters) throw std::runtime_error("attn_decode: counters buffer required ([B][n_heads])");
  if (a.max_ctx % 128) throw std::runtime_error("attn_decode: max_ctx must be a multiple of 128");
  const int G = a.n_heads / a.n_kv_heads;
  const AttnDecodeArgs b = attn_resolve(a);
  if (b.split % ATTN_CHUNK) throw std::runtime_error("attn_decode: split must be a multiple of ATTN_CHUNK");
  if (a.head_dim == 128) {
    if (a.kv_fp8) launch_hd<128, true>(b, G, st);
    else launch_hd<128, false>(b, G, st);
  } else if (a.head_dim == 64) {
    if (a.kv_fp8) launch_hd<64, true>(b, G, st);
    else launch_hd<64, false>(b, G, st);
  } else {
    throw std::runtime_error("attn_decode: head_dim must be 64 or 128");
  }
}

}  // namespace aios
