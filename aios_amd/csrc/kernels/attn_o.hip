// Batch-1 decode: attention and the O projection in ONE launch, communicating through each XCD's
// own L2 (MI355X in-launch dependency).
//
// Two launches (profiles/decode_mistral_rocprof_r4_final.txt): attention 5.3 us on 32 of 256 CUs,
// then the row-pair O GEMV (4096 x 4096 Q4_K, 9.4 MB) 5.4-6.0 us -- its bytes need ~1.8 us, the rest
// was its launch, the first weight round trip and the x staging, all serial behind attention.
//
// Short contexts (seq_len <= short_len; agent turns): grid = 256 workgroups, one per CU, dealt
// round-robin to the 8 XCDs (a residue class b % 8 on one XCD; HW_REG_XCC_ID in probes).  EVERY XCD
// computes the whole attention -- its 32 workgroups one query head each (the K/V of a head group
// hits that XCD's L2 after the first read; the 8x re-read of a short context comes from MALL) --
// and then 1/8 of the O rows.  Each workgroup first issues the weight loads of its O row pairs
// (registers; they land while attention runs), runs its head, writes the head's output to its
// XCD's private copy of x and adds 1 to its XCD's counter -- both in that XCD's L2 (workgroup-scope
// atomics execute there).  One lane polls the counter with L1-bypassing (sc0) loads until all 32
// heads of the XCD are in, then x is staged and the pairs computed.  Every hand-off is an L2 round
// trip, not a memory one: the cross-XCD variant (agent-scope write-through outputs, counters in
// memory, 224 dedicated O workgroups beside 32 attention ones) measured 10.3-10.6 us per launch --
// five memory round trips after attention -- against 10.8 us for the two launches.
//
// Long contexts: split-K attention over all workgroups (attention.hip's long mode, combine fused),
// outputs with agent-scope write-through stores and the arrival count in memory (one copy per XCD,
// each in its own 128-B line); then every workgroup takes O row pairs (weights loaded after its
// attention share).
//
// MEASURED, NOT A WIN (so AIOS_ATTN_O defaults to 0; the engine launches attention and O
// separately): in the captured Mistral-7B step this launch takes 10.8 us against 5.3 + 5.3 us for
// the two (bench 666-667 vs 677-678 tok/s same box; --prompt 1500: 609 vs 615).  With the x
// copies and counters XCD-local, the poll still needs sc1 loads (below) -- a memory round trip --
// and the chain after attention (store ack, count, poll, x staging, dot, residual) costs what the
// second launch's ramp did.  Kept as the tested reference for the in-launch hand-off.
//
// Forward progress: one workgroup per CU (the attention core's registers), so the 32 workgroups of
// an XCD are resident together once dispatched; a co-tenant's kernels only delay them.  Every wait
// is bounded (1 s), so a fault gives wrong numbers, never a hang.  Counters are re-armed by the
// NEXT layer's launch (`rearm`; every B = 1 step runs all layers in order).
#include "gemv_impl.h"
#include "attn_decode.h"

namespace aios {

constexpr int AO_XCDS = 8;
// counter block per layer (ATTN_O_CNT_INTS ints): [0, 256) short-mode per-XCD counters (stride 32
// ints = 128 B), [256, 512) long-mode copies, [768, 1024) probes: each workgroup's physical XCD
static_assert(ATTN_O_CNT_INTS >= 1024, "counter block");

__device__ __forceinline__ int ao_xcc_id() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return (int)(v & 15);
}

template <int QT, int U, int PIPE>
struct ORows {
  RawChunk buf[PIPE][U][GEMV_ROWS];
};

// issue the weight loads of this wave's row pairs p0 + k * pstride (k < PIPE, p < pend)
template <int QT, int U, int PIPE>
__device__ __forceinline__ void o_issue(const GemvArgs& a, ORows<QT, U, PIPE>& r, int p0, int pstride, int pend) {
  const int nch = a.K / QFmt<QT>::W;
  const SegRs w0 = seg_rsrc(a, 0);
  const __amdgpu_buffer_rsrc_t rx = mk_rsrc((const uint8_t*)a.x);
#pragma unroll
  for (int k = 0; k < PIPE; ++k) {
    const int p = p0 + k * pstride;
    SegRs w = w0;
    if (p >= pend) w.r0 = w.r1 = w.r2 = w.r3 = rx;  // past the end: in-bounds dummy reads, no branch
    q8_load_item<QT, U>(w, p < pend ? 2 * p : 0, 0, nch, r.buf[k]);
  }
}

// bounded poll of *c >= need by one lane.  The XCD-local hand-off (SCOPE workgroup) polls with
// sc1 loads too (AIOS_ATTN_O_POLL=2, default): an sc0 (workgroup-scope) load, or a plain load after
// an L1 invalidate (mode 1), never saw the other workgroups' increments and spun to the 1 s bound
// (measured: 1 s per launch, counts complete in memory afterwards)
__device__ __forceinline__ int ao_ld_l2(const int* c) {
  int v;
  asm volatile("buffer_inv sc0\n\tglobal_load_dword %0, %1, off\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(c) : "memory");
  return v;
}
template <int SCOPE>
__device__ __forceinline__ void ao_wait(const int* c, int need, int mode = 0) {
  constexpr uint64_t TIMEOUT = 100ull * 1000 * 1000;  // 1 s of the 100 MHz wall clock: no hang
  const uint64_t t0 = wall_clock64();
  auto ld = [&]() __attribute__((always_inline)) {
    if (SCOPE == __HIP_MEMORY_SCOPE_WORKGROUP && mode == 1) return ao_ld_l2(c);
    if (SCOPE == __HIP_MEMORY_SCOPE_WORKGROUP && mode == 2)
      return __hip_atomic_load(const_cast<int*>(c), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __hip_atomic_load(const_cast<int*>(c), __ATOMIC_RELAXED, SCOPE);
  };
  while (ld() < need && wall_clock64() - t0 < TIMEOUT) __builtin_amdgcn_s_sleep(1);
}

// x (the attention output, fp32 [K]) -> int8 staging, then this wave's pairs with the residual /
// store epilogue
template <int QT, int U, int PIPE>
__device__ __forceinline__ void o_finish(const GemvArgs& a, const float* x, ORows<QT, U, PIPE>& r, int p0,
                                         int pstride, int pend) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  constexpr int W = QFmt<QT>::W, R = QFmt<QT>::RUNS;
  const int nch = a.K / W;
  float* red = smem;
  float2* ms = (float2*)(smem + 64);
  int8_t* xq = (int8_t*)(ms + (size_t)nch * R);
  GemvArgs ax = a;  // (the staging reads ax.x)
  ax.x = x;
  StagePre<1> pf;
  q8_stage_prefetch(ax, pf);
  q8_stage<QT, 1, 1>(ax, xq, ms, red, pf);
  __syncthreads();
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < PIPE; ++k) {
    const int p = p0 + k * pstride;
    if (p < pend) {
      float acc[GEMV_ROWS][1] = {{0.f}, {0.f}};
      q8_compute<QT, 1, U>(r.buf[k], 0, nch, xq, ms, acc);
      const float2 v = wave_sum_pair(acc[0][0], acc[1][0]);
      if (lane == 0) {
        float* y = a.y + a.row_base + 2 * p;
        if (a.epi == EPI_RESID) {
          unsafeAtomicAdd(y, v.x);
          unsafeAtomicAdd(y + 1, v.y);
        } else {
          *(float2*)y = v;
        }
      }
    }
  }
}

template <int HD, int G, int QT, int U, int PIPE>
__global__ void __launch_bounds__(512) attn_o_kernel(AttnDecodeArgs aa, AttnSplit sp, GemvArgs ga, int* cnt,
                                                     int* rearm, float* xloc) {
  kernarg_warm<sizeof(AttnDecodeArgs) + sizeof(AttnSplit) + sizeof(GemvArgs) + 24>();
  const int b = blockIdx.x, wave = threadIdx.x >> 6;
  const int npairs = ga.N >> 1;
  if (b == 0 && threadIdx.x < 2 * AO_XCDS)
    __hip_atomic_store(rearm + ATTN_O_CSTRIDE * threadIdx.x, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int len = aa.seq_len[0];
  ORows<QT, U, PIPE> rows;
  if (len <= aa.short_len) {
    // ---- short: XCD-local.  XCD x = b % 8 owns pairs [x * P8, (x + 1) * P8); its workgroup j = b / 8
    // (query head j) takes ppw * 8 of them, wave w pairs j * 8 * ppw + w + 8 k
    const int x = b % AO_XCDS, j = b / AO_XCDS;
    const int nper = gridDim.x / AO_XCDS;  // workgroups per XCD (= query heads)
    const int P8 = npairs / AO_XCDS, pw = P8 / nper;
    const int p0 = x * P8 + j * pw + wave, pend = x * P8 + (j + 1) * pw;
    o_issue<QT, U, PIPE>(ga, rows, p0, 8, pend);
    // (the XCDs take the workgroups round-robin from a rotating start -- workgroup b on XCD
    // (b + r) % 8 for the launch's r, measured -- so a residue class b % 8 shares one L2)
    if ((sp.xcd & 2) && threadIdx.x == 0 && b < 256)  // probes (AIOS_ATTN_XCD bit 1): [768 + b] physical XCD
      __hip_atomic_store(cnt + 768 + b, 100 + ao_xcc_id(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    float* xo = xloc + (size_t)x * aa.n_heads * HD;
    AttnDecodeArgs ah = aa;
    ah.out = xo;
    ah.out_wt = 0;  // plain stores: this XCD's L2
    attn_core<HD, 1>(ah, 0, j / G, j, j, 1, 1);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the head's output stored to L2
    __syncthreads();
    int* c = cnt + ATTN_O_CSTRIDE * x;
    if (threadIdx.x == 0) {
      __hip_atomic_fetch_add(c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);  // (an L2 atomic)
      ao_wait<__HIP_MEMORY_SCOPE_WORKGROUP>(c, nper, sp.xcd >> 2);
    }
    __syncthreads();
    o_finish<QT, U, PIPE>(ga, xo, rows, p0, 8, pend);
  } else {
    // ---- long: split-K attention over the whole grid, arrival count in memory, then O everywhere
    AttnDecodeArgs al = aa;
    al.out_wt = 1;
    attn_role<HD, G>(al, sp, b);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's write-through outputs retired
    __syncthreads();
    int* cl = cnt + AO_XCDS * ATTN_O_CSTRIDE;
    if (threadIdx.x < AO_XCDS)
      __hip_atomic_fetch_add(cl + ATTN_O_CSTRIDE * threadIdx.x, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int p0 = b * 8 + wave, pstride = gridDim.x * 8;
    o_issue<QT, U, PIPE>(ga, rows, p0, pstride, npairs);
    if (threadIdx.x == 0) ao_wait<__HIP_MEMORY_SCOPE_AGENT>(cl + ATTN_O_CSTRIDE * (b % AO_XCDS), gridDim.x);
    __syncthreads();
    // (plain x loads: this launch's acquire emptied every L2 of x's lines and nothing reads x before
    // the count, so each XCD's first miss fetches the write-through data)
    o_finish<QT, U, PIPE>(ga, aa.out, rows, p0, pstride, npairs);
  }
}

template <int HD, int G, int QT, int U, int PIPE>
static void attn_o_go(const AttnDecodeArgs& b, const AttnSplit& sp, const GemvArgs& g, int grid, int* cnt, int* rearm,
                      float* xloc, hipStream_t st) {
  const size_t lds = q8_lds_bytes<QT, QT, 1>(g.K);
  hipLaunchKernelGGL((attn_o_kernel<HD, G, QT, U, PIPE>), dim3(grid), dim3(512), lds, st, b, sp, g, cnt, rearm, xloc);
}

template <int HD, int G, int QT>
static void attn_o_fmt(const AttnDecodeArgs& b, const AttnSplit& sp, const GemvArgs& g, int U, int PIPE, int grid,
                       int* cnt, int* rearm, float* xloc, hipStream_t st) {
  if (U == 1 && PIPE == 1) attn_o_go<HD, G, QT, 1, 1>(b, sp, g, grid, cnt, rearm, xloc, st);
  else if (U == 1) attn_o_go<HD, G, QT, 1, 2>(b, sp, g, grid, cnt, rearm, xloc, st);
  else if (PIPE == 1) attn_o_go<HD, G, QT, 2, 1>(b, sp, g, grid, cnt, rearm, xloc, st);
  else attn_o_go<HD, G, QT, 2, 2>(b, sp, g, grid, cnt, rearm, xloc, st);
}

template <int HD, int G>
static void attn_o_g(const AttnDecodeArgs& b, const AttnSplit& sp, const GemvArgs& g, int U, int PIPE, int grid,
                     int* cnt, int* rearm, float* xloc, hipStream_t st) {
  if (g.seg[0].qtype == QT_Q4_K) attn_o_fmt<HD, G, QT_Q4_K>(b, sp, g, U, PIPE, grid, cnt, rearm, xloc, st);
  else attn_o_fmt<HD, G, QT_Q6_K>(b, sp, g, U, PIPE, grid, cnt, rearm, xloc, st);
}

static int attn_o_env() {  // read per call: tests flip it inside one process (captures call it once per layer)
  const char* e = std::getenv("AIOS_ATTN_O");
  return e ? std::atoi(e) : 0;
}

// Attention (a) then O (g: x = a.out, batch 1) as one launch; false (nothing launched) when the pair
// is outside what the fused kernel serves -- the caller then launches the two kernels.
bool launch_attn_o(const AttnDecodeArgs& a, const GemvArgs& g, int* cnt, int* rearm, float* xloc, hipStream_t st) {
  if (!attn_o_env() || !cnt || !rearm || !xloc || rearm == cnt) return false;
  if (a.B != 1 || g.B != 1 || a.out16 || !a.out || g.x != a.out || g.x16 || g.norm_w) return false;
  if (!g.act_q8 || g.force_v1 || g.nseg != 1 || g.tp || g.tune_dbg || g.tune_grid > 0) return false;
  if (g.epi != EPI_RESID && g.epi != EPI_STORE) return false;
  const int qt = g.seg[0].qtype;
  if (qt != QT_Q4_K && qt != QT_Q6_K) return false;
  if (g.N % 2 || g.K % 256) return false;
  if (a.n_heads % a.n_kv_heads || a.max_ctx % 128 || !a.counters) return false;
  const int G = a.n_heads / a.n_kv_heads;
  if (!((a.head_dim == 128 && (G == 1 || G == 4 || G == 8)) || (a.head_dim == 64 && G == 8))) return false;
  // one workgroup per CU; in the short mode an XCD's workgroups take one query head each
  const int cus = device_cu_count();
  if (cus % AO_XCDS || a.n_heads != cus / AO_XCDS) return false;
  // every pair's K slice in registers (U chunks per lane), one or two pairs per wave in both modes
  const int nch = g.K / 32;  // QFmt<Q4_K / Q6_K>::W
  const int npairs = g.N / 2;
  if (nch > 128 || npairs % (8 * cus)) return false;
  const int U = nch <= 64 ? 1 : 2;
  const int PIPE = npairs / (8 * cus);
  if (PIPE < 1 || PIPE > 2) return false;
  AttnDecodeArgs b = attn_resolve(a);
  // the long mode's split-K roles must fit the grid
  const int GL = (G % 4 == 0) ? 4 : G;
  const int pmax = std::max(1, cus / (a.n_kv_heads * (G / GL)));
  if (b.split / ATTN_CHUNK > pmax) b.split = pmax * ATTN_CHUNK;
  AttnSplit sp;
  const int nwg = attn_plan(b, G, sp);
  sp.xcd = attn_env_int("AIOS_ATTN_XCD", 1) | (attn_env_int("AIOS_ATTN_O_POLL", 2) << 2);
  sp.n_attn = nwg;
  if (nwg > cus) return false;
  if (a.head_dim == 128) {
    if (G == 1) attn_o_g<128, 1>(b, sp, g, U, PIPE, cus, cnt, rearm, xloc, st);
    else if (G == 4) attn_o_g<128, 4>(b, sp, g, U, PIPE, cus, cnt, rearm, xloc, st);
    else attn_o_g<128, 8>(b, sp, g, U, PIPE, cus, cnt, rearm, xloc, st);
  } else {
    attn_o_g<64, 8>(b, sp, g, U, PIPE, cus, cnt, rearm, xloc, st);
  }
  return true;
}

}  // namespace aios
