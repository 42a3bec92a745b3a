// Split-K flash-decode GQA attention over the bf16 KV cache (decode shape),
// with the log-sum-exp combine fused in (last-arriving workgroup per (row, kv-head)).
//
// grid = (ceil(max_ctx / ATTN_SPLIT), n_kv_heads, B); a 256-thread workgroup handles one KV head x
// one split of ATTN_SPLIT keys (walked in ATTN_CHUNK-key chunks, online softmax) for all
// G = n_heads/n_kv_heads query heads of the group, so each K/V byte is read once per group (GQA
// reuse).  Latency is what matters at decode sizes, so every global load
// a lane needs (its q slice, and its K and V rows) is issued up front: K/V rows below max_ctx are
// always valid memory, so the loads do not wait for seq_len -- keys past it are masked after.
// K/V go straight to VGPRs (16 B per lane, LPK = hd/8 lanes per key: the 'attention decode' row
// of the CDNA guide's Appendix B); scores and the chunk softmax live in LDS.
//
// Combine: each chunk writes its unnormalised partial (o, m, l) with write-through (sc1, agent
// scope) stores, drains them (s_waitcnt vmcnt(0)), and after a workgroup barrier one lane bumps
// an agent-scope counter for (row, kv head).  The workgroup that draws the last ticket reads all
// partials with sc1 loads and writes the normalised output, then re-arms the counter -- the
// write-through hand-off of CDNA guide §6 Guideline 16 / split-K item 2 (no release/acquire
// fences, placement independent).  Splits past seq_len exit before arriving; the expected
// arrivals are ceil(seq_len / ATTN_SPLIT) -- one, i.e. no hand-off at all, up to ATTN_SPLIT keys.
#include "../common.h"
#include "../ops.h"

namespace aios {

__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void bf16x8_to_f32(const uint4& v, float f[8]) {
  f[0] = bf16_to_f32(v.x & 0xffff); f[1] = bf16_to_f32(v.x >> 16);
  f[2] = bf16_to_f32(v.y & 0xffff); f[3] = bf16_to_f32(v.y >> 16);
  f[4] = bf16_to_f32(v.z & 0xffff); f[5] = bf16_to_f32(v.z >> 16);
  f[6] = bf16_to_f32(v.w & 0xffff); f[7] = bf16_to_f32(v.w >> 16);
}

// keys per workgroup ("split"): the workgroup walks its split in ATTN_CHUNK-key chunks with an
// online softmax, prefetching chunk c+1 into registers while chunk c is scored -- so a context of
// up to ATTN_SPLIT keys needs one workgroup per KV head and no cross-workgroup combine at all.
constexpr int ATTN_CPW = 8;
constexpr int ATTN_SPLIT = ATTN_CHUNK * ATTN_CPW;

template <int HD, int G>
__global__ void __launch_bounds__(256) attn_decode_kernel(AttnDecodeArgs a) {
  constexpr int LPK = HD / 8;        // lanes per key (8 dims per lane)
  constexpr int KPS = 64 / LPK;      // keys per wave step
  constexpr int CH = ATTN_CHUNK;
  constexpr int KPW = CH / 4;        // keys per wave per chunk
  constexpr int STEPS = KPW / KPS;
  __shared__ float s_p[2][G][CH];
  __shared__ float s_o[4][G][HD];
  __shared__ float s_m[G], s_l[G], s_alpha[G];
  __shared__ int s_last;

  const int sp = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int start = sp * ATTN_SPLIT;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ksub = lane / LPK, dsl = lane % LPK;
  const int slot = a.slot ? a.slot[b] : b;
  const size_t kv_base = (((size_t)slot * a.n_kv_heads + kvh) * a.max_ctx) * HD;
  const bf16_t* kc = a.k_cache + kv_base;
  const bf16_t* vc = a.v_cache + kv_base;
  const int koff = wave * KPW + ksub;  // this lane's key within a chunk (+ s * KPS)

  // ---- first chunk's loads up front (rows below max_ctx are always valid memory)
  uint4 kraw[STEPS], vraw[STEPS];
#pragma unroll
  for (int s = 0; s < STEPS; ++s) kraw[s] = *(const uint4*)(kc + (size_t)(start + koff + s * KPS) * HD + dsl * 8);
  float q[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float* qp = a.q + ((size_t)b * a.n_heads + kvh * G + g) * HD + dsl * 8;
    const float4 q0 = *(const float4*)qp, q1 = *(const float4*)(qp + 4);
    q[g][0] = q0.x; q[g][1] = q0.y; q[g][2] = q0.z; q[g][3] = q0.w;
    q[g][4] = q1.x; q[g][5] = q1.y; q[g][6] = q1.z; q[g][7] = q1.w;
  }
#pragma unroll
  for (int s = 0; s < STEPS; ++s) vraw[s] = *(const uint4*)(vc + (size_t)(start + koff + s * KPS) * HD + dsl * 8);
  const int len = a.seq_len[b];
  if (start >= len) return;
  const int nkeys = min(ATTN_SPLIT, len - start);
  const int nch = (nkeys + CH - 1) / CH;
  if (threadIdx.x < G) {
    s_m[threadIdx.x] = -INFINITY;
    s_l[threadIdx.x] = 0.f;
  }
  float o[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int i = 0; i < 8; ++i) o[g][i] = 0.f;

  for (int c = 0; c < nch; ++c) {
    const int cstart = start + c * CH;
    const int n = min(CH, len - cstart);
    float(*pb)[CH] = s_p[c & 1];
    // prefetch the next chunk (address clamped into the cache; only used when it exists)
    const int nstart = min(cstart + CH, a.max_ctx - CH);
    uint4 kn[STEPS], vn[STEPS];
#pragma unroll
    for (int s = 0; s < STEPS; ++s) kn[s] = *(const uint4*)(kc + (size_t)(nstart + koff + s * KPS) * HD + dsl * 8);
#pragma unroll
    for (int s = 0; s < STEPS; ++s) vn[s] = *(const uint4*)(vc + (size_t)(nstart + koff + s * KPS) * HD + dsl * 8);
    // ---- scores
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      const int kl = koff + s * KPS;
      float kf[8];
      bf16x8_to_f32(kraw[s], kf);
      float dot[G];
#pragma unroll
      for (int g = 0; g < G; ++g) {
        dot[g] = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) dot[g] = fmaf(q[g][i], kf[i], dot[g]);
#pragma unroll
        for (int off = LPK / 2; off > 0; off >>= 1) dot[g] += __shfl_xor(dot[g], off, 64);
      }
      if (dsl == 0) {
#pragma unroll
        for (int g = 0; g < G; ++g) pb[g][kl] = kl < n ? dot[g] * a.scale : -INFINITY;
      }
    }
    __syncthreads();
    // ---- online softmax: wave w owns heads w, w+4, ... (CH = 64 keys = one per lane)
    for (int g = wave; g < G; g += 4) {
      const float v = pb[g][lane];
      const float mc = wave_max(v);
      const float m_old = s_m[g];
      const float m_new = fmaxf(m_old, mc);
      const float p = (lane < n) ? __expf(v - m_new) : 0.f;
      const float l = wave_sum(p);
      pb[g][lane] = p;
      if (lane == 0) {
        const float alpha = __expf(m_old - m_new);  // 0 on the first chunk (m_old = -inf)
        s_alpha[g] = alpha;
        s_l[g] = s_l[g] * alpha + l;
        s_m[g] = m_new;
      }
    }
    __syncthreads();
    // ---- rescale + P.V
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const float al = s_alpha[g];
#pragma unroll
      for (int i = 0; i < 8; ++i) o[g][i] *= al;
    }
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      const int kl = koff + s * KPS;
      float vf[8];
      bf16x8_to_f32(vraw[s], vf);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float p = pb[g][kl];  // 0 for masked keys
#pragma unroll
        for (int i = 0; i < 8; ++i) o[g][i] = fmaf(p, vf[i], o[g][i]);
      }
    }
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      kraw[s] = kn[s];
      vraw[s] = vn[s];
    }
  }
  // ---- reduce o over the keys of a wave (lanes with equal dsl), then over the 4 waves
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int off = LPK; off < 64; off <<= 1) o[g][i] += __shfl_xor(o[g][i], off, 64);
  if (ksub == 0) {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int i = 0; i < 8; ++i) s_o[wave][g][dsl * 8 + i] = o[g][i];
  }
  __syncthreads();

  const int nact = (len + ATTN_SPLIT - 1) / ATTN_SPLIT;  // splits that arrive
  if (nact == 1) {  // whole context in this workgroup: normalise directly, no hand-off
    for (int idx = threadIdx.x; idx < G * HD; idx += 256) {
      const int g = idx / HD, d = idx - g * HD;
      const float v = s_o[0][g][d] + s_o[1][g][d] + s_o[2][g][d] + s_o[3][g][d];
      a.out[((size_t)b * a.n_heads + kvh * G + g) * HD + d] = v / s_l[g];
    }
    return;
  }
  // ---- publish this split's partial (write-through), then take a ticket
  for (int idx = threadIdx.x; idx < G * HD; idx += 256) {
    const int g = idx / HD, d = idx - g * HD;
    const float v = s_o[0][g][d] + s_o[1][g][d] + s_o[2][g][d] + s_o[3][g][d];
    const int h = kvh * G + g;
    st_wt(a.o_part + (((size_t)b * a.n_heads + h) * a.n_chunks + sp) * HD + d, v);
    if (d == 0) {
      float* ml = a.ml + (((size_t)b * a.n_heads + h) * a.n_chunks + sp) * 2;
      st_wt(ml, s_m[g]);
      st_wt(ml + 1, s_l[g]);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  int* cnt = a.counters + (size_t)b * a.n_kv_heads + kvh;
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == nact - 1);
  }
  __syncthreads();
  if (!s_last) return;
  // ---- last arriver: log-sum-exp combine over the nact splits (sc1 loads of every partial)
  for (int idx = threadIdx.x; idx < G * HD; idx += 256) {
    const int g = idx / HD, d = idx - g * HD;
    const int h = kvh * G + g;
    const float* ml = a.ml + ((size_t)b * a.n_heads + h) * a.n_chunks * 2;
    const float* op = a.o_part + ((size_t)b * a.n_heads + h) * a.n_chunks * HD;
    float M = -INFINITY;
    for (int c = 0; c < nact; ++c) M = fmaxf(M, ld_wt(ml + 2 * c));
    float L = 0.f, acc = 0.f;
    for (int c = 0; c < nact; ++c) {
      const float w = __expf(ld_wt(ml + 2 * c) - M);
      L += w * ld_wt(ml + 2 * c + 1);
      acc += w * ld_wt(op + (size_t)c * HD + d);
    }
    a.out[((size_t)b * a.n_heads + h) * HD + d] = acc / L;
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
}

template <int HD>
static void launch_hd(const AttnDecodeArgs& a, int G, hipStream_t st) {
  dim3 grid((a.max_ctx + ATTN_SPLIT - 1) / ATTN_SPLIT, a.n_kv_heads, a.B);
  if ((int)grid.x > a.n_chunks) throw std::runtime_error("attn_decode: partial buffers smaller than the split count");
  switch (G) {
    case 1: hipLaunchKernelGGL((attn_decode_kernel<HD, 1>), grid, dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((attn_decode_kernel<HD, 2>), grid, dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL((attn_decode_kernel<HD, 4>), grid, dim3(256), 0, st, a); break;
    case 5: hipLaunchKernelGGL((attn_decode_kernel<HD, 5>), grid, dim3(256), 0, st, a); break;
    case 8: hipLaunchKernelGGL((attn_decode_kernel<HD, 8>), grid, dim3(256), 0, st, a); break;
    default: throw std::runtime_error("attn_decode: unsupported GQA group size " + std::to_string(G));
  }
}

void launch_attn_decode(const AttnDecodeArgs& a, hipStream_t st) {
  if (a.n_heads % a.n_kv_heads) throw std::runtime_error("attn_decode: n_heads % n_kv_heads != 0");
  if (!a.counters) throw std::runtime_error("attn_decode: counters buffer required");
  if (a.max_ctx % ATTN_CHUNK) throw std::runtime_error("attn_decode: max_ctx must be a multiple of ATTN_CHUNK");
  const int G = a.n_heads / a.n_kv_heads;
  if (a.head_dim == 128) launch_hd<128>(a, G, st);
  else if (a.head_dim == 64) launch_hd<64>(a, G, st);
  else throw std::runtime_error("attn_decode: head_dim must be 64 or 128");
}

}  // namespace aios
