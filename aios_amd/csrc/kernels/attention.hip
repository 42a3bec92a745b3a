// Split-K flash-decode GQA attention over the bf16 KV cache (decode shape),
// with the log-sum-exp combine fused in (last-arriving workgroup per (row, kv-head)).
//
// grid = (Pmax, n_kv_heads, B), 256 threads.  The context is cut into 64-key chunks; with P
// active workgroups chunk c belongs to workgroup c % P (pass c / P).  P is 1 up to 3 chunks (a
// pass is cheaper than the cross-workgroup combine) and min(chunks, Pmax) beyond, Pmax (host,
// ~256 workgroups per grid) spreading one KV head over up to 64 CUs -- one CU streams only tens
// of GB/s, so the previous one-workgroup-per-head chunk walk was bandwidth- and latency-bound
// (2.2 us per serial 64-key chunk, 142 us at 4000 keys on MI355X; now 12 us, tools/attn_probe.py).
// Workgroup 0 issues chunk 0 before seq_len arrives (it always exists).
//
// Inside a pass every lane issues all its K and V loads at once (16 B = 8 dims per lane, LPK =
// hd/8 lanes per key, 16 keys per wave) and the next pass's loads are issued before the current
// pass is scored.  Each WAVE keeps its own online-softmax state (m, l, o) for the G = H/Hkv query
// heads of the group -- scores are reduced over the LPK lanes of a key with DPP (no LDS), and no
// workgroup barrier is needed until the four waves merge their states in LDS at the end.
//
// Combine: with more than one active workgroup each writes its partial (o, m, l) with
// write-through (sc1, agent scope) stores, drains them (s_waitcnt vmcnt(0)), and after a
// workgroup barrier one lane takes an agent-scope ticket for (row, kv head).  The last arriver
// reads every partial's (m, l) in one parallel sweep (one lane per partial), then each thread
// sums its outputs over the partials with independent loads -- the write-through hand-off of
// CDNA guide §6 Guideline 16 / split-K item 2 -- and re-arms the counter.
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

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, false));
}
// sum over aligned groups of N lanes (N = 8 or 16), result in every lane of the group
template <int N>
__device__ __forceinline__ float group_sum(float v) {
  v += dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += dpp<0x141>(v);  // row_half_mirror: lane i <-> 7-i within 8
  if constexpr (N == 16) v += dpp<0x140>(v);  // row_mirror: lane i <-> 15-i within 16
  return v;
}
// max / sum over the lanes that share (lane % LPK), i.e. across the 64/LPK key groups of a wave
template <int LPK>
__device__ __forceinline__ float keys_max(float v) {
#pragma unroll
  for (int off = LPK; off < 64; off <<= 1) v = fmaxf(v, __shfl_xor(v, off, 64));
  return v;
}
template <int LPK>
__device__ __forceinline__ float keys_sum(float v) {
#pragma unroll
  for (int off = LPK; off < 64; off <<= 1) v += __shfl_xor(v, off, 64);
  return v;
}

constexpr float kLog2e = 1.4426950408889634f;

template <int HD, int G>
__global__ void __launch_bounds__(256) attn_decode_kernel(AttnDecodeArgs a) {
  constexpr int LPK = HD / 8;          // lanes per key (8 dims per lane)
  constexpr int KPS = 64 / LPK;        // keys per wave-instruction
  constexpr int CH = ATTN_CHUNK;       // keys per workgroup pass
  constexpr int KPW = CH / 4;          // keys per wave per pass
  constexpr int STEPS = KPW / KPS;     // loads per lane per pass (each of K and V)
  constexpr int NG0 = 64 / LPK;        // key groups per wave
  // per (wave, key group) unnormalised outputs in LDS when that fits in 32 KB; otherwise the key
  // groups are first summed with cross-lane shuffles and only one group per wave is stored
  constexpr int NG = (4 * NG0 * G * HD * 4 <= 32768) ? NG0 : 1;
  __shared__ float s_o[4][NG][G][HD];
  __shared__ float s_m[4][G], s_l[4][G];
  __shared__ int s_last;

  const int sp = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ksub = lane / LPK, dsl = lane % LPK;
  const int slot = a.slot ? a.slot[b] : b;
  const size_t kv_base = (((size_t)slot * a.n_kv_heads + kvh) * a.max_ctx) * HD;
  const bf16_t* kc = a.k_cache + kv_base + dsl * 8;
  const bf16_t* vc = a.v_cache + kv_base + dsl * 8;
  const int koff = wave * KPW + ksub;  // this lane's key within a chunk (+ s * KPS)

  uint4 kr[STEPS], vr[STEPS];
  auto issue = [&](int chunk) {  // chunk < max_ctx / CH: always valid memory
    const int k0 = chunk * CH + koff;
#pragma unroll
    for (int s = 0; s < STEPS; ++s) kr[s] = *(const uint4*)(kc + (size_t)(k0 + s * KPS) * HD);
#pragma unroll
    for (int s = 0; s < STEPS; ++s) vr[s] = *(const uint4*)(vc + (size_t)(k0 + s * KPS) * HD);
  };
  // chunk 0 always exists (seq_len >= 1): workgroup 0 issues it before seq_len arrives
  if (sp == 0) issue(0);
  const int len = a.seq_len[b];
  const int nchunk = (len + CH - 1) / CH;
  // active workgroups: up to 3 chunks are walked by one workgroup (a pass costs less than the
  // cross-workgroup combine), beyond that one chunk per workgroup up to the grid's P
  const int P = nchunk <= 3 ? 1 : min(nchunk, (int)gridDim.x);
  if (sp >= P) return;  // uniform: this workgroup has no chunk, issues no K/V traffic
  if (sp != 0) issue(sp);
  const float qs = a.scale * kLog2e;  // scores in the log2 domain: exp2 below
  float q[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float* qp = a.q + ((size_t)b * a.n_heads + kvh * G + g) * HD + dsl * 8;
    const float4 q0 = *(const float4*)qp, q1 = *(const float4*)(qp + 4);
    q[g][0] = q0.x * qs; q[g][1] = q0.y * qs; q[g][2] = q0.z * qs; q[g][3] = q0.w * qs;
    q[g][4] = q1.x * qs; q[g][5] = q1.y * qs; q[g][6] = q1.z * qs; q[g][7] = q1.w * qs;
  }
  float m[G], l[G], o[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) o[g][i] = 0.f;
  }
  for (int c = sp; c < nchunk; c += P) {
    uint4 kc_[STEPS], vc_[STEPS];
#pragma unroll
    for (int s = 0; s < STEPS; ++s) { kc_[s] = kr[s]; vc_[s] = vr[s]; }
    if (c + P < nchunk) issue(c + P);  // next pass in flight while this one is scored
    // ---- scores of this lane's STEPS keys for the G heads (reduced over the key's LPK lanes)
    float sc[STEPS][G];
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      float kf[8];
      bf16x8_to_f32(kc_[s], kf);
      const bool valid = c * CH + koff + s * KPS < len;
#pragma unroll
      for (int g = 0; g < G; ++g) {
        float d = 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i) d = fmaf(q[g][i], kf[i], d);
        d = group_sum<LPK>(d);
        sc[s][g] = valid ? d : -INFINITY;
      }
    }
    // ---- per-wave online softmax over this pass's KPW keys
#pragma unroll
    for (int g = 0; g < G; ++g) {
      float mx = sc[0][g];
#pragma unroll
      for (int s = 1; s < STEPS; ++s) mx = fmaxf(mx, sc[s][g]);
      mx = keys_max<LPK>(mx);
      const float mn = fmaxf(m[g], mx);  // finite: the pass holds >= 1 valid key per wave? not always
      const float alpha = (mn == -INFINITY) ? 1.f : exp2f(m[g] - mn);
      float ps = 0.f;
#pragma unroll
      for (int s = 0; s < STEPS; ++s) {
        const float p = (sc[s][g] == -INFINITY) ? 0.f : exp2f(sc[s][g] - mn);
        sc[s][g] = p;
        ps += p;
      }
      l[g] = l[g] * alpha + keys_sum<LPK>(ps);
      m[g] = mn;
#pragma unroll
      for (int i = 0; i < 8; ++i) o[g][i] *= alpha;
    }
    // ---- P.V (lane-local over its keys; merged across key groups and waves at the end)
#pragma unroll
    for (int s = 0; s < STEPS; ++s) {
      float vf[8];
      bf16x8_to_f32(vc_[s], vf);
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 8; ++i) o[g][i] = fmaf(sc[s][g], vf[i], o[g][i]);
    }
  }
  // ---- merge the 4 waves x NG key groups (one barrier)
  if constexpr (NG == 1) {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int i = 0; i < 8; ++i) o[g][i] = keys_sum<LPK>(o[g][i]);
    if (ksub == 0) {
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 8; ++i) s_o[wave][0][g][dsl * 8 + i] = o[g][i];
    }
  } else {
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int i = 0; i < 8; ++i) s_o[wave][ksub][g][dsl * 8 + i] = o[g][i];
  }
  if (lane < G) {
    // m/l are wave-uniform after keys_max/keys_sum; lane g publishes head g
    float mv = m[0], lv = l[0];
#pragma unroll
    for (int g = 1; g < G; ++g)
      if (lane == g) { mv = m[g]; lv = l[g]; }
    s_m[wave][lane] = mv;
    s_l[wave][lane] = lv;
  }
  __syncthreads();
  const int nact = P;  // workgroups that arrive
  for (int idx = threadIdx.x; idx < G * HD; idx += 256) {
    const int g = idx / HD, d = idx - g * HD;
    float M = s_m[0][g];
#pragma unroll
    for (int w = 1; w < 4; ++w) M = fmaxf(M, s_m[w][g]);
    float L = 0.f, acc = 0.f;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const float sw = (s_m[w][g] == -INFINITY) ? 0.f : exp2f(s_m[w][g] - M);
      L += sw * s_l[w][g];
      float t = 0.f;
#pragma unroll
      for (int k = 0; k < NG; ++k) t += s_o[w][k][g][d];
      acc += sw * t;
    }
    const int h = kvh * G + g;
    if (nact == 1) {
      a.out[((size_t)b * a.n_heads + h) * HD + d] = acc / L;
    } else {
      st_wt(a.o_part + (((size_t)b * a.n_heads + h) * a.n_chunks + sp) * HD + d, acc);
      if (d == 0) {
        float* ml = a.ml + (((size_t)b * a.n_heads + h) * a.n_chunks + sp) * 2;
        st_wt(ml, M);
        st_wt(ml + 1, L);
      }
    }
  }
  if (nact == 1) return;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains its sc1 stores
  __syncthreads();
  int* cnt = a.counters + (size_t)b * a.n_kv_heads + kvh;
  if (threadIdx.x == 0) {
    const int t = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == nact - 1);
  }
  __syncthreads();
  if (!s_last) return;
  // ---- last arriver: each output sums its partials; m, l and o of 8 partials are loaded
  //      together (one memory round trip per 8 partials, online rescale across blocks)
  for (int idx = threadIdx.x; idx < G * HD; idx += 256) {
    const int g = idx / HD, d = idx - g * HD;
    const int h = kvh * G + g;
    const float* mlp = a.ml + ((size_t)b * a.n_heads + h) * a.n_chunks * 2;
    const float* op = a.o_part + ((size_t)b * a.n_heads + h) * a.n_chunks * HD + d;
    float M = -INFINITY, L = 0.f, acc = 0.f;
    for (int c = 0; c < nact; c += 8) {
      float mv[8], lv[8], ov[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int cc = min(c + j, nact - 1);
        mv[j] = ld_wt(mlp + 2 * cc);
        lv[j] = ld_wt(mlp + 2 * cc + 1);
        ov[j] = ld_wt(op + (size_t)cc * HD);
      }
      float mb = M;
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (c + j < nact) mb = fmaxf(mb, mv[j]);
      const float al = (M == -INFINITY) ? 0.f : exp2f(M - mb);
      L *= al;
      acc *= al;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (c + j < nact) {
          const float w = exp2f(mv[j] - mb);
          L = fmaf(w, lv[j], L);
          acc = fmaf(w, ov[j], acc);
        }
      }
      M = mb;
    }
    a.out[((size_t)b * a.n_heads + h) * HD + d] = acc / L;
  }
  if (threadIdx.x == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
}

template <int HD>
static void launch_hd(const AttnDecodeArgs& a, int G, hipStream_t st) {
  const int nch = (a.max_ctx + ATTN_CHUNK - 1) / ATTN_CHUNK;
  const int P = std::min(nch, a.split / ATTN_CHUNK);  // workgroups per (row, kv head)
  dim3 grid(P, a.n_kv_heads, a.B);
  if (P > a.n_chunks || P > 64) throw std::runtime_error("attn_decode: more splits than partial buffers / 64");
  switch (G) {
    case 1: hipLaunchKernelGGL((attn_decode_kernel<HD, 1>), grid, dim3(256), 0, st, a); break;
    case 2: hipLaunchKernelGGL((attn_decode_kernel<HD, 2>), grid, dim3(256), 0, st, a); break;
    case 4: hipLaunchKernelGGL((attn_decode_kernel<HD, 4>), grid, dim3(256), 0, st, a); break;
    case 5: hipLaunchKernelGGL((attn_decode_kernel<HD, 5>), grid, dim3(256), 0, st, a); break;
    case 8: hipLaunchKernelGGL((attn_decode_kernel<HD, 8>), grid, dim3(256), 0, st, a); break;
    default: throw std::runtime_error("attn_decode: unsupported GQA group size " + std::to_string(G));
  }
}

// `split` (kept in the args for the API) now encodes P * ATTN_CHUNK: the number of workgroups
// per (row, kv head).  Target ~256 workgroups for the whole grid (one per CU), 1..64 per head.
int attn_decode_split(int max_ctx, int B, int n_kv_heads) {
  const int nch = (max_ctx + ATTN_CHUNK - 1) / ATTN_CHUNK;
  const int P = std::max(1, std::min({64, nch, 256 / std::max(1, B * n_kv_heads)}));
  return P * ATTN_CHUNK;
}

void launch_attn_decode(const AttnDecodeArgs& a, hipStream_t st) {
  if (a.n_heads % a.n_kv_heads) throw std::runtime_error("attn_decode: n_heads % n_kv_heads != 0");
  if (!a.counters) throw std::runtime_error("attn_decode: counters buffer required");
  if (a.max_ctx % ATTN_CHUNK) throw std::runtime_error("attn_decode: max_ctx must be a multiple of ATTN_CHUNK");
  const int G = a.n_heads / a.n_kv_heads;
  AttnDecodeArgs b = a;
  if (b.split <= 0) b.split = attn_decode_split(a.max_ctx, a.B, a.n_kv_heads);
  if (b.split % ATTN_CHUNK) throw std::runtime_error("attn_decode: split must be a multiple of ATTN_CHUNK");
  if (a.head_dim == 128) launch_hd<128>(b, G, st);
  else if (a.head_dim == 64) launch_hd<64>(b, G, st);
  else throw std::runtime_error("attn_decode: head_dim must be 64 or 128");
}

}  // namespace aios
