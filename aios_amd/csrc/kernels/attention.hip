// Split-K flash-decode GQA attention over the bf16 KV cache (decode shape).
//
// grid = (n_chunks, n_kv_heads, B); a 256-thread workgroup handles one KV head x one chunk of
// ATTN_CHUNK keys for all G = n_heads/n_kv_heads query heads of the group, so each K/V byte is
// read once per group (GQA reuse).  K/V rows go straight to VGPRs (16 B per lane, LPK = hd/8
// lanes per key -- the 'attention decode' row of the CDNA guide's Appendix B); scores and the
// chunk softmax live in LDS; each chunk emits an unnormalised partial (o, m, l) that a tiny
// combine kernel merges (log-sum-exp).  Chunks past seq_len exit immediately, so the grid can be
// sized for max_ctx and captured once in a hipGraph while the context grows.
#include "../common.h"
#include "../ops.h"

namespace aios {

template <int HD, int G>
__global__ void __launch_bounds__(256) attn_decode_kernel(AttnDecodeArgs a) {
  constexpr int LPK = HD / 8;        // lanes per key (8 dims per lane)
  constexpr int KPS = 64 / LPK;      // keys per wave step
  constexpr int CH = ATTN_CHUNK;
  __shared__ float s_p[G][CH];
  __shared__ float s_o[4][G][HD];
  __shared__ float s_m[G], s_l[G];

  const int ch = blockIdx.x, kvh = blockIdx.y, b = blockIdx.z;
  const int len = a.seq_len[b];
  const int start = ch * CH;
  if (start >= len) return;
  const int n = min(CH, len - start);
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ksub = lane / LPK, dsl = lane % LPK;
  const int slot = a.slot ? a.slot[b] : b;
  const size_t kv_base = (((size_t)slot * a.n_kv_heads + kvh) * a.max_ctx) * HD;
  const bf16_t* kc = a.k_cache + kv_base;
  const bf16_t* vc = a.v_cache + kv_base;

  // q slice for the group's G heads: 8 dims per lane
  float q[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g) {
    const float* qp = a.q + ((size_t)b * a.n_heads + kvh * G + g) * HD + dsl * 8;
    const float4 q0 = *(const float4*)qp, q1 = *(const float4*)(qp + 4);
    q[g][0] = q0.x * a.scale; q[g][1] = q0.y * a.scale; q[g][2] = q0.z * a.scale; q[g][3] = q0.w * a.scale;
    q[g][4] = q1.x * a.scale; q[g][5] = q1.y * a.scale; q[g][6] = q1.z * a.scale; q[g][7] = q1.w * a.scale;
  }

  // ---- scores: wave w handles keys [w*CH/4, (w+1)*CH/4) of the chunk
  constexpr int KPW = CH / 4;
#pragma unroll
  for (int s = 0; s < KPW / KPS; ++s) {
    const int kl = wave * KPW + s * KPS + ksub;
    float dot[G];
#pragma unroll
    for (int g = 0; g < G; ++g) dot[g] = 0.f;
    if (kl < n) {
      const uint4 kv = *(const uint4*)(kc + (size_t)(start + kl) * HD + dsl * 8);
      float kf[8];
      kf[0] = bf16_to_f32(kv.x & 0xffff); kf[1] = bf16_to_f32(kv.x >> 16);
      kf[2] = bf16_to_f32(kv.y & 0xffff); kf[3] = bf16_to_f32(kv.y >> 16);
      kf[4] = bf16_to_f32(kv.z & 0xffff); kf[5] = bf16_to_f32(kv.z >> 16);
      kf[6] = bf16_to_f32(kv.w & 0xffff); kf[7] = bf16_to_f32(kv.w >> 16);
#pragma unroll
      for (int g = 0; g < G; ++g)
#pragma unroll
        for (int i = 0; i < 8; ++i) dot[g] = fmaf(q[g][i], kf[i], dot[g]);
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
#pragma unroll
      for (int o = LPK / 2; o > 0; o >>= 1) dot[g] += __shfl_xor(dot[g], o, 64);
    }
    if (dsl == 0) {
#pragma unroll
      for (int g = 0; g < G; ++g) s_p[g][kl] = kl < n ? dot[g] : -INFINITY;
    }
  }
  __syncthreads();

  // ---- chunk softmax: wave w handles heads w, w+4, ...  (CH = 64 keys = one per lane)
  for (int g = wave; g < G; g += 4) {
    const float v = s_p[g][lane];
    const float m = wave_max(v);
    const float p = (lane < n) ? __expf(v - m) : 0.f;
    const float l = wave_sum(p);
    s_p[g][lane] = p;
    if (lane == 0) { s_m[g] = m; s_l[g] = l; }
  }
  __syncthreads();

  // ---- P.V
  float o[G][8];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int i = 0; i < 8; ++i) o[g][i] = 0.f;
#pragma unroll
  for (int s = 0; s < KPW / KPS; ++s) {
    const int kl = wave * KPW + s * KPS + ksub;
    if (kl < n) {
      const uint4 vv = *(const uint4*)(vc + (size_t)(start + kl) * HD + dsl * 8);
      float vf[8];
      vf[0] = bf16_to_f32(vv.x & 0xffff); vf[1] = bf16_to_f32(vv.x >> 16);
      vf[2] = bf16_to_f32(vv.y & 0xffff); vf[3] = bf16_to_f32(vv.y >> 16);
      vf[4] = bf16_to_f32(vv.z & 0xffff); vf[5] = bf16_to_f32(vv.z >> 16);
      vf[6] = bf16_to_f32(vv.w & 0xffff); vf[7] = bf16_to_f32(vv.w >> 16);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const float p = s_p[g][kl];
#pragma unroll
        for (int i = 0; i < 8; ++i) o[g][i] = fmaf(p, vf[i], o[g][i]);
      }
    }
  }
  // reduce over the KPS key-lanes of the wave (lanes with equal dsl)
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
  // across the 4 waves, write the partial
  for (int idx = threadIdx.x; idx < G * HD; idx += 256) {
    const int g = idx / HD, d = idx - g * HD;
    const float v = s_o[0][g][d] + s_o[1][g][d] + s_o[2][g][d] + s_o[3][g][d];
    const int h = kvh * G + g;
    a.o_part[(((size_t)b * a.n_heads + h) * a.n_chunks + ch) * HD + d] = v;
    if (d == 0) {
      float* ml = a.ml + (((size_t)b * a.n_heads + h) * a.n_chunks + ch) * 2;
      ml[0] = s_m[g];
      ml[1] = s_l[g];
    }
  }
}

// grid (n_heads, B), block = hd threads
__global__ void attn_combine_kernel(AttnDecodeArgs a) {
  const int h = blockIdx.x, b = blockIdx.y, d = threadIdx.x;
  const int HD = a.head_dim;
  const int len = a.seq_len[b];
  const int nch = min(a.n_chunks, (len + ATTN_CHUNK - 1) / ATTN_CHUNK);
  const float* ml = a.ml + ((size_t)b * a.n_heads + h) * a.n_chunks * 2;
  float M = -INFINITY;
  for (int c = 0; c < nch; ++c) M = fmaxf(M, ml[2 * c]);
  float L = 0.f, acc = 0.f;
  const float* op = a.o_part + ((size_t)b * a.n_heads + h) * a.n_chunks * HD;
  for (int c = 0; c < nch; ++c) {
    const float w = __expf(ml[2 * c] - M);
    L += w * ml[2 * c + 1];
    acc += w * op[(size_t)c * HD + d];
  }
  a.out[((size_t)b * a.n_heads + h) * HD + d] = nch > 0 ? acc / L : 0.f;
}

template <int HD>
static void launch_hd(const AttnDecodeArgs& a, int G, hipStream_t st) {
  dim3 grid(a.n_chunks, a.n_kv_heads, a.B);
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
  const int G = a.n_heads / a.n_kv_heads;
  if (a.head_dim == 128) launch_hd<128>(a, G, st);
  else if (a.head_dim == 64) launch_hd<64>(a, G, st);
  else throw std::runtime_error("attn_decode: head_dim must be 64 or 128");
  hipLaunchKernelGGL(attn_combine_kernel, dim3(a.n_heads, a.B), dim3(a.head_dim), 0, st, a);
}

}  // namespace aios
