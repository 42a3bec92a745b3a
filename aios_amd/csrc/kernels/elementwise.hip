// Memory-bound elementwise ops: RMSNorm (K2), casts, residual add (K8), SwiGLU (K7), the
// per-head QK-norm + RoPE + KV-cache write (K4/K5) for the unfused paths, and the on-device
// sampler (K9: greedy / Gumbel-max temperature sampling with top-k / top-p and an optional
// grammar bitmask for JSON mode, K10).  All loads are float4-vectorised (CDNA guide G13).
#include <algorithm>

#include "../common.h"
#include "../ops.h"

namespace aios {

template <typename OutT>
__global__ void rmsnorm_kernel(const float* __restrict__ x, int ldx, const float* __restrict__ w, OutT* __restrict__ y,
                               int ldy, int n, float eps) {
  __shared__ float red[32];
  const float* xr = x + (size_t)blockIdx.x * ldx;
  float s = 0.f;
  for (int i = threadIdx.x * 4; i < n; i += blockDim.x * 4) {
    const float4 v = *(const float4*)(xr + i);
    s += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  s = block_sum(s, red);
  const float ir = rsqrtf(s / (float)n + eps);
  OutT* yr = y + (size_t)blockIdx.x * ldy;
  for (int i = threadIdx.x * 4; i < n; i += blockDim.x * 4) {
    const float4 v = *(const float4*)(xr + i);
    const float4 g = *(const float4*)(w + i);
    const float o0 = v.x * ir * g.x, o1 = v.y * ir * g.y, o2 = v.z * ir * g.z, o3 = v.w * ir * g.w;
    if constexpr (sizeof(OutT) == 4) {
      *(float4*)((float*)yr + i) = make_float4(o0, o1, o2, o3);
    } else {
      const uint32_t lo = f32_to_bf16(o0) | ((uint32_t)f32_to_bf16(o1) << 16);
      const uint32_t hi = f32_to_bf16(o2) | ((uint32_t)f32_to_bf16(o3) << 16);
      *(uint2*)((bf16_t*)yr + i) = make_uint2(lo, hi);
    }
  }
}

void launch_rmsnorm(const float* x, int ldx, const float* w, float* y, int ldy, int rows, int n, float eps,
                    hipStream_t st) {
  hipLaunchKernelGGL(rmsnorm_kernel<float>, dim3(rows), dim3(256), 0, st, x, ldx, w, y, ldy, n, eps);
}
void launch_rmsnorm_bf16(const float* x, int ldx, const float* w, bf16_t* y, int ldy, int rows, int n, float eps,
                         hipStream_t st) {
  hipLaunchKernelGGL(rmsnorm_kernel<bf16_t>, dim3(rows), dim3(256), 0, st, x, ldx, w, y, ldy, n, eps);
}

__global__ void f32_to_bf16_kernel(const float* __restrict__ x, bf16_t* __restrict__ y, size_t n) {
  for (size_t i = ((size_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i < n; i += (size_t)gridDim.x * blockDim.x * 4) {
    if (i + 4 <= n) {
      const float4 v = *(const float4*)(x + i);
      const uint32_t lo = f32_to_bf16(v.x) | ((uint32_t)f32_to_bf16(v.y) << 16);
      const uint32_t hi = f32_to_bf16(v.z) | ((uint32_t)f32_to_bf16(v.w) << 16);
      *(uint2*)(y + i) = make_uint2(lo, hi);
    } else {
      for (size_t k = i; k < n; ++k) y[k] = f32_to_bf16(x[k]);
    }
  }
}
void launch_f32_to_bf16(const float* x, bf16_t* y, size_t n, hipStream_t st) {
  const int g = (int)std::min<size_t>(2048, (n / 4 + 255) / 256 + 1);
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(g), dim3(256), 0, st, x, y, n);
}

__global__ void add_kernel(float* __restrict__ y, const float* __restrict__ x, size_t n) {
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) y[i] += x[i];
}
void launch_add(float* y, const float* x, size_t n, hipStream_t st) {
  const int g = (int)std::min<size_t>(2048, (n + 255) / 256);
  hipLaunchKernelGGL(add_kernel, dim3(g), dim3(256), 0, st, y, x, n);
}

__global__ void swiglu_kernel(const float* __restrict__ gu, int ldg, float* __restrict__ out, int ldo, int n) {
  const float* g = gu + (size_t)blockIdx.y * ldg;
  float* o = out + (size_t)blockIdx.y * ldo;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float2 v = *(const float2*)(g + 2 * i);
    o[i] = v.x / (1.f + __expf(-v.x)) * v.y;
  }
}
__global__ void swiglu_bf16_kernel(const float* __restrict__ gu, int ldg, bf16_t* __restrict__ out, int ldo, int n) {
  const float* g = gu + (size_t)blockIdx.y * ldg;
  bf16_t* o = out + (size_t)blockIdx.y * ldo;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const float2 v = *(const float2*)(g + 2 * i);
    o[i] = f32_to_bf16(v.x / (1.f + __expf(-v.x)) * v.y);
  }
}
void launch_swiglu_interleaved_bf16(const float* gu, int ldg, bf16_t* out, int ldo, int rows, int n, hipStream_t st) {
  const int gx = std::min(64, (n + 255) / 256);
  hipLaunchKernelGGL(swiglu_bf16_kernel, dim3(gx, rows), dim3(256), 0, st, gu, ldg, out, ldo, n);
}
void launch_swiglu_interleaved(const float* gu, int ldg, float* out, int ldo, int rows, int n, hipStream_t st) {
  const int gx = std::min(64, (n + 255) / 256);
  hipLaunchKernelGGL(swiglu_kernel, dim3(gx, rows), dim3(256), 0, st, gu, ldg, out, ldo, n);
}

// grid (T, n_heads + 2*n_kv_heads), one wave per head
__global__ void qkv_post_kernel(QkvPostArgs a) {
  const int t = blockIdx.x, h = blockIdx.y, lane = threadIdx.x;
  const int hd = a.head_dim, half = hd >> 1;
  const int qd = a.n_heads * hd, kvd = a.n_kv_heads * hd;
  int part, head;
  if (h < a.n_heads) { part = 0; head = h; }
  else if (h < a.n_heads + a.n_kv_heads) { part = 1; head = h - a.n_heads; }
  else { part = 2; head = h - a.n_heads - a.n_kv_heads; }
  const int col0 = (part == 0 ? 0 : (part == 1 ? qd : qd + kvd)) + head * hd;
  const float* src = a.qkv + (size_t)t * a.ldqkv + col0;
  const float* bias = a.bias ? a.bias + col0 : nullptr;  // QKV bias (Qwen2-style), before norm/RoPE
  auto val = [&](int i) { return bias ? src[i] + bias[i] : src[i]; };
  const int pos = a.pos[t];
  const int slot = a.slot ? a.slot[t] : 0;
  float inv = 1.f;
  const float* nw = part == 0 ? a.q_norm : (part == 1 ? a.k_norm : nullptr);
  if (nw) {
    float s = 0.f;
    for (int i = lane; i < hd; i += 64) s += val(i) * val(i);
    s = wave_sum(s);
    inv = rsqrtf(s / (float)hd + a.eps);
  }
  for (int p = lane; p < half; p += 64) {
    int ia, ib;
    if (part == 2) { ia = 2 * p; ib = 2 * p + 1; }
    else if (a.rope_neox) { ia = p; ib = p + half; }
    else { ia = 2 * p; ib = 2 * p + 1; }
    float v0 = val(ia), v1 = val(ib);
    if (nw) { v0 *= inv * nw[ia]; v1 *= inv * nw[ib]; }
    if (part < 2) {
      float sn, cs;
      if (a.rope_cs) {
        const float2 t = a.rope_cs[(size_t)pos * half + p];
        cs = t.x; sn = t.y;
      } else {
        const float theta = (float)pos * powf(a.rope_base, -2.f * (float)p / (float)hd);
        sincosf(theta, &sn, &cs);
      }
      const float o0 = v0 * cs - v1 * sn, o1 = v0 * sn + v1 * cs;
      v0 = o0; v1 = o1;
    }
    if (part == 0) {
      float* q = a.q_out + (size_t)t * qd + head * hd;
      q[ia] = v0; q[ib] = v1;
    } else {
      bf16_t* cache = part == 1 ? a.k_cache : a.v_cache;
      const size_t base = (((size_t)slot * a.n_kv_heads + head) * a.max_ctx + pos) * hd;
      cache[base + ia] = f32_to_bf16(v0);
      cache[base + ib] = f32_to_bf16(v1);
    }
  }
}
void launch_qkv_post(const QkvPostArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(qkv_post_kernel, dim3(a.T, a.n_heads + 2 * a.n_kv_heads), dim3(64), 0, st, a);
}

// ----------------------------------------------------------------------------------------------
// sampler: one 1024-thread workgroup per batch row
// ----------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mix32(uint64_t x) {
  x ^= x >> 33;
  x *= 0xff51afd7ed558ccdULL;
  x ^= x >> 33;
  x *= 0xc4ceb9fe1a85ec53ULL;
  x ^= x >> 33;
  return (uint32_t)x;
}

struct ArgMax {
  float v;
  int i;
};
__device__ __forceinline__ ArgMax am_better(ArgMax a, ArgMax b) {
  return (b.v > a.v || (b.v == a.v && b.i < a.i)) ? b : a;
}

__device__ ArgMax block_argmax(ArgMax m, float* sv, int* si) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    ArgMax t;
    t.v = __shfl_xor(m.v, o, 64);
    t.i = __shfl_xor(m.i, o, 64);
    m = am_better(m, t);
  }
  __syncthreads();
  if (lane == 0) { sv[wid] = m.v; si[wid] = m.i; }
  __syncthreads();
  ArgMax r{-INFINITY, 0x7fffffff};
  for (int k = 0; k < nw; ++k) r = am_better(r, ArgMax{sv[k], si[k]});
  return r;
}

__device__ float block_count_ge(const float* l, int V, const uint8_t* mask, float t, float* red) {
  float c = 0.f;
  for (int i = threadIdx.x; i < V; i += blockDim.x)
    if ((!mask || ((mask[i >> 3] >> (i & 7)) & 1)) && l[i] >= t) c += 1.f;
  return block_sum(c, red);
}

__global__ void __launch_bounds__(1024) sample_kernel(SampleArgs a, float top_p_unused) {
  __shared__ float sv[32];
  __shared__ int si[32];
  __shared__ float red[32];
  const int b = blockIdx.x;
  const float* l = a.logits + (size_t)b * a.ldl;
  const uint8_t* mask = a.mask ? a.mask + (size_t)b * ((a.V + 7) / 8) : nullptr;
  const float temp = a.temperature ? a.temperature[b] : 0.f;
  const int topk = a.top_k ? a.top_k[b] : 0;
  // RNG stream keyed by (seed, row, position): unique per step, replay-safe under hipGraph
  const uint32_t step = a.pos ? (uint32_t)a.pos[b] : 0u;

  // 1) plain argmax (also the max for the sampler)
  ArgMax m{-INFINITY, 0x7fffffff};
  for (int i = threadIdx.x; i < a.V; i += blockDim.x) {
    if (mask && !((mask[i >> 3] >> (i & 7)) & 1)) continue;
    m = am_better(m, ArgMax{l[i], i});
  }
  m = block_argmax(m, sv, si);
  int tok = m.i;
  if (temp > 0.f) {
    // 2) top-k threshold by bisection on the logit value
    float thr = -INFINITY;
    if (topk > 0 && topk < a.V) {
      float lo = m.v - 80.f * fmaxf(temp, 1e-3f) - 1e3f, hi = m.v;
      for (int it = 0; it < 24; ++it) {
        const float mid = 0.5f * (lo + hi);
        const float cnt = block_count_ge(l, a.V, mask, mid, red);
        if (cnt >= (float)topk) lo = mid; else hi = mid;
      }
      thr = lo;
    }
    // 3) Gumbel-max over the admissible set: argmax(l/T + G)
    ArgMax g{-INFINITY, 0x7fffffff};
    const float it_ = 1.f / temp;
    for (int i = threadIdx.x; i < a.V; i += blockDim.x) {
      if (mask && !((mask[i >> 3] >> (i & 7)) & 1)) continue;
      if (l[i] < thr) continue;
      const uint64_t seed = a.seed_dev ? *a.seed_dev : a.seed;
      const uint32_t h = mix32(seed * 0x9E3779B97F4A7C15ULL + ((uint64_t)step << 40) + ((uint64_t)b << 32) + i);
      const float u = ((h >> 8) + 0.5f) * (1.f / 16777216.f);
      const float gum = -__logf(-__logf(u));
      g = am_better(g, ArgMax{l[i] * it_ + gum, i});
    }
    g = block_argmax(g, sv, si);
    tok = g.i;
  }
  if (threadIdx.x == 0) {
    if (tok < 0 || tok >= a.V) tok = 0;
    a.tokens[b] = tok;
    if (a.advance && a.pos) {
      const int np = a.pos[b] + 1;
      a.pos[b] = np;
      if (a.seq_len) a.seq_len[b] = np + 1;
      if (a.history) a.history[(size_t)b * a.hist_stride + np] = tok;
    }
  }
}

void launch_sample(const SampleArgs& a, hipStream_t st) {
  hipLaunchKernelGGL(sample_kernel, dim3(a.B), dim3(1024), 0, st, a, 0.f);
}

}  // namespace aios

