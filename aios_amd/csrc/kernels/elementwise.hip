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

// rows of up to 256 * 4 * NV floats: the row stays in registers between the sum of squares and the
// scaled store (one HBM read per element; the two-pass kernel above re-read it: 12.5 us for a
// 2048 x 4096 prefill chunk, ~3.8 TB/s)
template <typename OutT, int NV>
__global__ void __launch_bounds__(256) rmsnorm_reg_kernel(const float* __restrict__ x, int ldx, const float* __restrict__ w,
                                                          OutT* __restrict__ y, int ldy, int n, float eps) {
  __shared__ float red[32];
  const float* xr = x + (size_t)blockIdx.x * ldx;
  float4 v[NV];
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = (threadIdx.x + 256 * k) * 4;
    v[k] = i < n ? *(const float4*)(xr + i) : make_float4(0.f, 0.f, 0.f, 0.f);
    s += v[k].x * v[k].x + v[k].y * v[k].y + v[k].z * v[k].z + v[k].w * v[k].w;
  }
  s = block_sum(s, red);
  const float ir = rsqrtf(s / (float)n + eps);
  OutT* yr = y + (size_t)blockIdx.x * ldy;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int i = (threadIdx.x + 256 * k) * 4;
    if (i >= n) break;
    const float4 g = *(const float4*)(w + i);
    const float o0 = v[k].x * ir * g.x, o1 = v[k].y * ir * g.y, o2 = v[k].z * ir * g.z, o3 = v[k].w * ir * g.w;
    if constexpr (sizeof(OutT) == 4) {
      *(float4*)((float*)yr + i) = make_float4(o0, o1, o2, o3);
    } else {
      const uint32_t lo = f32_to_bf16(o0) | ((uint32_t)f32_to_bf16(o1) << 16);
      const uint32_t hi = f32_to_bf16(o2) | ((uint32_t)f32_to_bf16(o3) << 16);
      *(uint2*)((bf16_t*)yr + i) = make_uint2(lo, hi);
    }
  }
}

template <typename OutT>
static void rmsnorm_go(const float* x, int ldx, const float* w, OutT* y, int ldy, int rows, int n, float eps,
                       hipStream_t st) {
  // (the register kernel's vector stores: float4 / 4 x bf16 at y + row * ldy + 4i -- ADVICE r5: y and
  // ldy are checked too, a misaligned output takes the scalar kernel)
  constexpr uintptr_t ymask = sizeof(OutT) == 4 ? 15 : 7;
  const bool al = n % 4 == 0 && ldx % 4 == 0 && ldy % 4 == 0 && ((uintptr_t)x & 15) == 0 && ((uintptr_t)w & 15) == 0 &&
                  ((uintptr_t)y & ymask) == 0;
  if (al && n <= 1024 * 4)
    hipLaunchKernelGGL((rmsnorm_reg_kernel<OutT, 4>), dim3(rows), dim3(256), 0, st, x, ldx, w, y, ldy, n, eps);
  else if (al && n <= 1024 * 8)
    hipLaunchKernelGGL((rmsnorm_reg_kernel<OutT, 8>), dim3(rows), dim3(256), 0, st, x, ldx, w, y, ldy, n, eps);
  else
    hipLaunchKernelGGL(rmsnorm_kernel<OutT>, dim3(rows), dim3(256), 0, st, x, ldx, w, y, ldy, n, eps);
}

void launch_rmsnorm(const float* x, int ldx, const float* w, float* y, int ldy, int rows, int n, float eps,
                    hipStream_t st) {
  rmsnorm_go<float>(x, ldx, w, y, ldy, rows, n, eps, st);
}
void launch_rmsnorm_bf16(const float* x, int ldx, const float* w, bf16_t* y, int ldy, int rows, int n, float eps,
                         hipStream_t st) {
  rmsnorm_go<bf16_t>(x, ldx, w, y, ldy, rows, n, eps, st);
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
// one wave per (token, head): 4 waves per workgroup (round 5: one 64-thread workgroup per (token,
// head) -- 98k of them for a 2048-token Mistral chunk -- ran 30.8 us, dispatch-bound)
__global__ void __launch_bounds__(256) qkv_post_kernel(QkvPostArgs a) {
  const int nh = a.n_heads + 2 * a.n_kv_heads;
  const int item = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (item >= a.T * nh) return;  // (wave-uniform; no barrier below)
  const int t = item / nh, h = item - t * nh, lane = threadIdx.x & 63;
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
    float v0, v1;
    if (ib == ia + 1 && !bias) {  // adjacent pair: one 8-B load
      const float2 u = *(const float2*)(src + ia);
      v0 = u.x; v1 = u.y;
    } else {
      v0 = val(ia); v1 = val(ib);
    }
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
      if (ib == ia + 1) *(float2*)(q + ia) = make_float2(v0, v1);  // (adjacent pairs: 8-B / 4-B stores)
      else { q[ia] = v0; q[ib] = v1; }
    } else {
      bf16_t* cache = part == 1 ? a.k_cache : a.v_cache;
      const size_t base = kv_offset(a.block_table, a.max_ctx / KV_BLOCK, slot, a.n_kv_heads, head, pos, hd);
      kv_store_pair(cache, base + ia, base + ib, v0, v1, a.kv_fp8, part == 1 ? a.kv_inv_k : a.kv_inv_v);
    }
  }
}
// The common case -- non-NeoX RoPE, no QK-norm, no bias (Llama / Mistral / TinyLlama) -- one
// workgroup per token row: pos, slot and the KV block are looked up ONCE per row (the per-(token,
// head) kernel above ran a pos -> block-table -> store chain per wave and was latency bound: 30.8
// us for a 2048-token Mistral chunk, ~3 TB/s of its 90 MB), then every thread walks row pairs
// (2 floats in, RoPE, fp32 pair / bf16 pair out) with 8 in flight.
__global__ void __launch_bounds__(256) qkv_post_row_kernel(QkvPostArgs a) {
  const int t = blockIdx.x;
  const int hd = a.head_dim, half = hd >> 1;
  const int qd = a.n_heads * hd, kvd = a.n_kv_heads * hd;
  const int npair = (qd + 2 * kvd) >> 1;
  const int pos = a.pos[t];
  const int slot = a.slot ? a.slot[t] : 0;
  const size_t kvbase = (((size_t)kv_block(a.block_table, a.max_ctx / KV_BLOCK, slot, pos) * a.n_kv_heads) * KV_BLOCK +
                         (pos % KV_BLOCK)) * hd;  // + head * KV_BLOCK * hd
  const float2* src = (const float2*)(a.qkv + (size_t)t * a.ldqkv);
  const float2* cs = a.rope_cs + (size_t)pos * half;
  constexpr int UNR = 8;
  for (int j0 = threadIdx.x; j0 < npair; j0 += 256 * UNR) {
    float2 v[UNR];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int j = j0 + 256 * u;
      v[u] = j < npair ? src[j] : make_float2(0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      const int j = j0 + 256 * u;
      if (j >= npair) break;
      const int c = 2 * j;
      const int part = c < qd ? 0 : (c < qd + kvd ? 1 : 2);
      const int r = c - (part == 0 ? 0 : (part == 1 ? qd : qd + kvd));
      const int head = r / hd, lr = r - head * hd;
      float v0 = v[u].x, v1 = v[u].y;
      if (part < 2) {
        const float2 tt = cs[lr >> 1];
        const float o0 = v0 * tt.x - v1 * tt.y, o1 = v0 * tt.y + v1 * tt.x;
        v0 = o0;
        v1 = o1;
      }
      if (part == 0) {
        *(float2*)(a.q_out + (size_t)t * qd + c) = make_float2(v0, v1);
      } else {
        bf16_t* cache = part == 1 ? a.k_cache : a.v_cache;
        const size_t i0 = kvbase + (size_t)head * KV_BLOCK * hd + lr;
        kv_store_pair(cache, i0, i0 + 1, v0, v1, a.kv_fp8, part == 1 ? a.kv_inv_k : a.kv_inv_v);
      }
    }
  }
}

void launch_qkv_post(const QkvPostArgs& a, hipStream_t st) {
  if (!a.rope_neox && !a.q_norm && !a.k_norm && !a.bias && a.rope_cs && a.head_dim % 2 == 0) {
    hipLaunchKernelGGL(qkv_post_row_kernel, dim3(a.T), dim3(256), 0, st, a);
    return;
  }
  const int items = a.T * (a.n_heads + 2 * a.n_kv_heads);
  hipLaunchKernelGGL(qkv_post_kernel, dim3((items + 3) / 4), dim3(256), 0, st, a);
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

// ----------------------------------------------------------------------------------------------
// Sampler, two phases in ONE launch: grid (NS = ceil(V / SAMPLE_SLICE), B), 256 threads.
//  A) every workgroup holds a 4096-logit slice in registers (16 per thread): masked argmax, and
//     for temperature > 0 either its Gumbel-max (plain temperature sampling: the max of the
//     slices' maxima is the global one) or its local top-K candidates (8-way bisection on the
//     register-resident values, no re-reads), published with write-through stores + a ticket;
//  B) the row's last arriving workgroup merges: argmax (greedy) / Gumbel winner / global top-K of
//     the candidates (bisection again), nucleus top-p over them (rank-ordered cumulative mass,
//     same rule as the host sampler: keep while the mass before a token is < p), and the
//     Gumbel-max among the survivors; then advances pos / seq_len / history and re-arms.
// Round 1 ran one 1024-thread workgroup per row over the whole vocabulary: 13-15 us per greedy
// step, and 24 bisection passes re-reading the logits when sampling; top-p was ignored.
// ----------------------------------------------------------------------------------------------
#ifndef AIOS_SAMPLE_PROBES
#define AIOS_SAMPLE_PROBES 0
#endif
constexpr int SAMPLE_THREADS = 256;
constexpr int SAMPLE_PER_THREAD = 16;
constexpr int SAMPLE_SLICE = SAMPLE_THREADS * SAMPLE_PER_THREAD;
constexpr int SAMPLE_KCAP = 256;          // candidates per slice (top-k above 256 is clamped)
constexpr int SAMPLE_MAX_CAND = 4096;     // candidates the merge holds (16 per thread)
constexpr int SAMPLE_TOPP_K = 256;        // candidate set of top-p when top-k is off

static inline int sample_slices(int V) { return (V + SAMPLE_SLICE - 1) / SAMPLE_SLICE; }

size_t sample_ws_bytes(int B, int V) {
  const size_t ns = sample_slices(V);
  return (size_t)B * ns * (8 + 4 + (size_t)SAMPLE_KCAP * 8) + 256;
}

struct SampleWs {
  float* part_v; int* part_i; int* cand_n; float* cand_v; int* cand_i;
};
__host__ __device__ inline SampleWs sample_ws(void* base, int B, int NS) {
  SampleWs w;
  char* p = (char*)base;
  w.part_v = (float*)p; p += (size_t)B * NS * 4;
  w.part_i = (int*)p; p += (size_t)B * NS * 4;
  w.cand_n = (int*)p; p += (size_t)B * NS * 4;
  w.cand_v = (float*)p; p += (size_t)B * NS * SAMPLE_KCAP * 4;
  w.cand_i = (int*)p;
  return w;
}

__device__ __forceinline__ float gumbel(uint64_t seed, uint32_t step, int b, int i) {
  const uint32_t h = mix32(seed * 0x9E3779B97F4A7C15ULL + ((uint64_t)step << 40) + ((uint64_t)b << 32) + i);
  const float u = ((h >> 8) + 0.5f) * (1.f / 16777216.f);
  return -__logf(-__logf(u));
}

// threshold thr <= hi such that #{v >= thr} >= K and (within ~span / 2^24) as high as possible; values below
// hi - span are treated as absent (probability < e^-30 relative at the temperatures served).  Round 6: a radix
// select on a 24-bit quantisation of (v - (hi - span)), 8 bits per pass (an LDS histogram of the digit under
// the prefix found so far, a block suffix scan, the digit where the count from the top reaches K) -- 3
// passes of 5 barriers instead of the 8 bisection passes' ~2.5 us each (profiles/sampler_r6.txt).
__device__ __forceinline__ int block_excl_scan(int c, int* s_w, int& total);
template <int N>
__device__ float topk_threshold(const float (&v)[N], float hi, float span, int K, float* /*red*/) {
  __shared__ int s_hist[SAMPLE_THREADS];
  __shared__ int s_w2[16], s_sel[2];
  static_assert(SAMPLE_THREADS == 256, "one histogram bin per thread");
  const int tid = threadIdx.x;
  const float lo = hi - span, scale = 16777216.f / span;
  int u[N];
#pragma unroll
  for (int j = 0; j < N; ++j) u[j] = v[j] >= lo ? min((int)((v[j] - lo) * scale), 16777215) : -1;
  int prefix = 0, above = 0;
#pragma unroll 1
  for (int pass = 0; pass < 3; ++pass) {
    const int shift = 16 - 8 * pass;
    s_hist[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < N; ++j)
      if (u[j] >= 0 && (u[j] >> (shift + 8)) == prefix) atomicAdd(&s_hist[(u[j] >> shift) & 255], 1);
    __syncthreads();
    const int c = s_hist[255 - tid];  // thread t: digit 255 - t (the scan runs from the top digit down)
    int tot;
    const int cum = block_excl_scan(c, s_w2, tot) + c;
    if (tid == 0) s_sel[0] = -1;
    __syncthreads();
    if (cum + above >= K && cum - c + above < K) {
      s_sel[0] = 255 - tid;
      s_sel[1] = above + cum - c;
    }
    __syncthreads();
    const int d = s_sel[0];
    if (d < 0) return lo;  // fewer than K values within the span: all of them
    prefix = (prefix << 8) | d;
    above = s_sel[1];
    __syncthreads();  // (s_sel / s_hist rewritten by the next pass)
  }
  return lo + (float)prefix / scale - span * 1e-7f;
}

// exclusive prefix sum of one int per thread over the block (wave scans + wave offsets); `total` = the sum
__device__ __forceinline__ int block_excl_scan(int c, int* s_w, int& total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  int x = c;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o);
    if (lane >= o) x += y;
  }
  __syncthreads();  // (s_w may still be read from a previous scan)
  if (lane == 63) s_w[wid] = x;
  __syncthreads();
  int off = 0, tot = 0;
  for (int w = 0; w < nw; ++w) {
    off += w < wid ? s_w[w] : 0;
    tot += s_w[w];
  }
  total = tot;
  return off + x - c;
}

__global__ void __launch_bounds__(SAMPLE_THREADS) sample_kernel(SampleArgs a) {
  __shared__ float sv[16];
  __shared__ int si[16];
  __shared__ __attribute__((aligned(16))) float red[7 * 16];
  __shared__ int s_cnt, s_last, s_w[16], s_off[65];
  __shared__ float s_kv[SAMPLE_MAX_CAND];
  __shared__ int s_ki[SAMPLE_MAX_CAND];
  __shared__ __attribute__((aligned(16))) float s_sv[SAMPLE_MAX_CAND + 4];
  __shared__ __attribute__((aligned(16))) float s_se[SAMPLE_MAX_CAND + 4];
  __shared__ __attribute__((aligned(16))) int s_si[SAMPLE_MAX_CAND + 4];
  const int b = blockIdx.y, slice = blockIdx.x, NS = gridDim.x, tid = threadIdx.x;
  const float* l = a.logits + (size_t)b * a.ldl;
  const uint8_t* mask = a.mask ? a.mask + (size_t)b * ((a.V + 7) / 8) : nullptr;
  const float temp = a.temperature ? a.temperature[b] : 0.f;
  const int topk = a.top_k ? a.top_k[b] : 0;
  const float topp = a.top_p ? a.top_p[b] : 1.f;
  const uint32_t step = a.pos ? (uint32_t)a.pos[b] : 0u;  // RNG stream (seed, row, position)
  // (not `c ? *p : a.seed`: a select between pointers made the compiler copy the kernel argument to scratch
  // to load it through a pointer)
  // (relaxed atomic loads: plain ones were sunk into one load through a select of the two pointers)
  uint64_t seed = a.seed;
  if (a.seeds) seed = __hip_atomic_load(a.seeds + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else if (a.seed_dev) seed = __hip_atomic_load(a.seed_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int rkey = a.seeds ? 0 : b;  // per-row seeds: row-independent streams
  const bool filt = temp > 0.f && (topk > 0 || topp < 1.f);
  const int K = topk > 0 ? min(topk, SAMPLE_KCAP) : SAMPLE_TOPP_K;
  SampleWs w = sample_ws(a.ws, a.B, NS);
  // probe stamps (tools/sample_probe.py; compiled into probe builds only, AIOS_BUILD_PROBES=1: the sites'
  // pointer checks pushed the kernel into SGPR spills)
  auto stamp = [&](int k) __attribute__((always_inline)) {
    if (AIOS_SAMPLE_PROBES && a.ts && tid == 0) a.ts[((size_t)b * NS + slice) * 16 + k] = __builtin_amdgcn_s_memrealtime();
  };
  stamp(0);

  // ---- A) this slice in registers
  float v[SAMPLE_PER_THREAD];
  ArgMax m{-INFINITY, 0x7fffffff};
#pragma unroll
  for (int j = 0; j < SAMPLE_PER_THREAD; ++j) {
    const int i = slice * SAMPLE_SLICE + j * SAMPLE_THREADS + tid;
    float x = -INFINITY;
    if (i < a.V && (!mask || ((mask[i >> 3] >> (i & 7)) & 1))) x = l[i];
    v[j] = x;
    m = am_better(m, ArgMax{x, i});
  }
  m = block_argmax(m, sv, si);
  stamp(1);
  ArgMax pub = m;
  if (temp > 0.f && !filt) {  // plain temperature sampling: this slice's Gumbel-max
    ArgMax g{-INFINITY, 0x7fffffff};
    const float it = 1.f / temp;
#pragma unroll
    for (int j = 0; j < SAMPLE_PER_THREAD; ++j) {
      const int i = slice * SAMPLE_SLICE + j * SAMPLE_THREADS + tid;
      if (v[j] > -INFINITY) g = am_better(g, ArgMax{v[j] * it + gumbel(seed, step, rkey, i), i});
    }
    pub = block_argmax(g, sv, si);
  }
  if (filt) {  // local top-K candidates (the global top-K is a subset of their union)
    const float thr = m.v > -INFINITY ? topk_threshold(v, m.v, 30.f * temp + 1.f, K, red) : INFINITY;
    stamp(2);
    // (slots by a block prefix sum in (thread, j) order: the candidate order -- and so every float sum over
    // candidates below -- is the same on every run)
    int c = 0;
#pragma unroll
    for (int j = 0; j < SAMPLE_PER_THREAD; ++j) c += (v[j] >= thr && v[j] > -INFINITY) ? 1 : 0;
    int total;
    int k = block_excl_scan(c, s_w, total);
#pragma unroll
    for (int j = 0; j < SAMPLE_PER_THREAD; ++j) {
      if (v[j] >= thr && v[j] > -INFINITY) {
        if (k < SAMPLE_KCAP) {
          const size_t o = ((size_t)b * NS + slice) * SAMPLE_KCAP + k;
          __hip_atomic_store(w.cand_v + o, v[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(w.cand_i + o, slice * SAMPLE_SLICE + j * SAMPLE_THREADS + tid, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
        ++k;
      }
    }
    if (tid == 0) s_cnt = total;
    __syncthreads();
  }
  if (tid == 0) {
    __hip_atomic_store(w.part_v + (size_t)b * NS + slice, pub.v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(w.part_i + (size_t)b * NS + slice, pub.i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(w.cand_n + (size_t)b * NS + slice, filt ? min(s_cnt, SAMPLE_KCAP) : 0, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const int t = __hip_atomic_fetch_add(a.counters + b, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (t == NS - 1);
  }
  __syncthreads();
  stamp(3);
  if (!s_last) return;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  stamp(4);

  // ---- B) the row's last arriver merges
  auto ldf = [](const float* p) { return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  auto ldi = [](const int* p) { return __hip_atomic_load(const_cast<int*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); };
  ArgMax r{-INFINITY, 0x7fffffff};
  for (int s = tid; s < NS; s += SAMPLE_THREADS)
    r = am_better(r, ArgMax{ldf(w.part_v + (size_t)b * NS + s), ldi(w.part_i + (size_t)b * NS + s)});
  r = block_argmax(r, sv, si);
  stamp(5);
  int tok = r.i;
  if (filt) {
    // gather every slice's candidates (slice-major, in their published order), all loads in flight at
    // once: the counts first (one round trip), then every candidate at its prefix offset (round 6: the
    // slice-serial gather cost a round trip per slice)
    if (tid < NS) s_off[tid + 1] = min(ldi(w.cand_n + (size_t)b * NS + tid), SAMPLE_KCAP);
    __syncthreads();
    if (tid == 0) {
      s_off[0] = 0;
      for (int s = 0; s < NS; ++s) s_off[s + 1] += s_off[s];
    }
    __syncthreads();
    const int nc = min(s_off[NS], SAMPLE_MAX_CAND);
    for (int o = tid; o < nc; o += SAMPLE_THREADS) {
      int s = 0;
      while (s + 1 < NS && s_off[s + 1] <= o) ++s;
      const size_t g = ((size_t)b * NS + s) * SAMPLE_KCAP + (o - s_off[s]);
      s_kv[o] = ldf(w.cand_v + g);
      s_ki[o] = ldi(w.cand_i + g);
    }
    __syncthreads();
    float cv[SAMPLE_MAX_CAND / SAMPLE_THREADS];
#pragma unroll
    for (int j = 0; j < SAMPLE_MAX_CAND / SAMPLE_THREADS; ++j) {
      const int o = j * SAMPLE_THREADS + tid;
      cv[j] = o < nc ? s_kv[o] : -INFINITY;
    }
    stamp(6);
    const float M = r.v;  // the global max is a candidate of its slice
    const float thr = topk_threshold(cv, M, 30.f * temp + 1.f, K, red);
    stamp(7);
    // survivors: top-K (ties kept), then the nucleus over them.  Round 6: the survivors are compacted
    // (block prefix sum, deterministic order) with their weights e = exp((v - M) / T) computed once, and
    // each survivor's rank-ordered mass before it sums over the S survivors only -- the old loop re-ran
    // exp over all nc candidates per survivor (~100 us per sampled token at nc ~ 2k, profiles/)
    const float it = 1.f / temp;
    int c = 0;
#pragma unroll
    for (int j = 0; j < SAMPLE_MAX_CAND / SAMPLE_THREADS; ++j) c += (cv[j] >= thr && cv[j] > -INFINITY) ? 1 : 0;
    int S;
    int k = block_excl_scan(c, s_w, S);
    float zs = 0.f;
#pragma unroll
    for (int j = 0; j < SAMPLE_MAX_CAND / SAMPLE_THREADS; ++j) {
      if (cv[j] >= thr && cv[j] > -INFINITY) {
        const float e = __expf((cv[j] - M) * it);
        zs += e;
        s_sv[k] = cv[j];
        s_si[k] = s_ki[j * SAMPLE_THREADS + tid];
        s_se[k] = e;
        ++k;
      }
    }
    if (tid < 4) {  // pad to a multiple of 4 (the float4 sweep below): never ranked before a survivor
      s_sv[S + tid] = -INFINITY;
      s_si[S + tid] = 0x7fffffff;
      s_se[S + tid] = 0.f;
    }
    const float Z = block_sum(zs, red);  // (its internal barriers also publish the survivor arrays)
    __syncthreads();
    stamp(8);
    if (AIOS_SAMPLE_PROBES && a.ts && tid == 0) {  // (probe: candidate / survivor counts)
      a.ts[((size_t)b * NS + slice) * 16 + 12] = nc;
      a.ts[((size_t)b * NS + slice) * 16 + 13] = S;
    }
    ArgMax g{-INFINITY, 0x7fffffff};
    for (int u = tid; u < S; u += SAMPLE_THREADS) {
      const float vu = s_sv[u];
      const int idx = s_si[u];
      bool keep = true;
      if (topp < 1.f) {  // mass of the survivors ranked before this one (value desc, index asc)
        // (float4 sweeps, four partial sums: the scalar loop waited one LDS round trip per survivor)
        float b0 = 0.f, b1 = 0.f, b2 = 0.f, b3 = 0.f;
        for (int q = 0; q < S; q += 4) {
          const float4 x = *(const float4*)(s_sv + q);
          const int4 xi = *(const int4*)(s_si + q);
          const float4 e = *(const float4*)(s_se + q);
          b0 += (x.x > vu || (x.x == vu && xi.x < idx)) ? e.x : 0.f;
          b1 += (x.y > vu || (x.y == vu && xi.y < idx)) ? e.y : 0.f;
          b2 += (x.z > vu || (x.z == vu && xi.z < idx)) ? e.z : 0.f;
          b3 += (x.w > vu || (x.w == vu && xi.w < idx)) ? e.w : 0.f;
        }
        keep = (b0 + b1) + (b2 + b3) < topp * Z;
      }
      if (keep) g = am_better(g, ArgMax{vu * it + gumbel(seed, step, rkey, idx), idx});
    }
    g = block_argmax(g, sv, si);
    stamp(9);
    if (g.i >= 0 && g.i < a.V) tok = g.i;
  } else if (temp > 0.f) {
    tok = r.i;  // r already holds the Gumbel winners' max
  }
  if (tid == 0) {
    if (tok < 0 || tok >= a.V) tok = 0;
    a.tokens[b] = tok;
    if (a.advance && a.pos) {
      const int np = a.pos[b] + 1;
      a.pos[b] = np;
      if (a.seq_len) a.seq_len[b] = np + 1;
      if (a.history) a.history[(size_t)b * a.hist_stride + np] = tok;
    }
    __hip_atomic_store(a.counters + b, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // re-arm
  }
  stamp(10);
}

void launch_sample(const SampleArgs& a, hipStream_t st) {
  if (!a.ws || !a.counters) throw std::runtime_error("sample: workspace and counters required");
  if (a.ws_bytes < sample_ws_bytes(a.B, a.V)) throw std::runtime_error("sample: workspace too small");
  hipLaunchKernelGGL(sample_kernel, dim3(sample_slices(a.V), a.B), dim3(SAMPLE_THREADS), 0, st, a);
}

}  // namespace aios

