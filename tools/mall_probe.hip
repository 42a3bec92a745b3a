// Infinity Cache (MALL) probe: is a weight matrix that was just read served faster the next time?
// For each size S: time a streaming read of an S-byte buffer from cold caches (after reading 1 GiB of
// another buffer) and right after a previous read of the same buffer (warm), with default-policy and
// non-temporal loads.  Decides whether prefetching the next decode matrices during the latency-bound
// attention step can pay (the GEMV reads are non-temporal).
//   hipcc --offload-arch=gfx950 -O3 -o build/mall_probe tools/mall_probe.hip && build/mall_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e = (x);                                                       \
    if (e != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      std::exit(1);                                                           \
    }                                                                         \
  } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

template <bool NT>
__global__ __launch_bounds__(512) void stream_read(const f4* __restrict__ p, size_t n, float* __restrict__ out) {
  float acc = 0.f;
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  for (; i + 3 * stride < n; i += 4 * stride) {
    f4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = NT ? __builtin_nontemporal_load(p + i + u * stride) : p[i + u * stride];
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += v[u].x + v[u].y + v[u].z + v[u].w;
  }
  for (; i < n; i += stride) {
    const f4 v = NT ? __builtin_nontemporal_load(p + i) : p[i];
    acc += v.x + v.y + v.z + v.w;
  }
  if (acc == 12345.678f) out[blockIdx.x] = acc;  // keeps the loads; never true for the zero-filled buffers
}

static float run(bool nt, const f4* p, size_t bytes, float* out, hipEvent_t a, hipEvent_t b) {
  const size_t n = bytes / 16;
  CK(hipEventRecord(a));
  if (nt) stream_read<true><<<2048, 512>>>(p, n, out);
  else stream_read<false><<<2048, 512>>>(p, n, out);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  return ms;
}

// --sol MB...: cold-cache single launches of the given sizes (flush, default-policy read, flush, nt read;
// 5 reps), for a kernel trace to time: the one-launch streaming-read speed of light at the decode
// matrices' sizes (rocprofv3 --kernel-trace; tools/sol_trace.py reads the trace)
static int sol(int argc, char** argv) {
  const size_t flush_bytes = (size_t)1 << 30;
  f4 *buf, *flush;
  float* out;
  CK(hipMalloc(&buf, (size_t)320 << 20));
  CK(hipMalloc(&flush, flush_bytes));
  CK(hipMalloc(&out, 4096 * sizeof(float)));
  CK(hipMemset(buf, 0, (size_t)320 << 20));
  CK(hipMemset(flush, 0, flush_bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 2; i < argc; ++i) {
    const size_t bytes = ((size_t)(std::atof(argv[i]) * 1048576.0) + 4095) & ~(size_t)4095;
    if (bytes > ((size_t)320 << 20)) return 2;
    for (int rep = 0; rep < 5; ++rep) {
      run(false, flush, flush_bytes, out, a, b);
      run(false, buf, bytes, out, a, b);
      run(false, flush, flush_bytes, out, a, b);
      run(true, buf, bytes, out, a, b);
    }
    std::printf("%s MB: %zu bytes\n", argv[i], bytes);
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc > 1 && std::string(argv[1]) == "--sol") return sol(argc, argv);
  const size_t flush_bytes = (size_t)1 << 30;
  const size_t sizes_mb[] = {8, 16, 32, 64, 96, 128, 192, 320};
  f4 *buf, *flush;
  float* out;
  CK(hipMalloc(&buf, (size_t)320 << 20));
  CK(hipMalloc(&flush, flush_bytes));
  CK(hipMalloc(&out, 4096 * sizeof(float)));
  CK(hipMemset(buf, 0, (size_t)320 << 20));
  CK(hipMemset(flush, 0, flush_bytes));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int w = 0; w < 3; ++w) run(false, flush, flush_bytes, out, a, b);
  std::printf("size_MB  cold_def_TBs  warm_def_TBs  cold_nt_TBs  warm_nt_TBs  warm_nt_after_nt_TBs\n");
  for (size_t mb : sizes_mb) {
    const size_t bytes = mb << 20;
    float best[5] = {1e9f, 1e9f, 1e9f, 1e9f, 1e9f};
    for (int rep = 0; rep < 5; ++rep) {
      float t;
      run(false, flush, flush_bytes, out, a, b);
      t = run(false, buf, bytes, out, a, b);  // cold, default policy
      best[0] = t < best[0] ? t : best[0];
      t = run(false, buf, bytes, out, a, b);  // warm (just read, default policy), default
      best[1] = t < best[1] ? t : best[1];
      run(false, flush, flush_bytes, out, a, b);
      t = run(true, buf, bytes, out, a, b);  // cold, nt
      best[2] = t < best[2] ? t : best[2];
      run(false, flush, flush_bytes, out, a, b);
      run(false, buf, bytes, out, a, b);  // prefetch with default policy
      t = run(true, buf, bytes, out, a, b);  // warm, nt
      best[3] = t < best[3] ? t : best[3];
      t = run(true, buf, bytes, out, a, b);  // after an nt read: did nt allocate?
      best[4] = t < best[4] ? t : best[4];
    }
    std::printf("%7zu", mb);
    for (float t : best) std::printf("  %12.2f", (double)bytes / (t * 1e-3) / 1e12);
    std::printf("\n");
  }
  return 0;
}
