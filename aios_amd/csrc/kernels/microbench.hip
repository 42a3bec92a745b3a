// Launch-overhead microbenchmarks (tools/bench_kernels.py): per-kernel cost of a chain of
// dependent launches, eager vs hipGraph replay, for trivial and for one-memory-round-trip kernels.
#include <vector>

#include "../common.h"

namespace aios {

__global__ void empty_kernel(int* p) {
  if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}

// reads one value written by the previous kernel and writes it back (+1): a dependent chain
__global__ void chain_kernel(int* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = p[i] + 1;
}

// returns microseconds per kernel
double bench_launch_chain(int n_kernels, int blocks, int use_graph, int reps) {
  hipStream_t st;
  HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  int* buf;
  const int n = blocks * 256;
  HIP_CHECK(hipMalloc(&buf, n * 4));
  HIP_CHECK(hipMemset(buf, 0, n * 4));
  auto enqueue = [&]() {
    for (int k = 0; k < n_kernels; ++k)
      hipLaunchKernelGGL(chain_kernel, dim3(blocks), dim3(256), 0, st, buf, n);
  };
  hipGraphExec_t ge = nullptr;
  if (use_graph) {
    hipGraph_t g;
    HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    enqueue();
    HIP_CHECK(hipStreamEndCapture(st, &g));
    HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    HIP_CHECK(hipGraphDestroy(g));
  }
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) {
    if (use_graph) HIP_CHECK(hipGraphLaunch(ge, st)); else enqueue();
  }
  HIP_CHECK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) {
    if (use_graph) HIP_CHECK(hipGraphLaunch(ge, st)); else enqueue();
  }
  HIP_CHECK(hipEventRecord(e1, st));
  HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0;
  HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  if (ge) hipGraphExecDestroy(ge);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  hipFree(buf);
  hipStreamDestroy(st);
  return (double)ms * 1e3 / ((double)reps * n_kernels);
}

// ---- streaming-read floor: what a decode projection of `bytes` could cost if the kernel did
// nothing but read its weights once.  Each launch reads a different buffer (rotation > the
// 256 MB Infinity Cache, so the bytes come from HBM as in the decode step), NT buffer loads,
// `U` 16-byte loads in flight per lane, grid = CUs x wg_per_cu workgroups of `threads`.
template <int U>
__global__ void stream_read_kernel(const uint8_t* __restrict__ buf, size_t bytes, uint32_t* out) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)buf, (short)0, 0x7fffffff, 0x00020000);
  const size_t nthreads = (size_t)gridDim.x * blockDim.x;
  const size_t tid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0;
  // chunk = U consecutive 16-B pieces per thread per step, strided so a wave's loads coalesce
  for (size_t base = 0; base < bytes; base += nthreads * 16 * U) {
    uint32_t v[U][4];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const size_t off = base + ((size_t)u * nthreads + tid) * 16;
      const int o = off < bytes ? (int)off : 0;
      const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, o, 0, 2);
      v[u][0] = x[0]; v[u][1] = x[1]; v[u][2] = x[2]; v[u][3] = x[3];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;  // keeps the loads alive, (almost) never stores
}

// Access-pattern variants of the same read (U = 4): MODE 1 = each workgroup streams its own
// contiguous 1/G of the buffer (the decode GEMVs' per-CU row slices), MODE 2 = 2 KB pieces dealt
// round-robin over the workgroups (piece p -> workgroup p % G).
template <int MODE>
__global__ void stream_read_part_kernel(const uint8_t* __restrict__ buf, size_t bytes, uint32_t* out) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)buf, (short)0, 0x7fffffff, 0x00020000);
  const size_t G = gridDim.x, T = blockDim.x;
  uint32_t acc = 0;
  if constexpr (MODE == 1) {
    const size_t per = (bytes / G) & ~(size_t)15;
    const size_t b0 = blockIdx.x * per;
    for (size_t base = 0; base < per; base += T * 64) {
      uint32_t v[4][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const size_t off = base + ((size_t)u * T + threadIdx.x) * 16;
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(b0 + (off < per ? off : 0)), 0, 2);
        v[u][0] = x[0]; v[u][1] = x[1]; v[u][2] = x[2]; v[u][3] = x[3];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
    }
  } else {
    const size_t np = bytes / 2048;
    // each thread: 16 B of a 2 KB piece (128 threads per piece), T / 128 pieces per pass, 4 passes in flight
    const size_t ppw = T / 128;
    for (size_t pb = blockIdx.x * ppw; pb < np; pb += G * ppw * 4) {
      uint32_t v[4][4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        size_t piece = pb + (size_t)u * G * ppw + threadIdx.x / 128;
        if (piece >= np) piece = 0;
        const auto x = __builtin_amdgcn_raw_buffer_load_b128(r, (int)(piece * 2048 + (threadIdx.x % 128) * 16), 0, 2);
        v[u][0] = x[0]; v[u][1] = x[1]; v[u][2] = x[2]; v[u][3] = x[3];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
    }
  }
  if (acc == 0x12345678u) out[blockIdx.x] = acc;
}

double bench_stream_read_part(size_t bytes, int nbuf, int mode, int threads, int reps) {
  hipStream_t st;
  HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  std::vector<uint8_t*> bufs(nbuf);
  for (auto& b : bufs) {
    HIP_CHECK(hipMalloc(&b, bytes));
    HIP_CHECK(hipMemset(b, 1, bytes));
  }
  uint32_t* out;
  HIP_CHECK(hipMalloc(&out, 1 << 20));
  int dev = 0, cus = 256;
  HIP_CHECK(hipGetDevice(&dev));
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const dim3 grid(cus), block(threads);
  hipGraph_t g;
  hipGraphExec_t ge;
  HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  for (int k = 0; k < nbuf; ++k) {
    if (mode == 1) hipLaunchKernelGGL(stream_read_part_kernel<1>, grid, block, 0, st, bufs[k], bytes, out);
    else hipLaunchKernelGGL(stream_read_part_kernel<2>, grid, block, 0, st, bufs[k], bytes, out);
  }
  HIP_CHECK(hipStreamEndCapture(st, &g));
  HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  HIP_CHECK(hipGraphDestroy(g));
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  HIP_CHECK(hipGraphLaunch(ge, st));
  HIP_CHECK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) HIP_CHECK(hipGraphLaunch(ge, st));
  HIP_CHECK(hipEventRecord(e1, st));
  HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0;
  HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  hipGraphExecDestroy(ge);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  for (auto b : bufs) hipFree(b);
  hipFree(out);
  hipStreamDestroy(st);
  return (double)ms * 1e3 / ((double)reps * nbuf);
}

double bench_stream_read(size_t bytes, int nbuf, int wg_per_cu, int u, int threads, int reps) {
  hipStream_t st;
  HIP_CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  std::vector<uint8_t*> bufs(nbuf);
  for (auto& b : bufs) {
    HIP_CHECK(hipMalloc(&b, bytes));
    HIP_CHECK(hipMemset(b, 1, bytes));
  }
  uint32_t* out;
  HIP_CHECK(hipMalloc(&out, 1 << 20));
  int dev = 0, cus = 256;
  HIP_CHECK(hipGetDevice(&dev));
  HIP_CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const dim3 grid(cus * wg_per_cu), block(threads);
  auto enqueue = [&]() {
    for (int k = 0; k < nbuf; ++k) {
      switch (u) {
        case 1: hipLaunchKernelGGL(stream_read_kernel<1>, grid, block, 0, st, bufs[k], bytes, out); break;
        case 2: hipLaunchKernelGGL(stream_read_kernel<2>, grid, block, 0, st, bufs[k], bytes, out); break;
        case 4: hipLaunchKernelGGL(stream_read_kernel<4>, grid, block, 0, st, bufs[k], bytes, out); break;
        default: hipLaunchKernelGGL(stream_read_kernel<8>, grid, block, 0, st, bufs[k], bytes, out); break;
      }
    }
  };
  hipGraph_t g;
  hipGraphExec_t ge;
  HIP_CHECK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
  enqueue();
  HIP_CHECK(hipStreamEndCapture(st, &g));
  HIP_CHECK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  HIP_CHECK(hipGraphDestroy(g));
  hipEvent_t e0, e1;
  HIP_CHECK(hipEventCreate(&e0));
  HIP_CHECK(hipEventCreate(&e1));
  HIP_CHECK(hipGraphLaunch(ge, st));
  HIP_CHECK(hipEventRecord(e0, st));
  for (int r = 0; r < reps; ++r) HIP_CHECK(hipGraphLaunch(ge, st));
  HIP_CHECK(hipEventRecord(e1, st));
  HIP_CHECK(hipEventSynchronize(e1));
  float ms = 0;
  HIP_CHECK(hipEventElapsedTime(&ms, e0, e1));
  hipGraphExecDestroy(ge);
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  for (auto b : bufs) hipFree(b);
  hipFree(out);
  hipStreamDestroy(st);
  return (double)ms * 1e3 / ((double)reps * nbuf);
}

}  // namespace aios
