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

}  // namespace aios
