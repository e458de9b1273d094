// Probe: host->device ingest bandwidth by a kernel that reads pinned host memory directly (zero-copy over
// PCIe) versus the runtime's copy engines.  Used to pick the ingress mechanism.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_pull(const f4* __restrict__ src, f4* __restrict__ dst, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    dst[i] = __builtin_nontemporal_load(src + i);
}

extern "C" int h2d_pull(const float* host_src, float* dst, int64_t n, int grid, void* stream) {
  hipLaunchKernelGGL(k_pull, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const f4*)host_src, (f4*)dst, n / 4);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
