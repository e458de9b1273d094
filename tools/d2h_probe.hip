// Probe: device->host egress bandwidth by a kernel that writes pinned host memory directly (zero-copy over
// PCIe) versus the runtime's copy engine (torch copy_ D2H).  Used to pick the egress mechanism.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void k_push(const f4* __restrict__ src, f4* __restrict__ host_dst, int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
    __builtin_nontemporal_store(src[i], host_dst + i);
}

extern "C" int d2h_push(const float* src, float* host_dst, int64_t n, int grid, void* stream) {
  hipLaunchKernelGGL(k_push, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const f4*)src, (f4*)host_dst, n / 4);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
