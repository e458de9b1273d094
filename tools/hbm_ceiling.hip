// Measured HBM stream-read ceiling on this GPU: a read-only kernel with the same access width
// (16 B/lane, non-temporal) as k_reduce and nothing else to do.  Used to report achieved / ceiling.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float f4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void k_read(const f4* __restrict__ x, int64_t n4, float* out) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + (U - 1) * stride < n4; i += U * stride) {
    f4 t[U];
#pragma unroll
    for (int u = 0; u < U; ++u) t[u] = __builtin_nontemporal_load(x + i + u * stride);
#pragma unroll
    for (int u = 0; u < U; ++u) acc += t[u];
  }
  for (; i < n4; i += stride) acc += __builtin_nontemporal_load(x + i);
  out[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

extern "C" int hbm_read(const float* x, int64_t n, float* out, int grid, int unroll, void* stream) {
  const int64_t n4 = n / 4;
  if (unroll == 16)
    hipLaunchKernelGGL(k_read<16>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const f4*)x, n4, out);
  else
    hipLaunchKernelGGL(k_read<8>, dim3(grid), dim3(256), 0, (hipStream_t)stream, (const f4*)x, n4, out);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
