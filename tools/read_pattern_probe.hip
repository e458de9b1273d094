// Round 6: does any read shape beat the round-1 stream-read ceiling (7.23 TB/s, grid-stride nt, 192 x 256, U = 8)?
// Shapes: grid-stride (nt / default / buffer loads with each cache-policy aux value), block-contiguous slices, and
// 512-thread workgroups; the host side (read_pattern_probe.py) sweeps the grid finely around 0.75 WG per CU.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float f4 __attribute__((ext_vector_type(4)));

// 0: grid-stride, nt loads; 1: grid-stride, default loads; 2: block-contiguous slice per workgroup, nt loads
template <int U, int MODE, int NT>
__global__ __launch_bounds__(NT) void k_read(const f4* __restrict__ x, int64_t n4, float* out) {
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  if (MODE == 2) {
    const int64_t per = (n4 + gridDim.x - 1) / gridDim.x;
    const int64_t b0 = (int64_t)blockIdx.x * per;
    const int64_t b1 = b0 + per < n4 ? b0 + per : n4;
    int64_t i = b0 + threadIdx.x;
    for (; i + (U - 1) * NT < b1; i += U * NT) {
      f4 t[U];
#pragma unroll
      for (int u = 0; u < U; ++u) t[u] = __builtin_nontemporal_load(x + i + u * NT);
#pragma unroll
      for (int u = 0; u < U; ++u) acc += t[u];
    }
    for (; i < b1; i += NT) acc += __builtin_nontemporal_load(x + i);
  } else {
    const int64_t stride = (int64_t)gridDim.x * NT;
    int64_t i = (int64_t)blockIdx.x * NT + threadIdx.x;
    for (; i + (U - 1) * stride < n4; i += U * stride) {
      f4 t[U];
#pragma unroll
      for (int u = 0; u < U; ++u) t[u] = MODE == 0 ? __builtin_nontemporal_load(x + i + u * stride) : x[i + u * stride];
#pragma unroll
      for (int u = 0; u < U; ++u) acc += t[u];
    }
    for (; i < n4; i += stride) acc += x[i];
  }
  out[(int64_t)blockIdx.x * NT + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

// grid-stride over one buffer resource per 2 GiB window, raw buffer loads with cache-policy bits AUX
template <int U, int AUX>
__global__ __launch_bounds__(256) void k_read_buf(const float* __restrict__ x, int64_t n4, float* out) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  const int64_t W = (int64_t)1 << 27;  // f4 per window (2 GiB)
  for (int64_t w0 = 0; w0 < n4; w0 += W) {
    const int64_t wn = n4 - w0 < W ? n4 - w0 : W;
    __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(x + w0 * 4), (short)0, (int)(wn * 16 > 0x7fffffff ? 0x7fffffff : wn * 16),
                                          0x00020000);
    int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    for (; i + (U - 1) * stride < wn; i += U * stride) {
      f4 t[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)((i + u * stride) * 16), 0, AUX);
        t[u] = __builtin_bit_cast(f4, v);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) acc += t[u];
    }
    for (; i < wn; i += stride) acc += __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(i * 16), 0, AUX));
  }
  out[(int64_t)blockIdx.x * 256 + threadIdx.x] = acc.x + acc.y + acc.z + acc.w;
}

extern "C" int probe_read(const float* x, int64_t n, float* out, int grid, int variant, void* stream) {
  const int64_t n4 = n / 4;
  hipStream_t s = (hipStream_t)stream;
  const f4* x4 = (const f4*)x;
  switch (variant) {
    case 0: hipLaunchKernelGGL((k_read<8, 0, 256>), dim3(grid), dim3(256), 0, s, x4, n4, out); break;
    case 1: hipLaunchKernelGGL((k_read<8, 1, 256>), dim3(grid), dim3(256), 0, s, x4, n4, out); break;
    case 2: hipLaunchKernelGGL((k_read<8, 2, 256>), dim3(grid), dim3(256), 0, s, x4, n4, out); break;
    case 3: hipLaunchKernelGGL((k_read<8, 0, 512>), dim3(grid), dim3(512), 0, s, x4, n4, out); break;
    case 4: hipLaunchKernelGGL((k_read<4, 0, 256>), dim3(grid), dim3(256), 0, s, x4, n4, out); break;
    case 5: hipLaunchKernelGGL((k_read<12, 0, 256>), dim3(grid), dim3(256), 0, s, x4, n4, out); break;
    case 10: hipLaunchKernelGGL((k_read_buf<8, 0>), dim3(grid), dim3(256), 0, s, x, n4, out); break;
    case 11: hipLaunchKernelGGL((k_read_buf<8, 1>), dim3(grid), dim3(256), 0, s, x, n4, out); break;
    case 12: hipLaunchKernelGGL((k_read_buf<8, 2>), dim3(grid), dim3(256), 0, s, x, n4, out); break;
    case 13: hipLaunchKernelGGL((k_read_buf<8, 3>), dim3(grid), dim3(256), 0, s, x, n4, out); break;
    case 14: hipLaunchKernelGGL((k_read_buf<8, 16>), dim3(grid), dim3(256), 0, s, x, n4, out); break;
    case 15: hipLaunchKernelGGL((k_read_buf<8, 18>), dim3(grid), dim3(256), 0, s, x, n4, out); break;
    default: return -2;
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
