// ptrattr_probe.hip — host cost of the HIP pointer queries an entry point's operand checks would make
// (hipPointerGetAttributes, hipMemGetAddressRange, hipStreamGetDevice), on device, pinned, pageable and
// interior pointers.  Decides how fa_device.h validates operands (ABI operand checks).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <chrono>

static double ns_per(int n, const std::chrono::steady_clock::time_point& t0) {
  return std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count() / n;
}

int main() {
  const int N = 200000;
  float* d = nullptr;
  float* h = nullptr;
  if (hipMalloc(&d, 64 << 20) != hipSuccess || hipHostMalloc(&h, 64 << 20, 0) != hipSuccess) return 1;
  // many live allocations, as a torch process holds (the lookup is a search over them)
  const int NA = 2000;
  void* many[NA];
  for (int i = 0; i < NA; ++i)
    if (hipMalloc(&many[i], 1 << 16) != hipSuccess) return 1;
  float* pg = (float*)malloc(64 << 20);
  hipStream_t st;
  if (hipStreamCreate(&st) != hipSuccess) return 1;
  const void* ptrs[4] = {d, d + 12345, h, pg};
  const char* names[4] = {"device", "device+interior", "pinned", "pageable"};
  for (int i = 0; i < 4; ++i) {
    hipPointerAttribute_t at;
    int type = -1, dev = -1;
    auto t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < N; ++r) {
      if (hipPointerGetAttributes(&at, ptrs[i]) == hipSuccess) {
        type = at.type;
        dev = at.device;
      } else {
        (void)hipGetLastError();
      }
    }
    const double a = ns_per(N, t0);
    void* base = nullptr;
    size_t sz = 0;
    hipError_t re = hipSuccess;
    t0 = std::chrono::steady_clock::now();
    for (int r = 0; r < N; ++r) {
      re = hipMemGetAddressRange((hipDeviceptr_t*)&base, &sz, (hipDeviceptr_t)ptrs[i]);
      if (re != hipSuccess) (void)hipGetLastError();
    }
    const double b = ns_per(N, t0);
    printf("{\"pointer\": \"%s\", \"type\": %d, \"device\": %d, \"getattr_ns\": %.1f, \"addr_range_ns\": %.1f, "
           "\"range_ok\": %d, \"range_size\": %zu}\n",
           names[i], type, dev, a, b, re == hipSuccess, sz);
  }
  int sdev = -1;
  auto t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < N; ++r) (void)hipStreamGetDevice(st, &sdev);
  printf("{\"stream_get_device_ns\": %.1f}\n", ns_per(N, t0));
  int cur = -1;
  t0 = std::chrono::steady_clock::now();
  for (int r = 0; r < N; ++r) (void)hipGetDevice(&cur);
  printf("{\"get_device_ns\": %.1f}\n", ns_per(N, t0));
  for (int i = 0; i < NA; ++i) (void)hipFree(many[i]);
  (void)hipFree(d);
  (void)hipHostFree(h);
  free(pg);
  return 0;
}
