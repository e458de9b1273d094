// Mock of the few HIP runtime calls fedscale_amd/csrc/fa_device.h makes, for a CPU-only unit test of the
// C ABI's device scope and operand checks (tests/csrc/devscope_test.cpp, tests/test_abi_operands.py).
// A process-wide table of allocations (base, size, kind, device) and streams (handle -> device) stands in
// for the runtime; the test registers "device" buffers of several GPUs on plain host memory (nothing is
// ever dereferenced by the checks) and counts the pointer queries.
#pragma once

#include <stddef.h>
#include <stdint.h>

#include <map>
#include <vector>

typedef enum hipError_t { hipSuccess = 0, hipErrorInvalidValue = 1, hipErrorInvalidDevice = 101 } hipError_t;
typedef enum hipMemoryType {
  hipMemoryTypeUnregistered = 0,
  hipMemoryTypeHost = 1,
  hipMemoryTypeDevice = 2,
  hipMemoryTypeManaged = 3,
} hipMemoryType;
typedef struct ihipStream_t* hipStream_t;
typedef void* hipDeviceptr_t;
#define hipStreamPerThread ((hipStream_t)2)

typedef struct hipPointerAttribute_t {
  hipMemoryType type;
  int device;
  void* devicePointer;
  void* hostPointer;
  int isManaged;
  unsigned allocationFlags;
} hipPointerAttribute_t;

namespace mockhip {
struct Alloc {
  uintptr_t base;
  size_t size;
  hipMemoryType type;
  int device;
  bool ranged = true;  // false: hipMemGetAddressRange knows nothing of it (hipHostRegister'd memory, VMM segments)
};
inline std::map<uintptr_t, Alloc>& allocs() {
  static std::map<uintptr_t, Alloc> m;
  return m;
}
inline std::map<uintptr_t, int>& streams() {
  static std::map<uintptr_t, int> m;
  return m;
}
inline int& ndev() {
  static int n = 8;
  return n;
}
inline thread_local int current = 0;
inline long queries = 0;  // hipPointerGetAttributes calls
inline void add(const void* base, size_t size, hipMemoryType type, int device, bool ranged = true) {
  allocs()[(uintptr_t)base] = Alloc{(uintptr_t)base, size, type, device, ranged};
}
inline hipStream_t new_stream(int device) {
  static uintptr_t next = 0x1000;
  next += 0x10;
  streams()[next] = device;
  return (hipStream_t)next;
}
inline const Alloc* find(const void* p) {
  auto& m = allocs();
  auto it = m.upper_bound((uintptr_t)p);
  if (it == m.begin()) return nullptr;
  --it;
  const Alloc& a = it->second;
  return ((uintptr_t)p < a.base + a.size) ? &a : nullptr;
}
}  // namespace mockhip

inline hipError_t hipGetLastError() { return hipSuccess; }
inline hipError_t hipGetDevice(int* d) {
  *d = mockhip::current;
  return hipSuccess;
}
inline hipError_t hipSetDevice(int d) {
  if (d < 0 || d >= mockhip::ndev()) return hipErrorInvalidDevice;
  mockhip::current = d;
  return hipSuccess;
}
inline hipError_t hipStreamGetDevice(hipStream_t s, int* d) {
  auto it = mockhip::streams().find((uintptr_t)s);
  if (it == mockhip::streams().end()) return hipErrorInvalidValue;
  *d = it->second;
  return hipSuccess;
}
// as ROCm 7 reports them (tools/ptrattr_probe.hip on the MI355X box): device memory type 2 with its ordinal,
// pinned host memory type 1 mapped at the same address, pageable memory type 0 with device -2, hipSuccess
inline hipError_t hipPointerGetAttributes(hipPointerAttribute_t* at, const void* p) {
  ++mockhip::queries;
  const mockhip::Alloc* a = mockhip::find(p);
  *at = hipPointerAttribute_t{};
  if (!a) {
    at->type = hipMemoryTypeUnregistered;
    at->device = -2;
    return hipSuccess;
  }
  at->type = a->type;
  at->device = a->device;
  at->devicePointer = const_cast<void*>(p);
  at->hostPointer = a->type == hipMemoryTypeHost ? const_cast<void*>(p) : nullptr;
  return hipSuccess;
}
inline hipError_t hipMemGetAddressRange(hipDeviceptr_t* base, size_t* size, hipDeviceptr_t p) {
  const mockhip::Alloc* a = mockhip::find(p);
  if (!a || !a->ranged) return hipErrorInvalidValue;
  *base = (void*)a->base;
  *size = a->size;
  return hipSuccess;
}
