// fa_device.h — which GPU an entry point's work belongs to (internal to libfedagg.so).
//
// One aggregator process may drive several GPUs from one host thread (ShardedModelAdapter: FedScale's
// aggregator is a single process, aggregator.py:177-192).  HIP resolves the NULL stream, and any kernel
// launch, against the thread's CURRENT device, so an entry point cannot trust it.  Every launching entry
// point opens a DevScope first:
//   * a non-NULL stream names the device (hipStreamGetDevice); an anchor pointer (the call's output) on
//     another device is rejected with FA_E_ARG before anything is launched;
//   * a NULL stream means the legacy default stream of the device that holds the anchor
//     (hipPointerGetAttributes), which the scope makes current for the call;
//   * the scope restores the caller's current device on exit, and the launch plan's CU-count and occupancy
//     queries read the scope's device (fa_scope_device), not whatever device happens to be current;
//   * every other operand is then checked against the scope's device (DevScope::operand / table, FA_OPERAND):
//     device memory of THAT device, or pinned host memory where the header allows it, and inside its allocation.
// tests/csrc/ compiles this header against a mock HIP runtime (a table of devices and allocations) to check
// the wrong-device and pageable cases on the CPU.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/fedagg.h"

extern "C" __attribute__((visibility("hidden"))) int fa_internal_set_error(int code, const char* msg);
// Operands HIP reports no address range for (round 6).  Host memory: its extent comes from the library's
// own fa_host_register registry (ingress_dma.cpp); *end = one past the registration holding p, 0 if none does.
extern "C" __attribute__((visibility("hidden"))) int fa_internal_registration_end(const void* p, uintptr_t* end);
// Device memory (VMM / expandable segments): no extent can be had; each acceptance is counted process-wide
// (fa_unranged_operands) and, with fa_set_strict_operands(1), refused instead.
extern "C" __attribute__((visibility("hidden"))) void fa_internal_note_unranged(void);
extern "C" __attribute__((visibility("hidden"))) int fa_internal_strict_operands(void);

// device of the entry point running on this thread (-1 outside any scope)
inline thread_local int fa_t_dev = -1;

inline int fa_scope_device() {
  if (fa_t_dev >= 0) return fa_t_dev;
  int d = 0;
  return hipGetDevice(&d) == hipSuccess ? d : -1;
}

// device of a device pointer, or -1 (host, unregistered, or NULL)
inline int fa_pointer_device(const void* p) {
  if (!p) return -1;
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();  // an unknown pointer is not a launch failure: clear it for check_launch
    return -1;
  }
  return at.type == hipMemoryTypeDevice ? at.device : -1;
}

// 1: host memory the GPU dereferences at the same address (pinned and mapped, e.g. hipHostMalloc / torch
// pin_memory); 0: device memory; -1: anything else (pageable, unregistered, managed, or mapped at another
// address) — a kernel must never be handed such a pointer (it would fault the GPU).  NULL: 0.
inline int fa_host_mapped(const void* p) {
  if (!p) return 0;
  hipPointerAttribute_t at;
  if (hipPointerGetAttributes(&at, p) != hipSuccess) {
    (void)hipGetLastError();
    return -1;
  }
  if (at.type == hipMemoryTypeDevice) return 0;
  // the same mapping on both sides (compared with each other, so it holds whether the runtime reports the
  // allocation's base or the queried address)
  if (at.type == hipMemoryTypeHost && at.hostPointer && at.devicePointer == at.hostPointer) return 1;
  return -1;
}

class DevScope {
 public:
  DevScope(const char* what, fa_stream_t stream, const void* anchor) : what_(what), saved_(fa_t_dev) {
    if (hipGetDevice(&prev_) != hipSuccess) {
      (void)hipGetLastError();
      rc_ = err(FA_E_HIP, what, "no current HIP device", -1, -1);
      prev_ = -1;
      return;
    }
    const int pdev = fa_pointer_device(anchor);
    hipStream_t st = (hipStream_t)stream;
    if (st != nullptr && st != hipStreamPerThread) {
      int sdev = -1;
      if (hipStreamGetDevice(st, &sdev) != hipSuccess) {
        (void)hipGetLastError();
        rc_ = err(FA_E_ARG, what, "invalid stream", -1, -1);
        return;
      }
      if (pdev >= 0 && pdev != sdev) {
        rc_ = err(FA_E_ARG, what, "output on device %d but the stream belongs to device %d", pdev, sdev);
        return;
      }
      dev_ = sdev;
    } else {
      dev_ = pdev >= 0 ? pdev : prev_;
    }
    if (dev_ != prev_ && hipSetDevice(dev_) != hipSuccess) {
      (void)hipGetLastError();
      rc_ = err(FA_E_HIP, what, "hipSetDevice(%d) failed", dev_, -1);
      dev_ = prev_;
      return;
    }
    fa_t_dev = dev_;
  }
  ~DevScope() {
    if (prev_ >= 0 && dev_ >= 0 && dev_ != prev_) (void)hipSetDevice(prev_);
    fa_t_dev = saved_;
  }
  DevScope(const DevScope&) = delete;
  DevScope& operator=(const DevScope&) = delete;

  int rc() const { return rc_; }
  int device() const { return dev_; }
  int unranged() const { return unranged_; }

  // Operand check (round 4): every buffer a launch of this call dereferences must be DEVICE memory of the
  // scope's device, or — only where the header allows it (host_ok) — pinned host memory the GPU reads at
  // the same address; and its `bytes` must lie inside the allocation holding it.  Anything else (pageable
  // memory, another GPU's memory, an undersized buffer) is rejected with FA_E_ARG before the call queues
  // anything, where the launch would fault the GPU or read over xGMI.  NULL (or bytes == 0) passes: the entry
  // point checks its required pointers for NULL itself.  Cost: one hipPointerGetAttributes +
  // hipMemGetAddressRange per allocation (~65 ns each on the MI355X host, tools/ptrattr_probe.hip); pointers
  // into an allocation this call already checked (a pointer table's tensors share the caching allocator's
  // segments) cost a range compare.  The checked ranges live for this call only, so a freed and reused
  // address is always re-queried.
  int operand(const char* name, const void* p, uint64_t bytes, bool host_ok = false) {
    if (!p || bytes == 0) return FA_OK;
    const uintptr_t a = (uintptr_t)p;
    for (int i = 0; i < nr_; ++i) {  // most recent first: a table's consecutive tensors share a segment
      const Range& r = rng_[(last_ + nr_ - i) % kRanges];
      if (a >= r.lo && a < r.hi && (r.host == 0 || (host_ok && r.host == 1))) {
        if (bytes > r.hi - a) return operr(name, "%s extends %llu bytes past the end of its allocation", bytes - (r.hi - a));
        return FA_OK;
      }
    }
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess) {
      (void)hipGetLastError();
      return operr(name, "%s is not memory the GPU can read (unknown to HIP)", 0);
    }
    int host = -1;
    if (at.type == hipMemoryTypeDevice) {
      if (at.device != dev_) {
        char m[96];
        snprintf(m, sizeof(m), "%%s is memory of device %d but the call runs on device %d", at.device, dev_);
        return operr(name, m, 0);
      }
      host = 0;
    } else if (at.type == hipMemoryTypeHost && at.hostPointer && at.devicePointer == at.hostPointer) {
      if (!host_ok)
        return operr(name, "%s is pinned host memory; this operand must be device memory (include/fedagg.h)", 0);
      host = 1;
    } else {
      return operr(name, "%s is pageable (or unmapped) host memory: a kernel reading it would fault the GPU", 0);
    }
    void* base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange((hipDeviceptr_t*)&base, &size, (hipDeviceptr_t)p) != hipSuccess || !base) {
      // The type and device checks above have passed, but HIP reports no range (hipHostRegister'd memory, VMM /
      // expandable segments).  Host memory takes its extent from the library's own registrations; host memory
      // nobody registered through the library has no known extent and is refused.  Device memory has none either:
      // it is accepted and counted (fa_unranged_operands), or refused under fa_set_strict_operands(1).
      (void)hipGetLastError();
      if (host == 1) {
        uintptr_t end = 0;
        if (!fa_internal_registration_end(p, &end) || end <= a)
          return operr(name, "%s is pinned host memory of unknown extent (HIP reports no range and it is not a "
                             "fa_host_register registration)", 0);
        if (bytes > end - a) return operr(name, "%s extends %llu bytes past the end of its registration", bytes - (end - a));
        return FA_OK;
      }
      if (fa_internal_strict_operands())
        return operr(name, "%s is device memory HIP reports no range for (VMM / expandable segments); its extent "
                           "cannot be checked and strict operand checks are on (fa_set_strict_operands)", 0);
      ++unranged_;
      fa_internal_note_unranged();
      return FA_OK;
    }
    const Range r{(uintptr_t)base, (uintptr_t)base + size, host};
    if (a < r.lo || a >= r.hi) return operr(name, "%s lies outside the allocation HIP reports for it", 0);
    last_ = (last_ + 1) % kRanges;
    rng_[last_] = r;
    if (nr_ < kRanges) ++nr_;
    if (bytes > r.hi - a) return operr(name, "%s extends %llu bytes past the end of its allocation", bytes - (r.hi - a));
    return FA_OK;
  }
  // the SOURCE of an H2D copy-engine transfer (fa_h2d_pieces): registered or pinned host memory — pageable memory
  // would turn the async copy into a synchronous staged one — and inside its registration
  int host_source(const char* name, const void* p, uint64_t bytes) {
    if (!p || bytes == 0) return FA_OK;
    const uintptr_t a = (uintptr_t)p;
    for (int i = 0; i < nr_; ++i) {
      const Range& r = rng_[(last_ + nr_ - i) % kRanges];
      if (a >= r.lo && a < r.hi && r.host >= 1) {
        if (bytes > r.hi - a) return operr(name, "%s extends %llu bytes past the end of its registration", bytes - (r.hi - a));
        return FA_OK;
      }
    }
    hipPointerAttribute_t at;
    if (hipPointerGetAttributes(&at, p) != hipSuccess || at.type != hipMemoryTypeHost) {
      (void)hipGetLastError();
      return operr(name, "%s is not registered (fa_host_register) or pinned host memory", 0);
    }
    void* base = nullptr;
    size_t size = 0;
    if (hipMemGetAddressRange((hipDeviceptr_t*)&base, &size, (hipDeviceptr_t)p) != hipSuccess || !base) {
      (void)hipGetLastError();
      return operr(name, "%s: no registration range for the pointer", 0);
    }
    const Range r{(uintptr_t)base, (uintptr_t)base + size, 2};
    if (a < r.lo || a >= r.hi) return operr(name, "%s lies outside the registration HIP reports for it", 0);
    last_ = (last_ + 1) % kRanges;
    rng_[last_] = r;
    if (nr_ < kRanges) ++nr_;
    if (bytes > r.hi - a) return operr(name, "%s extends %llu bytes past the end of its registration", bytes - (r.hi - a));
    return FA_OK;
  }
  // a HOST table of n device pointers, tensor i holding numel[i] elements of elem_bytes (numel[i] == 0: skipped)
  int table(const char* name, const void* const* ptrs, const int64_t* numel, int n, int elem_bytes,
            bool host_ok = false) {
    if (!ptrs) return FA_OK;
    char nm[64];
    for (int i = 0; i < n; ++i) {
      if (numel[i] <= 0 || !ptrs[i]) continue;
      const uintptr_t a = (uintptr_t)ptrs[i];
      const Range& r = rng_[last_];  // fast path: the same segment as the previous tensor
      if (nr_ > 0 && a >= r.lo && a < r.hi && (r.host == 0 || (host_ok && r.host == 1)) &&
          (uint64_t)numel[i] * elem_bytes <= r.hi - a)
        continue;
      snprintf(nm, sizeof(nm), "%s[%d]", name, i);
      const int e = operand(nm, ptrs[i], (uint64_t)numel[i] * elem_bytes, host_ok);
      if (e) return e;
    }
    return FA_OK;
  }

 private:
  static int err(int code, const char* what, const char* fmt, int a, int b) {
    char msg[160], buf[256];
    snprintf(msg, sizeof(msg), fmt, a, b);
    snprintf(buf, sizeof(buf), "%s: %s", what, msg);
    return fa_internal_set_error(code, buf);
  }
  int operr(const char* name, const char* fmt, unsigned long long v) {
    char msg[200], buf[300];
    snprintf(msg, sizeof(msg), fmt, name, v);
    snprintf(buf, sizeof(buf), "%s: %s (nothing was launched)", what_, msg);
    return fa_internal_set_error(FA_E_ARG, buf);
  }
  struct Range {
    uintptr_t lo, hi;
    int host;  // 1: pinned host memory mapped at the same address; 2: host memory only known to be registered
  };
  static constexpr int kRanges = 16;
  Range rng_[kRanges] = {};
  int nr_ = 0, last_ = 0;
  int unranged_ = 0;  // operands accepted without an extent check (HIP reported no range)
  const char* what_ = "";
  int prev_ = -1, dev_ = -1, saved_ = -1, rc_ = FA_OK;
};

// open the scope of an entry point; return its error code from the enclosing function on failure
#define FA_DEVICE_SCOPE(what, stream, anchor) \
  DevScope fa_scope_((what), (stream), (anchor)); \
  if (fa_scope_.rc() != FA_OK) return fa_scope_.rc()

// check an operand of the open scope (fa_scope_) — before the entry point launches anything
#define FA_OPERAND(name, p, bytes)                                                          \
  do {                                                                                      \
    const int fa_e_ = fa_scope_.operand((name), (const void*)(p), (uint64_t)(bytes), false); \
    if (fa_e_) return fa_e_;                                                                \
  } while (0)
#define FA_HOST_OK_OPERAND(name, p, bytes)                                                 \
  do {                                                                                     \
    const int fa_e_ = fa_scope_.operand((name), (const void*)(p), (uint64_t)(bytes), true); \
    if (fa_e_) return fa_e_;                                                               \
  } while (0)
#define FA_TABLE(name, ptrs, numel, n, elem_bytes)                                                       \
  do {                                                                                                   \
    const int fa_e_ = fa_scope_.table((name), (const void* const*)(ptrs), (numel), (n), (elem_bytes)); \
    if (fa_e_) return fa_e_;                                                                             \
  } while (0)
