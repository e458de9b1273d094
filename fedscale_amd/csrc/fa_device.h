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
//     queries read the scope's device (fa_scope_device), not whatever device happens to be current.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/fedagg.h"

extern "C" __attribute__((visibility("hidden"))) int fa_internal_set_error(int code, const char* msg);

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
  DevScope(const char* what, fa_stream_t stream, const void* anchor) : saved_(fa_t_dev) {
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

 private:
  static int err(int code, const char* what, const char* fmt, int a, int b) {
    char msg[160], buf[256];
    snprintf(msg, sizeof(msg), fmt, a, b);
    snprintf(buf, sizeof(buf), "%s: %s", what, msg);
    return fa_internal_set_error(code, buf);
  }
  int prev_ = -1, dev_ = -1, saved_ = -1, rc_ = FA_OK;
};

// open the scope of an entry point; return its error code from the enclosing function on failure
#define FA_DEVICE_SCOPE(what, stream, anchor) \
  DevScope fa_scope_((what), (stream), (anchor)); \
  if (fa_scope_.rc() != FA_OK) return fa_scope_.rc()
