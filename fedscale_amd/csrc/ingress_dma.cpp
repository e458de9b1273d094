// ingress_dma.cpp — N-GPU ingress straight out of the upload's own bytes (include/fedagg.h, "host ingress").
//
// The one aggregator process receives every upload into a pickled payload (CLIENT_EXECUTE_COMPLETION,
// aggregator.py:919-963; decoded without copies by fedscale_amd/ingress.py, aggregator.py:704).  Round 3 gathered
// each upload into a pinned full-model row and let every GPU copy its slice out of it: three passes over host DRAM
// per byte (payload read, pinned write, DMA read), so the host's memory bandwidth, not the N PCIe links, bounded
// an N-GPU node's ingress.  Here the payload's pages are registered in place (fa_host_register) and
// every GPU's copy engine reads its slice's pieces straight out of them (fa_h2d_pieces): one pass.  Measured on
// one card (tools/register_probe.py, profiles/r04_register_probe.log): registering a 100 MB payload takes 3-35 us.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include <mutex>
#include <vector>

#include "../../include/fedagg.h"
#include "fa_device.h"

namespace {
// The ranges registered through fa_host_register: hipMemGetAddressRange does not report registered host memory,
// so fa_h2d_pieces checks a piece's source extent against this list (pinned hipHostMalloc memory it asks HIP).
std::mutex g_reg_mu;
std::vector<std::pair<uintptr_t, uintptr_t>> g_regs;

bool registered(const void* p, uint64_t n) {
  const uintptr_t a = (uintptr_t)p;
  std::lock_guard<std::mutex> lk(g_reg_mu);
  for (const auto& r : g_regs)
    if (a >= r.first && a < r.second) return n <= r.second - a;
  return false;
}
}  // namespace

// fa_device.h: the extent of registered host memory, which hipMemGetAddressRange does not report
extern "C" __attribute__((visibility("hidden"))) int fa_internal_registration_end(const void* p, uintptr_t* end) {
  const uintptr_t a = (uintptr_t)p;
  std::lock_guard<std::mutex> lk(g_reg_mu);
  for (const auto& r : g_regs)
    if (a >= r.first && a < r.second) {
      *end = r.second;
      return 1;
    }
  *end = 0;
  return 0;
}

extern "C" int fa_host_register(void* p, int64_t nbytes) {
  if (!p || nbytes <= 0) return fa_internal_set_error(FA_E_ARG, "fa_host_register: NULL pointer or empty range");
  const hipError_t e = hipHostRegister(p, (size_t)nbytes, hipHostRegisterDefault);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    char buf[200];
    snprintf(buf, sizeof(buf), "fa_host_register: hipHostRegister(%lld bytes): %s", (long long)nbytes,
             hipGetErrorString(e));
    return fa_internal_set_error(FA_E_HIP, buf);
  }
  std::lock_guard<std::mutex> lk(g_reg_mu);
  g_regs.emplace_back((uintptr_t)p, (uintptr_t)p + (uintptr_t)nbytes);
  return FA_OK;
}

extern "C" int fa_host_unregister(void* p) {
  if (!p) return FA_OK;
  {
    std::lock_guard<std::mutex> lk(g_reg_mu);
    for (size_t i = 0; i < g_regs.size(); ++i)
      if (g_regs[i].first == (uintptr_t)p) {
        g_regs.erase(g_regs.begin() + (long)i);
        break;
      }
  }
  const hipError_t e = hipHostUnregister(p);
  if (e != hipSuccess) {
    (void)hipGetLastError();
    char buf[160];
    snprintf(buf, sizeof(buf), "fa_host_unregister: %s", hipGetErrorString(e));
    return fa_internal_set_error(FA_E_HIP, buf);
  }
  return FA_OK;
}

extern "C" int fa_h2d_pieces(void* const* dst, const void* const* src, const int64_t* nbytes, const int32_t* sidx,
                             int32_t n, void* const* streams, int32_t nstreams) {
  if (n < 0 || nstreams < 1 || !streams || (n > 0 && (!dst || !src || !nbytes || !sidx)))
    return fa_internal_set_error(FA_E_ARG, "fa_h2d_pieces: bad arguments");
  for (int i = 0; i < n; ++i)
    if (sidx[i] < 0 || sidx[i] >= nstreams || nbytes[i] < 0 || (nbytes[i] > 0 && (!dst[i] || !src[i])))
      return fa_internal_set_error(FA_E_ARG, "fa_h2d_pieces: bad piece");
  // pass 1: every piece checked against its stream's device before anything is enqueued
  for (int s = 0; s < nstreams; ++s) {
    if (!streams[s]) return fa_internal_set_error(FA_E_ARG, "fa_h2d_pieces: NULL stream");
    DevScope fa_scope_("fa_h2d_pieces", streams[s], nullptr);
    if (fa_scope_.rc() != FA_OK) return fa_scope_.rc();
    for (int i = 0; i < n; ++i) {
      if (sidx[i] != s || nbytes[i] == 0) continue;
      FA_OPERAND("dst", dst[i], (uint64_t)nbytes[i]);
      if (registered(src[i], (uint64_t)nbytes[i])) continue;  // inside one of our registrations
      const int e = fa_scope_.host_source("src", src[i], (uint64_t)nbytes[i]);  // else: pinned memory
      if (e) return e;
    }
  }
  // pass 2: the copies, in piece order on their streams
  for (int s = 0; s < nstreams; ++s) {
    DevScope scope("fa_h2d_pieces", streams[s], nullptr);
    if (scope.rc() != FA_OK) return scope.rc();
    for (int i = 0; i < n; ++i) {
      if (sidx[i] != s || nbytes[i] == 0) continue;
      const hipError_t e = hipMemcpyAsync(dst[i], src[i], (size_t)nbytes[i], hipMemcpyHostToDevice,
                                          (hipStream_t)streams[s]);
      if (e != hipSuccess) {
        (void)hipGetLastError();
        char buf[160];
        snprintf(buf, sizeof(buf), "fa_h2d_pieces: hipMemcpyAsync of piece %d: %s", i, hipGetErrorString(e));
        return fa_internal_set_error(FA_E_HIP, buf);
      }
    }
  }
  return FA_OK;
}
