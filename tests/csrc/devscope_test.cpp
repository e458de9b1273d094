// CPU unit test of fedscale_amd/csrc/fa_device.h (the C ABI's device scope and operand checks) against a
// mock HIP runtime with 8 "GPUs" (tests/csrc/mock_hip).  Built and run by tests/test_abi_operands.py:
//   g++ -std=c++17 -I tests/csrc/mock_hip tests/csrc/devscope_test.cpp
// The two entry points below use the scope exactly as fedagg.hip / client_update.hip do (FA_DEVICE_SCOPE,
// then FA_HOST_OK_OPERAND / FA_OPERAND / FA_TABLE before anything would be launched); `launched` counts the
// launches that would have happened.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "../../fedscale_amd/csrc/fa_device.h"

static std::string g_msg;
extern "C" int fa_internal_set_error(int code, const char* msg) {
  g_msg = msg;
  return code;
}

// the library's hooks (fedagg.hip / ingress_dma.cpp): a registry of fa_host_register ranges, the unranged counter and
// the strict switch
static std::vector<std::pair<uintptr_t, uintptr_t>> g_regs;
static int g_unranged = 0, g_strict = 0;
extern "C" int fa_internal_registration_end(const void* p, uintptr_t* end) {
  for (const auto& r : g_regs)
    if ((uintptr_t)p >= r.first && (uintptr_t)p < r.second) {
      *end = r.second;
      return 1;
    }
  *end = 0;
  return 0;
}
extern "C" void fa_internal_note_unranged(void) { ++g_unranged; }
extern "C" int fa_internal_strict_operands(void) { return g_strict; }

static int launched = 0;

// like fa_reduce: x may be pinned host memory, a / out must be device memory of the call's GPU
static int entry_reduce(const float* x, int64_t K, int64_t ld, int64_t P, const float* a, float* out, void* stream) {
  FA_DEVICE_SCOPE("entry_reduce", stream, out);
  FA_HOST_OK_OPERAND("x", x, (uint64_t)((K - 1) * ld + (P + 3) / 4 * 4) * 4);
  FA_OPERAND("a", a, (uint64_t)K * 4);
  FA_OPERAND("out", out, (uint64_t)(P + 3) / 4 * 16);
  if (mockhip::current != fa_scope_.device()) return -100;  // the scope made the call's GPU current
  ++launched;
  return FA_OK;
}

// like fa_prox_update: host tables of device pointers
static int entry_table(float* const* param, const float* const* global, const int64_t* numel, int T, void* stream) {
  const void* first = nullptr;
  for (int i = 0; i < T && !first; ++i)
    if (numel[i] > 0) first = param[i];
  FA_DEVICE_SCOPE("entry_table", stream, first);
  FA_TABLE("param", param, numel, T, 4);
  FA_TABLE("global", global, numel, T, 4);
  ++launched;
  return FA_OK;
}

static int failures = 0;
static void expect(bool ok, const char* name) {
  printf("%s %s%s%s\n", ok ? "ok" : "FAIL", name, ok ? "" : "  -- ", ok ? "" : g_msg.c_str());
  if (!ok) ++failures;
}
static bool has(const char* s) { return g_msg.find(s) != std::string::npos; }

// "device memory" of GPU d: an aligned host block registered in the mock (never dereferenced)
static float* dev_alloc(int d, size_t bytes) {
  void* p = aligned_alloc(256, (bytes + 255) / 256 * 256);
  mockhip::add(p, bytes, hipMemoryTypeDevice, d);
  return (float*)p;
}

int main() {
  const int64_t K = 8, ld = 1024, P = 1000;
  float* x0 = dev_alloc(0, K * ld * 4);
  float* x1 = dev_alloc(1, K * ld * 4);
  float* out0 = dev_alloc(0, ld * 4);
  float* out1 = dev_alloc(1, ld * 4);
  float* a0 = dev_alloc(0, K * 4);
  float* a1 = dev_alloc(1, K * 4);
  float* pinned = (float*)aligned_alloc(256, K * ld * 4);
  mockhip::add(pinned, K * ld * 4, hipMemoryTypeHost, 0);
  std::vector<float> pageable(K * ld);
  hipStream_t s0 = mockhip::new_stream(0), s1 = mockhip::new_stream(1);

  int rc = entry_reduce(x0, K, ld, P, a0, out0, s0);
  expect(rc == FA_OK && launched == 1, "device operands on the stream's device");
  rc = entry_reduce(x1, K, ld, P, a1, out1, s1);
  expect(rc == FA_OK && launched == 2 && mockhip::current == 0, "device 1 from a device-0 thread, restored after");

  // the wrong-device cases: an input (not the anchor) on another GPU
  rc = entry_reduce(x1, K, ld, P, a0, out0, s0);
  expect(rc == FA_E_ARG && launched == 2 && has("x is memory of device 1") && has("runs on device 0") &&
             has("nothing was launched"),
         "x on device 1, call on device 0: FA_E_ARG");
  rc = entry_reduce(x0, K, ld, P, a1, out0, s0);
  expect(rc == FA_E_ARG && launched == 2 && has("a is memory of device 1"), "weights on another device: FA_E_ARG");
  rc = entry_reduce(x0, K, ld, P, a0, out0, s1);
  expect(rc == FA_E_ARG && launched == 2 && has("stream belongs to device 1"), "stream of another device: FA_E_ARG");
  // NULL stream: the device of the output; its inputs must live there too
  mockhip::current = 3;
  rc = entry_reduce(x1, K, ld, P, a1, out1, nullptr);
  expect(rc == FA_OK && launched == 3 && mockhip::current == 3, "NULL stream follows the output's device");
  rc = entry_reduce(x0, K, ld, P, a1, out1, nullptr);
  expect(rc == FA_E_ARG && launched == 3 && has("x is memory of device 0") && mockhip::current == 3,
         "NULL stream, x on another device: FA_E_ARG, current device restored");
  mockhip::current = 0;

  // host memory
  rc = entry_reduce(pageable.data(), K, ld, P, a0, out0, s0);
  expect(rc == FA_E_ARG && launched == 3 && has("pageable"), "pageable x: FA_E_ARG");
  rc = entry_reduce(pinned, K, ld, P, a0, out0, s0);
  expect(rc == FA_OK && launched == 4, "pinned x where the header allows host memory");
  rc = entry_reduce(x0, K, ld, P, (const float*)pinned, out0, s0);
  expect(rc == FA_E_ARG && has("a is pinned host memory"), "pinned weights where device memory is required");

  // extents
  rc = entry_reduce(x0, K + 1, ld, P, a0, out0, s0);
  expect(rc == FA_E_ARG && has("past the end of its allocation"), "x one row longer than its allocation");
  rc = entry_reduce(x0 + 200, K, ld, P, a0, out0, s0);
  expect(rc == FA_E_ARG && has("past the end"), "interior pointer whose rows overrun the allocation");
  rc = entry_reduce(x0 + ld, K - 1, ld, P, a0, out0, s0);
  expect(rc == FA_OK, "interior pointer inside its allocation");

  // memory HIP reports no range for (hipHostRegister'd pinned memory, VMM / expandable segments): the type
  // and device checks still apply, only the extent check is skipped
  float* vmm0 = (float*)aligned_alloc(256, K * ld * 4);
  mockhip::add(vmm0, K * ld * 4, hipMemoryTypeDevice, 0, /*ranged=*/false);
  float* vmm1 = (float*)aligned_alloc(256, K * ld * 4);
  mockhip::add(vmm1, K * ld * 4, hipMemoryTypeDevice, 1, /*ranged=*/false);
  float* reg = (float*)aligned_alloc(256, K * ld * 4);
  mockhip::add(reg, K * ld * 4, hipMemoryTypeHost, 0, /*ranged=*/false);
  const int l0 = launched;
  rc = entry_reduce(vmm0, K, ld, P, a0, out0, s0);
  expect(rc == FA_OK && launched == l0 + 1 && g_unranged == 1,
         "device memory without a HIP range (VMM segment): accepted and counted");
  rc = entry_reduce(vmm1, K, ld, P, a0, out0, s0);
  expect(rc == FA_E_ARG && has("x is memory of device 1"), "rangeless memory of another device: still FA_E_ARG");
  g_strict = 1;
  rc = entry_reduce(vmm0, K, ld, P, a0, out0, s0);
  expect(rc == FA_E_ARG && launched == l0 + 1 && has("strict operand checks"),
         "strict operand checks: rangeless device memory refused");
  g_strict = 0;
  // rangeless host memory: only inside a fa_host_register registration, extent checked against it
  rc = entry_reduce(reg, K, ld, P, a0, out0, s0);
  expect(rc == FA_E_ARG && launched == l0 + 1 && has("unknown extent"),
         "rangeless pinned memory the library did not register: FA_E_ARG");
  g_regs.emplace_back((uintptr_t)reg, (uintptr_t)reg + K * ld * 4);
  rc = entry_reduce(reg, K, ld, P, a0, out0, s0);
  expect(rc == FA_OK && launched == l0 + 2, "registered pinned memory without a range where host memory is allowed");
  rc = entry_reduce(reg, K + 1, ld, P, a0, out0, s0);
  expect(rc == FA_E_ARG && launched == l0 + 2 && has("past the end of its registration"),
         "an undersized registered buffer (one row short): FA_E_ARG");
  g_regs.back().second -= 4096;
  rc = entry_reduce(reg, K, ld, P, a0, out0, s0);
  expect(rc == FA_E_ARG && has("past the end of its registration"), "registration shorter than the rows: FA_E_ARG");
  g_regs.back().second += 4096;
  rc = entry_reduce(x0, K, ld, P, (const float*)reg, out0, s0);
  expect(rc == FA_E_ARG && has("a is pinned host memory"), "rangeless pinned memory where device memory is required");
  expect(g_unranged == 1, "only the rangeless device operand was counted");

  // pointer tables: 96 tensors in 3 segments of device 1 -> 3 queries per table, not 96
  const int T = 96;
  float* seg[3] = {dev_alloc(1, 1 << 20), dev_alloc(1, 1 << 20), dev_alloc(1, 1 << 20)};
  float* gseg = dev_alloc(1, 3 << 20);
  std::vector<float*> param(T);
  std::vector<const float*> glob(T);
  std::vector<int64_t> numel(T, 1000);
  for (int i = 0; i < T; ++i) {
    param[i] = seg[i / 32] + (i % 32) * 1024;
    glob[i] = gseg + i * 1024;
  }
  numel[5] = 0;
  long q0 = mockhip::queries;
  rc = entry_table(param.data(), glob.data(), numel.data(), T, s1);
  expect(rc == FA_OK && launched == l0 + 3, "table of device-1 tensors");
  printf("queries for %d + %d table pointers: %ld\n", T, T, mockhip::queries - q0);
  expect(mockhip::queries - q0 <= 6, "one query per allocation, not per tensor");
  param[40] = dev_alloc(0, 4096);
  rc = entry_table(param.data(), glob.data(), numel.data(), T, s1);
  expect(rc == FA_E_ARG && has("param[40] is memory of device 0"), "one table entry on another device: FA_E_ARG");
  param[40] = (float*)pageable.data();
  rc = entry_table(param.data(), glob.data(), numel.data(), T, s1);
  expect(rc == FA_E_ARG && has("param[40] is pageable"), "one pageable table entry: FA_E_ARG");
  param[40] = seg[1] + 8 * 1024;
  numel[95] = (1 << 20) / 4;  // the last tensor runs past its segment
  rc = entry_table(param.data(), glob.data(), numel.data(), T, s1);
  expect(rc == FA_E_ARG && has("param[95] extends"), "table entry overrunning its allocation");
  numel[95] = 1000;
  param[5] = (float*)pageable.data();  // an empty tensor's pointer is never read
  rc = entry_table(param.data(), glob.data(), numel.data(), T, s1);
  expect(rc == FA_OK, "empty tensors are not checked");

  printf("%s: %d failure(s)\n", failures ? "FAILED" : "PASSED", failures);
  return failures ? 1 : 0;
}
