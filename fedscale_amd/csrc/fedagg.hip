// fedagg.hip — MI355X (gfx950, CDNA4) kernels for FedScale's aggregator update-reduction path.
//
// Everything here is memory-bound streaming arithmetic (~1 flop per 4 B for FedAvg), so the design
// target is the HBM3E read roofline, not MFMA:
//   * client updates are client-major [K][ld] fp32; a workgroup owns a contiguous column tile and walks
//     the client axis in ARRIVAL ORDER, so every element's chain is the reference's sequential
//     ((u0 + u1) + u2) + ... in fp32 — bit-identical to the numpy loop of aggregator.py:500-503;
//   * per client, one wave loads V KiB contiguous (16 B/lane dwordx4, non-temporal: every client byte
//     is read exactly once, so it must not evict anything from L2 / Infinity Cache);
//   * U clients are loaded before any of them is added (U*V KiB per wave in flight) to cover HBM latency;
//   * epilogues (÷K, FedYoGi) are fused into the same pass so the global model, m and v make exactly
//     one round trip; no fused multiply-add anywhere (the reference rounds every op).
// See DESIGN.md for the roofline arithmetic per kernel.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <unistd.h>

#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/fedagg.h"
#include "fa_device.h"

// 2: fa_qfed_accumulate gained `chain`, fa_sgd_prox_step's dampening became double, and every launching
//    entry point resolves its device from the stream / output pointer (fa_device.h)
// 3: fa_qfed_accumulate takes the workspace's size, fa_qfed_workspace_bytes the call's (ld, P) (deferred gathers)
// 4: fa_build_id / fa_build_defs, fa_rccl_comm_info
#define FA_ABI_VERSION 5

// The build id (fedscale_amd/buildinfo.py): a hash of the sources, headers and flags this library was compiled
// from, passed in by the build.  _native.load() recomputes it from the tree and refuses a library that differs.
#ifndef FA_BUILD_ID
#define FA_BUILD_ID "unset"  // a build outside buildinfo.py: no loader accepts it
#endif
#ifndef FA_BUILD_DEFS
#define FA_BUILD_DEFS ""
#endif
__attribute__((used)) static const char fa_build_marker[] = "FA_BUILD_ID=" FA_BUILD_ID;

// FA_TUNING 1 (tools/build_*variants.sh) compiles the measured-and-rejected alternatives kept for re-measurement:
// the second q-FedAvg design (k_qfed_accum2), the level cascade of fixed variants, the multi-round capped grid,
// raw-buffer / XCD-remapped / pipelined k_reduce loads and the fixed-variant builds (FA_RED_V).  The default
// library holds only what the drop-in launches.
#ifndef FA_TUNING
#define FA_TUNING 0
#endif

typedef float f4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------------------------------------
// error plumbing
// ------------------------------------------------------------------------------------------------
static thread_local char g_err[512] = "";

__attribute__((format(printf, 2, 3))) static int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}
static int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(FA_E_HIP, "%s: launch failed: %s", what, hipGetErrorString(e));
  return FA_OK;
}
static bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }
// bytes a kernel touches in a client-major [K][ld] buffer of P columns (float4 columns past P included) and in
// a per-column vector (operand extents for DevScope::operand)
static uint64_t rows_bytes(int64_t K, int64_t ld, int64_t P, int elem = 4) {
  return K > 0 ? (uint64_t)((K - 1) * ld + (P + 3) / 4 * 4) * elem : 0;
}
static uint64_t cols_bytes(int64_t P) { return (uint64_t)((P + 3) / 4) * 16; }

// shared with the other translation units of the library (client_update.hip)
extern "C" __attribute__((visibility("hidden"))) int fa_internal_set_error(int code, const char* msg) {
  snprintf(g_err, sizeof(g_err), "%s", msg);
  return code;
}

// operands accepted without an extent check (device memory HIP reports no range for), process-wide; and the switch
// that refuses them instead (fa_device.h, round 6)
static std::atomic<int64_t> g_unranged{0};
static std::atomic<int> g_strict_operands{0};
extern "C" __attribute__((visibility("hidden"))) void fa_internal_note_unranged(void) {
  g_unranged.fetch_add(1, std::memory_order_relaxed);
}
extern "C" __attribute__((visibility("hidden"))) int fa_internal_strict_operands(void) {
  return g_strict_operands.load(std::memory_order_relaxed);
}
extern "C" int64_t fa_unranged_operands(void) { return g_unranged.load(std::memory_order_relaxed); }
extern "C" int fa_set_strict_operands(int32_t on) { return g_strict_operands.exchange(on ? 1 : 0); }

extern "C" int fa_abi_version(void) { return FA_ABI_VERSION; }
extern "C" const char* fa_build_id(void) { return fa_build_marker + sizeof("FA_BUILD_ID=") - 1; }
extern "C" const char* fa_build_defs(void) { return FA_BUILD_DEFS; }
extern "C" int fa_pointer_kind(const void* p) { return fa_host_mapped(p); }
extern "C" const char* fa_last_error_string(void) { return g_err; }

// ------------------------------------------------------------------------------------------------
// small device helpers
// ------------------------------------------------------------------------------------------------
#ifndef FA_RED_NT
#define FA_RED_NT 1
#endif
// client rows are read exactly once: non-temporal loads keep them from evicting L2 / Infinity Cache lines
__device__ __forceinline__ f4 ldnt(const f4* p) {
#if FA_RED_NT
  return __builtin_nontemporal_load(p);
#else
  return *p;
#endif
}

#ifndef FA_RED_BUF
#define FA_RED_BUF 0  // tuning: 1 = k_reduce reads client rows with raw buffer loads of cache policy FA_RED_AUX
#endif
#if !FA_TUNING && (FA_RED_BUF || !FA_RED_NT)
#error "FA_RED_BUF / FA_RED_NT=0 are tuning knobs: build with -DFA_TUNING=1"
#endif
#ifndef FA_RED_AUX
#define FA_RED_AUX 2  // buffer-load cache policy bits (gfx950: 1 sc0, 2 nt, 16 sc1)
#endif
// the same float4 as ldnt(ub + lane + 64 * j): `ub` is the wave-uniform row/tile base, the lane offset a voffset
__device__ __forceinline__ f4 ldrow(const f4* ub, int lane, int j) {
#if FA_RED_BUF
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<f4*>(ub), (short)0, 0x7fffffff,
                                                                     0x00020000);
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(rs, (lane + 64 * j) * 16, 0, FA_RED_AUX));
#else
  return ldnt(ub + lane + 64 * j);
#endif
}

__device__ __forceinline__ float sgnf(float x) {  // torch.sign: -1, 0, +1 (NaN passes through)
  return x > 0.f ? 1.f : (x < 0.f ? -1.f : x);
}
__device__ __forceinline__ double sgnd(double x) { return x > 0.0 ? 1.0 : (x < 0.0 ? -1.0 : x); }

// FedYoGi element step, op order of yogi.py:22-31 + optimizers.py:52-58 (fp32, every op rounded).
__device__ __forceinline__ float yogi_elem(float cur, float last, float& m, float& v, float eta, float tau,
                                           float beta, float omb, float omb2) {
  const float g = cur - last;                       // optimizers.py:53  pb - pa
  const float g2 = g * g;                           // yogi.py:22        gradient**2
  m = beta * m + omb * g;                           // yogi.py:24
  v = v - (omb2 * g2) * sgnf(v - g2);               // yogi.py:26-28
  const float den = __builtin_sqrtf(v) + tau;            // yogi.py:29        sqrt(v) + tau
  const float lr = __frcp_rn(den) * eta;            //                   eta / t == t.reciprocal() * eta
  return last + lr * m;                             // yogi.py:31, optimizers.py:58
}

__device__ __forceinline__ f4 yogi4(f4 cur, f4 last, f4& M, f4& V, float eta, float tau, float beta, float omb,
                                    float omb2) {
  float m[4] = {M.x, M.y, M.z, M.w}, v[4] = {V.x, V.y, V.z, V.w};
  float c[4] = {cur.x, cur.y, cur.z, cur.w}, l[4] = {last.x, last.y, last.z, last.w}, o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = yogi_elem(c[i], l[i], m[i], v[i], eta, tau, beta, omb, omb2);
  M = f4{m[0], m[1], m[2], m[3]};
  V = f4{v[0], v[1], v[2], v[3]};
  return f4{o[0], o[1], o[2], o[3]};
}

// ------------------------------------------------------------------------------------------------
// K-way in-order column reduction (+ fused epilogues)
// ------------------------------------------------------------------------------------------------
enum { EPI_CHAIN = 0, EPI_MEAN = 1, EPI_YOGI = 2 };

struct RedArgs {
  const float* x;
  int64_t ld4;  // row stride in float4
  int64_t P4;   // float4 columns to produce (ceil(P/4))
  int64_t col0; // first float4 column of this launch (a launch covers [col0, min(P4, col0 + ntiles*span)))
  int64_t ntiles;  // tiles of this launch; workgroup b takes tiles b, b + grid, ...
  int sw;          // strips (64 float4 columns) per wave per tile, <= the variant's V
  int K;
  int flags;
  const float* a;
  const float* acc_in;
  float* out;
  float denom;
  const float* last;
  float* m;
  float* v;
  float* mean_out;  // EPI_YOGI: optional copy of chain/denom (the reference's model_weights)
  float eta, tau, beta, omb, omb2;
};

// V: float4 per lane per client (a wave covers V KiB contiguous of one client row)
// U: clients loaded ahead of the adds
#ifndef FA_XCD_REMAP
#define FA_XCD_REMAP 0  // 1: capped-grid workgroups of one XCD take adjacent tiles (tuning experiment)
#endif
#ifndef FA_RED_WAVES
#define FA_RED_WAVES 4
#endif
#ifndef FA_PIPE
#define FA_PIPE 0  // 1: every variant software-pipelines its client groups (tuning builds)
#endif
#if !FA_TUNING && (FA_XCD_REMAP || FA_PIPE || FA_RED_WAVES != 4)
#error "FA_XCD_REMAP / FA_PIPE / FA_RED_WAVES are tuning knobs: build with -DFA_TUNING=1"
#endif
// One tile: the workgroup's FA_RED_WAVES waves each own 64*sw float4 columns (sw <= V strips, a run-time
// width; FULL: sw == V, the compile-time width) and walk all K clients.
template <int V, int U, int EPI, bool W, bool FULL, bool PIPE = false>
__device__ __forceinline__ void reduce_tile(const RedArgs& r, int64_t tile, int lane, int wave) {
  const f4* __restrict__ xp = reinterpret_cast<const f4*>(r.x);
  const int sw = FULL ? V : r.sw;
  const int64_t c0 = r.col0 + (tile * FA_RED_WAVES + wave) * (64LL * sw) + lane;
#if FA_RED_BUF
  const f4* xu = xp + (int64_t)__builtin_amdgcn_readfirstlane((int)(c0 - lane));  // wave-uniform tile base
#else
  const f4* xu = xp + (c0 - lane);
#endif

  bool ok[V];
#pragma unroll
  for (int j = 0; j < V; ++j) ok[j] = (FULL || j < sw) && (c0 + 64 * j) < r.P4;

  f4 s[V];
  int k = 0;
  if (r.flags & FA_ACCUMULATE) {
    const f4* ain = reinterpret_cast<const f4*>(r.acc_in);
#pragma unroll
    for (int j = 0; j < V; ++j) s[j] = ok[j] ? ain[c0 + 64 * j] : f4{0.f, 0.f, 0.f, 0.f};
  } else {
    const float w0 = W ? r.a[0] : 1.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      f4 t = ok[j] ? ldrow(xu, lane, j) : f4{0.f, 0.f, 0.f, 0.f};
      s[j] = W ? t * w0 : t;
    }
    k = 1;
  }

  const f4* row = xu + (int64_t)k * r.ld4;  // client k's row at this wave's tile (lane offsets in ldrow)
  // U clients' loads, then their adds in arrival order
  auto load_group = [&](f4(&t)[U][V], const f4* rw) {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int j = 0; j < V; ++j)
        t[u][j] = ok[j] ? ldrow(rw + u * r.ld4, lane, j) : f4{0.f, 0.f, 0.f, 0.f};
  };
  auto add_group = [&](const f4(&t)[U][V], int k0) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const float w = W ? r.a[k0 + u] : 1.f;
#pragma unroll
      for (int j = 0; j < V; ++j) s[j] = W ? s[j] + w * t[u][j] : s[j] + t[u][j];
    }
  };
  if ((PIPE || FA_PIPE) && k + U <= r.K) {
    // software pipeline: the next group's loads are issued before the current group's adds, so every wave
    // keeps U*V KiB in flight through its add phase too (two register buffers, alternating)
    f4 ta[U][V], tb[U][V];
    load_group(ta, row);
    row += U * r.ld4;
    for (;;) {
      const bool more = k + 2 * U <= r.K;
      if (more) load_group(tb, row), row += U * r.ld4;
      add_group(ta, k);
      k += U;
      if (!more) break;
      const bool more2 = k + 2 * U <= r.K;
      if (more2) load_group(ta, row), row += U * r.ld4;
      add_group(tb, k);
      k += U;
      if (!more2) break;
    }
  }
  for (; k + U <= r.K; k += U) {
    f4 t[U][V];
    load_group(t, row);
    add_group(t, k);
    row += U * r.ld4;
  }
  for (; k < r.K; ++k) {
    const float w = W ? r.a[k] : 1.f;
#pragma unroll
    for (int j = 0; j < V; ++j) {
      f4 t = ok[j] ? ldrow(row, lane, j) : f4{0.f, 0.f, 0.f, 0.f};
      s[j] = W ? s[j] + w * t : s[j] + t;
    }
    row += r.ld4;
  }

#pragma unroll
  for (int j = 0; j < V; ++j) {
    if (!ok[j]) continue;
    const int64_t c = c0 + 64 * j;
    if (EPI == EPI_CHAIN) {
      reinterpret_cast<f4*>(r.out)[c] = s[j];
    } else if (EPI == EPI_MEAN) {
      f4 o;
      o.x = __fdiv_rn(s[j].x, r.denom);
      o.y = __fdiv_rn(s[j].y, r.denom);
      o.z = __fdiv_rn(s[j].z, r.denom);
      o.w = __fdiv_rn(s[j].w, r.denom);
      reinterpret_cast<f4*>(r.out)[c] = o;
      if (r.mean_out) reinterpret_cast<f4*>(r.mean_out)[c] = o;  // fa_reduce_mirror (may be pinned host)
    } else {  // EPI_YOGI
      const f4 L = reinterpret_cast<const f4*>(r.last)[c];
      f4 M, Vv;
      if (r.flags & FA_YOGI_INIT) {
        M = f4{0.f, 0.f, 0.f, 0.f};
        Vv = f4{r.tau, r.tau, r.tau, r.tau};
      } else {
        M = reinterpret_cast<const f4*>(r.m)[c];
        Vv = reinterpret_cast<const f4*>(r.v)[c];
      }
      const f4 cur = f4{__fdiv_rn(s[j].x, r.denom), __fdiv_rn(s[j].y, r.denom), __fdiv_rn(s[j].z, r.denom),
                        __fdiv_rn(s[j].w, r.denom)};
      const f4 o = yogi4(cur, L, M, Vv, r.eta, r.tau, r.beta, r.omb, r.omb2);
      if (r.mean_out) reinterpret_cast<f4*>(r.mean_out)[c] = cur;
      reinterpret_cast<f4*>(r.m)[c] = M;
      reinterpret_cast<f4*>(r.v)[c] = Vv;
      reinterpret_cast<f4*>(r.out)[c] = o;
    }
  }
}

// LOOP = false: workgroup b reduces tile b (grid = tiles).  LOOP = true: a capped grid, workgroup b
// reduces tiles b, b + grid, ... (r.ntiles in this launch): fewer concurrent column streams per round.
// FULL: the tiles are V strips wide (r.sw == V, compile-time masks); otherwise r.sw < V at run time.
template <int V, int U, int EPI, bool W, bool LOOP, bool FULL = true, bool PIPE = false>
__global__ __launch_bounds__(64 * FA_RED_WAVES) void k_reduce(RedArgs r) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  if (LOOP) {
    int64_t b = blockIdx.x;
#if FA_XCD_REMAP
    // workgroups are dispatched round-robin over the 8 XCDs (b -> XCD b % 8): give each XCD a contiguous
    // run of the grid's concurrent tiles instead of every 8th one (bijective for any grid size)
    {
      const int64_t G = gridDim.x, q = G / 8, rem = G % 8, x = b % 8;
      b = x * q + (x < rem ? x : rem) + b / 8;
    }
#endif
    for (int64_t tile = b; tile < r.ntiles; tile += gridDim.x) reduce_tile<V, U, EPI, W, FULL, PIPE>(r, tile, lane, wave);
  } else {
    reduce_tile<V, U, EPI, W, FULL, PIPE>(r, blockIdx.x, lane, wave);
  }
}

// Launch plan.  Each wave owns a column tile of V KiB (V float4 per lane) and walks all K clients, so a
// tile is K*V KiB of reads.  Two measured effects shape it (profiles/r01_tune_grid_sweep.log):
//   * wide tiles keep few DRAM pages open per client row: V=32 reads fastest, V=2 ~6 % slower;
//   * FEWER concurrent column streams read faster: ~0.75 workgroup of V=32 per CU (192 on 256 CUs),
//     each walking several tiles, beats one workgroup per CU by 3-4 % (7.08 vs 6.83 TB/s at 1000 x 25M;
//     6.76 vs 6.56 at 11.19 M; 7.0 vs 6.4 at 6.25 M) — the grid is capped and every workgroup takes the
//     same number of tiles (grid = ceil(tiles / ceil(tiles / cap))).
// So a bucket with at least ~0.85 x cap widest tiles is one capped V=32 launch.  Smaller buckets need
// the parallelism of narrower tiles: the widest variant takes as many FULL waves of workgroups as fit
// (occupancy x CUs, queried at run time), the next narrower variant the same on what is left, the
// narrowest the remainder.  Every column is still reduced by exactly one thread in arrival order, so no
// plan changes a bit of the result.
#if defined(FA_RED_V) && !FA_TUNING
#error "FA_RED_V (a single fixed variant) is a tuning build: add -DFA_TUNING=1"
#endif
#ifdef FA_RED_V  // tuning build: a single fixed variant
#define FA_LEVELS 1
#define FA_L0_V FA_RED_V
#define FA_L0_U FA_RED_U
#else
#define FA_LEVELS 4
#define FA_L0_V 32
#define FA_L0_U 1
#define FA_L1_V 16
#define FA_L1_U 4
#define FA_L2_V 8
#define FA_L2_U 4
#define FA_L3_V 2
#define FA_L3_U 8
#endif
#ifndef FA_GRID_CAP_PCT
#define FA_GRID_CAP_PCT 75  // concurrent V=32 workgroups as a percentage of the CU count
#endif

// CU count and occupancy of the device the running entry point works on (its DevScope), not the thread's
// current device
static int cu_count() {
  static int cache[64];  // per device ordinal (idempotent, benign race)
  const int dev = fa_scope_device();
  if (dev < 0 || dev >= 64) return 0;
  if (cache[dev] > 0) return cache[dev];
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) return 0;
  cache[dev] = cus;
  return cus;
}

// fa_reduce_launches() runs the launch plan with g_plan_count set: every k_reduce launch site then counts
// instead of launching, so the plan has one source of truth.
static thread_local int64_t* g_plan_count = nullptr;
#define FA_RED_LAUNCH(kern, grid, block, st, args)         \
  do {                                                     \
    if (g_plan_count)                                      \
      ++*g_plan_count;                                     \
    else                                                   \
      hipLaunchKernelGGL(kern, grid, block, 0, st, args);  \
  } while (0)

#if FA_TUNING
template <int V, int U, int EPI, bool W>
static int resident_blocks() {
  static int cache[64];  // per device ordinal: occupancy x CU count (idempotent, benign race)
  const int dev = fa_scope_device();
  if (dev < 0 || dev >= 64) return 0;
  if (cache[dev] > 0) return cache[dev];
  int per_cu = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(
          &per_cu, reinterpret_cast<const void*>(&k_reduce<V, U, EPI, W, false>), 64 * FA_RED_WAVES, 0) != hipSuccess)
    return 0;
  cache[dev] = per_cu * cu_count();
  return cache[dev];
}

// launch variant (V, U) over float4 columns [col, col_end); `full_waves_only` keeps only whole waves of
// workgroups (a last partial wave is kept when it would still occupy >= 90 % of the resident slots: a
// narrower variant is ~6 % slower per byte, so handing such a wave down costs more than its idle 10 %)
// and returns the first column it did not cover.  `cap` > 0: at most `cap` workgroups, each reducing an
// equal number of tiles (the LOOP kernel).
template <int V, int U, int EPI, bool W>
static int64_t launch_level(RedArgs r, int64_t col, int64_t col_end, bool full_waves_only, int64_t cap,
                            hipStream_t st) {
  const int64_t span = 64LL * FA_RED_WAVES * V;
  r.sw = V;
  int64_t nblk = (col_end - col + span - 1) / span;
  if (full_waves_only) {
    const int64_t R = resident_blocks<V, U, EPI, W>();
    if (R <= 0) return col;
    const int64_t total = nblk;  // including a partial last tile
    nblk = ((col_end - col) / span) / R * R;
    if (total - nblk >= (R * 9) / 10) nblk = total;  // rest < R + 1 blocks: finish it here
  }
  if (nblk <= 0) return col;
  r.col0 = col;
  r.ntiles = nblk;
  if (cap > 0 && nblk > cap) {
    const int64_t rounds = (nblk + cap - 1) / cap;
    const int64_t grid = (nblk + rounds - 1) / rounds;
    FA_RED_LAUNCH((k_reduce<V, U, EPI, W, true>), dim3((unsigned)grid), dim3(64 * FA_RED_WAVES), st, r);
  } else {
    FA_RED_LAUNCH((k_reduce<V, U, EPI, W, false>), dim3((unsigned)nblk), dim3(64 * FA_RED_WAVES), st, r);
  }
  const int64_t end = col + nblk * span;
  return (full_waves_only && end < col_end) ? end : col_end;
}
#endif  // FA_TUNING (the level cascade)

// Balanced launches (run-time tile width sw strips per wave, sw <= the variant's V; every workgroup gets
// the same number of equally wide tiles, the last tile ragged).  With S strips of 64 float4 columns:
//  * sw1 = ceil(S / (waves x cap)) > 32 (cap = FA_GRID_CAP_PCT of the CUs): R rounds of the capped grid,
//    R = ceil(S / (waves x 32 x cap)), sw = ceil(S / (waves x R x cap)) — the round-1 capped plan at
//    1000 x 25 M exactly; round 1 used full-width tiles only, so a bucket just above one round of them
//    (6.3-8.4 M) ran two rounds on half the cap;
//  * 8 <= sw1 <= 32: one round of sw1-wide tiles, one per workgroup, on ~cap workgroups;
//  * narrower: one round on ~FA_BAL_GRID workgroups per 256 CUs, unless the tiles would be narrower than
//    FA_BAL_MIN_SW or the round short (K x sw < FA_BAL_MIN_WORK): then the level cascade below (more,
//    narrower workgroups) reads faster;
//  * rounds of fewer than FA_BAL_SHORT_K clients take one round over every CU whenever sw <= 32.
// One-round launches use the narrowest variant that holds sw (V x U = 32 KiB of loads in flight per
// wave).  Measured: profiles/r02_tune_small_p.log (1000 x 3.125 M, config 4's bucket over 8 GPUs and the
// north star's per-GPU work at 8 GPUs: 6.2 -> 7.0 TB/s).
#ifndef FA_BAL_GRID
#define FA_BAL_GRID 224
#endif
#ifndef FA_BAL_MIN_SW
#define FA_BAL_MIN_SW 5
#endif
#ifndef FA_BAL_MIN_WORK
#define FA_BAL_MIN_WORK 1000  // K x sw: KiB one wave reads over the round
#endif
#ifndef FA_BAL_SHORT_K
#define FA_BAL_SHORT_K 200  // rounds of fewer clients: one round over every CU when the tiles fit
#endif
#ifndef FA_CAP_SW_MAX
#define FA_CAP_SW_MAX 32  // widest tile (strips per wave) of the multi-round capped plan (tuning knob, 8..32)
#endif
static_assert(FA_CAP_SW_MAX >= 8 && FA_CAP_SW_MAX <= 32, "FA_CAP_SW_MAX: 8..32");
#ifndef FA_WINDOWS
#define FA_WINDOWS 1
#endif
template <int V, int U, int EPI, bool W>
static void launch_balanced(RedArgs r, int64_t sw, int64_t rounds, hipStream_t st) {
  const int64_t S = (r.P4 + 63) / 64;
  r.col0 = 0;
  r.sw = (int)sw;
  r.ntiles = (S + (int64_t)FA_RED_WAVES * sw - 1) / ((int64_t)FA_RED_WAVES * sw);
  const int64_t grid = (r.ntiles + rounds - 1) / rounds;
  const dim3 blk(64 * FA_RED_WAVES);
#if FA_TUNING || !FA_WINDOWS || FA_CAP_SW_MAX != 32
  if (grid < r.ntiles) {  // several rounds of the capped grid in one launch (the window plan replaces it)
    if (sw == V)
      FA_RED_LAUNCH((k_reduce<V, U, EPI, W, true, true>), dim3((unsigned)grid), blk, st, r);
    else
      FA_RED_LAUNCH((k_reduce<V, U, EPI, W, true, false>), dim3((unsigned)grid), blk, st, r);
    return;
  }
#endif
  (void)grid;
  if (sw == V) {
    FA_RED_LAUNCH((k_reduce<V, U, EPI, W, false, true>), dim3((unsigned)r.ntiles), blk, st, r);
  } else {
    FA_RED_LAUNCH((k_reduce<V, U, EPI, W, false, false>), dim3((unsigned)r.ntiles), blk, st, r);
  }
}

// One round of tiles over the column window [s0, s0 + ns) strips (64 float4 columns each) on about `cap`
// workgroups: the kernel's col0 / P4 bound the window, outputs stay indexed by absolute column.
#ifndef FA_WIN_FULL_MIN
#define FA_WIN_FULL_MIN 33  // tuning knob: windows whose tiles would be >= this many strips wide take full 32-wide
                            // tiles on fewer workgroups instead (33: off)
#endif
template <int EPI, bool W>
static void launch_window(RedArgs r, int64_t s0, int64_t ns, int64_t cap, hipStream_t st) {
  int64_t sw = (ns + (int64_t)FA_RED_WAVES * cap - 1) / ((int64_t)FA_RED_WAVES * cap);
  if (sw >= FA_WIN_FULL_MIN && sw < 32) sw = 32;
  r.col0 = s0 * 64;
  r.P4 = (s0 + ns) * 64 < r.P4 ? (s0 + ns) * 64 : r.P4;
  r.sw = (int)sw;
  r.ntiles = (ns + (int64_t)FA_RED_WAVES * sw - 1) / ((int64_t)FA_RED_WAVES * sw);
  const dim3 grid((unsigned)r.ntiles), blk(64 * FA_RED_WAVES);
  if (sw == 32)
    FA_RED_LAUNCH((k_reduce<32, 1, EPI, W, false, true>), grid, blk, st, r);
  else if (sw > 16)
    FA_RED_LAUNCH((k_reduce<32, 1, EPI, W, false, false>), grid, blk, st, r);
  else if (sw == 16)
    FA_RED_LAUNCH((k_reduce<16, 2, EPI, W, false, true>), grid, blk, st, r);
  else
    FA_RED_LAUNCH((k_reduce<16, 2, EPI, W, false, false>), grid, blk, st, r);
}

// FA_WINDOWS 1: a plan of R > 1 rounds of the capped grid runs as R launches over equal column windows,
// one round each.  Over several rounds of ~1000 clients the workgroups drift apart; a launch boundary
// re-aligns them.  Measured interleaved on three boxes (tools/window_probe.py, profiles/r02_window_probe.log):
// 1000 x 25 M 7.07-7.09 -> 7.15-7.16 TB/s, 1000 x 12.5 M +0.6 %; the bits are the same (columns are
// independent).
// Short, narrow rounds (config 2: 100 x 1 M, 400 MB per round): one launch, one workgroup per tile of 4
// waves x 4 float4 per lane, the client groups software-pipelined (two register buffers of 4 clients: the
// next group's 16 KiB per wave is in flight while the current one is added, so 32 KiB per wave is
// outstanding through the add phase).  Round 2 ran a cascade of up to 4 launches of narrower variants here.
// Measured against a bare stream read of the same 400 MB in the same process (tools/c2_probe.py,
// profiles/r03_c2_probe.log): the cascade 97.4 %, this launch 98.3 %.
#ifndef FA_SHORT_PIPE
#define FA_SHORT_PIPE 1
#endif
template <int EPI, bool W>
static void launch_short(RedArgs r, hipStream_t st) {
  const int64_t span = 64LL * FA_RED_WAVES * 4;
  r.col0 = 0;
  r.sw = 4;
  r.ntiles = (r.P4 + span - 1) / span;
  FA_RED_LAUNCH((k_reduce<4, 4, EPI, W, false, true, true>), dim3((unsigned)r.ntiles), dim3(64 * FA_RED_WAVES), st, r);
}
template <int EPI, bool W>
static int launch_plan(const RedArgs& r, hipStream_t st) {
#if FA_LEVELS == 1  // tuning build: one fixed variant (FA_RED_V / FA_RED_U), optionally on a fixed grid cap
#if defined(FA_RED_GRID) && FA_RED_GRID > 0
  launch_level<FA_L0_V, FA_L0_U, EPI, W>(r, 0, r.P4, false, FA_RED_GRID, st);
#else
  launch_level<FA_L0_V, FA_L0_U, EPI, W>(r, 0, r.P4, false, 0, st);
#endif
  return FA_OK;
#else
  const int64_t cus = cu_count();
  if (cus <= 0) return fail(FA_E_HIP, "k_reduce launch plan: no CU count for device %d", fa_scope_device());
  const int64_t cap = cus * FA_GRID_CAP_PCT / 100;
#if FA_BAL_GRID > 0
  {
    const int64_t S = (r.P4 + 63) / 64;
    const int64_t g1 = r.K < FA_BAL_SHORT_K ? cus : cap;  // short rounds: one round, all CUs
    const int64_t sw1 = (S + (int64_t)FA_RED_WAVES * g1 - 1) / ((int64_t)FA_RED_WAVES * g1);
    if (sw1 > 32) {  // R rounds of the capped grid, tiles at most FA_CAP_SW_MAX strips wide
      const int64_t per_round = (int64_t)FA_RED_WAVES * FA_CAP_SW_MAX * cap;
      const int64_t R = (S + per_round - 1) / per_round;
      if (FA_WINDOWS && FA_CAP_SW_MAX == 32) {  // ... as R launches over column windows, one round each
        const int64_t Sw = (S + R - 1) / R;
        for (int64_t s0 = 0; s0 < S; s0 += Sw) launch_window<EPI, W>(r, s0, S - s0 < Sw ? S - s0 : Sw, cap, st);
        return FA_OK;
      }
      const int64_t sw = (S + (int64_t)FA_RED_WAVES * R * cap - 1) / ((int64_t)FA_RED_WAVES * R * cap);
      if (sw > 16)
        launch_balanced<32, 1, EPI, W>(r, sw, R, st);
      else
        launch_balanced<16, 2, EPI, W>(r, sw, R, st);
      return FA_OK;
    }
    if (sw1 >= 8) {  // one round of wide tiles on (about) the capped grid
      if (sw1 > 16)
        launch_balanced<32, 1, EPI, W>(r, sw1, 1, st);
      else
        launch_balanced<16, 2, EPI, W>(r, sw1, 1, st);
      return FA_OK;
    }
    // narrow tiles: one round on more workgroups, unless the round is short
    const int64_t gb = cus * FA_BAL_GRID / 256;
    const int64_t swb = (S + (int64_t)FA_RED_WAVES * gb - 1) / ((int64_t)FA_RED_WAVES * gb);
    if (swb >= FA_BAL_MIN_SW && (int64_t)r.K * swb >= FA_BAL_MIN_WORK) {
      if (swb > 8)
        launch_balanced<16, 2, EPI, W>(r, swb, 1, st);
      else
        launch_balanced<8, 4, EPI, W>(r, swb, 1, st);
      return FA_OK;
    }
  }
#endif
#if FA_SHORT_PIPE
  launch_short<EPI, W>(r, st);  // narrow, short round (K x sw < FA_BAL_MIN_WORK, e.g. config 2's 100 x 1 M)
  return FA_OK;
#elif FA_TUNING
  // rounds 1-2's level cascade (tuning builds with FA_SHORT_PIPE=0 or FA_BAL_GRID=0)
  const int64_t span0 = 64LL * FA_RED_WAVES * FA_L0_V;
  const int64_t tiles0 = (r.P4 + span0 - 1) / span0;
  if (tiles0 * 20 >= cap * 17) {  // enough widest tiles to keep ~cap workgroups busy
    launch_level<FA_L0_V, FA_L0_U, EPI, W>(r, 0, r.P4, false, cap, st);
    return FA_OK;
  }
  int64_t col = launch_level<FA_L0_V, FA_L0_U, EPI, W>(r, 0, r.P4, true, 0, st);
  if (col < r.P4) col = launch_level<FA_L1_V, FA_L1_U, EPI, W>(r, col, r.P4, true, 0, st);
  if (col < r.P4) col = launch_level<FA_L2_V, FA_L2_U, EPI, W>(r, col, r.P4, true, 0, st);
  if (col < r.P4) launch_level<FA_L3_V, FA_L3_U, EPI, W>(r, col, r.P4, false, 0, st);
  return FA_OK;
#else
#error "FA_SHORT_PIPE=0 / FA_BAL_GRID=0 fall back to the level cascade: a tuning build (-DFA_TUNING=1)"
#endif
#endif
}

template <int EPI>
static int launch_reduce(const RedArgs& r, hipStream_t st, const char* what) {
  if (r.P4 <= 0) return FA_OK;
  if (r.P4 / (64 * FA_RED_WAVES) > 0x7fffffffLL) return fail(FA_E_RANGE, "%s: P too large", what);
  const int e = r.a ? launch_plan<EPI, true>(r, st) : launch_plan<EPI, false>(r, st);
  if (e) return e;
  return check_launch(what);
}

// Kernel launches one fa_reduce / fa_reduce_yogi call makes at (K, P): the plan run in counting mode.
extern "C" int64_t fa_reduce_launches(int32_t K, int64_t P, int32_t weighted) {
  if (K <= 0 || P <= 0) return 0;
  RedArgs r{};
  r.P4 = (P + 3) / 4;
  r.K = K;
  int64_t n = 0;
  g_plan_count = &n;
  const int e = weighted ? launch_plan<EPI_MEAN, true>(r, nullptr) : launch_plan<EPI_MEAN, false>(r, nullptr);
  g_plan_count = nullptr;
  return e ? e : n;
}

static int check_reduce_args(const char* what, const float* x, int64_t ld, int32_t K, int64_t P,
                             const float* acc_in, const float* out, int32_t flags) {
  if (K < 0 || P < 0 || ld < P) return fail(FA_E_ARG, "%s: bad sizes (ld < P or negative)", what);
  if (ld % 4 != 0) return fail(FA_E_ARG, "%s: ld=%lld must be a multiple of 4", what, (long long)ld);
  if ((flags & FA_ACCUMULATE) && !acc_in) return fail(FA_E_ARG, "%s: FA_ACCUMULATE without acc_in", what);
  if (K == 0 && !(flags & FA_ACCUMULATE)) return fail(FA_E_ARG, "%s: K == 0 with nothing to accumulate", what);
  if (K > 0 && !x) return fail(FA_E_ARG, "%s: x is NULL", what);
  if (!out) return fail(FA_E_ARG, "%s: out is NULL", what);
  if (!aligned16(x) || !aligned16(out) || !aligned16(acc_in))
    return fail(FA_E_ARG, "%s: device pointers must be 16-byte aligned", what);
  return FA_OK;
}

extern "C" int fa_reduce(const float* x, int64_t ld, int32_t K, int64_t P, const float* a, const float* acc_in,
                         float* out, float denom, int32_t flags, fa_stream_t stream) {
  int e = check_reduce_args("fa_reduce", x, ld, K, P, acc_in, out, flags);
  if (e) return e;
  if (P == 0) return FA_OK;
  RedArgs r{};
  r.x = x; r.ld4 = ld / 4; r.P4 = (P + 3) / 4; r.K = K; r.flags = flags; r.a = a; r.acc_in = acc_in;
  r.out = out; r.denom = denom;
  FA_DEVICE_SCOPE("fa_reduce", stream, out);
  FA_HOST_OK_OPERAND("x", x, rows_bytes(K, ld, P));  // device, or pinned host (the zero-copy round)
  FA_OPERAND("a", a, (uint64_t)K * 4);
  FA_OPERAND("acc_in", (flags & FA_ACCUMULATE) ? acc_in : nullptr, cols_bytes(P));
  FA_OPERAND("out", out, cols_bytes(P));
  hipStream_t st = (hipStream_t)stream;
  if (flags & FA_FINALIZE) return launch_reduce<EPI_MEAN>(r, st, "fa_reduce");
  return launch_reduce<EPI_CHAIN>(r, st, "fa_reduce");
}

// The finishing reduce of every part of a model sharded over the GPUs of this process, in one call (round 4): the
// in-process N-GPU round's host cost per part drops from a Python call chain to a DevScope and the plan's launches.
// Every part is validated (sizes, stream, operands) before any part launches.
extern "C" int fa_reduce_parts(int32_t n, const float* const* x, const int64_t* ld, const int32_t* K,
                               const int64_t* P, const float* const* acc_in, float* const* out, float denom,
                               const int32_t* flags, void* const* streams) {
  if (n < 1 || !x || !ld || !K || !P || !acc_in || !out || !flags || !streams)
    return fail(FA_E_ARG, "fa_reduce_parts: NULL table or n < 1");
  char what[48];
  for (int i = 0; i < n; ++i) {
    snprintf(what, sizeof(what), "fa_reduce_parts[%d]", i);
    int e = check_reduce_args(what, x[i], ld[i], K[i], P[i], acc_in[i], out[i], flags[i]);
    if (e) return e;
    if (!streams[i]) return fail(FA_E_ARG, "%s: NULL stream (one stream per part's GPU)", what);
    if (P[i] == 0) continue;
    FA_DEVICE_SCOPE(what, streams[i], out[i]);
    char nx[24], na[24], no[24];
    snprintf(nx, sizeof(nx), "x[%d]", i);
    snprintf(na, sizeof(na), "acc_in[%d]", i);
    snprintf(no, sizeof(no), "out[%d]", i);
    FA_OPERAND(nx, x[i], rows_bytes(K[i], ld[i], P[i]));
    FA_OPERAND(na, (flags[i] & FA_ACCUMULATE) ? acc_in[i] : nullptr, cols_bytes(P[i]));
    FA_OPERAND(no, out[i], cols_bytes(P[i]));
  }
  for (int i = 0; i < n; ++i) {
    if (P[i] == 0) continue;
    snprintf(what, sizeof(what), "fa_reduce_parts[%d]", i);
    RedArgs r{};
    r.x = x[i]; r.ld4 = ld[i] / 4; r.P4 = (P[i] + 3) / 4; r.K = K[i]; r.flags = flags[i]; r.acc_in = acc_in[i];
    r.out = out[i]; r.denom = denom;
    FA_DEVICE_SCOPE(what, streams[i], out[i]);
    const int e = (flags[i] & FA_FINALIZE) ? launch_reduce<EPI_MEAN>(r, (hipStream_t)streams[i], what)
                                           : launch_reduce<EPI_CHAIN>(r, (hipStream_t)streams[i], what);
    if (e) return e;
  }
  return FA_OK;
}

extern "C" int fa_reduce_mirror(const float* x, int64_t ld, int32_t K, int64_t P, const float* a,
                                const float* acc_in, float* out, float* mirror, float denom, int32_t flags,
                                fa_stream_t stream) {
  int e = check_reduce_args("fa_reduce_mirror", x, ld, K, P, acc_in, out, flags);
  if (e) return e;
  if (!(flags & FA_FINALIZE)) return fail(FA_E_ARG, "fa_reduce_mirror: needs FA_FINALIZE");
  if (!mirror || !aligned16(mirror)) return fail(FA_E_ARG, "fa_reduce_mirror: mirror NULL or not 16-byte aligned");
  if (P == 0) return FA_OK;
  RedArgs r{};
  r.x = x; r.ld4 = ld / 4; r.P4 = (P + 3) / 4; r.K = K; r.flags = flags; r.a = a; r.acc_in = acc_in;
  r.out = out; r.denom = denom; r.mean_out = mirror;
  FA_DEVICE_SCOPE("fa_reduce_mirror", stream, out);
  FA_HOST_OK_OPERAND("x", x, rows_bytes(K, ld, P));
  FA_HOST_OK_OPERAND("mirror", mirror, cols_bytes(P));
  FA_OPERAND("a", a, (uint64_t)K * 4);
  FA_OPERAND("acc_in", (flags & FA_ACCUMULATE) ? acc_in : nullptr, cols_bytes(P));
  FA_OPERAND("out", out, cols_bytes(P));
  return launch_reduce<EPI_MEAN>(r, (hipStream_t)stream, "fa_reduce_mirror");
}

extern "C" int fa_reduce_yogi(const float* x, int64_t ld, int32_t K, int64_t P, const float* a,
                              const float* acc_in, float denom, const float* last, float* m, float* v,
                              float* out, float* mean_out, float eta, float tau, float beta, float omb,
                              float omb2, int32_t flags, fa_stream_t stream) {
  int e = check_reduce_args("fa_reduce_yogi", x, ld, K, P, acc_in, out, flags);
  if (e) return e;
  if (!last || !m || !v) return fail(FA_E_ARG, "fa_reduce_yogi: last/m/v NULL");
  if (!aligned16(last) || !aligned16(m) || !aligned16(v) || !aligned16(mean_out))
    return fail(FA_E_ARG, "fa_reduce_yogi: last/m/v must be 16-byte aligned");
  if (P == 0) return FA_OK;
  FA_DEVICE_SCOPE("fa_reduce_yogi", stream, out);
  FA_OPERAND("x", x, rows_bytes(K, ld, P));
  FA_OPERAND("a", a, (uint64_t)K * 4);
  FA_OPERAND("acc_in", (flags & FA_ACCUMULATE) ? acc_in : nullptr, cols_bytes(P));
  FA_OPERAND("last", last, cols_bytes(P));
  FA_OPERAND("m", m, cols_bytes(P));
  FA_OPERAND("v", v, cols_bytes(P));
  FA_OPERAND("out", out, cols_bytes(P));
  FA_OPERAND("mean_out", mean_out, cols_bytes(P));
  RedArgs r{};
  r.x = x; r.ld4 = ld / 4; r.P4 = (P + 3) / 4; r.K = K; r.flags = flags; r.a = a; r.acc_in = acc_in;
  r.out = out; r.denom = denom; r.last = last; r.m = m; r.v = v; r.mean_out = mean_out;
  r.eta = eta; r.tau = tau; r.beta = beta; r.omb = omb; r.omb2 = omb2;
  return launch_reduce<EPI_YOGI>(r, (hipStream_t)stream, "fa_reduce_yogi");
}

// ------------------------------------------------------------------------------------------------
// FedYoGi step alone (elementwise, grid-stride float4)
// ------------------------------------------------------------------------------------------------
// k_yogi_step touches every byte once per round.  NT: non-temporal loads and stores.  Measured back to back on
// rotating buffer sets (tools/yogi_step_probe.py, profiles/r05_yogi_step_probe.log): 25 M 0.133 -> 0.120 ms (5.27 ->
// 5.84 TB/s), 6.25 M 0.0314 -> 0.0299 ms, but 3.125 M 0.0148 -> 0.0164 ms: a step whose 28 P bytes fit in the
// 256 MiB Infinity Cache keeps hits the nt policy gives up (m, v and last of the previous round, the mean just
// written), so only steps of more than FA_YOGI_NT_MIN_BYTES take it.  Two float4 per thread per iteration: no
// faster (same log).
#ifndef FA_YOGI_NT_MIN_BYTES
#define FA_YOGI_NT_MIN_BYTES (256LL << 20)
#endif
template <bool NT, typename T>
__device__ __forceinline__ T ld_y(const T* p) {
  if (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT, typename T>
__device__ __forceinline__ void st_y(T* p, T v) {
  if (NT)
    __builtin_nontemporal_store(v, p);
  else
    *p = v;
}
template <bool NT>
__global__ __launch_bounds__(256) void k_yogi_step(const f4* __restrict__ cur, const f4* __restrict__ last,
                                                   f4* m, f4* v, f4* out, int64_t P4, float eta, float tau,
                                                   float beta, float omb, float omb2, int init) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < P4; i += (int64_t)gridDim.x * 256) {
    const f4 C = ld_y<NT>(cur + i), L = ld_y<NT>(last + i);
    f4 M = init ? f4{0.f, 0.f, 0.f, 0.f} : ld_y<NT>(m + i);
    f4 Vv = init ? f4{tau, tau, tau, tau} : ld_y<NT>(v + i);
    const f4 o = yogi4(C, L, M, Vv, eta, tau, beta, omb, omb2);
    st_y<NT>(m + i, M);
    st_y<NT>(v + i, Vv);
    st_y<NT>(out + i, o);
  }
}

static unsigned stride_grid(int64_t n4) {
  int64_t b = (n4 + 255) / 256;
  if (b > 8192) b = 8192;  // 256 CUs x 32 blocks: grid-stride the rest
  return (unsigned)(b < 1 ? 1 : b);
}

extern "C" int fa_yogi_step(const float* cur, const float* last, float* m, float* v, float* out, int64_t P,
                            float eta, float tau, float beta, float omb, float omb2, int32_t flags,
                            fa_stream_t stream) {
  if (P < 0) return fail(FA_E_ARG, "fa_yogi_step: negative P");
  if (P == 0) return FA_OK;
  if (!cur || !last || !m || !v || !out) return fail(FA_E_ARG, "fa_yogi_step: NULL pointer");
  if (!aligned16(cur) || !aligned16(last) || !aligned16(m) || !aligned16(v) || !aligned16(out))
    return fail(FA_E_ARG, "fa_yogi_step: pointers must be 16-byte aligned");
  FA_DEVICE_SCOPE("fa_yogi_step", stream, out);
  FA_OPERAND("cur", cur, cols_bytes(P));
  FA_OPERAND("last", last, cols_bytes(P));
  FA_OPERAND("m", m, cols_bytes(P));
  FA_OPERAND("v", v, cols_bytes(P));
  FA_OPERAND("out", out, cols_bytes(P));
  const int64_t P4 = (P + 3) / 4;
  hipLaunchKernelGGL(P4 * 16 * 7 > FA_YOGI_NT_MIN_BYTES ? k_yogi_step<true> : k_yogi_step<false>,
                     dim3(stride_grid(P4)), dim3(256), 0, (hipStream_t)stream,
                     (const f4*)cur, (const f4*)last, (f4*)m, (f4*)v, (f4*)out, P4, eta, tau, beta, omb, omb2,
                     (flags & FA_YOGI_INIT) ? 1 : 0);
  return check_launch("fa_yogi_step");
}

// fa_yogi_step over every part of a model sharded across this process's GPUs, in one call (round 4: with
// fa_reduce_parts, config 4's in-process N-GPU finish without a per-part host call chain).  All parts are checked
// before any launches.
extern "C" int fa_yogi_step_parts(int32_t n, const float* const* cur, const float* const* last, float* const* m,
                                  float* const* v, float* const* out, const int64_t* P, float eta, float tau,
                                  float beta, float omb, float omb2, int32_t flags, fa_stream_t const* streams) {
  if (n < 1 || !cur || !last || !m || !v || !out || !P || !streams)
    return fail(FA_E_ARG, "fa_yogi_step_parts: NULL table or n < 1");
  char what[48], nm[24];
  for (int i = 0; i < n; ++i) {
    snprintf(what, sizeof(what), "fa_yogi_step_parts[%d]", i);
    if (P[i] < 0) return fail(FA_E_ARG, "%s: negative P", what);
    if (P[i] == 0) continue;
    if (!cur[i] || !last[i] || !m[i] || !v[i] || !out[i] || !streams[i])
      return fail(FA_E_ARG, "%s: NULL pointer or stream", what);
    if (!aligned16(cur[i]) || !aligned16(last[i]) || !aligned16(m[i]) || !aligned16(v[i]) || !aligned16(out[i]))
      return fail(FA_E_ARG, "%s: pointers must be 16-byte aligned", what);
    FA_DEVICE_SCOPE(what, streams[i], out[i]);
    const uint64_t b = cols_bytes(P[i]);
    const void* ops[5] = {cur[i], last[i], m[i], v[i], out[i]};
    const char* names[5] = {"cur", "last", "m", "v", "out"};
    for (int j = 0; j < 5; ++j) {
      snprintf(nm, sizeof(nm), "%s[%d]", names[j], i);
      FA_OPERAND(nm, ops[j], b);
    }
  }
  for (int i = 0; i < n; ++i) {
    if (P[i] == 0) continue;
    snprintf(what, sizeof(what), "fa_yogi_step_parts[%d]", i);
    FA_DEVICE_SCOPE(what, streams[i], out[i]);
    const int64_t P4 = (P[i] + 3) / 4;
    hipLaunchKernelGGL(P4 * 16 * 7 > FA_YOGI_NT_MIN_BYTES ? k_yogi_step<true> : k_yogi_step<false>,
                       dim3(stride_grid(P4)), dim3(256), 0, (hipStream_t)streams[i], (const f4*)cur[i],
                       (const f4*)last[i], (f4*)m[i], (f4*)v[i], (f4*)out[i], P4, eta, tau, beta, omb, omb2,
                       (flags & FA_YOGI_INIT) ? 1 : 0);
    const int e = check_launch(what);
    if (e) return e;
  }
  return FA_OK;
}

// ------------------------------------------------------------------------------------------------
// q-FedAvg phase 1: delta chain + per-client sum of squares
// ------------------------------------------------------------------------------------------------
// Layout: a fixed grid of QF_GRID workgroups (4 waves each), each owning an equal contiguous run of
// columns that it walks in tiles of QF_V KiB per wave; the grid size is a constant so the fp64
// sum-of-squares order is deterministic across runs and devices.  Clients are taken in groups of QF_G
// (8 or 4): per client each lane sums its QF_V*4 squares in fp64 (v[j]); after the group, one
// "multi-reduce" butterfly (for 8: xor 32 / 16 / 8 halve the value set, xor 4 / 2 / 1 finish) leaves
// lane l with the wave total of client (l >> 3) & 7 — 10 fp64 shuffles per 8 clients instead of 48 —
// and the first lane of each client's lane group adds it into the LDS slot [wave][k].  At the end the
// block writes its 4-wave total per client to workspace[block][k]; k_qfed_gather sums the blocks in
// block order.  No atomics: bit-reproducible run to run.
#ifndef QF_V
#define QF_V 16
#endif
#ifndef QF_U
#define QF_U 1
#endif
#ifndef QF_G
#define QF_G 4  // clients per multi-reduce group: 4 or 8
#endif
static_assert(QF_G == 8 || QF_G == 4, "QF_G must be 4 or 8");
#ifndef QF_GRID
#define QF_GRID 256  // one workgroup per CU at 1 wave/SIMD (profiles/r01_tune_qfed.log)
#endif
#ifndef QF_CHAIN_GRID
#define QF_CHAIN_GRID QF_GRID  // the chain launches' grid (one workgroup per CU: 96 KiB of LDS each at QF_MAXK 2048)
#endif
static_assert(QF_GRID % 16 == 0 && QF_CHAIN_GRID % 16 == 0, "the norm gathers sum the grid's rows in 16 segments");
// workgroups of a k_qfed_accum launch (fixed per kind, so the fp64 norm order is the same on every run and device)
static inline int qf_grid(bool chain) { return chain ? QF_CHAIN_GRID : QF_GRID; }

#ifndef QF_BALANCE
#define QF_BALANCE 1  // 0: always full-width tiles (plain grid-stride)
#endif
// Clients per fa_qfed_accumulate call (a DeviceRound chunk).  LDS: 4 waves x QF_MAXK clients x 8 B per workgroup
// (64 KiB at 2048).  Round 4: 2048 halves the passes (and launch boundaries) of a 10,000-client round; config 5's
// shard of 8 (10,000 x 12.5 M) 70.9 ms every run against 71.0-74.1 ms at 1024, interleaved whole-library A/B on
// one box (tools/ab_c5.sh, profiles/r04_ab_c5_maxk.log).
#ifndef QF_MAXK
#define QF_MAXK 2048
#endif
static_assert(QF_MAXK % 4 == 0, "QF_MAXK: a multiple of 4 (its LDS bound is checked per kernel variant)");

struct QfArgs {
  const float* x;
  int64_t ld4, P4;
  int K;
  int flags;
  const float* last;
  const float* alpha;
  float lr, rlr;  // rlr = RN(1/lr)
  int fast;       // 0: lr outside [2^-20, 2^20] -> IEEE division for every element
  int sw;         // strips (64 f4 columns) per wave per tile, <= QF_V
  float* delta;
  float* chain;  // CHAIN: the plain FedAvg chain of the same rows (aggregator.py:500-503)
  double* part;  // [gridDim.x][K]
};

// a / b for a runtime-constant divisor b with r = RN(1/b): q = RN(a*r), then one exact-residual
// correction q + (a - b*q)*r.  Markstein's theorem: r correctly rounded and q within 1 ulp make the
// corrected quotient the correctly rounded a/b (a quotient has no midpoint cases).  It needs a normal
// residual and quotient: the host admits only 2^-20 <= |b| <= 2^20 for this path, and every element of
// the client must have |a| in [2^-80, 2^80) or a == 0 (NaN propagates correctly either way); otherwise
// (a denormal, huge or infinite element anywhere in the wave) the wave redoes that client with the
// IEEE division.  The range test is folded per lane into min/max of frexp exponents + max |a|, one wave
// vote per client.  The residual is formed negated, nrem = b*q - a, and the correction is q - nrem*r:
// the same exact values for a != 0, and the signed zero IEEE gives for a = -0 (b > 0: q = -0,
// nrem = +0, -0 + -0 = -0), where q + (a - b*q)*r would round -0 + +0 to +0.
// QF_DIV_MUL 1 (tuning builds only, WRONG BITS): the quotient is a * RN(1/b) with no correction — a power / clock
// probe of the division's cost at the card's power cap (tools/gpu/r6_div_power.sh), never a product.
#ifndef QF_DIV_MUL
#define QF_DIV_MUL 0
#endif
#if QF_DIV_MUL && !FA_TUNING
#error "QF_DIV_MUL changes results: a tuning build only (-DFA_TUNING=1)"
#endif
__device__ __forceinline__ float fast_div(float a, float b, float r) {
  const float q = a * r;
#if QF_DIV_MUL
  (void)b;
  return q;
#else
  const float nrem = __builtin_fmaf(q, b, -a);
  return __builtin_fmaf(-nrem, r, q);
#endif
}
// QF_INFCHK 1: +-inf inputs are caught per element (max |a|).  2: they are caught once per client and
// lane instead: an infinite a makes the fast quotient NaN (its residual is inf - inf), so the lane's
// sum of squares is not finite and the client is redone with the IEEE division.  A finite sum that
// overflows (|g| > 2^64) also triggers the redo, which then yields the same quotients: results never
// depend on the choice, only the VALU count does (one op per element fewer with 2).  Measured
// (profiles/r01_tune_qfed_infchk.log): 2 is no faster at 25 M / 12.5 M and 4 % slower at 11.19 M, so 1 stays.
#ifndef QF_INFCHK
#define QF_INFCHK 1
#endif
// QF_EMAX 0: the upper bound is tested on max |a| alone (|a| < 2^80 also excludes +-inf), so the frexp
// exponent feeds only the lower bound — one max3 per two elements fewer.  1: round 1's form.
#ifndef QF_EMAX
#define QF_EMAX 1
#endif
// QF_PART: squares per fp32 partial before the fp64 sum (4, 8 or 16; each partial is one cvt + one fp64 add)
#ifndef QF_PART
#define QF_PART 4
#endif
// The chain launches' own knobs (round 4).  Round 2 kept them equal to the plain launches' so that both summed
// the norms identically; since round 3's 8-float4 chain tiles sum them in another fp64 order anyway, the chain
// launches take the cheaper forms: the range test on max |a| alone and fp32 partials of 8 squares — one v_max3
// per two elements and one cvt + fp64 add per 8 squares fewer.  Measured interleaved on one box
// (tools/tune_qfed2.py, profiles/r04_tune_qfed_chain_knobs.log): 1024 x 12.5 M 7.354 -> 7.185 ms (first pass) and
// 7.361 -> 7.185 ms (later passes), 1000 x 25 M 14.47 -> 14.06 ms; the chain launches now read faster than the
// plain ones.  The norms move by <= 1e-10 relative (the fp32 value hs consumes: at most one ulp).
#ifndef QF_CHAIN_EMAX
#define QF_CHAIN_EMAX 0
#endif
#ifndef QF_CHAIN_PART
#define QF_CHAIN_PART 8
#endif
static_assert(QF_CHAIN_PART == 4 || QF_CHAIN_PART == 8 || QF_CHAIN_PART == 16, "QF_CHAIN_PART: 4, 8 or 16");
static_assert(QF_PART == 4 || QF_PART == 8 || QF_PART == 16, "QF_PART: 4, 8 or 16");
// EMAX picks which bound test admits an element to the fast division; both tests admit only elements the
// fast division gets correctly rounded, so the choice never changes a bit, only the VALU count.
template <bool EMAX>
struct DivRange {
  int emin = 0;  // frexp exponents (0 for +-0): |a| in [2^(e-1), 2^e)
  int emax = 0;
  float amax = 0.f;  // catches +-inf (frexp reports 0 for it)
  __device__ __forceinline__ void add(float a) {
    const int e = __builtin_amdgcn_frexp_expf(a);
    emin = e < emin ? e : emin;
    if (EMAX) emax = e > emax ? e : emax;
    if (QF_INFCHK == 1 || !EMAX) amax = __builtin_fmaxf(amax, __builtin_fabsf(a));
  }
  __device__ __forceinline__ bool ok() const {
    if (!EMAX) return emin >= -79 && amax < 0x1p80f;
    if (QF_INFCHK == 1) return emin >= -79 && emax <= 80 && amax < __builtin_inff();
    return emin >= -79 && emax <= 80;
  }
};

__device__ __forceinline__ double shfl_xor_d(double v, int m) { return __shfl_xor(v, m, 64); }

// Client rows are read through buffer descriptors (cdna guide T8) and every mask is an offset: a lane
// whose column is past P (or past its wave's sw strips) gets the voffset sentinel QF_OOB, which is past
// num_records, so the hardware returns zero without touching memory — one load path, no exec masking.
//  * WIDE (QF_G rows span < 2 GiB): ONE descriptor per client group, base = the group's first row,
//    num_records = its valid rows only; voffset = column + row * rowbytes, so rows of clients past K are
//    out of range too.
//  * otherwise: one descriptor per client row, num_records = the row's P4 * 16 bytes (rows past K: 0);
//    the host cuts P into column windows of < 2 GiB (fa_qfed_accumulate).
// aux 2 = non-temporal.
#define QF_OOB 0x80000000u
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rows_rsrc(const float* row0, uint32_t nbytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(row0), (short)0, (int)nbytes, 0x00020000);
}
__device__ __forceinline__ f4 rows_load(__amdgpu_buffer_rsrc_t r, uint32_t voff) {
  return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)voff, 0, 2));
}
// 16 B per lane HBM -> LDS (buffer_load_dwordx4 ... lds, non-temporal): lane i's bytes land at LDS address
// lds + 16 i.  A plain device function, so the kernel templates that call it stay valid in the host pass.
__device__ __forceinline__ void rows_load_lds(__amdgpu_buffer_rsrc_t r, uint32_t lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)(uintptr_t)lds, 16, voff, 0,
                                           0, 2);
}

#ifndef QF_MINW
#define QF_MINW 1
#endif
// WIDE: one descriptor spans all QF_G rows of a group (QF_G rows < 4 GiB); otherwise one per QF_U rows.
// GLDS > 0: the next GLDS clients' row slices stream HBM -> LDS (buffer_load_dwordx4 ... lds, no VGPR
// destination) while the wave computes the current client from registers; at the top of each client the
// wave copies its landed slice LDS -> registers (16 ds_read_b128) and re-arms the DMA, so loads stay in
// flight through the compute phase at no register cost (GLDS x 16 KiB of LDS per wave).  Measured
// (profiles/r02_tune_qfed2.log): 2-4 % SLOWER than register loads for the plain kernel, 1-5 % FASTER with
// the fused FedAvg chain (whose 64 extra live values otherwise go through AGPRs), so chain launches use it.
template <bool WIDE, bool CHAIN, int GLDS, int QV>
__global__ __launch_bounds__(256, QF_MINW) void k_qfed_accum(QfArgs q) {
  static_assert(GLDS == 0 || GLDS == 1 || (GLDS == 2 && (QV == 16 || QV == 12 || QV == 8)),
                "GLDS: 0, 1 or 2 LDS slices per wave (2: 16 or 12 float4 per lane)");
  constexpr int NB = GLDS > 0 ? GLDS : 1;
  // ONE static LDS array, so it sits at LDS offset 0: the row slices first (the DMA addresses them from
  // offset 0), then the per-client squared norms sq[4][QF_MAXK] (64 KiB at QF_MAXK 2048).  The chain launches
  // (GLDS 1, QV 8): 32 KiB + 64 KiB = 96 KiB, one workgroup per CU.
  constexpr int ROWB = GLDS > 0 ? GLDS * 4 * QV * 64 : 0;  // f4 elements of row slices
  static_assert(ROWB * 16 + 4 * QF_MAXK * 8 <= 160 * 1024,
                "k_qfed_accum: row slices + per-client norms exceed gfx950's 160 KiB of LDS (GLDS / QV / QF_MAXK)");
  __shared__ f4 lds_all[ROWB + 4 * QF_MAXK / 2];
  f4* const rowbuf = lds_all;
  double(*const sq)[QF_MAXK] = reinterpret_cast<double(*)[QF_MAXK]>(lds_all + ROWB);
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  for (int i = threadIdx.x; i < 4 * QF_MAXK; i += 256) (&sq[0][0])[i] = 0.0;
  __syncthreads();

  // Balanced grid-stride: the columns come in strips of 64 f4 (one wave-wide dwordx4 load).  A tile is
  // 4 waves x sw strips, sw <= QV chosen so that the tiles divide evenly over the grid (fa_qfed_
  // accumulate: q.sw) — no workgroup is left with an extra tile whatever P is — and the workgroups
  // stride over tiles so the grid's concurrent loads stay on adjacent addresses.
  const int64_t S = (q.P4 + 63) / 64;
  const int sw = q.sw;
  const int64_t ntiles = (S + 4 * sw - 1) / (4 * sw);
  const uint32_t rowbytes = (uint32_t)(q.ld4 * 16);
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const int64_t sw0 = tile * 4 * sw + (int64_t)wave * sw;  // this wave's first strip
    const int64_t c0 = sw0 * 64 + lane;
    bool ok[QV];
    f4 L[QV], D[QV], C[QV];
    uint32_t voff[QV];  // byte offset of this lane's column j in a row, or QF_OOB
#pragma unroll
    for (int j = 0; j < QV; ++j) {
      ok[j] = j < sw && (c0 + 64 * j) < q.P4;
      voff[j] = ok[j] ? (uint32_t)((c0 + 64 * j) * 16) : QF_OOB;
      L[j] = ok[j] ? reinterpret_cast<const f4*>(q.last)[c0 + 64 * j] : f4{0.f, 0.f, 0.f, 0.f};
      D[j] = (ok[j] && (q.flags & FA_ACCUMULATE)) ? reinterpret_cast<const f4*>(q.delta)[c0 + 64 * j]
                                                  : f4{0.f, 0.f, 0.f, 0.f};
      if (CHAIN)
        C[j] = (ok[j] && (q.flags & FA_ACCUMULATE)) ? reinterpret_cast<const f4*>(q.chain)[c0 + 64 * j]
                                                    : f4{0.f, 0.f, 0.f, 0.f};
    }
    // one client: g = (L - W)/lr from its loaded row slice t (overwritten with L - W), delta chain and the
    // lane's fp64 sum of squares
    auto client = [&](f4(&t)[QV], int kk, float al) -> double {
      const bool first = (kk == 0) && !(q.flags & FA_ACCUMULATE);
      f4 g[QV];
      DivRange<(CHAIN ? QF_CHAIN_EMAX : QF_EMAX) != 0> rng;
#pragma unroll
      for (int j = 0; j < QV; ++j) {
        if (CHAIN) C[j] = first ? t[j] : C[j] + t[j];  // the FedAvg chain of the same upload
        t[j] = L[j] - t[j];  // (last - W), optimizers.py:83; the "* 1.0" is exact
        g[j].x = fast_div(t[j].x, q.lr, q.rlr);
        g[j].y = fast_div(t[j].y, q.lr, q.rlr);
        g[j].z = fast_div(t[j].z, q.lr, q.rlr);
        g[j].w = fast_div(t[j].w, q.lr, q.rlr);
        rng.add(t[j].x);
        rng.add(t[j].y);
        rng.add(t[j].z);
        rng.add(t[j].w);
      }
      constexpr int PART = CHAIN ? QF_CHAIN_PART : QF_PART;
      static_assert(QV % (PART / 4) == 0, "a tile's float4 columns split into whole partials");
      double acc = 0.0;
#pragma unroll
      for (int j = 0; j < QV; j += PART / 4) {
        float s = 0.f;
#pragma unroll
        for (int i = 0; i < PART / 4; ++i) {
          const f4 g2 = g[j + i] * g[j + i];  // torch.square(grad), fp32
          const float s4 = (g2.x + g2.y) + (g2.z + g2.w);
          s = i == 0 ? s4 : s + s4;
        }
        acc += (double)s;  // PART-term fp32 partial, then fp64
      }
#if QF_INFCHK == 1
      const bool fast_ok = rng.ok();
#else
      const bool fast_ok = rng.ok() && __builtin_isfinite(acc);
#endif
      if (!q.fast || !__all(fast_ok)) {  // rare: redo this client with the IEEE division
        acc = 0.0;
#pragma unroll
        for (int j = 0; j < QV; ++j) {
          g[j].x = __fdiv_rn(t[j].x, q.lr);
          g[j].y = __fdiv_rn(t[j].y, q.lr);
          g[j].z = __fdiv_rn(t[j].z, q.lr);
          g[j].w = __fdiv_rn(t[j].w, q.lr);
        }
#pragma unroll
        for (int j = 0; j < QV; j += PART / 4) {  // the same partials as the fast path
          float s = 0.f;
#pragma unroll
          for (int i = 0; i < PART / 4; ++i) {
            const f4 g2 = g[j + i] * g[j + i];
            const float s4 = (g2.x + g2.y) + (g2.z + g2.w);
            s = i == 0 ? s4 : s + s4;
          }
          acc += (double)s;
        }
      }
#pragma unroll
      for (int j = 0; j < QV; ++j) {
        const f4 term = al * g[j];  // optimizers.py:89,93  float_power(...) * grad (fp32 product)
        D[j] = first ? term : D[j] + term;
      }
      return acc;
    };
    f4* myrow = rowbuf + (GLDS > 0 ? wave * (NB * QV * 64) + lane : 0);
    // the DMA takes an absolute LDS address: rowbuf is at offset 0 of the kernel's only LDS array (with two
    // LDS variables the compiler may place either first — round 2's layout worked by that accident)
    const uint32_t ldsbase = (uint32_t)__builtin_amdgcn_readfirstlane(wave) * (NB * QV * 64 * 16);
    // client k's row slice -> this wave's LDS buffer (OOB lanes write 0).  Issued for every client,
    // k == K included (an empty range: zeros, no memory access), so the wait counts stay the same on
    // every path and the compiler never falls back to draining the DMA mid-client.
    auto glds_rows = [&](int k) {
      const __amdgpu_buffer_rsrc_t rr =
          rows_rsrc(q.x + (int64_t)k * q.ld4 * 4, k < q.K ? (uint32_t)(q.P4 * 16) : 0u);
      const uint32_t slot = (uint32_t)(k % NB) * (QV * 64 * 16);
#pragma unroll
      for (int j = 0; j < QV; ++j) rows_load_lds(rr, ldsbase + slot + (uint32_t)(j * 64 * 16), voff[j]);
    };
    // prologue: the first GLDS clients' alphas and slices in flight (alpha before its slice)
    float al_q[NB];
    if constexpr (GLDS > 0) {
#pragma unroll
      for (int i = 0; i < GLDS; ++i) {
        al_q[i] = q.alpha[i < q.K ? i : q.K - 1];
        glds_rows(i);
      }
    }
    for (int kg = 0; kg < q.K; kg += QF_G) {
      double v[QF_G];
#pragma unroll
      for (int jj = 0; jj < QF_G; ++jj) v[jj] = 0.0;
      if constexpr (GLDS > 0) {
#pragma unroll
      for (int u = 0; u < QF_G; ++u) {
        const int kk = kg + u;
        if (kk >= q.K) break;  // uniform
        // client kk's slice has landed in LDS: everything issued before the last (GLDS-1) clients'
        // alpha + 16 slice loads has completed (the vector memory counter retires in order)
        if constexpr (GLDS == 1)
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        else  // (GLDS - 1) x (alpha + 16 slice loads) may stay in flight
          if constexpr (QV == 16)
            asm volatile("s_waitcnt vmcnt(17)" ::: "memory");
          else if constexpr (QV == 12)
            asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
          else
            asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
        f4 t[QV];
        const f4* src = myrow + (kk % NB) * (QV * 64);
#pragma unroll
        for (int j = 0; j < QV; ++j) t[j] = src[64 * j];
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // ... and is in registers: refill the slot
        const float al = al_q[0];
#pragma unroll
        for (int i = 0; i + 1 < NB; ++i) al_q[i] = al_q[i + 1];
        // the alpha of client kk + GLDS is requested BEFORE its slice, so waiting for it never drains
        // the DMA; past K: a repeated alpha and an empty range (zeros, no memory access)
        const int kn = kk + GLDS;
        al_q[NB - 1] = q.alpha[kn < q.K ? kn : q.K - 1];
        glds_rows(kn);
        v[u] = client(t, kk, al);
      }
      } else {
      const int nrows = q.K - kg < QF_G ? q.K - kg : QF_G;
      const float* row0 = q.x + (int64_t)kg * q.ld4 * 4;
      const __amdgpu_buffer_rsrc_t grp = rows_rsrc(row0, WIDE ? (uint32_t)nrows * rowbytes : 0u);
#pragma unroll
      for (int u0 = 0; u0 < QF_G; u0 += QF_U) {
        f4 t[QF_U][QV];
#pragma unroll
        for (int u = 0; u < QF_U; ++u) {
          if (WIDE) {
#pragma unroll
            for (int j = 0; j < QV; ++j) t[u][j] = rows_load(grp, voff[j] + (uint32_t)(u0 + u) * rowbytes);
          } else {
            const __amdgpu_buffer_rsrc_t rr =
                rows_rsrc(row0 + (int64_t)(u0 + u) * q.ld4 * 4, u0 + u < nrows ? (uint32_t)(q.P4 * 16) : 0u);
#pragma unroll
            for (int j = 0; j < QV; ++j) t[u][j] = rows_load(rr, voff[j]);
          }
        }
#pragma unroll
        for (int u = 0; u < QF_U; ++u) {
          const int kk = kg + u0 + u;
          if (kk >= q.K) break;  // uniform
          v[u0 + u] = client(t[u], kk, q.alpha[kk]);
        }
      }
      }
      // multi-reduce: QF_G values per lane -> lane l holds the wave sum of client (l >> s) & (QF_G-1)
      double y;
      const bool b5 = lane & 32, b4 = lane & 16, b3 = lane & 8;
#if QF_G == 8
      double w4[4], w2[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double keep = b5 ? v[i + 4] : v[i], send = b5 ? v[i] : v[i + 4];
        w4[i] = keep + shfl_xor_d(send, 32);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const double keep = b4 ? w4[i + 2] : w4[i], send = b4 ? w4[i] : w4[i + 2];
        w2[i] = keep + shfl_xor_d(send, 16);
      }
      {
        const double keep = b3 ? w2[1] : w2[0], send = b3 ? w2[0] : w2[1];
        y = keep + shfl_xor_d(send, 8);
      }
      constexpr int csh = 3;  // client index bits: lane bits 5..3
#else
      double w2[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const double keep = b5 ? v[i + 2] : v[i], send = b5 ? v[i] : v[i + 2];
        w2[i] = keep + shfl_xor_d(send, 32);
      }
      {
        const double keep = b4 ? w2[1] : w2[0], send = b4 ? w2[0] : w2[1];
        y = keep + shfl_xor_d(send, 16);
      }
      y += shfl_xor_d(y, 8);
      (void)b3;
      constexpr int csh = 4;  // client index bits: lane bits 5..4
#endif
      y += shfl_xor_d(y, 4);
      y += shfl_xor_d(y, 2);
      y += shfl_xor_d(y, 1);
      const int jcl = (lane >> csh) & (QF_G - 1);
      if ((lane & ((1 << csh) - 1)) == 0 && kg + jcl < q.K) sq[wave][kg + jcl] += y;
    }
#pragma unroll
    for (int j = 0; j < QV; ++j)
      if (ok[j]) {
        reinterpret_cast<f4*>(q.delta)[c0 + 64 * j] = D[j];
        if (CHAIN) reinterpret_cast<f4*>(q.chain)[c0 + 64 * j] = C[j];
      }
  }
  __syncthreads();
  for (int k = threadIdx.x; k < q.K; k += 256)
    q.part[(int64_t)blockIdx.x * q.K + k] = ((sq[0][k] + sq[1][k]) + sq[2][k]) + sq[3][k];
}

#if FA_TUNING
// ------------------------------------------------------------------------------------------------
// q-FedAvg phase 1, second design (QF_KERNEL / QF_CHAIN_KERNEL 2; measured slower, built off): 2 waves per SIMD
// ------------------------------------------------------------------------------------------------
// The first design (k_qfed_accum above) runs 1 wave per SIMD: `last`, the delta chain, the loaded row and
// the quotients all live in registers (256 VGPRs + AGPR parking), so a wave has no loads in flight while
// it computes (~20 % of its time) and the kernel reads HBM at 0.83 of peak.  Here:
//  * the wave's `last` tile lives in LDS (written and read back by the same lane: no barrier), 16 KiB per
//    wave, 8 waves = 128 KiB per workgroup, one workgroup per CU;
//  * per client, pass 1 forms a = last - W in place of the loaded row and folds the range test of the
//    constant-divisor division; the wave votes; pass 2 divides (fast or IEEE for the whole client),
//    squares and extends the delta chain — no quotient array, so t, D (and the FedAvg chain C) fit in
//    < 256 VGPRs: 2 waves per SIMD cover each other's compute phases with their loads;
//  * CHAIN: the plain FedAvg chain C += W (aggregator.py:500-503) rides along (+1 add per element and
//    +8P bytes per chunk), so the reference's model_weights (the mean, :505-507) exists for any K;
//  * per-client partial squared norms: each (workgroup, wave) owns a row of K fp64 in the workspace and
//    accumulates its tiles into it in tile order (read-add-write, the read issued ahead of the group's
//    loads); k_qfed_gather2a/b then sum the 2048 rows in a fixed two-level order.  No atomics, so the
//    result is the same bits on every run and every device.
#ifndef QF_KERNEL
#define QF_KERNEL 1  // the no-chain launches (profiles/r02_tune_qfed2.log: the 1-wave design reads faster)
#endif
#ifndef QF2_WAVES
#define QF2_WAVES 8
#endif
#ifndef QF2_V
#define QF2_V 16
#endif
#ifndef QF2_GRID
#define QF2_GRID 256
#endif
#define QF2_SEG 32  // first-level segments of the norm gather
#define QF2_ROWS (QF2_GRID * QF2_WAVES)

struct Qf2Args {
  const float* x;
  int64_t ld4, P4;
  int K;
  int flags;
  const float* last;
  const float* alpha;
  float lr, rlr;
  int fast;
  int sw;  // strips (64 f4 columns) per wave per tile, <= QF2_V
  float* delta;
  float* chain;
  double* part;  // [QF2_ROWS][K]
};

template <bool CHAIN>
__global__ __launch_bounds__(64 * QF2_WAVES, 1) void k_qfed_accum2(Qf2Args q) {
  __shared__ f4 Ls[QF2_WAVES * QF2_V * 64];
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  f4* myL = Ls + wave * (QF2_V * 64) + lane;  // slot j at myL[64 * j]: this lane's own bytes
  const int64_t S = (q.P4 + 63) / 64;
  const int sw = q.sw;
  const int64_t ntiles = (S + (int64_t)QF2_WAVES * sw - 1) / ((int64_t)QF2_WAVES * sw);
  const uint32_t rowbytes = (uint32_t)(q.P4 * 16);
  const bool acc_in = (q.flags & FA_ACCUMULATE) != 0;
  double* prow = q.part + ((int64_t)blockIdx.x * QF2_WAVES + wave) * q.K;
  const int jcl = (lane >> 4) & 3;           // the client whose wave total this lane ends up with
  const bool writer = (lane & 15) == 0;
  const f4 z4 = f4{0.f, 0.f, 0.f, 0.f};
  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const bool first_tile = tile == (int64_t)blockIdx.x;
    const int64_t c0 = (tile * QF2_WAVES + wave) * sw * 64 + lane;
    uint32_t voff[QF2_V];
    f4 D[QF2_V], C[QF2_V];
#pragma unroll
    for (int j = 0; j < QF2_V; ++j) {
      const bool ok = j < sw && c0 + 64 * j < q.P4;
      voff[j] = ok ? (uint32_t)((c0 + 64 * j) * 16) : QF_OOB;
      myL[64 * j] = ok ? reinterpret_cast<const f4*>(q.last)[c0 + 64 * j] : z4;
      D[j] = (ok && acc_in) ? reinterpret_cast<const f4*>(q.delta)[c0 + 64 * j] : z4;
      if (CHAIN) C[j] = (ok && acc_in) ? reinterpret_cast<const f4*>(q.chain)[c0 + 64 * j] : z4;
    }
    for (int kg = 0; kg < q.K; kg += 4) {
      // this (workgroup, wave) row's running norms of the group's clients, from the earlier tiles
      double old = 0.0;
      if (!first_tile && writer && kg + jcl < q.K) old = prow[kg + jcl];
      double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
      // not unrolled: one client's row slice in registers at a time (an unrolled loop lets the scheduler
      // hoist the next client's 16 loads and spill)
      const int un = q.K - kg < 4 ? q.K - kg : 4;
#pragma unroll 1
      for (int u = 0; u < un; ++u) {
        const int k = kg + u;
        // compiler barrier: the `last` tile is re-read from LDS for every client (hoisting those reads out
        // of the loop would put the tile back into 64 VGPRs and halve the occupancy)
        asm volatile("" ::: "memory");
        const __amdgpu_buffer_rsrc_t rr = rows_rsrc(q.x + (int64_t)k * q.ld4 * 4, rowbytes);
        f4 t[QF2_V];
#pragma unroll
        for (int j = 0; j < QF2_V; ++j) t[j] = rows_load(rr, voff[j]);
        const bool first = (k == 0) && !acc_in;
        DivRange<QF_EMAX != 0> rng;
#pragma unroll
        for (int j = 0; j < QF2_V; ++j) {  // pass 1: the FedAvg chain, a = last - W, the range test
          if (CHAIN) C[j] = first ? t[j] : C[j] + t[j];
          t[j] = myL[64 * j] - t[j];  // (last - W), optimizers.py:83; the "* 1.0" is exact
          rng.add(t[j].x);
          rng.add(t[j].y);
          rng.add(t[j].z);
          rng.add(t[j].w);
        }
        const float al = q.alpha[k];
        double acc = 0.0;
        if (q.fast && __all(rng.ok())) {  // pass 2: divide, square, extend the delta chain
#pragma unroll
          for (int j = 0; j < QF2_V; ++j) {
            f4 g;
            g.x = fast_div(t[j].x, q.lr, q.rlr);
            g.y = fast_div(t[j].y, q.lr, q.rlr);
            g.z = fast_div(t[j].z, q.lr, q.rlr);
            g.w = fast_div(t[j].w, q.lr, q.rlr);
            const f4 g2 = g * g;                             // torch.square(grad), fp32
            acc += (double)((g2.x + g2.y) + (g2.z + g2.w));  // 4-term fp32 partial, then fp64
            const f4 term = al * g;                          // float_power(...) * grad (fp32 product)
            D[j] = first ? term : D[j] + term;
          }
        } else {  // rare: the whole client with the IEEE division
#pragma unroll
          for (int j = 0; j < QF2_V; ++j) {
            f4 g;
            g.x = __fdiv_rn(t[j].x, q.lr);
            g.y = __fdiv_rn(t[j].y, q.lr);
            g.z = __fdiv_rn(t[j].z, q.lr);
            g.w = __fdiv_rn(t[j].w, q.lr);
            const f4 g2 = g * g;
            acc += (double)((g2.x + g2.y) + (g2.z + g2.w));
            const f4 term = al * g;
            D[j] = first ? term : D[j] + term;
          }
        }
        v0 = u == 0 ? acc : v0;
        v1 = u == 1 ? acc : v1;
        v2 = u == 2 ? acc : v2;
        v3 = u == 3 ? acc : v3;
      }
      // multi-reduce: lane l ends with the wave total of client kg + ((l >> 4) & 3)
      double y;
      {
        const double v[4] = {v0, v1, v2, v3};
        const bool b5 = lane & 32, b4 = lane & 16;
        double w2[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const double keep = b5 ? v[i + 2] : v[i], send = b5 ? v[i] : v[i + 2];
          w2[i] = keep + shfl_xor_d(send, 32);
        }
        const double keep = b4 ? w2[1] : w2[0], send = b4 ? w2[0] : w2[1];
        y = keep + shfl_xor_d(send, 16);
        y += shfl_xor_d(y, 8);
        y += shfl_xor_d(y, 4);
        y += shfl_xor_d(y, 2);
        y += shfl_xor_d(y, 1);
      }
      if (writer && kg + jcl < q.K) prow[kg + jcl] = first_tile ? y : old + y;
    }
#pragma unroll
    for (int j = 0; j < QF2_V; ++j) {
      if (voff[j] == QF_OOB) continue;
      reinterpret_cast<f4*>(q.delta)[c0 + 64 * j] = D[j];
      if (CHAIN) reinterpret_cast<f4*>(q.chain)[c0 + 64 * j] = C[j];
    }
  }
  // rows of waves that owned no tile at all (tiny P) must still be defined
  if ((int64_t)blockIdx.x >= ntiles)
    for (int k = lane; k < q.K; k += 64) prow[k] = 0.0;
}

// first level: segment s of the QF2_ROWS partial rows -> seg[s][k]; second: sqnorm[k] += sum_s seg[s][k]
__global__ __launch_bounds__(256) void k_qfed_gather2a(const double* __restrict__ part, int K, double* seg) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  constexpr int rps = QF2_ROWS / QF2_SEG;
  const double* p = part + (int64_t)blockIdx.y * rps * K + k;
  double s = 0.0;
#pragma unroll 8
  for (int r = 0; r < rps; ++r) s += p[(int64_t)r * K];
  seg[(int64_t)blockIdx.y * K + k] = s;
}
__global__ __launch_bounds__(256) void k_qfed_gather2b(const double* __restrict__ seg, int K, double* sqnorm) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  double s = 0.0;
  for (int i = 0; i < QF2_SEG; ++i) s += seg[(int64_t)i * K + k];
  sqnorm[k] += s;
}
static_assert(QF2_ROWS % QF2_SEG == 0, "gather segments must divide the partial rows");
#endif  // FA_TUNING (k_qfed_accum2)

#define QF_GATHER_SEG 16
__global__ __launch_bounds__(256) void k_qfed_gather_seg(const double* __restrict__ part, int nrows, int K,
                                                         double* seg) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  const int rps = nrows / QF_GATHER_SEG;
  const double* p = part + (int64_t)blockIdx.y * rps * K + k;
  double s = 0.0;
#pragma unroll 4
  for (int r = 0; r < rps; ++r) s += p[(int64_t)r * K];
  seg[(int64_t)blockIdx.y * K + k] = s;
}
static_assert(QF_GRID % QF_GATHER_SEG == 0 && QF_CHAIN_GRID % QF_GATHER_SEG == 0,
              "gather segments must divide the grid");

__global__ __launch_bounds__(256) void k_qfed_gather(const double* __restrict__ part, int nblk, int K,
                                                     double* sqnorm) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  double s = 0.0;
  for (int b = 0; b < nblk; ++b) s += part[(int64_t)b * K + k];
  sqnorm[k] += s;
}

// Deferred gathers (a call with several column windows and a workspace that holds every window's partials):
// seg[w][y][k] = the y-th 16-row segment sum of window w's QF_GRID partial rows, all windows in one launch, then
// per client, window by window in order: s = sum of the 16 segments from 0.0; sqnorm[k] += s — the same adds
// in the same order as the per-window pair above, so the norms are bit-identical; one pair of launches per
// call instead of one per window (each window's pair cost ~13 us: 2.5 % of config 5's 0.55 ms chain windows).
__global__ __launch_bounds__(256) void k_qfed_gather_seg_win(const double* __restrict__ part, int nrows, int K,
                                                             int64_t per_win, double* seg) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  const int rps = nrows / QF_GATHER_SEG;
  const double* p = part + (int64_t)blockIdx.z * per_win + (int64_t)blockIdx.y * rps * K + k;
  double s = 0.0;
#pragma unroll 4
  for (int r = 0; r < rps; ++r) s += p[(int64_t)r * K];
  seg[((int64_t)blockIdx.z * QF_GATHER_SEG + blockIdx.y) * K + k] = s;
}

__global__ __launch_bounds__(256) void k_qfed_gather_win(const double* __restrict__ seg, int K, int nwin,
                                                         double* sqnorm) {
  const int k = blockIdx.x * 256 + threadIdx.x;
  if (k >= K) return;
  double acc = sqnorm[k];
  for (int w = 0; w < nwin; ++w) {
    double s = 0.0;
    for (int b = 0; b < QF_GATHER_SEG; ++b) s += seg[((int64_t)w * QF_GATHER_SEG + b) * K + k];
    acc += s;
  }
  sqnorm[k] = acc;
}

// The same sums with one wave per client: lane l forms the window sums s_w of windows w = l, l + 64, ... (each from
// 0.0 over its 16 segments in order, as above) into LDS, then lane 0 adds them to sqnorm[k] in window order — the
// same adds in the same order, so the same bits.  One memory round trip per 64 windows instead of one per window:
// the thread-per-client form above waits on nwin dependent batches of loads (config 5 on one GPU: 50 windows, 57-68
// us per call, profiles/r05_prof_all_by_shape.jsonl).
#define QF_GWIN_MAX 1024  // windows per call this form takes (the host keeps the form above beyond it)
__global__ __launch_bounds__(256) void k_qfed_gather_win_wave(const double* __restrict__ seg, int K, int nwin,
                                                              double* sqnorm) {
  __shared__ double sw[4][QF_GWIN_MAX];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int k = blockIdx.x * 4 + wave;
  if (k < K) {
    for (int w = lane; w < nwin; w += 64) {
      double s = 0.0;
#pragma unroll
      for (int b = 0; b < QF_GATHER_SEG; ++b) s += seg[((int64_t)w * QF_GATHER_SEG + b) * K + k];
      sw[wave][w] = s;
    }
  }
  __syncthreads();
  if (k < K && lane == 0) {
    double acc = sqnorm[k];
    for (int w = 0; w < nwin; ++w) acc += sw[wave][w];
    sqnorm[k] = acc;
  }
}

extern "C" int fa_qfed_max_chunk(void) { return QF_MAXK; }

static int64_t qfed_window(int64_t ld, int64_t P, bool chain);
// one window's partials + segments (the per-window gathers), either kernel family
static int64_t qfed_ws_one(int64_t k) {
  const int64_t g = QF_GRID > QF_CHAIN_GRID ? QF_GRID : QF_CHAIN_GRID;
  const int64_t w1 = (g + QF_GATHER_SEG) * k * 8;
#if FA_TUNING  // (the workspace size is part of the ABI: tuning builds keep the default build's figure or more)
  const int64_t w2 = ((int64_t)QF2_ROWS + QF2_SEG) * k * 8;
#else
  const int64_t w2 = (2048LL + 32) * k * 8;  // = k_qfed_accum2's at its defaults: callers' workspaces stay valid
#endif
  return w1 > w2 ? w1 : w2;
}
// every window's partials + segments (deferred gathers) of a call at (K, ld, P), chain or not
static int64_t qfed_ws_deferred(int64_t k, int64_t ld, int64_t P, bool chain) {
  const int64_t win = qfed_window(ld, P, chain), nwin = P > win ? (P + win - 1) / win : 1;
  return nwin * ((int64_t)qf_grid(chain) + QF_GATHER_SEG) * k * 8;
}
extern "C" int64_t fa_qfed_workspace_bytes(int32_t K, int64_t ld, int64_t P) {
  const int64_t k = K > 0 ? K : 1;
  int64_t b = qfed_ws_one(k);
  if (ld >= P && P > 0) {
    const int64_t c = qfed_ws_deferred(k, ld, P, true), n = qfed_ws_deferred(k, ld, P, false);
    if (c > b) b = c;
    if (n > b) b = n;
  }
  return b;
}

#ifndef QF_CHAIN_KERNEL
#define QF_CHAIN_KERNEL 1
#endif
#if !FA_TUNING && ((defined(QF_KERNEL) && QF_KERNEL != 1) || QF_CHAIN_KERNEL != 1)
#error "QF_KERNEL / QF_CHAIN_KERNEL 2 (k_qfed_accum2) is a tuning build: add -DFA_TUNING=1"
#endif
#ifndef QF_GATHER_WAVE
#define QF_GATHER_WAVE 1  // deferred gathers: the wave-per-client window fold (k_qfed_gather_win_wave)
#endif
#ifndef QF_DEFER_GATHER
#define QF_DEFER_GATHER 1  // one gather pair per call over every window's partials (workspace permitting)
#endif
#ifndef QF_CHAIN_GLDS
#define QF_CHAIN_GLDS 1  // LDS-DMA slices per wave of the chain launches (profiles/r02_tune_qfed2.log)
#endif
#ifndef QF_PLAIN_GLDS
#define QF_PLAIN_GLDS 0
#endif
// Tile width (float4 per lane) of the chain launches.  The fused FedAvg chain adds 4*QV live values per
// lane; at 16 float4 the LDS-DMA design parks ~200 values in AGPRs (15.0 vs 14.1 ms at 1000 x 25 M).  Round 3
// measured 4..16 interleaved on three shapes (profiles/r03_tune_qfed_chain_width2.log): 8 is the fastest
// everywhere (1000 x 25 M and 1024 x 12.5 M at the plain kernel's time, 462 x 100 M 1.5-2 % above it; 12:
// +2-5 %, 10 and 6: +3-6 %, 4: +25 %).  The plain launches keep 16 (the register design at 12 is 10 %
// slower, LDS-DMA at 8 mixed: -1 % / +4 % by shape).  Tiles of another width sum each client's squares in
// another fp64 order: chain and plain launches' norms agree to ~1e-16 relative.
#ifndef QF_CHAIN_V
#define QF_CHAIN_V 8
#endif
#ifndef QF_WIN_ROUNDS
#define QF_WIN_ROUNDS 1  // column windows of this many rounds of full-width tiles (0: no windows)
#endif
#ifndef QF_CHAIN_WIN_ROUNDS
#define QF_CHAIN_WIN_ROUNDS QF_WIN_ROUNDS  // the same for the chain launches
#endif
#ifndef QF_WIDE_BYTES
#define QF_WIDE_BYTES (1LL << 31)  // largest QF_G-row span served by one descriptor (tuning knob; <= 2^31)
#endif
static_assert(QF_WIDE_BYTES <= (1LL << 31), "QF_WIDE_BYTES: the rows plus the OOB sentinel must stay below 2^32");

// Column window of one k_qfed_accum launch: per-row descriptors need windows of <= 2^28 columns, and long
// rows run as windows of one round of full-width tiles (QF_WIN_ROUNDS) — over several rounds of ~1000
// clients the workgroups drift apart and a launch boundary re-aligns them (tools/tune_qfed2.py,
// profiles/r02_tune_qfed_windows.log: 1000 x 25 M 6.87 -> 7.03 TB/s, 462 x 100 M 6.34 -> 6.89).  The
// windows' gathers add their per-client partial norms in window order (deterministic; fp64).
static int64_t qfed_window(int64_t ld, int64_t P, bool chain) {
  const bool wide = (int64_t)ld * 4 * QF_G <= QF_WIDE_BYTES;
  int64_t win = wide ? (P > 0 ? P : 1) : (1LL << 28);
  const int64_t qv = chain ? QF_CHAIN_V : QF_V, rounds = chain ? QF_CHAIN_WIN_ROUNDS : QF_WIN_ROUNDS;
  const int64_t cols = rounds * qf_grid(chain) * 4 * qv * 256;  // rounds of full-width tiles
  if (cols > 0 && win > cols) win = cols;
  return win;
}

extern "C" int64_t fa_qfed_launches(int64_t ld, int64_t P, int32_t chain) {
  if (P <= 0 || ld < P) return 0;
  const int64_t win = qfed_window(ld, P, chain != 0);
  return (P + win - 1) / win;
}

static int launch_qfed1(const float* x, int64_t ld, int32_t K, int64_t P, const float* last, const float* alpha,
                        float lr, int fast, float* delta, float* chain, double* sqnorm, void* workspace,
                        int64_t ws_bytes, int32_t flags, hipStream_t st) {
  QfArgs q{};
  q.x = x; q.ld4 = ld / 4; q.P4 = (P + 3) / 4; q.K = K; q.flags = flags; q.last = last; q.alpha = alpha;
  q.lr = lr; q.rlr = 1.0f / lr; q.delta = delta; q.chain = chain; q.part = (double*)workspace;
  q.fast = fast;
  // WIDE needs QF_G rows plus the sentinel below 2^32; otherwise per-row descriptors over column
  // windows of 2^28 floats (1 GiB), one launch each; the gathers add their partial norms in order.
  const bool wide = (int64_t)ld * 4 * QF_G <= QF_WIDE_BYTES;
  const int qv = chain ? QF_CHAIN_V : QF_V;
  const int64_t win = qfed_window(ld, P, chain != nullptr);
  const int64_t nwin = P > win ? (P + win - 1) / win : 1;
  const int grid = qf_grid(chain != nullptr);
  const int64_t per_win = (int64_t)grid * K;  // doubles of one window's partial rows
  // several windows and room for all their partials: one gather pair at the end (QF_DEFER_GATHER 0: off)
  const bool defer = QF_DEFER_GATHER && nwin > 1 && ws_bytes >= qfed_ws_deferred(K, ld, P, chain != nullptr);
  int64_t wi = 0;
  for (int64_t w0 = 0; w0 < P || w0 == 0; w0 += win, ++wi) {
    QfArgs qw = q;
    if (defer) qw.part = (double*)workspace + wi * per_win;
    const int64_t pw = P - w0 < win ? P - w0 : win;
    qw.x = x + w0; qw.last = last + w0; qw.delta = delta + w0; qw.chain = chain ? chain + w0 : nullptr;
    qw.P4 = (pw + 3) / 4;
    {  // rounds r = tiles per workgroup at full width; then the narrowest tile that still needs r rounds
      const int64_t S = (qw.P4 + 63) / 64;
      const int64_t r = (S + (int64_t)grid * 4 * qv - 1) / ((int64_t)grid * 4 * qv);
      const int64_t strips = r > 0 ? (S + (int64_t)grid * r - 1) / ((int64_t)grid * r) : 1;
      qw.sw = (int)((strips + 3) / 4);
      if (qw.sw < 1) qw.sw = 1;
      if (qw.sw > qv || !QF_BALANCE) qw.sw = qv;
    }
    // chain launches: LDS-DMA prefetch (QF_CHAIN_GLDS slices) on QF_CHAIN_V-wide tiles; the plain kernel:
    // register loads on QF_V-wide tiles
    if (wide && chain)
      hipLaunchKernelGGL((k_qfed_accum<true, true, QF_CHAIN_GLDS, QF_CHAIN_V>), dim3(grid), dim3(256), 0, st, qw);
    else if (wide)
      hipLaunchKernelGGL((k_qfed_accum<true, false, QF_PLAIN_GLDS, QF_V>), dim3(grid), dim3(256), 0, st, qw);
    else if (chain)
      hipLaunchKernelGGL((k_qfed_accum<false, true, QF_CHAIN_GLDS, QF_CHAIN_V>), dim3(grid), dim3(256), 0, st, qw);
    else
      hipLaunchKernelGGL((k_qfed_accum<false, false, QF_PLAIN_GLDS, QF_V>), dim3(grid), dim3(256), 0, st, qw);
    int e = check_launch("fa_qfed_accumulate");
    if (e) return e;
    if (!defer) {
      // the grid's partial rows, summed in a fixed two-level order (16 segments of grid/16 rows)
      double* seg = (double*)workspace + per_win;
      hipLaunchKernelGGL(k_qfed_gather_seg, dim3((K + 255) / 256, QF_GATHER_SEG), dim3(256), 0, st,
                         (const double*)workspace, grid, (int)K, seg);
      hipLaunchKernelGGL(k_qfed_gather, dim3((K + 255) / 256), dim3(256), 0, st, (const double*)seg,
                         (int)QF_GATHER_SEG, (int)K, sqnorm);
      e = check_launch("fa_qfed_accumulate(gather)");
      if (e) return e;
    }
    if (pw >= P - w0) break;
  }
  if (defer) {
    const int64_t nw = wi + 1;  // windows launched
    double* seg = (double*)workspace + nw * per_win;
    hipLaunchKernelGGL(k_qfed_gather_seg_win, dim3((K + 255) / 256, QF_GATHER_SEG, (unsigned)nw), dim3(256), 0, st,
                       (const double*)workspace, grid, (int)K, per_win, seg);
    if (QF_GATHER_WAVE && nw <= QF_GWIN_MAX)
      hipLaunchKernelGGL(k_qfed_gather_win_wave, dim3((K + 3) / 4), dim3(256), 0, st, (const double*)seg, (int)K,
                         (int)nw, sqnorm);
    else
      hipLaunchKernelGGL(k_qfed_gather_win, dim3((K + 255) / 256), dim3(256), 0, st, (const double*)seg, (int)K,
                         (int)nw, sqnorm);
    return check_launch("fa_qfed_accumulate(gather)");
  }
  return FA_OK;
}

#if FA_TUNING
static int launch_qfed2(const float* x, int64_t ld, int32_t K, int64_t P, const float* last, const float* alpha,
                        float lr, int fast, float* delta, float* chain, double* sqnorm, void* workspace,
                        int32_t flags, hipStream_t st) {
  // per-row descriptors: a row's num_records and the voffsets stay below 2^32 for windows of 2^28 floats
  const int64_t win = 1LL << 28;
  for (int64_t w0 = 0; w0 < P || w0 == 0; w0 += win) {
    const int64_t pw = P - w0 < win ? P - w0 : win;
    Qf2Args q{};
    q.x = x + w0; q.ld4 = ld / 4; q.P4 = (pw + 3) / 4; q.K = K; q.flags = flags; q.last = last + w0;
    q.alpha = alpha; q.lr = lr; q.rlr = 1.0f / lr; q.fast = fast; q.delta = delta + w0;
    q.chain = chain ? chain + w0 : nullptr; q.part = (double*)workspace;
    {  // rounds r = tiles per workgroup at full width; then the narrowest tile that still needs r rounds
      const int64_t S = (q.P4 + 63) / 64;
      const int64_t r = (S + (int64_t)QF2_ROWS * QF2_V - 1) / ((int64_t)QF2_ROWS * QF2_V);
      const int64_t strips = r > 0 ? (S + (int64_t)QF2_GRID * r - 1) / ((int64_t)QF2_GRID * r) : 1;
      q.sw = (int)((strips + QF2_WAVES - 1) / QF2_WAVES);
      if (q.sw < 1) q.sw = 1;
      if (q.sw > QF2_V) q.sw = QF2_V;
    }
    if (chain)
      hipLaunchKernelGGL(k_qfed_accum2<true>, dim3(QF2_GRID), dim3(64 * QF2_WAVES), 0, st, q);
    else
      hipLaunchKernelGGL(k_qfed_accum2<false>, dim3(QF2_GRID), dim3(64 * QF2_WAVES), 0, st, q);
    int e = check_launch("fa_qfed_accumulate");
    if (e) return e;
    double* seg = (double*)workspace + (int64_t)QF2_ROWS * K;
    hipLaunchKernelGGL(k_qfed_gather2a, dim3((K + 255) / 256, QF2_SEG), dim3(256), 0, st, (const double*)workspace,
                       (int)K, seg);
    hipLaunchKernelGGL(k_qfed_gather2b, dim3((K + 255) / 256), dim3(256), 0, st, (const double*)seg, (int)K, sqnorm);
    e = check_launch("fa_qfed_accumulate(gather)");
    if (e) return e;
    if (pw >= P - w0) break;
  }
  return FA_OK;
}
#endif  // FA_TUNING

extern "C" int fa_qfed_accumulate(const float* x, int64_t ld, int32_t K, int64_t P, const float* last,
                                  const float* alpha, float lr, float* delta, float* chain, double* sqnorm,
                                  void* workspace, int64_t workspace_bytes, int32_t flags, fa_stream_t stream) {
  if (K <= 0 || K > QF_MAXK) return fail(FA_E_RANGE, "fa_qfed_accumulate: K=%d outside [1, %d]", (int)K, QF_MAXK);
  if (P < 0 || ld < P || ld % 4) return fail(FA_E_ARG, "fa_qfed_accumulate: bad P/ld");
  if (!x || !last || !alpha || !delta || !sqnorm || !workspace)
    return fail(FA_E_ARG, "fa_qfed_accumulate: NULL pointer");
  if (workspace_bytes < qfed_ws_one(K))
    return fail(FA_E_ARG, "fa_qfed_accumulate: workspace of %lld bytes, needs >= %lld (fa_qfed_workspace_bytes)",
                (long long)workspace_bytes, (long long)qfed_ws_one(K));
  if (!aligned16(x) || !aligned16(last) || !aligned16(delta) || !aligned16(chain))
    return fail(FA_E_ARG, "fa_qfed_accumulate: x/last/delta/chain must be 16-byte aligned");
  if (!(lr > 1e-30f && lr < 1e30f)) return fail(FA_E_ARG, "fa_qfed_accumulate: lr=%g outside (1e-30, 1e30)", (double)lr);
  FA_DEVICE_SCOPE("fa_qfed_accumulate", stream, delta);
  FA_OPERAND("x", x, rows_bytes(K, ld, P));
  FA_OPERAND("last", last, cols_bytes(P));
  FA_OPERAND("alpha", alpha, (uint64_t)K * 4);
  FA_OPERAND("delta", delta, cols_bytes(P));
  FA_OPERAND("chain", chain, cols_bytes(P));
  FA_OPERAND("sqnorm", sqnorm, (uint64_t)K * 8);
  FA_OPERAND("workspace", workspace, (uint64_t)workspace_bytes);
  hipStream_t st = (hipStream_t)stream;
  const int fast = (lr >= 9.5367432e-07f && lr <= 1048576.f) ? 1 : 0;  // [2^-20, 2^20]
#if FA_TUNING
  const int kern = chain ? QF_CHAIN_KERNEL : QF_KERNEL;
  if (kern == 2) return launch_qfed2(x, ld, K, P, last, alpha, lr, fast, delta, chain, sqnorm, workspace, flags, st);
#endif
  return launch_qfed1(x, ld, K, P, last, alpha, lr, fast, delta, chain, sqnorm, workspace, workspace_bytes, flags,
                      st);
}

// hs (optimizers.py:96-98) is a sequential fp32 sum in arrival order, so its final add chain stays on one
// thread; everything around it is parallel: all 256 threads form the terms t_k = c1[k]*fp32(sqnorm[k]) +
// c2[k] (two fp32 roundings, no FMA) into LDS, a slab at a time, and thread 0 adds them from LDS (the
// loads no longer sit on the dependent chain: 10,000 clients take tens of µs instead of ~1 ms).
#define HS_SLAB 8192
__global__ __launch_bounds__(256) void k_qfed_hs(const double* sqnorm, const float* c1, const float* c2, int K,
                                                 float* hs_out) {
  __shared__ __attribute__((aligned(16))) float terms[HS_SLAB];
  float hs = 0.f;  // optimizers.py:70  hs = 0.0; the first `0.0 + t` is exact
  for (int k0 = 0; k0 < K; k0 += HS_SLAB) {
    const int n = K - k0 < HS_SLAB ? K - k0 : HS_SLAB;
    for (int i = threadIdx.x; i < n; i += 256) {
      const float sk = (float)sqnorm[k0 + i];               // torch.sum(...) of fp32 -> fp32
      terms[i] = c1[k0 + i] * sk + c2[k0 + i];             // (q*a^(q-1)) * S + (1/lr)*a^q
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      // the adds stay one dependent chain in k order; the LDS reads run one 32-term batch ahead of them, so the
      // chain waits on the adds alone (a read per 4 terms in the loop's critical path cost ~34 cycles per term:
      // 142 us at K = 10,000, profiles/r05_prof_all_by_shape.jsonl)
      int i = 0;
      if (n >= 32) {
        float4 cur[8], nxt[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) cur[j] = *reinterpret_cast<const float4*>(terms + 4 * j);
        for (; i + 64 <= n; i += 32) {
#pragma unroll
          for (int j = 0; j < 8; ++j) nxt[j] = *reinterpret_cast<const float4*>(terms + i + 32 + 4 * j);
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            hs = hs + cur[j].x;
            hs = hs + cur[j].y;
            hs = hs + cur[j].z;
            hs = hs + cur[j].w;
            cur[j] = nxt[j];
          }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          hs = hs + cur[j].x;
          hs = hs + cur[j].y;
          hs = hs + cur[j].z;
          hs = hs + cur[j].w;
        }
        i += 32;
      }
      for (; i < n; ++i) hs = hs + terms[i];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    hs_out[0] = hs;
    hs_out[1] = hs + 1e-10f;  // optimizers.py:102 (hs + 1e-10)
  }
}

extern "C" int fa_qfed_hs(const double* sqnorm, const float* c1, const float* c2, int32_t K, float* hs_out,
                          fa_stream_t stream) {
  if (K < 0 || !sqnorm || !c1 || !c2 || !hs_out) return fail(FA_E_ARG, "fa_qfed_hs: bad arguments");
  FA_DEVICE_SCOPE("fa_qfed_hs", stream, hs_out);
  FA_OPERAND("sqnorm", sqnorm, (uint64_t)K * 8);
  FA_OPERAND("c1", c1, (uint64_t)K * 4);
  FA_OPERAND("c2", c2, (uint64_t)K * 4);
  FA_OPERAND("hs_out", hs_out, 8);
  hipLaunchKernelGGL(k_qfed_hs, dim3(1), dim3(256), 0, (hipStream_t)stream, sqnorm, c1, c2, (int)K, hs_out);
  return check_launch("fa_qfed_hs");
}

__global__ __launch_bounds__(256) void k_qfed_finalize(const f4* __restrict__ last, const f4* __restrict__ delta,
                                                       const float* __restrict__ hs, f4* out, int64_t P4) {
  const float d = hs[1];
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < P4; i += (int64_t)gridDim.x * 256) {
    const f4 L = last[i], D = delta[i];
    f4 o;
    o.x = L.x - __fdiv_rn(D.x, d);
    o.y = L.y - __fdiv_rn(D.y, d);
    o.z = L.z - __fdiv_rn(D.z, d);
    o.w = L.w - __fdiv_rn(D.w, d);
    out[i] = o;
  }
}

extern "C" int fa_qfed_finalize(const float* last, const float* delta, const float* hs_dev, float* out, int64_t P,
                                fa_stream_t stream) {
  if (P < 0 || !last || !delta || !hs_dev || !out) return fail(FA_E_ARG, "fa_qfed_finalize: bad arguments");
  if (!aligned16(last) || !aligned16(delta) || !aligned16(out))
    return fail(FA_E_ARG, "fa_qfed_finalize: pointers must be 16-byte aligned");
  if (P == 0) return FA_OK;
  FA_DEVICE_SCOPE("fa_qfed_finalize", stream, out);
  FA_OPERAND("last", last, cols_bytes(P));
  FA_OPERAND("delta", delta, cols_bytes(P));
  FA_OPERAND("hs_dev", hs_dev, 8);
  FA_OPERAND("out", out, cols_bytes(P));
  const int64_t P4 = (P + 3) / 4;
  hipLaunchKernelGGL(k_qfed_finalize, dim3(stride_grid(P4)), dim3(256), 0, (hipStream_t)stream,
                     (const f4*)last, (const f4*)delta, hs_dev, (f4*)out, P4);
  return check_launch("fa_qfed_finalize");
}

// fixed-order sum of per-shard fp64 rows (after an all-gather of the shards' partial norms)
__global__ __launch_bounds__(256) void k_sum_rows_f64(const double* x, int64_t ld, int n, int64_t K,
                                                     double* out) {
  for (int64_t k = (int64_t)blockIdx.x * 256 + threadIdx.x; k < K; k += (int64_t)gridDim.x * 256) {
    double s = x[k];
    for (int r = 1; r < n; ++r) s += x[(int64_t)r * ld + k];
    out[k] = s;
  }
}

extern "C" int fa_sum_rows_f64(const double* x, int64_t ld, int32_t n, int64_t K, double* out, fa_stream_t stream) {
  if (n < 1 || K < 0 || ld < K || !x || !out) return fail(FA_E_ARG, "fa_sum_rows_f64: bad arguments");
  if (K == 0) return FA_OK;
  FA_DEVICE_SCOPE("fa_sum_rows_f64", stream, out);
  FA_OPERAND("x", x, (uint64_t)((n - 1) * ld + K) * 8);
  FA_OPERAND("out", out, (uint64_t)K * 8);
  hipLaunchKernelGGL(k_sum_rows_f64, dim3(stride_grid(K)), dim3(256), 0, (hipStream_t)stream, x, ld, (int)n, K, out);
  return check_launch("fa_sum_rows_f64");
}

// ------------------------------------------------------------------------------------------------
// side table (int64 state_dict entries): one thread per element, clients in arrival order
// ------------------------------------------------------------------------------------------------
__global__ void k_side_accum(const int64_t* xi, int ldq, int K, int Q, int mode, const double* w, int64_t* acc_i,
                             double* acc_d, int accumulate) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Q) return;
  if (mode == 0) {
    int64_t s = accumulate ? acc_i[q] : xi[q];
    for (int k = accumulate ? 0 : 1; k < K; ++k)
      s = (int64_t)((uint64_t)s + (uint64_t)xi[(int64_t)k * ldq + q]);  // numpy int64 add wraps
    acc_i[q] = s;
  } else {
    double s = accumulate ? acc_d[q] : (double)xi[q] * w[0];
    for (int k = accumulate ? 0 : 1; k < K; ++k) s = s + w[k] * (double)xi[(int64_t)k * ldq + q];
    acc_d[q] = s;
  }
}

extern "C" int fa_side_accumulate(const int64_t* xi, int32_t ldq, int32_t K, int32_t Q, int32_t mode,
                                  const double* w, int64_t* acc_i, double* acc_d, int32_t flags,
                                  fa_stream_t stream) {
  if (Q == 0) return FA_OK;
  if (Q < 0 || K < 0 || ldq < Q || (K > 0 && !xi)) return fail(FA_E_ARG, "fa_side_accumulate: bad sizes");
  if (mode == 0 && !acc_i) return fail(FA_E_ARG, "fa_side_accumulate: acc_i NULL");
  if (mode == 1 && (!acc_d || !w)) return fail(FA_E_ARG, "fa_side_accumulate: acc_d/w NULL");
  if (mode != 0 && mode != 1) return fail(FA_E_ARG, "fa_side_accumulate: mode %d", (int)mode);
  if (K == 0) return FA_OK;
  FA_DEVICE_SCOPE("fa_side_accumulate", stream, mode == 0 ? (const void*)acc_i : (const void*)acc_d);
  FA_HOST_OK_OPERAND("xi", xi, (uint64_t)((int64_t)(K - 1) * ldq + Q) * 8);  // device, or the pinned mirror
  FA_OPERAND("w", mode == 1 ? w : nullptr, (uint64_t)K * 8);
  FA_OPERAND(mode == 0 ? "acc_i" : "acc_d", mode == 0 ? (const void*)acc_i : (const void*)acc_d, (uint64_t)Q * 8);
  hipLaunchKernelGGL(k_side_accum, dim3((Q + 63) / 64), dim3(64), 0, (hipStream_t)stream, xi, ldq, K, Q, mode, w,
                     acc_i, acc_d, (flags & FA_ACCUMULATE) ? 1 : 0);
  return check_launch("fa_side_accumulate");
}

__global__ void k_side_close(const int64_t* acc_i, const double* acc_d, int Q, int mode, double denom, double* cur,
                             int64_t* model) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Q) return;
  const double c = (mode == 0 ? (double)acc_i[q] : acc_d[q]) / denom;
  if (cur) cur[q] = c;
  if (model) model[q] = (int64_t)(float)c;  // np.asarray(float32) then float32 -> int64 copy (truncation)
}

extern "C" int fa_side_close(const int64_t* acc_i, const double* acc_d, int32_t Q, int32_t mode, double denom,
                             double* cur, int64_t* model, fa_stream_t stream) {
  if (Q == 0) return FA_OK;
  if (Q < 0 || (mode == 0 && !acc_i) || (mode == 1 && !acc_d)) return fail(FA_E_ARG, "fa_side_close: bad args");
  FA_DEVICE_SCOPE("fa_side_close", stream, mode == 0 ? (const void*)acc_i : (const void*)acc_d);
  FA_OPERAND(mode == 0 ? "acc_i" : "acc_d", mode == 0 ? (const void*)acc_i : (const void*)acc_d, (uint64_t)Q * 8);
  FA_OPERAND("cur", cur, (uint64_t)Q * 8);
  FA_OPERAND("model", model, (uint64_t)Q * 8);
  hipLaunchKernelGGL(k_side_close, dim3((Q + 63) / 64), dim3(64), 0, (hipStream_t)stream, acc_i, acc_d, Q, mode,
                     denom, cur, model);
  return check_launch("fa_side_close");
}

__global__ void k_side_yogi(const double* cur, const int64_t* last, double* m, double* v, double* step,
                            int64_t* model, int Q, double eta, double tau, double beta, double omb, double omb2,
                            int init) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Q) return;
  const double L = last ? (double)last[q] : 0.0;
  const double g = cur[q] - L;
  const double g2 = g * g;
  double M = init ? 0.0 : m[q];
  double Vv = init ? tau : v[q];
  M = beta * M + omb * g;
  Vv = Vv - (omb2 * g2) * sgnd(Vv - g2);
  const double lr = __drcp_rn(__builtin_sqrt(Vv) + tau) * eta;
  const double st = lr * M;
  m[q] = M;
  v[q] = Vv;
  if (step) step[q] = st;
  if (model) model[q] = (int64_t)(float)(L + st);  // np.array(last + diff, float32) -> load_state_dict
}

extern "C" int fa_side_yogi(const double* cur, const int64_t* last, double* m, double* v, double* step,
                            int64_t* model, int32_t Q, double eta, double tau, double beta, double omb, double omb2,
                            int32_t flags, fa_stream_t stream) {
  if (Q == 0) return FA_OK;
  if (Q < 0 || !cur || !m || !v) return fail(FA_E_ARG, "fa_side_yogi: bad args");
  FA_DEVICE_SCOPE("fa_side_yogi", stream, m);
  FA_OPERAND("cur", cur, (uint64_t)Q * 8);
  FA_OPERAND("last", last, (uint64_t)Q * 8);
  FA_OPERAND("m", m, (uint64_t)Q * 8);
  FA_OPERAND("v", v, (uint64_t)Q * 8);
  FA_OPERAND("step", step, (uint64_t)Q * 8);
  FA_OPERAND("model", model, (uint64_t)Q * 8);
  hipLaunchKernelGGL(k_side_yogi, dim3((Q + 63) / 64), dim3(64), 0, (hipStream_t)stream, cur, last, m, v, step,
                     model, Q, eta, tau, beta, omb, omb2, (flags & FA_YOGI_INIT) ? 1 : 0);
  return check_launch("fa_side_yogi");
}

// q-FedAvg side: (a) one thread per element walks the clients (delta chain);
//                (b) one thread per client walks the elements (sum of g^2 in element order).
__device__ __forceinline__ float side_g(int64_t L, int64_t W, float lr) {
  // (u - v) int64, then "* 1.0" promotes to fp32 (int64 -> fp32 conversion, times 1.0f), then / lr
  return __fdiv_rn((float)(int64_t)((uint64_t)L - (uint64_t)W) * 1.0f, lr);
}

__global__ void k_side_qfed_delta(const int64_t* xi, int ldq, int K, int Q, const int64_t* last, const float* alpha,
                                  float lr, float* delta_s, int accumulate) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Q) return;
  float d = accumulate ? delta_s[q] : 0.f;
  for (int k = 0; k < K; ++k) {
    const float t = alpha[k] * side_g(last[q], xi[(int64_t)k * ldq + q], lr);
    d = (k == 0 && !accumulate) ? t : d + t;
  }
  delta_s[q] = d;
}

__global__ void k_side_qfed_sq(const int64_t* xi, int ldq, int K, int Q, const int64_t* last, float lr,
                               double* sqnorm) {
  const int k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= K) return;
  double s = 0.0;
  for (int q = 0; q < Q; ++q) {
    const float g = side_g(last[q], xi[(int64_t)k * ldq + q], lr);
    s += (double)(g * g);
  }
  sqnorm[k] += s;
}

extern "C" int fa_side_qfed_accumulate(const int64_t* xi, int32_t ldq, int32_t K, int32_t Q, const int64_t* last,
                                       const float* alpha, float lr, float* delta_s, double* sqnorm, int32_t flags,
                                       fa_stream_t stream) {
  if (Q == 0 || K == 0) return FA_OK;
  if (Q < 0 || K < 0 || ldq < Q || !xi || !last || !alpha || !delta_s || !sqnorm)
    return fail(FA_E_ARG, "fa_side_qfed_accumulate: bad args");
  FA_DEVICE_SCOPE("fa_side_qfed_accumulate", stream, delta_s);
  FA_OPERAND("xi", xi, (uint64_t)((int64_t)(K - 1) * ldq + Q) * 8);
  FA_OPERAND("last", last, (uint64_t)Q * 8);
  FA_OPERAND("alpha", alpha, (uint64_t)K * 4);
  FA_OPERAND("delta_s", delta_s, (uint64_t)Q * 4);
  FA_OPERAND("sqnorm", sqnorm, (uint64_t)K * 8);
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_side_qfed_delta, dim3((Q + 63) / 64), dim3(64), 0, st, xi, ldq, K, Q, last, alpha, lr, delta_s,
                     (flags & FA_ACCUMULATE) ? 1 : 0);
  int e = check_launch("fa_side_qfed_accumulate(delta)");
  if (e) return e;
  hipLaunchKernelGGL(k_side_qfed_sq, dim3((K + 63) / 64), dim3(64), 0, st, xi, ldq, K, Q, last, lr, sqnorm);
  return check_launch("fa_side_qfed_accumulate(sq)");
}

__global__ void k_side_qfed_finalize(const int64_t* last, const float* delta_s, const float* hs, int64_t* model,
                                     int Q) {
  const int q = blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Q) return;
  model[q] = (int64_t)((float)last[q] - __fdiv_rn(delta_s[q], hs[1]));
}

extern "C" int fa_side_qfed_finalize(const int64_t* last, const float* delta_s, const float* hs_dev, int64_t* model,
                                     int32_t Q, fa_stream_t stream) {
  if (Q == 0) return FA_OK;
  if (Q < 0 || !last || !delta_s || !hs_dev || !model) return fail(FA_E_ARG, "fa_side_qfed_finalize: bad args");
  FA_DEVICE_SCOPE("fa_side_qfed_finalize", stream, model);
  FA_OPERAND("last", last, (uint64_t)Q * 8);
  FA_OPERAND("delta_s", delta_s, (uint64_t)Q * 4);
  FA_OPERAND("hs_dev", hs_dev, 8);
  FA_OPERAND("model", model, (uint64_t)Q * 8);
  hipLaunchKernelGGL(k_side_qfed_finalize, dim3((Q + 63) / 64), dim3(64), 0, (hipStream_t)stream, last, delta_s,
                     hs_dev, model, Q);
  return check_launch("fa_side_qfed_finalize");
}

// ------------------------------------------------------------------------------------------------
// deterministic synthetic updates (bit-reproducible on the host: fedscale_amd/synth.py)
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
__device__ __forceinline__ float tri(uint32_t stream, int64_t p) {
  const uint32_t h = mix32(mix32((uint32_t)p + mix32(stream)) ^ (uint32_t)((uint64_t)p >> 32));
  const int32_t u1 = (int32_t)(h >> 8), u2 = (int32_t)(mix32(h) >> 8);
  return (float)(u1 + u2 - (1 << 24)) * 5.9604644775390625e-08f;  // exact: |n| <= 2^24, times 2^-24
}

__global__ __launch_bounds__(256) void k_fill(float* x, int64_t ld, int K, int64_t P, uint32_t seed, int k0,
                                              float sb, float sn) {
  const int k = blockIdx.y;
  float* row = x + (int64_t)k * ld;
  for (int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x; p < ld; p += (int64_t)gridDim.x * 256) {
    float val = 0.f;
    if (p < P) {
      const float b = tri(seed, p) * sb;
      const float n = tri(seed + 1u + (uint32_t)(k0 + k), p) * sn;
      val = b + n;
    }
    row[p] = val;
  }
}

extern "C" int fa_fill_synthetic(float* x, int64_t ld, int32_t K, int64_t P, uint32_t seed, int32_t k0,
                                 float scale_base, float scale_noise, fa_stream_t stream) {
  if (K < 0 || P < 0 || ld < P || !x) return fail(FA_E_ARG, "fa_fill_synthetic: bad args");
  if (K == 0 || ld == 0) return FA_OK;
  if (K > 65535) return fail(FA_E_RANGE, "fa_fill_synthetic: K=%d > 65535 per call", (int)K);
  FA_DEVICE_SCOPE("fa_fill_synthetic", stream, x);
  FA_OPERAND("x", x, (uint64_t)K * ld * 4);
  int64_t gx = (ld + 255) / 256;
  if (gx > 2048) gx = 2048;
  hipLaunchKernelGGL(k_fill, dim3((unsigned)gx, (unsigned)K), dim3(256), 0, (hipStream_t)stream, x, ld, K, P, seed, k0,
                     scale_base, scale_noise);
  return check_launch("fa_fill_synthetic");
}

// ------------------------------------------------------------------------------------------------
// HeteroFL sub-model combination (examples/heterofl/customized_aggregator.py:78-119)
// ------------------------------------------------------------------------------------------------
// A client at model rate r uploads, for every tensor of shape (O, I, S...), the prefix box
// [0:o) x [0:i) x S (examples/heterofl/customized_fllibs.py:25-70 only ever builds prefix index sets).
// Per global element, the reference sums the covering clients' values in client order into an fp32
// zero, counts them, and replaces the element by sum / count where count > 0.
//
// desc[(m*T + k)*4 + {0,1,2,3}] = {offset of client m's box of tensor k in xs, o_m, L_m = i_m*S, ld_m}:
// the box is o_m rows of L_m elements at row stride ld_m.  A chunk is (tensor k, row o, first column r0)
// in ROW mode: o is uniform, so "client m covers this row" is a scalar branch; the host pads every box
// row to ld_m = round_up(L_m, 4) with a 16-byte aligned offset, so each thread takes 4 consecutive
// columns with ONE dwordx4 load per client (the padding is read, never counted).  ELEMENT mode (k, -1,
// first element) serves tensors with short rows (1-D BatchNorm vectors ...) one element per thread.
#define HB_ELEMS 1024
#ifndef HB_U
#define HB_U 8
#endif  // HB_U: clients whose loads are issued before their (in-order) adds
#ifndef HB_NT
#define HB_NT 1
#endif  // HB_NT: non-temporal box loads (every upload element is read exactly once)
__device__ __forceinline__ f4 hb_load(const float* p) {
#if HB_NT
  return __builtin_nontemporal_load((const f4*)p);
#else
  return *(const f4*)p;
#endif
}

__device__ __forceinline__ void hb_add(float& acc, int& cnt, float v, bool hit) {
  if (hit) {
    acc = acc + v;  // tmp_v[idx] += local_parameters[k], clients in order
    ++cnt;          // count[k][idx] += 1
  }
}

// FLAT mode (rows of RL % 4 == 0 elements, boxes padded to 16-byte rows): the workgroup owns HB_FLAT_J x
// 1024 consecutive elements of the flattened tensor; thread t takes the float4 groups at
// c0 + j*1024 + 4t, j < HB_FLAT_J (a group never straddles a row).  A full-rate client's box rows are
// contiguous in its upload, so each client contributes HB_FLAT_J x 4 KiB of contiguous reads per
// workgroup — longer runs per DRAM page than ROW mode's one row segment.
#ifndef HB_FLAT_J
#define HB_FLAT_J 8
#endif
#ifndef HB_FLAT_U
#define HB_FLAT_U 1
#endif
#ifndef HB_DPREFETCH
#define HB_DPREFETCH 0  // 1: measured 2 % slower (profiles/r02_tune_heterofl_dprefetch.log)
#endif
__device__ __forceinline__ void prefix_box_flat(const float* __restrict__ xs, const int64_t* __restrict__ dk,
                                                int64_t dstride, int K, int64_t goff, int64_t RL, int64_t n,
                                                int64_t c0, float* glob) {
  int64_t o[HB_FLAT_J], r[HB_FLAT_J];
  bool in[HB_FLAT_J];
#pragma unroll
  for (int j = 0; j < HB_FLAT_J; ++j) {
    const int64_t e = c0 + j * 1024 + 4 * (int64_t)threadIdx.x;
    in[j] = e < n;
    o[j] = e / RL;
    r[j] = e - o[j] * RL;
  }
  float acc[HB_FLAT_J][4];
  int cnt[HB_FLAT_J][4];
#pragma unroll
  for (int j = 0; j < HB_FLAT_J; ++j)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[j][i] = 0.f;  // tmp_v = v.new_zeros(..., dtype=torch.float32)
      cnt[j][i] = 0;
    }
  // the clients' box descriptors are scalar loads; HB_DPREFETCH requests the next group's while this
  // group's vector loads are in flight
  int64_t dsc[HB_FLAT_U][4];
  auto desc_of = [&](int m, int64_t(&v)[4]) {
    const bool mv = m < K;
    const int64_t* d = dk + (int64_t)(mv ? m : 0) * dstride;
    v[0] = d[0], v[1] = mv ? d[1] : 0, v[2] = d[2], v[3] = d[3];
  };
#pragma unroll
  for (int u = 0; u < HB_FLAT_U; ++u) desc_of(u, dsc[u]);
  for (int m0 = 0; m0 < K; m0 += HB_FLAT_U) {
    f4 t[HB_FLAT_U][HB_FLAT_J];
    int64_t len[HB_FLAT_U][HB_FLAT_J];
#pragma unroll
    for (int u = 0; u < HB_FLAT_U; ++u) {
#if !HB_DPREFETCH
      desc_of(m0 + u, dsc[u]);
#endif
      const int64_t off = dsc[u][0], om = dsc[u][1], Lm = dsc[u][2], ldm = dsc[u][3];
#pragma unroll
      for (int j = 0; j < HB_FLAT_J; ++j) {
        len[u][j] = (in[j] && o[j] < om) ? Lm : 0;  // covered columns of this row: [0, L_m)
        t[u][j] = r[j] < len[u][j] ? hb_load(xs + off + o[j] * ldm + r[j]) : f4{0.f, 0.f, 0.f, 0.f};
      }
    }
#if HB_DPREFETCH
#pragma unroll
    for (int u = 0; u < HB_FLAT_U; ++u) desc_of(m0 + HB_FLAT_U + u, dsc[u]);
#endif
#pragma unroll
    for (int u = 0; u < HB_FLAT_U; ++u)
#pragma unroll
      for (int j = 0; j < HB_FLAT_J; ++j) {
        hb_add(acc[j][0], cnt[j][0], t[u][j].x, r[j] < len[u][j]);
        hb_add(acc[j][1], cnt[j][1], t[u][j].y, r[j] + 1 < len[u][j]);
        hb_add(acc[j][2], cnt[j][2], t[u][j].z, r[j] + 2 < len[u][j]);
        hb_add(acc[j][3], cnt[j][3], t[u][j].w, r[j] + 3 < len[u][j]);
      }
  }
#pragma unroll
  for (int j = 0; j < HB_FLAT_J; ++j) {
    if (!in[j]) continue;
    float* g = glob + goff + o[j] * RL + r[j];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (cnt[j][i] > 0) g[i] = __fdiv_rn(acc[j][i], (float)cnt[j][i]);  // tmp_v[count>0].div_(count[..])
  }
}

__device__ __forceinline__ void prefix_box_chunk(const float* __restrict__ xs, const int64_t* __restrict__ desc,
                                                 int K, int T, const int64_t* __restrict__ tens,
                                                 const int32_t* __restrict__ ck_t,
                                                 const int64_t* __restrict__ ck_first, float* glob, int c) {
  const int k = ck_t[2 * c];
  const int row = ck_t[2 * c + 1];
  const int64_t goff = tens[4 * k];
  const int64_t RL = tens[4 * k + 2] * tens[4 * k + 3];  // global row length I*S
  const int64_t* dk = desc + 4 * (int64_t)k;
  const int64_t dstride = 4 * (int64_t)T;
  if (row == -2) {  // FLAT mode: HB_FLAT_J x 1024 consecutive elements, rows a multiple of 4 long
    prefix_box_flat(xs, dk, dstride, K, goff, RL, tens[4 * k + 1] * RL, ck_first[c], glob);
    return;
  }
  if (row >= 0) {
    const int64_t o = row;
    const int64_t r = ck_first[c] + 4 * (int64_t)threadIdx.x;  // 4 columns per thread, 16-byte aligned
    if (r >= RL) return;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};  // tmp_v = v.new_zeros(..., dtype=torch.float32)
    int cnt[4] = {0, 0, 0, 0};
    int m = 0;
    for (; m + HB_U <= K; m += HB_U) {
      f4 t[HB_U];
      int64_t len[HB_U];
#pragma unroll
      for (int u = 0; u < HB_U; ++u) {
        const int64_t* d = dk + (int64_t)(m + u) * dstride;
        len[u] = o < d[1] ? d[2] : 0;  // row covered (scalar) -> its covered columns are [0, L_m)
        t[u] = r < len[u] ? hb_load(xs + d[0] + o * d[3] + r) : f4{0.f, 0.f, 0.f, 0.f};
      }
#pragma unroll
      for (int u = 0; u < HB_U; ++u) {
        hb_add(acc[0], cnt[0], t[u].x, r < len[u]);
        hb_add(acc[1], cnt[1], t[u].y, r + 1 < len[u]);
        hb_add(acc[2], cnt[2], t[u].z, r + 2 < len[u]);
        hb_add(acc[3], cnt[3], t[u].w, r + 3 < len[u]);
      }
    }
    for (; m < K; ++m) {
      const int64_t* d = dk + (int64_t)m * dstride;
      const int64_t len = o < d[1] ? d[2] : 0;
      if (r < len) {
        const f4 v = hb_load(xs + d[0] + o * d[3] + r);
        hb_add(acc[0], cnt[0], v.x, true);
        hb_add(acc[1], cnt[1], v.y, r + 1 < len);
        hb_add(acc[2], cnt[2], v.z, r + 2 < len);
        hb_add(acc[3], cnt[3], v.w, r + 3 < len);
      }
    }
    float* g = glob + goff + o * RL + r;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (r + j < RL && cnt[j] > 0) g[j] = __fdiv_rn(acc[j], (float)cnt[j]);  // tmp_v[count>0].div_(count[..])
    return;
  }
  const int64_t n = tens[4 * k + 1] * RL;
  for (int j = 0; j < HB_ELEMS / 256; ++j) {
    const int64_t e = ck_first[c] + j * 256 + threadIdx.x;
    if (e >= n) break;
    const int64_t o = e / RL, r = e - o * RL;
    float acc = 0.f;
    int cnt = 0;
    int m = 0;
    for (; m + HB_U <= K; m += HB_U) {
      float t[HB_U];
      bool hit[HB_U];
#pragma unroll
      for (int u = 0; u < HB_U; ++u) {
        const int64_t* d = dk + (int64_t)(m + u) * dstride;
        hit[u] = o < d[1] && r < d[2];
        t[u] = hit[u] ? xs[d[0] + o * d[3] + r] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < HB_U; ++u) hb_add(acc, cnt, t[u], hit[u]);
    }
    for (; m < K; ++m) {
      const int64_t* d = dk + (int64_t)m * dstride;
      if (o < d[1] && r < d[2]) hb_add(acc, cnt, xs[d[0] + o * d[3] + r], true);
    }
    if (cnt > 0) glob[goff + o * RL + r] = __fdiv_rn(acc, (float)cnt);
  }
}

// HB_GRID > 0 caps the grid; workgroup b then takes chunks b, b + grid, ... (fewer concurrent streams)
#ifndef HB_GRID
#define HB_GRID 0
#endif
__global__ __launch_bounds__(256) void k_prefix_box(const float* __restrict__ xs, const int64_t* __restrict__ desc,
                                                    int K, int T, const int64_t* __restrict__ tens,
                                                    const int32_t* __restrict__ ck_t,
                                                    const int64_t* __restrict__ ck_first, float* glob, int nchunks) {
  for (int c = blockIdx.x; c < nchunks; c += gridDim.x) prefix_box_chunk(xs, desc, K, T, tens, ck_t, ck_first, glob, c);
}

extern "C" int fa_prefix_box_combine(const float* xs, const int64_t* desc, int32_t K, const int64_t* tensors,
                                     int32_t T, const int32_t* chunk_tensor, const int64_t* chunk_first,
                                     int32_t nchunks, float* global, fa_stream_t stream) {
  if (K < 0 || T < 0 || nchunks < 0) return fail(FA_E_ARG, "fa_prefix_box_combine: negative sizes");
  if (nchunks == 0 || K == 0) return FA_OK;
  if (!xs || !desc || !tensors || !chunk_tensor || !chunk_first || !global)
    return fail(FA_E_ARG, "fa_prefix_box_combine: NULL pointer");
  if (!aligned16(xs)) return fail(FA_E_ARG, "fa_prefix_box_combine: xs must be 16-byte aligned");
  FA_DEVICE_SCOPE("fa_prefix_box_combine", stream, xs);
  // (the boxes' extents live in desc on the device: xs and global are checked at their base)
  FA_OPERAND("xs", xs, 16);
  FA_OPERAND("desc", desc, (uint64_t)K * T * 4 * 8);
  FA_OPERAND("tensors", tensors, (uint64_t)T * 4 * 8);
  FA_OPERAND("chunk_tensor", chunk_tensor, (uint64_t)nchunks * 2 * 4);
  FA_OPERAND("chunk_first", chunk_first, (uint64_t)nchunks * 8);
  FA_OPERAND("global", global, 4);
  const int grid = (HB_GRID > 0 && nchunks > HB_GRID) ? HB_GRID : nchunks;
  hipLaunchKernelGGL(k_prefix_box, dim3(grid), dim3(256), 0, (hipStream_t)stream, xs, desc, (int)K, (int)T, tensors,
                     chunk_tensor, chunk_first, global, (int)nchunks);
  return check_launch("fa_prefix_box_combine");
}

// ------------------------------------------------------------------------------------------------
// host ingress: multi-threaded gather of a client update's tensors into a pinned staging row
// ------------------------------------------------------------------------------------------------
// One call per arriving update (the reference's dict of numpy arrays, torch_client.py:76-78): the byte
// ranges are cut into equal shares, one per worker of a persistent pool, so the copy into pinned memory
// runs at several cores' memory bandwidth instead of one (a single memcpy stream is ~29 GB/s on the
// MI355X host, below the ~55 GB/s the H2D copy engine sustains).
namespace {
struct GatherPool {
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv, done_cv;
  std::function<void(int)> job;
  int gen = 0, pending = 0, nthreads = 0;
  bool stop = false;
  explicit GatherPool(int n) : nthreads(n) {
    for (int i = 0; i < n; ++i)
      th.emplace_back([this, i] {
        int seen = 0;
        for (;;) {
          std::function<void(int)> f;
          {
            std::unique_lock<std::mutex> lk(mu);
            cv.wait(lk, [&] { return stop || gen != seen; });
            if (stop) return;
            seen = gen;
            f = job;
          }
          f(i);
          std::lock_guard<std::mutex> lk(mu);
          if (--pending == 0) done_cv.notify_all();
        }
      });
  }
  ~GatherPool() {
    {
      std::lock_guard<std::mutex> lk(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
  void run(std::function<void(int)> f) {
    std::unique_lock<std::mutex> lk(mu);
    job = std::move(f);
    pending = nthreads;
    ++gen;
    cv.notify_all();
    done_cv.wait(lk, [&] { return pending == 0; });
  }
};
std::mutex g_pool_mu;
GatherPool* g_pool = nullptr;
pid_t g_pool_pid = 0;  // a forked child inherits the pointer but not the threads: rebuild there

// Pieces of >= 64 KiB are written with non-temporal (streaming) stores: the pinned row is read next by
// the H2D copy engine, not by this core, and a cached store first reads the line it overwrites
// (read-for-ownership), so a plain memcpy moves 3 bytes of host DRAM traffic per byte copied where this
// moves 2.  Source loads stay cached (they are read once either way).  FEDAGG_GATHER_NT=0 turns it off.
bool gather_nt() {
  static const bool on = [] {
    const char* e = getenv("FEDAGG_GATHER_NT");
    return !(e && e[0] == '0');
  }();
  return on;
}
void copy_piece(char* d, const char* s, size_t n) {
  if (n < (64u << 10) || !gather_nt()) {
    memcpy(d, s, n);
    return;
  }
  typedef float v4 __attribute__((ext_vector_type(4)));
  const size_t head = (64 - ((uintptr_t)d & 63)) & 63;  // align the destination to a cache line
  memcpy(d, s, head);
  d += head, s += head, n -= head;
  const size_t lines = n / 64;
  for (size_t i = 0; i < lines; ++i, d += 64, s += 64) {
    v4 a, b, c, e;
    memcpy(&a, s, 16), memcpy(&b, s + 16, 16), memcpy(&c, s + 32, 16), memcpy(&e, s + 48, 16);
    __builtin_nontemporal_store(a, reinterpret_cast<v4*>(d));
    __builtin_nontemporal_store(b, reinterpret_cast<v4*>(d + 16));
    __builtin_nontemporal_store(c, reinterpret_cast<v4*>(d + 32));
    __builtin_nontemporal_store(e, reinterpret_cast<v4*>(d + 48));
  }
  memcpy(d, s, n - lines * 64);
}
}  // namespace

extern "C" int fa_host_gather(void* dst, const void* const* srcs, const int64_t* dst_off, const int64_t* nbytes,
                              int32_t n, int32_t threads) {
  if (n < 0 || (n > 0 && (!dst || !srcs || !dst_off || !nbytes))) return fail(FA_E_ARG, "fa_host_gather: bad args");
  int64_t total = 0;
  for (int i = 0; i < n; ++i) {
    if (nbytes[i] < 0 || dst_off[i] < 0 || (nbytes[i] > 0 && !srcs[i])) return fail(FA_E_ARG, "fa_host_gather: piece %d", i);
    total += nbytes[i];
  }
  char* d = static_cast<char*>(dst);
  if (threads <= 1 || total < (4 << 20)) {
    for (int i = 0; i < n; ++i) copy_piece(d + dst_off[i], static_cast<const char*>(srcs[i]), (size_t)nbytes[i]);
    std::atomic_thread_fence(std::memory_order_seq_cst);
    return FA_OK;
  }
  if (threads > 64) threads = 64;
  std::lock_guard<std::mutex> serial(g_pool_mu);  // one gather at a time through the shared pool
  try {
    if (g_pool && g_pool_pid != getpid()) g_pool = nullptr;  // inherited across fork(): leak, do not join
    if (!g_pool || g_pool->nthreads != threads) {
      delete g_pool;
      g_pool = new GatherPool(threads);
      g_pool_pid = getpid();
    }
  } catch (...) {  // no exception crosses the C ABI: fall back to one thread
    g_pool = nullptr;
    for (int i = 0; i < n; ++i) memcpy(d + dst_off[i], srcs[i], (size_t)nbytes[i]);
    return FA_OK;
  }
  const int64_t share = (total + threads - 1) / threads;
  g_pool->run([&](int w) {
    const int64_t lo = (int64_t)w * share, hi = lo + share < total ? lo + share : total;
    int64_t pos = 0;
    for (int i = 0; i < n && pos < hi; ++i) {
      const int64_t a = pos, b = pos + nbytes[i];
      pos = b;
      const int64_t s0 = a > lo ? a : lo, s1 = b < hi ? b : hi;
      if (s0 < s1) copy_piece(d + dst_off[i] + (s0 - a), static_cast<const char*>(srcs[i]) + (s0 - a), (size_t)(s1 - s0));
    }
    // order the streaming stores before the pool reports done (the caller's H2D reads the row next)
    std::atomic_thread_fence(std::memory_order_seq_cst);
  });
  return FA_OK;
}
