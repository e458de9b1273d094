// client_update.hip — MI355X (gfx950) kernels for the client-side element-wise weight handlers of
// FedScale, run when an executor trains on the GPU:
//   * FedProx proximal step, fedscale/cloud/execution/optimizers.py:6-10, called after every local
//     optimizer step (torch_client.py:238-240):  p += lr*mu * (p - global);
//   * local differential privacy, examples/differential_privacy/customized_client.py:51-65 with
//     clip_norm.py:12-52:  delta = p - last; clip delta to max_norm by its global 2-norm (or inf-norm);
//     p = last + delta; upload = state_dict + N(0, sigma).
//
// A model is a list of T separately allocated tensors, so every kernel is a multi-tensor launch: the
// tensor table (pointers, sizes, per-tensor first workgroup) travels in the kernel arguments, up to
// MT_MAX tensors per launch, and a workgroup owns MT_CHUNK contiguous elements of one tensor.  One launch
// replaces T per-tensor torch ops; all of it is HBM streaming (12-16 B per element), no MFMA.
//
// Numerics: every fp32 op is rounded as the reference's torch CPU op is (no FMA), so FedProx is
// bit-exact.  The DP norm accumulates squares in fp64 in a fixed order (the reference's torch.norm
// accumulates in fp32 in an implementation-defined order); per-tensor norms are rounded to fp32 and
// combined like torch.norm(torch.stack(norms)).  Noise comes from a counter-based generator keyed by
// (seed, element), not from torch's CPU generator: same distribution, different stream.
#pragma clang fp contract(off)

#include <hip/hip_runtime.h>
#include <math.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>

#include "../../include/fedclient.h"
#include "fa_device.h"

// error plumbing shared with fedagg.hip (thread-local last-error string)
extern "C" __attribute__((visibility("hidden"))) int fa_internal_set_error(int code, const char* msg);

namespace {

__attribute__((format(printf, 2, 3))) int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  return fa_internal_set_error(code, buf);
}
int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return fail(FA_E_HIP, "%s: launch failed: %s", what, hipGetErrorString(e));
  return FA_OK;
}

typedef float f4 __attribute__((ext_vector_type(4)));

constexpr int MT_MAX = 64;               // tensors per launch (kernel-argument table 2.8 KiB, < 4 KiB; `vec` is 64 bits)
constexpr int MT_THREADS = 256;
#ifndef MT_UNROLL_N
#define MT_UNROLL_N 4
#endif
constexpr int MT_UNROLL = MT_UNROLL_N;   // float4 per thread per chunk
constexpr int64_t MT_CHUNK = MT_THREADS * 4 * MT_UNROLL;  // 4096 elements per workgroup

struct MtList {
  float* a[MT_MAX];        // param (read; written by prox / dp_apply)
  const float* b[MT_MAX];  // global model (prox) / last model (dp); NULL: buffer without a reference
  float* c[MT_MAX];        // upload (dp_apply, may be NULL)
  int64_t n[MT_MAX];
  int64_t noff[MT_MAX];    // noise counter offset of the tensor's first element
  int32_t blk0[MT_MAX + 1];  // first workgroup of each tensor; blk0[T] = grid size
  uint64_t vec;            // bit t: every pointer of tensor t is 16-byte aligned -> float4 path
  int32_t T;
  int32_t part0;           // index of this launch's first workgroup in the partials workspace
  int32_t t0;              // index of this launch's first tensor in the whole list
};

__device__ __forceinline__ int find_tensor(const MtList& L, int blk) {
  int lo = 0, hi = L.T - 1;  // largest t with blk0[t] <= blk
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (L.blk0[mid] <= blk) lo = mid; else hi = mid - 1;
  }
  return lo;
}

// ---- counter-based N(0,1): 32-bit integer hash -> two 24-bit uniforms -> Box-Muller --------------
__device__ __forceinline__ uint32_t mix32(uint32_t x) {
  x ^= x >> 16; x *= 0x7feb352du; x ^= x >> 15; x *= 0x846ca68bu; x ^= x >> 16;
  return x;
}
// returns the pair (z0, z1) for counter pair index j (elements 2j and 2j+1 of the noise stream)
__device__ __forceinline__ void normal_pair(uint64_t seed, uint64_t j, float& z0, float& z1) {
  const uint32_t s = mix32((uint32_t)seed ^ mix32((uint32_t)(seed >> 32) + 0x9e3779b9u));
  const uint32_t h1 = mix32(s ^ mix32((uint32_t)j ^ mix32((uint32_t)(j >> 32) + 0x85ebca6bu)));
  const uint32_t h2 = mix32(h1 + 0x27d4eb2fu);
  const float u1 = ((float)(h1 >> 8) + 1.0f) * 5.9604644775390625e-08f;  // (0, 1]
  const float u2 = (float)(h2 >> 8) * 5.9604644775390625e-08f;           // [0, 1)
  const float r = sqrtf(-2.0f * logf(u1));
  float sn, cs;
  sincosf(6.283185307179586f * u2, &sn, &cs);
  z0 = r * cs;
  z1 = r * sn;
}
// torch.normal(mean=0, std=sigma): z * sigma + 0 in fp32 (so sigma = 0 gives +0.0 exactly)
__device__ __forceinline__ float noise_at(uint64_t seed, uint64_t e, float sigma) {
  float z0, z1;
  normal_pair(seed, e >> 1, z0, z1);
  return ((e & 1) ? z1 : z0) * sigma + 0.0f;
}

// ------------------------------------------------------------------------------------------------
// FedProx: p = p + c * (p - g)   (optimizers.py:10: param.data += lr*mu*(param.data - global_model[idx]))
// ------------------------------------------------------------------------------------------------
__device__ __forceinline__ float prox1(float p, float g, float c) { return p + c * (p - g); }

__global__ __launch_bounds__(MT_THREADS) void k_prox(MtList L, float c) {
  const int t = find_tensor(L, blockIdx.x);
  const int64_t n = L.n[t];
  const int64_t e0 = (int64_t)(blockIdx.x - L.blk0[t]) * MT_CHUNK;
  float* __restrict__ p = L.a[t];
  const float* __restrict__ g = L.b[t];
  if ((L.vec >> t) & 1) {
    f4 P[MT_UNROLL], G[MT_UNROLL];
    int64_t idx[MT_UNROLL];
#pragma unroll
    for (int u = 0; u < MT_UNROLL; ++u) {
      idx[u] = e0 + ((int64_t)u * MT_THREADS + threadIdx.x) * 4;
      if (idx[u] + 4 <= n) {
        P[u] = *(const f4*)(p + idx[u]);
        G[u] = *(const f4*)(g + idx[u]);
      }
    }
#pragma unroll
    for (int u = 0; u < MT_UNROLL; ++u) {
      if (idx[u] + 4 <= n) {
        *(f4*)(p + idx[u]) = f4{prox1(P[u].x, G[u].x, c), prox1(P[u].y, G[u].y, c), prox1(P[u].z, G[u].z, c),
                                prox1(P[u].w, G[u].w, c)};
      } else {
        for (int64_t i = idx[u]; i < n && i < idx[u] + 4; ++i) p[i] = prox1(p[i], g[i], c);
      }
    }
  } else {
    for (int64_t i = e0 + threadIdx.x; i < n && i < e0 + MT_CHUNK; i += MT_THREADS) p[i] = prox1(p[i], g[i], c);
  }
}

// ------------------------------------------------------------------------------------------------
// Local SGD step fused with the FedProx step (torch_client.py:236-240): torch.optim.SGD(lr, momentum,
// dampening, weight_decay, nesterov) on every parameter, then p += c * (p - g) (optimizers.py:10).
// One pass over param, grad, momentum buffer and global model instead of torch's foreach SGD passes
// plus the proximal pass.  `fma`: torch's alpha-adds (add(x, alpha=a), mul_().add_()) as one fused
// multiply-add each, the way its elementwise kernels are contracted on ROCm; 0: every op rounded.
// ------------------------------------------------------------------------------------------------
constexpr int SGD_MAX = 48;  // tensors per SGD launch: pointers + per-tensor scalars stay < 3 KiB of arguments
struct SgdList {
  float* p[SGD_MAX];
  const float* g[SGD_MAX];      // gradient
  float* m[SGD_MAX];            // momentum buffer (NULL when the tensor's momentum == 0)
  const float* w[SGD_MAX];      // global model (NULL: no proximal step)
  int64_t n[SGD_MAX];
  // per tensor, from its param group (torch_client.py:100-108 builds one group per parameter for
  // detection): lr, momentum, fp32(1 - dampening) formed in double as torch does, weight decay, flags
  float lr[SGD_MAX], mom[SGD_MAX], omd[SGD_MAX], wd[SGD_MAX];
  uint8_t flags[SGD_MAX];       // SGD_NESTEROV | SGD_FIRST
  int32_t blk0[SGD_MAX + 1];
  uint64_t vec;
  int32_t T;
};
enum { SGD_NESTEROV = 1, SGD_FIRST = 2 };
struct SgdScalars {
  float lr, momentum, omd, wd, c;
  int32_t nesterov, first, fma, prox;
};
__device__ __forceinline__ float axpy(float a, float x, float y, int fma) {  // y + a * x
  return fma ? __builtin_fmaf(a, x, y) : y + a * x;
}
__device__ __forceinline__ void sgd1(float& p, float g, float& m, float w, const SgdScalars& k) {
  float d = g;
  if (k.wd != 0.f) d = axpy(k.wd, p, d, k.fma);                 // grad.add(param, alpha=weight_decay)
  if (k.momentum != 0.f) {
    m = k.first ? d : axpy(k.omd, d, m * k.momentum, k.fma);  // buf.mul_(mom).add_(d, alpha=1-damp)
    d = k.nesterov ? axpy(k.momentum, m, d, k.fma) : m;         // d.add(buf, alpha=mom) / buf
  }
  p = axpy(-k.lr, d, p, k.fma);                                 // param.add_(d, alpha=-lr)
  if (k.prox) p = p + k.c * (p - w);                            // optimizers.py:10 (separate torch ops)
}
__global__ __launch_bounds__(MT_THREADS) void k_sgd_prox(SgdList L, float c, int fma) {
  int lo = 0, hi = L.T - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (L.blk0[mid] <= (int)blockIdx.x) lo = mid; else hi = mid - 1;
  }
  const int t = lo;
  const int64_t n = L.n[t];
  const int64_t e0 = (int64_t)(blockIdx.x - L.blk0[t]) * MT_CHUNK;
  float* __restrict__ p = L.p[t];
  const float* __restrict__ g = L.g[t];
  float* __restrict__ m = L.m[t];
  const float* __restrict__ w = L.w[t];
  const SgdScalars k{L.lr[t], L.mom[t], L.omd[t], L.wd[t], c, (L.flags[t] & SGD_NESTEROV) ? 1 : 0,
                     (L.flags[t] & SGD_FIRST) ? 1 : 0, fma, w ? 1 : 0};
  const bool hasm = k.momentum != 0.f;
  if ((L.vec >> t) & 1) {
#pragma unroll
    for (int u = 0; u < MT_UNROLL; ++u) {
      const int64_t i = e0 + ((int64_t)u * MT_THREADS + threadIdx.x) * 4;
      if (i + 4 <= n) {
        f4 P = *(const f4*)(p + i), G = *(const f4*)(g + i);
        f4 M = (hasm && !k.first) ? *(const f4*)(m + i) : f4{0.f, 0.f, 0.f, 0.f};
        const f4 W = k.prox ? *(const f4*)(w + i) : f4{0.f, 0.f, 0.f, 0.f};
        float pv[4] = {P.x, P.y, P.z, P.w}, mv[4] = {M.x, M.y, M.z, M.w};
        const float gv[4] = {G.x, G.y, G.z, G.w}, wv[4] = {W.x, W.y, W.z, W.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) sgd1(pv[e], gv[e], mv[e], wv[e], k);
        P = f4{pv[0], pv[1], pv[2], pv[3]};
        M = f4{mv[0], mv[1], mv[2], mv[3]};
        *(f4*)(p + i) = P;
        if (hasm) *(f4*)(m + i) = M;
      } else {
        for (int64_t j = i; j < n && j < i + 4; ++j) {
          float mj = (hasm && !k.first) ? m[j] : 0.f;
          sgd1(p[j], g[j], mj, k.prox ? w[j] : 0.f, k);
          if (hasm) m[j] = mj;
        }
      }
    }
  } else {
    for (int64_t j = e0 + threadIdx.x; j < n && j < e0 + MT_CHUNK; j += MT_THREADS) {
      float mj = (hasm && !k.first) ? m[j] : 0.f;
      sgd1(p[j], g[j], mj, k.prox ? w[j] : 0.f, k);
      if (hasm) m[j] = mj;
    }
  }
}

// ------------------------------------------------------------------------------------------------
// DP, pass 1: per-workgroup partial of sum((a - b)^2) (norm_type 2) or max|a - b| (inf) in fp64
// ------------------------------------------------------------------------------------------------
// max that propagates NaN, like torch.max (fmax would drop it)
__device__ __forceinline__ double nanmax(double a, double b) { return (b > a || b != b) ? b : a; }
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = nanmax(v, __shfl_xor(v, o, 64));
  return v;
}

template <bool INF>
__global__ __launch_bounds__(MT_THREADS) void k_dp_partial(MtList L, double* __restrict__ part) {
  const int t = find_tensor(L, blockIdx.x);
  const int64_t n = L.n[t];
  const int64_t e0 = (int64_t)(blockIdx.x - L.blk0[t]) * MT_CHUNK;
  const float* __restrict__ a = L.a[t];
  const float* __restrict__ b = L.b[t];
  double acc = 0.0;
  auto take = [&](float x, float y) {
    const float d = b ? x - y : x;  // delta = param - last  (customized_client.py:51-52)
    if (INF) acc = nanmax(acc, (double)fabsf(d));
    else acc += (double)d * (double)d;  // exact square in fp64
  };
  if ((L.vec >> t) & 1) {
#pragma unroll
    for (int u = 0; u < MT_UNROLL; ++u) {
      const int64_t i = e0 + ((int64_t)u * MT_THREADS + threadIdx.x) * 4;
      if (i + 4 <= n) {
        const f4 A = *(const f4*)(a + i);
        const f4 B = b ? *(const f4*)(b + i) : f4{0.f, 0.f, 0.f, 0.f};
        take(A.x, B.x); take(A.y, B.y); take(A.z, B.z); take(A.w, B.w);
      } else {
        for (int64_t j = i; j < n && j < i + 4; ++j) take(a[j], b ? b[j] : 0.f);
      }
    }
  } else {
    for (int64_t i = e0 + threadIdx.x; i < n && i < e0 + MT_CHUNK; i += MT_THREADS) take(a[i], b ? b[i] : 0.f);
  }
  __shared__ double red[MT_THREADS / 64];
  acc = INF ? wave_max(acc) : wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double s = red[0];
    for (int w = 1; w < MT_THREADS / 64; ++w) s = INF ? nanmax(s, red[w]) : s + red[w];
    part[L.part0 + blockIdx.x] = s;
  }
}

// pass 2 (one wave per tensor): the tensor's total over its workgroup partials.  Lane l sums partials
// l, l+64, ... in order, then a fixed butterfly combines the lanes: deterministic for a given model.
template <bool INF>
__global__ __launch_bounds__(64) void k_dp_tensor_norm(MtList L, const double* __restrict__ part,
                                                      double* __restrict__ tsum) {
  const int t = blockIdx.x;
  double s = 0.0;
  for (int b = L.blk0[t] + threadIdx.x; b < L.blk0[t + 1]; b += 64)
    s = INF ? nanmax(s, part[L.part0 + b]) : s + part[L.part0 + b];
  s = INF ? wave_max(s) : wave_sum(s);
  if (threadIdx.x == 0) tsum[L.t0 + t] = s;
}

// pass 3 (one wave): clip_norm.py:36-52 on the per-tensor totals
//   norms[t] = fp32 torch.norm(p_t);  total = torch.norm(torch.stack(norms))  (or max for inf)
//   clip_coef = max_norm / (total + 1e-6)  (fp32);  apply = clip_coef < 1
template <bool INF>
__global__ __launch_bounds__(64) void k_dp_coef(const double* __restrict__ tsum, int T, float max_norm,
                                               float* __restrict__ out) {
  double s = 0.0;
  for (int t = threadIdx.x; t < T; t += 64) {
    if (INF) {
      s = nanmax(s, tsum[t]);
    } else {
      const float nt = (float)sqrt(tsum[t]);  // torch.norm(p, 2) -> fp32 0-d tensor
      s += (double)nt * (double)nt;
    }
  }
  s = INF ? wave_max(s) : wave_sum(s);
  if (threadIdx.x != 0) return;
  const float total = T == 0 ? 0.f : (INF ? (float)s : (float)sqrt(s));  // T == 0: clip_norm.py:35-36
  const float coef = max_norm / (total + 1e-6f);
  out[0] = total;
  out[1] = coef;
  out[2] = (T > 0 && coef < 1.0f) ? 1.0f : 0.0f;  // NaN coef compares false: no clipping, as in torch
}

// ------------------------------------------------------------------------------------------------
// DP, pass 4: recover + noise (customized_client.py:57-63)
//   b != NULL (a parameter):  d = a - b; d = apply ? d * coef : d; pn = b + d; a = pn (if write_param);
//                             c = pn + noise        (upload)
//   b == NULL (a buffer):      c = a + noise
// mode 1 (clip_grad_norm_ alone): a = apply ? a * coef : a, no upload.
// ------------------------------------------------------------------------------------------------
template <int MODE>
__global__ __launch_bounds__(MT_THREADS) void k_dp_apply(MtList L, const float* __restrict__ coefv, float sigma,
                                                       uint64_t seed, int write_param) {
  const int t = find_tensor(L, blockIdx.x);
  const int64_t n = L.n[t];
  const int64_t e0 = (int64_t)(blockIdx.x - L.blk0[t]) * MT_CHUNK;
  float* __restrict__ a = L.a[t];
  const float* __restrict__ b = L.b[t];
  float* __restrict__ c = L.c[t];
  const float coef = coefv[1];
  const bool apply = coefv[2] != 0.f;
  const uint64_t noff = (uint64_t)L.noff[t];
  auto one = [&](int64_t i, float x, float y, float& pn_out) -> float {
    if (MODE == 1) {
      pn_out = apply ? x * coef : x;
      return 0.f;
    }
    float pn = x;
    if (b) {
      float d = x - y;
      if (apply) d = d * coef;
      pn = y + d;
    }
    pn_out = pn;
    return c ? pn + noise_at(seed, noff + (uint64_t)i, sigma) : 0.f;
  };
  const bool write_a = MODE == 1 || (write_param && b);
  if ((L.vec >> t) & 1) {
#pragma unroll
    for (int u = 0; u < MT_UNROLL; ++u) {
      const int64_t i = e0 + ((int64_t)u * MT_THREADS + threadIdx.x) * 4;
      if (i + 4 <= n) {
        const f4 A = *(const f4*)(a + i);
        const f4 B = b ? *(const f4*)(b + i) : f4{0.f, 0.f, 0.f, 0.f};
        float pn[4];
        const float c0 = one(i, A.x, B.x, pn[0]), c1 = one(i + 1, A.y, B.y, pn[1]);
        const float c2 = one(i + 2, A.z, B.z, pn[2]), c3 = one(i + 3, A.w, B.w, pn[3]);
        if (write_a) *(f4*)(a + i) = f4{pn[0], pn[1], pn[2], pn[3]};
        if (MODE == 0 && c) __builtin_nontemporal_store(f4{c0, c1, c2, c3}, (f4*)(c + i));
      } else {
        for (int64_t j = i; j < n && j < i + 4; ++j) {
          float pn;
          const float cv = one(j, a[j], b ? b[j] : 0.f, pn);
          if (write_a) a[j] = pn;
          if (MODE == 0 && c) c[j] = cv;
        }
      }
    }
  } else {
    for (int64_t j = e0 + threadIdx.x; j < n && j < e0 + MT_CHUNK; j += MT_THREADS) {
      float pn;
      const float cv = one(j, a[j], b ? b[j] : 0.f, pn);
      if (write_a) a[j] = pn;
      if (MODE == 0 && c) c[j] = cv;
    }
  }
}

// int64 state_dict entries (BatchNorm num_batches_tracked): numpy int64 + float32 noise -> float64
// int64 state_dict entries (BatchNorm num_batches_tracked): numpy int64 + float32 noise -> float64.
// Multi-tensor like the fp32 kernels: a[t] holds the int64 source, c[t] the float64 destination.
__global__ __launch_bounds__(MT_THREADS) void k_dp_noise_i64(MtList L, float sigma, uint64_t seed) {
  const int t = find_tensor(L, blockIdx.x);
  const int64_t n = L.n[t];
  const int64_t e0 = (int64_t)(blockIdx.x - L.blk0[t]) * MT_CHUNK;
  const int64_t* __restrict__ x = (const int64_t*)L.a[t];
  double* __restrict__ out = (double*)L.c[t];
  for (int64_t i = e0 + threadIdx.x; i < n && i < e0 + MT_CHUNK; i += MT_THREADS)
    out[i] = (double)x[i] + (double)noise_at(seed, (uint64_t)(L.noff[t] + i), sigma);
}

// ---- host side: cut the tensor list into launch groups -----------------------------------------
bool al16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// Builds group g's table starting at tensor *t (advanced past the group).  Returns the group's grid.
int build_group(MtList& L, int32_t T, int32_t* t, float* const* a, const float* const* b, float* const* c,
                const int64_t* n, const int64_t* noff, int32_t part0) {
  L.T = 0;
  L.vec = 0;
  L.part0 = part0;
  L.t0 = *t;
  int32_t blk = 0;
  while (*t < T && L.T < MT_MAX) {
    const int i = *t;
    const int64_t nb = (n[i] + MT_CHUNK - 1) / MT_CHUNK;
    if (L.T > 0 && blk + nb > (int64_t)INT32_MAX / 2) break;  // a lone tensor always fits (check_list)
    L.a[L.T] = a ? a[i] : nullptr;
    L.b[L.T] = b ? b[i] : nullptr;
    L.c[L.T] = c ? c[i] : nullptr;
    L.n[L.T] = n[i];
    L.noff[L.T] = noff ? noff[i] : 0;
    L.blk0[L.T] = blk;
    if (al16(L.a[L.T]) && al16(L.b[L.T]) && al16(L.c[L.T])) L.vec |= (uint64_t)1 << L.T;
    blk += (int32_t)nb;
    ++L.T;
    ++*t;
  }
  L.blk0[L.T] = blk;
  return blk;
}

int check_list(const char* what, int32_t T, float* const* a, const float* const* b, const int64_t* n,
               bool need_b) {
  if (T < 0) return fail(FA_E_ARG, "%s: negative T", what);
  if (T > 0 && (!a || !n || (need_b && !b))) return fail(FA_E_ARG, "%s: NULL table", what);
  for (int i = 0; i < T; ++i) {
    if (n[i] < 0) return fail(FA_E_ARG, "%s: tensor %d has negative size", what, i);
    if (n[i] > 0 && !a[i]) return fail(FA_E_ARG, "%s: tensor %d: NULL pointer", what, i);
    if (need_b && n[i] > 0 && !b[i]) return fail(FA_E_ARG, "%s: tensor %d: NULL reference pointer", what, i);
    if (((uintptr_t)a[i] & 3u) || (b && ((uintptr_t)b[i] & 3u)))
      return fail(FA_E_ARG, "%s: tensor %d: pointers must be 4-byte aligned", what, i);
    if (n[i] > MT_CHUNK * (int64_t)(INT32_MAX / 4)) return fail(FA_E_RANGE, "%s: tensor %d too large", what, i);
  }
  return FA_OK;
}

// the device a pointer-table call works on: its first non-empty tensor's (fa_device.h)
const void* first_ptr(int32_t T, const void* const* a, const int64_t* n) {
  for (int i = 0; a && n && i < T; ++i)
    if (n[i] > 0 && a[i]) return a[i];
  return nullptr;
}

int64_t total_blocks(int32_t T, const int64_t* n) {
  int64_t s = 0;
  for (int i = 0; i < T; ++i) s += (n[i] + MT_CHUNK - 1) / MT_CHUNK;
  return s;
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// C ABI (include/fedclient.h)
// ------------------------------------------------------------------------------------------------
extern "C" int fa_prox_update(float* const* param, const float* const* global, const int64_t* numel, int32_t T,
                              float c, fa_stream_t stream) {
  int rc = check_list("fa_prox_update", T, param, global, numel, true);
  if (rc) return rc;
  FA_DEVICE_SCOPE("fa_prox_update", stream, first_ptr(T, (const void* const*)param, numel));
  FA_TABLE("param", param, numel, T, 4);
  FA_TABLE("global", global, numel, T, 4);
  int32_t t = 0;
  while (t < T) {
    MtList L;
    const int grid = build_group(L, T, &t, param, global, nullptr, numel, nullptr, 0);
    if (grid == 0) continue;
    hipLaunchKernelGGL(k_prox, dim3(grid), dim3(MT_THREADS), 0, (hipStream_t)stream, L, c);
    if ((rc = check_launch("fa_prox_update"))) return rc;
  }
  return FA_OK;
}

static int sgd_groups(const char* what, float* const* param, const float* const* grad,
                      float* const* momentum_buf, const float* const* global, const int64_t* numel, int32_t T,
                      const float* lr, const float* momentum, const double* dampening, const float* weight_decay,
                      const int32_t* flags, float c, int32_t fma, fa_stream_t stream) {
  int rc = check_list(what, T, param, grad, numel, true);
  if (rc) return rc;
  if (T > 0 && (!lr || !momentum || !dampening || !weight_decay || !flags))
    return fail(FA_E_ARG, "%s: NULL per-tensor scalar table", what);
  for (int i = 0; i < T; ++i) {
    if (numel[i] == 0) continue;
    if (momentum[i] != 0.f && (!momentum_buf || !momentum_buf[i]))
      return fail(FA_E_ARG, "%s: tensor %d: momentum != 0 needs a momentum buffer", what, i);
    if (global && !global[i]) return fail(FA_E_ARG, "%s: tensor %d: NULL global pointer", what, i);
    if ((momentum_buf && ((uintptr_t)momentum_buf[i] & 3u)) || (global && ((uintptr_t)global[i] & 3u)))
      return fail(FA_E_ARG, "%s: tensor %d: pointers must be 4-byte aligned", what, i);
    if ((flags[i] & SGD_NESTEROV) && (momentum[i] <= 0.f || dampening[i] != 0.0))
      return fail(FA_E_ARG, "%s: tensor %d: nesterov needs momentum > 0 and zero dampening", what, i);
  }
  FA_DEVICE_SCOPE(what, stream, first_ptr(T, (const void* const*)param, numel));
  FA_TABLE("param", param, numel, T, 4);
  FA_TABLE("grad", grad, numel, T, 4);
  FA_TABLE("global", global, numel, T, 4);
  for (int i = 0; momentum_buf && i < T; ++i)  // buffers are read only where the group's momentum != 0
    if (momentum[i] != 0.f && numel[i] > 0) {
      char nm[48];
      snprintf(nm, sizeof(nm), "momentum_buf[%d]", i);
      FA_OPERAND(nm, momentum_buf[i], (uint64_t)numel[i] * 4);
    }
  int32_t t = 0;
  while (t < T) {
    SgdList L;
    L.T = 0;
    L.vec = 0;
    int32_t blk = 0;
    while (t < T && L.T < SGD_MAX) {
      const int64_t nb = (numel[t] + MT_CHUNK - 1) / MT_CHUNK;
      if (L.T > 0 && blk + nb > (int64_t)INT32_MAX / 2) break;
      const int j = L.T;
      L.p[j] = param[t];
      L.g[j] = grad[t];
      L.m[j] = (momentum[t] != 0.f) ? momentum_buf[t] : nullptr;
      L.w[j] = global ? global[t] : nullptr;
      L.n[j] = numel[t];
      L.lr[j] = lr[t];
      L.mom[j] = momentum[t];
      // torch's buf.add_(d, alpha=1 - dampening): the Python double 1 - dampening, rounded to fp32 once
      L.omd[j] = (float)(1.0 - dampening[t]);
      L.wd[j] = weight_decay[t];
      L.flags[j] = (uint8_t)(flags[t] & (SGD_NESTEROV | SGD_FIRST));
      L.blk0[j] = blk;
      if (al16(L.p[j]) && al16(L.g[j]) && al16(L.m[j]) && al16(L.w[j])) L.vec |= (uint64_t)1 << j;
      blk += (int32_t)nb;
      ++L.T;
      ++t;
    }
    L.blk0[L.T] = blk;
    if (blk == 0) continue;
    hipLaunchKernelGGL(k_sgd_prox, dim3(blk), dim3(MT_THREADS), 0, (hipStream_t)stream, L, c, fma ? 1 : 0);
    if ((rc = check_launch(what))) return rc;
  }
  return FA_OK;
}

extern "C" int fa_sgd_prox_step(float* const* param, const float* const* grad, float* const* momentum_buf,
                                const float* const* global, const int64_t* numel, int32_t T, float lr,
                                float momentum, double dampening, float weight_decay, int32_t nesterov,
                                int32_t first, float c, int32_t fma, fa_stream_t stream) {
  if (T < 0) return fail(FA_E_ARG, "fa_sgd_prox_step: T=%d", (int)T);
  if (nesterov && (momentum <= 0.f || dampening != 0.0))
    return fail(FA_E_ARG, "fa_sgd_prox_step: nesterov needs momentum > 0 and zero dampening");
  // one group: every tensor takes the same scalars
  const int32_t f = (nesterov ? SGD_NESTEROV : 0) | (first ? SGD_FIRST : 0);
  int rc = FA_OK;
  for (int32_t t0 = 0; t0 < T && rc == FA_OK; t0 += SGD_MAX) {
    const int32_t n = T - t0 < SGD_MAX ? T - t0 : SGD_MAX;
    float lrs[SGD_MAX], moms[SGD_MAX], wds[SGD_MAX];
    double damps[SGD_MAX];
    int32_t flags[SGD_MAX];
    for (int i = 0; i < n; ++i) {
      lrs[i] = lr; moms[i] = momentum; wds[i] = weight_decay; damps[i] = dampening; flags[i] = f;
    }
    rc = sgd_groups("fa_sgd_prox_step", param + t0, grad + t0, momentum_buf ? momentum_buf + t0 : nullptr,
                    global ? global + t0 : nullptr, numel + t0, n, lrs, moms, damps, wds, flags, c, fma, stream);
  }
  if (T == 0) rc = check_list("fa_sgd_prox_step", T, param, grad, numel, true);
  return rc;
}

extern "C" int fa_sgd_prox_step_groups(float* const* param, const float* const* grad, float* const* momentum_buf,
                                       const float* const* global, const int64_t* numel, int32_t T, const float* lr,
                                       const float* momentum, const double* dampening, const float* weight_decay,
                                       const int32_t* flags, float c, int32_t fma, fa_stream_t stream) {
  return sgd_groups("fa_sgd_prox_step_groups", param, grad, momentum_buf, global, numel, T, lr, momentum,
                    dampening, weight_decay, flags, c, fma, stream);
}

extern "C" int64_t fa_dp_workspace_bytes(const int64_t* numel, int32_t T) {
  if (T < 0 || (T > 0 && !numel)) return -1;
  return 8 * (total_blocks(T, numel) + T + 1) + 16;
}

extern "C" int fa_dp_clip_coef(const float* const* param, const float* const* last, const int64_t* numel,
                               int32_t T, float max_norm, int32_t norm_inf, void* workspace, float* coef_out,
                               fa_stream_t stream) {
  int rc = check_list("fa_dp_clip_coef", T, const_cast<float* const*>(param), last, numel, false);
  if (rc) return rc;
  if (!workspace || !coef_out) return fail(FA_E_ARG, "fa_dp_clip_coef: NULL workspace / coef_out");
  if ((uintptr_t)workspace & 7u) return fail(FA_E_ARG, "fa_dp_clip_coef: workspace must be 8-byte aligned");
  const int64_t nblk = total_blocks(T, numel);
  if (nblk > INT32_MAX / 2) return fail(FA_E_RANGE, "fa_dp_clip_coef: model too large");
  FA_DEVICE_SCOPE("fa_dp_clip_coef", stream, coef_out);
  FA_TABLE("param", param, numel, T, 4);
  FA_TABLE("last", last, numel, T, 4);
  FA_OPERAND("workspace", workspace, (uint64_t)fa_dp_workspace_bytes(numel, T));
  FA_OPERAND("coef_out", coef_out, 12);
  double* part = (double*)workspace;
  double* tsum = part + nblk;
  hipStream_t s = (hipStream_t)stream;
  int32_t t = 0, part0 = 0;
  while (t < T) {
    MtList L;
    const int grid = build_group(L, T, &t, const_cast<float* const*>(param), last, nullptr, numel, nullptr, part0);
    if (grid > 0) {
      if (norm_inf) hipLaunchKernelGGL(k_dp_partial<true>, dim3(grid), dim3(MT_THREADS), 0, s, L, part);
      else hipLaunchKernelGGL(k_dp_partial<false>, dim3(grid), dim3(MT_THREADS), 0, s, L, part);
      if ((rc = check_launch("fa_dp_clip_coef"))) return rc;
    }
    if (norm_inf) hipLaunchKernelGGL(k_dp_tensor_norm<true>, dim3(L.T), dim3(64), 0, s, L, part, tsum);
    else hipLaunchKernelGGL(k_dp_tensor_norm<false>, dim3(L.T), dim3(64), 0, s, L, part, tsum);
    if ((rc = check_launch("fa_dp_clip_coef"))) return rc;
    part0 += grid;
  }
  if (norm_inf) hipLaunchKernelGGL(k_dp_coef<true>, dim3(1), dim3(64), 0, s, tsum, T, max_norm, coef_out);
  else hipLaunchKernelGGL(k_dp_coef<false>, dim3(1), dim3(64), 0, s, tsum, T, max_norm, coef_out);
  return check_launch("fa_dp_clip_coef");
}

extern "C" int fa_dp_apply(float* const* param, const float* const* last, float* const* upload,
                           const int64_t* numel, const int64_t* noise_offset, int32_t T, const float* coef,
                           float sigma, uint64_t seed, int32_t flags, fa_stream_t stream) {
  int rc = check_list("fa_dp_apply", T, param, last, numel, false);
  if (rc) return rc;
  if (!coef) return fail(FA_E_ARG, "fa_dp_apply: NULL coef");
  const bool scale_only = flags & FA_DP_SCALE_ONLY;
  if (!scale_only && (!upload || !noise_offset))
    return fail(FA_E_ARG, "fa_dp_apply: NULL upload / noise_offset table");
  for (int i = 0; !scale_only && i < T; ++i)
    if (numel[i] > 0 && (!upload[i] || ((uintptr_t)upload[i] & 3u)))
      return fail(FA_E_ARG, "fa_dp_apply: tensor %d: bad upload pointer", i);
  FA_DEVICE_SCOPE("fa_dp_apply", stream, coef);
  FA_TABLE("param", param, numel, T, 4);
  FA_TABLE("last", last, numel, T, 4);
  if (!scale_only) FA_TABLE("upload", upload, numel, T, 4);
  FA_OPERAND("coef", coef, 12);
  int32_t t = 0;
  hipStream_t s = (hipStream_t)stream;
  const int wp = (flags & FA_DP_WRITE_PARAM) ? 1 : 0;
  while (t < T) {
    MtList L;
    const int grid = build_group(L, T, &t, param, last, scale_only ? nullptr : upload, numel,
                                 scale_only ? nullptr : noise_offset, 0);
    if (grid == 0) continue;
    if (scale_only) hipLaunchKernelGGL(k_dp_apply<1>, dim3(grid), dim3(MT_THREADS), 0, s, L, coef, sigma, seed, wp);
    else hipLaunchKernelGGL(k_dp_apply<0>, dim3(grid), dim3(MT_THREADS), 0, s, L, coef, sigma, seed, wp);
    if ((rc = check_launch("fa_dp_apply"))) return rc;
  }
  return FA_OK;
}

extern "C" int fa_dp_noise_i64(const int64_t* const* x, double* const* out, const int64_t* numel,
                               const int64_t* noise_offset, int32_t T, float sigma, uint64_t seed,
                               fa_stream_t stream) {
  if (T < 0 || (T > 0 && (!x || !out || !numel || !noise_offset))) return fail(FA_E_ARG, "fa_dp_noise_i64: bad args");
  for (int i = 0; i < T; ++i) {
    if (numel[i] < 0 || (numel[i] > 0 && (!x[i] || !out[i])))
      return fail(FA_E_ARG, "fa_dp_noise_i64: tensor %d: bad pointer / size", i);
    if (((uintptr_t)x[i] & 7u) || ((uintptr_t)out[i] & 7u))
      return fail(FA_E_ARG, "fa_dp_noise_i64: tensor %d: pointers must be 8-byte aligned", i);
    if (numel[i] > MT_CHUNK * (int64_t)(INT32_MAX / 4)) return fail(FA_E_RANGE, "fa_dp_noise_i64: tensor %d too large", i);
  }
  FA_DEVICE_SCOPE("fa_dp_noise_i64", stream, first_ptr(T, (const void* const*)out, numel));
  FA_TABLE("x", x, numel, T, 8);
  FA_TABLE("out", out, numel, T, 8);
  int32_t t = 0;
  int rc;
  while (t < T) {
    MtList L;
    const int grid = build_group(L, T, &t, (float* const*)x, nullptr, (float* const*)out, numel, noise_offset, 0);
    if (grid == 0) continue;
    L.vec = 0;
    hipLaunchKernelGGL(k_dp_noise_i64, dim3(grid), dim3(MT_THREADS), 0, (hipStream_t)stream, L, sigma, seed);
    if ((rc = check_launch("fa_dp_noise_i64"))) return rc;
  }
  return FA_OK;
}

// reference normal stream for host-side tests: z[i] for counter i (host twin in fedscale_amd/synth.py)
__global__ void k_dp_normals(float* out, int64_t n, uint64_t seed, int64_t off) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    out[i] = noise_at(seed, (uint64_t)(off + i), 1.0f);
}

extern "C" int fa_dp_normals(float* out, int64_t n, uint64_t seed, int64_t noise_offset, fa_stream_t stream) {
  if (n < 0 || (n > 0 && !out)) return fail(FA_E_ARG, "fa_dp_normals: bad args");
  if (n == 0) return FA_OK;
  FA_DEVICE_SCOPE("fa_dp_normals", stream, out);
  FA_OPERAND("out", out, (uint64_t)n * 4);
  int64_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  hipLaunchKernelGGL(k_dp_normals, dim3((unsigned)g), dim3(256), 0, (hipStream_t)stream, out, n, seed, noise_offset);
  return check_launch("fa_dp_normals");
}
