/*
 * fedclient.h — C ABI of the client-side element-wise weight handlers on MI355X (gfx950), SURVEY §8f
 * row 4.  Built into the same libfedagg.so as fedagg.h and following its conventions (0 / negative FA_E*
 * codes, fa_last_error_string(), asynchronous on `stream`, caller-owned device memory, stateless).
 *
 * A model is a list of T separately allocated tensors: every entry point takes HOST arrays of T device
 * pointers and element counts and processes the whole list in a few multi-tensor launches (the table
 * travels in the kernel arguments).  Pointers must be 4-byte aligned; 16-byte aligned tensors take the
 * float4 path.
 *
 * The reference runs these handlers in the executor, on whatever device trains the model; there is no
 * native code or FFI on this path, so the "interface" replaced is the Python function cited per entry
 * point (fedscale_amd/cloud/execution/ binds them through ctypes).
 */
#ifndef FEDCLIENT_H
#define FEDCLIENT_H

#include <stdint.h>

#include "fedagg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* flags of fa_dp_apply */
enum {
  FA_DP_WRITE_PARAM = 1, /* also store the recovered parameter last + clip(delta) back into param[t] */
  FA_DP_SCALE_ONLY = 2,  /* clip_grad_norm_ alone: param[t] *= coef when coef < 1; no upload, no noise */
};

/*
 * FedProx proximal step, fedscale/cloud/execution/optimizers.py:6-10 (ClientOptimizer.update_client_weight,
 * called after every local step at torch_client.py:238-240):
 *   param[t][i] = param[t][i] + c * (param[t][i] - global[t][i])     c = fp32(learning_rate * proxy_mu)
 * every op rounded in fp32 as torch does it (bit-exact).
 */
int fa_prox_update(float* const* param, const float* const* global, const int64_t* numel, int32_t T, float c,
                   fa_stream_t stream);

/*
 * One local training step fused with the FedProx step: replaces torch_client.py:236-240
 * (torch.optim.SGD.step() as built by get_optimizer :95-130, then update_client_weight, optimizers.py:6-10).
 * Per element of every tensor t, as torch.optim.SGD (maximize False) then FedProx:
 *   d = grad + weight_decay * p;  buf = first ? d : buf * momentum + (1 - dampening) * d;
 *   d = nesterov ? d + momentum * buf : buf;  p = p - lr * d;  p = p + c * (p - global)
 * momentum_buf[t] is written (read unless `first`); ignored when momentum == 0.  global == NULL: no
 * proximal step.  fma != 0: each alpha-add is one fused multiply-add (torch's elementwise kernels on ROCm).
 * dampening is the Python double of the param group: 1 - dampening is formed in double and rounded to
 * fp32 once, as torch does for the alpha of buf.add_(d, alpha=1 - dampening).
 */
int fa_sgd_prox_step(float* const* param, const float* const* grad, float* const* momentum_buf,
                     const float* const* global, const int64_t* numel, int32_t T, float lr, float momentum,
                     double dampening, float weight_decay, int32_t nesterov, int32_t first, float c, int32_t fma,
                     fa_stream_t stream);

/*
 * fa_sgd_prox_step over every param group of an optimizer in one pass: the SGD scalars come per tensor
 * (host arrays of T: lr, momentum, dampening (the group's Python double), weight_decay, flags =
 * FA_SGD_NESTEROV | FA_SGD_FIRST), as torch.optim.SGD keeps them per param group.  The detection task
 * builds one group per parameter (torch_client.py:100-108), so this is one launch where the per-group
 * call would be one launch (and one host round trip) per parameter.
 */
enum { FA_SGD_NESTEROV = 1, FA_SGD_FIRST = 2 };
int fa_sgd_prox_step_groups(float* const* param, const float* const* grad, float* const* momentum_buf,
                            const float* const* global, const int64_t* numel, int32_t T, const float* lr,
                            const float* momentum, const double* dampening, const float* weight_decay,
                            const int32_t* flags, float c, int32_t fma, fa_stream_t stream);

/*
 * Local-DP clipping coefficient, examples/differential_privacy/clip_norm.py:12-52 applied to
 * delta[t] = param[t] - last[t] (customized_client.py:51-55; last[t] == NULL: delta[t] = param[t]):
 *   norms[t] = ||delta[t]||_2 (fp32)  ->  total = ||stack(norms)||_2   (norm_inf: max |delta|)
 *   coef = fp32(max_norm) / (total + 1e-6f);  apply = coef < 1
 * Writes coef_out[0] = total, coef_out[1] = coef, coef_out[2] = apply ? 1 : 0 (device fp32[3]).
 * Squares are summed in fp64 in a fixed order (deterministic).  workspace: fa_dp_workspace_bytes(numel, T)
 * bytes of device memory, 8-byte aligned.
 */
int64_t fa_dp_workspace_bytes(const int64_t* numel, int32_t T);
int fa_dp_clip_coef(const float* const* param, const float* const* last, const int64_t* numel, int32_t T,
                    float max_norm, int32_t norm_inf, void* workspace, float* coef_out, fa_stream_t stream);

/*
 * Local-DP recover + noise, customized_client.py:57-63, with coef from fa_dp_clip_coef:
 *   last[t] != NULL (a parameter): d = param - last; if apply: d = d * coef; pn = last + d;
 *                                  param = pn (FA_DP_WRITE_PARAM); upload = pn + z * sigma
 *   last[t] == NULL (a buffer):    upload = param + z * sigma
 * z = N(0,1) from a counter-based generator keyed by (seed, noise_offset[t] + i) — the same distribution
 * as the reference's torch.normal(mean=0, std=sigma), a different stream; sigma = 0 adds exactly +0.
 * FA_DP_SCALE_ONLY: param = apply ? param * coef : param (clip_norm.py:50-52 alone; upload/noise unused).
 */
int fa_dp_apply(float* const* param, const float* const* last, float* const* upload, const int64_t* numel,
                const int64_t* noise_offset, int32_t T, const float* coef, float sigma, uint64_t seed, int32_t flags,
                fa_stream_t stream);

/* int64 state_dict entries (customized_client.py:63 on BatchNorm num_batches_tracked), all T in one launch:
 *   out[t][i] = double(x[t][i]) + double(z(seed, noise_offset[t] + i) * sigma)
 * (numpy int64 + float32 -> float64).  Pointers 8-byte aligned. */
int fa_dp_noise_i64(const int64_t* const* x, double* const* out, const int64_t* numel, const int64_t* noise_offset,
                    int32_t T, float sigma, uint64_t seed, fa_stream_t stream);

/* The generator alone: out[i] = z(seed, noise_offset + i) (for the distribution tests). */
int fa_dp_normals(float* out, int64_t n, uint64_t seed, int64_t noise_offset, fa_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* FEDCLIENT_H */
