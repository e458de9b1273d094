/*
 * fedagg.h — C ABI of the MI355X (gfx950) aggregator update-reduction path.
 *
 * This library replaces the arithmetic of FedScale's aggregator hot path (FedScale v0.5,
 * /root/reference).  The reference has no native code and no FFI on this path: its "interface" is the
 * Python plugin surface listed per entry point below, and the binding a maintainer adds is the ctypes
 * layer in fedscale_amd/_native.py (INTEGRATION.md shows it).
 *
 * Conventions (all entry points):
 *   - return 0 on success, a negative FA_E* code on failure; fa_last_error_string() describes the
 *     last failure of the calling thread.  No exception crosses the ABI.
 *   - every pointer is DEVICE memory owned by the caller (16-byte aligned), except where an entry point
 *     says it may be pinned host memory (fa_reduce_mirror, fa_side_accumulate's xi); every launch is
 *     asynchronous on the caller's `stream` (a hipStream_t) with no implicit synchronisation.
 *     Functions are stateless and reentrant.
 *   - the device: a call's work runs on the GPU that holds its output.  A non-NULL `stream` must be a
 *     stream of that GPU (else FA_E_ARG, nothing launched); NULL means the legacy default stream of THAT
 *     GPU — the library makes it current for the call and restores the caller's current device after, so
 *     one host thread can drive several GPUs (fedscale_amd/csrc/fa_device.h).  Launch plans size their
 *     grids by that GPU's CU count.
 *   - operands (ABI 3, round 4): before anything is queued, EVERY buffer a call's kernels read or write is
 *     checked to be device memory of the call's GPU — or pinned host memory where an entry point says so —
 *     and to hold the call's extent inside its allocation; otherwise FA_E_ARG names the operand and nothing
 *     is launched (pageable memory would fault the GPU; another GPU's memory would be read over xGMI).
 *   - a "bucket" is the fp32 tensors of a state_dict concatenated in state_dict order: P elements,
 *     padded with zeros to a row stride `ld` (multiple of 64).  Client updates live client-major,
 *     x[k*ld + p].  Every per-column buffer (acc, out, last, m, v, delta) holds >= round_up(P, 4)
 *     elements.  Non-fp32 (int64) state_dict entries form the "side table" of Q elements.
 *   - reductions run strictly in arrival order per element (k = 0, 1, ..., K-1), in fp32 with IEEE
 *     round-to-nearest per operation and no fused multiply-add, so they are bit-identical to the
 *     reference's numpy/torch CPU arithmetic; chunked calls (FA_ACCUMULATE) continue the same chain.
 */
#ifndef FEDAGG_H
#define FEDAGG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* fa_stream_t; /* hipStream_t */

enum {
  FA_OK = 0,
  FA_E_ARG = -1,      /* bad size / null / alignment */
  FA_E_HIP = -2,      /* a HIP runtime call failed */
  FA_E_RANGE = -3,    /* size beyond what the kernel supports */
};

/* flags for fa_reduce / fa_reduce_yogi */
enum {
  FA_ACCUMULATE = 1, /* chain starts from acc_in[p] (a previous chunk) instead of client 0 */
  FA_FINALIZE = 2,   /* write chain / denom (true fp32 division) instead of the raw chain */
  FA_YOGI_INIT = 4,  /* fa_reduce_yogi / fa_yogi_step: first call, m := 0 and v := tau (yogi.py:17-19) */
};

int fa_abi_version(void);
const char* fa_last_error_string(void);

/* Build provenance (ABI 4).  fa_build_id(): 16 hex digits of SHA-256 over the compiler flags, the extra -D
 * definitions (fa_build_defs(), "" for the product build) and every source and header of this library
 * (fedscale_amd/buildinfo.py).  The loader recomputes it from the tree and refuses a library that differs.
 * No reference counterpart. */
const char* fa_build_id(void);
const char* fa_build_defs(void);

/* Operand extents HIP cannot report (ABI 5).  Device memory in VMM / expandable segments has no address range, so
 * its extent cannot be checked: such an operand is accepted after its type and device checks and counted;
 * fa_unranged_operands() returns that count for the process, and fa_set_strict_operands(1) refuses such operands
 * with FA_E_ARG instead (returns the previous setting).  Host memory without a range is accepted only inside a
 * fa_host_register registration, extent included.  No reference counterpart. */
int64_t fa_unranged_operands(void);
int fa_set_strict_operands(int32_t on);

/* What a pointer is to the GPU: 0 device memory (or NULL), 1 pinned host memory the GPU reads at the same
 * address (hipHostMalloc, torch pin_memory), -1 anything else (pageable, unregistered, managed) — no entry point
 * hands such a pointer to a kernel: fa_reduce, fa_reduce_mirror and fa_side_accumulate reject it with FA_E_ARG.
 * No reference counterpart (the host-memory operands of the zero-copy round). */
int fa_pointer_kind(const void* p);

/*
 * Weighted in-order K-way column reduction over one chunk of K client updates.
 *   chain_p = FA_ACCUMULATE ? acc_in[p] : w_0*x[0][p]      (w_k = a[k], or 1 when a == NULL)
 *   chain_p = chain_p + w_k*x[k][p]                          k = (FA_ACCUMULATE ? 0 : 1) .. K-1
 *   out[p]  = FA_FINALIZE ? chain_p / denom : chain_p
 * Replaces: Aggregator.update_weight_aggregation, aggregator.py:489-511 (a == NULL, denom = K) and
 *           AsyncAggregator.update_weight_aggregation, async_aggregator.py:115-137 (a = staleness
 *           weights 1/sqrt(1+s) rounded to fp32, denom = fp32(sum of the weights)).
 * `a` is a device array of K fp32 weights or NULL.  out may alias acc_in.
 */
int fa_reduce(const float* x, int64_t ld, int32_t K, int64_t P, const float* a, const float* acc_in,
              float* out, float denom, int32_t flags, fa_stream_t stream);

/*
 * fa_reduce for every part of a model sharded over the GPUs of ONE process (ShardedModelAdapter), in one call:
 * part i reduces x[i] (K[i] rows of ld[i] floats, P[i] columns) into out[i] (continuing acc_in[i] with
 * FA_ACCUMULATE) on streams[i], a stream of the GPU holding out[i] (never NULL), with fa_reduce's arithmetic,
 * denom and flags[i]; unweighted (FedAvg).  Every part is checked before any part launches.  Replaces the same
 * lines as fa_reduce (aggregator.py:497-507) for the finish of an in-process N-GPU round (the per-part host call
 * chain was the round's serial part: DESIGN.md §6).
 */
int fa_reduce_parts(int32_t n, const float* const* x, const int64_t* ld, const int32_t* K, const int64_t* P,
                    const float* const* acc_in, float* const* out, float denom, const int32_t* flags,
                    fa_stream_t const* streams);

/*
 * fa_reduce with FA_FINALIZE whose epilogue writes the mean twice: into out (device, the new global model)
 * and into `mirror` (round_up(P, 4) floats), which may be PINNED HOST memory (page-locked, mapped for the
 * GPU of `out`).  `x` may be pinned host memory too: the kernel then reads the client rows over PCIe.
 * For small rounds (config 1: 10 x 24,492) this replaces H2D + reduce + D2H with one launch
 * (tools/c1_zero_copy_probe.py: 49.8 -> 31.9 us on the device); the arithmetic and its order are fa_reduce's.
 * Replaces: the same lines as fa_reduce (aggregator.py:489-511, async_aggregator.py:115-137) followed by
 *           get_weights()'s copy of the model to the host (torch_model_adapter.py:41-47).
 * Host buffers are visible to the host once the stream has passed the launch (an event or a synchronize).
 */
int fa_reduce_mirror(const float* x, int64_t ld, int32_t K, int64_t P, const float* a, const float* acc_in,
                     float* out, float* mirror, float denom, int32_t flags, fa_stream_t stream);

/*
 * Number of kernel launches one fa_reduce (or fa_reduce_yogi) call makes at (K, P) on the current device:
 * long buckets run as several launches over column windows.  For reporting per-launch figures (bench.py);
 * no reference counterpart.  Needs a GPU (the plan depends on the CU count).
 */
int64_t fa_reduce_launches(int32_t K, int64_t P, int32_t weighted);

/*
 * fa_reduce with FA_FINALIZE, fused with the FedYoGi server step in the same pass over HBM:
 *   cur = chain/denom; g = cur - last; m = beta*m + omb*g; v = v - (omb2*g*g)*sign(v - g*g);
 *   out = last + (reciprocal(sqrt(v) + tau) * eta) * m
 * Replaces: TorchModelAdapter.set_weights (torch_model_adapter.py:23-39) ->
 *           TorchServerOptimizer.update_round_gradient fed-yogi branch (optimizers.py:43-63) ->
 *           YoGi.update (yogi.py:15-36).  omb = fp32(1-beta), omb2 = fp32(1-beta2) as the host computes
 *           them in double.  m, v are updated in place; FA_YOGI_INIT ignores their contents.
 *           mean_out (optional, may be NULL) receives cur, the FedAvg mean the reference keeps in
 *           Aggregator.model_weights.
 */
int fa_reduce_yogi(const float* x, int64_t ld, int32_t K, int64_t P, const float* a, const float* acc_in,
                   float denom, const float* last, float* m, float* v, float* out, float* mean_out, float eta,
                   float tau, float beta, float omb, float omb2, int32_t flags, fa_stream_t stream);

/* The FedYoGi step alone on an already-reduced model (cur = the new mean), same arithmetic as above.
 * Replaces: optimizers.py:43-63 + yogi.py:15-36 when set_weights() is handed a list of weights. */
int fa_yogi_step(const float* cur, const float* last, float* m, float* v, float* out, int64_t P, float eta,
                 float tau, float beta, float omb, float omb2, int32_t flags, fa_stream_t stream);

/* fa_yogi_step over every part of a model sharded across the GPUs of ONE process, in one call: part i steps cur[i],
 * last[i], m[i], v[i] -> out[i] (P[i] columns) on streams[i] (never NULL), the same scalars and flags for every part.
 * Every part is checked before any launches.  With fa_reduce_parts, config 4's in-process finish (optimizers.py:43-63,
 * yogi.py:15-36 over the model's shards). */
int fa_yogi_step_parts(int32_t n, const float* const* cur, const float* const* last, float* const* m, float* const* v,
                       float* const* out, const int64_t* P, float eta, float tau, float beta, float omb, float omb2,
                       int32_t flags, fa_stream_t const* streams);

/*
 * Number of k_qfed_accum launches one fa_qfed_accumulate call makes for rows of ld floats and P columns,
 * with (chain != 0) or without the fused FedAvg chain: long rows run as column windows of one round of tiles
 * (4,194,304 columns; 2,097,152 for chain launches, whose tiles are 8 float4 per lane wide).  For reporting
 * per-launch figures (bench.py); no reference counterpart.
 */
int64_t fa_qfed_launches(int64_t ld, int64_t P, int32_t chain);

/*
 * q-FedAvg phase 1 over one chunk of K (<= fa_qfed_max_chunk()) retained client updates:
 *   g_k = (last - x[k]) / lr                      (fp32 true division)
 *   delta = FA_ACCUMULATE ? delta + alpha_k*g_0 : alpha_0*g_0; delta = delta + alpha_k*g_k ...
 *   sqnorm[k] += sum_p fp32(g_k[p]^2)              (accumulated in fp64, deterministic order)
 *   chain (optional, may be NULL) = FA_ACCUMULATE ? chain + x[0] : x[0]; chain = chain + x[k] ...
 * Replaces: the per-client loop of optimizers.py:73-98 (client results retained at aggregator.py:466-467)
 * and, through `chain`, the FedAvg sum the reference computes on the same inputs (aggregator.py:497-503,
 * its model_weights): fa_reduce(chain, ld, 1, P, ..., FA_FINALIZE, denom = K) then gives the mean.
 * alpha: device fp32[K] = fp32(float_power(loss_k + 1e-10, q)).  sqnorm: device fp64[K].
 * workspace: device memory of `workspace_bytes` bytes, at least fa_qfed_workspace_bytes(K, 0, 0) (one column
 * window's per-workgroup partial norms: the gathers then run after every window).  fa_qfed_workspace_bytes(K, ld,
 * P) holds every window's partials of a call at (ld, P), chain or not: the gathers then run once per call
 * (ABI 3; the per-window form cost ~13 us a window).  Either way the norms are the same bits.
 * Reproducibility: a call's results are the same bits run to run (fixed grid, fixed gather order, no atomics).
 * delta and chain are per column, so calls with and without `chain` give the same delta bits; sqnorm is NOT
 * bit-reproducible across that choice — chain launches sum each client's squares over 8-float4 tiles, plain ones
 * over 16-float4 tiles (another fp64 order; ~1e-16 relative, the fp32 value hs consumes within one ulp).
 */
int fa_qfed_max_chunk(void);
int64_t fa_qfed_workspace_bytes(int32_t K, int64_t ld, int64_t P);
int fa_qfed_accumulate(const float* x, int64_t ld, int32_t K, int64_t P, const float* last, const float* alpha,
                       float lr, float* delta, float* chain, double* sqnorm, void* workspace, int64_t workspace_bytes,
                       int32_t flags, fa_stream_t stream);

/*
 * q-FedAvg Lipschitz estimate, the fp32 recurrence of optimizers.py:96-98 in arrival order:
 *   hs = 0; hs = hs + (c1[k]*fp32(sqnorm[k]) + c2[k])      k = 0..K-1
 *   hs_out[0] = hs; hs_out[1] = hs + fp32(1e-10)          (the divisor of optimizers.py:102)
 * c1[k] = fp32(q*float_power(loss_k+1e-10, q-1)), c2[k] = fp32((1/lr)*float_power(loss_k+1e-10, q)).
 */
int fa_qfed_hs(const double* sqnorm, const float* c1, const float* c2, int32_t K, float* hs_out,
               fa_stream_t stream);

/* q-FedAvg phase 2: out = last - delta / hs_dev[1]  (optimizers.py:101-104). */
int fa_qfed_finalize(const float* last, const float* delta, const float* hs_dev, float* out, int64_t P,
                     fa_stream_t stream);

/*
 * Side table (non-fp32 state_dict entries, BatchNorm num_batches_tracked etc.).
 * xi: int64 [K][Q] client-major, device or pinned host memory (read over PCIe: small rounds read the staging's
 *     pinned mirror, as fa_reduce_mirror does).  State: acc_i (int64 [Q]) and acc_d (fp64 [Q]).
 *   mode 0 FedAvg : acc_i = acc_i + xi[k]  (int64, aggregator.py:500-503)
 *   mode 1 FedBuff: acc_d = acc_d + w[k]*double(xi[k]), first = double(xi[0])*w[0] (async_aggregator.py:129-133)
 * w: device fp64[K] or NULL.  FA_ACCUMULATE continues a previous chunk.
 */
int fa_side_accumulate(const int64_t* xi, int32_t ldq, int32_t K, int32_t Q, int32_t mode, const double* w,
                       int64_t* acc_i, double* acc_d, int32_t flags, fa_stream_t stream);
/* cur[q] = (mode 0 ? double(acc_i) : acc_d) / denom  (np.divide -> float64, aggregator.py:505-507) and
 * model[q] = int64(fp32(cur[q]))  (np.asarray(float32) + load_state_dict truncation, torch_model_adapter.py:31-35). */
int fa_side_close(const int64_t* acc_i, const double* acc_d, int32_t Q, int32_t mode, double denom, double* cur,
                  int64_t* model, fa_stream_t stream);
/* FedYoGi on the side table, in fp64 (int64 - float64 promotes, optimizers.py:52-61, yogi.py:15-36):
 * g = cur - double(last) (last NULL -> 0); step = (reciprocal(sqrt(v)+tau)*eta)*m;
 * step[q] (optional) = step; model[q] (optional) = int64(fp32(double(last) + step)).  m, v: fp64 [Q]. */
int fa_side_yogi(const double* cur, const int64_t* last, double* m, double* v, double* step, int64_t* model,
                 int32_t Q, double eta, double tau, double beta, double omb, double omb2, int32_t flags,
                 fa_stream_t stream);
/* q-FedAvg on the side table: per element the delta chain over the chunk (fp32), per client the
 * fp64-accumulated sum of fp32 g^2 added to sqnorm[k]. delta_s: fp32 [Q]. */
int fa_side_qfed_accumulate(const int64_t* xi, int32_t ldq, int32_t K, int32_t Q, const int64_t* last,
                            const float* alpha, float lr, float* delta_s, double* sqnorm, int32_t flags,
                            fa_stream_t stream);
/* model[q] = int64( fp32(last[q]) - delta_s[q] / hs_dev[1] ) */
int fa_side_qfed_finalize(const int64_t* last, const float* delta_s, const float* hs_dev, int64_t* model,
                          int32_t Q, fa_stream_t stream);

/*
 * Deterministic synthetic client updates for benchmarks and full-size parity tests:
 *   x[k][p] = base(p) + noise(k, p), base ~ scale_base * tri(seed, p), noise ~ scale_noise * tri(seed+1+k0+k, p)
 * where tri() is a triangular variate built from a 32-bit integer hash (bit-reproducible on the host,
 * see fedscale_amd/synth.py).  Columns [P, ld) are zero-filled.
 */
int fa_fill_synthetic(float* x, int64_t ld, int32_t K, int64_t P, uint32_t seed, int32_t k0, float scale_base,
                      float scale_noise, fa_stream_t stream);

/*
 * HeteroFL sub-model combination: replaces Customized_Aggregator.combine_models,
 * examples/heterofl/customized_aggregator.py:78-119 (index sets from customized_fllibs.py:25-70 are
 * prefixes, so client m's upload of tensor k is the box [0:o) x [0:i) x S of the global (O, I, S)).
 *   xs       concatenated client uploads (fp32, 16-byte aligned),
 *            desc[(m*T + k)*4 + {0,1,2,3}] = {offset in xs, o, L = i*S, ld}: client m's box of tensor k is
 *            o rows of L elements at row stride ld.  For ROW-mode tensors the offset must be a multiple
 *            of 4 and ld = round_up(L, 4) (rows padded to 16 bytes; the padding is read, never counted);
 *            ELEMENT-mode tensors may use ld = L at any offset.
 *   tensors  [T][4] = {offset in global, O, I, S};  chunk_tensor[2c] = tensor of workgroup c,
 *            chunk_tensor[2c+1] = row o (>= 0: columns [chunk_first[c], +1024) of that row, chunk_first
 *            a multiple of 4), -1 (elements [chunk_first[c], +1024) of the flattened tensor, any layout)
 *            or -2 (FLAT: elements [chunk_first[c], +8192) of the flattened tensor; I*S a multiple of 4,
 *            chunk_first a multiple of 4, boxes in the padded ROW layout)
 * global[e] <- (sum over covering clients, client order, fp32 from 0) / fp32(count) where count > 0.
 */
int fa_prefix_box_combine(const float* xs, const int64_t* desc, int32_t K, const int64_t* tensors, int32_t T,
                          const int32_t* chunk_tensor, const int64_t* chunk_first, int32_t nchunks, float* global,
                          fa_stream_t stream);

/*
 * Host ingress (no GPU work): copy n host byte ranges srcs[i][0:nbytes[i]] to dst + dst_off[i] with up
 * to `threads` workers of a persistent pool (used to gather an arriving update's tensors into a pinned
 * staging row before its H2D copy).  Replaces the per-tensor numpy copies implied by
 * aggregator.py:494-503's list handling; no reference FFI exists for it.
 */
int fa_host_gather(void* dst, const void* const* srcs, const int64_t* dst_off, const int64_t* nbytes, int32_t n,
                   int32_t threads);

/*
 * N-GPU ingress straight out of the upload's own bytes (round 4; replaces, for a model sharded over several
 * GPUs of the one aggregator process, the pinned full-model row that fa_host_gather fills: one host-DRAM pass per
 * byte instead of three).  fa_host_register pins and registers the pages of host memory the caller owns — the
 * executor's pickled payload whose arrays fedscale_amd/ingress.py decoded as views (aggregator.py:704) — and
 * fa_host_unregister releases them once every copy out of them has completed.  fa_h2d_pieces enqueues, for each
 * piece i, an asynchronous H2D copy of nbytes[i] from src[i] to dst[i] on streams[sidx[i]] (a HOST table of
 * nstreams hipStream_t): dst[i] must be device memory of that stream's device, src[i] registered or pinned host
 * memory, both holding nbytes[i] — checked for every piece before any copy is enqueued (FA_E_ARG otherwise).
 * Copies run in piece order per stream.  No reference counterpart (the reference has no device, aggregator.py).
 */
int fa_host_register(void* p, int64_t nbytes);
int fa_host_unregister(void* p);
int fa_h2d_pieces(void* const* dst, const void* const* src, const int64_t* nbytes, const int32_t* sidx, int32_t n,
                  void* const* streams, int32_t nstreams);

/*
 * Host ingress (no GPU work): strip the large byte strings out of a pickled executor result so it can be
 * unpickled without copying them (replaces the copies inside pickle.loads of deserialize_response,
 * aggregator.py:704, on payloads made by pickle.dumps at torch_client.py:79-91).  Walks the opcode
 * stream of `in[0:n)` up to STOP: FRAME opcodes are dropped; every BINBYTES / BINBYTES8 argument of at
 * least `min_bytes` (>= 16) bytes is replaced by SHORT_BINBYTES of 12 bytes "FAPB" + uint64 LE region
 * index, and regions[2r], regions[2r+1] receive the raw bytes' offset in `in` and their length (for
 * r < max_regions).  Everything else is copied verbatim.  Returns the length of the stripped stream (it
 * is written only when it fits in out_cap; out may be NULL to size it) and sets *nregions, or a negative
 * FA_E* code for an unknown opcode (protocol 5 out-of-band buffers included) or a truncated stream.
 */
int64_t fa_pickle_strip(const uint8_t* in, int64_t n, int64_t min_bytes, uint8_t* out, int64_t out_cap,
                        int64_t* regions, int32_t max_regions, int32_t* nregions);

/*
 * Fixed-order sum of n rows of K fp64 values: out[k] = ((x[0][k] + x[1][k]) + x[2][k]) + ...  (row
 * stride ld).  Combines per-shard partial q-FedAvg squared norms (optimizers.py:96-97 summed over the
 * model's shards) after an all-gather, so the result does not depend on the collective's internal
 * order or on the transport.  out may alias x[0].
 */
int fa_sum_rows_f64(const double* x, int64_t ld, int32_t n, int64_t K, double* out, fa_stream_t stream);

/*
 * Shard group: RCCL collectives over the N GPUs that ONE aggregator process drives.
 *
 * Replaces nothing in the reference (its aggregator is one process on one device, aggregator.py:177-192,
 * 919-963); this is what lets the drop-in spread a round over a node's GPUs behind that unmodified
 * single-process event loop: the parameter shards (or client blocks) live on N devices of the one
 * process, and the cross-device steps are RCCL collectives over xGMI, issued for all N devices in one
 * ncclGroupStart/End from the calling thread.  RCCL is loaded at run time (the copy torch already
 * loaded is reused); fa_rccl_available() == 0 when it cannot be found.
 *
 * Tables (send / recv / bufs / streams) are HOST arrays of N device pointers / hipStream_t, indexed by
 * the position in `devs` given to fa_rccl_init.  count is in elements of `dtype` per device.  streams[i]
 * must be a stream of devs[i] (FA_E_ARG otherwise, nothing enqueued); NULL is accepted only by a one-device
 * communicator.
 *   fa_rccl_init       ncclCommInitAll over devs[0..ndev) (distinct device ordinals)
 *   fa_rccl_all_gather recv[i][r*count + j] = send[r][j]
 *   fa_rccl_all_reduce recv[i][j] = sum_r send[r][j]
 *   fa_rccl_gather     recv_root[r*count + j] = send[r][j]  (on device `root` only)
 *   fa_rccl_broadcast  bufs[i][j] = bufs[root][j]
 */
enum { FA_DT_F32 = 0, FA_DT_F64 = 1, FA_DT_I64 = 2 };
int fa_rccl_available(void);
int fa_rccl_init(int32_t ndev, const int32_t* devs, void** comm_out);
int fa_rccl_destroy(void* comm);
int fa_rccl_all_gather(void* comm, const void* const* send, void* const* recv, int64_t count, int32_t dtype,
                       void* const* streams);
int fa_rccl_all_reduce(void* comm, const void* const* send, void* const* recv, int64_t count, int32_t dtype,
                       void* const* streams);
int fa_rccl_gather(void* comm, const void* const* send, void* recv_root, int64_t count, int32_t dtype, int32_t root,
                   void* const* streams);
int fa_rccl_broadcast(void* comm, void* const* bufs, int64_t count, int32_t dtype, int32_t root,
                      void* const* streams);

/* What RCCL itself reports for a handle (ABI 4): *count = ncclCommCount (every communicator of the handle must
 * agree, else FA_E_HIP); ranks[i] = ncclCommUserRank and devs[i] = ncclCommCuDevice of the handle's i-th
 * communicator (one per device given to fa_rccl_init; one for fa_rccl_init_rank).  ranks / devs may be NULL.
 * The bench records it on every N > 1 line, so a multi-GPU record shows the rank count RCCL saw. */
int fa_rccl_comm_info(void* comm, int32_t* count, int32_t* ranks, int32_t* devs);
/* One rank of a communicator spanning processes (one process per GPU, the SPMD bench): fa_rccl_unique_id on one
 * rank writes NCCL_UNIQUE_ID_BYTES (128) bytes the caller broadcasts; every rank then calls fa_rccl_init_rank
 * with its rank and its device (collective: it returns once all nranks have joined).  Destroy with
 * fa_rccl_destroy.  No reference counterpart. */
int fa_rccl_unique_id(void* id_out);
int fa_rccl_init_rank(int32_t nranks, const void* id, int32_t rank, int32_t device, void** comm_out);

#ifdef __cplusplus
}
#endif
#endif /* FEDAGG_H */
