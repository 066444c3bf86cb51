/*
 * nfdpf.h -- C ABI of libnfdpf.so, the MI355X (gfx950) particle-update hot path of
 * normalizing-flow differentiable particle filters.
 *
 * The reference (xiongjiechen/Normalizing-Flows-DPFs) is pure Python/PyTorch and has no
 * FFI layer: its boundary for this path is the Python module API.  Each
 * entry point below replaces the PyTorch op chain of the reference function cited in its
 * comment; the Python mirror of the reference API (normalizing-flows-dpfs_amd/nf, model,
 * resamplers, utils, DPFs) binds them through ctypes (nfdpf/_lib.py).
 *
 * Conventions
 *   - every buffer is a DEVICE pointer owned by the caller; nothing is allocated inside,
 *     so every call is stream-ordered and capturable into a hipGraph;
 *   - fp32, row-major, contiguous unless a *_rs (row stride, in elements) says otherwise;
 *   - `stream` is a hipStream_t passed as void* (NULL = legacy default stream);
 *   - return 0 on success, NFDPF_EINVAL for bad arguments (nothing launched),
 *     NFDPF_ELAUNCH if the launch failed; nfdpf_last_error() gives the message.
 *
 * Packed parameter blobs (fp32, concatenated in this order, each tensor row-major as
 * nn.Linear stores it):
 *   FCNN(in,out,H)          : W1[H,in] b1[H] W2[H,H] b2[H] W3[out,H] b3[out]   (nf/flows.py:101-114)
 *   coupling net            : FCNN(h + O, h, H) of a RealNVP(_cond) flow, h = dim/2, O = obser_dim,
 *                             stored core-first: W1[:, :h] W2 b2 W3 b3, then W1[:, h:] b1
 *                             (the context columns are folded into a bias once per row)
 *   RealNVP(_cond) flow     : coupling halves (t1, s1), (t2, s2), the two nets of a half
 *                             interleaved elementwise ({t, s} float pairs)     (nf/flows.py:181-190)
 *   stack of n flows        : flow 0, flow 1, ... (model order, i.e. nf_dyn.flows[i])
 *   split suffix (optional) : behind a stack of RealNVP_cond(2, O) flows, for each flow and net
 *                             t1, s1, t2, s2 ninety floats: W1[:, 0], W2, b2, W3 with hidden
 *                             units 2m, 2m+1 adjacent, then {b3, 0} (csrc/split.hpp); the tiled
 *                             step reads it when split_nets is set
 *   MAF flow (dim d)        : initial_param[2], then FCNN(i, 2, H) for i = 1..d-1 (nf/flows.py:247-254)
 *   particle encoder        : Linear(2,16) Linear(16,32) Linear(32,E): W,b each  (model/models.py:130-150),
 *                             W1 in row-pair order [out/2][in][2], W2 and W3 in col-pair order
 *                             [in][out/2][2] (outputs 2m, 2m+1 adjacent in both)
 *   likelihood_est (NN)     : Linear(2E,64) Linear(64,64) Linear(64,1): W,b each (model/models.py:119-128)
 */
#ifndef NFDPF_H
#define NFDPF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__) || defined(__clang__)
#define NFDPF_API __attribute__((visibility("default")))
#else
#define NFDPF_API
#endif

#define NFDPF_OK 0
#define NFDPF_EINVAL 1
#define NFDPF_ELAUNCH 2

/* measurement kinds (arguments.py:24 --measurement) */
#define NFDPF_MEAS_COS 0
#define NFDPF_MEAS_CRNVP 1
#define NFDPF_MEAS_NN 2
#define NFDPF_MEAS_GAUSSIAN 3
#define NFDPF_MEAS_EXTERNAL 4 /* raw likelihood supplied in lik_ext (e.g. CGLOW kernel) */

/* resampler kinds (arguments.py:32 --resampler_type) */
#define NFDPF_RESAMPLE_SOFT 0
#define NFDPF_RESAMPLE_OT 1

/* nf_dyn values of nfdpf_filter_desc: the dynamic flow (--NF-dyn / --NF-dyn-flow) */
#define NFDPF_DYN_NONE 0
#define NFDPF_DYN_REALNVP 1 /* NormalizingFlowModel_cond over RealNVP_cond, [mean,std] context */
#define NFDPF_DYN_MAF 2     /* NormalizingFlowModel over MAF (context-free) */

/* RNG modes: DEVICE = counter-based Philox4x32-10 keyed by (seed, step, global row,
 * particle), shard invariant; HOST = caller uploads the draws of the reference's CPU
 * generator (parity mode) */
#define NFDPF_RNG_DEVICE 0
#define NFDPF_RNG_HOST 1

NFDPF_API int nfdpf_version(void);
NFDPF_API const char *nfdpf_last_error(void);

/* NormalizingFlowModel_cond.forward / .inverse over RealNVP_cond flows
 * (nf/models.py:45-61, nf/flows.py:215-239).  obser_dim = 0 gives the unconditional
 * RealNVP stack (nf/models.py:13-30, nf/flows.py:155-179).
 *   x       [rows, dim]
 *   cond    [ceil(rows / cond_group), obser_dim]: row r uses cond row r / cond_group
 *           (cond_group = 1 is the reference's materialised per-row obser; = N broadcasts a
 *           per-batch context without materialising (B*N, O))
 *   out     [rows, dim]; logdet [rows]; prior_logprob [rows] or NULL (forward only:
 *           log N(z; prior_mean, prior_std^2 I), nf/models.py:51)                        */
NFDPF_API int nfdpf_cond_stack(const float *params, int n_flows, int dim, int obser_dim, int hidden,
                     const float *x, const float *cond, int64_t rows, int64_t cond_group,
                     int inverse, float prior_mean, float prior_std,
                     float *out, float *logdet, float *prior_logprob, void *stream);

/* Backward of nfdpf_cond_stack (training); replaces the autograd graph the
 * reference builds over nf/flows.py:215-239 (RealNVP_cond.forward/.inverse) and
 * nf/models.py:45-61 (NormalizingFlowModel_cond.forward/.inverse, prior log-prob :51).
 * Per-row condition only (cond_group = 1: the reference's materialised obser).
 *   g_out [rows, dim], g_logdet [rows]: dL/d(out, logdet); g_prior_logprob [rows] or NULL
 *   (forward only)
 *   g_x [rows, dim]; g_cond [rows, obser_dim] (may be NULL); g_params [blob floats] in the
 *   blob layout of params (every entry a {t, s} pair, as nfdpf_cond_stack reads it)
 *   workspace: nfdpf_cond_stack_backward_workspace() bytes (per-workgroup parameter partials,
 *   summed in a fixed order: the result is deterministic)
 * Built for dim in {2, 4, 32}, hidden 8, n_flows 1..4, LDS-bound obser_dim (<= ~400 at dim 2). */
NFDPF_API int64_t nfdpf_cond_stack_backward_workspace(int n_flows, int dim, int obser_dim, int hidden,
                                                      int64_t rows);
NFDPF_API int nfdpf_cond_stack_backward(const float *params, int n_flows, int dim, int obser_dim,
                                        int hidden, const float *x, const float *cond, int64_t rows,
                                        int inverse, float prior_mean, float prior_std,
                                        const float *g_out, const float *g_logdet,
                                        const float *g_prior_logprob, float *g_x, float *g_cond,
                                        float *g_params, void *workspace, void *stream);

/* NormalizingFlowModel.forward / .inverse over MAF flows (nf/models.py:13-30,
 * nf/flows.py:259-284; forward flips the output).  x/out [rows, dim], logdet [rows]. */
NFDPF_API int nfdpf_maf_stack(const float *params, int n_flows, int dim, int hidden, const float *x,
                    int64_t rows, int inverse, float *out, float *logdet, void *stream);

/* soft_resampler (resamplers.py:20-60), bit-exact indices vs. the reference on CPU:
 *   x [B,N,D], p [B,N], lin [N] = torch.linspace(0,(N-1)/N,N) (host constant),
 *   offsets [B] (CPU-generator draw uniform_(0,1/N), resamplers.py:43)
 *   -> x_out [B,N,D], w_out [B,N], idx_out [B,N] int64 = local index + N*(row_base + b) */
NFDPF_API int nfdpf_soft_resample(const float *x, const float *p, const float *lin, const float *offsets,
                        int B, int N, int D, float alpha, int64_t row_base, float *x_out,
                        float *w_out, int64_t *idx_out, void *stream);

/* Backward of nfdpf_soft_resample (training): the gradient the reference's
 * autograd takes through resamplers.py:28-56 (q = (a p + (1-a)/N) / S, w = p / q, gather by
 * idx, w' normalised), without its B x N x N tensor.
 *   p [B, N]: the forward's input probabilities; idx [B, N], w_out [B, N]: its outputs
 *   g_x_out [B, N, D] / g_w_out [B, N]: dL/d(x', w') (either may be NULL: zero)
 *   g_x [B, N, D], g_p [B, N]: dL/d(x, p)
 *   workspace: nfdpf_soft_resample_backward_workspace(B, N) bytes
 * Each source's gradient is the in-order sum over its run of equal indices (idx is sorted):
 * deterministic, no atomics. */
NFDPF_API int64_t nfdpf_soft_resample_backward_workspace(int B, int N);
NFDPF_API int nfdpf_soft_resample_backward(const float *p, const int64_t *idx, const float *w_out,
                                           const float *g_x_out, const float *g_w_out, int B, int N,
                                           int D, float alpha, int64_t row_base, float *g_x,
                                           float *g_p, void *workspace, void *stream);

/* resampler_ot (resamplers.py:62-277): entropy-regularised OT, Sinkhorn in fp32 with the
 * reference's batch-coupled stop rule (the loop ends when ANY row converges, :126-129).
 *   x [B,N,2], w [B,N] -> x_out [B,N,2], w_out [B,N] (= 1/N), idx_out [B,N] (identity)
 *   iters_out [1] int32: the reference's returned count (total_iter + 2, :179)
 *   workspace: nfdpf_ot_workspace_bytes(B,N) bytes, 256-B aligned                   */
NFDPF_API int64_t nfdpf_ot_workspace_bytes(int B, int N);
NFDPF_API int nfdpf_ot_resample(const float *x, const float *w, int B, int N, float eps, float scaling,
                      float threshold, int max_iter, int64_t row_base, float *x_out,
                      float *w_out, int64_t *idx_out, int32_t *iters_out, void *workspace,
                      const int32_t *gate, const int32_t *stop_at, int poll, void *stream);
/* The same with row strides (in floats) for x and w: row b of the particles starts at
 * x + b * x_rs (x_rs >= 2N, its N points contiguous), of the weights at w + b * w_rs (w_rs >= N)
 * -- one time step of a [B, T, N, 2] history read in place (the outputs stay contiguous). */
NFDPF_API int nfdpf_ot_resample_rs(const float *x, int64_t x_rs, const float *w, int64_t w_rs, int B, int N,
                                   float eps, float scaling, float threshold, int max_iter, int64_t row_base,
                                   float *x_out, float *w_out, int64_t *idx_out, int32_t *iters_out,
                                   void *workspace, const int32_t *gate, const int32_t *stop_at, int poll,
                                   void *stream);

/* Backward of nfdpf_ot_resample for training: the reference's gradient
 * reaches the particles only through x' = bmm(T, x) with T treated as a constant (its
 * transport Function discards the autograd.grad it computes, resamplers.py:234-245), so
 *   g_x[b, j] = sum_i T[b, i, j] g_out[b, i]      (g_out, g_x [B, N, 2])
 * T is not formed: column j is summed over i from the forward's potentials and column
 * normalisers.  workspace = the forward call's workspace, untouched since that call (its
 * iteration tables are reused); gate = the forward's gate (off: g_x = g_out). */
NFDPF_API int nfdpf_ot_transport_backward(const float *g_out, int B, int N, float eps, float *g_x,
                                          void *workspace, const int32_t *gate, void *stream);
/*   gate: optional device flag; when non-NULL and *gate == 0 every kernel is a no-op (the
 *         ESS gate of DPFs.py:165 decided not to resample this step, without a host sync)
 *   stop_at: optional device int32, in the iters_out encoding (total_iter + 2).  NULL: the
 *         reference's rule -- stop after the first iteration at which ANY of these B rows
 *         has converged (resamplers.py:126-129).  Non-NULL: run exactly that many
 *         iterations.  (A batch sharded over ranks uses the two-phase form below instead of
 *         running once with NULL and again with stop_at = the MIN over ranks.)
 *   poll: 0 -- enqueue max_iter - 1 iteration launches (iterations after the stop exit at
 *         once; stream-ordered, graph-capturable, returns immediately).  1 -- the calling
 *         thread follows the device's progress through library-owned mapped host flags and
 *         stops enqueueing once the loop has stopped (at most 2 early-exit launches past the
 *         stop; the call returns when the last iteration has been enqueued, not capturable;
 *         the reference's own loop syncs the host every iteration, resamplers.py:126-129). */

/* nfdpf_ot_resample for a batch sharded over ranks, in two phases
 * around the caller's all-reduce, without running any Sinkhorn iteration twice:
 *   1. nfdpf_ot_sinkhorn_local: the loop with the stop rule over THIS rank's rows, keeping
 *      every state's potentials in `history` (nfdpf_ot_history_bytes(B, N, max_iter) bytes,
 *      [max_iter][2][B][N] fp64); iters_out = the local count (iters_out encoding).
 *   -- the caller: all-reduce(MIN) of iters_out over the ranks, on the stream (the first row
 *      to converge anywhere ends the unsharded loop, resamplers.py:126-129) --
 *   2. nfdpf_ot_sinkhorn_finish with stop_at = that minimum (<= the local count): rebuilds the
 *      state's tables from the history, then the final potential, column normalisers and the
 *      transport apply at that state.  iters_out (optional) = *stop_at.
 * The outputs equal nfdpf_ot_resample of the whole batch bit for bit (tests/test_gpu_parity.py).
 * Same workspace for both phases, untouched in between; it then serves
 * nfdpf_ot_transport_backward as after nfdpf_ot_resample. */
NFDPF_API int64_t nfdpf_ot_history_bytes(int B, int N, int max_iter);
NFDPF_API int nfdpf_ot_sinkhorn_local(const float *x, const float *w, int B, int N, float eps, float scaling,
                                      float threshold, int max_iter, int32_t *iters_out, void *workspace,
                                      void *history, const int32_t *gate, int poll, void *stream);
NFDPF_API int nfdpf_ot_sinkhorn_finish(const float *x, int B, int N, float eps, float scaling, float threshold,
                                       int max_iter, int64_t row_base, float *x_out, float *w_out,
                                       int64_t *idx_out, int32_t *iters_out, void *workspace, void *history,
                                       const int32_t *gate, const int32_t *stop_at, void *stream);

/* Diagnostics of the last nfdpf_ot_resample on `workspace` (synchronous device read):
 *   host_out[0] = iterations in the iters_out encoding (-1: ran to max_iter), host_out[1] =
 *   softmin evaluations that left the shifted fast path and were recomputed exactly. */
NFDPF_API int nfdpf_ot_stats(const void *workspace, int32_t *host_out);

/* Health of the wave-pair hand-offs of the tiled step (csrc/split.hpp): the number of
 * exchanges that gave up waiting for their partner wave since the last reset (a correct run
 * never does; the launch's outputs are then invalid).  Read in order on `stream` (the stream
 * the checked launches ran on), then that stream is synchronised; reset != 0 clears the count
 * (also in stream order).  Returns -1 if the read failed. */
NFDPF_API int nfdpf_split_fault(int reset, void *stream);

/* ESS gate of DPFs.py:163-165: gate = mean_b(inv_ess[b]) < 0.5 N (or force) -> int32 [1] */
NFDPF_API int nfdpf_ess_gate(const float *inv_ess, int B, int N, int force, int32_t *gate,
                   void *stream);

/* normalize_log_probs (utils.py:39-44) + add, and the per-row inverse ESS term
 * 1/sum(p^2) of DPFs.py:163.  logw [B,N] -> p [B,N]; inv_ess [B] or NULL */
NFDPF_API int nfdpf_normalize_log_probs(const float *logw, int B, int N, float add, float *p,
                              float *inv_ess, void *stream);

/* Measurement models (model/models.py:206-278): enc [B,E] frame encodings,
 * x [B,N,2] particles -> lik [B,N].  kind = NFDPF_MEAS_*; meas_params: CRNVP stack
 * (2 flows, dim E, obser E) or likelihood_est (NN); prior_std: CRNVP prior (2.5). */
NFDPF_API int nfdpf_measurement(int kind, const float *pe_params, const float *meas_params, int n_flows,
                      const float *enc, const float *x, int B, int N, int E, float prior_std,
                      float *lik, void *stream);

/* Backward of the cosine-distance measurement (kind NFDPF_MEAS_COS of nfdpf_measurement;
 * training): the autograd gradient of model/models.py:206-219 (particle
 * encoder :130-139, et_distance utils.py:8-15).
 *   pe_params: the same packed encoder blob; enc [B, E] frame encodings; x [B, N, 2];
 *   g_lik [B, N] = dL/dlik
 *   g_enc [B, E], g_x [B, N, 2]; g_params [1648]: the encoder's gradient in the plain
 *   nn.Linear layout W1 b1 W2 b2 W3 b3 (= the module's parameter order)
 *   workspace: nfdpf_cos_measurement_backward_workspace(B, N) bytes (fixed-order partials) */
/* The particle encoder alone (model/models.py:130-139), for models that feed its output on
 * (CRNVP: the flow's condition, model/models.py:256-278): mode 0 e_out [B*N, 32] = PE(x);
 * mode 1 the backward for a given g_e [B*N, 32] -> g_x [B, N, 2], g_params [1648] (nn.Linear
 * order), workspace nfdpf_cos_measurement_backward_workspace(B, N) bytes. */
NFDPF_API int nfdpf_particle_encoder(int mode, const float *pe_params, const float *x, int B, int N,
                                     const float *g_e, float *e_out, float *g_x, float *g_params,
                                     void *workspace, void *stream);
NFDPF_API int64_t nfdpf_cos_measurement_backward_workspace(int B, int N);
NFDPF_API int nfdpf_cos_measurement_backward(const float *pe_params, const float *enc, const float *x,
                                             const float *g_lik, int B, int N, int E, float *g_enc,
                                             float *g_x, float *g_params, void *workspace, void *stream);

/* Backward of the NN measurement's likelihood head (kind NFDPF_MEAS_NN; training, SURVEY.md
 * §8(f1)): lik = log sigmoid(likelihood_est([enc, PE(x)])) (model/models.py:221-235, the MLP of
 * :119-128).  Gradients stop at the particle encodings; the caller chains g_e through
 * nfdpf_particle_encoder mode 1.
 *   meas_params: the likelihood_est blob of nfdpf_measurement (NN); enc [B, E] frame encodings;
 *   e_particles [B*N, E] = PE(x) (nfdpf_particle_encoder mode 0); g_lik [B, N]
 *   g_e [B*N, E], g_enc [B, E]; g_params [8385]: likelihood_est's gradient in the plain
 *   nn.Linear layout W1 b1 W2 b2 W3 b3
 *   workspace: nfdpf_nn_measurement_backward_workspace(B, N) bytes (fixed-order partials) */
NFDPF_API int64_t nfdpf_nn_measurement_backward_workspace(int B, int N);
NFDPF_API int nfdpf_nn_measurement_backward(const float *meas_params, const float *enc, const float *e_particles,
                                            const float *g_lik, int B, int N, int E, float *g_e, float *g_enc,
                                            float *g_params, void *workspace, void *stream);

/* Conditional-GLOW measurement (model/models.py:280-303; nf/cglow/CGlowModel.py with the
 * default flow_depth K = 1, L = 1, x_size = y_size = (3,8,8)): particle (b,i) at
 * x + b*x_rs + 2i, frame encoding of row b at enc + b*enc_rs (192 floats) -> the RAW
 * likelihood -nll at lik + b*lik_rs + i (the row-max shift of :301-302 is the caller's:
 * the filter's EXTERNAL-measurement phase 2, or measurement_model_cglow).
 * pe_params: particle encoder 2->16->32->192 (encoder layout above); glow_params:
 * nfdpf_cglow_params_size(K) floats (layout: nfdpf.pack.cglow_tensors). */
NFDPF_API int64_t nfdpf_cglow_params_size(int K);
NFDPF_API int nfdpf_cglow_measurement(const float *pe_params, const float *glow_params, int K,
                            const float *enc, int64_t enc_rs, const float *x, int64_t x_rs,
                            int B, int N, float *lik, int64_t lik_rs, void *stream);

/* CondGlowModel.forward(x, y) (nf/cglow/CGlowModel.py:167-176) with the reference's default
 * configuration (K = 1, L = 1, learn_top off, 256 bins): x [M,3,8,8] the condition, y [M,3,8,8]
 * the flow input, both per sample -> z [M,12,4,4] (NULL: not written) and nll [M]
 * (= -(log-det + Gaussian log-prob) / (192 log 2)).  glow_params as nfdpf_cglow_measurement. */
NFDPF_API int nfdpf_cglow_flow(const float *glow_params, int K, const float *x, const float *y, int64_t M,
                               float *z, float *nll, void *stream);

/* Backward of the two CGLOW entry points above (training; the autograd
 * gradient of nf/cglow/modules.py + CGlowModel.py:167-176, d log|det W| / dW = W^-T).
 * Deterministic (fixed-order per-workgroup partials in the workspace, reduced in order).
 *   nfdpf_cglow_measurement_backward: inputs as nfdpf_cglow_measurement, g_lik (b, i) at
 *     g_lik + b*glik_rs + i = dL/d(raw lik) -> g_x [B, N, 2], g_y [B*N, 192] = dL/d(frame
 *     encoding) per particle (the caller sums each row's N), g_glow (glow blob layout),
 *     g_pe (encoder blob layout).
 *   nfdpf_cglow_flow_backward: inputs as nfdpf_cglow_flow, g_z [M, 192] (NULL = 0), g_nll [M]
 *     -> g_x, g_y [M, 192], g_glow.
 *   workspace: nfdpf_cglow_backward_workspace(B*N or M) bytes. */
NFDPF_API int64_t nfdpf_cglow_backward_workspace(int64_t M);
NFDPF_API int nfdpf_cglow_measurement_backward(const float *pe_params, const float *glow_params, int K,
                                               const float *enc, int64_t enc_rs, const float *x, int64_t x_rs,
                                               int B, int N, const float *g_lik, int64_t glik_rs, float *g_x,
                                               float *g_y, float *g_glow, float *g_pe, void *workspace,
                                               void *stream);
NFDPF_API int nfdpf_cglow_flow_backward(const float *glow_params, int K, const float *x, const float *y, int64_t M,
                                        const float *g_z, const float *g_nll, float *g_x, float *g_y,
                                        float *g_glow, void *workspace, void *stream);

/* Backward of nfdpf_maf_stack (training): g_out [rows, dim] = dL/d(output), g_logdet [rows]
 * (either may be NULL = 0) -> g_x [rows, dim] = dL/dx and g_params = dL/d(blob), the blob's
 * layout.  dim 2 or 4, hidden 8, n_flows <= 4 (dim 4: <= 2).  workspace: caller-owned,
 * nfdpf_maf_stack_backward_workspace bytes (-1 = unsupported sizes).  Deterministic.      */
NFDPF_API int64_t nfdpf_maf_stack_backward_workspace(int n_flows, int dim, int hidden, int64_t rows);
NFDPF_API int nfdpf_maf_stack_backward(const float *params, int n_flows, int dim, int hidden, const float *x,
                                       int64_t rows, int inverse, const float *g_out, const float *g_logdet,
                                       float *g_x, float *g_params, void *workspace, void *stream);

/* Block pseudo-likelihood of the semi-supervised objective (compute_block_density_nf,
 * losses.py:37-68) on the filter histories w, lik, prior [B,T,N] and the ancestor index
 * [B,T,N] (int64, flat into B*N): Q [B] (fp64) = the reference's Q / number of blocks.
 * Backward: g_Q [B] -> g_w, g_lik, g_prior [B,T,N]; the ancestor maps must be non-decreasing
 * over the flattened batch (the filter's always are: nfdpf_pseudo_lik_check sets *ok = 0
 * otherwise; *ok must be 1 on entry).  workspace: nfdpf_pseudo_lik_workspace bytes.        */
NFDPF_API int nfdpf_pseudo_lik_forward(const float *w, const float *lik, const float *prior, const int64_t *index,
                                       int B, int T, int N, int block_len, double *Q, void *stream);
NFDPF_API int64_t nfdpf_pseudo_lik_workspace(int B, int T, int N, int block_len);
NFDPF_API int nfdpf_pseudo_lik_check(const int64_t *index, int B, int T, int N, int32_t *ok, void *stream);
NFDPF_API int nfdpf_pseudo_lik_backward(const float *w, const float *lik, const float *prior, const int64_t *index,
                                        int B, int T, int N, int block_len, const float *g_Q, float *g_w,
                                        float *g_lik, float *g_prior, void *workspace, void *stream);

/* The rational-quadratic spline of the neural spline flows NSF_AR / NSF_CL (nf/flows.py:343-458)
 * on M elements with K bins each: RQS (nf/utils.py:55-147) on [left, right] x [bottom, top],
 * or, with tails = 1, unconstrained_RQS (:23-53): inputs outside [left, right] pass through
 * with log-det 0.  W, H: [M, K] unnormalised widths / heights; D: [M, K + 1] unnormalised
 * derivatives (full_derivatives = 1) or [M, K - 1] inner ones with the reference's constant at
 * both ends (0).  Out: y [M], logdet [M] (inverse = 1: the inverse map and its log-det).      */
NFDPF_API int nfdpf_rqs(const float *x, const float *W, const float *H, const float *D, int64_t M, int K,
                        int full_derivatives, int inverse, float left, float right, float bottom, float top,
                        int tails, float min_bin_width, float min_bin_height, float min_derivative, float *y,
                        float *logdet, void *stream);

/* particle_initialization (utils.py:46-62) in DEVICE rng mode:
 * uniform on [-width/2, width/2)^2 (or start + N(0,1) when true_state)        */
NFDPF_API int nfdpf_particle_init(const float *start_xy, int B, int N, float width, int true_state,
                        uint64_t seed, int64_t row_base, float *x, float *logw, void *stream);

/* torch.sum(x, -1) of each row of x [B][N] in ATen's CPU cascade order (the soft resampler's
 * q.sum() and w.sum(), resamplers.py:33-34, 56) -> out [B]: variant 0 the generic device sum,
 * 1 the one-launch pass's load-ahead sum for 8 <= N <= 1024 (same additions, same bits).  A test
 * probe of the bit-exact resampler's building block; no reference counterpart. */
NFDPF_API int nfdpf_cascade_row_sum(const float *x, int B, int N, int variant, float *out, void *stream);

/* One iteration of the T loop of DPF.filtering_pos (DPFs.py:160-214), fused:
 * ESS gate (batch-global, read from ess_all) -> [soft resample | OT result] -> motion ->
 * nf_dyn inverse -> NF proposal -> nf_dyn forward -> densities -> measurement ->
 * weight update -> normalise(+1e-12) -> inverse-ESS term, writing history slot t.
 * One workgroup per batch row.                                                    */
typedef struct nfdpf_filter_desc {
  /* sizes */
  int32_t B, N, T, E;       /* local rows, particles, history length, frame-encoding width */
  int32_t B_global;         /* rows whose inverse-ESS terms gate resampling (all ranks) */
  int32_t t;                /* step index */
  int32_t phase;            /* 0 = whole step; 1 = up to the proposal (EXTERNAL measurement
                               runs next on hist_x slot t); 2 = from the likelihood on */
  int64_t row_base;         /* global row of local row 0 (flat index base = N*row_base) */
  /* configuration */
  int32_t nf_dyn, nf_cond, measurement, resampler, rng_mode, force_resample, n_flows,
      hidden;
  int32_t defer_norm;       /* tiled step: normalise step t's weights inside step t+1's first
                               launch (p_prev / x_prev = history slot t-1, not yet normalised);
                               the caller clears it for the last step and to feed p_prev itself */
  int32_t split_nets;       /* tiled step: dyn_params / cond_params carry the split suffix
                               (below) and nf_dyn is RealNVP -- the coupling nets then run on
                               wave pairs (t-nets and s-nets on separate waves) */
  float alpha, pos_noise, dens_const, meas_prior_std;
  uint64_t seed;
  /* packed parameters */
  const float *dyn_params, *cond_params, *pe_params, *meas_params;
  /* inputs */
  const float *enc;         /* [B,T,E] frame encodings */
  const float *vel;         /* [B,2] velocity used by this step's motion */
  const float *lin;         /* [N] soft-resampler markers base (host torch.linspace) */
  const float *host_noise;  /* [B,N,2] parity-mode noise of this step (rng_mode HOST) */
  const float *host_offsets;/* [B] parity-mode offsets (rng_mode HOST, soft; read only when the
                               host-decided gate fires -- NULL there falls back to Philox) */
  const float *x_prev;      /* particles after the previous step, rows of x_prev_rs */
  const float *p_prev;      /* probabilities after the previous step, rows of p_prev_rs */
  int64_t x_prev_rs, p_prev_rs;
  const float *ess_all;     /* [B_global] 1/sum(p_prev^2) per row (tiled: see below) */
  const int32_t *gate;      /* optional [1]: precomputed gate (OT path), NULL = compute */
  const float *ot_x;        /* [B,N,2] OT-resampled particles (resampler OT, gate on) */
  const float *lik_ext;     /* [B,N] raw likelihood (measurement EXTERNAL) */
  /* outputs: history [B,T,...] slot t, plus per-step reductions */
  float *hist_x, *hist_p, *hist_noise, *hist_lik, *hist_jac, *hist_prior;
  int64_t *hist_idx;
  float *ess_out;           /* [B] 1/sum(p^2) of this step (tiled: see below) */
  float *lw_sum;            /* [B,T] row sums of the unnormalised log-weights (obs likelihood) */
  float *pred;              /* [B,T,2] sum_n p*x (losses.py:18-31 prediction) */
  float *scratch;           /* [2][B,N,4] per-particle hand-off between stages (x_dyn, propose, prior),
                               indexed by step parity: step t's values must not overwrite step t-1's,
                               which the deferred normalisation of slot t-1 reads during step t */
  void *prof_events;        /* optional hipEvent_t[2]: live kernel timing of the dominant launch
                               -- recorded around the whole step for nfdpf_filter_step; carried
                               by the proposal+measurement launch's own dispatch
                               (hipExtLaunchKernel: its begin / end timestamps) for
                               nfdpf_filter_step_tiled */
  int32_t ess_local;        /* tiled: 1 = ess_all holds this shard's B rows only (row b at b), the
                               gate coming from `gate` -- the speculative-gate mode of a sharded
                               batch (nfdpf_ess_gate_tiled_batch verifies it after the pass) */
  int32_t prof_front;       /* tiled, with prof_events: 1 = prof_events is hipEvent_t[4] and events
                               [2], [3] ride in the front launch's dispatch (ESS gate + resampling +
                               motion [+ nf_dyn]: the resampler's launch) */
  /* nfdpf_filter_pass_tiled only (NULL / 0 elsewhere): */
  int32_t pass_gate;        /* 0 = every ESS gate taken as off (speculative; verified after the
                               pass), 1 = the batch-global gate decided inside the launch at every
                               step (DPFs.py:163-165; needs B_global == B) */
  int32_t *pass_gates;      /* optional [T] out: step t's gate -- the in-launch decisions
                               (pass_gate 1) or the verification of a speculative pass */
  int32_t *pass_flags;      /* optional [3] out: {gates that fired, wave hand-off faults since the
                               last read (nfdpf_split_fault's counter, read and cleared), 1 written
                               last with a system-scope release (a completion word: host-mapped
                               flags can be waited on without a stream operation)} */
  float *pass_obs;          /* optional [1] out: the obs-likelihood sum_t mean_{b,n} logw (DPFs.py:191) */
  int32_t meas_mfma;        /* 1 = meas_params is the CRNVP measurement's MFMA fragment blob (encoder
                               included, pe_params unused by the measurement; nfdpf.pack.
                               crnvp_mfma_tensors, csrc/crnvp_mfma.hpp; n_flows <= 2): the features-
                               by-particles layout of the f32-MFMA measurement, read by the no-flow
                               one-launch pass (tiled_pass_cm_kernel); 0 = the pair layout above */
  const int32_t *pass_plan; /* nfdpf_filter_pass_tiled with pass_gate = 1, optional [T]: the ESS gate
                               decisions to follow instead of deciding them inside the launch (the
                               "plan" pass: step t resamples iff pass_plan[t]; no batch-wide
                               exchange, so a sharded batch (B_global != B) and a batch of more rows
                               than the device holds at once run it too).  With pass_gates and the
                               whole batch (B_global == B) the epilogue writes the ACTUAL gates of
                               the trajectory (from the pass's own partials) to pass_gates and
                               counts the steps where they differ from the plan in pass_flags[0];
                               the caller reruns with a corrected plan -- the result is the
                               reference's only when no step differs */
  void **gate_peers;        /* nfdpf_filter_pass_tiled with pass_gate = 1 on a sharded batch
                               (B_global != B, B_global <= 512), optional [gate_world] device array:
                               every rank's gate-exchange buffer (nfdpf_gate_xchg_alloc, the peers'
                               mapped by nfdpf_gate_xchg_open; entry gate_rank is this rank's own).
                               Each step, each row's 1 / sum p^2 goes to every rank's buffer (one
                               tagged 8-byte granule, system scope) and each rank sweeps its own
                               buffer's B_global granules in global row order: the batch-global
                               gate decided inside every rank's launch, identically (DPFs.py:163-165)
                               -- the gated pass sharded.  Every rank's pass must run concurrently
                               (the sweeps wait for each other; a wait that times out counts a
                               hand-off fault as a non-resident grid does) */
  int32_t gate_world;       /* ranks in gate_peers */
  int32_t gate_rank;        /* this rank's index in gate_peers */
} nfdpf_filter_desc;

NFDPF_API int nfdpf_filter_step(const nfdpf_filter_desc *d, void *stream);

/* The same step as a pipeline of launches over (particle tile of 256, batch row) workgroups
 * (gate + resample + motion -> dyn inverse -> proposal+measurement [-> normalise]), so a small
 * batch fills every CU.  In this mode ess_out / ess_all hold the per-(row, tile) softmax
 * partials of the step's log-weights u as 4 doubles {max u, sum e^(u-max), sum e^(2(u-max)),
 * max raw likelihood} ([B][tiles][4] / [B_global][tiles][4]; nfdpf_filter_tiled_tiles(N)
 * tiles per row): the next step's ESS gate and normalisation both derive from them.
 * pred / lw_sum are written after the last step (t == T-1) for all steps at once.
 * workspace: nfdpf_filter_tiled_workspace_bytes(B, N, T) bytes, 256-B aligned, shared by
 * the T steps of one sequence.                                                        */
NFDPF_API int64_t nfdpf_filter_tiled_workspace_bytes(int B, int N, int T);
NFDPF_API int nfdpf_filter_tiled_tiles(int N);
/* 1 when nfdpf_filter_step_tiled runs this step as ONE launch (tiled_step_fused_kernel: the
 * C2-shaped path -- split RealNVP nets, NF_cond, cosine measurement -- with every workgroup of
 * the (tiles, B) grid resident on the current device; opt-in: NFDPF_FUSED_STEP=1), else 0.
 * prof_front is then ignored (no separate front launch).  No reference counterpart: a query. */
NFDPF_API int nfdpf_filter_tiled_fused(const nfdpf_filter_desc *d);
/* sizeof(nfdpf_filter_desc) as this library was built: a binding checks its mirror of the
 * struct against it (nfdpf._lib does, at load).  No reference counterpart: a query. */
NFDPF_API int64_t nfdpf_filter_desc_size(void);
/* The WHOLE T-step pass (DPFs.py:160-214, all of filtering_pos's loop) as one persistent launch,
 * for a pass whose every ESS gate is taken as off (the speculative-gate mode: the caller verifies
 * the T gates afterwards with nfdpf_ess_gate_tiled_batch over ess_out, and reruns the pass step
 * by step with nfdpf_filter_step_tiled if one fired).  Replaces the T iterations of
 * nfdpf_filter_step_tiled (+ the last normalisation and the pred / lw_sum reduction) for the
 * configuration nfdpf_filter_pass_supported accepts: split RealNVP nf_dyn, NF_cond, the cosine
 * measurement, device RNG, N <= 1024, n_flows <= 2, the soft resampler when forced (every step
 * then resamples inside the launch and there is no gate to verify), B <= 256, and a (tiles, B)
 * grid of 1024-thread workgroups that is resident on the current device all at once -- except a
 * speculative or forced C2-shaped pass, which runs more rows than fit as consecutive launches
 * of resident rows, the last rows first (e.g. 96 rows of N = 1000 on 256 CUs: rows 64-95, then
 * 0-63); the C3-shaped pass needs all its rows resident (above that its step launches are faster).
 * Descriptor fields as nfdpf_filter_step_tiled at t = 0, except:
 *   dyn_params / cond_params: the PASS layout (nfdpf.pack.pass_flow_tensors: the pair layout with
 *   the tanh algebra folded into the weights -- W1, b1 x c, W2 x -2c, b2 -> c (b2 + rowsum W2),
 *   W3 x -2, b3 -> b3 + rowsum W3, c = 2 log2 e; no split suffix);
 *   x_prev / p_prev: the initial particles / probabilities;  vel: [T][B][2], every step's velocity;
 *   ess_all: [B][tiles][4], the initial partials (nfdpf_filter_tiled_init; step 0's gate input);
 *   ess_out: [T][B][tiles][4], step t's softmax partials (the gates' input; the next step's
 *   partials in include/nfdpf.h's tiled layout);  gate / scratch / defer_norm: unused;
 *   pass_gate / pass_gates / pass_flags / pass_obs: above (pass_gates with pass_gate 0 asks for
 *   the verification of a speculative pass of the whole batch, B_global == B);
 *   prof_events: optional hipEvent_t[2] riding in the pass launch's own dispatch.
 * Every history slot, pred and lw_sum are written as after the T steps of the tiled path.
 * workspace: nfdpf_filter_pass_workspace_bytes(B, N, T) bytes, 256-B aligned, ZEROED by the
 * caller when it is new or its (B, N, T) changed (its first 256 bytes carry the granule tags'
 * epoch from pass to pass).  A wait between the row's workgroups that times out is counted in
 * nfdpf_split_fault / pass_flags[1] (the outputs are then invalid).  No reference counterpart
 * for the query / workspace functions. */
NFDPF_API int nfdpf_filter_pass_supported(const nfdpf_filter_desc *d);
NFDPF_API int64_t nfdpf_filter_pass_workspace_bytes(int B, int N, int T);
NFDPF_API int nfdpf_filter_pass_tiled(const nfdpf_filter_desc *d, void *workspace, void *stream);
/* the t = 0 gate input from p0 [B,N] -> ess_parts [B][tiles][4] */
NFDPF_API int nfdpf_filter_tiled_init(const float *p0, int B, int N, double *ess_parts,
                            void *stream);
/* nfdpf_particle_init + nfdpf_normalize_log_probs (add 0) + nfdpf_filter_tiled_init in ONE launch
 * (one workgroup per row, N <= 1024), bit-identical to the three: particle_initialization
 * (utils.py:46-62, device RNG; start: [B][start_rs >= 4] rows of the start state, x, y, vx, vy)
 * -> x [B,N,2], logw [B,N]; p0 = normalize_log_probs(logw) (DPFs.py:153) -> p [B,N], inv_ess [B]
 * (nullable); the t = 0 gate input -> ess_parts [B][tiles][4]; and (vel nullable) every step's
 * velocity in the descriptor's [T][B][2] layout: the start velocity, then vel_in[b][t - 1][2]
 * (rows of vel_rs floats; DPFs.py:158, 173). */
NFDPF_API int nfdpf_filter_init(const float *start, int start_rs, const float *vel_in, int vel_rs, int T, int B,
                                int N, float width, int true_state, uint64_t seed, int64_t row_base, float *x,
                                float *logw, float *p, float *inv_ess, double *ess_parts, float *vel, void *stream);
/* Pinned, device-mapped, coherent host memory (hipHostMalloc Mapped | Coherent, zeroed): *host for
 * the caller, *dev for kernel arguments -- e.g. pass_flags, written by the pass epilogue with
 * system-scope stores and read on the host once an event behind the pass has completed (no copy
 * launch).  No reference counterpart. */
NFDPF_API int nfdpf_host_mapped_alloc(int64_t bytes, void **host, void **dev);
NFDPF_API int nfdpf_host_mapped_free(void *host);
/* The cross-rank gate exchange of the sharded gated pass (nfdpf_filter_desc.gate_peers): each rank
 * allocates one buffer of nfdpf_gate_xchg_bytes(B_global) bytes in uncached device memory
 * (zeroed; a 256-B header whose first word is the exchange's pass epoch, then [2][B_global]
 * tagged granules), exports it as a 64-byte IPC handle, and maps every peer's buffer from its
 * handle (hipIpcOpenMemHandle; over xGMI on one node).  close unmaps a peer's buffer, free
 * releases this rank's own.  Replaces the per-step all-gather of the gate partials (DPFs.py:163:
 * the batch-global mean) for the one-launch pass.  No reference counterpart. */
NFDPF_API int64_t nfdpf_gate_xchg_bytes(int B_global);
NFDPF_API int nfdpf_gate_xchg_alloc(int64_t bytes, void **dev, void *ipc_handle);
NFDPF_API int nfdpf_gate_xchg_open(const void *ipc_handle, void **dev);
NFDPF_API int nfdpf_gate_xchg_close(void *dev);
NFDPF_API int nfdpf_gate_xchg_free(void *dev);
NFDPF_API int nfdpf_filter_step_tiled(const nfdpf_filter_desc *d, void *workspace, void *stream);
/* the ESS gate (DPFs.py:163-165) of step t from the [B][tiles][4] partials of step t-1
 * -> int32 [1] (OT path) */
NFDPF_API int nfdpf_ess_gate_tiled(const double *parts, int B, int N, int t, int force, int32_t *gate,
                         void *stream);
/* The tiled gate of T steps at once: parts [T][B_global][tiles][4] (step t's input partials,
 * i.e. the previous step's outputs gathered over the shards) -> gates [T] int32 (step t uses
 * the +1e-12 terms iff t0 + t > 0).  Verifies a speculative pass (every gate assumed off). */
NFDPF_API int nfdpf_ess_gate_tiled_batch(const double *parts, int T, int B, int N, int t0, int force,
                                         int32_t *gates, void *stream);
/* The verification of a one-shard speculative pass, stream-ordered (capturable in a graph, no
 * host synchronisation): the T gates as nfdpf_ess_gate_tiled_batch (not forced) -> gates [T];
 * flags [2] int32 = {how many of the T gates fired, the wave hand-off fault count since the last
 * read -- nfdpf_split_fault's counter, read and cleared on the device}; obs [1] = the
 * obs-likelihood sum_t (sum_b lw_sum[b][t]) / (B N) (DPFs.py:191) from the pass's lw_sum [B][T].
 * The caller reads flags once after the pass.  No reference counterpart (the reference checks
 * each gate as it goes, DPFs.py:163-165). */
NFDPF_API int nfdpf_pass_verify(const double *parts, const float *lw_sum, int T, int B, int N, int t0,
                                int32_t *gates, int32_t *flags, float *obs, void *stream);
/* The verification of a SHARDED speculative pass from one small all-gather: each rank reduces its
 * [T][B][tiles][4] step partials to the rows' gate terms terms[t * B + b] = 1 / sum p^2 of row b at
 * step t (tiled_gate_batch_kernel's per-row arithmetic; the +1e-12 terms iff t0 + t > 0) and puts
 * its hand-off fault counter (read and cleared, as an int32) in terms[T * B]; after the ranks'
 * term arrays are gathered in global row order, nfdpf_ess_gate_terms takes the T batch-global
 * gates (DPFs.py:163-165: ATen's cascade mean over the B_global rows) from terms [T][B_global].
 * Bit-identical to nfdpf_ess_gate_tiled_batch on the gathered partials, at 1 / (4 tiles x 4)
 * of the gathered bytes.  No reference counterpart. */
NFDPF_API int nfdpf_ess_row_terms(const double *parts, int T, int B, int N, int t0, float *terms, void *stream);
NFDPF_API int nfdpf_ess_gate_terms(const float *terms, int T, int B, int N, int force, int32_t *gates, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* NFDPF_H */
