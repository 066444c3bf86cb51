// stages.hpp -- per-particle stages of one filtering step (DPFs.py:160-192), shared by the
// row-per-workgroup fused kernel (filter_step.hip) and the tiled multi-CU kernels
// (filter_tiled.hip).  Each stage reads / writes the particle's own history slot t, so a
// stage may run in a different launch than the one before it.
#pragma once

#include "measure.hpp"

namespace nfdpf {

struct Ctx4 {
  float m0, m1, s0, s1;  // per-row [mean, std (unbiased)] context (model/models.py:309-315)
};

// Row-local pointers into history slot t and the scratch row.
struct RowSlot {
  float *hx, *hp, *hlik, *hnoise, *hjac, *hprior, *scr;  // scr: x_dyn0, x_dyn1, propose, prior
  int64_t *hidx;
  const float *enc;
};

__device__ __forceinline__ RowSlot row_slot(const nfdpf_filter_desc &d, int b, int t) {
  const int64_t hrow = ((int64_t)b * d.T + t) * d.N;
  RowSlot s;
  s.hx = d.hist_x + hrow * 2;
  s.hp = d.hist_p + hrow;
  s.hlik = d.hist_lik + hrow;
  s.hnoise = d.hist_noise + hrow * 2;
  s.hidx = d.hist_idx + hrow;
  s.hjac = d.hist_jac ? d.hist_jac + hrow : nullptr;
  s.hprior = d.hist_prior ? d.hist_prior + hrow : nullptr;
  s.scr = d.scratch + ((int64_t)(t & 1) * d.B + b) * d.N * 4;  // double-buffered by step parity
  s.enc = d.enc + ((int64_t)b * d.T + t) * d.E;
  return s;
}
__device__ __forceinline__ RowSlot row_slot(const nfdpf_filter_desc &d, int b) { return row_slot(d, b, d.t); }

// context from (sum x, sum y, sum x^2, sum y^2) over N particles: mean = s / N and std =
// sqrt((q - s mean) / (N - 1)) as products with the fp64 reciprocals 1 / N, 1 / (N - 1) (the
// one-launch pass's chain takes them from registers: no fp64 division on its critical path)
__device__ __forceinline__ double ctx_mean(double s, double inv_n) { return s * inv_n; }
__device__ __forceinline__ double ctx_var(double s, double q, double m, double inv_n1) { return (q - s * m) * inv_n1; }
__device__ __forceinline__ Ctx4 ctx_from_sums(double a0, double a1, double b0, double b1, int N) {
  const double inv_n = 1.0 / N, inv_n1 = 1.0 / (N - 1);
  const double m0 = ctx_mean(a0, inv_n), m1 = ctx_mean(a1, inv_n);
  return Ctx4{(float)m0, (float)m1, (float)sqrt(ctx_var(a0, b0, m0, inv_n1)), (float)sqrt(ctx_var(a1, b1, m1, inv_n1))};
}

// source of the particle before motion
enum SrcMode { kSrcPrev = 0, kSrcSoft = 1, kSrcOt = 2 };

// motion (model/models.py:191-204) of a particle whose resampled state (x0, x1, log p) is
// known: x_phys = (x_res + vel) + eps, eps ~ N(0, pos_noise^2).  Writes hx = x_phys,
// hnoise = eps, hp = log p_res.
// the motion noise eps of particle i (model/models.py:200-202): device Philox or the
// uploaded parity-mode draw
__device__ __forceinline__ void motion_noise(const nfdpf_filter_desc &d, int b, int64_t grow, int i, float &e0,
                                             float &e1) {
  if (d.rng_mode == NFDPF_RNG_HOST) {
    e0 = d.host_noise[((int64_t)b * d.N + i) * 2];
    e1 = d.host_noise[((int64_t)b * d.N + i) * 2 + 1];
  } else {
    const U4 r = rng_draw(d.seed, kTagMotion, (uint32_t)d.t, grow, (uint32_t)i);
    box_muller(r.x, r.y, e0, e1);
    e0 *= d.pos_noise;
    e1 *= d.pos_noise;
  }
}

__device__ __forceinline__ void motion_apply_eps(const RowSlot &S, int i, float x0, float x1, float lr, float v0,
                                                 float v1, float e0, float e1, float &p0, float &p1) {
  p0 = (x0 + v0) + e0;
  p1 = (x1 + v1) + e1;
  S.hnoise[2 * i] = e0;
  S.hnoise[2 * i + 1] = e1;
  S.hx[2 * i] = p0;
  S.hx[2 * i + 1] = p1;
  S.hp[i] = lr;
}

__device__ __forceinline__ void motion_apply(const nfdpf_filter_desc &d, const RowSlot &S, int b,
                                             int64_t grow, int i, float x0, float x1, float lr,
                                             float v0, float v1, float &p0, float &p1) {
  float e0, e1;
  motion_noise(d, b, grow, i, e0, e1);
  p0 = (x0 + v0) + e0;
  p1 = (x1 + v1) + e1;
  S.hnoise[2 * i] = e0;
  S.hnoise[2 * i + 1] = e1;
  S.hx[2 * i] = p0;
  S.hx[2 * i + 1] = p1;
  S.hp[i] = lr;
}

// motion from the particle's source: kSrcSoft = resampled into slot t by the fused step's
// soft stage (hx = x_res, hp = unnormalised w', renormaliser S2); kSrcOt = the OT result;
// kSrcPrev = the previous step's particle (no resampling).  Also writes hidx for the
// non-soft modes (the soft stage wrote its own).
__device__ __forceinline__ void stage_motion(const nfdpf_filter_desc &d, const RowSlot &S, int b,
                                             int64_t grow, int i, int mode, const float *xprev,
                                             const float *pprev, float S2, float lr_ot, float v0,
                                             float v1, float &p0, float &p1) {
  const int N = d.N;
  float x0, x1, lr;
  if (mode == kSrcSoft) {
    x0 = S.hx[2 * i];
    x1 = S.hx[2 * i + 1];
    lr = logf(S.hp[i] / S2);
  } else {
    if (mode == kSrcOt) {
      x0 = d.ot_x[((int64_t)b * N + i) * 2];
      x1 = d.ot_x[((int64_t)b * N + i) * 2 + 1];
      lr = lr_ot;
    } else {
      x0 = xprev[2 * i];
      x1 = xprev[2 * i + 1];
      lr = logf(pprev[i]);
    }
    S.hidx[i] = (int64_t)N * grow + i;
  }
  motion_apply(d, S, b, grow, i, x0, x1, lr, v0, v1, p0, p1);
}

constexpr int kOctxDyn = 4;  // nf_dyn context [mean(2), std(2)]
constexpr int kNsDyn = net_size<1, kH>(kOctxDyn);  // pairs per coupling half
constexpr int kMafDyn = maf_size<kH>(2);           // floats per MAF flow of the dynamic stack

// Folded first-layer bias of one float of the [flow][half][j][t|s] table, thread tid:
// b1 + sum_c W1[j, 1 + c] ctx[c], accumulated in column order.  fold_acc adds the columns
// [c0, c1) to a running value, so a fold can be split across launches (the encoding columns
// of the proposal context are known before the row statistics) without changing the
// fma sequence.  The per-lane weight address is not uniform: generic loads, a few per row.
struct FoldRef {
  const float *w1c;
  int j, w;
};

__device__ __forceinline__ FoldRef fold_ref(const float *flows, int ns, int tid) {
  const int f = tid / (4 * kH), r = tid % (4 * kH);
  const int n = r / (2 * kH);
  return FoldRef{flows + 2 * ((f * 2 + n) * ns + net_core<1, kH>()), (r >> 1) % kH, r & 1};
}
__device__ __forceinline__ float fold_bias0(const FoldRef &r, int O) { return r.w1c[2 * (kH * O + r.j) + r.w]; }

__device__ __forceinline__ float fold_acc(const FoldRef &r, int O, float a, const float *ctx, int c0, int c1) {
  const float *wr = r.w1c + 2 * r.j * O + r.w;
  int c = c0;
  for (; c + 12 <= c1; c += 12) {  // 12 weight loads in flight, then the fmas in order
    float wv[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) wv[q] = wr[2 * (c + q)];
#pragma unroll
    for (int q = 0; q < 12; ++q) a = fmaf(wv[q], ctx[c + q - c0], a);
  }
  for (; c < c1; ++c) a = fmaf(wr[2 * c], ctx[c - c0], a);
  return a;
}

// fold_acc with the next 12 weights in flight while the current 12 are accumulated (the same
// fma sequence): for the long folds (the proposal's 192 encoding columns), whose 16 batches
// would otherwise each wait a full load latency
__device__ __forceinline__ float fold_acc_pipe(const FoldRef &r, int O, float a, const float *ctx, int c0, int c1) {
  const float *wr = r.w1c + 2 * r.j * O + r.w;
  int c = c0;
  if (c + 12 <= c1) {
    float wa[12], wb[12];
#pragma unroll
    for (int q = 0; q < 12; ++q) wa[q] = wr[2 * (c + q)];
    for (; c + 24 <= c1; c += 24) {
#pragma unroll
      for (int q = 0; q < 12; ++q) wb[q] = wr[2 * (c + 12 + q)];
#pragma unroll
      for (int q = 0; q < 12; ++q) a = fmaf(wa[q], ctx[c + q - c0], a);
      if (c + 36 <= c1) {
#pragma unroll
        for (int q = 0; q < 12; ++q) wa[q] = wr[2 * (c + 24 + q)];
      }
#pragma unroll
      for (int q = 0; q < 12; ++q) a = fmaf(wb[q], ctx[c + 12 + q - c0], a);
    }
    if (c + 12 <= c1) {  // an odd batch left in wa
#pragma unroll
      for (int q = 0; q < 12; ++q) a = fmaf(wa[q], ctx[c + q - c0], a);
      c += 12;
    }
  }
  for (; c < c1; ++c) a = fmaf(wr[2 * c], ctx[c - c0], a);
  return a;
}

__device__ __forceinline__ float fold_one(const float *flows, int ns, int O, int tid, const float *ctx) {
  const FoldRef r = fold_ref(flows, ns, tid);
  return fold_acc(r, O, fold_bias0(r, O), ctx, 0, O);
}

// per-row fold of the nf_dyn context into the first-layer biases (model/models.py:309-315)
__device__ __forceinline__ void fold_dyn(const float *dyn, int nfl, const Ctx4 &c, f2 *cb, int kind) {
  const int tid = threadIdx.x;
  if (kind == NFDPF_DYN_REALNVP && tid < nfl * 4 * kH) {  // MAF takes no context
    const float cc[4] = {c.m0, c.m1, c.s0, c.s1};
    reinterpret_cast<float *>(cb)[tid] = fold_one(dyn, kNsDyn, kOctxDyn, tid, cc);
  }
}

// per-row fold of the proposal context [enc, mean, std] (model/models.py:338-346); ctx in LDS
__device__ __forceinline__ void fold_cond(const float *cond, int nfl, int E, const float *ctx, f2 *cb) {
  const int tid = threadIdx.x;
  if (tid < nfl * 4 * kH)
    reinterpret_cast<float *>(cb)[tid] = fold_one(cond, net_size<1, kH>(E + 4), E + 4, tid, ctx);
}

// nf_dyn inverse (model/models.py:305-332) of x_phys = (x0, x1): writes scr x_dyn and hjac
__device__ __forceinline__ void stage_dyn_inverse(const nfdpf_filter_desc &d, const RowSlot &S, int i,
                                                  float x0, float x1, const f2 *cb, float &xd0,
                                                  float &xd1) {
  float lo[1] = {x0}, up[1] = {x1};
  float ld = 0.f;
  if (d.nf_dyn == NFDPF_DYN_MAF) {
    // NormalizingFlowModel.inverse over MAF flows, last flow first (nf/models.py:23-30)
    float v[2] = {x0, x1};
    for (int f = d.n_flows - 1; f >= 0; --f) ld += maf_inverse<2, kH>(wptr(d.dyn_params) + f * kMafDyn, v);
    lo[0] = v[0];
    up[0] = v[1];
  } else {
    for (int f = d.n_flows - 1; f >= 0; --f)
      ld += coupling_inverse<1, kH>(wptr2(d.dyn_params) + f * 2 * kNsDyn, kOctxDyn, lo, up,
                                    cb + f * 2 * kH);
  }
  S.scr[4 * i] = lo[0];
  S.scr[4 * i + 1] = up[0];
  if (S.hjac) S.hjac[i] = -ld;
  xd0 = lo[0];
  xd1 = up[0];
}

// Per-particle inputs of the proposal stage, loaded up front so the loads overlap the
// per-row prologue (context folds) instead of following it.
struct PropIn {
  float p0, p1, e0, e1, xd0, xd1, jac;
};

template <bool NFD>
__device__ __forceinline__ PropIn load_prop_in(const RowSlot &S, int i) {
  PropIn a;
  a.p0 = S.hx[2 * i];
  a.p1 = S.hx[2 * i + 1];
  a.e0 = S.hnoise[2 * i];
  a.e1 = S.hnoise[2 * i + 1];
  a.xd0 = a.p0;
  a.xd1 = a.p1;
  a.jac = 0.f;
  if (NFD) {
    a.xd0 = S.scr[4 * i];
    a.xd1 = S.scr[4 * i + 1];
    a.jac = S.hjac ? S.hjac[i] : 0.f;
  }
  return a;
}

// NF proposal inverse (model/models.py:334-356): q = cond_model.inverse(x_dyn, [enc, mean, std]),
// returns jac_prop = -log_det (0 and q = x_dyn without --NF-cond).
template <bool NFC>
__device__ __forceinline__ float stage_propose_inverse(const nfdpf_filter_desc &d, const PropIn &in,
                                                       const f2 *cb_cond, float &q0x, float &q1x) {
  q0x = in.xd0;
  q1x = in.xd1;
  if (!NFC) return 0.f;
  const int oC = d.E + 4;
  const int nsC = net_size<1, kH>(oC);
  float lo[1] = {in.xd0}, up[1] = {in.xd1};
  float ld = 0.f;
#ifndef NFDPF_EXP_NOCOND
  for (int f = d.n_flows - 1; f >= 0; --f)
    ld += coupling_inverse<1, kH>(wptr2(d.cond_params) + f * 2 * nsC, oC, lo, up, cb_cond + f * 2 * kH);
#endif
  q0x = lo[0];
  q1x = up[0];
  return -ld;
}

// nf_dyn forward of the proposal + densities (model/models.py:358-377): (propose, prior);
// writes hx = proposal, scr propose/prior, hprior.
template <bool NFD, bool NFC>
__device__ __forceinline__ void stage_prior(const nfdpf_filter_desc &d, const RowSlot &S, int i,
                                            const PropIn &in, const f2 *cb_dyn, float q0x, float q1x,
                                            float jac_prop, float &propose, float &prior) {
  const float K = d.dens_const;
  const float two_var = 2.0f * (d.pos_noise * d.pos_noise);
  const int nfl = d.n_flows;
  const float de = density(in.e0, in.e1, K, two_var);
  if (NFC) {
    const float r0 = in.p0 - in.e0, r1 = in.p1 - in.e1;
    if (NFD) {
      float lo[1] = {q0x}, up[1] = {q1x};
      float ld2 = 0.f;
#ifndef NFDPF_EXP_NODYNF
      if (d.nf_dyn == NFDPF_DYN_MAF) {
        // NormalizingFlowModel.forward over MAF flows (nf/models.py:13-21)
        float v[2] = {lo[0], up[0]};
        for (int f = 0; f < nfl; ++f) ld2 += maf_forward<2, kH>(wptr(d.dyn_params) + f * kMafDyn, v);
        lo[0] = v[0];
        up[0] = v[1];
      } else {
        for (int f = 0; f < nfl; ++f)
          ld2 += coupling_forward<1, kH>(wptr2(d.dyn_params) + f * 2 * kNsDyn, kOctxDyn, lo, up,
                                         cb_dyn + f * 2 * kH);
      }
#endif
      prior = density(lo[0] - r0, up[0] - r1, K, two_var) - (-ld2);
    } else {
      prior = density(q0x - r0, q1x - r1, K, two_var);
    }
    propose = (de + in.jac) + jac_prop;
  } else {
    prior = de + in.jac;
    propose = de + in.jac;
  }
  S.hx[2 * i] = q0x;
  S.hx[2 * i + 1] = q1x;
  S.scr[4 * i + 2] = propose;
  S.scr[4 * i + 3] = prior;
  if (S.hprior) S.hprior[i] = prior;
}

template <int MEAS>
__device__ __forceinline__ float stage_measure(const nfdpf_filter_desc &d, const StepShared &L, float q0x,
                                               float q1x) {
#ifdef NFDPF_EXP_NOMEAS
  return q0x * 1e-3f;
#endif
  if (MEAS != NFDPF_MEAS_EXTERNAL)
    return measure<MEAS>(MeasArgs{d.pe_params, d.meas_params, d.n_flows, d.meas_prior_std}, L, q0x, q1x);
  return 0.f;
}

// The whole proposal stage for one particle: inverse, prior/propose, measurement.  Returns the
// raw likelihood (0 for an EXTERNAL measurement).
template <bool NFD, bool NFC, int MEAS>
__device__ __forceinline__ float stage_proposal(const nfdpf_filter_desc &d, const RowSlot &S,
                                                const StepShared &L, int i, const PropIn &in,
                                                const f2 *cb_dyn, const f2 *cb_cond, float &q0x,
                                                float &q1x, float &propose, float &prior) {
  const float jp = stage_propose_inverse<NFC>(d, in, cb_cond, q0x, q1x);
  stage_prior<NFD, NFC>(d, S, i, in, cb_dyn, q0x, q1x, jp, propose, prior);
  return stage_measure<MEAS>(d, L, q0x, q1x);
}

// log-weight from registers: ((log p_res + lik) + prior) - propose
__device__ __forceinline__ float logw(float lr, float lik, float prior, float propose) {
  return ((lr + lik) + prior) - propose;
}

// log-weight update (DPFs.py:187): ((log p_res + lik) + prior) - propose
__device__ __forceinline__ float stage_logw(const RowSlot &S, int i, float lik) {
  return ((S.hp[i] + lik) + S.scr[4 * i + 3]) - S.scr[4 * i + 2];
}

template <int MEAS>
__host__ __device__ constexpr bool meas_shifted() {
  // measurement models that subtract the row max of the raw likelihood (model/models.py:276,301)
  return MEAS == NFDPF_MEAS_CRNVP || MEAS == NFDPF_MEAS_GAUSSIAN || MEAS == NFDPF_MEAS_EXTERNAL;
}

}  // namespace nfdpf
