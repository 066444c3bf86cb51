// filter_step.hip -- one iteration of the T loop of DPF.filtering_pos (DPFs.py:160-214),
// fused into ONE launch per step for the soft / no-resample path.
//
// One workgroup owns one batch row for the whole step, because every stage of the step
// is coupled through a per-row reduction:
//   ESS gate (batch mean, DPFs.py:163-165) -> soft resampling (row scan, resamplers.py:20-60)
//   -> motion (model/models.py:191-204) -> mean/std(x_phys) -> nf_dyn inverse (:305-332)
//   -> mean/std(x_dyn) -> NF proposal inverse (:334-356) -> nf_dyn forward + densities
//   (:358-377) -> measurement (:206-278; CRNVP/gaussian subtract a row max) -> log-weight
//   update (DPFs.py:187) -> row max / sum -> p + 1e-12 (:192) -> 1/sum p^2 (next gate).
// The per-row contexts ([mean, std], [enc, mean, std]) enter only the first layer of every
// coupling net, so they are folded once per row into a bias (fold_bias) and each particle
// pays just its own coordinate's column.
//
// Between stages a particle's intermediates are parked in its own history slot (written
// and re-read by the same lane, L1/L2-resident) and in `scratch`; the stage order and all
// reductions are fixed, so results do not depend on timing or placement.
#include "soft.hpp"
#include "stages.hpp"

namespace nfdpf {

// ESS gate (DPFs.py:163-165): every workgroup evaluates the same expression
__device__ __forceinline__ bool step_gate(const nfdpf_filter_desc &d) {
  if (d.gate) return d.gate[0] != 0;
  if (d.force_resample) return true;
  // torch.mean over the batch (ATen cascade order); every wave evaluates it
  const float *ess = d.ess_all;
  const float s = cascade_row_sum([&](int i) { return ess[i]; }, d.B_global);
  return (s / (float)d.B_global) < 0.5f * (float)d.N;
}

// Soft resampling of row b (resamplers.py:20-60) into slot t: hx = x_res, hp = w' (not yet
// renormalised), hidx.  Returns S2 = the cascade sum of w' (the renormaliser).  `Cbuf` is
// LDS of N floats.  All threads of the workgroup call it.
__device__ float soft_row(const nfdpf_filter_desc &d, const RowSlot &S, int b, int64_t grow,
                          const float *xprev, const float *pprev, float *Cbuf, StepShared &L) {
  const int N = d.N;
  float off;
  if (d.rng_mode == NFDPF_RNG_HOST && d.host_offsets)
    off = d.host_offsets[b];
  else
    off = u01(rng_draw(d.seed, kTagOffset, (uint32_t)d.t, grow, 0u).x) * (1.0f / (float)N);
  SoftRow row{pprev, N, d.alpha, 1.0f / (float)N, (float)(1.0 - (double)d.alpha), 1.0f};
  const int64_t flat0 = (int64_t)N * grow;
  soft_row_search(row, d.lin, off, Cbuf, L.d, L.f, [&](int i, int src) {
    const float *xs;
    float w;
    if (src < N) {
      xs = xprev + 2 * src;
      w = row.w(src);
    } else if (b + 1 < d.B) {  // reference edge: flat index N*(b+1) is the next row
      xs = xprev + d.x_prev_rs;
      w = 0.f;
    } else {
      xs = xprev + 2 * (N - 1);
      w = 0.f;
    }
    S.hx[2 * i] = xs[0];
    S.hx[2 * i + 1] = xs[1];
    S.hp[i] = w;
    S.hidx[i] = flat0 + src;
  });
  __syncthreads();
  if (threadIdx.x < 64) {
    const float s = cascade_row_sum([&](int j) { return S.hp[j]; }, N);
    if (threadIdx.x == 0) L.bc[0] = s;
  }
  __syncthreads();
  return L.bc[0];
}

template <int BLK, bool NFD, bool NFC, int MEAS>
__global__ __launch_bounds__(BLK) void filter_step_kernel(const nfdpf_filter_desc d) {
  extern __shared__ float Cbuf[];
  __shared__ StepShared L;
  const int b = blockIdx.x, tid = threadIdx.x, N = d.N;
  const int64_t grow = d.row_base + b;
  const RowSlot S = row_slot(d, b);
  const int nfl = d.n_flows;

  if (d.phase != 2) {
    if (MEAS != NFDPF_MEAS_EXTERNAL) measure_row_setup<MEAS>(S.enc, d.meas_params, L);
    const bool fire = step_gate(d);
    const int mode = !fire ? kSrcPrev : (d.resampler == NFDPF_RESAMPLE_SOFT ? kSrcSoft : kSrcOt);
    const float *xprev = d.x_prev + b * d.x_prev_rs;
    const float *pprev = d.p_prev + b * d.p_prev_rs;
    const float S2 = mode == kSrcSoft ? soft_row(d, S, b, grow, xprev, pprev, Cbuf, L) : 1.f;

    // ---------------- motion + mean/std of x_phys
    const float v0 = d.vel[2 * b], v1 = d.vel[2 * b + 1];
    const float lr_ot = logf(1.0f / (float)N);
    double s0 = 0, s1 = 0, q0 = 0, q1 = 0;
    for (int i = tid; i < N; i += BLK) {
      float p0, p1;
      stage_motion(d, S, b, grow, i, mode, xprev, pprev, S2, lr_ot, v0, v1, p0, p1);
      s0 += p0;
      s1 += p1;
      q0 += (double)p0 * p0;
      q1 += (double)p1 * p1;
    }
    auto row_ctx = [&](double a0, double a1, double b0, double b1) {
      a0 = block_sum(a0, L.d);
      a1 = block_sum(a1, L.d);
      b0 = block_sum(b0, L.d);
      b1 = block_sum(b1, L.d);
      return ctx_from_sums(a0, a1, b0, b1, N);
    };
    Ctx4 cphys{0.f, 0.f, 0.f, 0.f};
    if (NFD || NFC) cphys = row_ctx(s0, s1, q0, q1);

    // ---------------- nf_dyn inverse (model/models.py:305-332)
    if (NFD) {
      fold_dyn(d.dyn_params, nfl, cphys, L.cb_dyn, d.nf_dyn);
      __syncthreads();
      s0 = s1 = q0 = q1 = 0;
      for (int i = tid; i < N; i += BLK) {
        float x0, x1;
        stage_dyn_inverse(d, S, i, S.hx[2 * i], S.hx[2 * i + 1], L.cb_dyn, x0, x1);
        s0 += x0;
        s1 += x1;
        q0 += (double)x0 * x0;
        q1 += (double)x1 * x1;
      }
    }
    // ---------------- proposal context [enc, mean, std] (model/models.py:334-346)
    if (NFC) {
      const Ctx4 cp = NFD ? row_ctx(s0, s1, q0, q1) : cphys;
      if (tid < d.E) L.ctx[tid] = S.enc[tid];
      if (tid == 0) {
        L.ctx[d.E] = cp.m0;
        L.ctx[d.E + 1] = cp.m1;
        L.ctx[d.E + 2] = cp.s0;
        L.ctx[d.E + 3] = cp.s1;
      }
      __syncthreads();
      fold_cond(d.cond_params, nfl, d.E, L.ctx, L.cb_cond);
    }
    __syncthreads();
    float lmax = -INFINITY;
    for (int i = tid; i < N; i += BLK) {
      float q0x, q1x, propose, prior;
      const float lk = stage_proposal<NFD, NFC, MEAS>(d, S, L, i, load_prop_in<NFD>(S, i), L.cb_dyn,
                                                      L.cb_cond, q0x, q1x, propose, prior);
      if (MEAS != NFDPF_MEAS_EXTERNAL) {
        S.hlik[i] = lk;
        lmax = fmaxf(lmax, lk);
      }
    }
    if (d.phase == 1) return;
    if (MEAS == NFDPF_MEAS_CRNVP || MEAS == NFDPF_MEAS_GAUSSIAN) L.bc[1] = block_max(lmax, L.f);
  }

  // ---------------- likelihood -> log-weights (DPFs.py:187-191)
  float lshift = 0.f;
  if (MEAS == NFDPF_MEAS_EXTERNAL) {
    const float *lx = d.lik_ext + (int64_t)b * N;
    float m = -INFINITY;
    for (int i = tid; i < N; i += BLK) m = fmaxf(m, lx[i]);
    lshift = block_max(m, L.f);
  } else if (MEAS == NFDPF_MEAS_CRNVP || MEAS == NFDPF_MEAS_GAUSSIAN) {
    lshift = L.bc[1];
  }
  float wmax = -INFINITY;
  double wsum = 0.0;
  for (int i = tid; i < N; i += BLK) {
    float lk = MEAS == NFDPF_MEAS_EXTERNAL ? d.lik_ext[(int64_t)b * N + i] : S.hlik[i];
    if (meas_shifted<MEAS>()) {
      lk = lk - lshift;
      S.hlik[i] = lk;
    }
    const float lw = stage_logw(S, i, lk);
    S.hp[i] = lw;
    wmax = fmaxf(wmax, lw);
    wsum += lw;
  }
  wmax = block_max(wmax, L.f);
  wsum = block_sum(wsum, L.d);
  // ---------------- normalize_log_probs(...) + 1e-12 (utils.py:39-44, DPFs.py:192)
  double es = 0.0;
  for (int i = tid; i < N; i += BLK) {
    const float e = expf(S.hp[i] - wmax);
    S.hp[i] = e;
    es += e;
  }
  const float Ssum = (float)block_sum(es, L.d);
  double sp2 = 0.0, px = 0.0, py = 0.0;
  for (int i = tid; i < N; i += BLK) {
    const float p = S.hp[i] / Ssum + 1e-12f;
    S.hp[i] = p;
    sp2 += (double)p * p;
    px += (double)p * S.hx[2 * i];
    py += (double)p * S.hx[2 * i + 1];
  }
  sp2 = block_sum(sp2, L.d);
  px = block_sum(px, L.d);
  py = block_sum(py, L.d);
  if (tid == 0) {
    d.ess_out[b] = 1.0f / (float)sp2;
    const int64_t bt = (int64_t)b * d.T + d.t;
    d.lw_sum[bt] = (float)wsum;
    d.pred[2 * bt] = (float)px;
    d.pred[2 * bt + 1] = (float)py;
  }
}

template <int BLK, bool NFD, bool NFC, int MEAS>
static int launch_step(const nfdpf_filter_desc &d, hipStream_t st) {
  const size_t lds = (d.resampler == NFDPF_RESAMPLE_SOFT && d.phase != 2) ? d.N * sizeof(float) : 0;
  hipEvent_t *ev = (hipEvent_t *)d.prof_events;
  if (ev) (void)hipEventRecord(ev[0], st);
  filter_step_kernel<BLK, NFD, NFC, MEAS><<<d.B, BLK, lds, st>>>(d);
  if (ev) (void)hipEventRecord(ev[1], st);
  return launch_status("nfdpf_filter_step");
}

template <int BLK, int MEAS>
static int dispatch_nf(const nfdpf_filter_desc &d, hipStream_t st) {
  if (d.nf_dyn && d.nf_cond) return launch_step<BLK, true, true, MEAS>(d, st);
  if (d.nf_dyn) return launch_step<BLK, true, false, MEAS>(d, st);
  if (d.nf_cond) return launch_step<BLK, false, true, MEAS>(d, st);
  return launch_step<BLK, false, false, MEAS>(d, st);
}

}  // namespace nfdpf

using namespace nfdpf;

extern "C" int nfdpf_filter_step(const nfdpf_filter_desc *dp, void *stream) {
  NFDPF_REQUIRE(dp, "nfdpf_filter_step: null descriptor");
  const nfdpf_filter_desc &d = *dp;
  NFDPF_REQUIRE(d.B >= 0 && d.N >= 2 && d.T >= 1 && d.t >= 0 && d.t < d.T,
                "nfdpf_filter_step: bad sizes (B=%d N=%d T=%d t=%d); N >= 2 (std needs N-1)",
                d.B, d.N, d.T, d.t);
  NFDPF_REQUIRE(d.phase >= 0 && d.phase <= 2, "nfdpf_filter_step: bad phase");
  NFDPF_REQUIRE(!d.meas_mfma, "nfdpf_filter_step: the MFMA fragment blob (meas_mfma) is for the tiled launches");
  NFDPF_REQUIRE(d.n_flows >= 0 && d.n_flows <= kMaxFlows, "nfdpf_filter_step: n_flows <= %d",
                kMaxFlows);
  NFDPF_REQUIRE(d.hidden == kH, "nfdpf_filter_step: FCNN hidden width must be %d", kH);
  NFDPF_REQUIRE(d.hist_x && d.hist_p && d.hist_noise && d.hist_lik && d.hist_idx && d.scratch &&
                    d.ess_out && d.lw_sum && d.pred && d.enc && d.vel,
                "nfdpf_filter_step: null output/input pointer");
  NFDPF_REQUIRE(d.phase == 2 || (d.x_prev && d.p_prev && (d.gate || d.force_resample || d.ess_all)),
                "nfdpf_filter_step: previous-step state missing");
  NFDPF_REQUIRE(!d.nf_dyn || (d.dyn_params && d.hist_jac && d.hist_prior),
                "nfdpf_filter_step: nf_dyn needs dyn_params, hist_jac, hist_prior");
  NFDPF_REQUIRE(d.nf_dyn >= NFDPF_DYN_NONE && d.nf_dyn <= NFDPF_DYN_MAF, "nfdpf_filter_step: bad nf_dyn %d",
                d.nf_dyn);
  NFDPF_REQUIRE(!d.nf_cond || d.cond_params, "nfdpf_filter_step: nf_cond needs cond_params");
  NFDPF_REQUIRE(d.measurement == NFDPF_MEAS_EXTERNAL || (d.E == kE && d.pe_params),
                "nfdpf_filter_step: fused measurements need E == %d and pe_params (got E=%d)", kE,
                d.E);
  NFDPF_REQUIRE(!(d.measurement == NFDPF_MEAS_CRNVP || d.measurement == NFDPF_MEAS_NN) ||
                    d.meas_params,
                "nfdpf_filter_step: measurement parameters missing");
  NFDPF_REQUIRE(d.E + 4 <= kMaxCtx, "nfdpf_filter_step: E=%d too large (<= %d)", d.E, kMaxCtx - 4);
  NFDPF_REQUIRE(d.measurement != NFDPF_MEAS_EXTERNAL || d.phase != 0,
                "nfdpf_filter_step: EXTERNAL measurement runs as phase 1 + phase 2");
  NFDPF_REQUIRE(d.measurement != NFDPF_MEAS_EXTERNAL || d.phase != 2 || d.lik_ext,
                "nfdpf_filter_step: phase 2 needs lik_ext");
  if (d.resampler == NFDPF_RESAMPLE_SOFT) {
    NFDPF_REQUIRE(d.N <= kStepMaxN, "nfdpf_filter_step: soft resampling supports N <= %d",
                  kStepMaxN);
    NFDPF_REQUIRE(d.lin || d.phase == 2, "nfdpf_filter_step: soft resampling needs lin");
    NFDPF_REQUIRE(d.rng_mode == NFDPF_RNG_DEVICE || d.gate || d.phase == 2,
                  "nfdpf_filter_step: HOST rng mode needs the host-decided gate (host_offsets are "
                  "read only when it fires)");
  } else {
    NFDPF_REQUIRE(d.ot_x || d.phase == 2, "nfdpf_filter_step: OT path needs ot_x");
  }
  NFDPF_REQUIRE(d.rng_mode == NFDPF_RNG_DEVICE || d.host_noise || d.phase == 2,
                "nfdpf_filter_step: HOST rng mode needs host_noise");
  if (d.B == 0) return NFDPF_OK;
  hipStream_t st = as_stream(stream);
  switch (d.measurement) {
    case NFDPF_MEAS_COS: return dispatch_nf<512, NFDPF_MEAS_COS>(d, st);
    case NFDPF_MEAS_CRNVP: return dispatch_nf<256, NFDPF_MEAS_CRNVP>(d, st);
    case NFDPF_MEAS_GAUSSIAN: return dispatch_nf<512, NFDPF_MEAS_GAUSSIAN>(d, st);
    case NFDPF_MEAS_NN: return dispatch_nf<256, NFDPF_MEAS_NN>(d, st);
    case NFDPF_MEAS_EXTERNAL: return dispatch_nf<512, NFDPF_MEAS_EXTERNAL>(d, st);
  }
  set_error("nfdpf_filter_step: unknown measurement %d", d.measurement);
  return NFDPF_EINVAL;
}
