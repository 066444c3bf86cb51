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
#include "measure.hpp"
#include "soft.hpp"

namespace nfdpf {

struct Ctx4 {
  float m0, m1, s0, s1;  // per-row [mean, std] context (model/models.py:309-315)
};

template <int BLK, bool NFD, bool NFC, int MEAS>
__global__ __launch_bounds__(BLK) void filter_step_kernel(const nfdpf_filter_desc d) {
  extern __shared__ float Cbuf[];
  __shared__ StepShared L;
  const int b = blockIdx.x, tid = threadIdx.x, N = d.N;
  const int64_t grow = d.row_base + b;
  const int64_t flat0 = (int64_t)N * grow;
  const int64_t hrow = ((int64_t)b * d.T + d.t) * N;
  float *hx = d.hist_x + hrow * 2;
  float *hp = d.hist_p + hrow;
  float *hlik = d.hist_lik + hrow;
  float *hnoise = d.hist_noise + hrow * 2;
  int64_t *hidx = d.hist_idx + hrow;
  float *hjac = d.hist_jac ? d.hist_jac + hrow : nullptr;
  float *hprior = d.hist_prior ? d.hist_prior + hrow : nullptr;
  float *scr = d.scratch + (int64_t)b * N * 4;  // per particle: x_dyn0, x_dyn1, propose, prior
  const float K = d.dens_const;
  const float two_var = 2.0f * (d.pos_noise * d.pos_noise);
  const int nfl = d.n_flows;
  const float *enc = d.enc + ((int64_t)b * d.T + d.t) * d.E;

  if (d.phase != 2) {
    // ---------------- frame encoding of this row (+ per-row measurement constants)
    if (MEAS != NFDPF_MEAS_EXTERNAL) measure_row_setup<MEAS>(enc, d.meas_params, L);
    // ---------------- ESS gate (DPFs.py:163-165), identical in every workgroup
    bool fire;
    if (d.gate) {
      fire = d.gate[0] != 0;
    } else if (d.force_resample) {
      fire = true;
    } else {
      float s = 0.f;
      for (int i = 0; i < d.B_global; ++i) s += d.ess_all[i];
      fire = (s / (float)d.B_global) < 0.5f * (float)N;
    }
    const bool soft = fire && d.resampler == NFDPF_RESAMPLE_SOFT;
    const bool ot = fire && d.resampler == NFDPF_RESAMPLE_OT;
    const float *xprev = d.x_prev + b * d.x_prev_rs;
    const float *pprev = d.p_prev + b * d.p_prev_rs;

    float S2 = 1.f;
    if (soft) {
      float off;
      if (d.rng_mode == NFDPF_RNG_HOST && d.host_offsets)
        off = d.host_offsets[b];
      else
        off = u01(rng_draw(d.seed, kTagOffset, (uint32_t)d.t, grow, 0u).x) * (1.0f / (float)N);
      SoftRow row{pprev, N, d.alpha, 1.0f / (float)N, (float)(1.0 - (double)d.alpha), 1.0f};
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
        hx[2 * i] = xs[0];
        hx[2 * i + 1] = xs[1];
        hp[i] = w;
        hidx[i] = flat0 + src;
      });
      __syncthreads();
      if (tid < 64) {
        const float s = cascade_row_sum([&](int j) { return hp[j]; }, N);
        if (tid == 0) L.bc[0] = s;
      }
      __syncthreads();
      S2 = L.bc[0];
    }

    // ---------------- motion (model/models.py:191-204) + mean/std of x_phys
    const float v0 = d.vel[2 * b], v1 = d.vel[2 * b + 1];
    const float lr_ot = logf(1.0f / (float)N);
    double s0 = 0, s1 = 0, q0 = 0, q1 = 0;
    for (int i = tid; i < N; i += BLK) {
      float x0, x1, lr;
      if (soft) {
        x0 = hx[2 * i];
        x1 = hx[2 * i + 1];
        lr = logf(hp[i] / S2);
      } else {
        if (ot) {
          x0 = d.ot_x[((int64_t)b * N + i) * 2];
          x1 = d.ot_x[((int64_t)b * N + i) * 2 + 1];
          lr = lr_ot;
        } else {
          x0 = xprev[2 * i];
          x1 = xprev[2 * i + 1];
          lr = logf(pprev[i]);
        }
        hidx[i] = flat0 + i;
      }
      float e0, e1;
      if (d.rng_mode == NFDPF_RNG_HOST) {
        e0 = d.host_noise[((int64_t)b * N + i) * 2];
        e1 = d.host_noise[((int64_t)b * N + i) * 2 + 1];
      } else {
        const U4 r = rng_draw(d.seed, kTagMotion, (uint32_t)d.t, grow, (uint32_t)i);
        box_muller(r.x, r.y, e0, e1);
        e0 *= d.pos_noise;
        e1 *= d.pos_noise;
      }
      const float p0 = (x0 + v0) + e0, p1 = (x1 + v1) + e1;
      hnoise[2 * i] = e0;
      hnoise[2 * i + 1] = e1;
      hx[2 * i] = p0;
      hx[2 * i + 1] = p1;
      hp[i] = lr;
      s0 += p0;
      s1 += p1;
      q0 += (double)p0 * p0;
      q1 += (double)p1 * p1;
    }
    // context [mean, std(unbiased)] (model/models.py:309-315); reductions in f64
    auto row_ctx = [&](double a0, double a1, double b0, double b1) {
      a0 = block_sum(a0, L.d);
      a1 = block_sum(a1, L.d);
      b0 = block_sum(b0, L.d);
      b1 = block_sum(b1, L.d);
      const double m0 = a0 / N, m1 = a1 / N;
      return Ctx4{(float)m0, (float)m1, (float)sqrt((b0 - a0 * m0) / (N - 1)),
                  (float)sqrt((b1 - a1 * m1) / (N - 1))};
    };
    Ctx4 c4{0.f, 0.f, 0.f, 0.f};
    if (NFD || NFC) c4 = row_ctx(s0, s1, q0, q1);
    const float cdyn[4] = {c4.m0, c4.m1, c4.s0, c4.s1};

    // ---------------- nf_dyn inverse (model/models.py:305-332)
    constexpr int inD = 1 + 4;
    const int nsD = fcnn_size<kH>(inD, 1);
    if (NFD) {
      if (tid < nfl * 4 * kH) {
        const int f = tid / (4 * kH), n = (tid / kH) & 3, j = tid % kH;
        L.cb_dyn[tid] = fold_bias_c<kH, 4>(d.dyn_params + (int64_t)(f * 4 + n) * nsD, inD, 1, j, cdyn);
      }
      __syncthreads();
      s0 = s1 = q0 = q1 = 0;
      for (int i = tid; i < N; i += BLK) {
        float lo[1] = {hx[2 * i]}, up[1] = {hx[2 * i + 1]};
        float ld = 0.f;
        for (int f = nfl - 1; f >= 0; --f)
          ld += coupling_inverse<1, kH>(opaque(d.dyn_params) + (int64_t)f * 4 * nsD, inD, lo, up,
                                        L.cb_dyn + f * 4 * kH);
        scr[4 * i] = lo[0];
        scr[4 * i + 1] = up[0];
        if (hjac) hjac[i] = -ld;
        s0 += lo[0];
        s1 += up[0];
        q0 += (double)lo[0] * lo[0];
        q1 += (double)up[0] * up[0];
      }
    }

    // ---------------- proposal + densities + measurement (model/models.py:334-379)
    const int inC = 1 + d.E + 4;
    const int nsC = fcnn_size<kH>(inC, 1);
    if (NFC) {
      const Ctx4 cp = NFD ? row_ctx(s0, s1, q0, q1) : c4;
      const float cprop[4] = {cp.m0, cp.m1, cp.s0, cp.s1};
      if (tid < d.E) L.ctx[tid] = enc[tid];
      if (tid == 0) {
        L.ctx[d.E] = cprop[0];
        L.ctx[d.E + 1] = cprop[1];
        L.ctx[d.E + 2] = cprop[2];
        L.ctx[d.E + 3] = cprop[3];
      }
      __syncthreads();
      if (tid < nfl * 4 * kH) {
        const int f = tid / (4 * kH), n = (tid / kH) & 3, j = tid % kH;
        L.cb_cond[tid] =
            fold_bias<kH>(d.cond_params + (int64_t)(f * 4 + n) * nsC, inC, 1, j, L.ctx, d.E + 4);
      }
    }
    __syncthreads();
    float lmax = -INFINITY;
    for (int i = tid; i < N; i += BLK) {
      const float p0 = hx[2 * i], p1 = hx[2 * i + 1];
      const float e0 = hnoise[2 * i], e1 = hnoise[2 * i + 1];
      float xd0 = p0, xd1 = p1, jac = 0.f;
      if (NFD) {
        xd0 = scr[4 * i];
        xd1 = scr[4 * i + 1];
        jac = hjac ? hjac[i] : 0.f;
      }
      const float de = density(e0, e1, K, two_var);
      float q0x = xd0, q1x = xd1, prior, propose;
      if (NFC) {
        float lo[1] = {xd0}, up[1] = {xd1};
        float ld = 0.f;
        for (int f = nfl - 1; f >= 0; --f)
          ld += coupling_inverse<1, kH>(opaque(d.cond_params) + (int64_t)f * 4 * nsC, inC, lo, up,
                                        L.cb_cond + f * 4 * kH);
        q0x = lo[0];
        q1x = up[0];
        const float jac_prop = -ld;
        const float r0 = p0 - e0, r1 = p1 - e1;
        if (NFD) {
          float ld2 = 0.f;
          for (int f = 0; f < nfl; ++f)
            ld2 += coupling_forward<1, kH>(opaque(d.dyn_params) + (int64_t)f * 4 * nsD, inD, lo, up,
                                           L.cb_dyn + f * 4 * kH);
          prior = density(lo[0] - r0, up[0] - r1, K, two_var) - (-ld2);
        } else {
          prior = density(q0x - r0, q1x - r1, K, two_var);
        }
        propose = (de + jac) + jac_prop;
      } else {
        prior = de + jac;
        propose = de + jac;
      }
      hx[2 * i] = q0x;
      hx[2 * i + 1] = q1x;
      scr[4 * i + 2] = propose;
      scr[4 * i + 3] = prior;
      if (hprior) hprior[i] = prior;
      if (MEAS != NFDPF_MEAS_EXTERNAL) {
        const float lk = measure<MEAS>(MeasArgs{d.pe_params, d.meas_params, d.n_flows, d.meas_prior_std}, L, q0x, q1x);
        hlik[i] = lk;
        lmax = fmaxf(lmax, lk);
      }
    }
    if (d.phase == 1) return;
    // row max of the raw likelihood for the models that subtract it (model/models.py:276,301)
    if (MEAS == NFDPF_MEAS_CRNVP || MEAS == NFDPF_MEAS_GAUSSIAN)
      L.bc[1] = block_max(lmax, L.f);
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
    float lk = MEAS == NFDPF_MEAS_EXTERNAL ? d.lik_ext[(int64_t)b * N + i] : hlik[i];
    if (MEAS == NFDPF_MEAS_EXTERNAL || MEAS == NFDPF_MEAS_CRNVP || MEAS == NFDPF_MEAS_GAUSSIAN) {
      lk = lk - lshift;
      hlik[i] = lk;
    }
    const float lw = ((hp[i] + lk) + scr[4 * i + 3]) - scr[4 * i + 2];
    hp[i] = lw;
    wmax = fmaxf(wmax, lw);
    wsum += lw;
  }
  wmax = block_max(wmax, L.f);
  wsum = block_sum(wsum, L.d);
  // ---------------- normalize_log_probs(...) + 1e-12 (utils.py:39-44, DPFs.py:192)
  double es = 0.0;
  for (int i = tid; i < N; i += BLK) {
    const float e = expf(hp[i] - wmax);
    hp[i] = e;
    es += e;
  }
  const float S = (float)block_sum(es, L.d);
  double sp2 = 0.0, px = 0.0, py = 0.0;
  for (int i = tid; i < N; i += BLK) {
    const float p = hp[i] / S + 1e-12f;
    hp[i] = p;
    sp2 += (double)p * p;
    px += (double)p * hx[2 * i];
    py += (double)p * hx[2 * i + 1];
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
  filter_step_kernel<BLK, NFD, NFC, MEAS><<<d.B, BLK, lds, st>>>(d);
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
