// measure.hpp -- per-particle measurement models (model/models.py:206-278) and the per-row
// shared state of the fused filter step.
#pragma once

#include "flows.hpp"

namespace nfdpf {

constexpr int kH = 8;           // FCNN hidden width (nf/flows.py:183, fixed by the reference)
constexpr int kMaxFlows = 4;    // n_sequence (DPFs.py:46) is 2
constexpr int kE = 32;          // frame-encoding width of the fused measurements (--hiddensize)
constexpr int kNnH = 64;        // likelihood_est width (model/models.py:119-128)
constexpr int kStepMaxN = 12288;  // soft resampler C[] in LDS
constexpr int kMaxCtx = 260;      // proposal context [enc (E <= 256), mean, std]

struct StepShared {
  f2 cb_dyn[kMaxFlows * 2 * kH];   // folded bias pairs [flow][coupling half][j] of nf_dyn
  f2 cb_cond[kMaxFlows * 2 * kH];  // ... of the proposal flow
  float ctx[kMaxCtx];
  alignas(16) float encv[kE];  // this row's frame encoding (raw; 16-B aligned: crnvp_lik_mfma's b128 reads)
  double vinv;          // cos: 1 / max(|encv|, 1e-12), fp64
  float nnrow[kNnH];    // NN: folded first layer of the obs half
  float f[16];
  double d[16];
  float bc[4];
};

__device__ __forceinline__ float density(float e0, float e1, float K, float two_var) {
#pragma clang fp contract(off)
  // compute_normal_density (utils.py:22-37) with D = 2: K - (e0^2/(2s^2) + e1^2/(2s^2))
  return K - (e0 * e0 / two_var + e1 * e1 / two_var);
}

struct MeasArgs {
  const float *pe_params, *meas_params;
  int n_flows;
  float meas_prior_std;
};

// measurement_model_cnf (model/models.py:256-278): flow input = the row's frame encoding encv,
// condition = the particle encoding; N(0, prior_std^2 I) prior + log-det.  pe / mp: the encoder
// and flow blobs behind constant-address-space pointers (scalar loads) or plain pointers into
// LDS (tiled_prop_kernel stages them per workgroup) -- the same arithmetic either way.
template <class WF>
__device__ __forceinline__ float crnvp_lik(WF pe, WF mp, int n_flows, float prior_std, const float *encv,
                                           float x0, float x1) {
  float e[kE];
  particle_encode<kE>(pe, x0, x1, e);
  constexpr int HALF = kE / 2;
  constexpr int ns = net_size<HALF, kH>(kE);
  float lo[HALF], up[HALF];
#pragma unroll
  for (int k = 0; k < HALF; ++k) {
    lo[k] = encv[k];
    up[k] = encv[HALF + k];
  }
  float ld = 0.f;
  for (int f = 0; f < n_flows; ++f) {
    const auto fw = pair_ptr(mp) + f * 2 * ns;
    f2 cb[2 * kH];
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int j = 0; j < kH; ++j) cb[n * kH + j] = fold_pair_c<HALF, kH, kE>(fw + n * ns, j, e);
    ld += coupling_forward<HALF, kH>(fw, kE, lo, up, cb);
  }
  // the prior's quadratic form in fp64 (32 terms of ~10 each: fp32 lost ~1e-4 absolute)
  const double is = 1.0 / (double)prior_std;
  double m = 0.0;
#pragma unroll
  for (int k = 0; k < HALF; ++k) {
    const double a = lo[k] * is, c = up[k] * is;
    m = fma(a, a, m);
    m = fma(c, c, m);
  }
  const double lp = -0.5 * (kE * 1.8378770664093453 + m) - kE * log((double)prior_std);
  return (float)(lp + (double)ld);
}

template <int MEAS>
__device__ __forceinline__ float measure(const MeasArgs &d, const StepShared &L, float x0,
                                         float x1) {
  if constexpr (MEAS == NFDPF_MEAS_COS) {
    // measurement_model_cosine_distance + et_distance (model/models.py:206-219, utils.py:8-15)
    // <e/|e|, v/|v|> computed as <e, v>/(|e| |v|) in fp64 (flows.hpp cos_lik)
    double ss, dot;
    encode_dot<kE>(wptr(d.pe_params), x0, x1, L.encv, ss, dot);
    return cos_lik(ss, dot, L.vinv);
  } else if constexpr (MEAS == NFDPF_MEAS_CRNVP) {
    return crnvp_lik(wptr(d.pe_params), wptr(d.meas_params), d.n_flows, d.meas_prior_std, L.encv, x0, x1);
  } else if constexpr (MEAS == NFDPF_MEAS_GAUSSIAN) {
    // measurement_model_Gaussian with N(1, 100 I) (DPFs.py:84-86, model/models.py:237-254)
    float e[kE];
    particle_encode<kE>(wptr(d.pe_params), x0, x1, e);
    float m = 0.f;
#pragma unroll
    for (int j = 0; j < kE; ++j) {
      const float v = (L.encv[j] - e[j] - 1.0f) * 0.1f;
      m = fmaf(v, v, m);
    }
    return -0.5f * (kE * 1.8378770664093453f + m) - kE * 2.302585092994046f;
  } else if constexpr (MEAS == NFDPF_MEAS_NN) {
    // measurement_model_NN (model/models.py:221-235): sigmoid(MLP([enc_obs, enc_particle])).log()
    float e[kE];
    particle_encode<kE>(wptr(d.pe_params), x0, x1, e);
    // W1 [64, 2E] and W2 [64, 64] in row_pairs layout, W3 [1, 64] and biases plain
    cfloat *P = wptr(d.meas_params);
    cf2 *W1 = (cf2 *)P;
    f2 h[kNnH / 2];
#pragma unroll
    for (int m = 0; m < kNnH / 2; ++m) {
      f2 a = f2{L.nnrow[2 * m], L.nnrow[2 * m + 1]};
#pragma unroll
      for (int k = 0; k < kE; ++k) a = pfma(W1[m * 2 * kE + kE + k], splat(e[k]), a);
      h[m] = relu2(a);
    }
    cf2 *W2 = (cf2 *)(P + kNnH * 2 * kE + kNnH), *b2 = (cf2 *)(P + kNnH * 2 * kE + kNnH + kNnH * kNnH);
    cfloat *W3 = P + kNnH * 2 * kE + kNnH + kNnH * kNnH + kNnH, *b3 = W3 + kNnH;
    float o = b3[0];
    for (int m = 0; m < kNnH / 2; ++m) {
      f2 a = b2[m];
#pragma unroll
      for (int k = 0; k < kNnH; ++k) a = pfma(W2[m * kNnH + k], splat(k & 1 ? h[k >> 1].y : h[k >> 1].x), a);
      o = fmaf(W3[2 * m], relu(a.x), o);
      o = fmaf(W3[2 * m + 1], relu(a.y), o);
    }
    return logf(1.0f / (1.0f + expf(-o)));
  } else {
    return 0.f;  // EXTERNAL: supplied by lik_ext in phase 2
  }
}


// per-row constants of the measurement (frame encoding, NN obs-half fold); all threads call
template <int MEAS>
__device__ __forceinline__ void measure_row_setup(const float *enc, const float *meas_params,
                                                  StepShared &L) {
  const int tid = threadIdx.x;
  if (tid < 64) {
    const float v = tid < kE ? enc[tid] : 0.f;
    if (MEAS == NFDPF_MEAS_COS) {
      const double nrm = sqrt(wave_sum((double)v * v));
      if (tid < kE) L.encv[tid] = v;
      if (tid == 0) L.vinv = 1.0 / fmax(nrm, 1e-12);
    } else if (tid < kE) {
      L.encv[tid] = v;
    }
  }
  if (MEAS == NFDPF_MEAS_NN && tid < kNnH) {
    // obs half of likelihood_est's first layer (row_pairs layout: [m][k][2], m = tid / 2)
    float a = meas_params[kNnH * 2 * kE + tid];
    const float *w = meas_params + (tid >> 1) * 2 * kE * 2 + (tid & 1);
    for (int k = 0; k < kE; ++k) a = fmaf(w[2 * k], enc[k], a);
    L.nnrow[tid] = a;
  }
}

}  // namespace nfdpf
