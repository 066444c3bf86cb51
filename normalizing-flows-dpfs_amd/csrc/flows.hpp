// flows.hpp -- per-particle device functions for the flows and MLPs of the hot path.
//
// Weights come through `cfloat*` (constant address space, common.hpp): every offset inside
// a net is a compile-time constant, so hipcc emits s_load_dwordx16 and feeds v_fma_f32
// from SGPRs -- no LDS traffic, no VGPR per weight.  One particle per lane; the hidden
// width (8) is far too narrow for a 16x16 MFMA tile.
//
// Coupling-net layout (nfdpf.pack.realnvp_tensors, include/nfdpf.h):
//   [ W1[:, :HALF] (H x HALF) | W2 (H x H) | b2 (H) | W3 (HALF x H) | b3 (HALF)   <- "core",
//     W1[:, HALF:] (H x O) | b1 (H) ]                                              <- context
// The per-particle path touches only the core; the context columns are folded into a bias
// once per batch row (or per particle when the condition is per particle).
#pragma once

#include "common.hpp"

namespace nfdpf {

template <int HALF, int H>
__host__ __device__ constexpr int net_core() {
  return H * HALF + H * H + H + HALF * H + HALF;
}
template <int HALF, int H>
__host__ __device__ constexpr int net_size(int O) {
  return net_core<HALF, H>() + H * O + H;
}

// cb[j] = b1[j] + sum_c W1[j, HALF + c] * ctx[c]  (context folded into the first layer)
template <int HALF, int H>
__device__ __forceinline__ float fold_bias(cfloat *w, int O, int j, const float *ctx) {
  cfloat *w1c = w + net_core<HALF, H>();
  float a = w1c[H * O + j];
  for (int c = 0; c < O; ++c) a = fmaf(w1c[j * O + c], ctx[c], a);
  return a;
}
template <int HALF, int H, int O>
__device__ __forceinline__ float fold_bias_c(cfloat *w, int j, const float (&ctx)[O]) {
  cfloat *w1c = w + net_core<HALF, H>();
  float a = w1c[H * O + j];
#pragma unroll
  for (int c = 0; c < O; ++c) a = fmaf(w1c[j * O + c], ctx[c], a);
  return a;
}

// Nets t and s of one coupling half (same input u), first layer on the HALF leading columns
// plus the folded biases cbt/cbs.  Outputs t[HALF], s[HALF].
template <int HALF, int H>
__device__ __forceinline__ void ts_pair(cfloat *wt, cfloat *ws, const float (&u)[HALF],
                                        const float *cbt, const float *cbs, float (&t)[HALF],
                                        float (&s)[HALF]) {
  float ht[H], hs[H];
#pragma unroll
  for (int j = 0; j < H; ++j) {
    float at = cbt[j], as = cbs[j];
#pragma unroll
    for (int k = 0; k < HALF; ++k) {
      at = fmaf(wt[j * HALF + k], u[k], at);
      as = fmaf(ws[j * HALF + k], u[k], as);
    }
    ht[j] = tanh_fast(at);
    hs[j] = tanh_fast(as);
  }
  cfloat *w2t = wt + H * HALF, *w2s = ws + H * HALF;
  float gt[H], gs[H];
#pragma unroll
  for (int j = 0; j < H; ++j) {
    float at = w2t[H * H + j], as = w2s[H * H + j];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      at = fmaf(w2t[j * H + k], ht[k], at);
      as = fmaf(w2s[j * H + k], hs[k], as);
    }
    gt[j] = tanh_fast(at);
    gs[j] = tanh_fast(as);
  }
  cfloat *w3t = w2t + H * H + H, *w3s = w2s + H * H + H;
#pragma unroll
  for (int o = 0; o < HALF; ++o) {
    float at = w3t[HALF * H + o], as = w3s[HALF * H + o];
#pragma unroll
    for (int k = 0; k < H; ++k) {
      at = fmaf(w3t[o * H + k], gt[k], at);
      as = fmaf(w3s[o * H + k], gs[k], as);
    }
    t[o] = at;
    s[o] = as;
  }
}

// torch.sum(s, dim=1) over HALF entries in ATen's CPU order (oracle/cascade.py): for
// HALF = 16: sum_q (s[q] + s[q+8]) left to right; for HALF < 8: ((s0 + s1) + s2) ...
template <int HALF>
__device__ __forceinline__ float half_sum(const float (&s)[HALF]) {
  if constexpr (HALF >= 8 && HALF % 8 == 0) {
    float tot = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      float l = s[q];
#pragma unroll
      for (int r = 1; r < HALF / 8; ++r) l += s[q + 8 * r];
      tot += l;
    }
    return tot;
  } else {
    float tot = s[0];
#pragma unroll
    for (int q = 1; q < HALF; ++q) tot += s[q];
    return tot;
  }
}

// One RealNVP_cond flow (nets t1,s1,t2,s2 of net_size(O) floats each); cb = folded biases
// [4][H].  Forward: nf/flows.py:215-226; inverse: :228-239.  Returns the flow's log-det.
template <int HALF, int H>
__device__ __forceinline__ float coupling_forward(cfloat *fw, int O, float (&lo)[HALF],
                                                  float (&up)[HALF], const float *cb) {
  const int ns = net_size<HALF, H>(O);
  float t[HALF], s[HALF];
  ts_pair<HALF, H>(fw, fw + ns, lo, cb, cb + H, t, s);
#pragma unroll
  for (int k = 0; k < HALF; ++k) up[k] = t[k] + up[k] * expf(s[k]);
  const float l1 = half_sum<HALF>(s);
  ts_pair<HALF, H>(fw + 2 * ns, fw + 3 * ns, up, cb + 2 * H, cb + 3 * H, t, s);
#pragma unroll
  for (int k = 0; k < HALF; ++k) lo[k] = t[k] + lo[k] * expf(s[k]);
  return l1 + half_sum<HALF>(s);
}

template <int HALF, int H>
__device__ __forceinline__ float coupling_inverse(cfloat *fw, int O, float (&lo)[HALF],
                                                  float (&up)[HALF], const float *cb) {
  const int ns = net_size<HALF, H>(O);
  float t[HALF], s[HALF];
  ts_pair<HALF, H>(fw + 2 * ns, fw + 3 * ns, up, cb + 2 * H, cb + 3 * H, t, s);
#pragma unroll
  for (int k = 0; k < HALF; ++k) {
    lo[k] = (lo[k] - t[k]) * expf(-s[k]);
    s[k] = -s[k];
  }
  const float l2 = half_sum<HALF>(s);
  ts_pair<HALF, H>(fw, fw + ns, lo, cb, cb + H, t, s);
#pragma unroll
  for (int k = 0; k < HALF; ++k) {
    up[k] = (up[k] - t[k]) * expf(-s[k]);
    s[k] = -s[k];
  }
  return half_sum<HALF>(s) + l2;
}

// Plain FCNN(in, OUT, H): W1[H,in] b1 W2 b2 W3[OUT,H] b3 (nf/flows.py:101-114), used by MAF.
template <int H>
__host__ __device__ constexpr int fcnn_size(int in, int out) {
  return H * in + H + H * H + H + out * H + out;
}

template <int H, int OUT>
__device__ __forceinline__ void fcnn_small(cfloat *w, int in, const float *x, float (&o)[OUT]) {
  float h[H], g[H];
#pragma unroll
  for (int j = 0; j < H; ++j) {
    float a = w[H * in + j];
    for (int k = 0; k < in; ++k) a = fmaf(w[j * in + k], x[k], a);
    h[j] = tanh_fast(a);
  }
  cfloat *w2 = w + H * in + H;
#pragma unroll
  for (int j = 0; j < H; ++j) {
    float a = w2[H * H + j];
#pragma unroll
    for (int k = 0; k < H; ++k) a = fmaf(w2[j * H + k], h[k], a);
    g[j] = tanh_fast(a);
  }
  cfloat *w3 = w2 + H * H + H;
#pragma unroll
  for (int q = 0; q < OUT; ++q) {
    float a = w3[OUT * H + q];
#pragma unroll
    for (int k = 0; k < H; ++k) a = fmaf(w3[q * H + k], g[k], a);
    o[q] = a;
  }
}

// MAF flow size (nf/flows.py:247-254): initial_param[2] + FCNN(i,2,H) for i=1..D-1
template <int H>
__host__ __device__ constexpr int maf_size(int D) {
  int s = 2;
  for (int i = 1; i < D; ++i) s += fcnn_size<H>(i, 2);
  return s;
}

// MAF forward (nf/flows.py:259-270): z_i = (x_i - mu_i) / exp(alpha_i), output flipped.
template <int D, int H>
__device__ __forceinline__ float maf_forward(cfloat *fw, float (&x)[D]) {
  float z[D];
  float ld = 0.f;
  cfloat *w = fw + 2;
#pragma unroll
  for (int i = 0; i < D; ++i) {
    float mu, al;
    if (i == 0) {
      mu = fw[0];
      al = fw[1];
    } else {
      float o[2];
      fcnn_small<H, 2>(w, i, x, o);
      w += fcnn_size<H>(i, 2);
      mu = o[0];
      al = o[1];
    }
    z[i] = (x[i] - mu) / expf(al);
    ld -= al;
  }
#pragma unroll
  for (int i = 0; i < D; ++i) x[i] = z[D - 1 - i];
  return ld;
}

// MAF inverse (nf/flows.py:272-284): z flipped, then x_i = mu_i + exp(alpha_i) z_i.
template <int D, int H>
__device__ __forceinline__ float maf_inverse(cfloat *fw, float (&v)[D]) {
  float z[D], x[D];
#pragma unroll
  for (int i = 0; i < D; ++i) {
    z[i] = v[D - 1 - i];
    x[i] = 0.f;
  }
  float ld = 0.f;
  cfloat *w = fw + 2;
#pragma unroll
  for (int i = 0; i < D; ++i) {
    float mu, al;
    if (i == 0) {
      mu = fw[0];
      al = fw[1];
    } else {
      float o[2];
      fcnn_small<H, 2>(w, i, x, o);
      w += fcnn_size<H>(i, 2);
      mu = o[0];
      al = o[1];
    }
    x[i] = mu + expf(al) * z[i];
    ld += al;
  }
#pragma unroll
  for (int i = 0; i < D; ++i) v[i] = x[i];
  return ld;
}

// ----------------------------------------------------------------------------------------
// particle encoder (model/models.py:130-150): Linear(2,16) ReLU Linear(16,32) ReLU Linear(32,E)
// ----------------------------------------------------------------------------------------
constexpr int kPeH1 = 16, kPeH2 = 32;
__host__ __device__ constexpr int pe_size(int E) {
  return kPeH1 * 2 + kPeH1 + kPeH2 * kPeH1 + kPeH2 + E * kPeH2 + E;
}

__device__ __forceinline__ void pe_hidden(cfloat *pe, float x0, float x1, float (&h2)[kPeH2]) {
  float h1[kPeH1];
  cfloat *b1 = pe + kPeH1 * 2;
#pragma unroll
  for (int j = 0; j < kPeH1; ++j) h1[j] = relu(fmaf(pe[2 * j + 1], x1, fmaf(pe[2 * j], x0, b1[j])));
  cfloat *w2 = b1 + kPeH1, *b2 = w2 + kPeH2 * kPeH1;
#pragma unroll
  for (int j = 0; j < kPeH2; ++j) {
    float a = b2[j];
#pragma unroll
    for (int k = 0; k < kPeH1; ++k) a = fmaf(w2[j * kPeH1 + k], h1[k], a);
    h2[j] = relu(a);
  }
}

template <int E>
__device__ __forceinline__ void particle_encode(cfloat *pe, float x0, float x1, float (&e)[E]) {
  float h2[kPeH2];
  pe_hidden(pe, x0, x1, h2);
  cfloat *w3 = pe + kPeH1 * 2 + kPeH1 + kPeH2 * kPeH1 + kPeH2, *b3 = w3 + E * kPeH2;
#pragma unroll
  for (int j = 0; j < E; ++j) {
    float a = b3[j];
#pragma unroll
    for (int k = 0; k < kPeH2; ++k) a = fmaf(w3[j * kPeH2 + k], h2[k], a);
    e[j] = a;
  }
}

// Cosine-distance pieces for the particle encoder output, streamed: (|e|^2, <e, v>) without
// materialising e (model/models.py:130-139 then utils.py:8-15).
template <int E>
__device__ __forceinline__ void encode_dot(cfloat *pe, float x0, float x1, const float *v, float &ss,
                                           float &dot) {
  float h2[kPeH2];
  pe_hidden(pe, x0, x1, h2);
  cfloat *w3 = pe + kPeH1 * 2 + kPeH1 + kPeH2 * kPeH1 + kPeH2, *b3 = w3 + E * kPeH2;
  ss = 0.f;
  dot = 0.f;
#pragma unroll 4
  for (int j = 0; j < E; ++j) {
    float a = b3[j];
#pragma unroll
    for (int k = 0; k < kPeH2; ++k) a = fmaf(w3[j * kPeH2 + k], h2[k], a);
    ss = fmaf(a, a, ss);
    dot = fmaf(a, v[j], dot);
  }
}

}  // namespace nfdpf
