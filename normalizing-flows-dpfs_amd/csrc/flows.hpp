// flows.hpp -- per-particle device functions for the flows and MLPs of the hot path.
//
// Weights come through `cfloat*` (constant address space, common.hpp): every offset inside
// a net is a compile-time constant, so hipcc emits s_load_dwordx16 and feeds v_fma_f32
// from SGPRs -- no LDS traffic, no VGPR per weight.  One particle per lane; the hidden
// width (8) is far too narrow for a 16x16 MFMA tile.
//
// Coupling layout (nfdpf.pack.coupling_pair_tensors, include/nfdpf.h): the nets t and s of
// one coupling half share their input, so they are stored interleaved elementwise (float2
// {t, s}) and advance together, one v_pk_fma_f32 per weight pair:
//   [ W1[:, :HALF] (H x HALF) | W2 (H x H) | b2 (H) | W3 (HALF x H) | b3 (HALF)   <- core,
//     W1[:, HALF:] (H x O) | b1 (H) ]                                              <- context
// (every entry a {t, s} pair).  A flow is pair (t1, s1) then pair (t2, s2).  The per-particle
// path touches only the core; the context columns are folded into a bias pair once per batch
// row (or per particle when the condition is per particle).  Each component sees exactly the
// fma sequence of an unpacked net.
#pragma once

#include "common.hpp"

namespace nfdpf {

typedef float f2 __attribute__((ext_vector_type(2)));
typedef const f2 __attribute__((address_space(4))) cf2;

__device__ __forceinline__ f2 splat(float v) { return f2{v, v}; }
__device__ __forceinline__ f2 pfma(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }
// tanh_fast (common.hpp) on both components, the non-transcendental steps packed
__device__ __forceinline__ f2 tanh2(f2 x) {
  const f2 y = x * splat(2.8853900817779268f);
  const f2 d = f2{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)} + splat(1.0f);
  return pfma(splat(-2.0f), f2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)}, splat(1.0f));
}
__device__ __forceinline__ cf2 *wptr2(const float *p) { return (cf2 *)wptr(p); }
// The weight-pointer types the per-particle helpers below take: constant address space (cfloat /
// cf2: scalar loads, the default) or a plain pointer into LDS (weights staged per workgroup:
// ds_read, the address space inferred after inlining).  pair_ptr maps a float pointer to the
// pair pointer of the same kind.
__device__ __forceinline__ cf2 *pair_ptr(cfloat *p) { return (cf2 *)p; }
__device__ __forceinline__ const f2 *pair_ptr(const float *p) { return (const f2 *)p; }
__device__ __forceinline__ f2 relu2(f2 x) { return f2{relu(x.x), relu(x.y)}; }

// pairs in a (t, s) core / a whole (t, s) coupling half
template <int HALF, int H>
__host__ __device__ constexpr int net_core() {
  return H * HALF + H * H + H + HALF * H + HALF;
}
template <int HALF, int H>
__host__ __device__ constexpr int net_size(int O) {
  return net_core<HALF, H>() + H * O + H;
}

// cb[j] = b1[j] + sum_c W1[j, HALF + c] * ctx[c], for t and s at once
template <int HALF, int H>
__device__ __forceinline__ f2 fold_pair(cf2 *w, int O, int j, const float *ctx) {
  cf2 *w1c = w + net_core<HALF, H>();
  f2 a = w1c[H * O + j];
  for (int c = 0; c < O; ++c) a = pfma(w1c[j * O + c], splat(ctx[c]), a);
  return a;
}
template <int HALF, int H, int O, class WP>
__device__ __forceinline__ f2 fold_pair_c(WP w, int j, const float (&ctx)[O]) {
  const WP w1c = w + net_core<HALF, H>();
  f2 a = w1c[H * O + j];
#pragma unroll
  for (int c = 0; c < O; ++c) a = pfma(w1c[j * O + c], splat(ctx[c]), a);
  return a;
}

// Nets t and s of one coupling half on input u, first layer on the HALF leading columns plus
// the folded bias pairs cb[H].  Outputs t[HALF], s[HALF].
template <int HALF, int H, class WP>
__device__ __forceinline__ void ts_pair(WP w, const float (&u)[HALF], const f2 *cb,
                                        float (&t)[HALF], float (&s)[HALF]) {
  f2 h[H];
#pragma unroll
  for (int j = 0; j < H; ++j) {
    f2 a = cb[j];
#pragma unroll
    for (int k = 0; k < HALF; ++k) a = pfma(w[j * HALF + k], splat(u[k]), a);
    h[j] = tanh2(a);
  }
  const WP w2 = w + H * HALF;
  f2 g[H];
#pragma unroll
  for (int j = 0; j < H; ++j) {
    f2 a = w2[H * H + j];
#pragma unroll
    for (int k = 0; k < H; ++k) a = pfma(w2[j * H + k], h[k], a);
    g[j] = tanh2(a);
  }
  const WP w3 = w2 + H * H + H;
#pragma unroll
  for (int o = 0; o < HALF; ++o) {
    f2 a = w3[HALF * H + o];
#pragma unroll
    for (int k = 0; k < H; ++k) a = pfma(w3[o * H + k], g[k], a);
    t[o] = a.x;
    s[o] = a.y;
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

// One RealNVP_cond flow: pair (t1, s1) then pair (t2, s2), net_size(O) pairs each; cb = the
// folded bias pairs [2][H].  Forward: nf/flows.py:215-226; inverse: :228-239.  Returns the
// flow's log-det.
template <int HALF, int H, class WP>
__device__ __forceinline__ float coupling_forward(WP fw, int O, float (&lo)[HALF],
                                                  float (&up)[HALF], const f2 *cb) {
  const int ns = net_size<HALF, H>(O);
  float t[HALF], s[HALF];
  ts_pair<HALF, H>(fw, lo, cb, t, s);
#pragma unroll
  for (int k = 0; k < HALF; ++k) up[k] = t[k] + up[k] * expf(s[k]);
  const float l1 = half_sum<HALF>(s);
  ts_pair<HALF, H>(fw + ns, up, cb + H, t, s);
#pragma unroll
  for (int k = 0; k < HALF; ++k) lo[k] = t[k] + lo[k] * expf(s[k]);
  return l1 + half_sum<HALF>(s);
}

template <int HALF, int H>
__device__ __forceinline__ float coupling_inverse(cf2 *fw, int O, float (&lo)[HALF],
                                                  float (&up)[HALF], const f2 *cb) {
  const int ns = net_size<HALF, H>(O);
  float t[HALF], s[HALF];
  ts_pair<HALF, H>(fw + ns, up, cb + H, t, s);
#pragma unroll
  for (int k = 0; k < HALF; ++k) {
    lo[k] = (lo[k] - t[k]) * expf(-s[k]);
    s[k] = -s[k];
  }
  const float l2 = half_sum<HALF>(s);
  ts_pair<HALF, H>(fw, lo, cb, t, s);
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
// Layout (nfdpf.pack.encoder_tensors): W1 in row_pairs order ({W[2m, k], W[2m+1, k]} at
// [m][k]); W2 and W3 in col_pairs order ({W[2m, k], W[2m+1, k]} at [k][m]), so the layers run
// input-major: each input's weight run (16 pairs = 128 B, two s_load_dwordx16) feeds
// independent accumulators for every output pair -- full ILP instead of one long dependent
// chain per output.  Biases as stored by nn.Linear.
// ----------------------------------------------------------------------------------------
constexpr int kPeH1 = 16, kPeH2 = 32;
__host__ __device__ constexpr int pe_size(int E) {
  return kPeH1 * 2 + kPeH1 + kPeH2 * kPeH1 + kPeH2 + E * kPeH2 + E;
}
constexpr int kPeB1 = kPeH1 * 2, kPeW2 = kPeB1 + kPeH1, kPeB2 = kPeW2 + kPeH2 * kPeH1,
              kPeW3 = kPeB2 + kPeH2;

__device__ __forceinline__ float pick(const f2 *h, int k) { return (k & 1) ? h[k >> 1].y : h[k >> 1].x; }

template <class WF>
__device__ __forceinline__ void pe_hidden(WF pe, float x0, float x1, f2 (&h2)[kPeH2 / 2]) {
  const auto w1 = pair_ptr(pe), b1 = pair_ptr(pe + kPeB1);
  f2 h1[kPeH1 / 2];
#pragma unroll
  for (int m = 0; m < kPeH1 / 2; ++m)
    h1[m] = relu2(pfma(w1[2 * m + 1], splat(x1), pfma(w1[2 * m], splat(x0), b1[m])));
  const auto w2 = pair_ptr(pe + kPeW2), b2 = pair_ptr(pe + kPeB2);
  constexpr int M = kPeH2 / 2;
#pragma unroll
  for (int m = 0; m < M; ++m) h2[m] = b2[m];
#pragma unroll
  for (int k = 0; k < kPeH1; ++k) {
    const float hk = pick(h1, k);
#pragma unroll
    for (int m = 0; m < M; ++m) h2[m] = pfma(w2[k * M + m], splat(hk), h2[m]);
  }
#pragma unroll
  for (int m = 0; m < M; ++m) h2[m] = relu2(h2[m]);
}

// output pairs [m0, m0 + MP) of the last layer, input-major
template <int E, int MP, class WF>
__device__ __forceinline__ void pe_out(WF pe, const f2 (&h2)[kPeH2 / 2], int m0, f2 (&a)[MP]) {
  constexpr int M = E / 2;
  const auto w3 = pair_ptr(pe + kPeW3) + m0, b3 = pair_ptr(pe + kPeW3 + E * kPeH2) + m0;
#pragma unroll
  for (int m = 0; m < MP; ++m) a[m] = b3[m];
#pragma unroll
  for (int k = 0; k < kPeH2; ++k) {
    const float hk = pick(h2, k);
#pragma unroll
    for (int m = 0; m < MP; ++m) a[m] = pfma(w3[k * M + m], splat(hk), a[m]);
  }
}

template <int E, class WF>
__device__ __forceinline__ void particle_encode(WF pe, float x0, float x1, float (&e)[E]) {
  f2 h2[kPeH2 / 2];
  pe_hidden(pe, x0, x1, h2);
  f2 a[E / 2];
  pe_out<E, E / 2>(pe, h2, 0, a);
#pragma unroll
  for (int m = 0; m < E / 2; ++m) {
    e[2 * m] = a[m].x;
    e[2 * m + 1] = a[m].y;
  }
}

// Cosine-distance pieces for the particle encoder output (|e|^2, <e, v>) over output pairs
// [m0, m0 + MP) (model/models.py:130-139 then utils.py:8-15); a caller may split the E
// outputs over several waves.  v is the RAW frame encoding; both sums accumulate in fp64 (the
// cosine distance 1 - cos ~ 1e-2 at a likely particle cancels two digits of them, and
// -log(1e-7 + 1 - cos) amplifies what is left by 1 / (1 - cos): fp32 sums made the likelihood
// ~1.3x less accurate than the reference's own fp32 F.normalize-then-dot, fp64 sums make it
// ~10x more accurate -- tests/test_gpu_parity_full.py).
template <int E, int MP = E / 2>
__device__ __forceinline__ void encode_dot(cfloat *pe, float x0, float x1, const float *v, double &ss,
                                           double &dot, int m0 = 0) {
  f2 h2[kPeH2 / 2];
  pe_hidden(pe, x0, x1, h2);
  f2 a[MP];
  pe_out<E, MP>(pe, h2, m0, a);
  ss = 0.0;
  dot = 0.0;
#pragma unroll
  for (int m = 0; m < MP; ++m) {
    const double ax = a[m].x, ay = a[m].y;
    ss = fma(ax, ax, ss);
    dot = fma(ax, (double)v[2 * (m0 + m)], dot);
    ss = fma(ay, ay, ss);
    dot = fma(ay, (double)v[2 * (m0 + m) + 1], dot);
  }
}

// log(1 / (1e-7 + cosd)), cosd = 1 - <e / max(|e|, 1e-12), v / max(|v|, 1e-12)>
// (measurement_model_cosine_distance + et_distance, model/models.py:206-219, utils.py:8-15),
// from fp64 |e|^2, <e, v> and the row's 1 / max(|v|, 1e-12) (fp64).
__device__ __forceinline__ float cos_lik(double ss, double dot, double vinv) {
  const double cosd = 1.0 - dot * vinv / fmax(sqrt(ss), 1e-12);
  return -logf((float)(1e-7 + cosd));
}

}  // namespace nfdpf
