// measure_bwd.hip -- backward of the cosine-distance measurement (training):
//   lik = log(1 / (1e-7 + cosd)),  cosd = 1 - <v^, e^>,  e = PE(x),  v = frame encoding
//   (model/models.py:206-219, et_distance utils.py:8-15 with F.normalize(eps = 1e-12),
//    build_particle_encoder model/models.py:130-139: Linear(2,16) ReLU Linear(16,32) ReLU
//    Linear(32,32))
// One workgroup = one wave = 64 particles of ONE batch row (grid (ceil(N / 64), B)), one
// particle per lane: recompute the encoder, back-propagate g = dL/dlik to x and leave the
// weight-gradient factors (g_e, h2, g_h2, h1, g_h1, x) in LDS; the wave contracts them over
// its 64 particles (lane = weight) into a per-workgroup partial of the plain nn.Linear layout
// [W1 b1 W2 b2 W3 b3].  The frame encoding's gradient needs the row sum of g r e^ (r =
// 1 / (1e-7 + cosd)); each workgroup writes its 32-wide partial, nfdpf_cos_meas_finish sums
// them per row in order and applies the normalisation's Jacobian.  Fixed-order sums only.
#include "measure.hpp"

namespace nfdpf {

constexpr int kMbRows = 64;
constexpr int kPe1 = 16, kPe2 = 32;
constexpr int kPeParams = kPe1 * 2 + kPe1 + kPe2 * kPe1 + kPe2 + kE * kPe2 + kE;  // 1648
// factor row (floats): g_e[32] h2[32] g_h2[32] h1[16] g_h1[16] x[2] (+1 pad: odd stride)
constexpr int kFGe = 0, kFH2 = 32, kFGh2 = 64, kFH1 = 96, kFGh1 = 112, kFX = 128, kFRow = 131;

// weights of the packed encoder blob (nfdpf.pack.encoder_tensors): W1 row_pairs, W2 / W3
// col_pairs, biases plain
__device__ __forceinline__ float pe_w1(cfloat *pe, int o, int k) { return pe[((o >> 1) * 2 + k) * 2 + (o & 1)]; }
__device__ __forceinline__ float pe_w2(cfloat *pe, int o, int k) {
  return pe[kPeW2 + (k * (kPe2 / 2) + (o >> 1)) * 2 + (o & 1)];
}
__device__ __forceinline__ float pe_w3(cfloat *pe, int o, int k) {
  return pe[kPeW3 + (k * (kE / 2) + (o >> 1)) * 2 + (o & 1)];
}

// normalisation Jacobian of F.normalize(a, eps): d(a / max(|a|, eps)) applied to g
template <int n>
__device__ __forceinline__ void normalize_bwd(const float (&a)[n], float norm, const float (&g)[n], float (&out)[n]) {
  if (norm > 1e-12f) {
    float dot = 0.f;
#pragma unroll
    for (int k = 0; k < n; ++k) dot = fmaf(a[k], g[k], dot);
    const float inv = 1.f / norm, c = dot * inv * inv;
#pragma unroll
    for (int k = 0; k < n; ++k) out[k] = (g[k] - a[k] * c) * inv;
  } else {
#pragma unroll
    for (int k = 0; k < n; ++k) out[k] = g[k] * 1e12f;
  }
}

// MODE: kPeCos (the cosine measurement: g = dL/dlik), kPeGrad (dL/de given per particle in
// g_e [B*N, 32]: the particle encoder inside another model, e.g. the CRNVP condition),
// kPeFwd (forward only: write e to e_out -- the recompute those models' backward needs)
constexpr int kPeCos = 0, kPeGrad = 1, kPeFwd = 2;

template <int MODE>
__global__ __launch_bounds__(kMbRows) void cos_meas_bwd_kernel(const float *__restrict__ pe_params,
                                                               const float *__restrict__ enc,
                                                               const float *__restrict__ x,
                                                               const float *__restrict__ g_lik, int N,
                                                               float *__restrict__ g_x,
                                                               float *__restrict__ g_vpart,
                                                               float *__restrict__ partial) {
  __shared__ float fac[kMbRows * kFRow];
  __shared__ float vh[kE];
  cfloat *pe = wptr(pe_params);
  const int b = blockIdx.y, blk = blockIdx.x, lane = threadIdx.x;
  const int i = blk * kMbRows + lane;
  const bool valid = i < N;
  const int64_t o = (int64_t)b * N + i;
  if (MODE == kPeCos) {
    // the row's frame encoding, normalised (F.normalize, eps 1e-12)
    float vv = lane < kE ? enc[(int64_t)b * kE + lane] : 0.f;
    float ss = vv * vv;
#pragma unroll
    for (int m = 1; m < 64; m <<= 1) ss += __shfl_xor(ss, m);
    const float vn = fmaxf(sqrtf(ss), 1e-12f);
    if (lane < kE) vh[lane] = vv / vn;
    __syncthreads();
  }
  const float x0 = valid ? x[2 * o] : 0.f, x1 = valid ? x[2 * o + 1] : 0.f;
  const float g = (MODE == kPeCos && valid) ? g_lik[o] : 0.f;
  // ---- forward recompute ----
  float h1[kPe1], h2[kPe2], e[kE];
#pragma unroll
  for (int q = 0; q < kPe1; ++q)
    h1[q] = relu(fmaf(pe_w1(pe, q, 1), x1, fmaf(pe_w1(pe, q, 0), x0, pe[kPeB1 + q])));
#pragma unroll
  for (int q = 0; q < kPe2; ++q) {
    float a = pe[kPeB2 + q];
#pragma unroll
    for (int k = 0; k < kPe1; ++k) a = fmaf(pe_w2(pe, q, k), h1[k], a);
    h2[q] = relu(a);
  }
  float es = 0.f;
#pragma unroll
  for (int q = 0; q < kE; ++q) {
    float a = pe[kPeW3 + kE * kPe2 + q];
#pragma unroll
    for (int k = 0; k < kPe2; ++k) a = fmaf(pe_w3(pe, q, k), h2[k], a);
    e[q] = a;
    es = fmaf(a, a, es);
  }
  if (MODE == kPeFwd) {
    if (valid)
#pragma unroll
      for (int q = 0; q < kE; ++q) g_x[o * kE + q] = e[q];  // e_out
    return;
  }
  float ge[kE];
  if (MODE == kPeCos) {
    const float en = fmaxf(sqrtf(es), 1e-12f);
    float dot = 0.f;
#pragma unroll
    for (int q = 0; q < kE; ++q) dot = fmaf(e[q] / en, vh[q], dot);
    const float cosd = 1.f - dot;
    // dlik/dcosd = -1 / (1e-7 + cosd); dcosd/d e^ = -v^  ->  g_e^ = g r v^, g_v^ = g r e^
    const float gr = g / (1e-7f + cosd);
    float ge_hat[kE];
#pragma unroll
    for (int q = 0; q < kE; ++q) ge_hat[q] = gr * vh[q];
    normalize_bwd<kE>(e, sqrtf(es), ge_hat, ge);
    // this particle's share of the frame-encoding gradient, before the row's normalisation
    // Jacobian: g r e^ summed over the workgroup (wave reduction per component)
    float *vp = g_vpart + ((int64_t)b * gridDim.x + blk) * kE;
#pragma unroll
    for (int q = 0; q < kE; ++q) {
      float s = gr * (e[q] / en);
#pragma unroll
      for (int m = 1; m < 64; m <<= 1) s += __shfl_xor(s, m);
      if (lane == 0) vp[q] = s;
    }
  } else {
#pragma unroll
    for (int q = 0; q < kE; ++q) ge[q] = valid ? g_lik[o * kE + q] : 0.f;  // dL/de given
  }
  // ---- back-propagation through the encoder ----
  float gh2[kPe2], gh1[kPe1];
#pragma unroll
  for (int k = 0; k < kPe2; ++k) {
    float a = 0.f;
#pragma unroll
    for (int q = 0; q < kE; ++q) a = fmaf(pe_w3(pe, q, k), ge[q], a);
    gh2[k] = h2[k] > 0.f ? a : 0.f;
  }
#pragma unroll
  for (int k = 0; k < kPe1; ++k) {
    float a = 0.f;
#pragma unroll
    for (int q = 0; q < kPe2; ++q) a = fmaf(pe_w2(pe, q, k), gh2[q], a);
    gh1[k] = h1[k] > 0.f ? a : 0.f;
  }
  float gx0 = 0.f, gx1 = 0.f;
#pragma unroll
  for (int q = 0; q < kPe1; ++q) {
    gx0 = fmaf(pe_w1(pe, q, 0), gh1[q], gx0);
    gx1 = fmaf(pe_w1(pe, q, 1), gh1[q], gx1);
  }
  if (valid) {
    g_x[2 * o] = gx0;
    g_x[2 * o + 1] = gx1;
  }
  // ---- weight-gradient factors (zero for lanes past the row: g = 0 makes every g-factor 0) ----
  float *f = fac + lane * kFRow;
#pragma unroll
  for (int q = 0; q < kE; ++q) f[kFGe + q] = ge[q];
#pragma unroll
  for (int q = 0; q < kPe2; ++q) {
    f[kFH2 + q] = h2[q];
    f[kFGh2 + q] = gh2[q];
  }
#pragma unroll
  for (int q = 0; q < kPe1; ++q) {
    f[kFH1 + q] = h1[q];
    f[kFGh1 + q] = gh1[q];
  }
  f[kFX] = x0;
  f[kFX + 1] = x1;
  __syncthreads();
  // ---- contraction over the wave's 64 particles, lane = weight (plain nn.Linear layout) ----
  float *part = partial + ((int64_t)b * gridDim.x + blk) * kPeParams;
  for (int w = lane; w < kPeParams; w += kMbRows) {
    int ga, bi;  // g-factor index, activation index (-1: bias)
    if (w < kPe1 * 2) {
      ga = kFGh1 + w / 2, bi = kFX + w % 2;
    } else if (w < kPe1 * 3) {
      ga = kFGh1 + (w - kPe1 * 2), bi = -1;
    } else if (w < kPe1 * 3 + kPe2 * kPe1) {
      const int u = w - kPe1 * 3;
      ga = kFGh2 + u / kPe1, bi = kFH1 + u % kPe1;
    } else if (w < kPe1 * 3 + kPe2 * kPe1 + kPe2) {
      ga = kFGh2 + (w - kPe1 * 3 - kPe2 * kPe1), bi = -1;
    } else if (w < kPeParams - kE) {
      const int u = w - (kPe1 * 3 + kPe2 * kPe1 + kPe2);
      ga = kFGe + u / kPe2, bi = kFH2 + u % kPe2;
    } else {
      ga = kFGe + (w - (kPeParams - kE)), bi = -1;
    }
    float acc = 0.f;
    if (bi < 0) {
      for (int r = 0; r < kMbRows; ++r) acc += fac[r * kFRow + ga];
    } else {
      for (int r = 0; r < kMbRows; ++r) acc = fmaf(fac[r * kFRow + ga], fac[r * kFRow + bi], acc);
    }
    part[w] = acc;
  }
}

// per row: S = sum of the workgroups' g r e^ partials (in order); g_enc = Jacobian of
// F.normalize(v) applied to S
__global__ __launch_bounds__(64) void cos_meas_finish_kernel(const float *__restrict__ enc,
                                                             const float *__restrict__ g_vpart, int nblk,
                                                             float *__restrict__ g_enc) {
  const int b = blockIdx.x, lane = threadIdx.x;
  float v[kE], S[kE], out[kE];
  float ss = 0.f;
#pragma unroll
  for (int q = 0; q < kE; ++q) {
    v[q] = enc[(int64_t)b * kE + q];
    ss = fmaf(v[q], v[q], ss);
    float s = 0.f;
    for (int k = 0; k < nblk; ++k) s += g_vpart[((int64_t)b * nblk + k) * kE + q];
    S[q] = s;
  }
  normalize_bwd<kE>(v, sqrtf(ss), S, out);
  if (lane < kE) {
    float r = 0.f;
#pragma unroll
    for (int q = 0; q < kE; ++q) r = (q == lane) ? out[q] : r;
    g_enc[(int64_t)b * kE + lane] = r;
  }
}

__global__ __launch_bounds__(256) void meas_param_reduce_kernel(const float *__restrict__ partial, int64_t n_parts,
                                                                float *__restrict__ out) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int p = blockIdx.x * 64 + c;
  float acc = 0.f;
  if (p < kPeParams)
    for (int64_t k = g; k < n_parts; k += 4) acc += partial[k * kPeParams + p];
  red[g][c] = acc;
  __syncthreads();
  if (g == 0 && p < kPeParams) out[p] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
}

}  // namespace nfdpf

using namespace nfdpf;

extern "C" int64_t nfdpf_cos_measurement_backward_workspace(int B, int N) {
  if (B < 0 || N < 1) return -1;
  const int64_t nblk = (N + kMbRows - 1) / kMbRows;
  return (int64_t)B * nblk * (kPeParams + kE) * (int64_t)sizeof(float);
}

extern "C" int nfdpf_cos_measurement_backward(const float *pe_params, const float *enc, const float *x,
                                              const float *g_lik, int B, int N, int E, float *g_enc,
                                              float *g_x, float *g_params, void *workspace, void *stream) {
  NFDPF_REQUIRE(B >= 0 && N >= 1, "nfdpf_cos_measurement_backward: bad sizes");
  NFDPF_REQUIRE(E == kE, "nfdpf_cos_measurement_backward: built for E = %d (got %d)", kE, E);
  NFDPF_REQUIRE(g_params, "nfdpf_cos_measurement_backward: null pointer");
  hipStream_t st = as_stream(stream);
  if (B == 0) {
    (void)hipMemsetAsync(g_params, 0, sizeof(float) * kPeParams, st);
    return launch_status("nfdpf_cos_measurement_backward");
  }
  NFDPF_REQUIRE(pe_params && enc && x && g_lik && g_enc && g_x && workspace,
                "nfdpf_cos_measurement_backward: null pointer");
  const int nblk = (N + kMbRows - 1) / kMbRows;
  float *partial = (float *)workspace;
  float *vpart = partial + (int64_t)B * nblk * kPeParams;
  cos_meas_bwd_kernel<kPeCos><<<dim3(nblk, B), kMbRows, 0, st>>>(pe_params, enc, x, g_lik, N, g_x, vpart, partial);
  cos_meas_finish_kernel<<<B, 64, 0, st>>>(enc, vpart, nblk, g_enc);
  meas_param_reduce_kernel<<<(kPeParams + 63) / 64, 256, 0, st>>>(partial, (int64_t)B * nblk, g_params);
  return launch_status("nfdpf_cos_measurement_backward");
}

// The particle encoder alone (model/models.py:130-139), for the measurement models that feed
// its output into a further model (CRNVP: the flow's condition): mode 0 forward (e_out
// [B*N, 32] = PE(x)), mode 1 backward (g_e [B*N, 32] given -> g_x, g_params in nn.Linear
// order, fixed-order partials in the workspace of nfdpf_cos_measurement_backward_workspace).
extern "C" int nfdpf_particle_encoder(int mode, const float *pe_params, const float *x, int B, int N,
                                      const float *g_e, float *e_out, float *g_x, float *g_params,
                                      void *workspace, void *stream) {
  NFDPF_REQUIRE(B >= 0 && N >= 1 && (mode == 0 || mode == 1), "nfdpf_particle_encoder: bad arguments");
  hipStream_t st = as_stream(stream);
  if (B == 0) {
    if (mode == 1 && g_params) (void)hipMemsetAsync(g_params, 0, sizeof(float) * kPeParams, st);
    return launch_status("nfdpf_particle_encoder");
  }
  const int nblk = (N + kMbRows - 1) / kMbRows;
  if (mode == 0) {
    NFDPF_REQUIRE(pe_params && x && e_out, "nfdpf_particle_encoder: null pointer");
    cos_meas_bwd_kernel<kPeFwd><<<dim3(nblk, B), kMbRows, 0, st>>>(pe_params, nullptr, x, nullptr, N, e_out,
                                                                   nullptr, nullptr);
  } else {
    NFDPF_REQUIRE(pe_params && x && g_e && g_x && g_params && workspace, "nfdpf_particle_encoder: null pointer");
    float *partial = (float *)workspace;
    cos_meas_bwd_kernel<kPeGrad><<<dim3(nblk, B), kMbRows, 0, st>>>(pe_params, nullptr, x, g_e, N, g_x, nullptr,
                                                                    partial);
    meas_param_reduce_kernel<<<(kPeParams + 63) / 64, 256, 0, st>>>(partial, (int64_t)B * nblk, g_params);
  }
  return launch_status("nfdpf_particle_encoder");
}
