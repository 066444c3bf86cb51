// nn_bwd.hip -- backward of the NN measurement's likelihood head (training):
//   lik = log sigmoid(W3 relu(W2 relu(W1 [v, e] + b1) + b2) + b3)
//   (measurement_model_NN model/models.py:221-235, build_likelihood :119-128; v = the row's
//    frame encoding (32), e = the particle's encoding (32, from the particle encoder, whose
//    backward is nfdpf_particle_encoder mode 1)).
// One workgroup = one wave = 64 particles of ONE batch row, one particle per lane: recompute
// the head (the v half of layer 1 folded once per workgroup), back-propagate g = dL/dlik to e
// (written per particle) and to the layer-1 pre-activations; the weight gradient is left as
// outer-product factors in LDS -- first {g_z2, h1, h2, g_z3} (layers 2, 3), then {g_z1, e}
// (layer 1) in the same buffer -- and contracted over the wave's particles (lane = weight) into
// a per-workgroup partial in nn.Linear order [W1 b1 W2 b2 W3 b3]; the v half of dW1 is
// (sum_r g_z1) (x) v and dL/dv = W1v^T sum_r g_z1 (per-workgroup partial, summed per row in
// order).  Fixed-order sums only.
#include "measure.hpp"

namespace nfdpf {

constexpr int kNnRows = 64;
constexpr int kNnIn = 2 * kE;                                  // [v, e]
constexpr int kNnParams = kNnH * kNnIn + kNnH + kNnH * kNnH + kNnH + kNnH + 1;  // 8385
// blob (nfdpf.pack.paired_mlp_tensors): W1, W2 in row_pairs, W3 and the biases plain
constexpr int kNnB1 = kNnH * kNnIn, kNnW2 = kNnB1 + kNnH, kNnB2 = kNnW2 + kNnH * kNnH, kNnW3 = kNnB2 + kNnH,
              kNnB3 = kNnW3 + kNnH;
__device__ __forceinline__ float nn_w1(cfloat *P, int o, int k) { return P[((o >> 1) * kNnIn + k) * 2 + (o & 1)]; }
__device__ __forceinline__ float nn_w2(cfloat *P, int o, int k) {
  return P[kNnW2 + ((o >> 1) * kNnH + k) * 2 + (o & 1)];
}
// factor rows (floats, odd stride): phase A g_z2[64] h1[64] h2[64] g_z3; phase B g_z1[64] e[32]
constexpr int kFaGz2 = 0, kFaH1 = 64, kFaH2 = 128, kFaGz3 = 192, kFaRow = 193;
constexpr int kFbGz1 = 0, kFbE = 64, kFbRow = 97;

__global__ __launch_bounds__(kNnRows) void nn_meas_bwd_kernel(const float *__restrict__ params,
                                                              const float *__restrict__ enc,
                                                              const float *__restrict__ es,
                                                              const float *__restrict__ g_lik, int N,
                                                              float *__restrict__ g_es, float *__restrict__ g_vpart,
                                                              float *__restrict__ partial) {
  extern __shared__ float fac[];  // [kNnRows][kFaRow] (phase B reuses it as [kNnRows][kFbRow])
  __shared__ float vrow[kE], fold[kNnH], gz1sum[kNnH];
  const int b = blockIdx.y, lane = threadIdx.x;
  const int n = blockIdx.x * kNnRows + lane;
  const bool valid = n < N;
  const int64_t r = (int64_t)b * N + n;
  cfloat *P = wptr(params);
  if (lane < kE) vrow[lane] = enc[b * kE + lane];
  __syncthreads();
  {  // the v half of layer 1, folded with b1: lane o
    float a = P[kNnB1 + lane];
    for (int k = 0; k < kE; ++k) a = fmaf(nn_w1(P, lane, k), vrow[k], a);
    fold[lane] = a;
  }
  float e[kE];
#pragma unroll
  for (int k = 0; k < kE; ++k) e[k] = valid ? es[r * kE + k] : 0.f;
  const float g = valid ? g_lik[r] : 0.f;
  __syncthreads();
  float *fa = fac + lane * kFaRow;
  float h1[kNnH];  // outer loops rolled (scalar weight loads per row of W), inner unrolled
#pragma unroll
  for (int o = 0; o < kNnH; ++o) {
    float a = fold[o];
#pragma unroll
    for (int k = 0; k < kE; ++k) a = fmaf(nn_w1(P, o, kE + k), e[k], a);
    h1[o] = relu(a);
    fa[kFaH1 + o] = h1[o];
  }
  float z3 = P[kNnB3];
#pragma unroll 1
  for (int o = 0; o < kNnH; ++o) {
    float a = P[kNnB2 + o];
#pragma unroll
    for (int k = 0; k < kNnH; ++k) a = fmaf(nn_w2(P, o, k), h1[k], a);
    a = relu(a);  // h2
    fa[kFaH2 + o] = a;
    z3 = fmaf(P[kNnW3 + o], a, z3);
  }
  // lik = log sigmoid(z3): d/dz3 = 1 - sigmoid(z3)
  const float gz3 = g * (1.f - 1.f / (1.f + expf(-z3)));
  fa[kFaGz3] = gz3;
  float gz1[kNnH];
#pragma unroll
  for (int k = 0; k < kNnH; ++k) gz1[k] = 0.f;
#pragma unroll 1
  for (int o = 0; o < kNnH; ++o) {  // g_z2 (h2 > 0 <=> z2 > 0), then its W2^T product
    const float gz2 = fa[kFaH2 + o] > 0.f ? P[kNnW3 + o] * gz3 : 0.f;
    fa[kFaGz2 + o] = gz2;
#pragma unroll
    for (int k = 0; k < kNnH; ++k) gz1[k] = fmaf(nn_w2(P, o, k), gz2, gz1[k]);
  }
#pragma unroll
  for (int k = 0; k < kNnH; ++k) gz1[k] = h1[k] > 0.f ? gz1[k] : 0.f;
#pragma unroll 1
  for (int k = 0; k < kE; ++k) {
    float a = 0.f;
#pragma unroll
    for (int o = 0; o < kNnH; ++o) a = fmaf(nn_w1(P, o, kE + k), gz1[o], a);
    if (valid) g_es[r * kE + k] = a;
  }
  __syncthreads();
  // phase A contraction: W2 (row-major [o][k]), b2, W3, b3 -- lane = parameter
  float *part = partial + ((int64_t)b * gridDim.x + blockIdx.x) * kNnParams;
  for (int p = lane; p < kNnH * kNnH + kNnH + kNnH + 1; p += kNnRows) {
    float s = 0.f;
    if (p < kNnH * kNnH) {
      const int o = p / kNnH, k = p % kNnH;
      for (int q = 0; q < kNnRows; ++q) s = fmaf(fac[q * kFaRow + kFaGz2 + o], fac[q * kFaRow + kFaH1 + k], s);
      part[kNnW2 + p] = s;
    } else if (p < kNnH * kNnH + kNnH) {
      const int o = p - kNnH * kNnH;
      for (int q = 0; q < kNnRows; ++q) s += fac[q * kFaRow + kFaGz2 + o];
      part[kNnB2 + o] = s;
    } else if (p < kNnH * kNnH + 2 * kNnH) {
      const int k = p - kNnH * kNnH - kNnH;
      for (int q = 0; q < kNnRows; ++q) s = fmaf(fac[q * kFaRow + kFaGz3], fac[q * kFaRow + kFaH2 + k], s);
      part[kNnW3 + k] = s;
    } else {
      for (int q = 0; q < kNnRows; ++q) s += fac[q * kFaRow + kFaGz3];
      part[kNnB3] = s;
    }
  }
  __syncthreads();
  float *fb = fac + lane * kFbRow;
#pragma unroll
  for (int o = 0; o < kNnH; ++o) fb[kFbGz1 + o] = gz1[o];
#pragma unroll
  for (int k = 0; k < kE; ++k) fb[kFbE + k] = e[k];
  __syncthreads();
  {  // sum over the wave's particles of g_z1 (lane o), then db1 and the v half of dW1
    float s = 0.f;
    for (int q = 0; q < kNnRows; ++q) s += fac[q * kFbRow + kFbGz1 + lane];
    gz1sum[lane] = s;
    part[kNnB1 + lane] = s;
  }
  __syncthreads();
  for (int p = lane; p < kNnH * kNnIn; p += kNnRows) {
    const int o = p / kNnIn, k = p % kNnIn;
    float s = 0.f;
    if (k < kE) {
      s = gz1sum[o] * vrow[k];
    } else {
      for (int q = 0; q < kNnRows; ++q) s = fmaf(fac[q * kFbRow + kFbGz1 + o], fac[q * kFbRow + kFbE + k - kE], s);
    }
    part[p] = s;
  }
  if (lane < kE) {  // dL/dv partial: W1v^T (sum g_z1)
    float a = 0.f;
    for (int o = 0; o < kNnH; ++o) a = fmaf(nn_w1(P, o, lane), gz1sum[o], a);
    g_vpart[((int64_t)b * gridDim.x + blockIdx.x) * kE + lane] = a;
  }
}

__global__ void nn_vpart_sum_kernel(const float *__restrict__ vpart, int nblk, float *__restrict__ g_enc) {
  const int b = blockIdx.x, k = threadIdx.x;
  if (k >= kE) return;
  float s = 0.f;
  for (int q = 0; q < nblk; ++q) s += vpart[((int64_t)b * nblk + q) * kE + k];
  g_enc[b * kE + k] = s;
}

__global__ __launch_bounds__(256) void nn_param_reduce_kernel(const float *__restrict__ partial, int64_t n_parts,
                                                              float *__restrict__ out) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, gq = threadIdx.x >> 6;
  const int p = blockIdx.x * 64 + c;
  float acc = 0.f;
  if (p < kNnParams)
    for (int64_t k = gq; k < n_parts; k += 4) acc += partial[k * kNnParams + p];
  red[gq][c] = acc;
  __syncthreads();
  if (gq == 0 && p < kNnParams) out[p] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
}

}  // namespace nfdpf

using namespace nfdpf;

extern "C" int64_t nfdpf_nn_measurement_backward_workspace(int B, int N) {
  if (B < 0 || N < 1) return -1;
  const int64_t nblk = (N + kNnRows - 1) / kNnRows;
  return (int64_t)(B > 0 ? B : 1) * nblk * (kNnParams + kE) * (int64_t)sizeof(float);
}

extern "C" int nfdpf_nn_measurement_backward(const float *meas_params, const float *enc, const float *e_particles,
                                             const float *g_lik, int B, int N, int E, float *g_e, float *g_enc,
                                             float *g_params, void *workspace, void *stream) {
  NFDPF_REQUIRE(B >= 0 && N >= 1, "nfdpf_nn_measurement_backward: bad sizes");
  NFDPF_REQUIRE(E == kE, "nfdpf_nn_measurement_backward: built for E = %d (got %d)", kE, E);
  NFDPF_REQUIRE(g_params, "nfdpf_nn_measurement_backward: null pointer");
  hipStream_t st = as_stream(stream);
  if (B == 0) {
    if (hipMemsetAsync(g_params, 0, sizeof(float) * kNnParams, st) != hipSuccess)
      return launch_status("nfdpf_nn_measurement_backward (memset)");
    return NFDPF_OK;
  }
  NFDPF_REQUIRE(meas_params && enc && e_particles && g_lik && g_e && g_enc && workspace,
                "nfdpf_nn_measurement_backward: null pointer");
  const int nblk = (N + kNnRows - 1) / kNnRows;
  float *partial = (float *)workspace;
  float *vpart = partial + (int64_t)B * nblk * kNnParams;
  const size_t lds = sizeof(float) * kNnRows * kFaRow;
  nn_meas_bwd_kernel<<<dim3(nblk, B), kNnRows, lds, st>>>(meas_params, enc, e_particles, g_lik, N, g_e, vpart,
                                                         partial);
  nn_vpart_sum_kernel<<<B, 64, 0, st>>>(vpart, nblk, g_enc);
  nn_param_reduce_kernel<<<(kNnParams + 63) / 64, 256, 0, st>>>(partial, (int64_t)B * nblk, g_params);
  return launch_status("nfdpf_nn_measurement_backward");
}
