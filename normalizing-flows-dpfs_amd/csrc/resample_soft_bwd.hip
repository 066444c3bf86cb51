// resample_soft_bwd.hip -- backward of the soft resampler (training),
// the gradient the reference's autograd takes through resamplers.py:28-56:
//   q_j = (a p_j + b) / S,  S = sum_k (a p_k + b),  b = (1 - a) / N        (:30-33)
//   w_j = p_j / q_j = p_j S / (a p_j + b)              (a = 1: w_j = 1/N)    (:34, :37)
//   x'_i = x[idx_i],  w'_i = w[idx_i] / sum_k w[idx_k]                       (:52-56)
// idx is the forward's flat index (non-decreasing over the whole flattened batch: row b's
// entries lie in [N b, N b + N]), so every source j receives the contiguous run of outputs
// i with idx_i == j -- found by binary search, summed in order: no atomics, deterministic.
// The reference's out-of-range edge (idx_i = N (b + 1): the next row's first particle) is
// differentiated as this library's forward computes it: x' from that particle, weight 0 (in
// the last row: x' and w from its own particle N - 1).
//   K1 (row):   S, A = sum_i w[idx_i], G = sum_i g'_i w'_i;  g_a_i = (g'_i - G) / A
//   K2 (flat j): g_x[j] = sum_{i: idx_i = j} g_x'[i],  g_w[j] = sum over same-row i of g_a_i
//   K3 (row):   g_p_j = g_w_j S b / (a p_j + b)^2 + a sum_k g_w_k p_k / (a p_k + b)
#include "soft.hpp"

namespace nfdpf {

constexpr int kSbThreads = 256;

__device__ __forceinline__ double soft_w(float pj, double S, double a, double bb, int N) {
  return a < 1.0 ? (double)pj * S / (a * (double)pj + bb) : 1.0 / (double)N;
}

__global__ __launch_bounds__(kSbThreads) void soft_bwd_rows_kernel(
    const float *__restrict__ p, const int64_t *__restrict__ idx, const float *__restrict__ wo,
    const float *__restrict__ g_wo, int B, int N, float alpha, int64_t base, float *__restrict__ g_a,
    double *__restrict__ rowS) {
  __shared__ double shd[16];
  const int b = blockIdx.x;
  const int64_t r0 = (int64_t)b * N;
  const double a = alpha, bb = (1.0 - (double)alpha) / N;
  double s = 0.0;
  for (int j = threadIdx.x; j < N; j += blockDim.x) s += a * (double)p[r0 + j] + bb;
  const double S = block_sum(s, shd);
  double A = 0.0, G = 0.0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    // the forward's source (the last row's out-of-range edge reads its own particle N-1)
    const int64_t tg = min(idx[r0 + i] - base, (int64_t)B * N - 1);
    if (tg / N == b) A += soft_w(p[tg], S, a, bb, N);
    if (g_wo) G += (double)g_wo[r0 + i] * (double)wo[r0 + i];
  }
  A = block_sum(A, shd);
  G = block_sum(G, shd);
  for (int i = threadIdx.x; i < N; i += blockDim.x)
    g_a[r0 + i] = g_wo ? (float)(((double)g_wo[r0 + i] - G) / A) : 0.f;
  if (threadIdx.x == 0) rowS[b] = S;
}

// first i in [0, M) with target(i) >= v, target(i) = min(idx_i - base, M - 1) (non-decreasing)
__device__ __forceinline__ int64_t tgt_lower_bound(const int64_t *idx, int64_t M, int64_t base, int64_t v) {
  int64_t lo = 0, hi = M;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (min(idx[mid] - base, M - 1) < v)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

__global__ __launch_bounds__(kSbThreads) void soft_bwd_scatter_kernel(
    const int64_t *__restrict__ idx, const float *__restrict__ g_xo, const float *__restrict__ g_a,
    int B, int N, int D, int64_t base, float *__restrict__ g_x, float *__restrict__ g_w) {
  const int64_t M = (int64_t)B * N;
  const int64_t j = (int64_t)blockIdx.x * kSbThreads + threadIdx.x;
  if (j >= M) return;
  const int64_t lo = tgt_lower_bound(idx, M, base, j), hi = tgt_lower_bound(idx, M, base, j + 1);
  const int64_t row = j / N;
  float gw = 0.f;
  for (int64_t i = lo; i < hi; ++i)
    if (i / N == row) gw += g_a[i];
  g_w[j] = gw;
  for (int k = 0; k < D; ++k) {
    float gx = 0.f;
    if (g_xo)
      for (int64_t i = lo; i < hi; ++i) gx += g_xo[i * D + k];
    g_x[j * D + k] = gx;
  }
}

__global__ __launch_bounds__(kSbThreads) void soft_bwd_probs_kernel(const float *__restrict__ p,
                                                                   const float *__restrict__ g_w,
                                                                   const double *__restrict__ rowS,
                                                                   int N, float alpha,
                                                                   float *__restrict__ g_p) {
  __shared__ double shd[16];
  const int b = blockIdx.x;
  const int64_t r0 = (int64_t)b * N;
  if (!(alpha < 1.0f)) {  // hard resampling: w = 1/N does not depend on p
    for (int j = threadIdx.x; j < N; j += blockDim.x) g_p[r0 + j] = 0.f;
    return;
  }
  const double a = alpha, bb = (1.0 - (double)alpha) / N, S = rowS[b];
  double t = 0.0;
  for (int j = threadIdx.x; j < N; j += blockDim.x) {
    const double pj = p[r0 + j];
    t += (double)g_w[r0 + j] * pj / (a * pj + bb);
  }
  t = block_sum(t, shd);
  for (int j = threadIdx.x; j < N; j += blockDim.x) {
    const double d = a * (double)p[r0 + j] + bb;
    g_p[r0 + j] = (float)((double)g_w[r0 + j] * S * bb / (d * d) + a * t);
  }
}

}  // namespace nfdpf

using namespace nfdpf;

extern "C" int64_t nfdpf_soft_resample_backward_workspace(int B, int N) {
  if (B < 0 || N < 0) return -1;
  const int64_t M = (int64_t)B * N;
  return 2 * M * (int64_t)sizeof(float) + (int64_t)B * (int64_t)sizeof(double) + 256;
}

extern "C" int nfdpf_soft_resample_backward(const float *p, const int64_t *idx, const float *w_out,
                                            const float *g_x_out, const float *g_w_out, int B, int N,
                                            int D, float alpha, int64_t row_base, float *g_x,
                                            float *g_p, void *workspace, void *stream) {
  NFDPF_REQUIRE(B >= 0 && N >= 1 && D >= 1, "nfdpf_soft_resample_backward: bad sizes");
  NFDPF_REQUIRE(alpha > 0.f && alpha <= 1.f, "nfdpf_soft_resample_backward: alpha must be in (0, 1]");
  if (B == 0) return NFDPF_OK;
  NFDPF_REQUIRE(p && idx && g_x && g_p && workspace && (w_out || !g_w_out),
                "nfdpf_soft_resample_backward: null pointer");
  hipStream_t st = as_stream(stream);
  const int64_t M = (int64_t)B * N;
  const int64_t base = (int64_t)N * row_base;
  float *g_a = (float *)workspace;
  float *g_w = g_a + M;
  double *rowS = (double *)(((uintptr_t)(g_w + M) + 7) & ~(uintptr_t)7);
  soft_bwd_rows_kernel<<<B, kSbThreads, 0, st>>>(p, idx, w_out, g_w_out, B, N, alpha, base, g_a, rowS);
  soft_bwd_scatter_kernel<<<(unsigned)((M + kSbThreads - 1) / kSbThreads), kSbThreads, 0, st>>>(
      idx, g_x_out, g_a, B, N, D, base, g_x, g_w);
  soft_bwd_probs_kernel<<<B, kSbThreads, 0, st>>>(p, g_w, rowS, N, alpha, g_p);
  return launch_status("nfdpf_soft_resample_backward");
}
