// resample_soft.hip -- standalone soft resampler (resamplers.py:20-60) and
// normalize_log_probs (utils.py:39-44) behind the C ABI.  One workgroup per batch row.
#include "soft.hpp"

namespace nfdpf {

constexpr int kSoftMaxN = 16384;  // C[] lives in LDS (64 KiB)
constexpr size_t kSoftStageLds = 156 * 1024;  // C, p and the gathered weights in LDS: N <= 13 312

// STAGE: the row's p and the gathered weights live in LDS next to C (3 N floats), so the two
// cascade sums (one wave each, ~N / 32 dependent adds per lane) and the scan read LDS instead
// of global memory (round 3: C5 112 us per call with every cascade term a global load).  The
// arithmetic is the same either way (bit-identical, tests/test_gpu_backward.py / parity).
template <bool STAGE>
__global__ __launch_bounds__(1024) void soft_resample_kernel(
    const float *__restrict__ x, const float *__restrict__ p, const float *__restrict__ lin,
    const float *__restrict__ offsets, int B, int N, int D, float alpha, int64_t row_base,
    float *__restrict__ x_out, float *__restrict__ w_out, int64_t *__restrict__ idx_out) {
  extern __shared__ float C[];
  __shared__ double shd[16];
  __shared__ float shf[2];
  float *P = C + N, *Wg = C + 2 * N;
  const int b = blockIdx.x;
  const int64_t rowN = (int64_t)b * N;
  const float *prow = p + rowN;
  if (STAGE) {
    for (int j = threadIdx.x; j < N; j += blockDim.x) P[j] = prow[j];
    __syncthreads();
    prow = P;
  }
  SoftRow row{prow, N, alpha, 1.0f / (float)N, (float)(1.0 - (double)alpha), 1.0f};
  const int64_t flat_base = (int64_t)N * (row_base + b);
  soft_row_search(row, lin, offsets[b], C, shd, shf, [&](int i, int src) {
    // the reference gathers from the flattened batch: src == N reads the next row (:52-55)
    const int64_t g = min(rowN + src, (int64_t)B * N - 1);
    const int64_t gb = g / N;
    const int gj = (int)(g - gb * N);
    for (int k = 0; k < D; ++k) x_out[(rowN + i) * D + k] = x[g * D + k];
    const float wsrc = (gb == b) ? row.w(gj) : 0.0f;  // other-row weights: see DESIGN.md
    if (STAGE)
      Wg[i] = wsrc;
    else
      w_out[rowN + i] = wsrc;
    idx_out[rowN + i] = flat_base + src;
  });
  __syncthreads();
  const float *wr = STAGE ? Wg : w_out + rowN;
  if (threadIdx.x < 64) {
    const float S2 = cascade_row_sum([&](int j) { return wr[j]; }, N);
    if (threadIdx.x == 0) shf[1] = S2;
  }
  __syncthreads();
  const float S2 = shf[1];
  for (int i = threadIdx.x; i < N; i += blockDim.x) w_out[rowN + i] = wr[i] / S2;
}

// p = exp(lw - max) / sum + add ; inv_ess = 1 / sum(p^2)
__global__ __launch_bounds__(1024) void normalize_kernel(const float *__restrict__ lw, int N,
                                                         float add, float *__restrict__ p,
                                                         float *__restrict__ inv_ess) {
  __shared__ float shf[16];
  __shared__ double shd[16];
  const int64_t base = (int64_t)blockIdx.x * N;
  float m = -INFINITY;
  for (int i = threadIdx.x; i < N; i += blockDim.x) m = fmaxf(m, lw[base + i]);
  m = block_max(m, shf);
  double s = 0.0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) s += (double)expf(lw[base + i] - m);
  const float S = (float)block_sum(s, shd);
  double s2 = 0.0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const float v = expf(lw[base + i] - m) / S + add;
    p[base + i] = v;
    s2 += (double)v * (double)v;
  }
  s2 = block_sum(s2, shd);
  if (inv_ess && threadIdx.x == 0) inv_ess[blockIdx.x] = 1.0f / (float)s2;
}

}  // namespace nfdpf

using namespace nfdpf;

extern "C" int nfdpf_soft_resample(const float *x, const float *p, const float *lin,
                                   const float *offsets, int B, int N, int D, float alpha,
                                   int64_t row_base, float *x_out, float *w_out, int64_t *idx_out,
                                   void *stream) {
  NFDPF_REQUIRE(x && p && lin && offsets && x_out && w_out && idx_out,
                "nfdpf_soft_resample: null pointer");
  NFDPF_REQUIRE(B >= 0 && N >= 1 && D >= 1, "nfdpf_soft_resample: bad sizes");
  NFDPF_REQUIRE(N <= kSoftMaxN, "nfdpf_soft_resample: N=%d above the LDS-resident limit %d", N,
                kSoftMaxN);
  NFDPF_REQUIRE(alpha > 0.f && alpha <= 1.f, "nfdpf_soft_resample: need 0 < alpha <= 1");
  if (B == 0) return NFDPF_OK;
  const size_t stage_lds = 3 * (size_t)N * sizeof(float);
  if (stage_lds <= kSoftStageLds) {
    ensure_max_dynamic_lds((const void *)soft_resample_kernel<true>, (int)kSoftStageLds);
    soft_resample_kernel<true><<<B, row_threads(N), stage_lds, as_stream(stream)>>>(
        x, p, lin, offsets, B, N, D, alpha, row_base, x_out, w_out, idx_out);
  } else {
    soft_resample_kernel<false><<<B, row_threads(N), N * sizeof(float), as_stream(stream)>>>(
        x, p, lin, offsets, B, N, D, alpha, row_base, x_out, w_out, idx_out);
  }
  return launch_status("nfdpf_soft_resample");
}

extern "C" int nfdpf_normalize_log_probs(const float *logw, int B, int N, float add, float *p,
                                         float *inv_ess, void *stream) {
  NFDPF_REQUIRE(logw && p, "nfdpf_normalize_log_probs: null pointer");
  NFDPF_REQUIRE(B >= 0 && N >= 1, "nfdpf_normalize_log_probs: bad sizes");
  if (B == 0) return NFDPF_OK;
  normalize_kernel<<<B, row_threads(N), 0, as_stream(stream)>>>(logw, N, add, p, inv_ess);
  return launch_status("nfdpf_normalize_log_probs");
}
