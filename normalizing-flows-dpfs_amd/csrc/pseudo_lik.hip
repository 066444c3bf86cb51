// pseudo_lik.hip -- the block pseudo-likelihood of the semi-supervised objective
// (compute_block_density_nf, losses.py:37-68; training), forward and
// backward, on the filter's histories (weights, likelihood, prior, ancestor index: [B, T, N]).
//
// For every block end k (k + 1 divisible by L) and particle n, the reference walks the
// ancestry L steps back -- position n at step k, then index[b, j, .] from step j to j - 1 --
// and adds prior + likelihood at each visited (step, position) to eta_n; eta is NOT reset
// between blocks (it accumulates over the whole sequence, position by position), and
//   Q_b = sum over blocks of sum_n w[b, k, n] eta_n,   returned as Q_b / (number of blocks).
//
// Forward: one workgroup per row, one thread per particle, blocks in order (eta in a
// register), the row sum of w eta in fp64 per block (deterministic order).
// Backward (dL/dQ_b given): dw[b, k, n] = gQ_b eta_n(after block k); for the likelihood and
// prior, block K contributes G_K(n) = sum over blocks K' >= K of gQ_b w[b, k', n] at every
// position its chains visit: G starts at the block end (position n at step k) and moves one
// step back per launch through the ancestor map -- G'[m'] = sum of G[m] over m with
// index[j][m] = m'.  The ancestor maps of the filter are non-decreasing over the flattened
// batch (soft resampling sorts its sources; OT and no-resample steps are the identity), so
// the m of a target m' are one contiguous run found by two binary searches and summed in
// order: deterministic, no atomics.  (nfdpf_pseudo_lik_backward checks the order first and
// reports a non-monotone map, which the caller then differentiates in PyTorch.)
#include "common.hpp"

namespace nfdpf {

// flat (b', n') position p at step j of a [B, T, N] history
__device__ __forceinline__ int64_t hist_at(int64_t p, int j, int T, int N) {
  const int64_t b = p / N;
  return (b * T + j) * N + (p - b * N);
}

__global__ __launch_bounds__(256) void pl_forward_kernel(const float *__restrict__ w, const float *__restrict__ lik,
                                                         const float *__restrict__ prior,
                                                         const int64_t *__restrict__ idx, int B, int T, int N, int L,
                                                         double *__restrict__ Q) {
  __shared__ double sh[8];
  const int b = blockIdx.x;
  const int nb = T / L;
  double Qb = 0.0;
  // each thread owns particles n = threadIdx.x + 256 q; eta lives in registers over blocks
  constexpr int kMaxPer = 48;  // N <= 12288
  float eta[kMaxPer];
  for (int q = 0; q < kMaxPer; ++q) eta[q] = 0.f;
  for (int K = 0; K < nb; ++K) {
    const int k = (K + 1) * L - 1;
    double part = 0.0;
    for (int q = 0; q < kMaxPer; ++q) {
      const int n = threadIdx.x + 256 * q;
      if (n >= N) break;
      int64_t p = (int64_t)b * N + n;
      float e = eta[q];
      for (int s = 0; s < L; ++s) {
        const int j = k - s;
        const int64_t a = hist_at(p, j, T, N);
        e = (e + prior[a]) + lik[a];  // logyita = logyita + log_prior + lik_log (:65)
        if (s < L - 1) p = idx[a];
      }
      eta[q] = e;
      part += (double)w[((int64_t)b * T + k) * N + n] * (double)e;
    }
    part = wave_sum(part);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = part;
    __syncthreads();
    if (threadIdx.x == 0) Qb += ((sh[0] + sh[1]) + sh[2]) + sh[3];
    __syncthreads();
  }
  if (threadIdx.x == 0) Q[b] = nb > 0 ? Qb / nb : 0.0;
}

// dw at the block ends and G_K(n) = gQ_b sum_{K' >= K} w[b, k', n] (ws_g: [nb][B N])
__global__ __launch_bounds__(256) void pl_bwd_eta_kernel(const float *__restrict__ w, const float *__restrict__ lik,
                                                         const float *__restrict__ prior,
                                                         const int64_t *__restrict__ idx,
                                                         const float *__restrict__ gQ, int B, int T, int N, int L,
                                                         float *__restrict__ gw, float *__restrict__ Gk) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= (int64_t)B * N) return;
  const int b = (int)(o / N), n = (int)(o - (int64_t)b * N);
  const int nb = T / L;
  const float g = gQ[b] / (float)nb;
  float e = 0.f;
  for (int K = 0; K < nb; ++K) {
    const int k = (K + 1) * L - 1;
    int64_t p = o;
    for (int s = 0; s < L; ++s) {
      const int64_t a = hist_at(p, k - s, T, N);
      e = (e + prior[a]) + lik[a];
      if (s < L - 1) p = idx[a];
    }
    gw[((int64_t)b * T + k) * N + n] = g * e;
  }
  float acc = 0.f;  // suffix over blocks, from the last
  for (int K = nb - 1; K >= 0; --K) {
    acc += w[((int64_t)b * T + (K + 1) * L - 1) * N + n];
    Gk[(int64_t)K * B * N + o] = g * acc;
  }
}

// one step back for every block at once: offset s within the blocks (j = k - s).  Writes the
// likelihood / prior gradient of step j from G, then (s < L - 1) G_next[m'] = sum of G[m] over
// the run of m with idx[j][m] = m' (binary searches in the non-decreasing flat map).
__global__ __launch_bounds__(256) void pl_bwd_step_kernel(const int64_t *__restrict__ idx, int B, int T, int N,
                                                          int L, int s, const float *__restrict__ G,
                                                          float *__restrict__ Gn, float *__restrict__ glik,
                                                          float *__restrict__ gprior) {
  const int64_t BN = (int64_t)B * N;
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int K = blockIdx.y;
  if (o >= BN) return;
  const int j = (K + 1) * L - 1 - s;
  const float gv = G[(int64_t)K * BN + o];
  const int64_t a = hist_at(o, j, T, N);
  glik[a] = gv;
  gprior[a] = gv;
  if (s == L - 1) return;
  // idx at step j over the flattened batch: element m lives at hist_at(m, j)
  auto at = [&](int64_t m) { return idx[hist_at(m, j, T, N)]; };
  int64_t lo = 0, hi = BN;  // first m with at(m) >= o
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (at(mid) < o) lo = mid + 1; else hi = mid;
  }
  float acc = 0.f;
  for (int64_t m = lo; m < BN && at(m) == o; ++m) acc += G[(int64_t)K * BN + m];
  Gn[(int64_t)K * BN + o] = acc;
}

// 1 if every step's flat ancestor map is non-decreasing (out[0] must be 1 on entry)
__global__ void pl_check_kernel(const int64_t *__restrict__ idx, int B, int T, int N, int32_t *__restrict__ ok) {
  const int64_t BN = (int64_t)B * N;
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int j = blockIdx.y;
  if (o + 1 >= BN) return;
  if (idx[hist_at(o, j, T, N)] > idx[hist_at(o + 1, j, T, N)] || idx[hist_at(o, j, T, N)] < 0 ||
      idx[hist_at(o + 1, j, T, N)] >= BN)
    ok[0] = 0;
}

}  // namespace nfdpf

using namespace nfdpf;

extern "C" int nfdpf_pseudo_lik_forward(const float *w, const float *lik, const float *prior, const int64_t *index,
                                        int B, int T, int N, int block_len, double *Q, void *stream) {
  NFDPF_REQUIRE(w && lik && prior && index && Q, "nfdpf_pseudo_lik_forward: null pointer");
  NFDPF_REQUIRE(B >= 0 && T >= 0 && N >= 1 && N <= 48 * 256 && block_len >= 1,
                "nfdpf_pseudo_lik_forward: bad sizes (N <= 12288)");
  if (B == 0) return NFDPF_OK;
  pl_forward_kernel<<<B, 256, 0, as_stream(stream)>>>(w, lik, prior, index, B, T, N, block_len, Q);
  return launch_status("nfdpf_pseudo_lik_forward");
}

extern "C" int64_t nfdpf_pseudo_lik_workspace(int B, int T, int N, int block_len) {
  if (B < 0 || T < 0 || N < 1 || block_len < 1) return -1;
  const int64_t nb = T / block_len;
  return 4 * (2 * (nb > 0 ? nb : 1) * (int64_t)B * N + 64);
}

extern "C" int nfdpf_pseudo_lik_check(const int64_t *index, int B, int T, int N, int32_t *ok, void *stream) {
  NFDPF_REQUIRE(index && ok, "nfdpf_pseudo_lik_check: null pointer");
  if (B == 0 || T == 0) return NFDPF_OK;
  const int64_t BN = (int64_t)B * N;
  pl_check_kernel<<<dim3((unsigned)((BN + 255) / 256), T), 256, 0, as_stream(stream)>>>(index, B, T, N, ok);
  return launch_status("nfdpf_pseudo_lik_check");
}

extern "C" int nfdpf_pseudo_lik_backward(const float *w, const float *lik, const float *prior, const int64_t *index,
                                         int B, int T, int N, int block_len, const float *g_Q, float *g_w,
                                         float *g_lik, float *g_prior, void *workspace, void *stream) {
  NFDPF_REQUIRE(w && lik && prior && index && g_Q && g_w && g_lik && g_prior && workspace,
                "nfdpf_pseudo_lik_backward: null pointer");
  NFDPF_REQUIRE(B >= 0 && T >= 0 && N >= 1 && block_len >= 1, "nfdpf_pseudo_lik_backward: bad sizes");
  hipStream_t st = as_stream(stream);
  const size_t hist = sizeof(float) * (size_t)B * T * N;
  if (hipMemsetAsync(g_w, 0, hist, st) != hipSuccess || hipMemsetAsync(g_lik, 0, hist, st) != hipSuccess ||
      hipMemsetAsync(g_prior, 0, hist, st) != hipSuccess)
    return launch_status("nfdpf_pseudo_lik_backward (memset)");
  const int nb = T / block_len;
  if (B == 0 || nb == 0) return NFDPF_OK;
  const int64_t BN = (int64_t)B * N;
  float *Ga = (float *)workspace, *Gb = Ga + (int64_t)nb * BN;
  pl_bwd_eta_kernel<<<(unsigned)((BN + 255) / 256), 256, 0, st>>>(w, lik, prior, index, g_Q, B, T, N, block_len,
                                                                   g_w, Ga);
  for (int s = 0; s < block_len; ++s) {
    pl_bwd_step_kernel<<<dim3((unsigned)((BN + 255) / 256), nb), 256, 0, st>>>(index, B, T, N, block_len, s, Ga, Gb,
                                                                                g_lik, g_prior);
    float *t = Ga;
    Ga = Gb;
    Gb = t;
  }
  return launch_status("nfdpf_pseudo_lik_backward");
}
