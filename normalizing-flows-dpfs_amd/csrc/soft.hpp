// soft.hpp -- soft resampling of one batch row by one workgroup (resamplers.py:20-60).
//
// Bit-exact with the reference on CPU for the same (p, offsets, linspace):
//   q_j  = f32(p_j * a) + f32(u * (1 - a)),   u = f32(1/N)                 (:26-32)
//   S    = torch.sum(q) in ATen's CPU cascade order (cascade_row_sum)       (:33)
//   q_j /= S;  w_j = p_j / q_j                                              (:33-34)
//   C_j  = f32(sum_{k<=j} f64(q_k)), C_{N-1} = 1                            (:45-47)
//          the f64 prefix is EXACT (every q_k is a multiple of 2^-52 * 2^e with all
//          partial sums < 2), so a parallel scan equals the reference's serial one;
//   idx_i = #{j : C_j < off + lin_i}: binary search over the monotone C_0..C_{N-2} plus
//           the forced last entry                                           (:49-50)
//   w'_i  = w_{idx_i} / torch.sum(w_idx) (cascade order again)              (:55-56)
#pragma once

#include "common.hpp"

namespace nfdpf {

struct SoftRow {
  const float *p;  // [N] probabilities of this row
  int N;
  float alpha, u, one_minus_alpha;
  float S;         // cascade sum of q_raw
  __device__ __forceinline__ float q_raw(int j) const { return q_raw_of(p[j]); }
  __device__ __forceinline__ float q_raw_of(float pj) const {
#pragma clang fp contract(off)
    return alpha < 1.0f ? pj * alpha + u * one_minus_alpha : pj;
  }
  __device__ __forceinline__ float q(int j) const { return alpha < 1.0f ? q_raw(j) / S : p[j]; }
  __device__ __forceinline__ float w(int j) const { return alpha < 1.0f ? p[j] / q(j) : u; }
};

// Steps 1-3: S, C (into LDS `C`), per-thread marker search.  For every particle i of this
// thread (i = tid + k*blockDim) calls emit(i, src) with src = idx_i (may be N at the
// reference's own out-of-range edge).  `shd` >= 16 doubles, `shf` >= 1 float.
template <class Emit>
__device__ void soft_row_search(SoftRow &row, const float *lin, float off, float *C, double *shd,
                                float *shf, const Emit &emit) {
  const int N = row.N;
  const int tid = threadIdx.x, nth = blockDim.x;
  if (row.alpha < 1.0f) {
    if (tid < 64) {
      const float S = cascade_row_sum([&](int j) { return row.q_raw(j); }, N);
      if (tid == 0) shf[0] = S;
    }
    __syncthreads();
    row.S = shf[0];
  }
  // exact f64 prefix of q over per-thread contiguous chunks
  const int chunk = (N + nth - 1) / nth;
  const int j0 = min(N, tid * chunk), j1 = min(N, j0 + chunk);
  double part = 0.0;
  for (int j = j0; j < j1; ++j) part += (double)row.q(j);
  double run = block_exclusive_scan(part, shd, (double *)nullptr);
  for (int j = j0; j < j1; ++j) {
    run += (double)row.q(j);
    C[j] = (float)run;
  }
  __syncthreads();
  for (int i = tid; i < N; i += nth) {
    const float m = off + lin[i];
    int lo = 0, hi = N - 1;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (C[mid] < m)
        lo = mid + 1;
      else
        hi = mid;
    }
    emit(i, lo + (1.0f < m ? 1 : 0));
  }
}

}  // namespace nfdpf
