// flows.hip -- standalone flow-stack kernels behind the C ABI:
//   nfdpf_cond_stack  : NormalizingFlowModel_cond over RealNVP_cond (nf/models.py:37-61),
//                       obser_dim = 0 -> unconditional RealNVP stack (nf/models.py:5-30)
//   nfdpf_maf_stack   : NormalizingFlowModel over MAF flows (nf/flows.py:241-284)
// One particle (row) per lane; rows are independent, so the grid is rows/256 workgroups.
#include "flows.hpp"

namespace nfdpf {

constexpr int kStackBlock = 256;

// Conditional affine-coupling stack.  Context is either per row (cond_group == 1) or
// shared by cond_group consecutive rows; either way each lane folds it into the first
// layer itself (the fused filter step amortises that fold per batch row instead).
template <int HALF, int H, bool INV>
__global__ __launch_bounds__(kStackBlock) void cond_stack_kernel(
    const float *__restrict__ params, int n_flows, int O, const float *__restrict__ x,
    const float *__restrict__ cond, int64_t rows, int64_t cond_group, float prior_mean,
    float prior_std, float *__restrict__ out, float *__restrict__ logdet,
    float *__restrict__ prior_lp) {
  const int64_t r = (int64_t)blockIdx.x * kStackBlock + threadIdx.x;
  if (r >= rows) return;
  constexpr int D = 2 * HALF;
  const int ns = net_size<HALF, H>(O);
  float lo[HALF], up[HALF];
#pragma unroll
  for (int k = 0; k < HALF; ++k) {
    lo[k] = x[r * D + k];
    up[k] = x[r * D + HALF + k];
  }
  const float *c = cond ? cond + (r / cond_group) * O : nullptr;
  float ld = 0.f;
  f2 cb[2 * H];
  for (int f = 0; f < n_flows; ++f) {
    const int fi = INV ? n_flows - 1 - f : f;
    cf2 *fw = wptr2(params) + fi * 2 * ns;
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int j = 0; j < H; ++j) cb[n * H + j] = fold_pair<HALF, H>(fw + n * ns, O, j, c);
    const float l = INV ? coupling_inverse<HALF, H>(fw, O, lo, up, cb)
                        : coupling_forward<HALF, H>(fw, O, lo, up, cb);
    ld += l;
  }
#pragma unroll
  for (int k = 0; k < HALF; ++k) {
    out[r * D + k] = lo[k];
    out[r * D + HALF + k] = up[k];
  }
  logdet[r] = ld;
  if (!INV && prior_lp) {
    // MultivariateNormal(mean*1, std^2 I).log_prob (nf/models.py:51)
    float m = 0.f;
#pragma unroll
    for (int k = 0; k < HALF; ++k) {
      const float a = (lo[k] - prior_mean) / prior_std, b = (up[k] - prior_mean) / prior_std;
      m = fmaf(a, a, m);
      m = fmaf(b, b, m);
    }
    const float kLog2Pi = 1.8378770664093453f;
    prior_lp[r] = -0.5f * (D * kLog2Pi + m) - D * logf(prior_std);
  }
}

template <int HALF, int H>
static void launch_cond(bool inv, dim3 g, hipStream_t st, const float *params, int n_flows, int O,
                        const float *x, const float *cond, int64_t rows, int64_t cg, float pm,
                        float ps, float *out, float *ld, float *lp) {
  if (inv)
    cond_stack_kernel<HALF, H, true><<<g, kStackBlock, 0, st>>>(params, n_flows, O, x, cond, rows,
                                                                cg, pm, ps, out, ld, lp);
  else
    cond_stack_kernel<HALF, H, false><<<g, kStackBlock, 0, st>>>(params, n_flows, O, x, cond, rows,
                                                                 cg, pm, ps, out, ld, lp);
}

template <int D, int H, bool INV>
__global__ __launch_bounds__(kStackBlock) void maf_stack_kernel(const float *__restrict__ params,
                                                               int n_flows,
                                                               const float *__restrict__ x,
                                                               int64_t rows,
                                                               float *__restrict__ out,
                                                               float *__restrict__ logdet) {
  const int64_t r = (int64_t)blockIdx.x * kStackBlock + threadIdx.x;
  if (r >= rows) return;
  float v[D];
#pragma unroll
  for (int k = 0; k < D; ++k) v[k] = x[r * D + k];
  const int fs = maf_size<H>(D);
  float ld = 0.f;
  for (int f = 0; f < n_flows; ++f) {
    const int fi = INV ? n_flows - 1 - f : f;
    const float l = INV ? maf_inverse<D, H>(wptr(params) + fi * fs, v)
                        : maf_forward<D, H>(wptr(params) + fi * fs, v);
    ld += l;
  }
#pragma unroll
  for (int k = 0; k < D; ++k) out[r * D + k] = v[k];
  logdet[r] = ld;
}

template <int D, int H>
static void launch_maf(bool inv, dim3 g, hipStream_t st, const float *p, int nf, const float *x,
                       int64_t rows, float *out, float *ld) {
  if (inv)
    maf_stack_kernel<D, H, true><<<g, kStackBlock, 0, st>>>(p, nf, x, rows, out, ld);
  else
    maf_stack_kernel<D, H, false><<<g, kStackBlock, 0, st>>>(p, nf, x, rows, out, ld);
}

}  // namespace nfdpf

using namespace nfdpf;

extern "C" int nfdpf_cond_stack(const float *params, int n_flows, int dim, int obser_dim,
                                int hidden, const float *x, const float *cond, int64_t rows,
                                int64_t cond_group, int inverse, float prior_mean,
                                float prior_std, float *out, float *logdet, float *prior_logprob,
                                void *stream) {
  NFDPF_REQUIRE(params && x && out && logdet, "nfdpf_cond_stack: null pointer");
  NFDPF_REQUIRE(n_flows >= 0 && rows >= 0 && obser_dim >= 0, "nfdpf_cond_stack: bad sizes");
  NFDPF_REQUIRE(obser_dim == 0 || (cond && cond_group >= 1), "nfdpf_cond_stack: cond missing");
  NFDPF_REQUIRE(prior_std > 0.f, "nfdpf_cond_stack: prior_std must be > 0");
  if (rows == 0) return NFDPF_OK;
  const dim3 g((unsigned)((rows + kStackBlock - 1) / kStackBlock));
  hipStream_t st = as_stream(stream);
  const bool inv = inverse != 0;
#define NFDPF_COND(HALF, H)                                                                   \
  if (dim == 2 * HALF && hidden == H) {                                                       \
    launch_cond<HALF, H>(inv, g, st, params, n_flows, obser_dim, x, cond, rows, cond_group,   \
                         prior_mean, prior_std, out, logdet, prior_logprob);                  \
    return launch_status("nfdpf_cond_stack");                                                 \
  }
  NFDPF_COND(1, 8)
  NFDPF_COND(2, 8)
  NFDPF_COND(16, 8)
  NFDPF_COND(1, 16)
  NFDPF_COND(16, 16)
  NFDPF_COND(1, 32)
#undef NFDPF_COND
  set_error("nfdpf_cond_stack: unsupported (dim=%d, hidden=%d); built for dim in {2,4,32}, "
            "hidden in {8,16,32}",
            dim, hidden);
  return NFDPF_EINVAL;
}

extern "C" int nfdpf_maf_stack(const float *params, int n_flows, int dim, int hidden,
                               const float *x, int64_t rows, int inverse, float *out,
                               float *logdet, void *stream) {
  NFDPF_REQUIRE(params && x && out && logdet, "nfdpf_maf_stack: null pointer");
  NFDPF_REQUIRE(n_flows >= 0 && rows >= 0, "nfdpf_maf_stack: bad sizes");
  if (rows == 0) return NFDPF_OK;
  const dim3 g((unsigned)((rows + kStackBlock - 1) / kStackBlock));
  hipStream_t st = as_stream(stream);
  const bool inv = inverse != 0;
#define NFDPF_MAF(D, H)                                                      \
  if (dim == D && hidden == H) {                                             \
    launch_maf<D, H>(inv, g, st, params, n_flows, x, rows, out, logdet);     \
    return launch_status("nfdpf_maf_stack");                                 \
  }
  NFDPF_MAF(2, 8)
  NFDPF_MAF(3, 8)
  NFDPF_MAF(4, 8)
  NFDPF_MAF(6, 8)
  NFDPF_MAF(8, 8)
#undef NFDPF_MAF
  set_error("nfdpf_maf_stack: unsupported (dim=%d, hidden=%d); built for dim in {2,3,4,6,8}, "
            "hidden 8",
            dim, hidden);
  return NFDPF_EINVAL;
}
