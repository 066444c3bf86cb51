// rqs.hip -- the unconstrained rational-quadratic spline of the neural spline flows
// (nf/utils.py:23-147 of the reference: unconstrained_RQS + RQS, used by NSF_AR / NSF_CL,
// nf/flows.py:343-458), one element per lane with its K bins in registers.
//
// The per-element parameter rows (K widths, K heights, K-1 inner derivatives) are read
// once and the bin tables never leave the lane; the reference materialises them as
// (M, K+1) tensors through ~30 ATen ops.  Arithmetic follows the reference's op order in
// fp32: softmax (max shift, exp, sum, divide), the bin floor min + (1 - min K) w, cumsum
// accumulated in fp64 and rounded per prefix (ATen's CPU cumsum of a float tensor), the
// pinned end knots, softplus (threshold 20) derivatives with the constant boundary
// derivative, the searchsorted with its +1e-6 on the last knot, then the forward map or the
// quadratic root of the inverse.
#include "common.hpp"

#include <cmath>

namespace nfdpf {

constexpr int kRqsMaxK = 32;

__device__ __forceinline__ float softplus1(float v) { return v > 20.f ? v : log1pf(expf(v)); }

// knots of one axis (widths or heights): loc[0..K], len[0..K-1]
__device__ __forceinline__ void rqs_knots(const float *u, int K, float lo, float hi, float min_bin, float scale,
                                          float *loc, float *len) {
#pragma clang fp contract(off)
  float m = u[0];
  for (int k = 1; k < K; ++k) m = fmaxf(m, u[k]);
  float e[kRqsMaxK];
  float s = 0.f;
  for (int k = 0; k < K; ++k) {
    e[k] = expf(u[k] - m);
    s += e[k];
  }
  double acc = 0.0;
  loc[0] = lo;
  for (int k = 0; k < K; ++k) {
    const float w = min_bin + scale * (e[k] / s);
    acc += (double)w;
    loc[k + 1] = (hi - lo) * (float)acc + lo;
  }
  loc[K] = hi;
  for (int k = 0; k < K; ++k) len[k] = loc[k + 1] - loc[k];
}

__global__ void rqs_kernel(const float *__restrict__ x, const float *__restrict__ W, const float *__restrict__ H,
                           const float *__restrict__ D, int64_t M, int K, int full_d, int inverse, float left,
                           float right, float bottom, float top, int tails, float min_w, float min_h, float min_d,
                           float scale_w, float scale_h, float bound_d, float *__restrict__ y,
                           float *__restrict__ logdet) {
#pragma clang fp contract(off)
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= M) return;
  const float v = x[o];
  if (tails && !(v >= left && v <= right)) {  // outside the tail bound: identity (nf/utils.py:41-42)
    y[o] = v;
    logdet[o] = 0.f;
    return;
  }
  float cw[kRqsMaxK + 1], wd[kRqsMaxK], ch[kRqsMaxK + 1], ht[kRqsMaxK], dv[kRqsMaxK + 1];
  rqs_knots(W + o * K, K, left, right, min_w, scale_w, cw, wd);
  rqs_knots(H + o * K, K, bottom, top, min_h, scale_h, ch, ht);
  if (full_d) {  // RQS: all K + 1 derivatives given
    for (int k = 0; k <= K; ++k) dv[k] = min_d + softplus1(D[o * (K + 1) + k]);
  } else {       // unconstrained_RQS: inner K - 1, the two boundary ones the constant
    dv[0] = min_d + softplus1(bound_d);
    dv[K] = dv[0];
    for (int k = 1; k < K; ++k) dv[k] = min_d + softplus1(D[o * (K - 1) + k - 1]);
  }
  // searchsorted (nf/utils.py:16-21): #{k : v >= loc_k} - 1, the last knot lifted by 1e-6
  const float *loc = inverse ? ch : cw;
  int bin = -1;
  for (int k = 0; k <= K; ++k) bin += v >= (k == K ? loc[K] + 1e-6f : loc[k]);
  bin = bin < 0 ? 0 : (bin > K - 1 ? K - 1 : bin);  // in-domain inputs always land in [0, K-1]
  const float icw = cw[bin], iw = wd[bin], ich = ch[bin], ih = ht[bin];
  const float delta = ih / iw;
  const float d0 = dv[bin], d1 = dv[bin + 1];
  if (inverse) {
    const float r = v - ich;
    const float a = r * (d0 + d1 - 2.f * delta) + ih * (delta - d0);
    const float b = ih * d0 - r * (d0 + d1 - 2.f * delta);
    const float c = -delta * r;
    const float disc = b * b - 4.f * a * c;
    const float root = (2.f * c) / (-b - sqrtf(disc));
    y[o] = root * iw + icw;
    const float tt = root * (1.f - root);
    const float den = delta + (d0 + d1 - 2.f * delta) * tt;
    const float num = delta * delta * (d1 * (root * root) + 2.f * delta * tt + d0 * ((1.f - root) * (1.f - root)));
    logdet[o] = -(logf(num) - 2.f * logf(den));
  } else {
    const float th = (v - icw) / iw;
    const float tt = th * (1.f - th);
    const float num = ih * (delta * (th * th) + d0 * tt);
    const float den = delta + (d0 + d1 - 2.f * delta) * tt;
    y[o] = ich + num / den;
    const float dn = delta * delta * (d1 * (th * th) + 2.f * delta * tt + d0 * ((1.f - th) * (1.f - th)));
    logdet[o] = logf(dn) - 2.f * logf(den);
  }
}

}  // namespace nfdpf

using namespace nfdpf;

extern "C" int nfdpf_rqs(const float *x, const float *W, const float *H, const float *D, int64_t M, int K,
                         int full_derivatives, int inverse, float left, float right, float bottom, float top,
                         int tails, float min_bin_width, float min_bin_height, float min_derivative, float *y,
                         float *logdet, void *stream) {
  NFDPF_REQUIRE(M >= 0 && K >= 1 && K <= kRqsMaxK, "nfdpf_rqs: bad sizes (M=%lld, K=%d, K <= %d)", (long long)M,
                K, kRqsMaxK);
  NFDPF_REQUIRE(x && W && H && (D || (K == 1 && !full_derivatives)) && y && logdet, "nfdpf_rqs: null pointer");
  NFDPF_REQUIRE(min_bin_width * K <= 1.f, "nfdpf_rqs: Minimal bin width too large for the number of bins");
  NFDPF_REQUIRE(min_bin_height * K <= 1.f, "nfdpf_rqs: Minimal bin height too large for the number of bins");
  NFDPF_REQUIRE(right > left && top > bottom, "nfdpf_rqs: empty interval");
  if (M == 0) return NFDPF_OK;
  // the boundary derivatives' unnormalised value log(e^(1 - min_d) - 1) (nf/utils.py:35-37)
  const float bound_d = (float)std::log(std::exp(1.0 - (double)min_derivative) - 1.0);
  // 1 - min K, evaluated in double as the reference's Python scalars are, then rounded
  const float scale_w = (float)(1.0 - (double)min_bin_width * K), scale_h = (float)(1.0 - (double)min_bin_height * K);
  rqs_kernel<<<(unsigned)((M + 255) / 256), 256, 0, as_stream(stream)>>>(
      x, W, H, D, M, K, full_derivatives, inverse, left, right, bottom, top, tails, min_bin_width, min_bin_height,
      min_derivative, scale_w, scale_h, bound_d, y, logdet);
  return launch_status("nfdpf_rqs");
}
