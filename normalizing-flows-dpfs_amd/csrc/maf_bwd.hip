// maf_bwd.hip -- backward of the MAF stack (NormalizingFlowModel over MAF flows,
// nf/models.py:13-30, nf/flows.py:241-284; training):
//   nfdpf_maf_stack_backward : d/d(x, params) of the stack forward or inverse.
//
// One workgroup = one wave = 64 rows, one row per lane.  The lane re-runs the stack (each
// flow's input kept in registers), then walks the flows backwards.  Per flow and dimension i
// it recomputes FCNN_i(x_{<i}) and back-propagates (mu_i, alpha_i):
//   forward  z_i = (x_i - mu_i) e^{-alpha_i}, log-det -= alpha_i, output flipped;
//   inverse  x_i = mu_i + e^{alpha_i} z_i (z = flipped input), log-det += alpha_i, i from the
//            last dimension down (x_{<i} feed later dimensions' nets).
// The parameter gradient is left as outer-product factors in LDS (the net input u, g_z1, h1,
// g_z2, h2, g_o per FCNN; g of initial_param), contracted over the wave's 64 rows with lane =
// parameter into a per-workgroup partial, summed over workgroups in a fixed order by
// param_reduce (deterministic).
#include "flows.hpp"

namespace nfdpf {

constexpr int kMafRows = 64;
constexpr int kMafMaxFlows = 4;

// factors of one flow per row: [g_init 2] then per i = 1..D-1: [u (i) | g_z1 (H) | h1 (H) |
// g_z2 (H) | h2 (H) | g_o (2)]
template <int D, int H>
__host__ __device__ constexpr int maf_fac(int upto) {  // offset of FCNN_upto's block
  int s = 2;
  for (int i = 1; i < upto; ++i) s += i + 4 * H + 2;
  return s;
}

// FCNN_i (i -> H -> H -> 2, tanh) on u: outputs o, keeps h1, h2
template <int H>
__device__ __forceinline__ void fcnn_fwd(cfloat *w, int in, const float *u, float (&h1)[H], float (&h2)[H],
                                         float (&o)[2]) {
#pragma unroll
  for (int j = 0; j < H; ++j) {
    float a = w[H * in + j];
    for (int k = 0; k < in; ++k) a = fmaf(w[j * in + k], u[k], a);
    h1[j] = tanh_fast(a);
  }
  cfloat *w2 = w + H * in + H;
#pragma unroll
  for (int j = 0; j < H; ++j) {
    float a = w2[H * H + j];
#pragma unroll
    for (int k = 0; k < H; ++k) a = fmaf(w2[j * H + k], h1[k], a);
    h2[j] = tanh_fast(a);
  }
  cfloat *w3 = w2 + H * H + H;
#pragma unroll
  for (int q = 0; q < 2; ++q) {
    float a = w3[2 * H + q];
#pragma unroll
    for (int k = 0; k < H; ++k) a = fmaf(w3[q * H + k], h2[k], a);
    o[q] = a;
  }
}

// its backward for g_o: adds d/du into gu[0..in), writes the factors at fac (stride kMafRows)
template <int H>
__device__ __forceinline__ void fcnn_bwd(cfloat *w, int in, const float *u, const float (&h1)[H],
                                         const float (&h2)[H], const float (&go)[2], float *gu, float *fac) {
  cfloat *w2 = w + H * in + H, *w3 = w2 + H * H + H;
  float gz2[H], gz1[H];
#pragma unroll
  for (int k = 0; k < H; ++k) {
    const float g = fmaf(w3[H + k], go[1], w3[k] * go[0]);
    gz2[k] = g * (1.f - h2[k] * h2[k]);
  }
#pragma unroll
  for (int k = 0; k < H; ++k) {
    float g = 0.f;
#pragma unroll
    for (int j = 0; j < H; ++j) g = fmaf(w2[j * H + k], gz2[j], g);
    gz1[k] = g * (1.f - h1[k] * h1[k]);
  }
  for (int k = 0; k < in; ++k) {
    float g = 0.f;
#pragma unroll
    for (int j = 0; j < H; ++j) g = fmaf(w[j * in + k], gz1[j], g);
    gu[k] += g;
  }
  int o = 0;
  for (int k = 0; k < in; ++k) fac[(o++) * kMafRows] = u[k];
#pragma unroll
  for (int j = 0; j < H; ++j) fac[(o + j) * kMafRows] = gz1[j];
#pragma unroll
  for (int j = 0; j < H; ++j) fac[(o + H + j) * kMafRows] = h1[j];
#pragma unroll
  for (int j = 0; j < H; ++j) fac[(o + 2 * H + j) * kMafRows] = gz2[j];
#pragma unroll
  for (int j = 0; j < H; ++j) fac[(o + 3 * H + j) * kMafRows] = h2[j];
  fac[(o + 4 * H) * kMafRows] = go[0];
  fac[(o + 4 * H + 1) * kMafRows] = go[1];
}

// one flow's backward (forward or inverse map) on its input v; g: dL/d(output) in, dL/d(input)
// out; gl: dL/d log-det.  fac: this flow's factor block (row lane).
template <int D, int H, bool INV>
__device__ __forceinline__ void maf_flow_bwd(cfloat *fw, const float (&v)[D], float (&g)[D], float gl, float *fac) {
  float x[D], z[D], mu[D], al[D];
  // recompute (maf_forward / maf_inverse of flows.hpp)
  {
    cfloat *w = fw + 2;
#pragma unroll
    for (int i = 0; i < D; ++i) {
      if (INV) z[i] = v[D - 1 - i];
      if (i == 0) {
        mu[0] = fw[0];
        al[0] = fw[1];
      } else {
        float h1[H], h2[H], o[2];
        fcnn_fwd<H>(w, i, INV ? x : v, h1, h2, o);
        w += fcnn_size<H>(i, 2);
        mu[i] = o[0];
        al[i] = o[1];
      }
      if (INV) {
        x[i] = mu[i] + expf(al[i]) * z[i];
      } else {
        x[i] = v[i];
        z[i] = (v[i] - mu[i]) / expf(al[i]);
      }
    }
  }
  float gxi[D];  // dL/dx_i (forward: the input; inverse: the output)
#pragma unroll
  for (int i = 0; i < D; ++i) gxi[i] = INV ? g[i] : 0.f;
  float gz[D];
#pragma unroll
  for (int i = D - 1; i >= 0; --i) {
    float gm, ga;
    if (INV) {  // x_i = mu_i + e^{alpha_i} z_i, log-det += alpha_i
      const float e = expf(al[i]);
      gm = gxi[i];
      ga = fmaf(gxi[i] * e, z[i], gl);
      gz[i] = gxi[i] * e;
    } else {    // z_i = (x_i - mu_i) / e^{alpha_i}, log-det -= alpha_i; output flipped
      const float e = expf(al[i]), gzi = g[D - 1 - i];
      gxi[i] += gzi / e;
      gm = -gzi / e;
      ga = -gzi * z[i] - gl;
    }
    if (i == 0) {
      fac[0] = gm;
      fac[kMafRows] = ga;
    } else {
      cfloat *w = fw + 2;
      for (int k = 1; k < i; ++k) w += fcnn_size<H>(k, 2);
      float h1[H], h2[H], o[2];
      fcnn_fwd<H>(w, i, x, h1, h2, o);
      const float go[2] = {gm, ga};
      fcnn_bwd<H>(w, i, x, h1, h2, go, gxi, fac + maf_fac<D, H>(i) * kMafRows);
    }
  }
#pragma unroll
  for (int i = 0; i < D; ++i) g[i] = INV ? gz[D - 1 - i] : gxi[i];
}

// parameter p of one flow's blob segment -> its contraction over the wave's rows
template <int D, int H>
__device__ __forceinline__ float maf_contract(const float *fac, int p) {
  auto dot = [&](int a, int b) {
    float s = 0.f;
    for (int r = 0; r < kMafRows; ++r) s = fmaf(fac[a * kMafRows + r], b < 0 ? 1.f : fac[b * kMafRows + r], s);
    return s;
  };
  if (p < 2) return dot(p, -1);
  p -= 2;
  for (int i = 1; i < D; ++i) {
    const int f0 = maf_fac<D, H>(i), u = f0, gz1 = f0 + i, h1 = gz1 + H, gz2 = h1 + H, h2 = gz2 + H, go = h2 + H;
    if (p < H * i) return dot(gz1 + p / i, u + p % i);
    p -= H * i;
    if (p < H) return dot(gz1 + p, -1);
    p -= H;
    if (p < H * H) return dot(gz2 + p / H, h1 + p % H);
    p -= H * H;
    if (p < H) return dot(gz2 + p, -1);
    p -= H;
    if (p < 2 * H) return dot(go + p / H, h2 + p % H);
    p -= 2 * H;
    if (p < 2) return dot(go + p, -1);
    p -= 2;
  }
  return 0.f;
}

template <int D, int H, bool INV>
__global__ __launch_bounds__(kMafRows) void maf_bwd_kernel(const float *__restrict__ params, int nf,
                                                           const float *__restrict__ x, int64_t rows,
                                                           const float *__restrict__ gout,
                                                           const float *__restrict__ gld, float *__restrict__ gx,
                                                           float *__restrict__ partial) {
  extern __shared__ float fac[];  // [nf][maf_fac<D,H>(D)][kMafRows]
  constexpr int F = maf_fac<D, H>(D);
  const int lane = threadIdx.x;
  const int64_t r = (int64_t)blockIdx.x * kMafRows + lane;
  const bool valid = r < rows;
  const int fs = maf_size<H>(D);
  cfloat *P = wptr(params);
  float cur[D], g[D];
#pragma unroll
  for (int k = 0; k < D; ++k) {
    cur[k] = valid ? x[r * D + k] : 0.f;
    g[k] = valid && gout ? gout[r * D + k] : 0.f;
  }
  const float gl = valid && gld ? gld[r] : 0.f;
  float xin[kMafMaxFlows][D];
  for (int s = 0; s < nf; ++s) {  // the stack in application order, each flow's input kept
    const int f = INV ? nf - 1 - s : s;
#pragma unroll
    for (int k = 0; k < D; ++k) xin[s][k] = cur[k];
    if (INV)
      maf_inverse<D, H>(P + f * fs, cur);
    else
      maf_forward<D, H>(P + f * fs, cur);
  }
  for (int s = nf - 1; s >= 0; --s) {
    const int f = INV ? nf - 1 - s : s;
    float v[D];
#pragma unroll
    for (int k = 0; k < D; ++k) v[k] = xin[s][k];
    maf_flow_bwd<D, H, INV>(P + f * fs, v, g, gl, fac + (size_t)f * F * kMafRows + lane);
  }
  if (valid)
#pragma unroll
    for (int k = 0; k < D; ++k) gx[r * D + k] = g[k];
  __syncthreads();
  // contraction: lane = parameter of the stack's blob
  const int Ptot = nf * fs;
  for (int p = lane; p < Ptot; p += kMafRows) {
    const int f = p / fs;
    partial[(int64_t)blockIdx.x * Ptot + p] = maf_contract<D, H>(fac + (size_t)f * F * kMafRows, p - f * fs);
  }
}

__global__ __launch_bounds__(256) void maf_param_reduce_kernel(const float *__restrict__ partial, int64_t n_parts,
                                                               int64_t P, float *__restrict__ out) {
  __shared__ float red[4][64];
  const int c = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t p = (int64_t)blockIdx.x * 64 + c;
  float acc = 0.f;
  if (p < P)
    for (int64_t b = g; b < n_parts; b += 4) acc += partial[b * P + p];
  red[g][c] = acc;
  __syncthreads();
  if (g == 0 && p < P) out[p] = ((red[0][c] + red[1][c]) + red[2][c]) + red[3][c];
}

template <int D>
static int maf_bwd_launch(bool inv, hipStream_t st, const float *params, int nf, const float *x, int64_t rows,
                          const float *gout, const float *gld, float *gx, float *g_params, float *ws) {
  constexpr int H = 8;
  const int64_t nb = (rows + kMafRows - 1) / kMafRows;
  const int64_t P = (int64_t)nf * maf_size<H>(D);
  const size_t lds = sizeof(float) * (size_t)nf * maf_fac<D, H>(D) * kMafRows;
  if (inv)
    maf_bwd_kernel<D, H, true><<<(unsigned)nb, kMafRows, lds, st>>>(params, nf, x, rows, gout, gld, gx, ws);
  else
    maf_bwd_kernel<D, H, false><<<(unsigned)nb, kMafRows, lds, st>>>(params, nf, x, rows, gout, gld, gx, ws);
  maf_param_reduce_kernel<<<(unsigned)((P + 63) / 64), 256, 0, st>>>(ws, nb, P, g_params);
  return launch_status("nfdpf_maf_stack_backward");
}

}  // namespace nfdpf

using namespace nfdpf;

extern "C" int64_t nfdpf_maf_stack_backward_workspace(int n_flows, int dim, int hidden, int64_t rows) {
  if (hidden != 8 || (dim != 2 && dim != 4) || n_flows < 1 || n_flows > kMafMaxFlows || rows < 0) return -1;
  const int64_t nb = (rows + kMafRows - 1) / kMafRows;
  const int64_t P = (int64_t)n_flows * (dim == 2 ? maf_size<8>(2) : maf_size<8>(4));
  return 4 * (nb > 0 ? nb : 1) * P;
}

extern "C" int nfdpf_maf_stack_backward(const float *params, int n_flows, int dim, int hidden, const float *x,
                                        int64_t rows, int inverse, const float *g_out, const float *g_logdet,
                                        float *g_x, float *g_params, void *workspace, void *stream) {
  NFDPF_REQUIRE(params && x && g_x && g_params && workspace, "nfdpf_maf_stack_backward: null pointer");
  NFDPF_REQUIRE(hidden == 8 && (dim == 2 || dim == 4), "nfdpf_maf_stack_backward: dim 2 or 4, hidden 8");
  NFDPF_REQUIRE(n_flows >= 1 && n_flows <= kMafMaxFlows && rows >= 0, "nfdpf_maf_stack_backward: bad sizes");
  const size_t lds = sizeof(float) * (size_t)n_flows * (dim == 2 ? maf_fac<2, 8>(2) : maf_fac<4, 8>(4)) * kMafRows;
  NFDPF_REQUIRE(lds <= 65536, "nfdpf_maf_stack_backward: %d flows of dim %d exceed the LDS factor budget", n_flows,
                dim);
  if (rows == 0) {
    if (hipMemsetAsync(g_params, 0, sizeof(float) * (size_t)n_flows * (dim == 2 ? maf_size<8>(2) : maf_size<8>(4)),
                       as_stream(stream)) != hipSuccess)
      return launch_status("nfdpf_maf_stack_backward (memset)");
    return NFDPF_OK;
  }
  hipStream_t st = as_stream(stream);
  float *ws = (float *)workspace;
  return dim == 2 ? maf_bwd_launch<2>(inverse != 0, st, params, n_flows, x, rows, g_out, g_logdet, g_x, g_params, ws)
                  : maf_bwd_launch<4>(inverse != 0, st, params, n_flows, x, rows, g_out, g_logdet, g_x, g_params, ws);
}
