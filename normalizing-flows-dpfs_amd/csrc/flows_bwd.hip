// flows_bwd.hip -- backward of the coupling-flow stack (training):
//   nfdpf_cond_stack_backward : d/d(x, cond, params) of NormalizingFlowModel_cond.forward /
//                               .inverse over RealNVP_cond flows (nf/models.py:45-61,
//                               nf/flows.py:215-239), prior log-prob term included (:51)
//
// One workgroup = one wave = 64 rows, one row per lane.  Each lane re-runs the stack forward
// (flow inputs kept in LDS), then walks the coupling halves backwards.  Per half it needs the
// net's activations again (recomputed from the half's input: one forward of the t/s pair), and
// leaves the outer-product factors of the parameter gradient in LDS:
//   dW1 = g_z1 (x) [u, c],  dW2 = g_z2 (x) h1,  dW3 = g_o (x) h2,  db = g_z / g_o
// The wave then contracts them over its 64 rows (lane = parameter pair) into this workgroup's
// partial -- a deterministic per-workgroup sum, reduced over workgroups in a fixed order by
// nfdpf_cond_stack_param_reduce.  d/d cond is the same contraction the other way round
// (per row: sum over halves and hidden units of W1c^T g_z1), done once at the end with
// lane = (row, context column) so its stores are coalesced.
#include "flows.hpp"

namespace nfdpf {

constexpr int kBwdRows = 64;
constexpr int kBwdMaxFlows = 4;

template <int HALF, int H>
struct BwdLds {
  static constexpr int D = 2 * HALF;
  static constexpr int PF = 4 * H + HALF;  // f2 factors per row: g_z1, h1, g_z2, h2, g_o
  // byte offsets of the regions (dynamic LDS)
  static __host__ __device__ int sfs(int O) { return HALF + O; }  // f32 per row: u, c
  static __host__ __device__ size_t pf_off() { return 0; }
  static __host__ __device__ size_t gz_off() { return sizeof(f2) * kBwdRows * PF; }
  static __host__ __device__ size_t sf_off(int nf) {
    return gz_off() + sizeof(f2) * (size_t)nf * 2 * kBwdRows * H;
  }
  static __host__ __device__ size_t xin_off(int nf, int O) {
    return sf_off(nf) + sizeof(float) * (size_t)kBwdRows * sfs(O);
  }
  static __host__ __device__ size_t cbs_off(int nf, int O) {
    return xin_off(nf, O) + sizeof(float) * (size_t)nf * D * kBwdRows;
  }
  // folded first-layer biases of every flow ([flow][2H][row] f2), kept from the recompute
  static __host__ __device__ size_t bytes(int nf, int O) {
    return cbs_off(nf, O) + sizeof(f2) * (size_t)nf * 2 * H * kBwdRows;
  }
};

// One coupling half: nets t, s on input u; forward y' = t + y e^s (log-det += sum s),
// inverse y' = (y - t) e^{-s} (log-det -= sum s).  In: gy = dL/dy', gl = dL/dlogdet.
// Out: gy = dL/dy, gu = dL/du; the row's gradient factors go to pf (f2) / uf (f32).
template <int HALF, int H, bool INV>
__device__ __forceinline__ void half_bwd(cf2 *w, const f2 *cb, const float (&u)[HALF],
                                         const float (&y)[HALF], float (&gy)[HALF], float gl,
                                         float (&gu)[HALF], f2 *pf, float *uf, f2 *gz_keep) {
  f2 h1[H], h2[H];
#pragma unroll
  for (int j = 0; j < H; ++j) {
    f2 a = cb[j];
#pragma unroll
    for (int k = 0; k < HALF; ++k) a = pfma(w[j * HALF + k], splat(u[k]), a);
    h1[j] = tanh2(a);
  }
  cf2 *w2 = w + H * HALF;
#pragma unroll
  for (int j = 0; j < H; ++j) {
    f2 a = w2[H * H + j];
#pragma unroll
    for (int k = 0; k < H; ++k) a = pfma(w2[j * H + k], h1[k], a);
    h2[j] = tanh2(a);
  }
  cf2 *w3 = w2 + H * H + H;
  f2 go[HALF];
#pragma unroll
  for (int o = 0; o < HALF; ++o) {
    f2 a = w3[HALF * H + o];
#pragma unroll
    for (int k = 0; k < H; ++k) a = pfma(w3[o * H + k], h2[k], a);
    const float t = a.x, s = a.y;
    if (!INV) {  // nf/flows.py:220,225: y' = t + y * exp(s)
      const float e = expf(s);
      go[o] = f2{gy[o], fmaf(gy[o] * y[o], e, gl)};
      gy[o] *= e;
    } else {     // nf/flows.py:233,237: y' = (y - t) * exp(-s)
      const float e = expf(-s);
      const float yp = (y[o] - t) * e;
      go[o] = f2{-gy[o] * e, -fmaf(gy[o], yp, gl)};
      gy[o] *= e;
    }
  }
  f2 gz2[H], gz1[H];
#pragma unroll
  for (int k = 0; k < H; ++k) {
    f2 a = splat(0.f);
#pragma unroll
    for (int o = 0; o < HALF; ++o) a = pfma(w3[o * H + k], go[o], a);
    gz2[k] = a * (splat(1.f) - h2[k] * h2[k]);
  }
#pragma unroll
  for (int k = 0; k < H; ++k) {
    f2 a = splat(0.f);
#pragma unroll
    for (int j = 0; j < H; ++j) a = pfma(w2[j * H + k], gz2[j], a);
    gz1[k] = a * (splat(1.f) - h1[k] * h1[k]);
  }
#pragma unroll
  for (int k = 0; k < HALF; ++k) {
    f2 a = splat(0.f);
#pragma unroll
    for (int j = 0; j < H; ++j) a = pfma(w[j * HALF + k], gz1[j], a);
    gu[k] = a.x + a.y;
  }
#pragma unroll
  for (int j = 0; j < H; ++j) {
    pf[j] = gz1[j];
    pf[H + j] = h1[j];
    pf[2 * H + j] = gz2[j];
    pf[3 * H + j] = h2[j];
    gz_keep[j] = gz1[j];
  }
#pragma unroll
  for (int o = 0; o < HALF; ++o) pf[4 * H + o] = go[o];
#pragma unroll
  for (int k = 0; k < HALF; ++k) uf[k] = u[k];
}

// Contract the wave's 64 rows of factors into the half's parameter-gradient pairs, in the
// blob layout of coupling_pair_tensors (core W1u W2 b2 W3 b3, context W1c b1); lane = pair.
template <int HALF, int H>
__device__ __forceinline__ void half_reduce(const f2 *pf, const float *sf, int O, f2 *out) {
  using L = BwdLds<HALF, H>;
  constexpr int PF = L::PF;
  const int SF = L::sfs(O);
  constexpr int cW2 = H * HALF, cB2 = cW2 + H * H, cW3 = cB2 + H, cB3 = cW3 + HALF * H,
                cCore = cB3 + HALF;
  const int cB1 = cCore + H * O, ns = cB1 + H;
  for (int e = threadIdx.x; e < ns; e += kBwdRows) {
    // A: the g-factor (pf index); B: 1, an f32 input (sf index) or an f2 activation (pf index)
    int ai, bi, mode;  // mode 0: B = 1, 1: B = sf[bi] (both nets), 2: B = pf[bi] (per net)
    if (e < cW2) {
      ai = e / HALF, bi = e % HALF, mode = 1;
    } else if (e < cB2) {
      ai = 2 * H + (e - cW2) / H, bi = H + (e - cW2) % H, mode = 2;
    } else if (e < cW3) {
      ai = 2 * H + (e - cB2), bi = 0, mode = 0;
    } else if (e < cB3) {
      ai = 4 * H + (e - cW3) / H, bi = 3 * H + (e - cW3) % H, mode = 2;
    } else if (e < cCore) {
      ai = 4 * H + (e - cB3), bi = 0, mode = 0;
    } else if (e < cB1) {
      ai = (e - cCore) / O, bi = HALF + (e - cCore) % O, mode = 1;
    } else {
      ai = e - cB1, bi = 0, mode = 0;
    }
    f2 acc = splat(0.f);
    if (mode == 0) {
      for (int r = 0; r < kBwdRows; ++r) acc += pf[r * PF + ai];
    } else if (mode == 1) {
      for (int r = 0; r < kBwdRows; ++r) acc = pfma(pf[r * PF + ai], splat(sf[r * SF + bi]), acc);
    } else {
      for (int r = 0; r < kBwdRows; ++r) acc = pfma(pf[r * PF + ai], pf[r * PF + bi], acc);
    }
    out[e] = acc;
  }
}

template <int HALF, int H, bool INV>
__global__ __launch_bounds__(kBwdRows) void cond_stack_bwd_kernel(
    const float *__restrict__ params, int n_flows, int O, const float *__restrict__ x,
    const float *__restrict__ cond, int64_t rows, float prior_mean, float prior_std,
    const float *__restrict__ g_out, const float *__restrict__ g_ld,
    const float *__restrict__ g_lp, float *__restrict__ g_x, float *__restrict__ g_cond,
    float *__restrict__ partial) {
  using L = BwdLds<HALF, H>;
  constexpr int D = 2 * HALF, PF = L::PF;
  extern __shared__ __align__(16) unsigned char lds[];
  f2 *pf = (f2 *)(lds + L::pf_off());
  f2 *gzall = (f2 *)(lds + L::gz_off());
  float *sf = (float *)(lds + L::sf_off(n_flows));
  float *xin = (float *)(lds + L::xin_off(n_flows, O));
  f2 *cbs = (f2 *)(lds + L::cbs_off(n_flows, O));
  const int SF = L::sfs(O);
  const int lane = threadIdx.x;
  const int64_t row0 = (int64_t)blockIdx.x * kBwdRows;
  const int64_t r = row0 + lane;
  const bool valid = r < rows;
  const int nrows = (int)min<int64_t>(kBwdRows, rows - row0);
  // the block's context rows, coalesced, into sf[:, HALF:] (0 past the end)
  for (int i = lane; i < kBwdRows * O; i += kBwdRows) {
    const int rr = i / O, c = i - rr * O;
    sf[rr * SF + HALF + c] = rr < nrows ? cond[(row0 + rr) * O + c] : 0.f;
  }
  __syncthreads();
  const float *c_row = sf + lane * SF + HALF;
  const int ns = net_size<HALF, H>(O);

  // ---- forward recompute; inputs of every flow (application order) to LDS ----
  float lo[HALF], up[HALF];
#pragma unroll
  for (int k = 0; k < HALF; ++k) {
    lo[k] = valid ? x[r * D + k] : 0.f;
    up[k] = valid ? x[r * D + HALF + k] : 0.f;
  }
  f2 cb[2 * H];
  for (int q = 0; q < n_flows; ++q) {
    const int fi = INV ? n_flows - 1 - q : q;
    cf2 *fw = wptr2(params) + fi * 2 * ns;
#pragma unroll
    for (int k = 0; k < HALF; ++k) {
      xin[(q * D + k) * kBwdRows + lane] = lo[k];
      xin[(q * D + HALF + k) * kBwdRows + lane] = up[k];
    }
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int j = 0; j < H; ++j) {
        cb[n * H + j] = fold_pair<HALF, H>(fw + n * ns, O, j, c_row);
        cbs[(q * 2 * H + n * H + j) * kBwdRows + lane] = cb[n * H + j];
      }
    if (INV)
      coupling_inverse<HALF, H>(fw, O, lo, up, cb);
    else
      coupling_forward<HALF, H>(fw, O, lo, up, cb);
  }

  // ---- incoming gradients ----
  float glo[HALF], gup[HALF];
  const float gl = valid ? g_ld[r] : 0.f;
#pragma unroll
  for (int k = 0; k < HALF; ++k) {
    glo[k] = valid ? g_out[r * D + k] : 0.f;
    gup[k] = valid ? g_out[r * D + HALF + k] : 0.f;
  }
  if (!INV && g_lp && valid) {  // lp = -0.5 sum ((z - m) / s)^2 - ...  (nf/models.py:51)
    const float glp = g_lp[r], is2 = 1.f / (prior_std * prior_std);
#pragma unroll
    for (int k = 0; k < HALF; ++k) {
      glo[k] = fmaf(-glp * is2, lo[k] - prior_mean, glo[k]);
      gup[k] = fmaf(-glp * is2, up[k] - prior_mean, gup[k]);
    }
  }

  // ---- backward over flows (reverse application order), two halves each ----
  const int P = n_flows * 2 * ns;  // pairs in the blob
  f2 *part = (f2 *)partial + (size_t)blockIdx.x * P;
  for (int q = n_flows - 1; q >= 0; --q) {
    const int fi = INV ? n_flows - 1 - q : q;
    cf2 *fw = wptr2(params) + fi * 2 * ns;
    float a_lo[HALF], a_up[HALF];
#pragma unroll
    for (int k = 0; k < HALF; ++k) {
      a_lo[k] = xin[(q * D + k) * kBwdRows + lane];
      a_up[k] = xin[(q * D + HALF + k) * kBwdRows + lane];
    }
#pragma unroll
    for (int j = 0; j < 2 * H; ++j) cb[j] = cbs[(q * 2 * H + j) * kBwdRows + lane];
    // the half applied first (pair 0 forward, pair 1 inverse) and the intermediate it made
    float mid[HALF], gu[HALF];
    {
      float t[HALF], s[HALF];
      if (!INV) {
        ts_pair<HALF, H>(fw, a_lo, cb, t, s);
#pragma unroll
        for (int k = 0; k < HALF; ++k) mid[k] = t[k] + a_up[k] * expf(s[k]);  // up after half A
      } else {
        ts_pair<HALF, H>(fw + ns, a_up, cb + H, t, s);
#pragma unroll
        for (int k = 0; k < HALF; ++k) mid[k] = (a_lo[k] - t[k]) * expf(-s[k]);  // lo after half B
      }
    }
    for (int hh = 0; hh < 2; ++hh) {
      // forward: second-applied half is B (pair 1: u = mid (up'), y = lo), then A (pair 0:
      // u = lo, y = up).  Inverse: A (pair 0: u = mid (lo'), y = up), then B (pair 1: u = up, y = lo)
      const int pair = INV ? hh : 1 - hh;
      const bool second = hh == 0;
      const int hidx = fi * 2 + pair;
      f2 *gz_keep = gzall + ((size_t)hidx * kBwdRows + lane) * H;
      if (!INV) {
        if (second) {
          half_bwd<HALF, H, false>(fw + ns, cb + H, mid, a_lo, glo, gl, gu, pf + lane * PF, sf + lane * SF, gz_keep);
#pragma unroll
          for (int k = 0; k < HALF; ++k) gup[k] += gu[k];
        } else {
          half_bwd<HALF, H, false>(fw, cb, a_lo, a_up, gup, gl, gu, pf + lane * PF, sf + lane * SF, gz_keep);
#pragma unroll
          for (int k = 0; k < HALF; ++k) glo[k] += gu[k];
        }
      } else {
        if (second) {
          half_bwd<HALF, H, true>(fw, cb, mid, a_up, gup, gl, gu, pf + lane * PF, sf + lane * SF, gz_keep);
#pragma unroll
          for (int k = 0; k < HALF; ++k) glo[k] += gu[k];
        } else {
          half_bwd<HALF, H, true>(fw + ns, cb + H, a_up, a_lo, glo, gl, gu, pf + lane * PF, sf + lane * SF, gz_keep);
#pragma unroll
          for (int k = 0; k < HALF; ++k) gup[k] += gu[k];
        }
      }
      __syncthreads();
      half_reduce<HALF, H>(pf, sf, O, part + (size_t)hidx * ns);
      __syncthreads();
    }
  }
  if (valid) {
#pragma unroll
    for (int k = 0; k < HALF; ++k) {
      g_x[r * D + k] = glo[k];
      g_x[r * D + HALF + k] = gup[k];
    }
  }
  // ---- d/d cond: sum over halves of W1c^T g_z1, lane = (row, column) ----
  if (g_cond && O > 0) {
    for (int i = lane; i < nrows * O; i += kBwdRows) {
      const int rr = i / O, c = i - rr * O;
      float acc = 0.f;
      for (int hidx = 0; hidx < n_flows * 2; ++hidx) {
        cf2 *w1c = wptr2(params) + hidx * ns + net_core<HALF, H>();
        const f2 *gz = gzall + ((size_t)hidx * kBwdRows + rr) * H;
#pragma unroll
        for (int j = 0; j < H; ++j) {
          const f2 wv = w1c[j * O + c];
          acc = fmaf(wv.x, gz[j].x, fmaf(wv.y, gz[j].y, acc));
        }
      }
      g_cond[(row0 + rr) * O + c] = acc;
    }
  }
}

// g_params[p] = sum over workgroups b (in order) of partial[b][p]; block = 64 parameters x 4
// workgroup strides, combined in LDS in a fixed order.
__global__ __launch_bounds__(256) void param_reduce_kernel(const float *__restrict__ partial,
                                                           int64_t n_parts, int64_t P,
                                                           float *__restrict__ out) {
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

template <int HALF, int H>
static int launch_bwd(bool inv, hipStream_t st, const float *params, int n_flows, int O,
                      const float *x, const float *cond, int64_t rows, float pm, float ps,
                      const float *go, const float *gl, const float *glp, float *gx,
                      float *gc, float *partial) {
  using L = BwdLds<HALF, H>;
  const size_t lds = L::bytes(n_flows, O);
  NFDPF_REQUIRE(lds <= 160 * 1024, "nfdpf_cond_stack_backward: %zu B of LDS needed (obser_dim %d too large)",
                lds, O);
  const dim3 g((unsigned)((rows + kBwdRows - 1) / kBwdRows));
  if (inv) {
    (void)hipFuncSetAttribute((const void *)cond_stack_bwd_kernel<HALF, H, true>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    cond_stack_bwd_kernel<HALF, H, true><<<g, kBwdRows, lds, st>>>(
        params, n_flows, O, x, cond, rows, pm, ps, go, gl, glp, gx, gc, partial);
  } else {
    (void)hipFuncSetAttribute((const void *)cond_stack_bwd_kernel<HALF, H, false>,
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    cond_stack_bwd_kernel<HALF, H, false><<<g, kBwdRows, lds, st>>>(
        params, n_flows, O, x, cond, rows, pm, ps, go, gl, glp, gx, gc, partial);
  }
  return NFDPF_OK;
}

}  // namespace nfdpf

using namespace nfdpf;

// floats in the packed blob of a RealNVP(_cond) stack (include/nfdpf.h, coupling layout)
static int64_t stack_param_floats(int n_flows, int dim, int obser_dim, int hidden) {
  const int64_t half = dim / 2, h = hidden;
  const int64_t ns = h * half + h * h + h + half * h + half + h * obser_dim + h;  // pairs per half
  return (int64_t)n_flows * 2 * ns * 2;
}

extern "C" int64_t nfdpf_cond_stack_backward_workspace(int n_flows, int dim, int obser_dim, int hidden,
                                                       int64_t rows) {
  if (n_flows < 0 || dim < 2 || dim % 2 || obser_dim < 0 || hidden < 1 || rows < 0) return -1;
  const int64_t blocks = (rows + kBwdRows - 1) / kBwdRows;
  return blocks * stack_param_floats(n_flows, dim, obser_dim, hidden) * (int64_t)sizeof(float);
}

extern "C" int nfdpf_cond_stack_backward(const float *params, int n_flows, int dim, int obser_dim,
                                         int hidden, const float *x, const float *cond, int64_t rows,
                                         int inverse, float prior_mean, float prior_std,
                                         const float *g_out, const float *g_logdet,
                                         const float *g_prior_logprob, float *g_x, float *g_cond,
                                         float *g_params, void *workspace, void *stream) {
  NFDPF_REQUIRE(g_params, "nfdpf_cond_stack_backward: null pointer");
  NFDPF_REQUIRE(n_flows >= 1 && n_flows <= kBwdMaxFlows && rows >= 0 && obser_dim >= 0,
                "nfdpf_cond_stack_backward: bad sizes (n_flows in 1..%d)", kBwdMaxFlows);
  NFDPF_REQUIRE(dim >= 2 && dim % 2 == 0 && hidden >= 1, "nfdpf_cond_stack_backward: bad sizes");
  NFDPF_REQUIRE(prior_std > 0.f, "nfdpf_cond_stack_backward: prior_std must be > 0");
  const int64_t P = stack_param_floats(n_flows, dim, obser_dim, hidden);
  hipStream_t st = as_stream(stream);
  if (rows == 0) {
    (void)hipMemsetAsync(g_params, 0, sizeof(float) * (size_t)P, st);
    return launch_status("nfdpf_cond_stack_backward");
  }
  NFDPF_REQUIRE(params && x && g_out && g_logdet && g_x, "nfdpf_cond_stack_backward: null pointer");
  NFDPF_REQUIRE(obser_dim == 0 || cond, "nfdpf_cond_stack_backward: cond missing");
  NFDPF_REQUIRE(workspace, "nfdpf_cond_stack_backward: workspace missing");
  const int O = obser_dim;
  const bool inv = inverse != 0;
  float *part = (float *)workspace;
  int rc = NFDPF_EINVAL;
  bool done = false;
#define NFDPF_BWD(HALF, H)                                                                      \
  if (!done && dim == 2 * HALF && hidden == H) {                                                \
    rc = launch_bwd<HALF, H>(inv, st, params, n_flows, O, x, O ? cond : nullptr, rows,          \
                             prior_mean, prior_std, g_out, g_logdet, inv ? nullptr : g_prior_logprob, \
                             g_x, O ? g_cond : nullptr, part);                                  \
    done = true;                                                                                \
  }
  NFDPF_BWD(1, 8)
  NFDPF_BWD(2, 8)
  NFDPF_BWD(16, 8)
#undef NFDPF_BWD
  if (!done) {
    set_error("nfdpf_cond_stack_backward: unsupported (dim=%d, hidden=%d); built for dim in "
              "{2,4,32}, hidden 8",
              dim, hidden);
    return NFDPF_EINVAL;
  }
  if (rc != NFDPF_OK) return rc;
  const int64_t nb = (rows + kBwdRows - 1) / kBwdRows;
  param_reduce_kernel<<<dim3((unsigned)((P + 63) / 64)), 256, 0, st>>>(part, nb, P, g_params);
  return launch_status("nfdpf_cond_stack_backward");
}
