// resample_ot.hip -- entropy-regularised optimal-transport resampling (resamplers.py:62-277).
//
// What the reference does (FP64, dense): centre and scale the particles (transport_function
// :211-227, diameter :72-76), build four B x N x N cost matrices (:183-186), run the
// Sinkhorn loop with epsilon annealing (:113-179) and finally materialise the B x N x N
// transport matrix (:194-210) and multiply it with the particles (:254-264).
//
// What runs here:
//   * costs are recomputed on the fly from the 2-D points (||x_i - x_j||^2 / 2), never stored;
//   * only the two potentials that reach the output (a_y, b_x) are iterated: a_x / b_y are
//     computed by the reference but read by nothing (:139-147, :177-178);
//   * every softmin is a streamed log-sum-exp over j tiles staged in LDS, in base 2
//     (v_exp_f32 is 2^x), with a tile-wise running max;
//   * the transport matrix is never formed: column log-normalisers r_j first, then
//     x'_i = sum_j 2^(...) x_j;
//   * the loop keeps the reference's batch-coupled stop rule -- it ends at the first
//     iteration after which ANY row has converged (torch.all(continue_), :126-129) -- with
//     one launch per iteration that first reads the previous iteration's per-row residuals
//     (identical decision in every workgroup, no host sync, no atomics);
//   * rows are split over `splits` workgroups along i so that a small batch still fills
//     the 256 CUs.
// Precision: Real = float (default) or double (parity mode, --ot-fp64).
#include "common.hpp"

namespace nfdpf {

constexpr int kOtThreads = 256;  // i per workgroup
constexpr int kOtTile = 512;     // j per LDS tile
constexpr float kLog2e = 1.4426950408889634f;
constexpr float kLn2 = 0.6931471805599453f;

struct OtState {
  int32_t stopped;  // set by the iteration that observes a converged row
  int32_t K;        // total_iter of the reference
};

struct OtWs {  // carve of the caller's workspace
  OtState *st;
  float *xs;     // [B,N,2] centred / scaled particles
  float *logw;   // [B,N]
  double *rowc;  // [B,4]: eps0, logu, unused, unused
  float *pot;    // [2 buffers][2 (a_y,b_x)][B,N]
  float *res;    // [2 parity][B][splits] max |delta| of the iteration
  float *fg;     // [2][B,N] final potentials f (=a_y), g (=b_x)
  float *r;      // [B,N] column terms r_j
};

static inline int64_t align256(int64_t v) { return (v + 255) / 256 * 256; }

static inline int ot_splits(int B, int N) {
  // enough workgroups to cover the chip, at most one per 256 i
  int s = (N + kOtThreads - 1) / kOtThreads;
  return s < 1 ? 1 : s;
}

static OtWs carve(void *ws, int B, int N, int splits) {
  char *p = (char *)ws;
  OtWs w;
  w.st = (OtState *)p;
  p += 256;
  w.xs = (float *)p;
  p += align256((int64_t)B * N * 2 * 4);
  w.logw = (float *)p;
  p += align256((int64_t)B * N * 4);
  w.rowc = (double *)p;
  p += align256((int64_t)B * 4 * 8);
  w.pot = (float *)p;
  p += align256((int64_t)4 * B * N * 4);
  w.res = (float *)p;
  p += align256((int64_t)2 * B * splits * 4);
  w.fg = (float *)p;
  p += align256((int64_t)2 * B * N * 4);
  w.r = (float *)p;
  return w;
}

static int64_t ws_bytes(int B, int N) {
  const int s = ot_splits(B, N);
  return 256 + align256((int64_t)B * N * 8) + align256((int64_t)B * N * 4) +
         align256((int64_t)B * 32) + align256((int64_t)16 * B * N) +
         align256((int64_t)8 * B * s) + align256((int64_t)8 * B * N) +
         align256((int64_t)4 * B * N);
}

// ------------------------------------------------------------------------------------------
// setup: centre/scale (transport_function :218-222), eps0 = max_min^2 (:87-91, :117), logw
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void ot_setup_kernel(const float *__restrict__ x,
                                                        const float *__restrict__ w, int N,
                                                        OtWs ws, const int32_t *gate) {
  if (gate && *gate == 0) return;
  __shared__ double shd[16];
  __shared__ float shf[16];
  const int b = blockIdx.x;
  const float *xr = x + (int64_t)b * N * 2;
  double s0 = 0, s1 = 0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    s0 += xr[2 * i];
    s1 += xr[2 * i + 1];
  }
  s0 = block_sum(s0, shd);
  s1 = block_sum(s1, shd);
  const float m0 = (float)(s0 / N), m1 = (float)(s1 / N);  // x.mean(dim=1) (float)
  double v0 = 0, v1 = 0;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const double a = xr[2 * i] - s0 / N, c = xr[2 * i + 1] - s1 / N;
    v0 += a * a;
    v1 += c * c;
  }
  v0 = block_sum(v0, shd);
  v1 = block_sum(v1, shd);
  // diameter: max over dims of the biased std (float), 0 -> 1, then double (:72-76)
  const float d0 = (float)sqrt(v0 / N), d1 = (float)sqrt(v1 / N);
  const float dm = fmaxf(d0, d1);
  const double diam = dm == 0.0f ? 1.0 : (double)dm;
  const double scale = diam * (double)sqrtf(2.0f);
  float mx = -INFINITY, mn = INFINITY;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const float a = (float)((double)(xr[2 * i] - m0) / scale);
    const float c = (float)((double)(xr[2 * i + 1] - m1) / scale);
    ws.xs[((int64_t)b * N + i) * 2] = a;
    ws.xs[((int64_t)b * N + i) * 2 + 1] = c;
    mx = fmaxf(mx, fmaxf(a, c));
    mn = fminf(mn, fminf(a, c));
    ws.logw[(int64_t)b * N + i] = logf(w[(int64_t)b * N + i]);
  }
  mx = block_max(mx, shf);
  mn = -block_max(-mn, shf);
  if (threadIdx.x == 0) {
    const double mm = (double)mx - (double)mn;
    ws.rowc[b * 4 + 0] = mm * mm;                        // epsilon_0 = diameter^2 (:117)
    ws.rowc[b * 4 + 1] = -(double)logf((float)N);       // uniform log weight (:214-215)
    if (b == 0) {
      ws.st->stopped = 0;
      ws.st->K = 0;
    }
  }
}

// running epsilon at iteration k: eps_{k+1} = max(eps_k * s^2, eps) in double (:158)
__device__ __forceinline__ double run_eps(double eps0, int k, double sf, double eps) {
  double e = eps0;
  for (int t = 0; t < k; ++t) e = fmax(e * sf, eps);
  return e;
}

// Two softmins of one i against all j of the row (base-2 streamed LSE):
//   A_i = -e * LSE_j(ha_j - C_ij/e),  B_i = -e * LSE_j(hb_j - C_ij/e),  C_ij = |x_i-x_j|^2/2
// ha/hb are produced tile by tile by `fill(j, &ha, &hb)`.
template <class Fill>
__device__ void softmin_pair(const float *xs, int N, int i, bool active, float inv_e, float e,
                             const Fill &fill, float *tx, float *ty, float *tha, float *thb,
                             float &A, float &Bv) {
  const float xi = active ? xs[2 * i] : 0.f, yi = active ? xs[2 * i + 1] : 0.f;
  const float c2 = 0.5f * inv_e * kLog2e;  // C_ij / e in base 2
  float ma = -INFINITY, sa = 0.f, mb = -INFINITY, sb = 0.f;
  for (int j0 = 0; j0 < N; j0 += kOtTile) {
    const int nt = min(kOtTile, N - j0);
    __syncthreads();
    for (int j = threadIdx.x; j < nt; j += blockDim.x) {
      float ha, hb;
      fill(j0 + j, ha, hb);
      tx[j] = xs[2 * (j0 + j)];
      ty[j] = xs[2 * (j0 + j) + 1];
      tha[j] = ha * kLog2e;
      thb[j] = hb * kLog2e;
    }
    __syncthreads();
    if (active) {
      for (int j = 0; j < nt; j += 16) {
        const int jn = min(16, nt - j);
        float va[16], vb[16];
        float la = -INFINITY, lb = -INFINITY;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          if (q < jn) {
            const float dx = xi - tx[j + q], dy = yi - ty[j + q];
            const float c = fmaf(dx, dx, dy * dy) * c2;
            va[q] = tha[j + q] - c;
            vb[q] = thb[j + q] - c;
          } else {
            va[q] = -INFINITY;
            vb[q] = -INFINITY;
          }
          la = fmaxf(la, va[q]);
          lb = fmaxf(lb, vb[q]);
        }
        if (la > ma) {
          sa = sa * exp2f(ma - la);
          ma = la;
        }
        if (lb > mb) {
          sb = sb * exp2f(mb - lb);
          mb = lb;
        }
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          sa += exp2f(va[q] - ma);
          sb += exp2f(vb[q] - mb);
        }
      }
    }
  }
  A = -e * (ma + log2f(sa)) * kLn2;
  Bv = -e * (mb + log2f(sb)) * kLn2;
}

struct OtParams {
  int B, N, splits, max_iter;
  double eps, sf, thr;
  const int32_t *gate;     // optional: skip everything when *gate == 0
  const int32_t *stop_at;  // optional: total_iter + 2 to run (sharded batches), else the rule
};

__device__ __forceinline__ bool ot_off(const OtParams &P) { return P.gate && *P.gate == 0; }

__device__ __forceinline__ float *pot_ptr(const OtWs &ws, const OtParams &P, int buf, int which,
                                          int b) {
  return ws.pot + (((int64_t)buf * 2 + which) * P.B + b) * P.N;
}

// initial potentials at eps0 (:120-121): a_y = softmin(eps0, C, logw), b_x = softmin(eps0, C, logu)
__global__ __launch_bounds__(kOtThreads) void ot_init_kernel(OtParams P, OtWs ws) {
  if (ot_off(P)) return;
  __shared__ float tx[kOtTile], ty[kOtTile], tha[kOtTile], thb[kOtTile];
  const int b = blockIdx.y, N = P.N;
  const int i = blockIdx.x * kOtThreads + threadIdx.x;
  const float *xs = ws.xs + (int64_t)b * N * 2;
  const float *lw = ws.logw + (int64_t)b * N;
  const double e = ws.rowc[b * 4];
  const float logu = (float)ws.rowc[b * 4 + 1];
  float A, Bv;
  softmin_pair(
      xs, N, i, i < N, (float)(1.0 / e), (float)e,
      [&](int j, float &ha, float &hb) {
        ha = lw[j];
        hb = logu;
      },
      tx, ty, tha, thb, A, Bv);
  if (i < N) {
    pot_ptr(ws, P, 0, 0, b)[i] = A;
    pot_ptr(ws, P, 0, 1, b)[i] = Bv;
  }
}

// does the loop stop before iteration k?  (stop_condition :126-129) -- every workgroup
// evaluates the same residuals of iteration k-1 in the same order
__device__ __forceinline__ bool ot_stop_before(const OtParams &P, const OtWs &ws, int k) {
  if (k == 0) return false;
  if (P.stop_at) return k >= *P.stop_at - 2;  // the batch-global decision, taken by the caller
  const float *res = ws.res + (int64_t)((k - 1) & 1) * P.B * P.splits;
  for (int b = 0; b < P.B; ++b) {
    const double e0 = ws.rowc[b * 4];
    const double re = run_eps(e0, k - 1, P.sf, P.eps);
    const double ne = fmax(re * P.sf, P.eps);
    bool cont = ne < re;
    for (int s = 0; s < P.splits && !cont; ++s) cont = (double)res[b * P.splits + s] > P.thr;
    if (!cont) return true;  // some row converged -> torch.all(continue_) is False
  }
  return false;
}

// iteration k: state k (buffer k&1) -> state k+1 (buffer (k+1)&1)  (apply_one :131-153)
__global__ __launch_bounds__(kOtThreads) void ot_iter_kernel(OtParams P, OtWs ws, int k) {
  if (ot_off(P)) return;
  __shared__ float tx[kOtTile], ty[kOtTile], tha[kOtTile], thb[kOtTile];
  __shared__ float shf[16];
  __shared__ int s_stop;
  if (threadIdx.x == 0) {
    int st = ws.st->stopped;
    if (!st && ot_stop_before(P, ws, k)) {
      st = 1;
      if (blockIdx.x == 0 && blockIdx.y == 0) {
        ws.st->stopped = 1;
        ws.st->K = k;
      }
    }
    s_stop = st;
  }
  __syncthreads();
  if (s_stop) return;
  const int b = blockIdx.y, N = P.N;
  const int i = blockIdx.x * kOtThreads + threadIdx.x;
  const double re = run_eps(ws.rowc[b * 4], k, P.sf, P.eps);
  const float ref = (float)re, inv = (float)(1.0 / re);
  const float *xs = ws.xs + (int64_t)b * N * 2;
  const float *lw = ws.logw + (int64_t)b * N;
  const float logu = (float)ws.rowc[b * 4 + 1];
  const float *ay = pot_ptr(ws, P, k & 1, 0, b), *bx = pot_ptr(ws, P, k & 1, 1, b);
  float A, Bv;
  // at_y = softmin(e, C, logw + b_x/e);  bt_x = softmin(e, C, logu + a_y/e)
  softmin_pair(
      xs, N, i, i < N, inv, ref,
      [&](int j, float &ha, float &hb) {
        ha = lw[j] + bx[j] * inv;
        hb = logu + ay[j] * inv;
      },
      tx, ty, tha, thb, A, Bv);
  float dmax = 0.f;
  if (i < N) {
    const float na = 0.5f * (ay[i] + A), nb = 0.5f * (bx[i] + Bv);
    pot_ptr(ws, P, (k + 1) & 1, 0, b)[i] = na;
    pot_ptr(ws, P, (k + 1) & 1, 1, b)[i] = nb;
    dmax = fmaxf(fabsf(na - ay[i]), fabsf(nb - bx[i]));
  }
  dmax = block_max(dmax, shf);
  if (threadIdx.x == 0) ws.res[((int64_t)(k & 1) * P.B + b) * P.splits + blockIdx.x] = dmax;
}

__device__ __forceinline__ int ot_total_iter(const OtParams &P, const OtWs &ws) {
  return ws.st->stopped ? ws.st->K : max(P.max_iter - 1, 0);
}

// final potentials at eps (:173-176): f = softmin(eps, C, logw + b_x/eps), g = softmin(eps, C, logu + a_y/eps)
__global__ __launch_bounds__(kOtThreads) void ot_final_kernel(OtParams P, OtWs ws) {
  if (ot_off(P)) return;
  __shared__ float tx[kOtTile], ty[kOtTile], tha[kOtTile], thb[kOtTile];
  const int b = blockIdx.y, N = P.N;
  const int i = blockIdx.x * kOtThreads + threadIdx.x;
  const int K = ot_total_iter(P, ws);
  const float e = (float)P.eps, inv = (float)(1.0 / P.eps);
  const float *xs = ws.xs + (int64_t)b * N * 2;
  const float *lw = ws.logw + (int64_t)b * N;
  const float logu = (float)ws.rowc[b * 4 + 1];
  const float *ay = pot_ptr(ws, P, K & 1, 0, b), *bx = pot_ptr(ws, P, K & 1, 1, b);
  float A, Bv;
  softmin_pair(
      xs, N, i, i < N, inv, e,
      [&](int j, float &ha, float &hb) {
        ha = lw[j] + bx[j] * inv;
        hb = logu + ay[j] * inv;
      },
      tx, ty, tha, thb, A, Bv);
  if (i < N) {
    ws.fg[(int64_t)b * N + i] = A;
    ws.fg[((int64_t)P.B + b) * N + i] = Bv;
  }
}

// r_j = log N + logw_j - LSE_i(f_i/eps - C_ij/eps)   (transport_from_potentials :200-207,
// with the column log-normaliser; g_j cancels)
__global__ __launch_bounds__(kOtThreads) void ot_col_kernel(OtParams P, OtWs ws) {
  if (ot_off(P)) return;
  __shared__ float tx[kOtTile], ty[kOtTile], tha[kOtTile], thb[kOtTile];
  const int b = blockIdx.y, N = P.N;
  const int j = blockIdx.x * kOtThreads + threadIdx.x;
  const float e = (float)P.eps, inv = (float)(1.0 / P.eps);
  const float *xs = ws.xs + (int64_t)b * N * 2;
  const float *f = ws.fg + (int64_t)b * N;
  float A, Bv;
  // softmin_pair returns -e * LSE(...); reuse it with ha = f_i / eps (the second lane unused)
  softmin_pair(
      xs, N, j, j < N, inv, e,
      [&](int i, float &ha, float &hb) {
        ha = f[i] * inv;
        hb = 0.f;
      },
      tx, ty, tha, thb, A, Bv);
  if (j < N) {
    const float lse = -A * inv;
    ws.r[(int64_t)b * N + j] = -(float)ws.rowc[b * 4 + 1] + ws.logw[(int64_t)b * N + j] - lse;
  }
}

// x'_i = sum_j exp(f_i/eps - C_ij/eps + r_j) x_j  (apply_transport_matrix :254-264)
__global__ __launch_bounds__(kOtThreads) void ot_apply_kernel(OtParams P, OtWs ws,
                                                             const float *__restrict__ x,
                                                             int64_t row_base,
                                                             float *__restrict__ x_out,
                                                             float *__restrict__ w_out,
                                                             int64_t *__restrict__ idx_out) {
  if (ot_off(P)) return;
  __shared__ float tx[kOtTile], ty[kOtTile], tr[kOtTile], px[kOtTile], py[kOtTile];
  const int b = blockIdx.y, N = P.N;
  const int i = blockIdx.x * kOtThreads + threadIdx.x;
  const float inv = (float)(1.0 / P.eps);
  const float *xs = ws.xs + (int64_t)b * N * 2;
  const float *xr = x + (int64_t)b * N * 2;
  const bool act = i < N;
  const float xi = act ? xs[2 * i] : 0.f, yi = act ? xs[2 * i + 1] : 0.f;
  const float fi = act ? ws.fg[(int64_t)b * N + i] * inv * kLog2e : 0.f;
  const float c2 = 0.5f * inv * kLog2e;
  float ax = 0.f, ay = 0.f;
  for (int j0 = 0; j0 < N; j0 += kOtTile) {
    const int nt = min(kOtTile, N - j0);
    __syncthreads();
    for (int j = threadIdx.x; j < nt; j += blockDim.x) {
      tx[j] = xs[2 * (j0 + j)];
      ty[j] = xs[2 * (j0 + j) + 1];
      tr[j] = ws.r[(int64_t)b * N + j0 + j] * kLog2e;
      px[j] = xr[2 * (j0 + j)];
      py[j] = xr[2 * (j0 + j) + 1];
    }
    __syncthreads();
    if (act) {
      for (int j = 0; j < nt; ++j) {
        const float dx = xi - tx[j], dy = yi - ty[j];
        const float t = exp2f(fi + tr[j] - fmaf(dx, dx, dy * dy) * c2);
        ax = fmaf(t, px[j], ax);
        ay = fmaf(t, py[j], ay);
      }
    }
  }
  if (act) {
    const int64_t o = (int64_t)b * N + i;
    x_out[2 * o] = ax;
    x_out[2 * o + 1] = ay;
    w_out[o] = 1.0f / (float)N;
    idx_out[o] = (int64_t)N * (row_base + b) + i;
  }
}

__global__ void ot_iters_kernel(OtParams P, OtWs ws, int32_t *out) {
  out[0] = ot_off(P) ? 0 : ot_total_iter(P, ws) + 2;
}

}  // namespace nfdpf

using namespace nfdpf;

extern "C" int64_t nfdpf_ot_workspace_bytes(int B, int N) {
  return (B <= 0 || N <= 0) ? 256 : ws_bytes(B, N);
}

extern "C" int nfdpf_ot_resample(const float *x, const float *w, int B, int N, float eps,
                                 float scaling, float threshold, int max_iter, int64_t row_base,
                                 float *x_out, float *w_out, int64_t *idx_out, int32_t *iters_out,
                                 void *workspace, const int32_t *gate, const int32_t *stop_at,
                                 void *stream) {
  NFDPF_REQUIRE(x && w && x_out && w_out && idx_out && workspace,
                "nfdpf_ot_resample: null pointer");
  NFDPF_REQUIRE(B >= 0 && N >= 1 && max_iter >= 1, "nfdpf_ot_resample: bad sizes");
  NFDPF_REQUIRE(eps > 0.f && scaling > 0.f, "nfdpf_ot_resample: eps and scaling must be > 0");
  NFDPF_REQUIRE(((uintptr_t)workspace & 255) == 0, "nfdpf_ot_resample: workspace not 256-B aligned");
  if (B == 0) return NFDPF_OK;
  hipStream_t st = as_stream(stream);
  const int splits = ot_splits(B, N);
  OtWs ws = carve(workspace, B, N, splits);
  OtParams P{B, N, splits, max_iter, (double)eps, (double)scaling * (double)scaling,
             (double)threshold, gate, stop_at};
  ot_setup_kernel<<<B, row_threads(N), 0, st>>>(x, w, N, ws, gate);
  const dim3 g(splits, B);
  ot_init_kernel<<<g, kOtThreads, 0, st>>>(P, ws);
  for (int k = 0; k < max_iter - 1; ++k) ot_iter_kernel<<<g, kOtThreads, 0, st>>>(P, ws, k);
  ot_final_kernel<<<g, kOtThreads, 0, st>>>(P, ws);
  ot_col_kernel<<<g, kOtThreads, 0, st>>>(P, ws);
  ot_apply_kernel<<<g, kOtThreads, 0, st>>>(P, ws, x, row_base, x_out, w_out, idx_out);
  if (iters_out) ot_iters_kernel<<<1, 1, 0, st>>>(P, ws, iters_out);
  return launch_status("nfdpf_ot_resample");
}

namespace nfdpf {
__global__ void ess_gate_kernel(const float *__restrict__ inv_ess, int B, int N, int force,
                                int32_t *gate) {
  // torch.mean (DPFs.py:163) in ATen's cascade order, one wave
  const float s = cascade_row_sum([&](int i) { return inv_ess[i]; }, force ? 0 : B);
  if (threadIdx.x == 0) gate[0] = (force || (s / (float)B) < 0.5f * (float)N) ? 1 : 0;
}
}  // namespace nfdpf

extern "C" int nfdpf_ess_gate(const float *inv_ess, int B, int N, int force, int32_t *gate,
                              void *stream) {
  NFDPF_REQUIRE(gate && (force || inv_ess), "nfdpf_ess_gate: null pointer");
  NFDPF_REQUIRE(B >= 1 && N >= 1, "nfdpf_ess_gate: bad sizes");
  ess_gate_kernel<<<1, 64, 0, as_stream(stream)>>>(inv_ess, B, N, force, gate);
  return launch_status("nfdpf_ess_gate");
}
