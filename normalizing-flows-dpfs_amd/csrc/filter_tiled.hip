// filter_tiled.hip -- one filtering step (DPFs.py:160-192) as a short pipeline of launches
// over (particle tile, batch row) workgroups, so a batch of 64 rows fills all 256 CUs.
//
// The stages are coupled only through per-row reductions (mean/std before each flow, the
// weight normalisation, the ESS gate), so each stage ends at a launch boundary and leaves
// per-(row, tile) partial sums in the workspace; the next stage's workgroups combine the
// partials of their row in a fixed order (deterministic, no atomics, no inter-workgroup
// hand-off inside a launch):
//
//   K0 soft   (row)        : ESS gate; soft resampling of fired rows (resamplers.py:20-60)
//   K1 motion (tile, row)  : motion (model/models.py:191-204)         -> sum x, x^2 partials
//   K2 dyn    (tile, row)  : nf_dyn inverse (model/models.py:305-332)  -> sum x, x^2 partials
//   K3 prop   (tile, row)  : NF proposal, nf_dyn forward, densities, measurement
//                            (model/models.py:334-379)                 -> max / sum-exp partials
//   K4 norm   (tile, row)  : log-weights, normalize_log_probs + 1e-12 (DPFs.py:187-192)
//                            -> sum p^2 (next gate), sum p x, sum logw partials
//
// ess_all / ess_out of the descriptor hold per-(row, tile) sums of p^2 as doubles
// ([B_global][tiles] / [B][tiles]); everything else has the fused kernel's meaning.
#include "soft.hpp"
#include "stages.hpp"

namespace nfdpf {

constexpr int kTile = 256;  // particles per workgroup, one per lane

#ifdef NFDPF_EXP_TRACE
// experiment-only: per-workgroup phase timestamps (s_memrealtime, 100 MHz) of one launch
__device__ unsigned long long g_trace[4][2048][8];
#define TRACE(K, P)                                                                        \
  if (threadIdx.x == 0 && blockIdx.y * gridDim.x + blockIdx.x < 2048)                     \
    g_trace[K][blockIdx.y * gridDim.x + blockIdx.x][P] = __builtin_amdgcn_s_memrealtime();
#else
#define TRACE(K, P)
#endif

struct TiledWs {
  double *st_phys;  // [B][tiles][4] sum x0, x1, x0^2, x1^2 of x_phys
  double *st_dyn;   // [B][tiles][4] same for x_dyn
  float *lmax;      // [B][tiles] max raw likelihood
  float *umax;      // [B][tiles] max of the unshifted log-weight u
  double *usum;     // [B][tiles] sum exp(u - umax)
  float *S2;        // [B] soft-resampling renormaliser
  int *fire;        // [B] gate decision taken by K0 (soft resampler)
  float *cb_dyn;    // [B][kCb] folded nf_dyn biases of the row (K2, tile 0)
  float *cb_cond;   // [B][kCb] proposal fold over the encoding columns (K1, tile 0)
  double *fin;      // [B][T][tiles][4] sum p^2, sum p x0, sum p x1, sum logw
};

constexpr int kCb = kMaxFlows * 4 * kH;  // floats of one row's folded-bias table

static inline int64_t al256(int64_t v) { return (v + 255) / 256 * 256; }
__host__ __device__ static inline int n_tiles(int N) { return (N + kTile - 1) / kTile; }

static int64_t tiled_bytes(int B, int N, int T) {
  const int64_t bt = (int64_t)B * n_tiles(N);
  return al256(bt * 32) * 2 + al256(bt * 4) * 2 + al256(bt * 8) + al256((int64_t)B * 4) * 2 +
         al256((int64_t)B * kCb * 4) * 2 + al256(bt * T * 32);
}

static TiledWs tiled_carve(void *ws, int B, int N, int T) {
  char *p = (char *)ws;
  const int64_t bt = (int64_t)B * n_tiles(N);
  TiledWs w;
  w.st_phys = (double *)p;
  p += al256(bt * 32);
  w.st_dyn = (double *)p;
  p += al256(bt * 32);
  w.lmax = (float *)p;
  p += al256(bt * 4);
  w.umax = (float *)p;
  p += al256(bt * 4);
  w.usum = (double *)p;
  p += al256(bt * 8);
  w.S2 = (float *)p;
  p += al256((int64_t)B * 4);
  w.fire = (int *)p;
  p += al256((int64_t)B * 4);
  w.cb_dyn = (float *)p;
  p += al256((int64_t)B * kCb * 4);
  w.cb_cond = (float *)p;
  p += al256((int64_t)B * kCb * 4);
  w.fin = (double *)p;
  return w;
}

// ESS gate from per-(row, tile) sums of p^2 (DPFs.py:163-165): torch.mean over the batch of
// 1 / sum p^2, in ATen's cascade order.  Every wave evaluates it (lanes in parallel over
// rows), so all workgroups take the same decision without a hand-off.
__device__ __forceinline__ bool tiled_gate(const nfdpf_filter_desc &d, int tiles) {
  if (d.gate) return d.gate[0] != 0;
  if (d.force_resample) return true;
  const double *parts = reinterpret_cast<const double *>(d.ess_all);
  const float s = cascade_row_sum(
      [&](int r) {
        double s2 = 0.0;
        for (int k = 0; k < tiles; ++k) s2 += parts[(int64_t)r * tiles + k];
        return 1.0f / (float)s2;
      },
      d.B_global);
  return (s / (float)d.B_global) < 0.5f * (float)d.N;
}

// The same gate, block-parallel (all threads call): thread r stages row r's 1 / sum p^2 in
// `buf` (one round trip for the whole batch), wave 0 folds them in cascade order.
__device__ bool tiled_gate_block(const nfdpf_filter_desc &d, int tiles, float *buf, int *flag) {
  if (d.gate) return d.gate[0] != 0;
  if (d.force_resample) return true;
  const double *parts = reinterpret_cast<const double *>(d.ess_all);
  for (int r = threadIdx.x; r < d.B_global; r += blockDim.x) {
    double s2 = 0.0;
    for (int k = 0; k < tiles; ++k) s2 += parts[(int64_t)r * tiles + k];
    buf[r] = 1.0f / (float)s2;
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const float s = cascade_row_sum([&](int r) { return buf[r]; }, d.B_global);
    if (threadIdx.x == 0) *flag = (s / (float)d.B_global) < 0.5f * (float)d.N;
  }
  __syncthreads();
  return *flag != 0;
}

// combine the 4-sum partials of row b -> context
__device__ __forceinline__ Ctx4 tiled_ctx(const double *st, int b, int tiles, int N) {
  double a0 = 0, a1 = 0, b0 = 0, b1 = 0;
  const double *p = st + (int64_t)b * tiles * 4;
#pragma unroll 4
  for (int k = 0; k < tiles; ++k) {
    a0 += p[4 * k];
    a1 += p[4 * k + 1];
    b0 += p[4 * k + 2];
    b1 += p[4 * k + 3];
  }
  return ctx_from_sums(a0, a1, b0, b1, N);
}

__device__ __forceinline__ void store_sums4(double *dst, double a, double b, double c, double e,
                                            double *sh) {
  block_sum4_store(a, b, c, e, sh, dst);
}

// ---- K1: ESS gate + resampling + motion, per (tile, row).  The gate (DPFs.py:163-165) is
// evaluated block-parallel in every workgroup (same inputs, same order, same decision).  Soft
// resampling (resamplers.py:20-60) of the row: every tile of the row builds the row's CDF in
// LDS and searches all N markers (the renormaliser is a cascade sum over the whole row's
// gathered weights), keeping its own particles' sources in registers -- so resampling and
// motion share one launch and the resampled state never round-trips through HBM.
// Dynamic LDS: C[max(N, B_global)] then w'[N].
__global__ __launch_bounds__(kTile) void tiled_front_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  extern __shared__ float dyn_lds[];
  __shared__ double shd[16];
  __shared__ float shf[16];
  __shared__ int fire_sh;
  __shared__ float xr_sh[kTile][2];
  __shared__ int src_sh[kTile];
  TRACE(0, 0)
  const int tiles = n_tiles(d.N), N = d.N;
  const int b = blockIdx.y, tile = blockIdx.x;
  const int i = tile * kTile + threadIdx.x;
  const int64_t grow = d.row_base + b;
  float *Cbuf = dyn_lds;
  const bool fire = tiled_gate_block(d, tiles, Cbuf, &fire_sh);
  const int mode = !fire ? kSrcPrev : (d.resampler == NFDPF_RESAMPLE_SOFT ? kSrcSoft : kSrcOt);
  const RowSlot S = row_slot(d, b);
  const float *xprev = d.x_prev + b * d.x_prev_rs;
  const float *pprev = d.p_prev + b * d.p_prev_rs;
  float x0 = 0.f, x1 = 0.f, lr = 0.f;
  if (mode == kSrcSoft) {
    float *wbuf = dyn_lds + max(N, d.B_global);
    SoftRow row{pprev, N, d.alpha, 1.0f / (float)N, (float)(1.0 - (double)d.alpha), 1.0f};
    float off;
    if (d.rng_mode == NFDPF_RNG_HOST && d.host_offsets)
      off = d.host_offsets[b];
    else
      off = u01(rng_draw(d.seed, kTagOffset, (uint32_t)d.t, grow, 0u).x) * (1.0f / (float)N);
    const int i0 = tile * kTile;
    soft_row_search(row, d.lin, off, Cbuf, shd, shf, [&](int j, int src) {
      // src == N: the reference's out-of-range edge (next row's first particle, weight 0)
      float w = 0.f;
      if (src < N) w = row.w(src);
      wbuf[j] = w;
      if (j >= i0 && j < i0 + kTile) {
        const float *xs = src < N ? xprev + 2 * src : (b + 1 < d.B ? xprev + d.x_prev_rs : xprev + 2 * (N - 1));
        xr_sh[j - i0][0] = xs[0];
        xr_sh[j - i0][1] = xs[1];
        src_sh[j - i0] = src;
      }
    });
    __syncthreads();
    if (threadIdx.x < 64) {
      const float s2 = cascade_row_sum([&](int j) { return wbuf[j]; }, N);
      if (threadIdx.x == 0) shf[8] = s2;
    }
    __syncthreads();
    if (i < N) {
      x0 = xr_sh[threadIdx.x][0];
      x1 = xr_sh[threadIdx.x][1];
      lr = logf(wbuf[i] / shf[8]);
      S.hidx[i] = (int64_t)N * grow + src_sh[threadIdx.x];
    }
  } else if (i < N) {
    if (mode == kSrcOt) {
      x0 = d.ot_x[((int64_t)b * N + i) * 2];
      x1 = d.ot_x[((int64_t)b * N + i) * 2 + 1];
      lr = logf(1.0f / (float)N);
    } else {
      x0 = xprev[2 * i];
      x1 = xprev[2 * i + 1];
      lr = logf(pprev[i]);
    }
    S.hidx[i] = (int64_t)N * grow + i;
  }
  double s0 = 0, s1 = 0, q0 = 0, q1 = 0;
  if (i < N) {
    float p0, p1;
    motion_apply(d, S, b, grow, i, x0, x1, lr, d.vel[2 * b], d.vel[2 * b + 1], p0, p1);
    s0 = p0;
    s1 = p1;
    q0 = (double)p0 * p0;
    q1 = (double)p1 * p1;
  }
  if (d.nf_cond && tile == 0 && threadIdx.x < d.n_flows * 4 * kH) {
    // proposal fold over the encoding columns (model/models.py:338-346); K3 adds mean/std
    const FoldRef r = fold_ref(d.cond_params, net_size<1, kH>(d.E + 4), threadIdx.x);
    ws.cb_cond[b * kCb + threadIdx.x] = fold_acc(r, d.E + 4, fold_bias0(r, d.E + 4), S.enc, 0, d.E);
  }
  TRACE(0, 2)
  store_sums4(ws.st_phys + ((int64_t)b * tiles + tile) * 4, s0, s1, q0, q1, shd);
  TRACE(0, 3)
}

// ---- K2: nf_dyn inverse
__global__ __launch_bounds__(kTile) void tiled_dyn_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  __shared__ double shd[16];
  __shared__ f2 cb[kMaxFlows * 2 * kH];
  TRACE(1, 0)
  const int tiles = n_tiles(d.N);
  const int b = blockIdx.y, tile = blockIdx.x;
  const int i = tile * kTile + threadIdx.x;
  const RowSlot S = row_slot(d, b);
  float p0 = 0.f, p1 = 0.f;
  if (i < d.N) {  // before the fold, so the loads overlap it
    p0 = S.hx[2 * i];
    p1 = S.hx[2 * i + 1];
  }
  fold_dyn(d.dyn_params, d.n_flows, tiled_ctx(ws.st_phys, b, tiles, d.N), cb, d.nf_dyn);
  __syncthreads();
  if (tile == 0 && threadIdx.x < d.n_flows * 4 * kH)  // K3's nf_dyn forward uses the same fold
    ws.cb_dyn[b * kCb + threadIdx.x] = reinterpret_cast<const float *>(cb)[threadIdx.x];
  TRACE(1, 1)
  double s0 = 0, s1 = 0, q0 = 0, q1 = 0;
  if (i < d.N) {
    float x0, x1;
    stage_dyn_inverse(d, S, i, p0, p1, cb, x0, x1);
    s0 = x0;
    s1 = x1;
    q0 = (double)x0 * x0;
    q1 = (double)x1 * x1;
  }
  TRACE(1, 2)
  store_sums4(ws.st_dyn + ((int64_t)b * tiles + tile) * 4, s0, s1, q0, q1, shd);
  TRACE(1, 3)
}

// softmax partials of the unshifted log-weight u over this tile
__device__ __forceinline__ void store_softmax(float u, bool valid, float *umax, double *usum, float *shf,
                                              double *shd) {
  // per wave (max, sum exp(u - max)), merged over the waves with one barrier
  const float mw = wave_max_dpp(valid ? u : -INFINITY);
  const double ew = wave_sum_dpp(valid ? (double)expf(u - mw) : 0.0);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    shf[w] = mw;
    shd[w] = ew;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    float m = shf[0];
    for (int k = 1; k < nw; ++k) m = fmaxf(m, shf[k]);
    double sum = 0.0;
    for (int k = 0; k < nw; ++k)
      if (shf[k] > -INFINITY) sum += shd[k] * (double)expf(shf[k] - m);
    *umax = m;
    *usum = sum;
  }
}

// ---- K3: proposal + measurement
template <bool NFD, bool NFC, int MEAS>
__global__ __launch_bounds__(kTile) void tiled_prop_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  __shared__ StepShared L;
  TRACE(2, 0)
  const int tiles = n_tiles(d.N);
  const int b = blockIdx.y, tile = blockIdx.x;
  const int i = tile * kTile + threadIdx.x;
  const RowSlot S = row_slot(d, b);
  const bool valid = i < d.N;
  PropIn in{};
  float lr = 0.f;
  if (valid) {  // issued before the row prologue so they overlap it
    in = load_prop_in<NFD>(S, i);
    lr = S.hp[i];
  }
  if (MEAS != NFDPF_MEAS_EXTERNAL) measure_row_setup<MEAS>(S.enc, d.meas_params, L);
  const int ncb = d.n_flows * 4 * kH;
  if (NFD && threadIdx.x < ncb)
    reinterpret_cast<float *>(L.cb_dyn)[threadIdx.x] = ws.cb_dyn[b * kCb + threadIdx.x];
  if (NFC && threadIdx.x < ncb) {
    // finish the proposal fold: the encoding columns came from K1, add [mean, std] of x_dyn
    const Ctx4 cp = tiled_ctx(NFD ? ws.st_dyn : ws.st_phys, b, tiles, d.N);
    const float c4[4] = {cp.m0, cp.m1, cp.s0, cp.s1};
    const FoldRef r = fold_ref(d.cond_params, net_size<1, kH>(d.E + 4), threadIdx.x);
    reinterpret_cast<float *>(L.cb_cond)[threadIdx.x] =
        fold_acc(r, d.E + 4, ws.cb_cond[b * kCb + threadIdx.x], c4, d.E, d.E + 4);
  }
  __syncthreads();
  TRACE(2, 1)
  float lk = -INFINITY, u = 0.f;
  if (valid) {
    float q0x, q1x, propose, prior;
    lk = stage_proposal<NFD, NFC, MEAS>(d, S, L, i, in, L.cb_dyn, L.cb_cond, q0x, q1x, propose, prior);
    if (MEAS != NFDPF_MEAS_EXTERNAL) {
      S.hlik[i] = lk;
      u = logw(lr, lk, prior, propose);
    }
  }
  TRACE(2, 2)
  if (MEAS == NFDPF_MEAS_EXTERNAL) return;  // phase 1: the external likelihood comes next
  const int64_t bt = (int64_t)b * tiles + tile;
  if (meas_shifted<MEAS>()) {
    const float m = block_max(lk, L.f);
    if (threadIdx.x == 0) ws.lmax[bt] = m;
  }
  store_softmax(u, valid, ws.umax + bt, ws.usum + bt, L.f + 8, L.d);  // L.f[0:8] held block_max
  TRACE(2, 3)
}

// ---- K3, two roles: 512 threads for a tile of 256 particles.  Waves 0-3 ("flows") run the
// proposal inverse, hand the proposal to waves 4-7 ("measurement") through LDS, and go on with
// the nf_dyn forward and densities while the measurement waves evaluate the likelihood of the
// same particles -- two independent chains per SIMD instead of one, at a batch size where one
// wave per SIMD is all the particles there are.
// With the cosine measurement a third role splits the encoder's output layer: waves 4-7 and
// 8-11 each produce half of the 32 outputs and their partial (|e|^2, <e, v>).
template <bool NFD, bool NFC, int MEAS, int ROLES>
__global__ __launch_bounds__(ROLES * kTile) void tiled_prop2_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  __shared__ StepShared L;
  __shared__ float qx[kTile][2];
  __shared__ float lx[kTile];
  __shared__ float ssx[ROLES][kTile], dotx[ROLES][kTile];
  __shared__ float smf[16];   // per-wave softmax partials (up to 12 waves)
  __shared__ double smd[16];
  TRACE(2, 0)
  const int tiles = n_tiles(d.N);
  const int b = blockIdx.y, tile = blockIdx.x;
  const int pl = threadIdx.x & (kTile - 1);
  const bool flows = threadIdx.x < kTile;
  const int i = tile * kTile + pl;
  const RowSlot S = row_slot(d, b);
  const bool valid = i < d.N;
  PropIn in{};
  float lr = 0.f;
  if (valid && flows) {  // issued before the row prologue so they overlap it
    in = load_prop_in<NFD>(S, i);
    lr = S.hp[i];
  }
  measure_row_setup<MEAS>(S.enc, d.meas_params, L);
  const int ncb = d.n_flows * 4 * kH;
  if (NFD && threadIdx.x < ncb)
    reinterpret_cast<float *>(L.cb_dyn)[threadIdx.x] = ws.cb_dyn[b * kCb + threadIdx.x];
  if (threadIdx.x >= kTile && threadIdx.x - kTile < ncb) {
    // finish the proposal fold: the encoding columns came from K1, add [mean, std] of x_dyn
    const int k = threadIdx.x - kTile;
    const Ctx4 cp = tiled_ctx(NFD ? ws.st_dyn : ws.st_phys, b, tiles, d.N);
    const float c4[4] = {cp.m0, cp.m1, cp.s0, cp.s1};
    const FoldRef r = fold_ref(d.cond_params, net_size<1, kH>(d.E + 4), k);
    reinterpret_cast<float *>(L.cb_cond)[k] = fold_acc(r, d.E + 4, ws.cb_cond[b * kCb + k], c4, d.E, d.E + 4);
  }
  __syncthreads();
  TRACE(2, 1)
  float q0x = 0.f, q1x = 0.f, jp = 0.f;
  if (flows && valid) {
    jp = stage_propose_inverse<NFC>(d, in, L.cb_cond, q0x, q1x);
    qx[pl][0] = q0x;
    qx[pl][1] = q1x;
  }
  __syncthreads();
  float lk = -INFINITY, u = 0.f, propose = 0.f, prior = 0.f;
  const int role = threadIdx.x / kTile;
  if (valid) {
    if (flows) {
      stage_prior<NFD, NFC>(d, S, i, in, L.cb_dyn, q0x, q1x, jp, propose, prior);
    } else if (ROLES == 3) {
      // cosine measurement, half of the encoder outputs per role (model/models.py:206-219)
      static_assert(ROLES != 3 || MEAS == NFDPF_MEAS_COS, "three roles: cosine measurement only");
      constexpr int HP = kE / 4;  // output pairs per role
      float ss, dot;
      encode_dot<kE>(wptr(d.pe_params), qx[pl][0], qx[pl][1], L.encv, ss, dot, (role - 1) * HP, role * HP);
      ssx[role][pl] = ss;
      dotx[role][pl] = dot;
    } else {
      lk = stage_measure<MEAS>(d, L, qx[pl][0], qx[pl][1]);
      S.hlik[i] = lk;
      lx[pl] = lk;
    }
  }
  __syncthreads();
  if (flows && valid) {
    float lik;
    if (ROLES == 3) {
      const float ss = ssx[1][pl] + ssx[2][pl], dot = dotx[1][pl] + dotx[2][pl];
      const float cosd = 1.0f - dot / fmaxf(sqrtf(ss), 1e-12f);
      lik = logf(1.0f / (1e-7f + cosd));
      S.hlik[i] = lik;
    } else {
      lik = lx[pl];
    }
    u = logw(lr, lik, prior, propose);
  }
  TRACE(2, 2)
  const int64_t bt = (int64_t)b * tiles + tile;
  if (meas_shifted<MEAS>()) {
    const float m = block_max(lk, L.f);  // the measurement waves hold lk, the others -inf
    if (threadIdx.x == 0) ws.lmax[bt] = m;
  }
  store_softmax(u, valid && flows, ws.umax + bt, ws.usum + bt, smf, smd);
  TRACE(2, 3)
}

// ---- K3b (phase 2 of an EXTERNAL measurement): raw likelihood from lik_ext
__global__ __launch_bounds__(kTile) void tiled_extlik_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  __shared__ float shf[16];
  __shared__ double shd[16];
  const int tiles = n_tiles(d.N);
  const int b = blockIdx.y, tile = blockIdx.x;
  const int i = tile * kTile + threadIdx.x;
  const RowSlot S = row_slot(d, b);
  const bool valid = i < d.N;
  float lk = -INFINITY, u = 0.f;
  if (valid) {
    lk = d.lik_ext[(int64_t)b * d.N + i];
    S.hlik[i] = lk;
    u = stage_logw(S, i, lk);
  }
  const int64_t bt = (int64_t)b * tiles + tile;
  const float m = block_max(lk, shf);
  if (threadIdx.x == 0) ws.lmax[bt] = m;
  store_softmax(u, valid, ws.umax + bt, ws.usum + bt, shf + 8, shd);  // shf[0:8] held block_max
}

// ---- K4: log-weights, normalisation, per-tile sums for the gate / prediction / obs-likelihood
template <bool SHIFT>
__global__ __launch_bounds__(kTile) void tiled_norm_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  TRACE(3, 0)
  __shared__ double shd[16];
  const int tiles = n_tiles(d.N);
  const int b = blockIdx.y, tile = blockIdx.x;
  const int i = tile * kTile + threadIdx.x;
  const int64_t rb = (int64_t)b * tiles;
  float M = -INFINITY, Lmax = -INFINITY;
  for (int k = 0; k < tiles; ++k) {
    M = fmaxf(M, ws.umax[rb + k]);
    if (SHIFT) Lmax = fmaxf(Lmax, ws.lmax[rb + k]);
  }
  double Sd = 0.0;
  for (int k = 0; k < tiles; ++k) Sd += ws.usum[rb + k] * (double)expf(ws.umax[rb + k] - M);
  const float Ssum = (float)Sd;
  // u = logw + Lmax for the shifted models: normalise with the same shift
  const float shift = SHIFT ? M - Lmax : M;
  const RowSlot S = row_slot(d, b);
  double sp2 = 0, px = 0, py = 0, sw = 0;
  if (i < d.N) {
    float lk = S.hlik[i];
    if (SHIFT) {
      lk = lk - Lmax;
      S.hlik[i] = lk;
    }
    const float lw = stage_logw(S, i, lk);
    const float p = expf(lw - shift) / Ssum + 1e-12f;
    S.hp[i] = p;
    sp2 = (double)p * p;
    px = (double)p * S.hx[2 * i];
    py = (double)p * S.hx[2 * i + 1];
    sw = lw;
  }
  double *fin = ws.fin + (((int64_t)b * d.T + d.t) * tiles + tile) * 4;
  TRACE(3, 2)
  store_sums4(fin, sp2, px, py, sw, shd);
  if (threadIdx.x == 0) reinterpret_cast<double *>(d.ess_out)[rb + tile] = fin[0];
  TRACE(3, 3)
}

// per-row prediction / obs-likelihood sums of every step (after the last step)
__global__ void tiled_finalize_kernel(const double *__restrict__ fin, int BT, int tiles,
                                      float *__restrict__ pred, float *__restrict__ lw_sum) {
  const int bt = blockIdx.x * blockDim.x + threadIdx.x;
  if (bt >= BT) return;
  double px = 0, py = 0, sw = 0;
  for (int k = 0; k < tiles; ++k) {
    const double *f = fin + ((int64_t)bt * tiles + k) * 4;
    px += f[1];
    py += f[2];
    sw += f[3];
  }
  pred[2 * bt] = (float)px;
  pred[2 * bt + 1] = (float)py;
  lw_sum[bt] = (float)sw;
}

// initial per-tile sums of p^2 (t = 0 gate) from p0 [B,N]
__global__ __launch_bounds__(kTile) void tiled_ess_init_kernel(const float *__restrict__ p, int N,
                                                               double *__restrict__ parts) {
  __shared__ double shd[16];
  const int tiles = n_tiles(N);
  const int b = blockIdx.y, tile = blockIdx.x;
  const int i = tile * kTile + threadIdx.x;
  double v = 0.0;
  if (i < N) {
    const float x = p[(int64_t)b * N + i];
    v = (double)x * x;
  }
  v = block_sum(v, shd);
  if (threadIdx.x == 0) parts[(int64_t)b * tiles + tile] = v;
}

__global__ void tiled_gate_kernel(const double *__restrict__ parts, int B, int tiles, int N, int force,
                                  int32_t *gate) {
  const float s = cascade_row_sum(
      [&](int r) {
        double s2 = 0.0;
        for (int k = 0; k < tiles; ++k) s2 += parts[(int64_t)r * tiles + k];
        return 1.0f / (float)s2;
      },
      force ? 0 : B);
  if (threadIdx.x == 0) gate[0] = (force || (s / (float)B) < 0.5f * (float)N) ? 1 : 0;
}

template <bool NFD, bool NFC, int MEAS>
static void launch_prop(const nfdpf_filter_desc &d, TiledWs ws, dim3 g, hipStream_t st) {
  // the two-role kernel needs a flow chain to overlap with the measurement
  // (a third role splitting the cosine encoder's output layer was measured slower: 16.7 vs
  // 11.4 us for the compute phase at C2 -- the extra waves duplicate the encoder's first layers)
  if constexpr (NFC && MEAS != NFDPF_MEAS_EXTERNAL)
    tiled_prop2_kernel<NFD, NFC, MEAS, 2><<<g, 2 * kTile, 0, st>>>(d, ws);
  else
    tiled_prop_kernel<NFD, NFC, MEAS><<<g, kTile, 0, st>>>(d, ws);
}

template <int MEAS>
static void dispatch_prop(const nfdpf_filter_desc &d, TiledWs ws, dim3 g, hipStream_t st) {
  if (d.nf_dyn && d.nf_cond)
    launch_prop<true, true, MEAS>(d, ws, g, st);
  else if (d.nf_dyn)
    launch_prop<true, false, MEAS>(d, ws, g, st);
  else if (d.nf_cond)
    launch_prop<false, true, MEAS>(d, ws, g, st);
  else
    launch_prop<false, false, MEAS>(d, ws, g, st);
}

}  // namespace nfdpf

using namespace nfdpf;

extern "C" int64_t nfdpf_filter_tiled_workspace_bytes(int B, int N, int T) {
  return (B <= 0 || N <= 0 || T <= 0) ? 256 : tiled_bytes(B, N, T);
}

extern "C" int nfdpf_filter_tiled_tiles(int N) { return N <= 0 ? 0 : n_tiles(N); }

extern "C" int nfdpf_ess_gate_tiled(const double *parts, int B, int N, int force, int32_t *gate,
                                    void *stream) {
  NFDPF_REQUIRE(gate && (force || parts) && B >= 1 && N >= 1, "nfdpf_ess_gate_tiled: bad arguments");
  tiled_gate_kernel<<<1, 64, 0, as_stream(stream)>>>(parts, B, n_tiles(N), N, force, gate);
  return launch_status("nfdpf_ess_gate_tiled");
}

extern "C" int nfdpf_filter_tiled_init(const float *p0, int B, int N, double *ess_parts,
                                       void *stream) {
  NFDPF_REQUIRE(p0 && ess_parts && B >= 0 && N >= 1, "nfdpf_filter_tiled_init: bad arguments");
  if (B == 0) return NFDPF_OK;
  tiled_ess_init_kernel<<<dim3(n_tiles(N), B), kTile, 0, as_stream(stream)>>>(p0, N, ess_parts);
  return launch_status("nfdpf_filter_tiled_init");
}

#ifdef NFDPF_EXP_TRACE
extern "C" NFDPF_API int nfdpf_exp_trace_read(void *host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_trace), sizeof(g_trace)) == hipSuccess ? 0 : 1;
}
#endif

extern "C" int nfdpf_filter_step_tiled(const nfdpf_filter_desc *dp, void *workspace, void *stream) {
  NFDPF_REQUIRE(dp && workspace, "nfdpf_filter_step_tiled: null argument");
  const nfdpf_filter_desc &d = *dp;
  NFDPF_REQUIRE(d.B >= 0 && d.N >= 2 && d.T >= 1 && d.t >= 0 && d.t < d.T,
                "nfdpf_filter_step_tiled: bad sizes (B=%d N=%d T=%d t=%d)", d.B, d.N, d.T, d.t);
  NFDPF_REQUIRE(((uintptr_t)workspace & 255) == 0, "nfdpf_filter_step_tiled: workspace not 256-B aligned");
  NFDPF_REQUIRE(d.n_flows >= 0 && d.n_flows <= kMaxFlows && d.hidden == kH,
                "nfdpf_filter_step_tiled: n_flows <= %d and hidden == %d", kMaxFlows, kH);
  NFDPF_REQUIRE(d.hist_x && d.hist_p && d.hist_noise && d.hist_lik && d.hist_idx && d.scratch &&
                    d.ess_out && d.enc && d.vel,
                "nfdpf_filter_step_tiled: null output/input pointer");
  NFDPF_REQUIRE(d.phase == 2 || (d.x_prev && d.p_prev && (d.gate || d.force_resample || d.ess_all)),
                "nfdpf_filter_step_tiled: previous-step state missing");
  NFDPF_REQUIRE(!d.nf_dyn || (d.dyn_params && d.hist_jac && d.hist_prior),
                "nfdpf_filter_step_tiled: nf_dyn needs dyn_params, hist_jac, hist_prior");
  NFDPF_REQUIRE(d.nf_dyn >= NFDPF_DYN_NONE && d.nf_dyn <= NFDPF_DYN_MAF,
                "nfdpf_filter_step_tiled: bad nf_dyn %d", d.nf_dyn);
  NFDPF_REQUIRE(!d.nf_cond || d.cond_params, "nfdpf_filter_step_tiled: nf_cond needs cond_params");
  NFDPF_REQUIRE(d.measurement == NFDPF_MEAS_EXTERNAL || (d.E == kE && d.pe_params),
                "nfdpf_filter_step_tiled: fused measurements need E == %d", kE);
  NFDPF_REQUIRE(!(d.measurement == NFDPF_MEAS_CRNVP || d.measurement == NFDPF_MEAS_NN) || d.meas_params,
                "nfdpf_filter_step_tiled: measurement parameters missing");
  NFDPF_REQUIRE(d.E + 4 <= kMaxCtx, "nfdpf_filter_step_tiled: E too large");
  NFDPF_REQUIRE(d.measurement != NFDPF_MEAS_EXTERNAL || d.phase != 0,
                "nfdpf_filter_step_tiled: EXTERNAL measurement runs as phase 1 + phase 2");
  NFDPF_REQUIRE(d.measurement != NFDPF_MEAS_EXTERNAL || d.phase != 2 || d.lik_ext,
                "nfdpf_filter_step_tiled: phase 2 needs lik_ext");
  if (d.resampler == NFDPF_RESAMPLE_SOFT) {
    NFDPF_REQUIRE(d.N <= kStepMaxN, "nfdpf_filter_step_tiled: soft resampling supports N <= %d", kStepMaxN);
    NFDPF_REQUIRE(d.lin || d.phase == 2, "nfdpf_filter_step_tiled: soft resampling needs lin");
    NFDPF_REQUIRE(d.B_global <= kStepMaxN, "nfdpf_filter_step_tiled: soft resampling supports B_global <= %d",
                  kStepMaxN);
  } else {
    NFDPF_REQUIRE(d.ot_x || d.phase == 2, "nfdpf_filter_step_tiled: OT path needs ot_x");
  }
  NFDPF_REQUIRE(d.rng_mode == NFDPF_RNG_DEVICE || (d.gate && d.host_noise) || d.phase == 2,
                "nfdpf_filter_step_tiled: HOST rng mode needs gate and host_noise");
  if (d.B == 0) return NFDPF_OK;
  hipStream_t st = as_stream(stream);
  TiledWs ws = tiled_carve(workspace, d.B, d.N, d.T);
  const dim3 g(n_tiles(d.N), d.B);
  if (d.phase != 2) {
    const size_t lds = d.resampler == NFDPF_RESAMPLE_SOFT ? (size_t)(std::max(d.N, d.B_global) + d.N) * 4
                                                         : (size_t)d.B_global * 4;
    tiled_front_kernel<<<g, kTile, lds, st>>>(d, ws);
    if (d.nf_dyn) tiled_dyn_kernel<<<g, kTile, 0, st>>>(d, ws);
    hipEvent_t *ev = (hipEvent_t *)d.prof_events;
    if (ev) (void)hipEventRecord(ev[0], st);
    switch (d.measurement) {
      case NFDPF_MEAS_COS: dispatch_prop<NFDPF_MEAS_COS>(d, ws, g, st); break;
      case NFDPF_MEAS_CRNVP: dispatch_prop<NFDPF_MEAS_CRNVP>(d, ws, g, st); break;
      case NFDPF_MEAS_NN: dispatch_prop<NFDPF_MEAS_NN>(d, ws, g, st); break;
      case NFDPF_MEAS_GAUSSIAN: dispatch_prop<NFDPF_MEAS_GAUSSIAN>(d, ws, g, st); break;
      case NFDPF_MEAS_EXTERNAL: dispatch_prop<NFDPF_MEAS_EXTERNAL>(d, ws, g, st); break;
      default: set_error("nfdpf_filter_step_tiled: unknown measurement %d", d.measurement); return NFDPF_EINVAL;
    }
    if (ev) (void)hipEventRecord(ev[1], st);
    if (d.phase == 1) return launch_status("nfdpf_filter_step_tiled");
  }
  if (d.measurement == NFDPF_MEAS_EXTERNAL) tiled_extlik_kernel<<<g, kTile, 0, st>>>(d, ws);
  const bool shift = d.measurement == NFDPF_MEAS_CRNVP || d.measurement == NFDPF_MEAS_GAUSSIAN ||
                     d.measurement == NFDPF_MEAS_EXTERNAL;
  if (shift)
    tiled_norm_kernel<true><<<g, kTile, 0, st>>>(d, ws);
  else
    tiled_norm_kernel<false><<<g, kTile, 0, st>>>(d, ws);
  if (d.t == d.T - 1 && d.pred && d.lw_sum) {
    const int BT = d.B * d.T;
    tiled_finalize_kernel<<<(BT + 255) / 256, 256, 0, st>>>(ws.fin, BT, n_tiles(d.N), d.pred, d.lw_sum);
  }
  return launch_status("nfdpf_filter_step_tiled");
}
