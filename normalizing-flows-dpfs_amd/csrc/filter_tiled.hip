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
#include <hip/hip_ext.h>

#ifdef NFDPF_EXP_QTRACE
// experiment-only: per-WAVE phase timestamps of the quad proposal launch (last step run)
__device__ unsigned long long g_qtrace[1024][16][16];
#define QTRACE(P)                                                                           \
  if ((threadIdx.x & 63) == 0 && blockIdx.y * gridDim.x + blockIdx.x < 1024)                \
    g_qtrace[blockIdx.y * gridDim.x + blockIdx.x][threadIdx.x >> 6][P] = __builtin_amdgcn_s_memrealtime();
#else
#define QTRACE(P)
#endif

#include "split.hpp"
#include "crnvp_mfma.hpp"

// front + dyn in one launch (tiled_fdyn_kernel) for rows up to this length (LDS)
constexpr int kMergedMaxN_ = 4096;

namespace nfdpf {

constexpr int kTile = 256;  // particles per workgroup, one per lane

#ifdef NFDPF_EXP_TRACE
// experiment-only: per-workgroup phase timestamps (s_memrealtime, 100 MHz) of one launch
__device__ unsigned long long g_trace[4][2048][8];
#define TRACE(K, P)                                                                        \
  if (threadIdx.x == 0 && blockIdx.y * gridDim.x + blockIdx.x < 2048)                     \
    g_trace[K][blockIdx.y * gridDim.x + blockIdx.x][P] = __builtin_amdgcn_s_memrealtime();
// the same from lane 0 of the executing wave (several waves of one workgroup record slots)
#define TRACEW(K, P)                                                                       \
  if ((threadIdx.x & 63) == 0 && blockIdx.y * gridDim.x + blockIdx.x < 2048)              \
    g_trace[K][blockIdx.y * gridDim.x + blockIdx.x][P] = __builtin_amdgcn_s_memrealtime();
#else
#define TRACE(K, P)
#define TRACEW(K, P)
#endif

// (row b, tile) of this workgroup.  -DNFDPF_XCD_REMAP: blocks are dealt round-robin over the 8
// XCDs (blocks k and k + 8 share one, MI355X_MICROARCH.md §Workgroup dispatch), so a row's tiles
// (blocks 4b .. 4b + 3) sat on 4 different L2s; the remap gives each XCD group whole rows, so the
// row-level data of the previous launch (the row's particles and partials) is read from the
// reader's own L2.  Any bijection is correct: every kernel derives (b, tile) here.  Measured
// SLOWER at C2 (2.05e9 vs 2.13e9: both launches ~0.5-0.8 us longer, one box) -- not the default.
__device__ __forceinline__ void tile_row(int &b, int &tile) {
#ifdef NFDPF_XCD_REMAP
  const int n = gridDim.x * gridDim.y;
  if ((n & 7) == 0) {
    const int id = blockIdx.x + gridDim.x * blockIdx.y;
    const int lin = (id & 7) * (n >> 3) + (id >> 3);
    tile = lin % gridDim.x;
    b = lin / gridDim.x;
    return;
  }
#endif
  b = blockIdx.y;
  tile = blockIdx.x;
}

struct TiledWs {
  double *st_phys;  // [B][tiles][4] sum x0, x1, x0^2, x1^2 of x_phys
  double *st_dyn;   // [B][tiles][4] same for x_dyn
  float *cb_dyn;    // [B][kCb] folded nf_dyn biases of the row (K2, tile 0)
  float *cb_cond;   // [B][kCb] proposal fold over the encoding columns (K1, tile 0)
  double *fin;      // [B][T][tiles][4] sum p^2, sum p x0, sum p x1, sum logw
  uint64_t *rowx;   // [B][tiles][8] the fused step's x_dyn partials as tagged granules
  // tiled_rows_kernel's outputs (long rows, soft resampler): the step's gate, each row's
  // normaliser of the deferred slot t-1 and, when the gate fired, each particle's source and
  // resampled log-weight
  int32_t *rs_gate;  // [1]
  float *rs_rn;      // [B][4] RowNorm {shift, Ssum, Lmax}
  int32_t *rs_src;   // [B][N]
  float *rs_lr;      // [B][N]
};
// The step's softmax partials live in the caller's ess_out / ess_all (include/nfdpf.h):
// per (row, tile) {max u, sum e^(u-max), sum e^(2(u-max)), max raw likelihood}.
constexpr int kSm = 4;

constexpr int kCb = kMaxFlows * 4 * kH;  // floats of one row's folded-bias table

static inline int64_t al256(int64_t v) { return (v + 255) / 256 * 256; }
__host__ __device__ static inline int n_tiles(int N) { return (N + kTile - 1) / kTile; }

static int64_t tiled_bytes(int B, int N, int T) {
  const int64_t bt = (int64_t)B * n_tiles(N);
  return al256(bt * 32) * 2 + al256((int64_t)B * kCb * 4) * 2 + al256(bt * T * 32) + al256(bt * 64) + al256(4) +
         al256((int64_t)B * 16) + al256((int64_t)B * N * 4) * 2;
}

static TiledWs tiled_carve(void *ws, int B, int N, int T) {
  char *p = (char *)ws;
  const int64_t bt = (int64_t)B * n_tiles(N);
  TiledWs w;
  w.st_phys = (double *)p;
  p += al256(bt * 32);
  w.st_dyn = (double *)p;
  p += al256(bt * 32);
  w.cb_dyn = (float *)p;
  p += al256((int64_t)B * kCb * 4);
  w.cb_cond = (float *)p;
  p += al256((int64_t)B * kCb * 4);
  w.fin = (double *)p;
  p += al256(bt * T * 32);
  w.rowx = (uint64_t *)p;
  p += al256(bt * 64);
  w.rs_gate = (int32_t *)p;
  p += al256(4);
  w.rs_rn = (float *)p;
  p += al256((int64_t)B * 16);
  w.rs_src = (int32_t *)p;
  p += al256((int64_t)B * N * 4);
  w.rs_lr = (float *)p;
  return w;
}

// 1 / sum_n p_n^2 of one row from its per-tile softmax partials (DPFs.py:163).  With
// e_n = e^(u_n - M) and S = sum e_n, p_n = e_n / S (+ 1e-12 after a filter step, DPFs.py:192):
// sum p^2 = sum e^2 / S^2 + 2e-12 + N 1e-24.  fp64 throughout; the reference sums fp32 p^2 in
// cascade order, so the two agree to ~1e-7 relative.
// The tile partials through an accessor sm(i) = partial word i of the row: a global pointer
// (row_inv_ess / row_norm below), or a register array indexed by constants (KT: the tiles loop
// fully unrolled, k < tiles masked -- the same operations in the same order, tiles <= KT).
// Through a generic pointer these reads compiled to flat_load (which also counts on lgkmcnt);
// a register array reached through a pointer lived in scratch.
typedef const double __attribute__((address_space(1))) gdouble;
template <int KT, class SM>
__device__ __forceinline__ float row_inv_ess_t(const SM &sm, int tiles, int N, bool eps) {
  double M = -INFINITY;
#pragma unroll
  for (int k = 0; k < KT; ++k)
    if (KT == 0 || k < tiles) M = sm(kSm * k) > M ? sm(kSm * k) : M;
  double S = 0.0, Q = 0.0;
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    if (!(KT == 0 || k < tiles)) continue;
    // the tile rescale factors in f32 (relative error ~1e-7, the gate's own resolution)
    const float f = expf((float)(sm(kSm * k) - M));
    S += sm(kSm * k + 1) * (double)f;
    Q += sm(kSm * k + 2) * ((double)f * (double)f);
  }
  double sp2 = Q / (S * S);
  if (eps) sp2 += 2e-12 + (double)N * 1e-24;
  return 1.0f / (float)sp2;
}
__device__ __forceinline__ float row_inv_ess(const double *sm_, int tiles, int N, bool eps) {
  gdouble *sm = (gdouble *)sm_;
  double M = -INFINITY;
  for (int k = 0; k < tiles; ++k) M = sm[kSm * k] > M ? sm[kSm * k] : M;
  double S = 0.0, Q = 0.0;
  for (int k = 0; k < tiles; ++k) {
    const float f = expf((float)(sm[kSm * k] - M));
    S += sm[kSm * k + 1] * (double)f;
    Q += sm[kSm * k + 2] * ((double)f * (double)f);
  }
  double sp2 = Q / (S * S);
  if (eps) sp2 += 2e-12 + (double)N * 1e-24;
  return 1.0f / (float)sp2;
}

// normalize_log_probs of a row (utils.py:39-44) from its softmax partials:
// p = e^(lw - shift) / S + 1e-12, shift = max u (- max raw likelihood for the shifted models)
struct RowNorm {
  float shift, Ssum, Lmax;
};
template <int KT, class SM>
__device__ __forceinline__ RowNorm row_norm_t(const SM &sm, int tiles, bool shifted) {
  float M = -INFINITY, Lmax = -INFINITY;
#pragma unroll
  for (int k = 0; k < KT; ++k) {
    if (!(k < tiles)) continue;
    M = fmaxf(M, (float)sm(kSm * k));
    if (shifted) Lmax = fmaxf(Lmax, (float)sm(kSm * k + 3));
  }
  double Sd = 0.0;
#pragma unroll
  for (int k = 0; k < KT; ++k)
    if (k < tiles) Sd += sm(kSm * k + 1) * (double)expf((float)sm(kSm * k) - M);
  return RowNorm{shifted ? M - Lmax : M, (float)Sd, Lmax};
}
__device__ __forceinline__ RowNorm row_norm(const double *sm_, int tiles, bool shifted) {
  gdouble *sm = (gdouble *)sm_;
  float M = -INFINITY, Lmax = -INFINITY;
  for (int k = 0; k < tiles; ++k) {
    M = fmaxf(M, (float)sm[kSm * k]);
    if (shifted) Lmax = fmaxf(Lmax, (float)sm[kSm * k + 3]);
  }
  double Sd = 0.0;
  for (int k = 0; k < tiles; ++k) Sd += sm[kSm * k + 1] * (double)expf((float)sm[kSm * k] - M);
  // u = logw + Lmax for the shifted models: normalise with the same shift
  return RowNorm{shifted ? M - Lmax : M, (float)Sd, Lmax};
}

// ESS gate: torch.mean over the batch of the rows' 1/sum p^2 (ATen's cascade order),
// evaluated by every wave (lanes in parallel over rows) -- the same decision everywhere.
__device__ __forceinline__ bool tiled_gate(const nfdpf_filter_desc &d, int tiles) {
  if (d.gate) return d.gate[0] != 0;
  if (d.force_resample) return true;
  const double *parts = reinterpret_cast<const double *>(d.ess_all);
  const float s = cascade_row_sum(
      [&](int r) { return row_inv_ess(parts + (int64_t)r * tiles * kSm, tiles, d.N, d.t > 0); }, d.B_global);
  return (s / (float)d.B_global) < 0.5f * (float)d.N;
}

// The same gate, block-parallel (all threads call): thread r stages row r's 1 / sum p^2 in
// `buf` (one round trip for the whole batch), wave 0 folds them in cascade order.
// With `rn_row` >= 0 the thread that stages that row also leaves its RowNorm in *rn (LDS),
// readable by every thread on return (the deferred normalisation needs it, same data).
__device__ bool tiled_gate_block(const nfdpf_filter_desc &d, int tiles, float *buf, int *flag,
                                 int64_t rn_row = -1, RowNorm *rn = nullptr, bool shifted = false) {
  const double *parts = reinterpret_cast<const double *>(d.ess_all);
  if (d.gate || d.force_resample) {
    if (rn_row >= 0 && threadIdx.x == 0) *rn = row_norm(parts + rn_row * tiles * kSm, tiles, shifted);
    __syncthreads();
    return d.gate ? d.gate[0] != 0 : true;
  }
  for (int r = threadIdx.x; r < d.B_global; r += blockDim.x) {
    buf[r] = row_inv_ess(parts + (int64_t)r * tiles * kSm, tiles, d.N, d.t > 0);
    if (r == rn_row) *rn = row_norm(parts + (int64_t)r * tiles * kSm, tiles, shifted);
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const float s = cascade_row_sum([&](int r) { return buf[r]; }, d.B_global);
    if (threadIdx.x == 0) *flag = (s / (float)d.B_global) < 0.5f * (float)d.N;
  }
  __syncthreads();
  return *flag != 0;
}

__host__ __device__ constexpr bool shifted_meas(int meas) {
  return meas == NFDPF_MEAS_CRNVP || meas == NFDPF_MEAS_GAUSSIAN || meas == NFDPF_MEAS_EXTERNAL;
}

// the normalised weight of particle i of slot S (hp still holding log p_res, hlik the raw
// likelihood): returns p, the log-weight lw and the (shifted) likelihood lk; writes nothing
__device__ __forceinline__ float norm_value(const RowSlot &S, int i, const RowNorm &rn, bool shifted, float &lw,
                                            float &lk) {
  lk = S.hlik[i];
  if (shifted) lk = lk - rn.Lmax;
  lw = stage_logw(S, i, lk);
  return expf(lw - rn.shift) / rn.Ssum + 1e-12f;
}
// ... and stores it: hp = p, hlik = shifted likelihood
__device__ __forceinline__ float norm_particle(const RowSlot &S, int i, const RowNorm &rn, bool shifted,
                                               float &lw) {
  float lk;
  const float p = norm_value(S, i, rn, shifted, lw, lk);
  if (shifted) S.hlik[i] = lk;
  S.hp[i] = p;
  return p;
}

// The previous step's per-particle values a deferred normalisation needs, loaded up front.
struct PrevIn {
  float lr, lik, prop, prior, x0, x1;
};
__device__ __forceinline__ PrevIn load_prev_in(const RowSlot &Sp, int i) {
  return PrevIn{Sp.hp[i], Sp.hlik[i], Sp.scr[4 * i + 2], Sp.scr[4 * i + 3], Sp.hx[2 * i], Sp.hx[2 * i + 1]};
}
// p of a prefetched particle (the arithmetic of norm_value)
__device__ __forceinline__ float prev_p_of(const PrevIn &v, const RowNorm &rn, bool shifted, float &lw, float &lk) {
  lk = shifted ? v.lik - rn.Lmax : v.lik;
  lw = ((v.lr + lk) + v.prior) - v.prop;
  return expf(lw - rn.shift) / rn.Ssum + 1e-12f;
}
// row b's softmax partials inside ess_all (global rows when the batch is sharded)
// row of ess_all holding local row b: the global row of a sharded batch, unless the
// speculative-gate mode keeps only this shard's rows (ess_local)
__device__ __forceinline__ int64_t ess_row(const nfdpf_filter_desc &d, int b) {
  return (!d.ess_local && d.row_base + d.B <= d.B_global) ? d.row_base + b : b;
}
__device__ __forceinline__ const double *prev_sm(const nfdpf_filter_desc &d, int b, int tiles) {
  return reinterpret_cast<const double *>(d.ess_all) + ess_row(d, b) * tiles * kSm;
}

// Deferred normalisation of step t-1 (defer_norm, t > 0): slot t-1's weights are written by
// the second launch of step t -- after every workgroup of the first launch has read slot t-1
// (the gate / resampler / motion) and before anything overwrites the step-t-1 values of the
// scratch (propose, prior).  All threads call (block reduction inside).
__device__ __forceinline__ void finish_prev(const nfdpf_filter_desc &d, TiledWs ws, int b, int tile, int i,
                                            bool own, const PrevIn &v, double *shd) {
  const int tiles = n_tiles(d.N);
  const bool shifted = shifted_meas(d.measurement);
  const RowNorm rn = row_norm(prev_sm(d, b, tiles), tiles, shifted);
  const RowSlot Sp = row_slot(d, b, d.t - 1);
  double sp2 = 0, px = 0, py = 0, sw = 0;
  if (own && i < d.N) {
    float lw, lk;
    const float p = prev_p_of(v, rn, shifted, lw, lk);
    if (shifted) Sp.hlik[i] = lk;
    Sp.hp[i] = p;
    sp2 = (double)p * p;
    px = (double)p * v.x0;
    py = (double)p * v.x1;
    sw = lw;
  }
  block_sum4_store(sp2, px, py, sw, shd, ws.fin + (((int64_t)b * d.T + d.t - 1) * tiles + tile) * 4);
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
//
// ROWS (long rows: tiled_rows_kernel ran first): the gate, the deferred slot's row normaliser
// and -- when the gate fired -- every particle's source and resampled log-weight come from
// that launch, so this one holds no dynamic LDS and no per-tile copy of the row's search.

// ---- K0 for long rows with the soft resampler, one 1024-thread workgroup per row: the step's
// ESS gate (the same block-parallel cascade-order evaluation, every workgroup alike), the row
// normaliser of the deferred slot t-1 and, when the gate fires, the row's soft resampling
// (resamplers.py:20-60, the soft.hpp recipe) ONCE per row.  tiled_front_kernel otherwise
// rebuilds the row's CDF and searches all N markers in each of the row's N / 256 tiles and
// evaluates the batch gate in every one of them (C5: 2,560 workgroups each reading the 64 x 40
// partials, with 120 KB of LDS each: one workgroup per CU -- 235 us per step, round 2).
__global__ __launch_bounds__(1024) void tiled_rows_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  extern __shared__ float dyn_lds[];
  __shared__ double shd[16];
  __shared__ float shf[16];
  __shared__ int fire_sh;
  __shared__ RowNorm rn_sh;
  const int tiles = n_tiles(d.N), N = d.N;
  const int b = blockIdx.x;
  const int64_t grow = d.row_base + b;
  const bool defer = d.defer_norm && d.t > 0;
  const bool shifted = shifted_meas(d.measurement);
  float *Cbuf = dyn_lds;
  const bool fire = tiled_gate_block(d, tiles, Cbuf, &fire_sh, defer ? ess_row(d, b) : -1, &rn_sh, shifted);
  if (threadIdx.x == 0) {
    if (b == 0) ws.rs_gate[0] = fire ? 1 : 0;
    if (defer) {
      ws.rs_rn[4 * b] = rn_sh.shift;
      ws.rs_rn[4 * b + 1] = rn_sh.Ssum;
      ws.rs_rn[4 * b + 2] = rn_sh.Lmax;
    }
  }
  if (!fire || d.resampler != NFDPF_RESAMPLE_SOFT) return;
  const float *pprev = d.p_prev + b * d.p_prev_rs;
  float *wbuf = dyn_lds + max(N, d.B_global);
  if (defer) {  // the row's p_{t-1} into LDS for the resampler
    const RowNorm rn = rn_sh;
    const RowSlot Sp = row_slot(d, b, d.t - 1);
    float *pbuf = wbuf + N;
    for (int j = threadIdx.x; j < N; j += blockDim.x) {
      float lw, lk;
      pbuf[j] = norm_value(Sp, j, rn, shifted, lw, lk);
    }
    __syncthreads();
    pprev = pbuf;
  }
  SoftRow row{pprev, N, d.alpha, 1.0f / (float)N, (float)(1.0 - (double)d.alpha), 1.0f};
  float off;
  if (d.rng_mode == NFDPF_RNG_HOST && d.host_offsets)
    off = d.host_offsets[b];
  else
    off = u01(rng_draw(d.seed, kTagOffset, (uint32_t)d.t, grow, 0u).x) * (1.0f / (float)N);
  int32_t *src_out = ws.rs_src + (int64_t)b * N;
  soft_row_search(row, d.lin, off, Cbuf, shd, shf, [&](int j, int src) {
    // src == N: the reference's out-of-range edge (next row's first particle, weight 0)
    wbuf[j] = src < N ? row.w(src) : 0.f;
    src_out[j] = src;
  });
  __syncthreads();
  if (threadIdx.x < 64) {
    const float s2 = cascade_row_sum([&](int j) { return wbuf[j]; }, N);
    if (threadIdx.x == 0) shf[8] = s2;
  }
  __syncthreads();
  const float s2 = shf[8];
  float *lr_out = ws.rs_lr + (int64_t)b * N;
  for (int j = threadIdx.x; j < N; j += blockDim.x) lr_out[j] = logf(wbuf[j] / s2);
}

template <bool ROWS>
__global__ __launch_bounds__(kTile) void tiled_front_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  extern __shared__ float dyn_lds[];
  __shared__ double shd[16];
  __shared__ float shf[16];
  __shared__ int fire_sh;
  __shared__ float xr_sh[ROWS ? 1 : kTile][2];
  __shared__ int src_sh[ROWS ? 1 : kTile];
  TRACE(0, 0)
  const int tiles = n_tiles(d.N), N = d.N;
  int b, tile;
  tile_row(b, tile);
  const int i = tile * kTile + threadIdx.x;
  const int64_t grow = d.row_base + b;
  float *Cbuf = dyn_lds;
  PrevIn pv{};
  const bool defer = d.defer_norm && d.t > 0;
  if (defer && i < N) pv = load_prev_in(row_slot(d, b, d.t - 1), i);  // overlaps the gate
  float e0 = 0.f, e1 = 0.f;
  if (i < N) motion_noise(d, b, grow, i, e0, e1);  // independent of the gate: computed under its latency
  __shared__ RowNorm rn_sh;
  bool fire;
  if constexpr (ROWS) {
    fire = ws.rs_gate[0] != 0;
  } else {
    const int64_t my_row = ess_row(d, b);
    fire = tiled_gate_block(d, tiles, Cbuf, &fire_sh, defer ? my_row : -1, &rn_sh, shifted_meas(d.measurement));
  }
  TRACE(0, 1)
  const int mode = !fire ? kSrcPrev : (d.resampler == NFDPF_RESAMPLE_SOFT ? kSrcSoft : kSrcOt);
  const RowSlot S = row_slot(d, b);
  const float *xprev = d.x_prev + b * d.x_prev_rs;
  const float *pprev = d.p_prev + b * d.p_prev_rs;
  // defer_norm: step t-1 is not normalised yet; its weights are derived here on the fly from
  // slot t-1 (read only -- the second launch of this step writes them, finish_prev)
  RowNorm rn{0.f, 1.f, 0.f};
  RowSlot Sp = S;
  if (defer) {
    if constexpr (ROWS)
      rn = RowNorm{ws.rs_rn[4 * b], ws.rs_rn[4 * b + 1], ws.rs_rn[4 * b + 2]};
    else
      rn = rn_sh;  // left by the gate staging (same partials)
    Sp = row_slot(d, b, d.t - 1);
  }
  auto prev_p = [&](int j) {
    float lw, lk;
    return norm_value(Sp, j, rn, shifted_meas(d.measurement), lw, lk);
  };
  float x0 = 0.f, x1 = 0.f, lr = 0.f;
  if (ROWS && mode == kSrcSoft) {
    if (i < N) {  // the row's resampling, done once by tiled_rows_kernel
      const int src = ws.rs_src[(int64_t)b * N + i];
      const float *xs = src < N ? xprev + 2 * src : (b + 1 < d.B ? xprev + d.x_prev_rs : xprev + 2 * (N - 1));
      x0 = xs[0];
      x1 = xs[1];
      lr = ws.rs_lr[(int64_t)b * N + i];
      S.hidx[i] = (int64_t)N * grow + src;
    }
  } else if (mode == kSrcSoft) {
    float *wbuf = dyn_lds + max(N, d.B_global);
    if (defer) {  // the row's p_{t-1} into LDS for the resampler
      float *pbuf = wbuf + N;
      for (int j = threadIdx.x; j < N; j += blockDim.x) pbuf[j] = prev_p(j);
      __syncthreads();
      pprev = pbuf;
    }
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
      if (defer) {
        float lw, lk;
        x0 = pv.x0;
        x1 = pv.x1;
        lr = logf(prev_p_of(pv, rn, shifted_meas(d.measurement), lw, lk));
      } else {
        x0 = xprev[2 * i];
        x1 = xprev[2 * i + 1];
        lr = logf(pprev[i]);
      }
    }
    S.hidx[i] = (int64_t)N * grow + i;
  }
  double s0 = 0, s1 = 0, q0 = 0, q1 = 0;
  if (i < N) {
    float p0, p1;
    motion_apply_eps(S, i, x0, x1, lr, d.vel[2 * b], d.vel[2 * b + 1], e0, e1, p0, p1);
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

// ---- the fused step (tiled_step_fused_kernel, below; opt-in, see use_fused): the merged front
// launch and the quad proposal launch as ONE launch per step.  Their only coupling inside a step is the row's x_dyn
// sums (the proposal's [mean, std] context): instead of a launch boundary, the four workgroups
// of a row exchange their partials through data-tagged 8-byte granules {32 data bits, tag}
// (agent-scope stores / loads: L2, no flag, no fence; MI355X_MICROARCH.md handoff-1to1).  The
// tag is (pass epoch << 16) + t + 1 -- the epoch is bumped by a one-lane kernel at the start
// of every pass (graph replays included), so granules of an earlier pass never match.  Needs
// every workgroup of the grid resident at once (the host checks grid <= CUs, one 1024-thread
// workgroup per CU); a poll that never sees its tag gives up at kSpinCap and counts a fault.
__device__ uint32_t g_step_epoch = 0;
constexpr int kFusedMaxTiles = kMergedMaxN_ / kTile;
struct FusedLds {
  float cb[kMaxFlows * 4 * kH];       // nf_dyn fold of the row (tiled_fdyn_kernel's cb, flat)
  float encfold[kMaxFlows * 4 * kH];  // the proposal fold over the encoding columns
  double rowst[kFusedMaxTiles * 4];   // the row's x_dyn partials, tile order (tiled_ctx input)
};
__device__ __forceinline__ void publish_granules(uint64_t *g, double v, uint32_t tag) {
  const uint64_t bits = (uint64_t)__double_as_longlong(v);
  __hip_atomic_store(g, ((uint64_t)tag << 32) | (bits & 0xffffffffull), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store(g + 1, ((uint64_t)tag << 32) | (bits >> 32), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// wave 0 polls the row's granules (8 per tile) until every tag matches, then leaves the
// doubles in fx->rowst; all threads call (one barrier)
__device__ __forceinline__ void row_sync(const nfdpf_filter_desc &d, const TiledWs &ws, FusedLds *fx, uint32_t tag) {
  const int tiles = n_tiles(d.N);
  const int ng = tiles * 8;
  if (threadIdx.x < 64) {
    int b, tile;
    tile_row(b, tile);
    const uint64_t *g = ws.rowx + (int64_t)b * tiles * 8;
    for (int base = 0; base < ng; base += 64) {
      const int q = base + (int)threadIdx.x;
      uint64_t v = 0;
      bool ok = q >= ng;
      for (int it = 0;; ++it) {
        if (!ok) {
          v = __hip_atomic_load(g + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          ok = (uint32_t)(v >> 32) == tag;
        }
        if (__all(ok)) break;
        if (it >= kSpinCap) {
          if (threadIdx.x == 0) atomicAdd(&g_split_fault, 1);
          break;
        }
        __builtin_amdgcn_s_sleep(1);
      }
      if (q < ng) reinterpret_cast<uint32_t *>(fx->rowst)[q] = (uint32_t)v;
    }
  }
  __syncthreads();
}

// ---- K2: nf_dyn inverse; with defer_norm also the normalisation of slot t-1 (finish_prev's
// arithmetic, its sums reduced together with this launch's in one barrier).  SPLIT: the
// RealNVP nets on wave pairs (split.hpp) -- role 0 = t-nets (and the stores), role 1 =
// s-nets (and the deferred normalisation).
// Each role's waves reduce their own four sums; thread k < 8 adds the wave partials of role
// k / 4 in particle-group order (waves k / 4, 2 + k / 4, ...) -- the order of block_sum8_store
// over the same particles.
__device__ __forceinline__ void block_sum_roles_store(const double (&v)[4], double *dst0, double *dst1,
                                                      double *sh, uint64_t *gran = nullptr, uint32_t tag = 0) {
  const int w = threadIdx.x >> 6;
  // a role whose destination is null skips its reductions (wave-uniform; fp64 DPP sums of 8
  // waves are a visible share of a short launch's epilogue)
  if (w < 8 && (w & 1 ? dst1 : dst0) != nullptr) {  // waves >= 8 (the fused step's) hold nothing here
    double w4[4] = {v[0], v[1], v[2], v[3]};
    wave_sum_dpp_n(w4);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
      for (int k = 0; k < 4; ++k) sh[4 * w + k] = w4[k];
  }
  __syncthreads();
  if (threadIdx.x < 8) {
    const int r = threadIdx.x >> 2, k = threadIdx.x & 3;
    double *dst = r ? dst1 : dst0;
    if (dst) {
      double a = sh[4 * r + k];
      for (int q = 1; q < 4; ++q) a += sh[4 * (2 * q + r) + k];
      dst[k] = a;
      if (gran && r == 0) publish_granules(gran + 2 * k, a, tag);  // the fused step's row exchange
    }
  }
}

template <bool SPLIT>
__global__ __launch_bounds__(SPLIT ? 2 * kTile : kTile) void tiled_dyn_kernel(const nfdpf_filter_desc d,
                                                                               TiledWs ws) {
  __shared__ double shd[64];
  __shared__ f2 cb[kMaxFlows * 2 * kH];
  __shared__ f2 cbs[SPLIT ? kMaxFlows * 2 * kH : 1];  // split order (split_cb_index)
  __shared__ __attribute__((aligned(8))) float xbuf[SPLIT ? 8 * kTile : 1];
  __shared__ int xflag[16];
  TRACE(1, 0)
  const int tiles = n_tiles(d.N);
  int b, tile;
  tile_row(b, tile);
  const SplitLane sl = SPLIT ? split_lane(8) : SplitLane{0, (int)threadIdx.x};
  const int role = sl.role, slot = sl.slot;
  const int i = tile * kTile + slot;
  const RowSlot S = row_slot(d, b);
  float p0 = 0.f, p1 = 0.f;
  PrevIn pv{};
  const bool defer = d.defer_norm && d.t > 0;
  const bool defer_here = defer && role == (SPLIT ? 1 : 0);
  const bool shifted = shifted_meas(d.measurement);
  if (i < d.N) {  // before the fold, so the loads overlap it
    p0 = S.hx[2 * i];
    p1 = S.hx[2 * i + 1];
    if (defer_here) pv = load_prev_in(row_slot(d, b, d.t - 1), i);
  }
  const RowNorm rn = defer_here ? row_norm(prev_sm(d, b, tiles), tiles, shifted) : RowNorm{0.f, 1.f, 0.f};
  if (SPLIT) {
    if (threadIdx.x < 16) xflag[threadIdx.x] = 0;
    pair_clear(xbuf, kTile);
    if (threadIdx.x < d.n_flows * 4 * kH) {
      const Ctx4 c = tiled_ctx(ws.st_phys, b, tiles, d.N);
      const float cv[4] = {c.m0, c.m1, c.s0, c.s1};
      const float v = fold_one(d.dyn_params, kNsDyn, kOctxDyn, threadIdx.x, cv);
      reinterpret_cast<float *>(cb)[threadIdx.x] = v;
      reinterpret_cast<float *>(cbs)[split_cb_index(threadIdx.x)] = v;
    }
  } else {
    fold_dyn(d.dyn_params, d.n_flows, tiled_ctx(ws.st_phys, b, tiles, d.N), cb, d.nf_dyn);
  }
  __syncthreads();
  if (tile == 0 && threadIdx.x < d.n_flows * 4 * kH)  // K3's nf_dyn forward uses the same fold
    ws.cb_dyn[b * kCb + threadIdx.x] = reinterpret_cast<const float *>(cb)[threadIdx.x];
  TRACE(1, 1)
  double sd[4] = {0, 0, 0, 0}, sf[4] = {0, 0, 0, 0};
  if (i < d.N) {
    float x0 = 0.f, x1 = 0.f;
    if (SPLIT) {
      PairX x = pair_of(xbuf, xflag, role, slot);
      stage_dyn_inverse_split(d, S, i, p0, p1, cbs, x, kTile, x0, x1);
    } else {
      stage_dyn_inverse(d, S, i, p0, p1, cb, x0, x1);
    }
    if (role == 0) {
      sd[0] = x0;
      sd[1] = x1;
      sd[2] = (double)x0 * x0;
      sd[3] = (double)x1 * x1;
    }
    if (defer_here) {
      const RowSlot Sp = row_slot(d, b, d.t - 1);
      float lw, lk;
      const float p = prev_p_of(pv, rn, shifted, lw, lk);
      if (shifted) Sp.hlik[i] = lk;
      Sp.hp[i] = p;
      sf[0] = (double)p * p;
      sf[1] = (double)p * pv.x0;
      sf[2] = (double)p * pv.x1;
      sf[3] = lw;
    }
  }
  TRACE(1, 2)
  double *dst = ws.st_dyn + ((int64_t)b * tiles + tile) * 4;
  double *dfin = defer ? ws.fin + (((int64_t)b * d.T + d.t - 1) * tiles + tile) * 4 : nullptr;
  if (SPLIT)
    block_sum_roles_store(role ? sf : sd, dst, dfin, shd);
  else if (defer)
    block_sum8_store(sd, dst, sf, dfin, shd);
  else
    store_sums4(dst, sd[0], sd[1], sd[2], sd[3], shd);
  TRACE(1, 3)
}

// ---- K1+K2 merged (the split-net path of --NF-dyn RealNVP with --NF-cond and the cosine
// measurement; tiled_prop_split_kernel finishes the step).  The nf_dyn context is the row's
// mean / std of the particles AFTER motion, a row reduction that otherwise costs a launch
// boundary: here every workgroup of a row runs the gate, the resampling source selection and
// the motion of the WHOLE row (the motion is a Philox draw and two adds per particle; soft
// resampling already builds the row's CDF in every tile), reduces the row's x, x^2 sums
// itself (same inputs, same order in every workgroup of the row -> the same context) and then
// runs the nf_dyn inverse of its own 256 particles on wave pairs.  Slot t-1 is read only here;
// its deferred normalisation moves to the proposal launch (the scratch row is double-
// buffered by step parity, so step t's propose / prior do not overwrite step t-1's).
// Dynamic LDS: C[max(N, B_global)], w'[N], p_{t-1}[N].
template <bool FUSED>
__device__ __forceinline__ void fdyn_part(const nfdpf_filter_desc &d, const TiledWs &ws, FusedLds *fx,
                                          uint32_t tag) {
  extern __shared__ float dyn_lds[];
  __shared__ double shd[64];
  __shared__ float shf[16];
  __shared__ int fire_sh;
  __shared__ RowNorm rn_sh;
  __shared__ float xr_sh[kTile][2];
  __shared__ int src_sh[kTile];
  __shared__ float w_sh[kTile];
  __shared__ f2 cb[kMaxFlows * 2 * kH];
  __shared__ f2 cbs[kMaxFlows * 2 * kH];
  __shared__ __attribute__((aligned(8))) float xbuf[8 * kTile];
  __shared__ int xflag[16];
  TRACE(0, 0)
  const int tiles = n_tiles(d.N), N = d.N;
  int b, tile;
  tile_row(b, tile);
  const SplitLane sl = split_lane(8);
  const int role = sl.role, slot = sl.slot;
  const int i = tile * kTile + slot;
  const bool valid = i < N && (!FUSED || role < 2);  // fused: waves 8-15 carry no particle here
  const int64_t grow = d.row_base + b;
  const bool defer = d.defer_norm && d.t > 0;
  const bool shifted = shifted_meas(d.measurement);
  float *Cbuf = dyn_lds;
  if (threadIdx.x < 16) xflag[threadIdx.x] = 0;
  pair_clear(xbuf, kTile);
  float e0 = 0.f, e1 = 0.f;
  const int64_t my_row = ess_row(d, b);
  const RowSlot S = row_slot(d, b);
  const float *xprev = d.x_prev + b * d.x_prev_rs;
  const float *pprev = d.p_prev + b * d.p_prev_rs;
  const RowSlot Sp = defer ? row_slot(d, b, d.t - 1) : S;
  const float v0 = d.vel[2 * b], v1 = d.vel[2 * b + 1];
  const double *parts = reinterpret_cast<const double *>(d.ess_all);
  // Phase 1 is memory latency (the previous launch's outputs: ~2.4 us from the workgroup's start,
  // round-3 trace) plus Philox draws that depend on no load: every wave issues its loads first
  // and draws while they are in flight.  The gate wave's partials of rows lane (tiles <= 4, the
  // merged C2 path) are loaded into registers before anything else.
  const bool gate_wave = threadIdx.x < 64 && !d.gate && !d.force_resample;
  constexpr int kPreT = 4;
  double pre[kPreT * kSm];
  const bool pre_ok = gate_wave && tiles <= kPreT && (int)threadIdx.x < d.B_global;
  if (pre_ok) {
    gdouble *pr = (gdouble *)(parts + (int64_t)threadIdx.x * tiles * kSm);
#pragma unroll
    for (int k = 0; k < kPreT * kSm; ++k) pre[k] = pr[k < tiles * kSm ? k : 0];
  }
  // fold operands that depend on nothing computed in this launch, loaded now so their latency
  // hides under the gate / speculative motion: the nf_dyn fold's bias and context weights
  // (threads < n_flows*4*H) and, in tile 0, the proposal fold over the encoding columns
  // this thread's own particle of slot t-1 (the no-resample source), loaded up front too
  PrevIn pv{};
  float xp0 = 0.f, xp1 = 0.f, pp = 1.f;
  if (valid) {
    if (defer) {
      pv = load_prev_in(Sp, i);
    } else {
      xp0 = xprev[2 * i];
      xp1 = xprev[2 * i + 1];
      pp = pprev[i];
    }
  }
  const bool dyn_fold_lane = threadIdx.x < d.n_flows * 4 * kH;
  float fw[1 + kOctxDyn] = {};
  if (dyn_fold_lane) {
    const FoldRef r = fold_ref(d.dyn_params, kNsDyn, threadIdx.x);
    fw[0] = fold_bias0(r, kOctxDyn);
#pragma unroll
    for (int c = 0; c < kOctxDyn; ++c) fw[1 + c] = r.w1c[2 * (r.j * kOctxDyn + c) + r.w];
  }
  // fused: every workgroup folds for itself, on the otherwise idle waves 8-15
  const int enc_fold_t0 = FUSED ? 2 * kTile : kTile;
  const bool enc_fold_lane = d.nf_cond && (FUSED || tile == 0) && threadIdx.x >= enc_fold_t0 &&
                             threadIdx.x - enc_fold_t0 < d.n_flows * 4 * kH;
  float enc_fold = 0.f;
  if (enc_fold_lane) {  // proposal fold over the encoding columns (model/models.py:338-346); K3 adds mean/std
    const FoldRef r = fold_ref(d.cond_params, net_size<1, kH>(d.E + 4), threadIdx.x - enc_fold_t0);
    enc_fold = fold_acc_pipe(r, d.E + 4, fold_bias0(r, d.E + 4), S.enc, 0, d.E);
  }
  // the row's sums over x_phys = (x_src + vel) + eps (motion_apply_eps's arithmetic)
  double a0 = 0, a1 = 0, c0 = 0, c1 = 0;
  auto acc_n = [&](float xs0, float xs1, float n0, float n1) {
    const float p0 = (xs0 + v0) + n0, p1 = (xs1 + v1) + n1;
    a0 += p0;
    a1 += p1;
    c0 += (double)p0 * p0;
    c1 += (double)p1 * p1;
  };
  auto acc = [&](int j, float xs0, float xs1) {
    float n0, n1;
    motion_noise(d, b, grow, j, n0, n1);
    acc_n(xs0, xs1, n0, n1);
  };
  // The ESS gate (DPFs.py:163-165) is a chain of dependent loads and fp64 arithmetic on one
  // wave: wave 0 evaluates it (tiled_gate_block's arithmetic) while waves 1..7 run the
  // no-resampling motion of the row speculatively -- kept when the gate stays off (every
  // step of the C2 bench), recomputed from the resampled sources when it fires.
  const bool spec = !d.force_resample && !(d.gate && d.gate[0] != 0);
  if (threadIdx.x < 64) {
    if (valid) motion_noise(d, b, grow, i, e0, e1);  // under the partials' latency
    if (d.gate || d.force_resample) {
      if (threadIdx.x == 0) {
        fire_sh = d.gate ? d.gate[0] != 0 : 1;
        if (defer) rn_sh = row_norm(parts + my_row * tiles * kSm, tiles, shifted);
      }
    } else {
      for (int r = threadIdx.x; r < d.B_global; r += 64) {
        // rows < 64 from the registers loaded at the launch's start (the row normaliser of this
        // workgroup's own row too: no second round trip)
        if (pre_ok && r == (int)threadIdx.x) {
          // every lane evaluates its row's normaliser beside its 1 / sum p^2 (two independent
          // chains the compiler interleaves) and the lane of this workgroup's row keeps it --
          // instead of one lane's normaliser run after the batch's ESS terms, a divergent tail
          // on the gate wave's critical path (same arithmetic: bit-identical)
          const auto sm = [&](int k) { return pre[k]; };
          const float ie = row_inv_ess_t<kPreT>(sm, tiles, N, d.t > 0);
          RowNorm rn_lane{0.f, 1.f, 0.f};
          if (defer) rn_lane = row_norm_t<kPreT>(sm, tiles, shifted);
          Cbuf[r] = ie;
          if (defer && r == my_row) rn_sh = rn_lane;
        } else {
          const double *sm = parts + (int64_t)r * tiles * kSm;
          Cbuf[r] = row_inv_ess(sm, tiles, N, d.t > 0);
          if (defer && r == my_row) rn_sh = row_norm(sm, tiles, shifted);
        }
      }
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): this wave's LDS writes have landed
      __builtin_amdgcn_wave_barrier();
      TRACEW(0, 4)
      const float s = cascade_row_sum([&](int r) { return Cbuf[r]; }, d.B_global);
      if (threadIdx.x == 0) fire_sh = (s / (float)d.B_global) < 0.5f * (float)N;
      TRACEW(0, 5)
    }
  } else if (spec && (!FUSED || threadIdx.x < 2 * kTile)) {
    // every source load of this thread first (one memory latency instead of one per
    // particle), then the draws and sums; N <= kMergedMaxN = 4096 -> <= 10 per thread
    constexpr int kPer = 10;
    const float *src = defer ? Sp.hx : xprev;
    const int j0 = threadIdx.x - 64, js = 2 * kTile - 64;  // waves 1-7 (fused too: the same sums)
    float xs0[kPer], xs1[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int j = j0 + k * js;
      xs0[k] = j < N ? src[2 * j] : 0.f;
      xs1[k] = j < N ? src[2 * j + 1] : 0.f;
    }
    // the draws while the sources are in flight (they depend on no load), then the sums
    float n0[kPer], n1[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int j = j0 + k * js;
      n0[k] = n1[k] = 0.f;
      if (j < N) motion_noise(d, b, grow, j, n0[k], n1[k]);
    }
    if (valid) motion_noise(d, b, grow, i, e0, e1);
#ifdef NFDPF_EXP_TRACE
    if (threadIdx.x >> 6 == 1) {  // wave 1: draws done / its source loads landed
      TRACEW(0, 6)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#endif
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const int j = j0 + k * js;
      if (j < N) acc_n(xs0[k], xs1[k], n0[k], n1[k]);
    }
#ifdef NFDPF_EXP_TRACE
    if (threadIdx.x >> 6 == 1) TRACEW(0, 7)
#endif
  } else if (valid) {
    motion_noise(d, b, grow, i, e0, e1);
  }
  __syncthreads();
  const bool fire = fire_sh != 0;
  TRACE(0, 1)
  const int mode = !fire ? kSrcPrev : (d.resampler == NFDPF_RESAMPLE_SOFT ? kSrcSoft : kSrcOt);
  const RowNorm rn = defer ? rn_sh : RowNorm{0.f, 1.f, 0.f};
  auto prev_p = [&](int j) {
    float lw, lk;
    return norm_value(Sp, j, rn, shifted, lw, lk);
  };
  if (mode != kSrcPrev || !spec) a0 = a1 = c0 = c1 = 0;  // the speculation does not apply
  const int i0 = tile * kTile;
  float x0 = 0.f, x1 = 0.f, lr = 0.f;
  int src = i;
  if (mode == kSrcSoft) {
    float *wbuf = dyn_lds + max(N, d.B_global);
    if (defer) {  // the row's p_{t-1} into LDS for the resampler
      float *pbuf = wbuf + N;
      for (int j = threadIdx.x; j < N; j += blockDim.x) pbuf[j] = prev_p(j);
      __syncthreads();
      pprev = pbuf;
    }
    SoftRow row{pprev, N, d.alpha, 1.0f / (float)N, (float)(1.0 - (double)d.alpha), 1.0f};
    float off;
    if (d.rng_mode == NFDPF_RNG_HOST && d.host_offsets)
      off = d.host_offsets[b];
    else
      off = u01(rng_draw(d.seed, kTagOffset, (uint32_t)d.t, grow, 0u).x) * (1.0f / (float)N);
    soft_row_search(row, d.lin, off, Cbuf, shd, shf, [&](int j, int sj) {
      // sj == N: the reference's out-of-range edge (next row's first particle, weight 0)
      float w = 0.f;
      if (sj < N) w = row.w(sj);
      wbuf[j] = w;
      const float *xs = sj < N ? xprev + 2 * sj : (b + 1 < d.B ? xprev + d.x_prev_rs : xprev + 2 * (N - 1));
      const float xs0 = xs[0], xs1 = xs[1];
      acc(j, xs0, xs1);
      if (j >= i0 && j < i0 + kTile) {
        xr_sh[j - i0][0] = xs0;
        xr_sh[j - i0][1] = xs1;
        src_sh[j - i0] = sj;
        w_sh[j - i0] = w;
      }
    });
    __syncthreads();
    if (threadIdx.x < 64) {
      const float s2 = cascade_row_sum([&](int j) { return wbuf[j]; }, N);
      if (threadIdx.x == 0) shf[8] = s2;
    }
    __syncthreads();
    if (valid) {
      x0 = xr_sh[slot][0];
      x1 = xr_sh[slot][1];
      lr = logf(w_sh[slot] / shf[8]);
      src = src_sh[slot];
    }
  } else {
    if (mode == kSrcOt || !spec) {
      for (int j = threadIdx.x; j < N; j += blockDim.x) {
        if (mode == kSrcOt)
          acc(j, d.ot_x[((int64_t)b * N + j) * 2], d.ot_x[((int64_t)b * N + j) * 2 + 1]);
        else if (defer)
          acc(j, Sp.hx[2 * j], Sp.hx[2 * j + 1]);
        else
          acc(j, xprev[2 * j], xprev[2 * j + 1]);
      }
    }
    if (valid) {
      if (mode == kSrcOt) {
        x0 = d.ot_x[((int64_t)b * N + i) * 2];
        x1 = d.ot_x[((int64_t)b * N + i) * 2 + 1];
        lr = logf(1.0f / (float)N);
      } else if (defer) {
        float lw, lk;
        x0 = pv.x0;
        x1 = pv.x1;
        lr = logf(prev_p_of(pv, rn, shifted, lw, lk));
      } else {
        x0 = xp0;
        x1 = xp1;
        lr = logf(pp);
      }
    }
  }
  // the row context: wave sums (DPP), then the 8 wave partials in wave order, in every thread
  {
    double w4[4] = {a0, a1, c0, c1};
    const int w = threadIdx.x >> 6;
    // the fused step's waves 8-15 accumulated nothing unless they resampled: zeros, no DPP
    if (!FUSED || w < 8 || mode != kSrcPrev || !spec) wave_sum_dpp_n(w4);
    if ((threadIdx.x & 63) == 0)
#pragma unroll
      for (int k = 0; k < 4; ++k) shd[4 * w + k] = w4[k];
    __syncthreads();
    a0 = shd[0];
    a1 = shd[1];
    c0 = shd[2];
    c1 = shd[3];
    for (int q = 1; q < (int)(blockDim.x >> 6); ++q) {
      a0 += shd[4 * q];
      a1 += shd[4 * q + 1];
      c0 += shd[4 * q + 2];
      c1 += shd[4 * q + 3];
    }
  }
  const Ctx4 c = ctx_from_sums(a0, a1, c0, c1, N);
  if (dyn_fold_lane) {  // fold_one's fma sequence on the prefetched weights
    const float cv[4] = {c.m0, c.m1, c.s0, c.s1};
    float v = fw[0];
#pragma unroll
    for (int q = 0; q < kOctxDyn; ++q) v = fmaf(fw[1 + q], cv[q], v);
    reinterpret_cast<float *>(cb)[threadIdx.x] = v;
    reinterpret_cast<float *>(cbs)[split_cb_index(threadIdx.x)] = v;
    if (FUSED) fx->cb[threadIdx.x] = v;
  }
  if (enc_fold_lane) {
    if (FUSED)
      fx->encfold[threadIdx.x - enc_fold_t0] = enc_fold;
    else
      ws.cb_cond[b * kCb + threadIdx.x - kTile] = enc_fold;
  }
  __syncthreads();
  if (!FUSED && tile == 0 && threadIdx.x < d.n_flows * 4 * kH)  // K3's nf_dyn forward uses the same fold
    ws.cb_dyn[b * kCb + threadIdx.x] = reinterpret_cast<const float *>(cb)[threadIdx.x];
  TRACE(0, 2)
  double sd[4] = {0, 0, 0, 0};
  if (valid) {
    float p0, p1;
    if (role == 0) {
      motion_apply_eps(S, i, x0, x1, lr, v0, v1, e0, e1, p0, p1);
      S.hidx[i] = (int64_t)N * grow + (mode == kSrcSoft ? src : i);
    } else {
      p0 = (x0 + v0) + e0;
      p1 = (x1 + v1) + e1;
    }
    PairX x = pair_of(xbuf, xflag, role, slot);
    float xd0, xd1;
    stage_dyn_inverse_split(d, S, i, p0, p1, cbs, x, kTile, xd0, xd1);
    if (role == 0) {
      sd[0] = xd0;
      sd[1] = xd1;
      sd[2] = (double)xd0 * xd0;
      sd[3] = (double)xd1 * xd1;
    }
  }
  block_sum_roles_store(sd, ws.st_dyn + ((int64_t)b * tiles + tile) * 4, nullptr, shd,
                        FUSED ? ws.rowx + ((int64_t)b * tiles + tile) * 8 : nullptr, tag);
  TRACE(0, 3)
}

__global__ __launch_bounds__(2 * kTile) void tiled_fdyn_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  fdyn_part<false>(d, ws, nullptr, 0u);
}

// softmax partials of the unshifted log-weight u over this tile
__device__ __forceinline__ void store_softmax(float u, bool valid, double *sm, float *shf, double *shd) {
  // per wave (max, sum e^(u - max), sum e^(2(u - max))), merged over the waves with one
  // barrier into this tile's {max, sum, sum of squares} (sm[0..2])
  const float mw = wave_max_dpp(valid ? u : -INFINITY);
  const float ev = valid ? expf(u - mw) : 0.f;
  const double ew = wave_sum_dpp((double)ev);
  const double qw = wave_sum_dpp((double)ev * ev);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    shf[w] = mw;
    shd[2 * w] = ew;
    shd[2 * w + 1] = qw;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    float m = shf[0];
    for (int k = 1; k < nw; ++k) m = fmaxf(m, shf[k]);
    double sum = 0.0, sq = 0.0;
    for (int k = 0; k < nw; ++k)
      if (shf[k] > -INFINITY) {
        const double f = (double)expf(shf[k] - m);
        sum += shd[2 * k] * f;
        sq += shd[2 * k + 1] * f * f;
      }
    sm[0] = m;
    sm[1] = sum;
    sm[2] = sq;
  }
}

// store_softmax (role-0 lanes carry u) plus, with the same barrier, the four deferred-
// normalisation sums of the role-1 waves (block_sum_roles_store's order) into fin.
// smd >= 48 doubles.
__device__ __forceinline__ void store_softmax_fin(float u, bool valid, double *sm, const double (&sf)[4],
                                                  double *fin, float *shf, double *shd) {
  const float mw = wave_max_dpp(valid ? u : -INFINITY);
  const float ev = valid ? expf(u - mw) : 0.f;
  const double ew = wave_sum_dpp((double)ev);
  const double qw = wave_sum_dpp((double)ev * ev);
  double f4[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) f4[k] = wave_sum_dpp(sf[k]);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    shf[w] = mw;
    shd[2 * w] = ew;
    shd[2 * w + 1] = qw;
#pragma unroll
    for (int k = 0; k < 4; ++k) shd[16 + 4 * w + k] = f4[k];
  }
  __syncthreads();
  const int nw = (blockDim.x + 63) >> 6;
  if (threadIdx.x == 0) {
    float m = shf[0];
    for (int k = 1; k < nw; ++k) m = fmaxf(m, shf[k]);
    double sum = 0.0, sq = 0.0;
    for (int k = 0; k < nw; ++k)
      if (shf[k] > -INFINITY) {
        const double f = (double)expf(shf[k] - m);
        sum += shd[2 * k] * f;
        sq += shd[2 * k + 1] * f * f;
      }
    sm[0] = m;
    sm[1] = sum;
    sm[2] = sq;
  } else if (threadIdx.x >= 64 && threadIdx.x < 68) {  // role-1 waves 1, 3, 5, 7 in order
    const int k = threadIdx.x - 64;
    double a = shd[16 + 4 * 1 + k];
    for (int q = 1; q < 4; ++q) a += shd[16 + 4 * (2 * q + 1) + k];
    fin[k] = a;
  }
}

// ---- K3: proposal + measurement
// STAGE (CRNVP, use_stage, opt-in): the measurement's encoder and flow weights copied into LDS
// once per workgroup and read from there (ds_read) instead of streamed through the scalar cache
// (26 KB, more than it holds).  Measured slower: not the default.
// MV (CRNVP): 0 = the measurement per lane with its weights through the scalar cache, 1 = the
// same with the weights staged in LDS (STAGE), 2 = on f32 MFMA, 64 particles per wave with the
// fragment blob (d.meas_mfma, csrc/crnvp_mfma.hpp) staged in LDS -- the step launch of the C3
// shape when a gate fires (the no-flow pass reruns step by step with the Sinkhorn)
constexpr int kCrnvpPe = pe_size(kE);                                  // encoder floats
constexpr int kCrnvpFlow = 2 * 2 * net_size<kE / 2, kH>(kE);           // floats per flow
template <bool NFD, bool NFC, int MEAS, int MV = 0>
__global__ __launch_bounds__(kTile) void tiled_prop_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  constexpr bool STAGE = MV == 1, MF = MV == 2;
  static_assert(!MF || (MEAS == NFDPF_MEAS_CRNVP && !NFC), "MFMA measurement: CRNVP, bootstrap or nf_dyn proposal");
  __shared__ StepShared L;
  extern __shared__ float4 wstage[];  // STAGE: [encoder | flows] weights; MF: the fragment blob
  __shared__ float xw[MF ? kTile : 1][2];  // MF: the proposals, per wave, for its MFMA measurement
  TRACE(2, 0)
  const int tiles = n_tiles(d.N);
  int b, tile;
  tile_row(b, tile);
  const int i = tile * kTile + threadIdx.x;
  const RowSlot S = row_slot(d, b);
  const bool valid = i < d.N;
  PropIn in{};
  float lr = 0.f;
  if constexpr (STAGE) {  // 16-B aligned blobs, whole float4s (checked on the host)
    const float4 *pe4 = reinterpret_cast<const float4 *>(d.pe_params);
    const float4 *mp4 = reinterpret_cast<const float4 *>(d.meas_params);
    const int nmp4 = d.n_flows * kCrnvpFlow / 4;
    for (int k = threadIdx.x; k < kCrnvpPe / 4; k += kTile) wstage[k] = pe4[k];
    for (int k = threadIdx.x; k < nmp4; k += kTile) wstage[kCrnvpPe / 4 + k] = mp4[k];
  }
  if constexpr (MF) {  // 16-B aligned blob of whole float4s (checked on the host)
    const float4 *mp4 = reinterpret_cast<const float4 *>(d.meas_params);
    for (int k = threadIdx.x; k < crnvp_mfma_floats(d.n_flows) / 4; k += kTile) wstage[k] = mp4[k];
  }
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
  if (!NFD && d.defer_norm && d.t > 0)  // no K2 in this config
    finish_prev(d, ws, b, tile, i, true, i < d.N ? load_prev_in(row_slot(d, b, d.t - 1), i) : PrevIn{}, L.d);
  TRACE(2, 1)
  float lk = -INFINITY, u = 0.f;
  if constexpr (MF) {  // the proposal per lane, then the wave's 64 likelihoods on MFMA
    float q0x = 0.f, q1x = 0.f, propose = 0.f, prior = 0.f;
    if (valid) {
      const float jp = stage_propose_inverse<NFC>(d, in, L.cb_cond, q0x, q1x);
      stage_prior<NFD, NFC>(d, S, i, in, L.cb_dyn, q0x, q1x, jp, propose, prior);
    }
    xw[threadIdx.x][0] = q0x;
    xw[threadIdx.x][1] = q1x;
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const float r = crnvp_lik_mfma(reinterpret_cast<const float *>(wstage), d.n_flows, d.meas_prior_std, L.encv,
                                   &xw[threadIdx.x & ~63][0]);
    if (valid) {
      lk = r;
      S.hlik[i] = lk;
      u = logw(lr, lk, prior, propose);
    }
  } else if (valid) {
    float q0x, q1x, propose, prior;
    if constexpr (STAGE) {
      static_assert(!STAGE || MEAS == NFDPF_MEAS_CRNVP, "staged weights: CRNVP only");
      const float jp = stage_propose_inverse<NFC>(d, in, L.cb_cond, q0x, q1x);
      stage_prior<NFD, NFC>(d, S, i, in, L.cb_dyn, q0x, q1x, jp, propose, prior);
      const float *wl = reinterpret_cast<const float *>(wstage);
      lk = crnvp_lik(wl, wl + kCrnvpPe, d.n_flows, d.meas_prior_std, L.encv, q0x, q1x);
    } else {
      lk = stage_proposal<NFD, NFC, MEAS>(d, S, L, i, in, L.cb_dyn, L.cb_cond, q0x, q1x, propose, prior);
    }
    if (MEAS != NFDPF_MEAS_EXTERNAL) {
      S.hlik[i] = lk;
      u = logw(lr, lk, prior, propose);
    }
  }
  TRACE(2, 2)
  if (MEAS == NFDPF_MEAS_EXTERNAL) return;  // phase 1: the external likelihood comes next
  double *sm = reinterpret_cast<double *>(d.ess_out) + ((int64_t)b * tiles + tile) * kSm;
  const float lm = meas_shifted<MEAS>() ? block_max_dpp(lk, L.f) : 0.f;
  if (threadIdx.x == 0) sm[3] = lm;
  __shared__ double smd[48];
  store_softmax(u, valid, sm, L.f + 8, smd);  // L.f[0:8] held block_max
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
  __shared__ double ssx[ROLES][kTile], dotx[ROLES][kTile];
  __shared__ float smf[16];   // per-wave softmax partials (up to 12 waves)
  __shared__ double smd[48];
  TRACE(2, 0)
  const int tiles = n_tiles(d.N);
  int b, tile;
  tile_row(b, tile);
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
  if (!NFD && d.defer_norm && d.t > 0)  // no K2 in this config
    finish_prev(d, ws, b, tile, i, flows, flows && i < d.N ? load_prev_in(row_slot(d, b, d.t - 1), i) : PrevIn{},
                L.d);
  TRACE(2, 1)
  float q0x = 0.f, q1x = 0.f, jp = 0.f;
  if (flows && valid) {
    jp = stage_propose_inverse<NFC>(d, in, L.cb_cond, q0x, q1x);
    qx[pl][0] = q0x;
    qx[pl][1] = q1x;
  }
  __syncthreads();
  TRACE(2, 4)
  float lk = -INFINITY, u = 0.f, propose = 0.f, prior = 0.f;
  const int role = threadIdx.x / kTile;
  if (valid) {
    if (flows) {
      stage_prior<NFD, NFC>(d, S, i, in, L.cb_dyn, q0x, q1x, jp, propose, prior);
    } else if (ROLES == 3) {
      // cosine measurement, half of the encoder outputs per role (model/models.py:206-219)
      static_assert(ROLES != 3 || MEAS == NFDPF_MEAS_COS, "three roles: cosine measurement only");
      constexpr int HP = kE / 4;  // output pairs per role
      double ss, dot;
      encode_dot<kE, HP>(wptr(d.pe_params), qx[pl][0], qx[pl][1], L.encv, ss, dot, (role - 1) * HP);
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
    if constexpr (ROLES == 3) {
      lik = cos_lik(ssx[1][pl] + ssx[2][pl], dotx[1][pl] + dotx[2][pl], L.vinv);
      S.hlik[i] = lik;
    } else {
      lik = lx[pl];
    }
    u = logw(lr, lik, prior, propose);
  }
  TRACE(2, 2)
  double *sm = reinterpret_cast<double *>(d.ess_out) + ((int64_t)b * tiles + tile) * kSm;
  // the measurement waves hold lk, the others -inf
  const float lm = meas_shifted<MEAS>() ? block_max_dpp(lk, L.f) : 0.f;
  if (threadIdx.x == 0) sm[3] = lm;
  store_softmax(u, valid && flows, sm, smf, smd);
  TRACE(2, 3)
}

// ---- K3 for the conditional-RealNVP measurement without an NF proposal (C3, DPF-CM): 512
// threads per tile of 256 particles.  The measurement's flow input is the row's frame encoding
// and its condition the particle encoding (model/models.py:256-278), so a particle's work is two
// chains: waves 4-7 ("cond") encode the proposal and fold the encoding into every coupling
// half's first-layer bias pairs (the context columns of nf/flows.py:215-226's nets), publishing
// them half by half through LDS; waves 0-3 ("flow", the same particles as cond wave w + 4) take
// the densities while the encoder runs, then the coupling nets on the frame encoding as each
// half's biases arrive.  Two waves per SIMD instead of one at C3's 64 000 particles: one chain's
// scalar-load stalls are the other's issue slots.  The arithmetic is measure<CRNVP>'s, split at
// the fold (bit-identical).  Not the default: measured slower (use_cm).
static __host__ __device__ constexpr size_t cm_lds_bytes(int n_flows) {
  return (size_t)2 * n_flows * kH * kTile * sizeof(f2);
}
template <bool NFD>
__global__ __launch_bounds__(2 * kTile) void tiled_prop_cm_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  extern __shared__ f2 cbx[];  // [half h = 2 flow + n][kH][kTile] folded bias pairs
  __shared__ StepShared L;
  __shared__ int cflag[4];     // halves published by cond wave w + 4 (for flow wave w)
  __shared__ float smf[16];
  __shared__ double smd[48];
  TRACE(2, 0)
  constexpr int HALF = kE / 2;
  constexpr int ns = net_size<HALF, kH>(kE);
  const int tiles = n_tiles(d.N);
  int b, tile;
  tile_row(b, tile);
  const int pl = threadIdx.x & (kTile - 1);
  const bool flows = threadIdx.x < kTile;
  const int i = tile * kTile + pl;
  const RowSlot S = row_slot(d, b);
  const bool valid = i < d.N;
  PropIn in{};
  float lr = 0.f;
  if (valid) {  // issued before the row prologue so they overlap it
    if (flows) {
      in = load_prop_in<NFD>(S, i);
      lr = S.hp[i];
    } else {  // the proposal (= x_dyn without --NF-cond, stage_propose_inverse)
      in.xd0 = NFD ? S.scr[4 * i] : S.hx[2 * i];
      in.xd1 = NFD ? S.scr[4 * i + 1] : S.hx[2 * i + 1];
    }
  }
  measure_row_setup<NFDPF_MEAS_CRNVP>(S.enc, d.meas_params, L);
  if (threadIdx.x < 4) cflag[threadIdx.x] = 0;
  __syncthreads();
  if (!NFD && d.defer_norm && d.t > 0)  // no K2 in this config
    finish_prev(d, ws, b, tile, i, flows, flows && i < d.N ? load_prev_in(row_slot(d, b, d.t - 1), i) : PrevIn{},
                L.d);
  TRACE(2, 1)
  const int nh = 2 * d.n_flows;
  lds_vint *flag = (lds_vint *)&cflag[__builtin_amdgcn_readfirstlane(threadIdx.x >> 6) & 3];
  float lk = -INFINITY, u = 0.f;
  if (!flows) {
    float e[kE];
    particle_encode<kE>(wptr(d.pe_params), in.xd0, in.xd1, e);
    for (int h = 0; h < nh; ++h) {
      cf2 *fw = wptr2(d.meas_params) + h * ns;  // flow h / 2, coupling half h % 2
#pragma unroll
      for (int j = 0; j < kH; ++j) cbx[(h * kH + j) * kTile + pl] = fold_pair_c<HALF, kH, kE>(fw, j, e);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the pairs land before the count
      *flag = h + 1;
    }
  } else {
    float propose = 0.f, prior = 0.f;
    if (valid) stage_prior<NFD, false>(d, S, i, in, nullptr, in.xd0, in.xd1, 0.f, propose, prior);
    float lo[HALF], up[HALF];
#pragma unroll
    for (int k = 0; k < HALF; ++k) {
      lo[k] = L.encv[k];
      up[k] = L.encv[HALF + k];
    }
    float ld = 0.f;
    for (int f = 0; f < d.n_flows; ++f) {
      cf2 *fw = wptr2(d.meas_params) + f * 2 * ns;
      f2 cb[kH];
      float t[HALF], s[HALF];
      // coupling_forward, half by half as the cond wave publishes the bias pairs
      int it = 0;
      for (; __builtin_amdgcn_readfirstlane(*flag) < 2 * f + 1 && it < kSpinCap; ++it) __builtin_amdgcn_s_sleep(1);
      if (it == kSpinCap && (threadIdx.x & 63) == 0) atomicAdd(&g_split_fault, 1);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < kH; ++j) cb[j] = cbx[(2 * f * kH + j) * kTile + pl];
      ts_pair<HALF, kH>(fw, lo, cb, t, s);
#pragma unroll
      for (int k = 0; k < HALF; ++k) up[k] = t[k] + up[k] * expf(s[k]);
      const float l1 = half_sum<HALF>(s);
      it = 0;
      for (; __builtin_amdgcn_readfirstlane(*flag) < 2 * f + 2 && it < kSpinCap; ++it) __builtin_amdgcn_s_sleep(1);
      if (it == kSpinCap && (threadIdx.x & 63) == 0) atomicAdd(&g_split_fault, 1);
      asm volatile("" ::: "memory");
#pragma unroll
      for (int j = 0; j < kH; ++j) cb[j] = cbx[((2 * f + 1) * kH + j) * kTile + pl];
      ts_pair<HALF, kH>(fw + ns, up, cb, t, s);
#pragma unroll
      for (int k = 0; k < HALF; ++k) lo[k] = t[k] + lo[k] * expf(s[k]);
      ld += l1 + half_sum<HALF>(s);
    }
    // the prior's quadratic form in fp64, as measure<CRNVP>
    const double is = 1.0 / (double)d.meas_prior_std;
    double m = 0.0;
#pragma unroll
    for (int k = 0; k < HALF; ++k) {
      const double a = lo[k] * is, c = up[k] * is;
      m = fma(a, a, m);
      m = fma(c, c, m);
    }
    const double lp = -0.5 * (kE * 1.8378770664093453 + m) - kE * log((double)d.meas_prior_std);
    if (valid) {
      lk = (float)(lp + (double)ld);
      S.hlik[i] = lk;
      u = logw(lr, lk, prior, propose);
    }
  }
  TRACE(2, 2)
  double *sm = reinterpret_cast<double *>(d.ess_out) + ((int64_t)b * tiles + tile) * kSm;
  const float lm = block_max_dpp(lk, L.f);  // the cond waves hold -inf
  if (threadIdx.x == 0) sm[3] = lm;
  store_softmax(u, valid && flows, sm, smf, smd);
  TRACE(2, 3)
}

// ---- K3 on wave pairs (split.hpp; --NF-dyn RealNVP, --NF-cond, cosine measurement): the
// t-wave and the s-wave of a particle group run the proposal inverse and the nf_dyn forward
// net by net, then split the particle encoder's output layer (each computes the hidden
// layers, then half of the 32 outputs) and exchange their partial |e|^2 and <e, v>.  No
// wave idles and no workgroup barrier separates the stages.  512 threads per tile.
template <bool MERGED>
__global__ __launch_bounds__(2 * kTile) void tiled_prop_split_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  __shared__ StepShared L;  // cb_dyn / cb_cond in split order
  __shared__ __attribute__((aligned(8))) float xbuf[8 * kTile];
  __shared__ float hbuf[2 * kPeH2 / 2 * kTile];  // the encoder's hidden halves (encode_dot_pair)
  __shared__ float dbuf[2 * 4 * kTile];          // the fp64 cosine partials (pair_swap_once2)
  __shared__ int xflag[16];
  __shared__ float smf[16];
  __shared__ double smd[48];
  TRACE(2, 0)
  const int tiles = n_tiles(d.N);
  int b, tile;
  tile_row(b, tile);
  const SplitLane sl = split_lane(8);
  const int role = sl.role, slot = sl.slot;
  const int i = tile * kTile + slot;
  const RowSlot S = row_slot(d, b);
  const bool valid = i < d.N;
  PropIn in{};
  float lr = 0.f;
  // with the merged front + dyn launch, slot t-1's deferred normalisation runs here (role 1)
  const bool defer_here = MERGED && d.defer_norm && d.t > 0 && role == 1;
  PrevIn pv{};
  if (valid) {  // issued before the row prologue so they overlap it
    in = load_prop_in<true>(S, i);
    if (role == 0) lr = S.hp[i];
    if (defer_here) pv = load_prev_in(row_slot(d, b, d.t - 1), i);
  }
  // slot t-1's row normaliser (softmax partials of the previous launch): read now, so its
  // global latency hides under the prologue instead of the epilogue
  const RowNorm rn_prev = defer_here && valid ? row_norm(prev_sm(d, b, tiles), tiles, shifted_meas(d.measurement))
                                              : RowNorm{0.f, 1.f, 0.f};
  measure_row_setup<NFDPF_MEAS_COS>(S.enc, d.meas_params, L);
  if (threadIdx.x < 16) xflag[threadIdx.x] = 0;
  pair_clear(xbuf, kTile);
  const int ncb = d.n_flows * 4 * kH;
  if (threadIdx.x < ncb)
    reinterpret_cast<float *>(L.cb_dyn)[split_cb_index(threadIdx.x)] = ws.cb_dyn[b * kCb + threadIdx.x];
  if (threadIdx.x >= kTile && threadIdx.x - kTile < ncb) {
    // finish the proposal fold: the encoding columns came from K1, add [mean, std] of x_dyn
    const int k = threadIdx.x - kTile;
    const Ctx4 cp = tiled_ctx(ws.st_dyn, b, tiles, d.N);
    const float c4[4] = {cp.m0, cp.m1, cp.s0, cp.s1};
    const FoldRef r = fold_ref(d.cond_params, net_size<1, kH>(d.E + 4), k);
    reinterpret_cast<float *>(L.cb_cond)[split_cb_index(k)] =
        fold_acc(r, d.E + 4, ws.cb_cond[b * kCb + k], c4, d.E, d.E + 4);
  }
  __syncthreads();
  TRACE(2, 1)
  PairX x = pair_of(xbuf, xflag, role, slot);
  float u = 0.f;
  if (valid) {
    float q0x, q1x, propose, prior;
    const float jp = stage_propose_inverse_split(d, in, L.cb_cond, x, kTile, q0x, q1x);
    stage_prior_split(d, S, i, in, L.cb_dyn, q0x, q1x, jp, x, kTile, propose, prior);
    // cosine measurement (model/models.py:206-219): outputs [16 role, 16 role + 16) here
    double ss, dot;
    double ss_o, dot_o;
#ifdef NFDPF_EXP_NOENC  // experiment builds only: the cosine encoder left out (prices it)
    ss = 1.0 + q0x * 1e-9, dot = 0.5 + q1x * 1e-9, ss_o = 1.0, dot_o = 0.25;
#else
    encode_dot_pair<kE>(wptr(d.pe_params), q0x, q1x, L.encv, ss, dot, x, hbuf, kTile);
    pair_swap_once2(x, ss, dot, dbuf, kTile, ss_o, dot_o);
#endif
    ss = role ? ss_o + ss : ss + ss_o;
    dot = role ? dot_o + dot : dot + dot_o;
    const float lk = cos_lik(ss, dot, L.vinv);
    if (role == 0) {
      S.hlik[i] = lk;
      u = logw(lr, lk, prior, propose);
    }
  }
  TRACE(2, 2)
  double *sm = reinterpret_cast<double *>(d.ess_out) + ((int64_t)b * tiles + tile) * kSm;
  if (threadIdx.x == 0) sm[3] = 0.f;
  if (MERGED && d.defer_norm && d.t > 0) {
    // finish_prev's arithmetic for slot t-1 on role 1; its four sums and this step's softmax
    // partials share one barrier
    double sf[4] = {0, 0, 0, 0};
    if (defer_here && valid) {
      const bool shifted = shifted_meas(d.measurement);
      const RowSlot Sp = row_slot(d, b, d.t - 1);
      float lw, lk;
      const float p = prev_p_of(pv, rn_prev, shifted, lw, lk);
      if (shifted) Sp.hlik[i] = lk;
      Sp.hp[i] = p;
      sf[0] = (double)p * p;
      sf[1] = (double)p * pv.x0;
      sf[2] = (double)p * pv.x1;
      sf[3] = lw;
    }
    store_softmax_fin(u, valid && role == 0, sm, sf, ws.fin + (((int64_t)b * d.T + d.t - 1) * tiles + tile) * 4,
                      smf, smd);
  } else {
    store_softmax(u, valid && role == 0, sm, smf, smd);
  }
  TRACE(2, 3)
}

// The quad launch's softmax / deferred-normalisation partials: the encoder t-waves 8, 10, 12,
// 14 (groups 0-3) carry u and the slot t-1 sums and leave their wave partials in LDS before
// the launch's one closing barrier (wave_partials_quad); after it thread 0 merges the tile's
// {max, sum e, sum e^2} and threads 64-67 the four sums -- the same lanes, values and
// summation order as the split launch's (u on waves 0, 2, 4, 6, sums on 1, 3, 5, 7).
// shf >= 16 floats, shd >= 96 doubles.
__device__ __forceinline__ void wave_partials_quad(float u, bool valid, bool carry, const double (&sf)[4],
                                                   float *shf, double *shd) {
  const int w = threadIdx.x >> 6;
  if (!carry) {  // wave-uniform: this wave holds no partials
    if ((threadIdx.x & 63) == 0) shf[w] = -INFINITY;
    return;
  }
  const float mw = wave_max_dpp(valid ? u : -INFINITY);
  const float ev = valid ? expf(u - mw) : 0.f;
  double r[6] = {(double)ev, (double)ev * ev, sf[0], sf[1], sf[2], sf[3]};
  wave_sum_dpp_n(r);
  if ((threadIdx.x & 63) == 0) {
    shf[w] = mw;
    shd[2 * w] = r[0];
    shd[2 * w + 1] = r[1];
#pragma unroll
    for (int k = 0; k < 4; ++k) shd[32 + 4 * w + k] = r[2 + k];
  }
}
// after the barrier
__device__ __forceinline__ void merge_partials_quad(double *sm, double *fin, const float *shf, const double *shd) {
  if (threadIdx.x == 0) {
    float m = shf[0];
    for (int k = 1; k < 16; ++k) m = fmaxf(m, shf[k]);
    double sum = 0.0, sq = 0.0;
    for (int k = 0; k < 16; ++k)
      if (shf[k] > -INFINITY) {
        const double f = (double)expf(shf[k] - m);
        sum += shd[2 * k] * f;
        sq += shd[2 * k + 1] * f * f;
      }
    sm[0] = m;
    sm[1] = sum;
    sm[2] = sq;
    sm[3] = 0.0;
  } else if (fin && threadIdx.x >= 64 && threadIdx.x < 68) {  // encoder t-waves 8, 10, 12, 14 in order
    const int k = threadIdx.x - 64;
    double a = shd[32 + 4 * 8 + k];
    for (int q = 1; q < 4; ++q) a += shd[32 + 4 * (8 + 2 * q) + k];
    fin[k] = a;
  }
}

// ---- K3 on wave quads (--NF-dyn RealNVP, --NF-cond, cosine measurement): per particle group
// of 64, a flow pair (waves 2g, 2g + 1: the t- and s-nets of the proposal inverse, then of the
// nf_dyn forward, split.hpp) and an encoder pair (waves 8 + 2g, 9 + 2g: the particle encoder
// split over two waves, encode_dot_pair).  The measurement needs only the proposal
// (model/models.py:358-377), so the encoder pair takes it from the flow t-wave through LDS and
// runs BESIDE the nf_dyn forward: the launch costs proposal + max(nf_dyn forward, encoder)
// instead of their sum, at four waves per SIMD.  While it waits for the proposal the encoder
// t-wave normalises slot t-1's particles (the deferred normalisation).  1024 threads per tile.
template <bool MERGED, bool FUSED>
__device__ __forceinline__ void quad_part(const nfdpf_filter_desc &d, const TiledWs &ws, const FusedLds *fx) {
  __shared__ StepShared L;
  __shared__ __attribute__((aligned(8))) float xbuf[8 * kTile];              // flow-pair hand-offs (pair_swap)
#ifdef NFDPF_ENC_VALU
  __shared__ float hbuf[2 * kPeH2 / 2 * kTile];  // encoder hidden halves (encode_dot_pair)
  __shared__ float dbuf[2 * 4 * kTile];          // fp64 cosine partials (pair_swap_once2)
#else
  __shared__ float Hws[8][32 * kHPitch];         // each encoder wave's layer-2 / layer-3 outputs
#endif
  __shared__ float qbuf[2 * kTile];              // the proposal, flow t-wave -> encoder pair
  __shared__ float rbuf[3 * kTile];              // likelihood | prior | propose per particle
  __shared__ float encq[8][kE];                  // each encoder wave's copy of the frame encoding
  __shared__ int xflag[16];
  __shared__ int qflag[4];
  __shared__ int rflag[4];
  __shared__ float smf[16];
  __shared__ double smd[96];
  TRACE(2, 0)
  QTRACE(0)
  const int tiles = n_tiles(d.N);
  int b, tile;
  tile_row(b, tile);
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool enc = w >= 8;
  const int role = w & 1, g = (w >> 1) & 3;
  const int slot = g * 64 + (threadIdx.x & 63);
  const int i = tile * kTile + slot;
  const RowSlot S = row_slot(d, b);
  const bool valid = i < d.N;
  PropIn in{};
  float lr = 0.f;
  // with the merged front + dyn launch, slot t-1's deferred normalisation runs here (encoder t-wave)
  const bool defer_here = MERGED && d.defer_norm && d.t > 0 && enc && role == 0;
  PrevIn pv{};
#ifndef NFDPF_ENC_VALU
  EncFrag2 ef{};
  if (enc) ef = enc_frag2_load(d.pe_params);  // the encoder's weight fragments, once
  // an encoder wave's measured particles: lanes 0-31 <- particles [32 role, 32 role + 32) of the group
  const int slot_e = g * 64 + 32 * role + (threadIdx.x & 31), i_e = tile * kTile + slot_e;
  const bool valid_e = enc && (threadIdx.x & 63) < 32 && i_e < d.N;
#else
  const int slot_e = slot, i_e = i;
  const bool valid_e = enc && role == 0 && valid;
#endif
  if (valid) {  // issued before the row prologue so they overlap it
    if (!enc) in = load_prop_in<true>(S, i);
    if (defer_here) pv = load_prev_in(row_slot(d, b, d.t - 1), i);
  }
  if (valid_e) lr = S.hp[i_e];
  // the encoder waves' row constants (the frame encoding, slot t-1's normaliser) are read after
  // the prologue barrier: they are needed only once the proposal has arrived
  if (threadIdx.x < 16) xflag[threadIdx.x] = 0;
  pair_clear(xbuf, kTile);
  if (threadIdx.x < 4) qflag[threadIdx.x] = 0;
  if (threadIdx.x >= 4 && threadIdx.x < 8) rflag[threadIdx.x - 4] = 0;
  const int ncb = d.n_flows * 4 * kH;
  if (threadIdx.x < ncb)
    reinterpret_cast<float *>(L.cb_dyn)[split_cb_index(threadIdx.x)] =
        FUSED ? fx->cb[threadIdx.x] : ws.cb_dyn[b * kCb + threadIdx.x];
  if (threadIdx.x >= kTile && threadIdx.x - kTile < ncb) {
    // finish the proposal fold: the encoding columns came from K1, add [mean, std] of x_dyn
    const int k = threadIdx.x - kTile;
    const Ctx4 cp = FUSED ? tiled_ctx(fx->rowst, 0, tiles, d.N) : tiled_ctx(ws.st_dyn, b, tiles, d.N);
    const float c4[4] = {cp.m0, cp.m1, cp.s0, cp.s1};
    const FoldRef r = fold_ref(d.cond_params, net_size<1, kH>(d.E + 4), k);
    reinterpret_cast<float *>(L.cb_cond)[split_cb_index(k)] =
        fold_acc(r, d.E + 4, FUSED ? fx->encfold[k] : ws.cb_cond[b * kCb + k], c4, d.E, d.E + 4);
  }
  __syncthreads();
  TRACE(2, 1)
  QTRACE(1)
  double sf[4] = {0, 0, 0, 0};
  float u = 0.f;
  lds_vint *qf = (lds_vint *)(qflag + g), *rf = (lds_vint *)(rflag + g);
  if (!enc) {
    PairX x = pair_of(xbuf, xflag, role, slot);
    float q0x = 0.f, q1x = 0.f, jp = 0.f;
    if (valid) {
      jp = stage_propose_inverse_split(d, in, L.cb_cond, x, kTile, q0x, q1x);
      if (role == 0) {
        qbuf[slot] = q0x;
        qbuf[kTile + slot] = q1x;
      }
    }
    if (role == 0) {  // publish the proposal to the encoder pair (values land first)
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      *qf = 1;
    }
    QTRACE(2)
    if (valid) {
      float propose, prior;
      stage_prior_split(d, S, i, in, L.cb_dyn, q0x, q1x, jp, x, kTile, propose, prior);
      if (role == 0) {
        rbuf[kTile + slot] = prior;
        rbuf[2 * kTile + slot] = propose;
      }
    }
    if (role == 0) {  // publish prior / propose to the encoder t-wave
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      *rf = 1;
    }
    QTRACE(3)
  } else {
    // measure_row_setup (cosine), per encoder wave into its own LDS copy (no barrier needed)
    const int lane = threadIdx.x & 63;
    float *encv = encq[w - 8];
    const float ve = lane < kE ? S.enc[lane] : 0.f;
    const double vinv = 1.0 / fmax(sqrt(wave_sum((double)ve * ve)), 1e-12);
    if (lane < kE) encv[lane] = ve;
    __builtin_amdgcn_wave_barrier();
    asm volatile("" ::: "memory");
    const RowNorm rn_prev = defer_here && valid ? row_norm(prev_sm(d, b, tiles), tiles, shifted_meas(d.measurement))
                                                : RowNorm{0.f, 1.f, 0.f};
    if (defer_here && valid) {  // finish_prev's arithmetic for slot t-1 while the proposal runs
      const bool shifted = shifted_meas(d.measurement);
      const RowSlot Sp = row_slot(d, b, d.t - 1);
      float lw, lk;
      const float p = prev_p_of(pv, rn_prev, shifted, lw, lk);
      if (shifted) Sp.hlik[i] = lk;
      Sp.hp[i] = p;
      sf[0] = (double)p * p;
      sf[1] = (double)p * pv.x0;
      sf[2] = (double)p * pv.x1;
      sf[3] = lw;
    }
    // valid lanes are a prefix of the wave: it has work iff its first lane has
    if (tile * kTile + g * 64 < d.N) {
      int it = 0;
      for (; __builtin_amdgcn_readfirstlane(*qf) == 0 && it < kSpinCap; ++it) __builtin_amdgcn_s_sleep(1);
      if (it == kSpinCap && (threadIdx.x & 63) == 0) atomicAdd(&g_split_fault, 1);
      asm volatile("" ::: "memory");
      QTRACE(2)
      // cosine measurement (model/models.py:206-219)
      double ss, dot;
#ifdef NFDPF_ENC_VALU  // the pair splits the outputs: [16 role, 16 role + 16) here, then exchanges
      PairX xe = pair_of(xbuf, xflag, role, slot);  // flags 8..15: the encoder pairs' own
      double ss_o, dot_o;
      encode_dot_pair<kE>(wptr(d.pe_params), qbuf[slot], qbuf[kTile + slot], encv, ss, dot, xe, hbuf, kTile);
      pair_swap_once2(xe, ss, dot, dbuf, kTile, ss_o, dot_o);
      ss = role ? ss_o + ss : ss + ss_o;
      dot = role ? dot_o + dot : dot + dot_o;
#else  // the pair splits the particles: no hand-off
      encode_dot_mfma_half<kE>(ef, role, qbuf + g * 64, qbuf + kTile + g * 64, encv, ss, dot, Hws[w - 8]);
#endif
      QTRACE(11)
      const float lk = cos_lik(ss, dot, vinv);
      if (valid_e) {
        S.hlik[i_e] = lk;
        // the log-weight (DPFs.py:187) once the flow t-wave has left prior / propose
        int it2 = 0;
        for (; __builtin_amdgcn_readfirstlane(*rf) == 0 && it2 < kSpinCap; ++it2) __builtin_amdgcn_s_sleep(1);
        if (it2 == kSpinCap && (threadIdx.x & 63) == 0) atomicAdd(&g_split_fault, 1);
        asm volatile("" ::: "memory");
        u = logw(lr, lk, rbuf[kTile + slot_e], rbuf[2 * kTile + slot_e]);
      }
    }
    QTRACE(3)
  }
  // the encoder waves' softmax and slot t-1 partials, then the launch's one closing barrier
#ifdef NFDPF_ENC_VALU
  wave_partials_quad(u, valid_e, enc && role == 0, sf, smf, smd);
#else
  wave_partials_quad(u, valid_e, enc, sf, smf, smd);
#endif
  __syncthreads();
  TRACE(2, 2)
  QTRACE(4)
  double *sm = reinterpret_cast<double *>(d.ess_out) + ((int64_t)b * tiles + tile) * kSm;
  const bool fin = MERGED && d.defer_norm && d.t > 0;
  merge_partials_quad(sm, fin ? ws.fin + (((int64_t)b * d.T + d.t - 1) * tiles + tile) * 4 : nullptr, smf, smd);
  TRACE(2, 3)
  QTRACE(5)
}

template <bool MERGED>
__global__ __launch_bounds__(4 * kTile) void tiled_prop_quad_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  quad_part<MERGED, false>(d, ws, nullptr);
}

// ---- the fused step: front + nf_dyn inverse (fdyn_part), the row's x_dyn exchange
// (row_sync), proposal + nf_dyn forward + cosine measurement (quad_part) -- one launch
__global__ __launch_bounds__(4 * kTile) void tiled_step_fused_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  __shared__ FusedLds fx;
  const uint32_t tag = (g_step_epoch << 16) + (uint32_t)d.t + 1u;
  fdyn_part<true>(d, ws, &fx, tag);
  TRACE(1, 0)
  row_sync(d, ws, &fx, tag);
  TRACE(1, 3)
  quad_part<true, true>(d, ws, &fx);
}
__global__ void tiled_epoch_kernel() { g_step_epoch = g_step_epoch + 1u; }

// ---- K3b (phase 2 of an EXTERNAL measurement): raw likelihood from lik_ext
__global__ __launch_bounds__(kTile) void tiled_extlik_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  __shared__ double shd2[32];
  __shared__ float shf[16];
  const int tiles = n_tiles(d.N);
  int b, tile;
  tile_row(b, tile);
  const int i = tile * kTile + threadIdx.x;
  const RowSlot S = row_slot(d, b);
  const bool valid = i < d.N;
  float lk = -INFINITY, u = 0.f;
  if (valid) {
    lk = d.lik_ext[(int64_t)b * d.N + i];
    S.hlik[i] = lk;
    u = stage_logw(S, i, lk);
  }
  double *sm = reinterpret_cast<double *>(d.ess_out) + ((int64_t)b * tiles + tile) * kSm;
  const float m = block_max_dpp(lk, shf);
  if (threadIdx.x == 0) sm[3] = m;
  store_softmax(u, valid, sm, shf + 8, shd2);  // shf[0:8] held block_max
}

// ---- K4: log-weights, normalisation, per-tile sums for the prediction / obs-likelihood, for
// the step's own slot (every step with OT or a caller-fed p_prev; otherwise only after the
// last step -- the front kernel of the next step does it, see tiled_front_kernel)
template <bool SHIFT>
__global__ __launch_bounds__(kTile) void tiled_norm_kernel(const nfdpf_filter_desc d, TiledWs ws) {
  TRACE(3, 0)
  __shared__ double shd[16];
  const int tiles = n_tiles(d.N);
  int b, tile;
  tile_row(b, tile);
  const int i = tile * kTile + threadIdx.x;
  const RowNorm rn = row_norm(reinterpret_cast<const double *>(d.ess_out) + (int64_t)b * tiles * kSm, tiles, SHIFT);
  const RowSlot S = row_slot(d, b);
  double sp2 = 0, px = 0, py = 0, sw = 0;
  if (i < d.N) {
    float lw;
    const float p = norm_particle(S, i, rn, SHIFT, lw);
    sp2 = (double)p * p;
    px = (double)p * S.hx[2 * i];
    py = (double)p * S.hx[2 * i + 1];
    sw = lw;
  }
  double *fin = ws.fin + (((int64_t)b * d.T + d.t) * tiles + tile) * 4;
  TRACE(3, 2)
  store_sums4(fin, sp2, px, py, sw, shd);
  TRACE(3, 3)
}

// per-row prediction / obs-likelihood sums of every step (after the last step)
// (entries read 8 at a time so the loads overlap, the rest one by one; added in entry order:
// `tiles` entries per (row, step) -- n_tiles for the step launches, n_tiles * 8 for the pass)
__global__ void tiled_finalize_kernel(const double *__restrict__ fin, int BT, int tiles,
                                      float *__restrict__ pred, float *__restrict__ lw_sum) {
  const int bt = blockIdx.x * blockDim.x + threadIdx.x;
  if (bt >= BT) return;
  double px = 0, py = 0, sw = 0;
  int k0 = 0;
  for (; k0 + 8 <= tiles; k0 += 8) {
    double a[8][3];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const double *f = fin + ((int64_t)bt * tiles + k0 + j) * 4;
      a[j][0] = f[1];
      a[j][1] = f[2];
      a[j][2] = f[3];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      px += a[j][0];
      py += a[j][1];
      sw += a[j][2];
    }
  }
  for (; k0 < tiles; ++k0) {
    const double *f = fin + ((int64_t)bt * tiles + k0) * 4;
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
  int b, tile;
  tile_row(b, tile);
  const int i = tile * kTile + threadIdx.x;
  double v = 0.0;
  if (i < N) {
    const float x = p[(int64_t)b * N + i];
    v = (double)x * x;
  }
  v = block_sum(v, shd);
  if (threadIdx.x == 0) {
    // partials of p0 itself: max 0, sum 1 (tile 0 only), sum p0^2 -> row_inv_ess = 1/sum p0^2
    double *sm = parts + ((int64_t)b * tiles + tile) * kSm;
    sm[0] = 0.0;
    sm[1] = tile == 0 ? 1.0 : 0.0;
    sm[2] = v;
    sm[3] = 0.0;
  }
}

// particle_initialization (utils.py:46-62, device RNG) + p0 = normalize_log_probs (DPFs.py:153) +
// the t = 0 gate's per-tile partials, one workgroup per row (N <= 1024, one particle per thread):
// particle_init_kernel's, normalize_kernel's and tiled_ess_init_kernel's arithmetic in their
// orders (the same bits) in one launch instead of three.  The tile sums reuse the wave sums of
// normalize's sum p^2 (a tile is waves 4k..4k+3, summed in order as block_sum sums a tile's).
// Also every step's velocity in the [T][B][2] layout the step and pass launches read: the start
// velocity, then vel_in[:, t - 1] (DPFs.py:158, 173).
__global__ __launch_bounds__(1024) void filter_init_kernel(const float *__restrict__ start, int start_rs,
                                                           const float *__restrict__ vel_in, int vel_rs, int T,
                                                           int N, float width, int true_state, uint64_t seed,
                                                           int64_t row_base, float *__restrict__ x,
                                                           float *__restrict__ logw, float *__restrict__ p,
                                                           float *__restrict__ inv_ess, double *__restrict__ parts,
                                                           float *__restrict__ vel) {
  __shared__ float shf[16];
  __shared__ double shd[16];
  const int b = blockIdx.x, i = threadIdx.x;
  if (vel)
    for (int k = i; k < 2 * T; k += blockDim.x) {
      const int t = k >> 1, c = k & 1;
      vel[((int64_t)t * gridDim.x + b) * 2 + c] =
          t == 0 ? start[(int64_t)b * start_rs + 2 + c] : vel_in[(int64_t)b * vel_rs + 2 * (t - 1) + c];
    }
  const bool valid = i < N;
  const int64_t o = (int64_t)b * N + i;
  float lw = -INFINITY;
  if (valid) {
    const int64_t grow = row_base + b;
    float a0, a1;
    if (true_state) {
      const U4 r = rng_draw(seed, kTagInitNormal, 0u, grow, (uint32_t)i);
      box_muller(r.x, r.y, a0, a1);
      a0 += start[(int64_t)b * start_rs];
      a1 += start[(int64_t)b * start_rs + 1];
    } else {
      const U4 r = rng_draw(seed, kTagInitPos, 0u, grow, (uint32_t)i);
      const float hi = width / 2.0f, lo = -width / 2.0f;
      a0 = (hi - lo) * u01(r.x) + lo;
      a1 = (hi - lo) * u01(r.y) + lo;
    }
    x[2 * o] = a0;
    x[2 * o + 1] = a1;
    lw = logf(1.0f / (float)N);
    logw[o] = lw;
  }
  const float m = block_max(lw, shf);
  const float S = (float)block_sum(valid ? (double)expf(lw - m) : 0.0, shd);
  float v = 0.f;
  if (valid) {
    v = expf(lw - m) / S + 0.0f;
    p[o] = v;
  }
  const double w2 = wave_sum(valid ? (double)v * (double)v : 0.0);
  __syncthreads();
  if ((i & 63) == 0) shd[i >> 6] = w2;
  __syncthreads();
  const int nw = (blockDim.x + 63) >> 6, tiles = n_tiles(N);
  if (i == 0 && inv_ess) {
    double r = shd[0];
    for (int k = 1; k < nw; ++k) r += shd[k];
    inv_ess[b] = 1.0f / (float)r;
  }
  if (i < tiles) {
    const int w0 = 4 * i;
    double r = shd[w0];
    for (int k = w0 + 1; k < w0 + 4 && k < nw; ++k) r += shd[k];
    double *sm = parts + ((int64_t)b * tiles + i) * kSm;
    sm[0] = 0.0;
    sm[1] = i == 0 ? 1.0 : 0.0;
    sm[2] = r;
    sm[3] = 0.0;
  }
}

__global__ void tiled_gate_kernel(const double *__restrict__ parts, int B, int tiles, int N, int t, int force,
                                  int32_t *gate) {
  const float s = cascade_row_sum([&](int r) { return row_inv_ess(parts + (int64_t)r * tiles * kSm, tiles, N, t > 0); },
                                  force ? 0 : B);
  if (threadIdx.x == 0) gate[0] = (force || (s / (float)B) < 0.5f * (float)N) ? 1 : 0;
}

// the same for T steps, one wave each (block = step)
__global__ void tiled_gate_batch_kernel(const double *__restrict__ parts, int B, int tiles, int N, int t0,
                                        int force, int32_t *gates) {
  const int k = blockIdx.x;
  const double *p = parts + (int64_t)k * B * tiles * kSm;
  const float s = cascade_row_sum([&](int r) { return row_inv_ess(p + (int64_t)r * tiles * kSm, tiles, N, t0 + k > 0); },
                                  force ? 0 : B);
  if (threadIdx.x == 0) gates[k] = (force || (s / (float)B) < 0.5f * (float)N) ? 1 : 0;
}

// The verification of a speculative pass, stream-ordered and capturable (the host then reads
// one word pair instead of synchronising for the fault counter and again for the gates): the T
// gates by tiled_gate_batch_kernel, then this one-wave launch -- the number that fired, the
// hand-off fault counter (read and cleared) and the obs-likelihood sum_t (sum_b lw[b, t]) / (B N)
// (DPFs.py:191; fp64 in row order per step, then step order) from the pass's lw_sum [B][T].
__global__ __launch_bounds__(64) void tiled_verify_flags_kernel(const int32_t *__restrict__ gates,
                                                                const float *__restrict__ lw_sum, int T, int B,
                                                                double BN, int32_t *flags, float *obs) {
  const int l = threadIdx.x;
  int f = 0;
  for (int k = l; k < T; k += 64) f += gates[k];
  for (int o = 32; o >= 1; o >>= 1) f += __shfl_xor(f, o);
  double acc = 0.0;  // lane 0 adds the steps in order; lanes hold the step sums of 64 steps at a time
  for (int t0 = 0; t0 < T; t0 += 64) {
    const int t = t0 + l;
    double tot = 0.0;
    if (t < T)
      for (int b = 0; b < B; ++b) tot += (double)lw_sum[(int64_t)b * T + t];
    const double q = tot / BN;
    for (int k = 0; k < 64 && t0 + k < T; ++k) acc += readlane_d(q, k);
  }
  if (l == 0) {
    flags[0] = f;
    flags[1] = atomicExch(&g_split_fault, 0);
    obs[0] = (float)acc;
  }
}

// the flows run on wave pairs when the blobs carry the split suffix (RealNVP nf_dyn)
static bool use_split(const nfdpf_filter_desc &d) { return d.split_nets && d.nf_dyn == NFDPF_DYN_REALNVP; }
// front + dyn in one launch (tiled_fdyn_kernel), the deferred normalisation in the proposal
// launch: the split-net path with the cosine measurement, rows short enough for LDS
constexpr int kMergedMaxN = kMergedMaxN_;
static bool use_merged(const nfdpf_filter_desc &d) {
  return use_split(d) && d.nf_cond && d.measurement == NFDPF_MEAS_COS && d.N <= kMergedMaxN &&
         d.B_global <= kMergedMaxN;
}

// Rows longer than this (soft resampler, not the merged path) take the gate, the deferred row
// normaliser and the row's resampling from tiled_rows_kernel, once per row.
// (NFDPF_TILED_ROWS_MIN_N overrides the threshold, read per call: tests compare both paths.)
constexpr int kRowsMinN = 1024;
static bool use_rows(const nfdpf_filter_desc &d) {
  const char *e = getenv("NFDPF_TILED_ROWS_MIN_N");
  const int min_n = e ? atoi(e) : kRowsMinN;
  return d.resampler == NFDPF_RESAMPLE_SOFT && !use_merged(d) && d.N > min_n;
}

// CRNVP weights staged in LDS per workgroup (tiled_prop_kernel<..., true>), opt-in with
// NFDPF_CRNVP_STAGE=1 (read per call: tests compare both): 16-B aligned blobs and at most
// kMaxFlows flows (<= 58 KB).  Measured SLOWER than the scalar-cache stream at C3 (48 vs 31 us
// per launch, 1.11e9 vs 1.58e9; one ds_read_b128 per two v_pk_fma, 254 VGPRs leave the
// compiler two or three reads in flight).
static bool use_stage(const nfdpf_filter_desc &d) {
  const char *e = getenv("NFDPF_CRNVP_STAGE");
  if (!(e && e[0] == '1')) return false;
  return d.n_flows >= 0 && d.n_flows <= kMaxFlows && ((uintptr_t)d.pe_params & 15) == 0 &&
         ((uintptr_t)d.meas_params & 15) == 0;
}

// The two-chain CRNVP proposal launch (tiled_prop_cm_kernel), opt-in with NFDPF_CM_TWO_CHAIN=1
// (read per call: tests compare both).  Measured SLOWER than the one-chain tiled_prop_kernel at
// C3 (33.7 vs 30.7 us per launch, 1.455e9 vs 1.566e9 particle-steps/s, one box, bit-identical).
static bool use_cm(const nfdpf_filter_desc &d) {
  const char *e = getenv("NFDPF_CM_TWO_CHAIN");
  return e && e[0] == '1' && d.n_flows <= kMaxFlows;
}

// One launch per step (tiled_step_fused_kernel), opt-in with NFDPF_FUSED_STEP=1, when every
// workgroup of the grid can be resident at once -- one 1024-thread workgroup per CU -- since a
// row's four workgroups wait for each other inside it.  Measured SLOWER than the two launches
// at C2 (1.483 vs 1.471 ms per pass, one box; profiles/r02_experiments.md): the granule
// exchange itself costs ~0.8 us against the 1.65 us launch gap it removes, but the front half
// runs 2.3 us longer inside the 16-wave workgroup than as its own 8-wave launch, and the
// proposal half's prologue stays at 2 us.  Kept, bit-identical, for that record and as a base.
static bool use_fused(const nfdpf_filter_desc &d) {
  const char *e = getenv("NFDPF_FUSED_STEP");  // read per call: tests compare both paths
  if (!(e && e[0] == '1') || !use_merged(d) || d.phase != 0 || n_tiles(d.N) > kFusedMaxTiles) return false;
  // a sharded pass shares the device with the collectives' kernels on other streams, which can
  // hold CUs while the row's workgroups spin on each other: never there
  if (d.B_global != d.B) return false;
  int dev = 0, cus = 0, occ = 0;
  const size_t mlds = (size_t)(std::max(d.N, d.B_global) + 2 * d.N) * 4;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, tiled_step_fused_kernel, 4 * kTile, mlds) != hipSuccess ||
      occ < 1)
    return false;
  return (int64_t)n_tiles(d.N) * d.B <= (int64_t)cus * occ;
}

// The proposal launch.  With live timing requested (prof_events) the two events ride in the
// launch's own dispatch (hipExtLaunchKernel: the kernel's begin / end timestamps), not in
// separate event packets around it, so the measured time is the kernel's, as rocprof sees it.
template <bool NFD, bool NFC, int MEAS>
static void launch_prop(const nfdpf_filter_desc &d, TiledWs ws, dim3 g, hipStream_t st, hipEvent_t *ev) {
  // the two-role kernel needs a flow chain to overlap with the measurement
  // (a third role splitting the cosine encoder's output layer was measured slower: 16.7 vs
  // 11.4 us for the compute phase at C2 -- the extra waves duplicate the encoder's first layers)
  if constexpr (NFD && NFC && MEAS == NFDPF_MEAS_COS) {
    if (use_merged(d)) {
#ifndef NFDPF_PROP_SPLIT  // the quad launch (flow pair beside encoder pair); -DNFDPF_PROP_SPLIT: the pair launch
      if (ev)
        hipExtLaunchKernelGGL(tiled_prop_quad_kernel<true>, g, dim3(4 * kTile), 0, st, ev[0], ev[1], 0, d, ws);
      else
        tiled_prop_quad_kernel<true><<<g, 4 * kTile, 0, st>>>(d, ws);
#else
      if (ev)
        hipExtLaunchKernelGGL(tiled_prop_split_kernel<true>, g, dim3(2 * kTile), 0, st, ev[0], ev[1], 0, d, ws);
      else
        tiled_prop_split_kernel<true><<<g, 2 * kTile, 0, st>>>(d, ws);
#endif
      return;
    }
    if (use_split(d)) {
      if (ev)
        hipExtLaunchKernelGGL(tiled_prop_split_kernel<false>, g, dim3(2 * kTile), 0, st, ev[0], ev[1], 0, d, ws);
      else
        tiled_prop_split_kernel<false><<<g, 2 * kTile, 0, st>>>(d, ws);
      return;
    }
  }
  if constexpr (!NFC && MEAS == NFDPF_MEAS_CRNVP) {
    if (use_cm(d) && !d.meas_mfma) {
      const size_t lds = cm_lds_bytes(d.n_flows);
      // the fold buffer exceeds the default 64 KB at 3-4 flows
      ensure_max_dynamic_lds((const void *)tiled_prop_cm_kernel<NFD>, (int)cm_lds_bytes(kMaxFlows));
      if (ev)
        hipExtLaunchKernelGGL(tiled_prop_cm_kernel<NFD>, g, dim3(2 * kTile), lds, st, ev[0], ev[1], 0, d, ws);
      else
        tiled_prop_cm_kernel<NFD><<<g, 2 * kTile, lds, st>>>(d, ws);
      return;
    }
  }
  if constexpr (NFC && MEAS != NFDPF_MEAS_EXTERNAL) {
    if (ev)
      hipExtLaunchKernelGGL(tiled_prop2_kernel<NFD, NFC, MEAS, 2>, g, dim3(2 * kTile), 0, st, ev[0], ev[1], 0, d,
                            ws);
    else
      tiled_prop2_kernel<NFD, NFC, MEAS, 2><<<g, 2 * kTile, 0, st>>>(d, ws);
  } else {
    if constexpr (MEAS == NFDPF_MEAS_CRNVP) {
      if (d.meas_mfma) {  // (NFC is false here: the tiled_prop2 branch above takes the conditional proposal)
        const size_t lds = (size_t)crnvp_mfma_floats(d.n_flows) * sizeof(float);
        if (ev)
          hipExtLaunchKernelGGL(tiled_prop_kernel<NFD, NFC, MEAS, 2>, g, dim3(kTile), lds, st, ev[0], ev[1], 0, d,
                                ws);
        else
          tiled_prop_kernel<NFD, NFC, MEAS, 2><<<g, kTile, lds, st>>>(d, ws);
        return;
      }
      if (use_stage(d)) {
        const size_t lds = (size_t)(kCrnvpPe + d.n_flows * kCrnvpFlow) * sizeof(float);
        if (ev)
          hipExtLaunchKernelGGL(tiled_prop_kernel<NFD, NFC, MEAS, 1>, g, dim3(kTile), lds, st, ev[0], ev[1], 0,
                                d, ws);
        else
          tiled_prop_kernel<NFD, NFC, MEAS, 1><<<g, kTile, lds, st>>>(d, ws);
        return;
      }
    }
    if (ev)
      hipExtLaunchKernelGGL(tiled_prop_kernel<NFD, NFC, MEAS>, g, dim3(kTile), 0, st, ev[0], ev[1], 0, d, ws);
    else
      tiled_prop_kernel<NFD, NFC, MEAS><<<g, kTile, 0, st>>>(d, ws);
  }
}

template <int MEAS>
static void dispatch_prop(const nfdpf_filter_desc &d, TiledWs ws, dim3 g, hipStream_t st, hipEvent_t *ev) {
  if (d.nf_dyn && d.nf_cond)
    launch_prop<true, true, MEAS>(d, ws, g, st, ev);
  else if (d.nf_dyn)
    launch_prop<true, false, MEAS>(d, ws, g, st, ev);
  else if (d.nf_cond)
    launch_prop<false, true, MEAS>(d, ws, g, st, ev);
  else
    launch_prop<false, false, MEAS>(d, ws, g, st, ev);
}

}  // namespace nfdpf

#include "filter_pass.hpp"     // the whole pass as one persistent launch (C2 shape)
#include "filter_pass_cm.hpp"  // ... the C3 shape (bootstrap proposal, CRNVP measurement, speculative gate)

using namespace nfdpf;

extern "C" int nfdpf_filter_pass_supported(const nfdpf_filter_desc *d) {
  return d && (pass_config_ok(*d) || pass_cm_config_ok(*d)) ? 1 : 0;
}

extern "C" int64_t nfdpf_filter_pass_workspace_bytes(int B, int N, int T) {
  return (B <= 0 || N <= 0 || T <= 0) ? 256 : pass_bytes(B, N, T);
}

extern "C" int nfdpf_filter_pass_tiled(const nfdpf_filter_desc *dp, void *workspace, void *stream) {
  NFDPF_REQUIRE(dp && workspace, "nfdpf_filter_pass_tiled: null argument");
  const nfdpf_filter_desc &d = *dp;
  NFDPF_REQUIRE(((uintptr_t)workspace & 255) == 0, "nfdpf_filter_pass_tiled: workspace not 256-B aligned");
  NFDPF_REQUIRE(d.t == 0, "nfdpf_filter_pass_tiled: a pass starts at t = 0 (got t=%d)", d.t);
  NFDPF_REQUIRE(d.hist_x && d.hist_p && d.hist_noise && d.hist_lik && d.hist_idx && d.ess_out && d.enc && d.vel &&
                    d.x_prev && d.p_prev && d.lw_sum && d.pred,
                "nfdpf_filter_pass_tiled: null input/output pointer");
  if (pass_cm_config_ok(d)) {  // the C3 / C1 shape: no flows on the particle path (CRNVP, cosine, gaussian)
    NFDPF_REQUIRE(d.pe_params && (d.meas_params || d.measurement != NFDPF_MEAS_CRNVP) && d.ess_all,
                  "nfdpf_filter_pass_tiled: parameters / ess_all missing");
    NFDPF_REQUIRE(!d.meas_mfma || ((uintptr_t)d.meas_params & 15) == 0,
                  "nfdpf_filter_pass_tiled: the MFMA fragment blob must be 16-B aligned");
    const int verify_cm = d.pass_gates && d.B_global == d.B;
    NFDPF_REQUIRE(!d.pass_gates || verify_cm, "nfdpf_filter_pass_tiled: pass_gates needs a pass of the whole batch");
    hipStream_t st = as_stream(stream);
    PassWs ws = pass_carve(workspace, d.B, d.N, d.T);
    ws.wait_ticks = kPassWaitTicks;
    if (const char *e = getenv("NFDPF_PASS_WAIT_US"))  // read per call (tests force a timeout)
      ws.wait_ticks = (uint64_t)std::max(1L, atol(e)) * 100ull;
    const auto kern = pass_cm_kernel_of(d);
    const int rows = pass_resident_rows(kern, pass_cm_threads(d), n_tiles(d.N));
    NFDPF_REQUIRE(rows >= 1, "nfdpf_filter_pass_tiled: no row of the pass fits on the device");
    pass_launch_rows(kern, d, ws, pass_cm_threads(d), std::min(rows, d.B), st);
    tiled_pass_epilogue_kernel<<<d.T, 64, 0, st>>>(d, ws, verify_cm, 4);
    return launch_status("nfdpf_filter_pass_tiled");
  }
  NFDPF_REQUIRE(d.hist_jac && d.hist_prior, "nfdpf_filter_pass_tiled: null input/output pointer");
  NFDPF_REQUIRE(d.dyn_params && d.cond_params && d.pe_params, "nfdpf_filter_pass_tiled: parameters missing");
  NFDPF_REQUIRE(!d.force_resample || (d.lin && ((uintptr_t)d.hist_x & 7) == 0),
                "nfdpf_filter_pass_tiled: a forced pass needs lin and an 8-B aligned hist_x");
  NFDPF_REQUIRE(pass_config_ok(d),
                "nfdpf_filter_pass_tiled: configuration not supported here (nfdpf_filter_pass_supported == 0)");
  const int mode = pass_mode_of(d);
  NFDPF_REQUIRE(d.ess_all || mode == kModeForce, "nfdpf_filter_pass_tiled: ess_all (the initial partials) missing");
  NFDPF_REQUIRE(!d.gate_peers || (mode == kModeGate && !d.pass_plan && d.gate_rank >= 0 && d.gate_rank < d.gate_world &&
                                  d.gate_world <= 64 && d.B_global <= kXgMaxRows && d.row_base + d.B <= d.B_global),
                "nfdpf_filter_pass_tiled: gate_peers needs a gated pass (no plan), 0 <= gate_rank < gate_world <= 64 "
                "and B_global <= %d", kXgMaxRows);
  // the epilogue's gates: those of a speculative pass of the whole batch (a sharded one is
  // verified by the caller over the gathered partials, nfdpf_ess_gate_tiled_batch), or the
  // decisions the gated pass took itself
  // (a plan pass's epilogue verifies the plan from the partials, as a speculative pass's)
  const int verify = (mode == kModeSpec || (mode == kModeGate && d.pass_plan)) && d.pass_gates && d.B_global == d.B;
  NFDPF_REQUIRE(!d.pass_gates || verify || (mode == kModeGate && !d.pass_plan),
                "nfdpf_filter_pass_tiled: pass_gates needs a pass of the whole batch (B_global == B) that is not forced");
  hipStream_t st = as_stream(stream);
  PassWs ws = pass_carve(workspace, d.B, d.N, d.T);
  ws.wait_ticks = kPassWaitTicks;
  if (const char *e = getenv("NFDPF_PASS_WAIT_US"))  // read per call (tests force a timeout)
    ws.wait_ticks = (uint64_t)std::max(1L, atol(e)) * 100ull;
  const auto kern = pass_kernel_of(d);
  const int rows = pass_resident_rows(kern, 4 * kTile, n_tiles(d.N));
  // (pass_config_ok: the gated pass has all its rows resident in one launch)
  NFDPF_REQUIRE(rows >= d.B || (rows >= 1 && (mode != kModeGate || d.pass_plan)),
                "nfdpf_filter_pass_tiled: the pass's rows do not fit on the device");
  pass_launch_rows(kern, d, ws, 4 * kTile, std::min(rows, d.B), st);
  tiled_pass_epilogue_kernel<<<d.T, 64, 0, st>>>(d, ws, mode == kModeGate && !d.pass_plan ? 2 : verify, 8);
  return launch_status("nfdpf_filter_pass_tiled");
}

extern "C" int64_t nfdpf_filter_tiled_workspace_bytes(int B, int N, int T) {
  return (B <= 0 || N <= 0 || T <= 0) ? 256 : tiled_bytes(B, N, T);
}

extern "C" int nfdpf_filter_tiled_tiles(int N) { return N <= 0 ? 0 : n_tiles(N); }

extern "C" int nfdpf_filter_tiled_fused(const nfdpf_filter_desc *d) { return d && use_fused(*d) ? 1 : 0; }

extern "C" int nfdpf_ess_gate_tiled(const double *parts, int B, int N, int t, int force, int32_t *gate,
                                    void *stream) {
  NFDPF_REQUIRE(gate && (force || parts) && B >= 1 && N >= 1, "nfdpf_ess_gate_tiled: bad arguments");
  tiled_gate_kernel<<<1, 64, 0, as_stream(stream)>>>(parts, B, n_tiles(N), N, t, force, gate);
  return launch_status("nfdpf_ess_gate_tiled");
}

extern "C" int nfdpf_ess_gate_tiled_batch(const double *parts, int T, int B, int N, int t0, int force,
                                          int32_t *gates, void *stream) {
  NFDPF_REQUIRE(gates && (force || parts) && T >= 0 && B >= 1 && N >= 1 && t0 >= 0,
                "nfdpf_ess_gate_tiled_batch: bad arguments");
  if (T == 0) return NFDPF_OK;
  tiled_gate_batch_kernel<<<T, 64, 0, as_stream(stream)>>>(parts, B, n_tiles(N), N, t0, force, gates);
  return launch_status("nfdpf_ess_gate_tiled_batch");
}

namespace nfdpf {
// row b's gate term of step t (block = step, lanes over rows); the last block also reads and
// clears the hand-off fault counter into terms[T * B]
__global__ __launch_bounds__(64) void ess_row_terms_kernel(const double *__restrict__ parts, int B, int tiles, int N,
                                                           int t0, float *terms) {
  const int k = blockIdx.x;
  const double *p = parts + (int64_t)k * B * tiles * kSm;
  for (int r = threadIdx.x; r < B; r += 64)
    terms[(int64_t)k * B + r] = row_inv_ess(p + (int64_t)r * tiles * kSm, tiles, N, t0 + k > 0);
  if (k == (int)gridDim.x - 1 && threadIdx.x == 0)
    reinterpret_cast<int32_t *>(terms)[(int64_t)gridDim.x * B] = atomicExch(&g_split_fault, 0);
}
// tiled_gate_batch_kernel's cascade over the gathered rows' terms (one wave per step)
__global__ __launch_bounds__(64) void ess_gate_terms_kernel(const float *__restrict__ terms, int B, int N, int force,
                                                            int32_t *gates) {
  const int k = blockIdx.x;
  const float *p = terms + (int64_t)k * B;
  const float s = cascade_row_sum([&](int r) { return p[r]; }, force ? 0 : B);
  if (threadIdx.x == 0) gates[k] = (force || (s / (float)B) < 0.5f * (float)N) ? 1 : 0;
}
}  // namespace nfdpf

extern "C" int nfdpf_ess_row_terms(const double *parts, int T, int B, int N, int t0, float *terms, void *stream) {
  NFDPF_REQUIRE(parts && terms && T >= 1 && B >= 1 && N >= 1 && t0 >= 0, "nfdpf_ess_row_terms: bad arguments");
  ess_row_terms_kernel<<<T, 64, 0, as_stream(stream)>>>(parts, B, n_tiles(N), N, t0, terms);
  return launch_status("nfdpf_ess_row_terms");
}

extern "C" int nfdpf_ess_gate_terms(const float *terms, int T, int B, int N, int force, int32_t *gates, void *stream) {
  NFDPF_REQUIRE(gates && (force || terms) && T >= 0 && B >= 1 && N >= 1, "nfdpf_ess_gate_terms: bad arguments");
  if (T == 0) return NFDPF_OK;
  ess_gate_terms_kernel<<<T, 64, 0, as_stream(stream)>>>(terms, B, N, force, gates);
  return launch_status("nfdpf_ess_gate_terms");
}

extern "C" int nfdpf_pass_verify(const double *parts, const float *lw_sum, int T, int B, int N, int t0,
                                 int32_t *gates, int32_t *flags, float *obs, void *stream) {
  NFDPF_REQUIRE(parts && lw_sum && gates && flags && obs && T >= 1 && B >= 1 && N >= 1 && t0 >= 0,
                "nfdpf_pass_verify: bad arguments");
  hipStream_t st = as_stream(stream);
  tiled_gate_batch_kernel<<<T, 64, 0, st>>>(parts, B, n_tiles(N), N, t0, 0, gates);
  tiled_verify_flags_kernel<<<1, 64, 0, st>>>(gates, lw_sum, T, B, (double)B * (double)N, flags, obs);
  return launch_status("nfdpf_pass_verify");
}

extern "C" int nfdpf_filter_tiled_init(const float *p0, int B, int N, double *ess_parts,
                                       void *stream) {
  NFDPF_REQUIRE(p0 && ess_parts && B >= 0 && N >= 1, "nfdpf_filter_tiled_init: bad arguments");
  if (B == 0) return NFDPF_OK;
  tiled_ess_init_kernel<<<dim3(n_tiles(N), B), kTile, 0, as_stream(stream)>>>(p0, N, ess_parts);
  return launch_status("nfdpf_filter_tiled_init");
}

extern "C" int nfdpf_filter_init(const float *start, int start_rs, const float *vel_in, int vel_rs, int T, int B,
                                 int N, float width, int true_state, uint64_t seed, int64_t row_base, float *x,
                                 float *logw, float *p, float *inv_ess, double *ess_parts, float *vel, void *stream) {
  NFDPF_REQUIRE(x && logw && p && ess_parts && (!true_state || start) && (!vel || (start && (T <= 1 || vel_in))),
                "nfdpf_filter_init: null pointer");
  NFDPF_REQUIRE(B >= 0 && N >= 1 && N <= 1024 && T >= 0 && start_rs >= 4 && vel_rs >= 2 * (T > 1 ? T - 1 : 0),
                "nfdpf_filter_init: bad sizes (need 1 <= N <= 1024, start rows >= 4, vel rows >= 2 (T - 1); got N=%d)",
                N);
  if (B == 0) return NFDPF_OK;
  filter_init_kernel<<<B, row_threads(N), 0, as_stream(stream)>>>(start, start_rs, vel_in, vel_rs, T, N, width,
                                                                  true_state, seed, row_base, x, logw, p, inv_ess,
                                                                  ess_parts, vel);
  return launch_status("nfdpf_filter_init");
}

extern "C" int nfdpf_split_fault(int reset, void *stream) {
  // stream-ordered after the launches it checks (the caller's stream, not the null stream); the
  // host words are this call's own (the stream is synchronised before they go out of scope)
  int v = 0;
  const int z = 0;
  hipStream_t st = as_stream(stream);
  if (hipMemcpyFromSymbolAsync(&v, HIP_SYMBOL(g_split_fault), sizeof(int), 0, hipMemcpyDeviceToHost, st) !=
          hipSuccess ||
      hipStreamSynchronize(st) != hipSuccess) {
    set_error("nfdpf_split_fault: reading the fault counter failed");
    return -1;
  }
  const int n = v;
  if (reset && n != 0) {
    if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_split_fault), &z, sizeof(int), 0, hipMemcpyHostToDevice, st) !=
            hipSuccess ||
        hipStreamSynchronize(st) != hipSuccess)
      return -1;
  }
  return n;
}

#ifdef NFDPF_EXP_PTRACE
extern "C" NFDPF_API int nfdpf_exp_ptrace_read(void *host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ptrace), sizeof(g_ptrace)) == hipSuccess ? 0 : 1;
}
#endif
#ifdef NFDPF_EXP_QTRACE
extern "C" NFDPF_API int nfdpf_exp_qtrace_read(void *host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_qtrace), sizeof(g_qtrace)) == hipSuccess ? 0 : 1;
}
#endif
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
  NFDPF_REQUIRE(!d.meas_mfma || (d.measurement == NFDPF_MEAS_CRNVP && !d.nf_cond && d.n_flows <= 2 &&
                                 ((uintptr_t)d.meas_params & 15) == 0),
                "nfdpf_filter_step_tiled: meas_mfma needs the CRNVP measurement without --NF-cond, n_flows <= 2 "
                "and a 16-B aligned fragment blob");
  NFDPF_REQUIRE(d.E + 4 <= kMaxCtx, "nfdpf_filter_step_tiled: E too large");
  NFDPF_REQUIRE(d.measurement != NFDPF_MEAS_EXTERNAL || d.phase != 0,
                "nfdpf_filter_step_tiled: EXTERNAL measurement runs as phase 1 + phase 2");
  NFDPF_REQUIRE(d.measurement != NFDPF_MEAS_EXTERNAL || d.phase != 2 || d.lik_ext,
                "nfdpf_filter_step_tiled: phase 2 needs lik_ext");
  // OT reads p_prev before the step, so its steps defer only in a speculative pass (every gate
  // taken as off: d.gate given and zero, the shard's own partials -- ess_local)
  NFDPF_REQUIRE(!d.defer_norm || d.resampler == NFDPF_RESAMPLE_SOFT || (d.ess_local && d.gate && !d.force_resample),
                "nfdpf_filter_step_tiled: defer_norm needs the soft resampler or a speculative OT pass");
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
    // C / gate staging [max(N, B_global)], gathered weights [N], deferred p_{t-1} [N]
    const size_t lds = d.resampler == NFDPF_RESAMPLE_SOFT ? (size_t)(std::max(d.N, d.B_global) + 2 * d.N) * 4
                                                         : (size_t)d.B_global * 4;
    // live timing of the front launch (the resampler's) in its own dispatch, as launch_prop
    hipEvent_t *fev = d.prof_events && d.prof_front ? (hipEvent_t *)d.prof_events + 2 : nullptr;
    if (use_fused(d)) {  // the whole step in one launch (the live timing on it)
      const size_t mlds = (size_t)(std::max(d.N, d.B_global) + 2 * d.N) * 4;
      if (d.t == 0) tiled_epoch_kernel<<<1, 1, 0, st>>>();  // new tags for this pass
      hipEvent_t *ev = (hipEvent_t *)d.prof_events;
      if (ev)
        hipExtLaunchKernelGGL(tiled_step_fused_kernel, g, dim3(4 * kTile), mlds, st, ev[0], ev[1], 0, d, ws);
      else
        tiled_step_fused_kernel<<<g, 4 * kTile, mlds, st>>>(d, ws);
    } else if (use_merged(d)) {
      const size_t mlds = (size_t)(std::max(d.N, d.B_global) + 2 * d.N) * 4;
      if (fev)
        hipExtLaunchKernelGGL(tiled_fdyn_kernel, g, dim3(2 * kTile), mlds, st, fev[0], fev[1], 0, d, ws);
      else
        tiled_fdyn_kernel<<<g, 2 * kTile, mlds, st>>>(d, ws);
    } else if (use_rows(d)) {
      // the gate / row normaliser / row resampling once per row, then the tiles without LDS
      tiled_rows_kernel<<<d.B, 1024, lds, st>>>(d, ws);
      if (fev)
        hipExtLaunchKernelGGL(tiled_front_kernel<true>, g, dim3(kTile), 0, st, fev[0], fev[1], 0, d, ws);
      else
        tiled_front_kernel<true><<<g, kTile, 0, st>>>(d, ws);
    } else if (fev) {
      hipExtLaunchKernelGGL(tiled_front_kernel<false>, g, dim3(kTile), lds, st, fev[0], fev[1], 0, d, ws);
    } else {
      tiled_front_kernel<false><<<g, kTile, lds, st>>>(d, ws);
    }
    if (use_fused(d))
      ;  // the whole step ran in tiled_step_fused_kernel
    else if (use_merged(d))
      ;  // nf_dyn ran in tiled_fdyn_kernel
    else if (use_split(d))
      tiled_dyn_kernel<true><<<g, 2 * kTile, 0, st>>>(d, ws);
    else if (d.nf_dyn)
      tiled_dyn_kernel<false><<<g, kTile, 0, st>>>(d, ws);
    hipEvent_t *ev = (hipEvent_t *)d.prof_events;
    if (!use_fused(d)) switch (d.measurement) {
      case NFDPF_MEAS_COS: dispatch_prop<NFDPF_MEAS_COS>(d, ws, g, st, ev); break;
      case NFDPF_MEAS_CRNVP: dispatch_prop<NFDPF_MEAS_CRNVP>(d, ws, g, st, ev); break;
      case NFDPF_MEAS_NN: dispatch_prop<NFDPF_MEAS_NN>(d, ws, g, st, ev); break;
      case NFDPF_MEAS_GAUSSIAN: dispatch_prop<NFDPF_MEAS_GAUSSIAN>(d, ws, g, st, ev); break;
      case NFDPF_MEAS_EXTERNAL: dispatch_prop<NFDPF_MEAS_EXTERNAL>(d, ws, g, st, ev); break;
      default: set_error("nfdpf_filter_step_tiled: unknown measurement %d", d.measurement); return NFDPF_EINVAL;
    }
    if (d.phase == 1) return launch_status("nfdpf_filter_step_tiled");
  }
  if (d.measurement == NFDPF_MEAS_EXTERNAL) tiled_extlik_kernel<<<g, kTile, 0, st>>>(d, ws);
  const bool shift = d.measurement == NFDPF_MEAS_CRNVP || d.measurement == NFDPF_MEAS_GAUSSIAN ||
                     d.measurement == NFDPF_MEAS_EXTERNAL;
  if (!d.defer_norm || d.t == d.T - 1) {  // deferred: the next step's launches normalise slot t
    if (shift)
      tiled_norm_kernel<true><<<g, kTile, 0, st>>>(d, ws);
    else
      tiled_norm_kernel<false><<<g, kTile, 0, st>>>(d, ws);
  }
  if (d.t == d.T - 1 && d.pred && d.lw_sum) {
    const int BT = d.B * d.T;
    tiled_finalize_kernel<<<(BT + 255) / 256, 256, 0, st>>>(ws.fin, BT, n_tiles(d.N), d.pred, d.lw_sum);
  }
  return launch_status("nfdpf_filter_step_tiled");
}
