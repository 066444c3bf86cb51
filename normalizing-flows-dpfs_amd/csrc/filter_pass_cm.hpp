// filter_pass_cm.hpp -- the whole T-step filtering pass of DPF.filtering_pos (DPFs.py:160-214) as
// ONE persistent launch for the C3 shape: no dynamic flow, no conditional proposal (the bootstrap
// proposal x_t = (x_{t-1} + vel) + eps), the conditional-RealNVP measurement (model/models.py:
// 256-278, shifted by the row max of the raw likelihood), every ESS gate taken as off (the
// speculative mode: the caller verifies the T gates afterwards from the per-step partials this
// launch leaves, and a fired gate reruns the pass step by step -- OT or soft resampling there).
// Included by filter_tiled.hip after filter_pass.hpp (its workspace, granules and epilogue).
//
// Why this shape pipelines: without resampling a particle never leaves its lane and its path
// x_0, x_1, ... needs nothing from the row (the bootstrap proposal has no context exchange), so
// the measurement of every step -- all the arithmetic (12.7 k FLOP per particle-step) -- is
// independent of the weights.  Only the log-weights form a chain across steps: step t's
// u_t = ((log p_{t-1} + lik_t) + prior) - propose needs slot t - 1 normalised, i.e. the row's
// softmax partials of u_{t-1} (exchange C, the granules of filter_pass.hpp) and the row max of
// the raw likelihood (the CRNVP shift, model/models.py:276).  That chain is short (a sweep and a
// few VALU ops per particle); the likelihoods run ahead of it.
//
// Grid (tiles, B) of 4 K-wave workgroups (K = 2: 512 threads; K = 3: 768, NFDPF_CM_K), all
// resident (pass_cm_config_ok).  Wave w handles particle group g = w & 3 (64 particles of the
// tile, one per lane; waves w, w + 4, ... share a SIMD) on the steps t = k mod K, k = w >> 2: K
// steps of a group in flight per SIMD.  The step-indexed buffers stay double-buffered for any K:
// the x hand-over is serialised by the xf flags, and nb / rn / the C granules of slot s are
// reused by slot s + 2 only after the C(s + 1) sweep, which needs every wave that read them.
// Per step t, wave (g, t mod K):
//   1. x_t from x_{t-1} (LDS xr, from the group's other wave; flag xf[g]) + vel_t + eps_t ->
//      xr, hist_x / noise / index;
//   2. lik_t = crnvp_lik(x_t) (raw), the step's frame encoding in the wave's own LDS copy;
//   3. [group 0's wave: sweep C(t - 1) -> slot t - 1's row normaliser rn (LDS, flag fR) and
//      the tile's merged partial -> ess_out[t - 1]] -> normalise slot t - 1 of the group from
//      the other wave's hand-over nb (finish_prev's arithmetic: hist_p, hist_lik shifted, the
//      fin partials) -> log p_{t-1};
//   4. u_t, the group's partials {max u, sum e, sum e^2, max lik} -> C(t) granules.
// The waves of k = T mod K normalise the last slot after their loop.
//
// Every wait is bounded (pass_spin: 200 ms, the workspace's abort word), as in filter_pass.hpp.

#include "crnvp_mfma.hpp"

namespace nfdpf {

// steps in flight per particle group (waves per group): 2 (512 threads, <= 256 VGPRs per wave) or
// 3 (768 threads, <= 168 VGPRs: the MFMA measurement, whose MFMA and VALU phases then overlap
// across three waves per SIMD)
// (tiled_pass_cm_kernel<MEAS, MF, K>; pass_cm_k: NFDPF_CM_K, read per call)
constexpr int kCmMaxK = 3;
constexpr int kCmMfmaFlows = 2;  // the MFMA measurement's LDS blob holds up to 2 flows (DPFs.py:46: n_sequence 2)

struct PassCmLds {
  // x_t in buffer t mod K: the group's next wave reads it for step t + 1, and the MFMA measurement
  // of step t reads it back (its particles per N tile) while the next waves move on -- only the
  // wave of step t + K, this same wave, overwrites it
  float xr[kCmMaxK][4][64][2];
  float nb[2][5][kTile];     // slot t's hand-over by parity: lr, raw lik, prior, x0, x1
  alignas(16) float encq[4 * kCmMaxK][kE];  // each wave's copy of its step's frame encoding (crnvp_lik's encv)
  uint32_t rowc[kPassMaxTiles * 4 * kGC];
  // a one-tile row (N <= 256, C1): exchange C stays in the workgroup -- the 4 groups' tagged
  // granules by slot parity in LDS instead of the global granules (one LDS round trip, not an L2 one)
  uint64_t cx[2][4 * kGC];
  RowNorm rn[2];
  int xf[4];                 // x_t of group g written (t + 1)
  int fR;                    // slot t's row normaliser in rn[t & 1] (t + 1)
};

// the row normaliser of slot s from its C(s) granules (tiles x 4 groups, each {max u, sum e,
// sum e^2, max raw lik}): the tile's merge over its groups in order (ess_out[s], the gate's
// input), then row_norm's arithmetic over the tiles in order with the CRNVP shift.  One wave.
// LDSC: the LDS exchange may apply (one-tile rows; compiled out of the MFMA measurement's kernel,
// whose C3 rows have 4 tiles and whose registers are tight)
template <bool SHIFT, bool LDSC>
__device__ __forceinline__ void pass_cm_poll_c(const nfdpf_filter_desc &d, const PassWs &ws, PassCmLds &L, int b,
                                               int tile, uint32_t tag0, int s) {
  const int tiles = n_tiles(d.N), lane = threadIdx.x & 63;
  const int64_t row0 = (((int64_t)(s & 1) * d.B + b) * tiles) * 4;
  bool got;
  if (LDSC && tiles == 1) {  // the row's four groups in this workgroup: their granules in LDS
    const uint32_t tag = tag0 + (uint32_t)s + 1u;
    volatile uint64_t *cx = L.cx[s & 1];
    uint64_t v = 0;
    bool ok = lane >= 4 * kGC;
    Spin sp;
    for (;;) {
      if (!ok) {
        v = cx[lane];
        ok = (uint32_t)(v >> 32) == tag;
      }
      if (__all(ok)) break;
      if (!pass_spin(sp)) break;
    }
    got = __all(ok);
    if (got && lane < 4 * kGC) L.rowc[lane] = (uint32_t)v;
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  } else {
    got = poll_row(ws.gc + row0 * kGC, tiles * 4 * kGC, tag0 + (uint32_t)s + 1u, L.rowc);
  }
  if (got) {
    const int k = lane < tiles ? lane : 0;
    float m = -INFINITY, lm = -INFINITY;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      m = fmaxf(m, __uint_as_float(L.rowc[(k * 4 + v) * kGC]));
      lm = fmaxf(lm, __uint_as_float(L.rowc[(k * 4 + v) * kGC + 5]));
    }
    double sum = 0.0, sq = 0.0;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int q = (k * 4 + v) * kGC;
      const float mv = __uint_as_float(L.rowc[q]);
      if (mv > -INFINITY) {
        const double f = (double)expf(mv - m);
        sum += lds_double(L.rowc, q + 1) * f;
        sq += lds_double(L.rowc, q + 3) * f * f;
      }
    }
    if (lane == tile) {
      double *sm = reinterpret_cast<double *>(d.ess_out) + (((int64_t)s * d.B + b) * tiles + tile) * kSm;
      sm[0] = m;
      sm[1] = sum;
      sm[2] = sq;
      sm[3] = lm;
    }
    // row_norm (filter_tiled.hip) over the tiles in order, shifted by the row max raw likelihood
    float M = -INFINITY, Lmax = -INFINITY;
    for (int kk = 0; kk < tiles; ++kk) {
      M = fmaxf(M, (float)(double)readlane_f(m, kk));
      Lmax = fmaxf(Lmax, readlane_f(lm, kk));
    }
    double Sd = 0.0;
    for (int kk = 0; kk < tiles; ++kk) Sd += readlane_d(sum, kk) * (double)expf(readlane_f(m, kk) - M);
    if (lane == 0) L.rn[s & 1] = SHIFT ? RowNorm{M - Lmax, (float)Sd, Lmax} : RowNorm{M, (float)Sd, 0.f};
  }
  set_flag(&L.fR, s + 1);
}

// normalise slot s of this wave's group from the hand-over nb[s & 1] (finish_prev / prev_p_of's
// arithmetic, shifted): hist_p, hist_lik (the shifted likelihood), the group's fin partials
// (entry g of the tile); returns log p
template <bool SHIFT>
__device__ __forceinline__ float pass_cm_norm(const nfdpf_filter_desc &d, const PassWs &ws, PassCmLds &L, int b,
                                              int tile, int g, int s, int slot, int i, bool valid) {
  wait_flag(&L.fR, s + 1);
  const RowNorm rn = L.rn[s & 1];
  double sf[4] = {0.0, 0.0, 0.0, 0.0};
  float lp = 0.f;
  if (valid) {
    const int par = s & 1;
    const float lr = L.nb[par][0][slot], raw = L.nb[par][1][slot], pr = L.nb[par][2][slot];
    const float lk = SHIFT ? raw - rn.Lmax : raw;
    const float lw = ((lr + lk) + pr) - pr;
    const float p = expf(lw - rn.shift) / rn.Ssum + 1e-12f;
    const int64_t o = ((int64_t)b * d.T + s) * d.N + i;
    d.hist_p[o] = p;
    d.hist_lik[o] = lk;
    lp = logf(p);
    sf[0] = (double)p * p;
    sf[1] = (double)p * L.nb[par][3][slot];
    sf[2] = (double)p * L.nb[par][4][slot];
    sf[3] = lw;
  }
  wave_sum_dpp_n(sf);
  const int lane = threadIdx.x & 63, tiles = n_tiles(d.N);
  if (lane < 4)
    ws.fin[((((int64_t)b * d.T + s) * tiles + tile) * 4 + g) * 4 + lane] =
        lane == 0 ? sf[0] : lane == 1 ? sf[1] : lane == 2 ? sf[2] : sf[3];
  return lp;
}

// MF (CRNVP with d.meas_mfma): the measurement on f32 MFMA (crnvp_mfma.hpp), 64 particles per
// wave, its fragment blob staged in LDS once per launch; else crnvp_lik per lane (scalar-cache
// weights, VALU)
template <int MEAS, bool MF = false, int K = 2>
__global__ __launch_bounds__(4 * K * 64, 1) void tiled_pass_cm_kernel(const nfdpf_filter_desc d, PassWs ws) {
  static_assert(MEAS == NFDPF_MEAS_CRNVP || MEAS == NFDPF_MEAS_COS || MEAS == NFDPF_MEAS_GAUSSIAN,
                "the no-flow pass: the CRNVP, cosine or gaussian measurement");
  static_assert(!MF || MEAS == NFDPF_MEAS_CRNVP, "MFMA: the CRNVP measurement");
  constexpr bool SHIFT = meas_shifted<MEAS>();  // CRNVP / gaussian: lik - the row max (model/models.py:276)
  __shared__ PassCmLds L;
  __shared__ f4v wfr[MF ? crnvp_mfma_floats(kCmMfmaFlows) / 4 : 1];  // MF: the fragment blob
  int b, tile;
  pass_tile_row(b, tile);
  const uint32_t tag0 = __hip_atomic_load(&ws.hdr->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) << 12;
  if (threadIdx.x < 4) L.xf[threadIdx.x] = 0;
  if (threadIdx.x == 0) L.fR = 0;
  if (threadIdx.x < 2 * 4 * kGC) (&L.cx[0][0])[threadIdx.x] = 0;  // (no tag: never a match)
  if constexpr (MF) {  // (16-B aligned blob of whole float4s: checked on the host)
    const f4v *src = reinterpret_cast<const f4v *>(d.meas_params);
    for (int q = threadIdx.x; q < crnvp_mfma_floats(d.n_flows) / 4; q += blockDim.x) wfr[q] = src[q];
  }
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int g = w & 3, k = w >> 2, slot = g * 64 + lane, N = d.N, tiles = n_tiles(N);  // k: t mod K
  const int km1 = k == 0 ? K - 1 : k - 1;  // (t - 1) mod K
  const int i = tile * kTile + slot;
  const bool valid = i < N;
  const int64_t grow = d.row_base + b;
  __syncthreads();
  float lr = 0.f;  // log p of this wave's particle in the slot before its next step
  if (k == 0) {  // x_0 = the initial particles (step 0 is parity 0's)
    if (valid) {
      L.xr[K - 1][g][lane][0] = d.x_prev[(int64_t)b * d.x_prev_rs + 2 * i];  // "x_{-1}": buffer -1 mod K
      L.xr[K - 1][g][lane][1] = d.x_prev[(int64_t)b * d.x_prev_rs + 2 * i + 1];
      lr = logf(d.p_prev[(int64_t)b * d.p_prev_rs + i]);
    }
  }
  for (int t = k; t < d.T; t += K) {
    const nfdpf_filter_desc &d = *(const nfdpf_filter_desc *)kernarg_desc();  // (kernarg_desc)
    const PassWs &ws = *(const PassWs *)kernarg_ws();
    const int par = t & 1;
    const RowSlot S = row_slot(d, b, t);
    // 1. motion (model/models.py:191-204): the bootstrap proposal, prior = propose = density(eps)
    float e0 = 0.f, e1 = 0.f;
    if (valid) pass_noise(d, t, grow, i, e0, e1);
    const float v0 = d.vel[2 * ((int64_t)t * d.B + b)], v1 = d.vel[2 * ((int64_t)t * d.B + b) + 1];
    if (lane < kE) L.encq[w][lane] = d.enc[((int64_t)b * d.T + t) * d.E + lane];
    wait_flag(&L.xf[g], t);  // x_{t-1} of the group
    float x0 = 0.f, x1 = 0.f, de = 0.f;
    if (valid) {
      x0 = (L.xr[km1][g][lane][0] + v0) + e0;
      x1 = (L.xr[km1][g][lane][1] + v1) + e1;
      L.xr[k][g][lane][0] = x0;
      L.xr[k][g][lane][1] = x1;
    }
    set_flag(&L.xf[g], t + 1);
    if (valid) {
      S.hx[2 * i] = x0;
      S.hx[2 * i + 1] = x1;
      S.hnoise[2 * i] = e0;
      S.hnoise[2 * i + 1] = e1;
      S.hidx[i] = (int64_t)N * grow + i;
      de = density(e0, e1, d.dens_const, 2.0f * (d.pos_noise * d.pos_noise)) + 0.0f;
    }
    // 2. the measurement of x_t (model/models.py:256-278), unshifted
    float raw = -INFINITY;
    double vinv = 0.0;
    if constexpr (MEAS == NFDPF_MEAS_COS) {  // measure_row_setup's 1 / max(|v|, 1e-12), per wave
      const float ve = lane < kE ? d.enc[((int64_t)b * d.T + t) * d.E + lane] : 0.f;
      vinv = 1.0 / fmax(sqrt(wave_sum((double)ve * ve)), 1e-12);
    }
    if constexpr (MF) {  // the whole wave: its 64 particles x_t are in xr[t mod K][g]
      const float r = crnvp_lik_mfma(reinterpret_cast<const float *>(wfr), d.n_flows, d.meas_prior_std, L.encq[w],
                                     &L.xr[k][g][0][0]);
      if (valid) raw = r;
    } else if (valid) {
      if constexpr (MEAS == NFDPF_MEAS_CRNVP) {
        raw = crnvp_lik(wptr(d.pe_params), wptr(d.meas_params), d.n_flows, d.meas_prior_std, L.encq[w], x0, x1);
      } else if constexpr (MEAS == NFDPF_MEAS_COS) {  // model/models.py:206-219 (measure<COS>'s arithmetic)
        double ss, dot;
        encode_dot<kE>(wptr(d.pe_params), x0, x1, L.encq[w], ss, dot);
        raw = cos_lik(ss, dot, vinv);
      } else {  // the gaussian measurement, model/models.py:237-254 (measure<GAUSSIAN>'s arithmetic)
        float e[kE];
        particle_encode<kE>(wptr(d.pe_params), x0, x1, e);
        float m = 0.f;
#pragma unroll
        for (int j = 0; j < kE; ++j) {
          const float vv = (L.encq[w][j] - e[j] - 1.0f) * 0.1f;
          m = fmaf(vv, vv, m);
        }
        raw = -0.5f * (kE * 1.8378770664093453f + m) - kE * 2.302585092994046f;
      }
    }
    // 3. slot t - 1: its row normaliser (group 0's wave sweeps C(t - 1)), its normalisation
    if (t > 0) {
      if (g == 0) pass_cm_poll_c<SHIFT, !MF>(d, ws, L, b, tile, tag0, t - 1);
      lr = pass_cm_norm<SHIFT>(d, ws, L, b, tile, g, t - 1, slot, i, valid);
    }
    // 4. the log-weight (DPFs.py:187) and exchange C(t): this group's softmax partials
    float u = -INFINITY;
    if (valid) {
      u = ((lr + raw) + de) - de;
      L.nb[par][0][slot] = lr;
      L.nb[par][1][slot] = raw;
      L.nb[par][2][slot] = de;
      L.nb[par][3][slot] = x0;
      L.nb[par][4][slot] = x1;
    }
    const float mw = wave_max_dpp(u), lmw = wave_max_dpp(raw);
    const float ev = valid ? expf(u - mw) : 0.f;
    double r[2] = {(double)ev, (double)ev * ev};
    wave_sum_dpp_n(r);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // nb written before C(t) can be swept
    if (lane < kGC) {
      const uint64_t eb = (uint64_t)__double_as_longlong(r[0]), qb = (uint64_t)__double_as_longlong(r[1]);
      const uint32_t word = lane == 0 ? __float_as_uint(mw)
                            : lane == 1 ? (uint32_t)eb
                            : lane == 2 ? (uint32_t)(eb >> 32)
                            : lane == 3 ? (uint32_t)qb
                            : lane == 4 ? (uint32_t)(qb >> 32)
                                        : __float_as_uint(lmw);
      const int64_t gslot = (((int64_t)par * d.B + b) * tiles + tile) * 4 + g;
      if (!MF && tiles == 1)
        *(volatile uint64_t *)&L.cx[par][g * kGC + lane] = ((uint64_t)(tag0 + (uint32_t)t + 1u) << 32) | word;
      else
        gran_store(ws.gc + gslot * kGC + lane, word, tag0 + (uint32_t)t + 1u);
    }
  }
  // the last slot's normalisation: the waves of parity T & 1 (they would have run step T)
  if (k == d.T % K) {
    if (g == 0) pass_cm_poll_c<SHIFT, !MF>(d, ws, L, b, tile, tag0, d.T - 1);
    pass_cm_norm<SHIFT>(d, ws, L, b, tile, g, d.T - 1, slot, i, valid);
  }
}

typedef void (*pass_cm_kernel_t)(const nfdpf_filter_desc, PassWs);
// steps in flight per particle group: 3 for the MFMA measurement (three waves per SIMD overlap its
// MFMA and VALU phases: 0.594 -> 0.560 ms per C3 pass, A/B on one box), else 2 (the per-lane VALU
// measurement spills at 168 VGPRs); NFDPF_CM_K=2|3 (read per call) overrides
static int pass_cm_k(const nfdpf_filter_desc &d) {
  const char *e = getenv("NFDPF_CM_K");
  if (e && (e[0] == '2' || e[0] == '3')) return e[0] - '0';
  return d.meas_mfma ? 3 : 2;
}
static int pass_cm_threads(const nfdpf_filter_desc &d) { return 4 * pass_cm_k(d) * 64; }
template <int K>
static pass_cm_kernel_t pass_cm_kernel_k(const nfdpf_filter_desc &d) {
  return d.measurement == NFDPF_MEAS_COS        ? tiled_pass_cm_kernel<NFDPF_MEAS_COS, false, K>
         : d.measurement == NFDPF_MEAS_GAUSSIAN ? tiled_pass_cm_kernel<NFDPF_MEAS_GAUSSIAN, false, K>
         : d.meas_mfma                          ? tiled_pass_cm_kernel<NFDPF_MEAS_CRNVP, true, K>
                                                : tiled_pass_cm_kernel<NFDPF_MEAS_CRNVP, false, K>;
}
static pass_cm_kernel_t pass_cm_kernel_of(const nfdpf_filter_desc &d) {
  return pass_cm_k(d) == 3 ? pass_cm_kernel_k<3>(d) : pass_cm_kernel_k<2>(d);
}

// The C3-shaped pass applies: the configuration, the speculative gate (not forced, not gated in
// the launch), and every workgroup of its grid resident at once.
static bool pass_cm_config_ok(const nfdpf_filter_desc &d) {
  const char *e = getenv("NFDPF_PASS");  // read per call: NFDPF_PASS=0 keeps the step-by-step launches
  if (e && e[0] == '0') return false;
  if (d.nf_dyn != NFDPF_DYN_NONE || d.nf_cond ||
      (d.measurement != NFDPF_MEAS_CRNVP && d.measurement != NFDPF_MEAS_COS && d.measurement != NFDPF_MEAS_GAUSSIAN))
    return false;
  if (d.rng_mode != NFDPF_RNG_DEVICE || d.phase != 0 || d.E != kE || d.force_resample || d.pass_gate) return false;
  if (d.meas_mfma && (d.measurement != NFDPF_MEAS_CRNVP || d.n_flows > kCmMfmaFlows)) return false;
  if (d.N < 2 || n_tiles(d.N) > kPassMaxTiles || d.n_flows < 0 || d.n_flows > kMaxFlows || d.T < 1 ||
      d.T > kPassMaxT || d.B < 1 || d.B > 256)
    return false;
  // every row resident in one launch: above that the step launches are faster for this shape
  // (C3 x 128 rows on one MI355X: 3.14e9 particle-steps/s step by step against 2.90e9 for two
  // resident chunks of the pass -- unlike the C2 shape, its step launches fill the device)
  return pass_resident_rows(pass_cm_kernel_of(d), pass_cm_threads(d), n_tiles(d.N)) >= d.B;
}

}  // namespace nfdpf
