// filter_pass.hpp -- the whole T-step filtering pass of DPF.filtering_pos (DPFs.py:160-214) as
// ONE persistent launch, for the C2-shaped path (--NF-dyn RealNVP, --NF-cond, the cosine
// measurement, N <= 1024) when every ESS gate of the pass is taken as off (the speculative-gate
// mode: nfdpf_pass_verify / nfdpf_ess_gate_tiled_batch verify the T gates after the pass from the
// per-step partials this launch leaves, and a fired gate reruns the pass step by step), or with
// the soft resampler forced every step (the row's resampling inside the launch, pass_resample).
// Included by filter_tiled.hip (same translation unit: it shares g_split_fault).
//
// Why: the two-launch step (tiled_fdyn_kernel + tiled_prop_quad_kernel) is a chain of
// latency-bound phases whose every launch starts by re-reading what the previous launch left in
// HBM (the row's particles, partials and folds, from other XCDs) -- 50 steps x 2 launches of
// ~13 + 15 us.  Without resampling a particle never leaves its lane: its state stays in
// registers for the whole pass, and a step needs only three ROW-LOCAL reductions, exchanged
// between the row's workgroups inside the launch as 8-byte {32 data bits, tag} granules
// (agent-scope sc1 stores / loads, MI355X_MICROARCH.md handoff-1to1, ~1 us each):
//
//   A  sum x, x^2 of x_phys after motion      -> nf_dyn context [mean, std]   (model/models.py:309-315)
//   B  sum x, x^2 of x_dyn after nf_dyn^-1    -> proposal context            (model/models.py:338-346)
//   C  softmax partials {max, sum e, sum e^2} -> slot t's normalisation      (DPFs.py:187-192, utils.py:39-44)
//
// Grid (tiles, B) of 1024-thread workgroups, one per CU, ALL resident (the host checks the grid
// against the occupancy; a row's workgroups wait for each other; pass_tile_row puts a row's
// tiles on one XCD).  Each of the 4 particle groups of a tile (64 particles, one per lane) has
// one wave per stage, the stages running independent loops over the steps and meeting only
// through LDS flags (step-tagged, monotonic):
//
//   chain t (waves 0-3, issue priority 3): motion -> publish A -> [wave 0: sweep A, nf_dyn
//            fold -> fA] -> nf_dyn inverse -> publish B -> [wave 0: sweep B, proposal fold
//            (encoding columns from prior wave 4: fE) -> fB] -> proposal inverse -> qbuf,
//            pbuf, rbuf's propose half (qf)
//   prior t (waves 4-7): [wave 4: the encoding-column fold of step t+1 -> fE] -> wait qf ->
//            nf_dyn forward of the proposal + the prior density -> rbuf (rf, pf)
//   enc  t (waves 8-15, a pair per group): encoder on qbuf (MFMA) -> [wave 8: sweep C(t-1) ->
//            slot t-1's row normaliser (fR), its ESS partial] -> normalise slot t-1 (hp, the
//            prediction / obs-likelihood partials) -> log-weight (ef) -> publish C(t)
//            (forced: the C(t-1) sweep and the normalisation first, then the encoder after the
//            row's resampling, fS)
//
// so the prior and the encoder of step t run beside the chain's step t+1.  Every step-indexed
// buffer (LDS and granules) is double-buffered by step parity: the exchanges are safe by the
// dependency chains (a tile can publish exchange X of step t+2 only after every tile of its row
// has consumed X of step t), the LDS hand-offs by explicit flags (pf before wave 0 refolds
// cbd, ef before a chain wave refills qbuf / pbuf / rbuf, qf[0](t-1) before wave 4 refolds
// encfold).
//
// Every wait is bounded (kPassWaitTicks of wall time) and a timed-out wait raises g_pass_abort so the whole grid
// drains promptly; the host reads g_split_fault (nfdpf_split_fault) and fails loudly.
//
// Reductions have a fixed order (deterministic): A / B = per chain wave DPP sums, the row
// total over (tile, wave) in order -- the order of the three-launch tiled path (tiled_front_kernel
// -> store_sums4, block_sum_roles_store -> tiled_ctx); the tile's softmax partial = the quad
// launch's merge over encoder waves 8..15.

namespace nfdpf {

constexpr int kPassMaxTiles = 4;   // N <= 1024: one poll sweep of <= 192 granules per exchange
constexpr int kPassMaxT = 4000;    // tag = (epoch << 12) + t + 1
constexpr uint32_t kPassEpochMask = (1u << 20) - 1;  // the epoch's 20 bits of the 32-bit tag
// the sharded gated pass's cross-rank gate exchange (d.gate_peers, nfdpf_gate_xchg_alloc): a
// 256-B header (word 0: the exchange's pass epoch), then [2][B_global] tagged granules
constexpr int kXgMaxRows = 512;
constexpr int kXgHdr = 32;  // header, in granules
constexpr int kGA = 8;             // granules per flow-wave publish: 4 doubles
constexpr int kGC = 6;             // per encoder-wave publish: max (f32), sum e, sum e^2 (f64), pad

// The pass workspace's first 256 bytes (zeroed by the caller when the workspace is new or its
// (B, N, T) layout changed, include/nfdpf.h): the granule tags' epoch -- bumped by the epilogue
// of every pass, so consecutive passes (and graph replays) never read each other's granules --,
// the abort word a timed-out wait raises to drain the grid (cleared by the epilogue), and the
// epilogue's arrival counter.  Per workspace: two passes on two streams with two workspaces do
// not interfere.
struct PassHdr {
  uint32_t epoch;
  int abort;
  uint32_t done;
};

#ifdef NFDPF_EXP_PTRACE
// experiment-only: per-step phase timestamps (s_memrealtime, 100 MHz) of waves 0, 1 and 8 of
// every workgroup, steps < 64 (scripts/archive/exp_ptrace.py)
__device__ unsigned long long g_ptrace[256][16][64][20];
#define PT(t, k)                                                                                   \
  do {                                                                                             \
    const int w_ = threadIdx.x >> 6, wi_ = w_;          \
    const int wg_ = (b) * gridDim.x + (tile); /* logical (row, tile) */                              \
    if (wi_ >= 0 && (threadIdx.x & 63) == 0 && wg_ < 256 && (t) < 64)                             \
      g_ptrace[wg_][wi_][(t)][(k)] = __builtin_amdgcn_s_memrealtime();                             \
  } while (0)
#else
#define PT(t, k) \
  do {           \
  } while (0)
#endif

// SPEC: the prior wave, not the chain, stores the step's histories (hist_x, noise, index, jac):
// five vector stores per step off the chain's critical path (experiment knob)
#ifndef NFDPF_PASS_HSTORE
#define NFDPF_PASS_HSTORE 1
#endif
// SPEC: the next step's motion and exchange A published at the end of the step, before its
// commit (A/B: pass 0.595-0.614 vs 0.621-0.630 ms, three pairs on one box)
#ifndef NFDPF_PASS_PRE
#define NFDPF_PASS_PRE 1
#endif

// pass modes (tiled_pass_kernel<MODE>)
constexpr int kModeSpec = 0;   // every ESS gate taken as off (verified after the pass)
constexpr int kModeForce = 1;  // --force-resample: the row resampled at the top of every step
constexpr int kModeGate = 2;   // the batch-global ESS gate decided inside the launch, every step

struct PassWs {
  PassHdr *hdr;
  // exchanges A and B by [variant][step parity]: variant 0 = the step without resampling, 1 = the
  // step after the row's resampling (kModeGate: a step speculated as not resampling and then
  // redone leaves variant 0 granules behind that nobody waits for any more)
  uint64_t *ga;  // [2][2][B][tiles][4 role-0 flow waves][kGA]  exchange A (x_phys sums)
  uint64_t *gb;  // [2][2][B][tiles][4][kGA]                   exchange B (x_dyn sums)
  uint64_t *gc;  // [2][B][tiles][8 encoder waves][kGC]         exchange C (softmax partials)
  uint64_t *ge;  // [2][B] kModeGate: each row's 1 / sum p^2 of slot s (by the parity of s)
  double *fin;   // [B][T][tiles * 8][4] per encoder wave: sum p^2, sum p x0, sum p x1, sum logw
  // forced resampling (FORCE): slot s's unnormalised log-weights, written through (sc1) by the
  // encoder waves before their C(s) granules, by slot parity
  float *gu;    // [2][B][N]
  double *eq;   // [T] the epilogue's per-step obs-likelihood terms
  int32_t *eg;  // [T] the epilogue's per-step gates
  uint64_t wait_ticks;  // the bound of every wait (s_memrealtime ticks; kPassWaitTicks)
  // the first row of this launch: a speculative or forced pass of more rows than the device
  // holds at once runs as several launches of resident rows (pass_launch_rows), every table
  // indexed by the batch row row0 + the grid's row
  int row0;
};

__host__ __device__ static inline int64_t pass_granule_bytes(int B, int N) {
  const int64_t bt = (int64_t)B * n_tiles(N);
  auto a256 = [](int64_t v) { return (v + 255) / 256 * 256; };
  return a256(4 * bt * 4 * kGA * 8) * 2 + a256(2 * bt * 8 * kGC * 8) + a256(2 * (int64_t)B * 8);
}

static int64_t pass_bytes(int B, int N, int T) {
  const int64_t bt = (int64_t)B * n_tiles(N);
  return 256 + pass_granule_bytes(B, N) + al256(bt * T * 8 * 32) + al256(2 * (int64_t)B * N * 4) +
         al256((int64_t)T * 8) + al256((int64_t)T * 4);
}

static PassWs pass_carve(void *ws, int B, int N, int T) {
  char *p = (char *)ws;
  const int64_t bt = (int64_t)B * n_tiles(N);
  PassWs w;
  w.row0 = 0;
  w.hdr = (PassHdr *)p;
  p += 256;
  w.ga = (uint64_t *)p;
  p += al256(4 * bt * 4 * kGA * 8);
  w.gb = (uint64_t *)p;
  p += al256(4 * bt * 4 * kGA * 8);
  w.gc = (uint64_t *)p;
  p += al256(2 * bt * 8 * kGC * 8);
  w.ge = (uint64_t *)p;
  p += al256(2 * (int64_t)B * 8);
  w.fin = (double *)p;
  p += al256(bt * T * 8 * 32);
  w.gu = (float *)p;
  p += al256(2 * (int64_t)B * N * 4);
  w.eq = (double *)p;
  p += al256((int64_t)T * 8);
  w.eg = (int32_t *)p;
  return w;
}

// forced resampling of the row (FORCE), at the top of a step while no wave is encoding
struct PassRs {
  float pl[kPassMaxTiles * kTile];   // the row's weights of the previous slot
  float qr[kPassMaxTiles * kTile];   // their mixture q_raw (SoftRow::q_raw, written beside pl)
  float cdf[kPassMaxTiles * kTile];  // its CDF (soft_row_search)
  float wg[kPassMaxTiles * kTile];   // the gathered weights w[idx_i] of every marker i
  float xr_l[kTile][2];              // source position,
  int src_l[kTile];                  // source index (N: the reference's out-of-range edge)
  double shd[16];
  float shf[16];
};
struct PassLds {
  union {
    float Hws[8][32 * kHPitch];    // each encoder wave's MFMA layer outputs
    PassRs rs;
  };
  float qbuf[2][2 * kTile];        // the proposal, chain wave -> prior wave + encoder pair, by step parity
  float pbuf[2][2 * kTile];        // x_phys - eps, chain wave -> prior wave
  float rbuf[2][2 * kTile];        // prior (prior wave) | propose (chain wave) -> encoder pair
  float encq[8][kE];               // each encoder wave's copy of the step's frame encoding
  f2 cbd[2][kMaxFlows * 2 * kH];   // nf_dyn folded biases (split order), by step parity
  f2 cbc[2][kMaxFlows * 2 * kH];   // proposal folded biases (split order)
  float encfold[2][kMaxFlows * 4 * kH];  // proposal fold over the encoding columns (pair order)
  uint32_t rowa[kPassMaxTiles * 4 * kGA];  // wave 0's A / B sweep
  uint32_t rowc[kPassMaxTiles * 8 * kGC];  // wave 8's C sweep
  RowNorm rn[2];                   // slot s's row normaliser, by parity of s
  int fA, fB, fE, fR;              // step-tagged flags (see the header comment; fA / fB: 4 (t + 1) + code)
  int qf[4], rf[4];
  alignas(8) int pf[4];
  alignas(8) int ef[8];
#if NFDPF_PASS_HSTORE
  float ebuf[2][3 * kTile];        // SPEC: the chain's motion noise and log|det J|, to the prior wave
#endif
  float lr_l[kTile];               // FORCE / GATE: this tile's resampled log-weights (outside the union:
                                   // the encoder waves read it while others may start their MFMA layers)
  int fS, fbar;                    // FORCE: resampling done, flow-wave barrier
  // kModeGate: the decisions (dec[t & 1] of step t, valid once fD >= t + 1; wave 8), the chain's
  // redo request to the prior waves (rq = t + 1: join the row's resampling of step t), each chain
  // wave's "slot t - 1's hist_x stores have landed" (hxf[g] = t), wave 8's batch sweep
  int fD, rq;
  int dec[2];
  int hxf[4];
  uint32_t rowe[kXgMaxRows];       // (B_global rows: the sharded gated pass's sweep of every rank's rows)
};

// A loop-invariant lane value made opaque inside a persistent step loop: the compiler would
// otherwise hoist the 64-bit addresses derived from it out of the loop and, short of VGPRs,
// spill them to scratch (reloaded every step on the critical path)
__device__ __forceinline__ int opaque_int(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

__device__ __forceinline__ void gran_store(uint64_t *g, uint32_t data, uint32_t tag) {
  __hip_atomic_store(g, ((uint64_t)tag << 32) | data, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// The kernel's arguments re-read from the kernarg segment where needed: LICM would otherwise
// keep every step-invariant field and address live in SGPRs across the step loop, and the
// nets' weight loads would then spill them through VGPR lanes (v_writelane / v_readlane around
// every coupling)
typedef const __attribute__((address_space(4))) nfdpf_filter_desc kdesc_t;
typedef const __attribute__((address_space(4))) PassWs kws_t;
__device__ __forceinline__ kdesc_t *kernarg_desc() {
  kdesc_t *p = (kdesc_t *)__builtin_amdgcn_kernarg_segment_ptr();
  asm volatile("" : "+s"(p));
  return p;
}
__device__ __forceinline__ kws_t *kernarg_ws() {
  constexpr size_t off = (sizeof(nfdpf_filter_desc) + alignof(PassWs) - 1) / alignof(PassWs) * alignof(PassWs);
  kws_t *p = (kws_t *)((const __attribute__((address_space(4))) char *)__builtin_amdgcn_kernarg_segment_ptr() + off);
  asm volatile("" : "+s"(p));
  return p;
}

// A bounded spin: false once the wait has timed out (counted once, and the whole grid told to
// drain through the workspace's abort word) or another wave's has.  The bound is wall time
// (s_memrealtime, 100 MHz): kPassWaitTicks from the wait's first miss, far above any legitimate
// wait (a step takes ~20 us) and short enough that a grid that cannot make progress drains
// within a second.  (NFDPF_PASS_WAIT_US overrides it per call: tests force the timeout path.)
constexpr uint64_t kPassWaitTicks = 20000000ull;  // 200 ms
struct Spin {
  uint64_t t0 = 0;
  int it = 0;
};
#ifndef NFDPF_PASS_FLAG_SLEEP
#define NFDPF_PASS_FLAG_SLEEP 1
#endif
template <int SLEEP = 1>
__device__ __forceinline__ bool pass_spin(Spin &s) {
  if ((s.it++ & 63) == 0) {
    int *abort_w = &kernarg_ws()->hdr->abort;
    if (__hip_atomic_load(abort_w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return false;
    const uint64_t now = __builtin_amdgcn_s_memrealtime();
    if (s.it == 1) {
      s.t0 = now;
    } else if (now - s.t0 > kernarg_ws()->wait_ticks) {
      if ((int)(threadIdx.x & 63) == __ffsll((unsigned long long)__ballot(1)) - 1) {  // first active lane
        atomicAdd(&g_split_fault, 1);
        __hip_atomic_store(abort_w, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      return false;
    }
  }
  __builtin_amdgcn_s_sleep(SLEEP);
  return true;
}

// wait until the LDS flag reaches v (wave-uniform)
__device__ __forceinline__ void wait_flag(const int *f, int v) {
  Spin s;
  while (__builtin_amdgcn_readfirstlane(*(lds_vint *)f) < v && pass_spin<NFDPF_PASS_FLAG_SLEEP>(s)) {
  }
  asm volatile("" ::: "memory");
}
// publish an LDS flag after this wave's LDS data writes have landed
__device__ __forceinline__ void set_flag(int *f, int v) {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  *(lds_vint *)f = v;
#ifdef NFDPF_PASS_WAKE
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_wakeup" ::: "memory");
#endif
}

// four wave-uniform doubles as 8 granules (lanes 0..7: value l / 2, low / high word by l & 1)
__device__ __forceinline__ void publish4(uint64_t *g, const double (&v)[4], uint32_t tag) {
  const int l = threadIdx.x & 63;
  if (l < 8) {
    const int k = l >> 1;
    const double x = k == 0 ? v[0] : k == 1 ? v[1] : k == 2 ? v[2] : v[3];
    const uint64_t bits = (uint64_t)__double_as_longlong(x);
    gran_store(g + l, (l & 1) ? (uint32_t)(bits >> 32) : (uint32_t)bits, tag);
  }
}

// one wave sweeps granules [0, n) of a row (n <= 64 NC) until every tag is `tag`, leaving the
// data words in dst (LDS): 0; 1 on abort; 2 when `stop()` (an LDS read, checked between sweeps)
// became true first (kModeGate: the step being speculated must be redone).
// `work` (register-only arithmetic) runs once while the first sweep's loads are in flight.
struct NoWork {
  __device__ void operator()() const {}
};
struct NoStop {
  __device__ bool operator()() const { return false; }
};
template <int NC = 3, class Work = NoWork, class Stop = NoStop, int SCOPE = __HIP_MEMORY_SCOPE_AGENT>
__device__ int poll_rowx(const uint64_t *g, int n, uint32_t tag, uint32_t *dst, Work work = Work(),
                         Stop stop = Stop()) {
  const int l = threadIdx.x & 63;
  uint64_t v[NC];
  bool ok[NC];
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    v[c] = 0;
    ok[c] = 64 * c + l >= n;
  }
  Spin sp;
  auto sweep = [&]() {
#pragma unroll
    for (int c = 0; c < NC; ++c)
      if (!ok[c]) v[c] = __hip_atomic_load(g + 64 * c + l, __ATOMIC_RELAXED, SCOPE);
  };
  sweep();
  work();
  for (;;) {
    bool all = true;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (!ok[c]) ok[c] = (uint32_t)(v[c] >> 32) == tag;
      all = all && ok[c];
    }
    if (__all(all)) break;
    if (stop()) return 2;
    if (!pass_spin(sp)) return 1;
    sweep();
  }
#pragma unroll
  for (int c = 0; c < NC; ++c)
    if (64 * c + l < n) dst[64 * c + l] = (uint32_t)v[c];
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  return 0;
}
template <class Work = NoWork>
__device__ bool poll_row(const uint64_t *g, int n, uint32_t tag, uint32_t *dst, Work work = Work()) {
  return poll_rowx<3>(g, n, tag, dst, work) == 0;
}

__device__ __forceinline__ double lds_double(const uint32_t *w, int q) {
  return __longlong_as_double((long long)(((uint64_t)w[q + 1] << 32) | w[q]));
}

// the row context from an A / B sweep: lanes c < 4 add component c over (tile, wave) in order
// (block_sum_roles_store, then tiled_ctx), every lane gets the context
__device__ __forceinline__ Ctx4 row_ctx(const uint32_t *rw, int tiles, double inv_n, double inv_n1) {
  const int c = threadIdx.x & 3;
  double a = 0.0;
  for (int k = 0; k < tiles; ++k) {
    double tk = lds_double(rw, (k * 4 + 0) * kGA + 2 * c);
#pragma unroll
    for (int g = 1; g < 4; ++g) tk += lds_double(rw, (k * 4 + g) * kGA + 2 * c);
    a += tk;
  }
  // ctx_from_sums's arithmetic with its two components on two lanes (lane k: mean and std of
  // component k); the selects branch-free (both readlanes uniform, then one v_cndmask per half)
  const int k = threadIdx.x & 1;
  const double s0 = readlane_d(a, 0), s1 = readlane_d(a, 1), q0 = readlane_d(a, 2), q1 = readlane_d(a, 3);
  const double s = k ? s1 : s0, q = k ? q1 : q0;
  const double m = ctx_mean(s, inv_n);
  const float sd = (float)sqrt(ctx_var(s, q, m, inv_n1));
  const float mf = (float)m;
  return Ctx4{readlane_f(mf, 0), readlane_f(mf, 1), readlane_f(sd, 0), readlane_f(sd, 1)};
}
// wait until both adjacent LDS flags f[0], f[1] reach v (one 8-byte read per poll)
__device__ __forceinline__ void wait_flag2(const int *f, int v) {
  Spin s;
  for (;;) {
    const uint64_t w = *(volatile __attribute__((address_space(3))) uint64_t *)f;
    const int a = __builtin_amdgcn_readfirstlane((int)(uint32_t)w), c = __builtin_amdgcn_readfirstlane((int)(w >> 32));
    if ((a >= v && c >= v) || !pass_spin<NFDPF_PASS_FLAG_SLEEP>(s)) break;
  }
  asm volatile("" ::: "memory");
}

// the motion noise of step t (motion_noise's device-RNG branch with an explicit step)
__device__ __forceinline__ void pass_noise(const nfdpf_filter_desc &d, int t, int64_t grow, int i, float &e0,
                                           float &e1) {
  const U4 r = rng_draw(d.seed, kTagMotion, (uint32_t)t, grow, (uint32_t)i);
  box_muller(r.x, r.y, e0, e1);
  e0 *= d.pos_noise;
  e1 *= d.pos_noise;
}

// write-through (sc1) stores of slot values another tile reads (FORCE)
__device__ __forceinline__ void store_wt(float *p, float v) {
  __hip_atomic_store(reinterpret_cast<uint32_t *>(p), __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void store_wt2(float *p, float a, float b) {  // p 8-B aligned
  __hip_atomic_store(reinterpret_cast<uint64_t *>(p), ((uint64_t)__float_as_uint(b) << 32) | __float_as_uint(a),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float load_wt(const float *p) {
  return __uint_as_float(__hip_atomic_load(reinterpret_cast<const uint32_t *>(p), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void load_wt2(const float *p, float &a, float &b) {
  const uint64_t v =
      __hip_atomic_load(reinterpret_cast<const uint64_t *>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  a = __uint_as_float((uint32_t)v);
  b = __uint_as_float((uint32_t)(v >> 32));
}

// barrier of the 8 flow waves (the encoder waves run their own loop meanwhile): each wave adds
// to a monotonic LDS counter once its LDS writes have landed, then waits for the round's total
__device__ __forceinline__ void flow_barrier(int *cnt, int &round) {
  round += 8;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  if ((threadIdx.x & 63) == 0) atomicAdd(cnt, 1);
#ifdef NFDPF_PASS_WAKE
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_wakeup" ::: "memory");
#endif
  wait_flag(cnt, round);
}

// ---- FORCE: the soft resampling of the row at the top of step t (resamplers.py:20-60, the
// soft.hpp recipe: bit-exact indices), by the 8 flow waves (512 threads) while the encoder
// waves wait for its log-weights (flag fS).  Input: slot t-1's normalised weights (hist_p,
// normalised here from the row's unnormalised log-weights, gu) and particles (hist_x) of the
// whole row, both written through (sc1) by the row's tiles before the C(t-1) granules that wave
// 8 has swept when it sets fR(t-1): an encoder wave publishes its granule after its own gu
// stores and vmcnt(0), and after its chain wave's qf(t-1), which that wave sets behind its own
// hist_x stores and vmcnt(0) (MI355X_MICROARCH.md inter-workgroup visibility, row 1; the sweeping
// wave, then an LDS word it sets, then sc1 loads) -- or the initial state at t = 0.  The weights
// are pass_norm's expression on the same u and row normaliser, so bit-equal to hist_p.  Every
// tile searches all N markers (the gathered weights' renormaliser is a cascade sum over the whole
// row in ATen's order) and keeps its own particles' source, position and log-weight in LDS.
// History slots are never overwritten inside the pass, so the rare read of the NEXT row's first
// particle (the reference's out-of-range edge, src == N) only waits for that row's tile-0
// encoder wave 0 to have published C(t-1) or a later C.
// fR(t-1) also means that every encoder wave of this tile has finished its MFMA layers of step
// t-1 (it publishes C(t-1) after them): the resampling scratch (PassRs) aliases their LDS.
#ifndef NFDPF_GATE_LATE
#define NFDPF_GATE_LATE 1
#endif
// late = true (FORCE; GATE unless NFDPF_GATE_LATE=0): the tail needs no barrier -- each chain
// wave gathers its own slots' sources (slot == tid) and reads them back itself, and wave 7, a
// prior wave idle until the proposal, sums the gathered weights and writes lr_l, then raises fS:
// the encoder waves wait for fS before their MFMA layers reuse this scratch (GATE: after the
// chain's commit, when step t or t - 1 fired).
__device__ __forceinline__ void pass_resample(const nfdpf_filter_desc &d, const PassWs &ws, PassLds &L, int b,
                                              int tile, uint32_t tag0, int t, int &round, bool late) {
  PassRs &R = L.rs;
  const int N = d.N, tiles = n_tiles(N), tid = threadIdx.x, nth = 8 * 64;
  const int64_t grow = d.row_base + b;
  const uint32_t tag = tag0 + (uint32_t)t;  // C(t - 1)'s
  const float *xs;  // the previous slot's particles of this row
  int64_t xs_next;  // ... and the offset of the next row's
  // the marker phase's inputs, in flight before the wait for the row's weights: markers tid and
  // tid + 512 (N <= 1024) of the fixed linspace, the step's offset draw
  const int ia = tid, ib = tid + nth;
  const bool va = ia < N, vb = ib < N;
  const float lin_a = va ? d.lin[ia] : 0.f, lin_b = vb ? d.lin[ib] : 0.f;
  const float off = u01(rng_draw(d.seed, kTagOffset, (uint32_t)t, grow, 0u).x) * (1.0f / (float)N);
  // soft_row_search's steps on 512 threads (soft.hpp); q_raw of every weight kept beside it
  SoftRow row{R.pl, N, d.alpha, 1.0f / (float)N, (float)(1.0 - (double)d.alpha), 1.0f};
  const bool mix = row.alpha < 1.0f;
  auto put = [&](int j, float pj) {
    R.pl[j] = pj;
    R.qr[j] = row.q_raw_of(pj);
  };
  if (t > 0) {
    wait_flag(&L.fR, t);  // wave 8 has swept C(t - 1): slot t - 1's row normaliser in L.rn
    PT(t, 12);
    const RowNorm rn = L.rn[(t - 1) & 1];
    const float *us = ws.gu + ((int64_t)((t - 1) & 1) * d.B + b) * N;
    for (int j = tid; j < N; j += nth) put(j, expf(load_wt(us + j) - rn.shift) / rn.Ssum + 1e-12f);  // pass_norm's p
    xs = d.hist_x + ((int64_t)b * d.T + t - 1) * N * 2;
    xs_next = (int64_t)d.T * N * 2;
  } else {
    for (int j = tid; j < N; j += nth) put(j, d.p_prev[(int64_t)b * d.p_prev_rs + j]);
    xs = d.x_prev + (int64_t)b * d.x_prev_rs;
    xs_next = d.x_prev_rs;
  }
  flow_barrier(&L.fbar, round);
  PT(t, 13);
  // SoftRow's q and w on the stored q_raw (the same values, not recomputed)
  auto qv = [&](int j) { return mix ? R.qr[j] / row.S : R.pl[j]; };
  auto wv = [&](int j) { return mix ? R.pl[j] / qv(j) : row.u; };
  if (mix) {
    if (tid < 64) {
      PT(t, 19);
      const float S = (N >= 8 ? cascade_row_sum_1k<kPassMaxTiles * kTile>([&](int j) { return R.qr[j]; }, N)
                              : cascade_row_sum([&](int j) { return R.qr[j]; }, N));
      if (tid == 0) R.shf[0] = S;
      PT(t, 11);
    }
    flow_barrier(&L.fbar, round);
  PT(t, 14);
    row.S = R.shf[0];
  }
  // the exact f64 prefix of q: 2 consecutive j per thread (N <= 1024), wave scans, wave order
  {
    const int j0 = 2 * tid;
    const double a = j0 < N ? (double)qv(j0) : 0.0, c = j0 + 1 < N ? (double)qv(j0 + 1) : 0.0;
    const double part = a + c;
    const int lane = tid & 63, w = tid >> 6;
    // f64 sums of fp32 q terms: with the uniform mixture every q >= (1 - alpha) / (N S) and the
    // partial sums stay below ~1, so when that floor is >= 2^-19 every partial sum is exact and the
    // DPP scan's addition order gives the bits of any order; otherwise the shfl_up scan
    double inc = part;
    if ((1.0f - row.alpha) * row.u >= 0x1p-18f) {
      inc = wave_incl_scan_dpp_d(part);
    } else {
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const double u = __shfl_up(inc, o);
        if (lane >= o) inc += u;
      }
    }
    if (lane == 63) R.shd[w] = inc;
    flow_barrier(&L.fbar, round);
  PT(t, 15);
    double base = 0.0, sh[8];  // (the 8 wave totals loaded at once, then added in wave order)
#pragma unroll
    for (int k = 0; k < 8; ++k) sh[k] = R.shd[k];
#pragma unroll
    for (int k = 0; k < 8; ++k)
      if (k < w) base += sh[k];
    double run = base + inc - part;
    if (j0 < N) {
      run += a;
      R.cdf[j0] = (float)run;
    }
    if (j0 + 1 < N) {
      run += c;
      R.cdf[j0 + 1] = (float)run;
    }
  }
  flow_barrier(&L.fbar, round);
  PT(t, 16);
  const int i0 = tile * kTile;
  {  // markers tid and tid + 512 (N <= 1024), their two searches interleaved (two LDS probes in
     // flight per step instead of one search after the other); the same lower bound
    const float ma = va ? off + lin_a : 0.f, mb = vb ? off + lin_b : 0.f;
    // branch-free lower bound (the first j with cdf[j] >= m, N if none) in fixed halving steps,
    // clamped to N - 1: the binary search's result, without divergent loop exits
    int loa = 0, lob = 0;
#pragma unroll
    for (int step = kPassMaxTiles * kTile / 2; step >= 1; step >>= 1) {
      const int ja = loa + step - 1, jb = lob + step - 1;
      const float ca = R.cdf[min(ja, N - 1)], cb = R.cdf[min(jb, N - 1)];
      loa += (ja < N && ca < ma) ? step : 0;
      lob += (jb < N && cb < mb) ? step : 0;
    }
    loa = min(loa, N - 1);
    lob = min(lob, N - 1);
    // sj == N: the reference's out-of-range edge (next row's first particle, weight 0)
    if (va) {
      const int sj = loa + (1.0f < ma ? 1 : 0);
      R.wg[ia] = sj < N ? wv(sj) : 0.f;
      if (ia >= i0 && ia < i0 + kTile) R.src_l[ia - i0] = sj;
    }
    if (vb) {
      const int sj = lob + (1.0f < mb ? 1 : 0);
      R.wg[ib] = sj < N ? wv(sj) : 0.f;
      if (ib >= i0 && ib < i0 + kTile) R.src_l[ib - i0] = sj;
    }
  }
  PT(t, 6);
  flow_barrier(&L.fbar, round);
  PT(t, 17);
  // the tile's sources' positions (their loads in flight while wave 0 sums the gathered weights),
  // then wave 0 turns every particle of the tile into its resampled log-weight
  if (tid < kTile && i0 + tid < N) {
    // (clamped: after an abort the barriers no longer order anything and src_l may hold stale
    // LDS words -- an address must never come from them)
    const int sj = min(max(R.src_l[tid], 0), N);
    const float *src = xs + 2 * (sj < N ? sj : N - 1);
    if (sj >= N && b + 1 < d.B) {
      src = xs + xs_next;
      if (t > 0) {  // row b + 1's tile-0 encoder wave 0 has published C(t - 1) (or a later C)
        const uint64_t *g = ws.gc + ((((int64_t)((t - 1) & 1) * d.B + b + 1) * tiles) * 8) * kGC;
        Spin sp;
        for (;;) {
          const uint32_t v = (uint32_t)(__hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> 32);
          if ((v >= tag && v < tag0 + (1u << 12)) || !pass_spin(sp)) break;
        }
      }
    }
    float x0, x1;
    if (t > 0) {
      load_wt2(src, x0, x1);
    } else {
      x0 = src[0];
      x1 = src[1];
    }
    R.xr_l[tid][0] = x0;
    R.xr_l[tid][1] = x1;
  }
  PT(t, 10);
  const int sw = late ? nth - 64 : 0;  // the wave that sums the gathered weights
  if (tid >= sw && tid < sw + 64) {
    const float s2 = (N >= 8 ? cascade_row_sum_1k<kPassMaxTiles * kTile>([&](int j) { return R.wg[j]; }, N)
                             : cascade_row_sum([&](int j) { return R.wg[j]; }, N));
    PT(t, 9);
#pragma unroll
    for (int k = 0; k < kTile / 64; ++k) {
      const int s = k * 64 + tid - sw;
      if (i0 + s < N) L.lr_l[s] = logf(R.wg[i0 + s] / s2);
    }
  }
  if (!late) flow_barrier(&L.fbar, round);
  PT(t, 18);
  if (tid >= sw && tid < sw + 64) set_flag(&L.fS, t + 1);  // the encoder waves may read lr_l
}

// The pass's (row, tile) of this workgroup: a row's tiles on ONE XCD where the grid allows
// (workgroups are dealt round-robin over the 8 XCDs: ids x, x + 8, ... share one), so the
// row's exchanges never wait on a tile that another XCD's load or clock holds back (+0.9 % at
// C2 on one box; any bijection is correct -- placement is for speed only)
__device__ __forceinline__ void pass_tile_row(int &b, int &tile) {
  const int n = gridDim.x * gridDim.y, id = blockIdx.x + gridDim.x * blockIdx.y;
  const int lin = (n & 7) == 0 ? (id & 7) * (n >> 3) + (id >> 3) : id;
  tile = lin % gridDim.x;
  b = lin / gridDim.x + kernarg_ws()->row0;
}

// Rows of (tiles) workgroups of `kern` the device holds at once (0: not even one row, or the
// query failed)
template <class K>
static int pass_resident_rows(K kern, int threads, int tiles) {
  int dev = 0, cus = 0, occ = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, kern, threads, 0) != hipSuccess || occ < 1)
    return 0;
  return (int)((int64_t)cus * occ / tiles);
}

// Launch `kern` over the pass's rows in chunks of `rows` resident rows (one launch when all fit),
// the LAST chunk first: a row reads nothing of another row except, in the forced pass, the next
// row's slot t - 1 particles at the reference's out-of-range edge (pass_resample) -- which a
// later chunk has then written in full, every granule tag of it at or past the one waited for.
// (The gated pass's rows wait for the batch's decision: it is never chunked.)  The profiling
// events (if any) bracket the first launch and the last.
template <class K>
static void pass_launch_rows(K kern, const nfdpf_filter_desc &d, PassWs ws, int threads, int rows,
                             hipStream_t st) {
  hipEvent_t *ev = (hipEvent_t *)d.prof_events;
  const int tiles = n_tiles(d.N), nch = (d.B + rows - 1) / rows;
  for (int c = nch - 1; c >= 0; --c) {
    const int r0 = c * rows;
    ws.row0 = r0;
    const dim3 g(tiles, std::min(rows, d.B - r0));
    hipEvent_t e0 = ev && c == nch - 1 ? ev[0] : nullptr, e1 = ev && c == 0 ? ev[1] : nullptr;
    if (e0 || e1)
      hipExtLaunchKernelGGL(kern, g, dim3(threads), 0, st, e0, e1, 0, d, ws);
    else
      kern<<<g, threads, 0, st>>>(d, ws);
  }
}

// ---- waves 0-7: the flows, one wave per particle group and stage ---------------------------
// The t- and s-nets of one coupling half on input u from the PASS layout (nfdpf.pack.
// pass_coupling_tensors: the pair layout of flows.hpp ts_pair, HALF = 1 -- one v_pk_fma_f32
// advances hidden unit j of both nets -- with the tanh algebra folded into the weights): every
// hidden unit is r = 1 / (1 + 2^y) of its scaled argument y (tanh = 1 - 2 r, the -2 and the next
// layer's 2 log2(e) live in the weights), so a unit costs exp2 + add + rcp: the tanh2 of the step
// launches' layout also multiplies by 2 log2(e) and evaluates 1 - 2 r (two packed ops per unit
// pair more).  Layer 3 summed the way split.hpp's net_split sums it (even and odd hidden units in
// two chains, then (even + odd) + b3).  cb = the half's folded bias pairs (fold_ref order).
#ifndef NFDPF_PASS_SB
#define NFDPF_PASS_SB 1
#endif
// {1 / (1 + 2^y.x), 1 / (1 + 2^y.y)}: 2^y = inf -> 0, 2^y = 0 -> 1 (no NaN anywhere)
__device__ __forceinline__ f2 sig2(f2 y) {
  const f2 d = f2{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)} + splat(1.0f);
  return f2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)};
}
__device__ __forceinline__ f2 ts_half(cf2 *w, float u, const f2 *cb) {
#if NFDPF_PASS_SB
  __builtin_amdgcn_sched_barrier(0);  // no weight loads hoisted from here into the previous half
#endif
  f2 h[kH];
#pragma unroll
  for (int j = 0; j < kH; ++j) h[j] = sig2(pfma(w[j], splat(u), cb[j]));
  cf2 *w2 = w + kH;
  f2 g[kH];
#pragma unroll
  for (int j = 0; j < kH; ++j) {
    f2 a = w2[kH * kH + j];
#pragma unroll
    for (int k = 0; k < kH; ++k) a = pfma(w2[j * kH + k], h[k], a);
    g[j] = sig2(a);
  }
  cf2 *w3 = w2 + kH * kH + kH;
  f2 e = w3[0] * g[0], o = w3[1] * g[1];
#pragma unroll
  for (int m = 1; m < kH / 2; ++m) {
    e = pfma(w3[2 * m], g[2 * m], e);
    o = pfma(w3[2 * m + 1], g[2 * m + 1], o);
  }
  return (e + o) + w3[kH];
}
// RealNVP_cond flow inverse (nf/flows.py:228-239) / forward (:215-226) on one wave: fw = the
// flow's pair-layout block (half 1 at fw, half 2 at fw + ns), cb = its 16 folded bias pairs
// (half 2 at cb + kH); the update arithmetic of split.hpp's coupling_*_split
// exp(s) of the coupling update: expf, as split.hpp's step launches.  (One v_exp_f32 of s log2(e)
// measured neutral on the pass's time, and its extra rounding of s log2(e) took the forced pass's
// indices against the step launches' from > 99 % to 94 % agreement over 8 steps of resampling --
// test_split_nets_match_pair_layout: not worth it.)
__device__ __forceinline__ float exp_s(float s) { return expf(s); }
__device__ __forceinline__ float pass_inverse(cf2 *fw, int ns, float &lo, float &up, const f2 *cb) {
  f2 ts = ts_half(fw + ns, up, cb + kH);
  lo = (lo - ts.x) * exp_s(-ts.y);
  const float l2 = -ts.y;
  ts = ts_half(fw, lo, cb);
  up = (up - ts.x) * exp_s(-ts.y);
  return -ts.y + l2;
}
__device__ __forceinline__ float pass_forward(cf2 *fw, int ns, float &lo, float &up, const f2 *cb) {
  f2 ts = ts_half(fw, lo, cb);
  up = ts.x + up * exp_s(ts.y);
  const float l1 = ts.y;
  ts = ts_half(fw + ns, up, cb + kH);
  lo = ts.x + lo * exp_s(ts.y);
  return l1 + ts.y;
}

// kModeGate: the prediction of step t's decision from the decisions so far -- a 2-bit saturating
// counter per history of the last two decisions (bits 0-1: the history, last decision in bit 0;
// bits 2 + 2h: counter h).  The chain, prior and encoder waves each keep a copy, updated with the
// same committed decisions, so all predict alike (the row's resampling barriers match).  It starts
// as "the previous step's decision" and learns e.g. the alternation of a filter whose resampling
// restores the ESS for a step (c2_full: 17 of 50 steps fire, every other one).
struct GatePred {
  int s = (1 << 2) | (2 << 4) | (1 << 6) | (2 << 8);
  __device__ __forceinline__ int get() const { return ((s >> (2 + 2 * (s & 3))) & 3) >= 2 ? 1 : 0; }
  __device__ __forceinline__ void update(int d) {
    const int h = s & 3, sh = 2 + 2 * h;
    int c = (s >> sh) & 3;
    c = d ? min(c + 1, 3) : max(c - 1, 0);
    s = (s & ~(3 << sh)) | (c << sh);
    s = (s & ~3) | (((h << 1) | (d ? 1 : 0)) & 3);
  }
};

// kModeGate: step t's decision once wave 8 has taken it (fD >= t + 1): 1 = the batch-global ESS
// gate fired (DPFs.py:163-165); the same value in every workgroup of the grid
__device__ __forceinline__ int wait_dec(PassLds &L, int t) {
  wait_flag(&L.fD, t + 1);
  return __builtin_amdgcn_readfirstlane(*(lds_vint *)&L.dec[t & 1]);
}
__device__ __forceinline__ bool dec_fired(PassLds &L, int t) {
  return __builtin_amdgcn_readfirstlane(*(lds_vint *)&L.fD) >= t + 1 &&
         __builtin_amdgcn_readfirstlane(*(lds_vint *)&L.dec[t & 1]) != 0;
}

// waves 0-3 ("chain", group g = w): motion -> A -> nf_dyn inverse -> B -> proposal inverse, the
// path from one step's particles to the next's; the proposal goes to the group's prior wave and
// encoder pair through LDS (qbuf, pbuf, rbuf's propose half; flag qf[g]).
// kModeGate: the step's gate is decided by wave 8 from slot t - 1 (after the C(t - 1) sweep, one
// batch-wide granule sweep); the chain PREDICTS it from step t - 1's decision:
//   * predicted to fire: the row is resampled first (as kModeForce, the 8 flow waves), then the
//     decision -- known by then -- picks the resampled or the own particles;
//   * predicted not to fire: the step runs on the own particles at once (variant 0) and the
//     decision is checked while wave 0 waits for A / B and before anything is committed; if the
//     gate fired after all, the attempt is dropped, the prior waves are called in (rq) and the
//     step is redone after the row's resampling (variant 1: its own exchange buffers).
// Nothing of step t leaves the chain (histories, qbuf, qf) before its decision is known, so the
// prior and encoder waves only ever see the committed step.
template <int MODE>
__device__ __forceinline__ void pass_chain(const nfdpf_filter_desc &d, const PassWs &ws, PassLds &L, int b, int tile,
                                           uint32_t tag0) {
  constexpr bool FORCE = MODE == kModeForce, GATE = MODE == kModeGate;
  const int tiles = n_tiles(d.N), N = d.N, nfl = d.n_flows, ncb = nfl * 4 * kH;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int g = w, slot = g * 64 + lane;
  const int i = tile * kTile + slot;
  const bool valid = i < N;
  const int64_t grow = d.row_base + b;
  float x0 = 0.f, x1 = 0.f;
  if (valid) {
    x0 = d.x_prev[(int64_t)b * d.x_prev_rs + 2 * i];
    x1 = d.x_prev[(int64_t)b * d.x_prev_rs + 2 * i + 1];
  }
  // wave 0 folds both contexts: the weights of the context columns, once per launch
  const bool fold_lane = w == 0 && lane < ncb;
  // the fold weights: held in registers for the whole pass (SPEC), or loaded per step under the
  // exchange's poll (FORCE / GATE: their VGPR pressure spilled the held copies to scratch, whose
  // reloads sat on the fold)
  constexpr bool HOLD = MODE == kModeSpec;
  float fwd[1 + kOctxDyn] = {}, fwc[4] = {};
  auto load_fwd = [&](const nfdpf_filter_desc &dd) {
    const FoldRef r = fold_ref(dd.dyn_params, kNsDyn, lane);
    fwd[0] = fold_bias0(r, kOctxDyn);
#pragma unroll
    for (int c = 0; c < kOctxDyn; ++c) fwd[1 + c] = r.w1c[2 * (r.j * kOctxDyn + c) + r.w];
  };
  auto load_fwc = [&](const nfdpf_filter_desc &dd) {
    const int O = dd.E + 4;
    const FoldRef rc = fold_ref(dd.cond_params, net_size<1, kH>(O), lane);
#pragma unroll
    for (int c = 0; c < 4; ++c) fwc[c] = rc.w1c[2 * (rc.j * O + dd.E + c) + rc.w];
  };
  if (HOLD && fold_lane) {
    load_fwd(d);
    load_fwc(d);
  }
  constexpr int nsd = kNsDyn, nsc = net_size<1, kH>(kE + 4);
  const double inv_n = 1.0 / N, inv_n1 = 1.0 / (N - 1);  // the row contexts' (ctx_from_sums)
  int round = 0;  // flow_barrier rounds (FORCE / GATE)
  GatePred gp;  // GATE: the prediction of step t's decision
  float en0 = 0.f, en1 = 0.f;  // the next step's motion noise
  // the step's velocity, loaded one step ahead (beside the next step's noise): no scalar-load
  // latency at the head of the step
  float nv0 = d.vel[2 * (int64_t)b], nv1 = d.vel[2 * (int64_t)b + 1];
  // SPEC (NFDPF_PASS_PRE): the next step's x_phys / noise, its A already published (pre)
  constexpr bool PRE = NFDPF_PASS_PRE && MODE == kModeSpec;
  float pp0 = 0.f, pp1 = 0.f, pe0 = 0.f, pe1 = 0.f;
  bool pre = false;
  const int i_ = i, slot_ = slot;
  for (int t = 0; t < d.T; ++t) {
    const nfdpf_filter_desc &d = *(const nfdpf_filter_desc *)kernarg_desc();  // (kernarg_desc)
    const PassWs &ws = *(const PassWs *)kernarg_ws();
    const int i = opaque_int(i_), slot = opaque_int(slot_);
    const float K = d.dens_const, two_var = 2.0f * (d.pos_noise * d.pos_noise);
    const int par = t & 1;
    const uint32_t tag = tag0 + (uint32_t)t + 1u;
    const float v0 = nv0, v1 = nv1;
    PT(t, 0);
    if (t == 0 && valid) pass_noise(d, 0, grow, i, en0, en1);
    // the step's input particles: own (x0, x1) or the row's resampling's
    float xs0 = x0, xs1 = x1;
    // the step's motion noise: kept aside -- the first attempt draws step t + 1's into (en0, en1)
    // while its A exchange is in flight, and a redone step (GATE) must move with step t's own
    const float sn0 = en0, sn1 = en1;
    int src = i, variant = 0, fire = FORCE ? 1 : 0;
    // (a plan pass follows d.pass_plan: the decision is known, never speculated)
    const int32_t *plan = GATE ? d.pass_plan : nullptr;
    const int pred = GATE ? (plan ? (plan[t] ? 1 : 0) : t == 0 ? wait_dec(L, 0) : gp.get()) : 0;
    bool known = !GATE || t == 0 || plan;  // the step's decision is in hand (GATE: else speculated)
    auto take_resampled = [&]() {
      if (valid) {
        xs0 = L.rs.xr_l[slot][0];
        xs1 = L.rs.xr_l[slot][1];
        src = min(max(L.rs.src_l[slot], 0), N);  // (a value, never an address; clamped all the same)
      }
    };
    if (FORCE || (GATE && pred)) {  // soft resampling of the row (--force-resample / predicted)
      if (GATE && t > 0) {  // slot t - 1's hist_x stores landed: this tile's C(t - 1) may go out
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        set_flag(&L.hxf[g], t);
      }
      pass_resample(d, ws, L, b, tile, tag0, t, round, FORCE || NFDPF_GATE_LATE);
      if (GATE) {
        fire = plan ? pred : wait_dec(L, t);
        known = true;
      }
      if (fire) take_resampled();
      variant = GATE && fire ? 1 : 0;
    }
    float e0 = 0.f, e1 = 0.f, p0 = 0.f, p1 = 0.f, jac = 0.f, q0 = 0.f, q1 = 0.f, ldp = 0.f;
    // one attempt at step t from (xs0, xs1): 0 done; 2 dropped (GATE: the gate fired while the
    // attempt speculated that it would not; `spec` enables the checks)
    auto attempt = [&](bool first, bool spec) -> int {
      // motion (model/models.py:191-204): x_phys = (x_src + vel) + eps; eps drawn during the
      // previous step's A exchange (en0, en1)
      const int64_t vb = (int64_t)(variant * 2 + par) * d.B;
      const int64_t gslot = ((vb + b) * tiles + tile) * 4 + g;
      const int64_t grow0 = (vb + b) * tiles * 4;
      if (PRE && pre) {  // SPEC: step t's motion and A were done at the end of step t - 1
        e0 = pe0;
        e1 = pe1;
        p0 = pp0;
        p1 = pp1;
      } else {
        e0 = e1 = p0 = p1 = 0.f;
        if (valid) {
          e0 = sn0;
          e1 = sn1;
          p0 = (xs0 + v0) + e0;
          p1 = (xs1 + v1) + e1;
        }
        {  // exchange A: this wave's sums of x_phys
          double s[4] = {p0, p1, (double)p0 * p0, (double)p1 * p1};
          wave_sum_dpp_n(s);
          publish4(ws.ga + gslot * kGA, s, tag);
        }
      }
      PT(t, 1);
      // the next step's motion noise, drawn while the A sweep is in flight / fA is awaited
      auto next_noise = [&]() {
        if (first && t + 1 < d.T) {
          if (valid) pass_noise(d, t + 1, grow, i, en0, en1);
          nv0 = d.vel[2 * ((int64_t)(t + 1) * d.B + b)];
          nv1 = d.vel[2 * ((int64_t)(t + 1) * d.B + b) + 1];
        }
      };
      auto stop = [&]() { return spec && dec_fired(L, t); };
      const int fa = 4 * (t + 1) + 2 * variant;
      if (w == 0) {  // the row's nf_dyn context and fold (fold_one's fma sequence)
        // cbd[par] was last read by the prior waves at step t - 2
        if (t >= 2) {
          wait_flag2(&L.pf[0], t - 1);
          wait_flag2(&L.pf[2], t - 1);
        }
        if (!HOLD && fold_lane) load_fwd(d);
        const int st = poll_rowx<3>(ws.ga + grow0 * kGA, tiles * 4 * kGA, tag, L.rowa, next_noise, stop);
        if (GATE && first) {  // (the poll's loads drained this wave's slot t - 1 stores too)
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          set_flag(&L.hxf[g], t);
        }
        PT(t, 7);
        if (st == 0) {
          const Ctx4 c = row_ctx(L.rowa, tiles, inv_n, inv_n1);
          if (fold_lane) {
            const float cv[4] = {c.m0, c.m1, c.s0, c.s1};
            float v = fwd[0];
#pragma unroll
            for (int q = 0; q < kOctxDyn; ++q) v = fmaf(fwd[1 + q], cv[q], v);
            reinterpret_cast<float *>(L.cbd[par])[lane] = v;
          }
        }
        set_flag(&L.fA, st == 2 ? fa + 1 : fa);
        if (st == 2) return 2;
      } else {
        if (GATE && first) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          set_flag(&L.hxf[g], t);
        }
        next_noise();
        wait_flag(&L.fA, fa);
        if (spec && __builtin_amdgcn_readfirstlane(*(lds_vint *)&L.fA) == fa + 1) return 2;
      }
      PT(t, 2);
      // nf_dyn inverse (model/models.py:305-332)
      cf2 *dyn = wptr2(d.dyn_params), *cond = wptr2(d.cond_params);
      float xd0 = p0, xd1 = p1, ld = 0.f;
      if (valid)
        for (int f = nfl - 1; f >= 0; --f)
          ld += pass_inverse(dyn + f * 2 * nsd, nsd, xd0, xd1, L.cbd[par] + f * 2 * kH);
      jac = -ld;
      PT(t, 3);
      {
        double s[4] = {valid ? xd0 : 0.0, valid ? xd1 : 0.0, valid ? (double)xd0 * xd0 : 0.0,
                       valid ? (double)xd1 * xd1 : 0.0};
        wave_sum_dpp_n(s);
        publish4(ws.gb + gslot * kGA, s, tag);  // exchange B
      }
      if (w == 0) {  // the proposal fold: encoding columns (from prior wave 4), then [mean, std] of x_dyn
        if (!HOLD && fold_lane) load_fwc(d);
        const int st = poll_rowx<3>(ws.gb + grow0 * kGA, tiles * 4 * kGA, tag, L.rowa, NoWork(), stop);
        if (st == 0) {
          PT(t, 8);
          const Ctx4 c = row_ctx(L.rowa, tiles, inv_n, inv_n1);
          wait_flag(&L.fE, t + 1);
          if (fold_lane) {
            const float c4[4] = {c.m0, c.m1, c.s0, c.s1};
            float a = L.encfold[par][lane];
#pragma unroll
            for (int q = 0; q < 4; ++q) a = fmaf(fwc[q], c4[q], a);
            reinterpret_cast<float *>(L.cbc[par])[lane] = a;
          }
        }
        set_flag(&L.fB, st == 2 ? fa + 1 : fa);
        if (st == 2) return 2;
      } else {
        wait_flag(&L.fB, fa);
        if (spec && __builtin_amdgcn_readfirstlane(*(lds_vint *)&L.fB) == fa + 1) return 2;
      }
      PT(t, 4);
      // NF proposal inverse (model/models.py:334-356)
      q0 = xd0;
      q1 = xd1;
      ldp = 0.f;
      if (valid)
        for (int f = nfl - 1; f >= 0; --f)
          ldp += pass_inverse(cond + f * 2 * nsc, nsc, q0, q1, L.cbc[par] + f * 2 * kH);
      if (PRE && t + 1 < d.T) {
        // SPEC: step t + 1's motion (its noise and velocity are in hand) and its exchange A go
        // out now, before step t's commit, whose LDS hand-offs then overlap A's visibility.  (A
        // of step t + 1 reuses the parity of step t - 1's, which every tile of the row consumed
        // before publishing B(t), swept above.)
        pe0 = pe1 = pp0 = pp1 = 0.f;
        if (valid) {
          pe0 = en0;
          pe1 = en1;
          pp0 = (q0 + nv0) + pe0;
          pp1 = (q1 + nv1) + pe1;
        }
        const int64_t gslot1 = (((int64_t)(par ^ 1) * d.B + b) * tiles + tile) * 4 + g;
        double s[4] = {pp0, pp1, (double)pp0 * pp0, (double)pp1 * pp1};
        wave_sum_dpp_n(s);
        publish4(ws.ga + gslot1 * kGA, s, tag + 1u);
      }
      return 0;
    };
    for (int a = 0;; ++a) {  // (one copy of the attempt's code: a loop, not two calls)
      attempt(a == 0, GATE && !known);
      if (!GATE || known) break;
      // the speculated step's decision: commit, or drop the attempt and redo after resampling
      fire = wait_dec(L, t);
      PT(t, 9);
      known = true;
      if (!fire) break;
      if (w == 0) set_flag(&L.rq, t + 1);  // the prior waves join the row's resampling
      pass_resample(d, ws, L, b, tile, tag0, t, round, FORCE || NFDPF_GATE_LATE);
      take_resampled();
      variant = 1;
    }
    // commit step t: the histories, and the proposal to the prior wave and the encoder pair
    constexpr bool HS = NFDPF_PASS_HSTORE && MODE == kModeSpec;  // the prior wave stores them
    const RowSlot S = row_slot(d, b, t);
    if (valid && !HS) {
      S.hnoise[2 * i] = e0;
      S.hnoise[2 * i + 1] = e1;
      S.hidx[i] = (int64_t)N * grow + src;
      if (S.hjac) S.hjac[i] = jac;
    }
    // the group's encoder pair has read qbuf / rbuf[par] of step t - 2 (HS: its prior wave ebuf)
    if (t >= 2) wait_flag2(&L.ef[2 * g], t - 1);
#if NFDPF_PASS_HSTORE
    if (HS && t >= 2) wait_flag(&L.pf[g], t - 1);
#endif
    if (valid) {  // to the prior wave and the encoder pair
      L.qbuf[par][slot] = q0;
      L.qbuf[par][kTile + slot] = q1;
      L.pbuf[par][slot] = p0 - e0;
      L.pbuf[par][kTile + slot] = p1 - e1;
      L.rbuf[par][kTile + slot] = (density(e0, e1, K, two_var) + jac) + (-ldp);  // propose
#if NFDPF_PASS_HSTORE
      if (HS) {
        L.ebuf[par][slot] = e0;
        L.ebuf[par][kTile + slot] = e1;
        L.ebuf[par][2 * kTile + slot] = jac;
      }
#endif
      if (FORCE || GATE) {  // a later step's resampling reads the row's particles from other tiles
        store_wt2(S.hx + 2 * i, q0, q1);
      } else if (!HS) {
        S.hx[2 * i] = q0;
        S.hx[2 * i + 1] = q1;
      }
    }
    // FORCE: drained before qf, which the encoder pair's C(t) granules then cover (GATE: drained
    // by the next step's A sweep / resampling, hxf)
    if (FORCE) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    set_flag(&L.qf[g], t + 1);
    PT(t, 5);
    x0 = q0;
    x1 = q1;
    if (GATE) gp.update(fire);
    pre = PRE;
  }
  if (GATE) {  // the last slot's stores (the encoder pair's C(T - 1) waits for them)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    set_flag(&L.hxf[g], d.T);
  }
}

// waves 4-7 ("prior", group g = w - 4): the nf_dyn forward of the proposal and the prior density
// (model/models.py:358-377, stage_prior_split) off the chain, into rbuf's prior half (flag rf[g]).
// They are half of the 8 flow waves that resample the row (pass_resample): every step (FORCE),
// or (GATE) at the top of a step predicted to fire, or when the chain drops a step it had
// speculated not to fire (rq) -- the same steps as the chain waves, so their barriers match.
template <int MODE>
__device__ __forceinline__ void pass_prior(const nfdpf_filter_desc &d, const PassWs &ws, PassLds &L, int b, int tile,
                                           uint32_t tag0) {
  constexpr bool FORCE = MODE == kModeForce, GATE = MODE == kModeGate;
  const int N = d.N, nfl = d.n_flows;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const int g = w - 4, slot = g * 64 + lane;
  const int i = tile * kTile + slot;
  const bool valid = i < N;
  constexpr int nsd = kNsDyn;
  int round = 0;
  GatePred gp;  // GATE: the prediction of step t's decision (pass_chain's, from the same decisions)
  const int i_ = i, slot_ = slot;
  for (int t = 0; t < d.T; ++t) {
    const nfdpf_filter_desc &d = *(const nfdpf_filter_desc *)kernarg_desc();  // (kernarg_desc)
    const PassWs &ws = *(const PassWs *)kernarg_ws();
    const int i = opaque_int(i_), slot = opaque_int(slot_);
    cf2 *dyn = wptr2(d.dyn_params);
    const float K = d.dens_const, two_var = 2.0f * (d.pos_noise * d.pos_noise);
    const int par = t & 1;
    const RowSlot S = row_slot(d, b, t);
    const int32_t *plan = GATE ? d.pass_plan : nullptr;
    const int pred = GATE ? (plan ? (plan[t] ? 1 : 0) : t == 0 ? wait_dec(L, 0) : gp.get()) : 0;
    if (FORCE || pred) pass_resample(d, ws, L, b, tile, tag0, t, round, FORCE || NFDPF_GATE_LATE);
    PT(t, 0);
    if (g == 0) {
      // the proposal fold over the encoding columns (model/models.py:338-346) one step ahead,
      // while this wave waits for the proposal: step t + 1's (and step 0's at t = 0), so wave
      // 0's B fold never waits for it.  encfold[(t + 1) & 1] was last read by wave 0's fold of
      // step t - 1, before qf[0](t - 1), which this wave has waited for
      const int O = d.E + 4, ncb = nfl * 4 * kH;
      for (int s = t == 0 ? 0 : t + 1; s <= t + 1 && s < d.T; ++s) {
        if (lane < ncb) {
          const FoldRef r = fold_ref(d.cond_params, net_size<1, kH>(O), lane);
          L.encfold[s & 1][lane] = fold_acc(r, O, fold_bias0(r, O), d.enc + ((int64_t)b * d.T + s) * d.E, 0, d.E);
        }
        set_flag(&L.fE, s + 1);
      }
    }
    if (GATE && !pred && t > 0 && !plan) {
      // the proposal, or the chain's call to resample the row after all (a dropped speculation;
      // rq is only ever raised before qf of the same step)
      Spin sp;
      for (;;) {
        const int q = __builtin_amdgcn_readfirstlane(*(lds_vint *)&L.qf[g]);
        const int r = __builtin_amdgcn_readfirstlane(*(lds_vint *)&L.rq);
        if (q >= t + 1 || r >= t + 1 || !pass_spin<NFDPF_PASS_FLAG_SLEEP>(sp)) break;
      }
      asm volatile("" ::: "memory");
      if (__builtin_amdgcn_readfirstlane(*(lds_vint *)&L.rq) >= t + 1)
        pass_resample(d, ws, L, b, tile, tag0, t, round, FORCE || NFDPF_GATE_LATE);
    }
    wait_flag(&L.qf[g], t + 1);
    PT(t, 1);
    if (valid) {
      float lo = L.qbuf[par][slot], up = L.qbuf[par][kTile + slot], ld2 = 0.f;
      const float r0 = L.pbuf[par][slot], r1 = L.pbuf[par][kTile + slot];
#if NFDPF_PASS_HSTORE
      if constexpr (MODE == kModeSpec) {  // the chain's histories of step t (pass_chain's commit)
        S.hx[2 * i] = lo;
        S.hx[2 * i + 1] = up;
        S.hnoise[2 * i] = L.ebuf[par][slot];
        S.hnoise[2 * i + 1] = L.ebuf[par][kTile + slot];
        S.hidx[i] = (int64_t)N * (d.row_base + b) + i;
        if (S.hjac) S.hjac[i] = L.ebuf[par][2 * kTile + slot];
      }
#endif
#ifndef NFDPF_EXP_NOFWD
      for (int f = 0; f < nfl; ++f)
#else
      for (int f = 0; f < nfl && lo == 12345.f; ++f)  // experiment only: timing without the prior's forward
#endif
        ld2 += pass_forward(dyn + f * 2 * nsd, nsd, lo, up, L.cbd[par] + f * 2 * kH);
      const float prior = density(lo - r0, up - r1, K, two_var) - (-ld2);
      L.rbuf[par][slot] = prior;
      if (S.hprior) S.hprior[i] = prior;
    }
    set_flag(&L.rf[g], t + 1);
    set_flag(&L.pf[g], t + 1);
    if (GATE) gp.update(__builtin_amdgcn_readfirstlane(*(lds_vint *)&L.dec[par]));  // committed: known
    PT(t, 2);
  }
}

// ---- waves 8-15 -----------------------------------------------------------------------------
// wave 8: sweep C(s) of the row, leave its tile's merged ESS partial (the quad launch's merge,
// include/nfdpf.h) at ess_out[s] and the row normaliser of slot s (row_norm) in L.rn
__device__ __forceinline__ float pass_poll_c(const nfdpf_filter_desc &d, const PassWs &ws, PassLds &L, int b,
                                             int tile, uint32_t tag0, int s) {
  const int tiles = n_tiles(d.N), lane = threadIdx.x & 63;
  const int64_t row0 = (((int64_t)(s & 1) * d.B + b) * tiles) * 8;
  float inv = 0.f;
  if (poll_row(ws.gc + row0 * kGC, tiles * 8 * kGC, tag0 + (uint32_t)s + 1u, L.rowc)) {
    // lane k < tiles: tile k's {max, sum e, sum e^2} over its encoder waves in order
    const int k = lane < tiles ? lane : 0;
    float m = -INFINITY;
#pragma unroll
    for (int v = 0; v < 8; ++v) m = fmaxf(m, __uint_as_float(L.rowc[(k * 8 + v) * kGC]));
    double sum = 0.0, sq = 0.0;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
      const int q = (k * 8 + v) * kGC;
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
      sm[3] = 0.0;
    }
    // row_norm's arithmetic over the tiles in order (the cosine likelihood is not shifted)
    float M = -INFINITY;
    for (int kk = 0; kk < tiles; ++kk) M = fmaxf(M, (float)(double)readlane_f(m, kk));
    double Sd = 0.0;
    for (int kk = 0; kk < tiles; ++kk) Sd += readlane_d(sum, kk) * (double)expf(readlane_f(m, kk) - M);
    if (lane == 0) L.rn[s & 1] = RowNorm{M, (float)Sd, 0.f};
    // the row's 1 / sum p^2 of slot s (the next step's gate term): row_inv_ess's arithmetic on
    // the same per-tile partials it would read from ess_out (filter_tiled.hip), + 1e-12 terms
    double Mx = -INFINITY;
    for (int kk = 0; kk < tiles; ++kk) {
      const double mk = (double)readlane_f(m, kk);
      Mx = mk > Mx ? mk : Mx;
    }
    double Sg = 0.0, Q = 0.0;
    for (int kk = 0; kk < tiles; ++kk) {
      const float f = expf((float)((double)readlane_f(m, kk) - Mx));
      Sg += readlane_d(sum, kk) * (double)f;
      Q += readlane_d(sq, kk) * ((double)f * (double)f);
    }
    const double sp2 = Q / (Sg * Sg) + (2e-12 + (double)d.N * 1e-24);
    inv = 1.0f / (float)sp2;
  }
  set_flag(&L.fR, s + 1);
  return inv;
}

// kModeGate on a sharded batch (d.gate_peers): this row's term goes to every rank's exchange buffer
// (one granule per rank, system scope: over xGMI to the peers), then this rank's own buffer is
// swept for all B_global terms -- in global row order, so every rank sums the same words in the
// same order and takes the same decision.  The slot parity follows the exchange's running step
// count (epoch x T + t): a rank may run one step ahead of the slowest, also across passes.
// (t = 0: the row's term from its initial partials, as the unsharded t = 0 sum.)  -> the decision
__device__ __forceinline__ int pass_gate_xrank(const nfdpf_filter_desc &d, PassLds &L, int b, int tile, int t,
                                               float inv) {
  const int tiles = n_tiles(d.N), lane = threadIdx.x & 63, Bg = d.B_global;
  uint64_t *const *peers = reinterpret_cast<uint64_t *const *>(d.gate_peers);
  const uint64_t *own = peers[d.gate_rank];
  const uint32_t xep =
      __hip_atomic_load(reinterpret_cast<const uint32_t *>(own), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const uint32_t tag = (xep << 12) + (uint32_t)t + 1u;
  const int64_t slot = kXgHdr + (int64_t)(((uint64_t)xep * (uint64_t)d.T + (uint64_t)t) & 1u) * Bg;
  const float r = t == 0 ? row_inv_ess(reinterpret_cast<const double *>(d.ess_all) + (int64_t)b * tiles * kSm,
                                       tiles, d.N, false)
                         : inv;
  if (tile == 0 && lane < d.gate_world)
    __hip_atomic_store(peers[lane] + slot + d.row_base + b, ((uint64_t)tag << 32) | __float_as_uint(r),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  for (int h = 0; h < Bg; h += 256)  // (256 granules a sweep)
    if (poll_rowx<4, NoWork, NoStop, __HIP_MEMORY_SCOPE_SYSTEM>(own + slot + h, min(256, Bg - h), tag, L.rowe + h))
      break;  // (timed out: the pass drains)
  const float s = cascade_row_sum([&](int q) { return __uint_as_float(L.rowe[q]); }, Bg);
  return (s / (float)Bg) < 0.5f * (float)d.N ? 1 : 0;
}

// kModeGate, wave 8 of every workgroup: the batch-global ESS gate of step t (DPFs.py:163-165:
// torch.mean over the rows of 1 / sum p^2 of slot t - 1, < 0.5 N), tiled_gate_batch_kernel's
// arithmetic.  t = 0: from the initial partials (ess_all).  t > 0: this row's term `inv` (from the
// C(t - 1) sweep) goes out as one granule from its tile 0, the B rows' granules are swept, and
// the mean follows ATen's cascade order over them.  Every workgroup decides alike, from the same
// words.  The decision goes to dec[t & 1] / fD; workgroup (0, 0) also records it (pass_gates,
// the epilogue's count).
// With a plan (d.pass_plan) the decision is the plan's: no exchange, nothing recorded here (the
// epilogue verifies the plan against the pass's own partials).
template <bool XR>
__device__ __forceinline__ void pass_gate(const nfdpf_filter_desc &d, const PassWs &ws, PassLds &L, int b, int tile,
                                          uint32_t tag0, int t, float inv) {
  const int tiles = n_tiles(d.N), lane = threadIdx.x & 63, B = d.B;
  if (d.pass_plan) {
    if (lane == 0) L.dec[t & 1] = d.pass_plan[t] ? 1 : 0;
    set_flag(&L.fD, t + 1);
    return;
  }
  float s;
  if constexpr (XR) {  // sharded: every rank's rows (its own kernel instance: the registers of the step loop)
    const int fire = pass_gate_xrank(d, L, b, tile, t, inv);
    if (lane == 0) L.dec[t & 1] = fire;
    set_flag(&L.fD, t + 1);
    if (b == 0 && tile == 0 && lane == 0) {
      ws.eg[t] = fire;
      if (d.pass_gates) d.pass_gates[t] = fire;
    }
    return;
  }
  if (t == 0) {
    const double *parts = reinterpret_cast<const double *>(d.ess_all);
    s = cascade_row_sum([&](int r) { return row_inv_ess(parts + (int64_t)r * tiles * kSm, tiles, d.N, false); }, B);
  } else {
    uint64_t *ge = ws.ge + (int64_t)((t - 1) & 1) * B;
    const uint32_t tag = tag0 + (uint32_t)t;  // slot t - 1's
    if (tile == 0 && lane == 0) gran_store(ge + b, __float_as_uint(inv), tag);
    poll_rowx<4>(ge, B, tag, L.rowe);
    s = cascade_row_sum([&](int r) { return __uint_as_float(L.rowe[r]); }, B);
  }
  const int fire = (s / (float)B) < 0.5f * (float)d.N ? 1 : 0;
  if (lane == 0) L.dec[t & 1] = fire;
  set_flag(&L.fD, t + 1);
  if (b == 0 && tile == 0 && lane == 0) {
    ws.eg[t] = fire;
    if (d.pass_gates) d.pass_gates[t] = fire;
  }
}

// normalise slot s of this wave's particles (finish_prev's arithmetic, the cosine measurement:
// unshifted): hp, and the wave's prediction / obs-likelihood partials; returns log p
__device__ __forceinline__ float pass_norm(const nfdpf_filter_desc &d, const PassWs &ws, PassLds &L, int b, int tile,
                                           int s, int i_e, bool valid_e, float u, float qx0, float qx1) {
  wait_flag(&L.fR, s + 1);
  const RowNorm rn = L.rn[s & 1];
  double sf[4] = {0.0, 0.0, 0.0, 0.0};
  float lp = 0.f;
  if (valid_e) {
    const float p = expf(u - rn.shift) / rn.Ssum + 1e-12f;
    d.hist_p[((int64_t)b * d.T + s) * d.N + i_e] = p;
    lp = logf(p);
    sf[0] = (double)p * p;
    sf[1] = (double)p * qx0;
    sf[2] = (double)p * qx1;
    sf[3] = u;
  }
  wave_sum_dpp_n(sf);
  const int lane = threadIdx.x & 63, we = (threadIdx.x >> 6) - 8, tiles = n_tiles(d.N);
  if (lane < 4)
    ws.fin[((((int64_t)b * d.T + s) * tiles + tile) * 8 + we) * 4 + lane] =
        lane == 0 ? sf[0] : lane == 1 ? sf[1] : lane == 2 ? sf[2] : sf[3];
  return lp;
}

// waves 8-15 (a pair per group): the cosine measurement on the MFMA encoder, the log-weights,
// exchange C and (wave 8) its sweep, slot t's normalisation; kModeGate: wave 8 also decides the
// next step's gate right after the C sweep (pass_gate), and a step whose gate fired takes the
// resampled log-weight of its particle's source (lr_l) instead of its own log p
// issue priority: the chain waves carry the pass's critical path (chain 3 / others 0: +0.8 %
// at C2 over equal priorities, two A/B rounds on one box)
#ifndef NFDPF_PRIO_CHAIN
#define NFDPF_PRIO_CHAIN 3
#define NFDPF_PRIO_PRIOR 0
#define NFDPF_PRIO_ENC 0
#endif
#ifndef NFDPF_GPRIO_PRIOR
#define NFDPF_GPRIO_PRIOR 0
#endif
// Which encoder wave sweeps exchange C (and, GATE, decides the gate), and the issue priority it
// takes meanwhile: in the gated and forced passes that sweep is on the step's critical path
// (the decision / the row's resampling wait for it), while its SIMD also carries a chain wave
// at priority 3.
#ifndef NFDPF_SWEEP_WE
#define NFDPF_SWEEP_WE 0
#endif
#ifndef NFDPF_SWEEP_PRIO
#define NFDPF_SWEEP_PRIO 0
#endif
template <int MODE>
__device__ __forceinline__ void sweep_prio(bool on) {
  if constexpr (MODE != kModeSpec && NFDPF_SWEEP_PRIO != 0) {
    if (on)
      __builtin_amdgcn_s_setprio(NFDPF_SWEEP_PRIO);
    else
      __builtin_amdgcn_s_setprio(NFDPF_PRIO_ENC);
  }
}

template <int MODE, bool XR = false>
__device__ __forceinline__ void pass_encoder(const nfdpf_filter_desc &d, const PassWs &ws, PassLds &L, int b, int tile,
                                             uint32_t tag0) {
  constexpr bool FORCE = MODE == kModeForce, GATE = MODE == kModeGate;
  const int sweeper = MODE == kModeSpec ? 0 : NFDPF_SWEEP_WE;  // (encoder-wave index, 0..7)
  const int tiles = n_tiles(d.N), N = d.N;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63, we = w - 8;
  const int role = w & 1, g = (w >> 1) & 3;
  // lanes 0-31: particles [32 role, 32 role + 32) of group g (encode_dot_mfma_half)
  const int slot_e = g * 64 + 32 * role + (lane & 31), i_e = tile * kTile + slot_e;
  const bool valid_e = lane < 32 && i_e < N;
  const bool grp = tile * kTile + g * 64 < N;
  const EncFrag2 ef = enc_frag2_load(d.pe_params);  // the encoder's weight fragments, once
  float lr = valid_e ? logf(d.p_prev[(int64_t)b * d.p_prev_rs + i_e]) : 0.f;
  float u = 0.f, qx0 = 0.f, qx1 = 0.f;
  int pdec = 0;  // GATE: step t's decision, once committed
  GatePred gp;   // GATE: the flow waves' prediction (they resampled at step t iff it or step t's decision fired)
  if (GATE && we == sweeper) pass_gate<XR>(d, ws, L, b, tile, tag0, 0, 0.f);
  const int slot_e_ = slot_e, i_e_ = i_e;
  for (int t = 0; t < d.T; ++t) {
    // (opaque_int where the VGPR pressure spilled their addresses: FORCE / GATE)
    const int slot_e = MODE == kModeSpec ? slot_e_ : opaque_int(slot_e_);
    const int i_e = MODE == kModeSpec ? i_e_ : opaque_int(i_e_);
    const int par = t & 1;
    const float *enc_t = d.enc + ((int64_t)b * d.T + t) * d.E;
    PT(t, 0);
    // measure_row_setup (cosine), per wave into its own LDS copy
    const float ve = lane < kE ? enc_t[lane] : 0.f;
    const double vinv = 1.0 / fmax(sqrt(wave_sum((double)ve * ve)), 1e-12);
    if (lane < kE) L.encq[we][lane] = ve;
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    // the cosine measurement (model/models.py:206-219) of step t's proposal
    auto encode = [&]() {
      double ss, dot;
      wait_flag(&L.qf[g], t + 1);
      // GATE: a resampling at step t (predicted, or the chain's redo) may still be summing its
      // gathered weights in the scratch the MFMA layers reuse -- until fS (qf implies fD >= t + 1)
      // (a plan pass: the flow waves resampled at step t iff the plan's gate fired -- nothing is
      // speculated from step t - 1's decision there)
      if (GATE && (d.pass_plan ? d.pass_plan[t] != 0
                               : ((t > 0 && gp.get()) || __builtin_amdgcn_readfirstlane(*(lds_vint *)&L.dec[par]) != 0)))
        wait_flag(&L.fS, t + 1);
      PT(t, 4);
#ifndef NFDPF_EXP_NOENC
      encode_dot_mfma_half<kE>(ef, role, L.qbuf[par] + g * 64, L.qbuf[par] + kTile + g * 64, L.encq[we], ss, dot,
                               L.Hws[we]);
#else
      ss = 1.0; dot = 0.5;  // experiment only: timing without the encoder
#endif
      PT(t, 5);
      return cos_lik(ss, dot, vinv);
    };
    float lk = 0.f;
    if constexpr (MODE == kModeSpec) {
      // the encoder first: it needs only the proposal, and it hides the C(t - 1) exchange
      if (grp) lk = encode();
      if (we == 0 && t > 0) pass_poll_c(d, ws, L, b, tile, tag0, t - 1);
      PT(t, 2);
      if (t > 0) lr = pass_norm(d, ws, L, b, tile, t - 1, i_e, valid_e, u, qx0, qx1);
    } else if constexpr (FORCE) {
      // the row's resampling at the top of step t needs slot t - 1 normalised first (fR(t - 1))
      if (we == sweeper && t > 0) {
        sweep_prio<MODE>(true);
        pass_poll_c(d, ws, L, b, tile, tag0, t - 1);
        sweep_prio<MODE>(false);
      }
      PT(t, 2);
      if (t > 0) lr = pass_norm(d, ws, L, b, tile, t - 1, i_e, valid_e, u, qx0, qx1);
      wait_flag(&L.fS, t + 1);  // the flow waves resampled the row: the log-weight of the source
      lr = valid_e ? L.lr_l[slot_e] : 0.f;
      if (grp) lk = encode();
    } else {
      // GATE: slot t - 1's exchange, its normaliser and step t's decision first (the chain's
      // speculation of step t waits for it), then the measurement
      if (we == sweeper && t > 0) {
        sweep_prio<MODE>(true);
        const float inv = pass_poll_c(d, ws, L, b, tile, tag0, t - 1);
        PT(t, 10);
        pass_gate<XR>(d, ws, L, b, tile, tag0, t, inv);
        sweep_prio<MODE>(false);
      }
      PT(t, 2);
      if (t > 0) lr = pass_norm(d, ws, L, b, tile, t - 1, i_e, valid_e, u, qx0, qx1);
      if (grp) lk = encode();
      // step t is committed (qf): its decision is known; a fired gate resampled the row and
      // this particle's log-weight is its source's (the chain's resampling left it in lr_l)
      pdec = d.pass_plan ? (d.pass_plan[t] ? 1 : 0) : __builtin_amdgcn_readfirstlane(*(lds_vint *)&L.dec[par]);
      if (pdec != 0) lr = valid_e ? L.lr_l[slot_e] : 0.f;
      gp.update(pdec);
    }
    // the log-weight (DPFs.py:187)
    PT(t, 3);
    u = 0.f;
    if (grp) {
      if (valid_e) {
        d.hist_lik[((int64_t)b * d.T + t) * N + i_e] = lk;
        qx0 = L.qbuf[par][slot_e];
        qx1 = L.qbuf[par][kTile + slot_e];
      }
      wait_flag(&L.rf[g], t + 1);
      if (valid_e) u = logw(lr, lk, L.rbuf[par][slot_e], L.rbuf[par][kTile + slot_e]);
    }
    set_flag(&L.ef[we], t + 1);  // qbuf / rbuf[par] read: the chain wave may reuse them at t + 2
    PT(t, 6);
    if (FORCE || GATE) {  // the row's next resampling reads u from every tile: written through, drained
      if (valid_e) store_wt(ws.gu + ((int64_t)par * d.B + b) * N + i_e, u);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    if (GATE) wait_flag(&L.hxf[g], t + 1);  // ... and the particles (the chain's slot-t stores)
    // exchange C: this wave's softmax partials (wave_partials_quad's arithmetic)
    const float mw = wave_max_dpp(valid_e ? u : -INFINITY);
    const float ev = valid_e ? expf(u - mw) : 0.f;
    double r[2] = {(double)ev, (double)ev * ev};
    wave_sum_dpp_n(r);
    if (lane < kGC) {
      const uint64_t eb = (uint64_t)__double_as_longlong(r[0]), qb = (uint64_t)__double_as_longlong(r[1]);
      const uint32_t word = lane == 0 ? __float_as_uint(mw)
                            : lane == 1 ? (uint32_t)eb
                            : lane == 2 ? (uint32_t)(eb >> 32)
                            : lane == 3 ? (uint32_t)qb
                            : lane == 4 ? (uint32_t)(qb >> 32)
                                        : 0u;
      const int64_t gslot = (((int64_t)par * d.B + b) * tiles + tile) * 8 + we;
      gran_store(ws.gc + gslot * kGC + lane, word, tag0 + (uint32_t)t + 1u);
    }
    PT(t, 7);
  }
  // the last slot's normalisation
  if (we == sweeper) pass_poll_c(d, ws, L, b, tile, tag0, d.T - 1);
  pass_norm(d, ws, L, b, tile, d.T - 1, i_e, valid_e, u, qx0, qx1);
}

// XR: kModeGate on a sharded batch (d.gate_peers: the cross-rank gate exchange, pass_gate_xrank)
template <int MODE, bool XR = false>
__global__ __launch_bounds__(4 * kTile, 1) void tiled_pass_kernel(const nfdpf_filter_desc d, PassWs ws) {
  __shared__ PassLds L;
  int b, tile;
  pass_tile_row(b, tile);
  const uint32_t tag0 = __hip_atomic_load(&ws.hdr->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) << 12;
  // LDS is not cleared between workgroups: zero every flag first
  if (threadIdx.x < 4) {
    L.qf[threadIdx.x] = 0;
    L.rf[threadIdx.x] = 0;
    L.pf[threadIdx.x] = 0;
    L.hxf[threadIdx.x] = 0;
  }
  if (threadIdx.x < 8) L.ef[threadIdx.x] = 0;
  if (threadIdx.x == 0) L.fA = L.fB = L.fE = L.fR = L.fS = L.fbar = L.fD = L.rq = 0;
  __syncthreads();
  if (threadIdx.x < 4 * 64) {
    __builtin_amdgcn_s_setprio(NFDPF_PRIO_CHAIN);
    pass_chain<MODE>(d, ws, L, b, tile, tag0);
  } else if (threadIdx.x < 8 * 64) {
    if constexpr (MODE == kModeSpec)
      __builtin_amdgcn_s_setprio(NFDPF_PRIO_PRIOR);
    else  // the prior's nf_dyn forward feeds the weights every decision / resampling waits for
      __builtin_amdgcn_s_setprio(NFDPF_GPRIO_PRIOR);
    pass_prior<MODE>(d, ws, L, b, tile, tag0);
  } else {
    __builtin_amdgcn_s_setprio(NFDPF_PRIO_ENC);
    pass_encoder<MODE, XR>(d, ws, L, b, tile, tag0);
  }
}

// After the pass, on its stream: one 64-lane workgroup per step k --
//   * pred[b][k] and lw_sum[b][k] of every row (tiled_finalize_kernel's sums over the row's
//     tiles x 8 encoder-wave entries, in order);
//   * with `gates_from` (a speculative one-shard pass): step k's ESS gate from its input
//     partials (k = 0: ess_all, else the pass's ess_out[k - 1]), tiled_gate_batch_kernel's
//     arithmetic;
//   * q_k = sum_b lw_sum[b][k] (fp64, row order) / (B N);
// the LAST workgroup to arrive (hdr->done) adds the q_k in step order (the obs-likelihood,
// DPFs.py:191), counts the fired gates, reads and clears the hand-off fault counter (flags, when
// asked), clears the abort word and bumps the epoch -- the granules of the current layout are
// cleared when its 20 bits wrap.  Replaces the epoch, finalize, gate-batch and verify launches
// of round 4 (one 64-lane wave walked 64 steps x B rows serially there: 18 us per pass).
// gates: 0 none, 1 verify (the speculative pass's gates from its partials), 2 the pass decided
// them itself (kModeGate: ws.eg already holds them; only counted here)
// ept: fin entries per tile (8 encoder waves in tiled_pass_kernel, 4 particle groups in
// tiled_pass_cm_kernel)
__global__ __launch_bounds__(64) void tiled_pass_epilogue_kernel(const nfdpf_filter_desc d, PassWs ws, int gates,
                                                                 int ept) {
  __shared__ float lw_l[256], inv_l[256];
  __shared__ int last;
  const int k = blockIdx.x, l = threadIdx.x, T = d.T, B = d.B, tiles = n_tiles(d.N), ent = tiles * ept;
  // gates == 1: step k's gate input (k = 0: ess_all, else the pass's ess_out[k - 1]), each row's
  // partials loaded beside its fin entries (one memory round trip for both)
  const double *parts = gates != 1 ? nullptr
                        : k == 0   ? reinterpret_cast<const double *>(d.ess_all)
                                   : reinterpret_cast<const double *>(d.ess_out) + (int64_t)(k - 1) * B * tiles * kSm;
  for (int b = l; b < B; b += 64) {
    const int64_t bt = (int64_t)b * T + k;
    double px = 0, py = 0, sw = 0;
    double gp[kPassMaxTiles * kSm];
    if (gates == 1) {
#pragma unroll
      for (int q = 0; q < kPassMaxTiles * kSm; ++q)
        if (q < tiles * kSm) gp[q] = parts[(int64_t)b * tiles * kSm + q];
    }
    // every entry's loads in flight at once (ent <= kPassMaxTiles * 8 = 32), then the adds in
    // entry order: one memory round trip per row instead of one per 8 entries
    double a[kPassMaxTiles * 8][3];
#pragma unroll
    for (int j = 0; j < kPassMaxTiles * 8; ++j) {
      if (j < ent) {
        const double *f = ws.fin + (bt * ent + j) * 4;
        a[j][0] = f[1];
        a[j][1] = f[2];
        a[j][2] = f[3];
      }
    }
#pragma unroll
    for (int j = 0; j < kPassMaxTiles * 8; ++j) {
      if (j < ent) {
        px += a[j][0];
        py += a[j][1];
        sw += a[j][2];
      }
    }
    d.pred[2 * bt] = (float)px;
    d.pred[2 * bt + 1] = (float)py;
    d.lw_sum[bt] = (float)sw;
    lw_l[b] = (float)sw;
    // the row's 1 / sum p^2 (row_inv_ess's arithmetic, row_inv_ess_t)
    if (gates == 1) inv_l[b] = row_inv_ess_t<kPassMaxTiles>([&](int q) { return gp[q]; }, tiles, d.N, k > 0);
  }
  __syncthreads();
  int fired = 0;
  if (gates == 1) {  // tiled_gate_batch_kernel's cascade over the rows' terms
    const float s = cascade_row_sum([&](int r) { return inv_l[r]; }, B);
    fired = (s / (float)B) < 0.5f * (float)d.N ? 1 : 0;
  }
  if (l == 0) {
    double tot = 0.0;
    for (int b = 0; b < B; ++b) tot += (double)lw_l[b];
    ws.eq[k] = tot / ((double)B * (double)d.N);
    if (gates != 2) ws.eg[k] = fired;
    if (d.pass_gates && gates == 1) d.pass_gates[k] = fired;
    // release the step's terms, then count this workgroup in
    const uint32_t n = __hip_atomic_fetch_add(&ws.hdr->done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    last = n == (uint32_t)T - 1;
  }
  __syncthreads();
  if (!last) return;
  __atomic_thread_fence(__ATOMIC_ACQUIRE);
  const uint32_t ep = __hip_atomic_load(&ws.hdr->epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u;
  if (ep > kPassEpochMask) {  // the tags' epoch wraps: no granule of this layout may keep an old tag
    const int64_t n = pass_granule_bytes(B, d.N) / 8;
    for (int64_t i = l; i < n; i += 64) ws.ga[i] = 0;  // ga, gb and gc are contiguous
  }
  // every step's terms in flight at once (lane t: steps t, t + 64, ...), then added in step order
  __shared__ double eq_l[kPassMaxT];
  __shared__ int eg_l[kPassMaxT];
  for (int t = l; t < T; t += 64) {
    eq_l[t] = __hip_atomic_load(&ws.eq[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    eg_l[t] = __hip_atomic_load(&ws.eg[t], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  if (l == 0) {
    double acc = 0.0;
    int nf = 0;
    for (int t = 0; t < T; ++t) {
      acc += eq_l[t];
      // a plan pass: the steps whose actual gate differs from the plan's
      nf += d.pass_plan ? (eg_l[t] != (d.pass_plan[t] ? 1 : 0)) : eg_l[t];
    }
    if (d.pass_obs) d.pass_obs[0] = (float)acc;
    if (d.pass_flags) {  // (system scope: the caller may map them from pinned host memory)
      __hip_atomic_store(&d.pass_flags[0], nf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&d.pass_flags[1], atomicExch(&g_split_fault, 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      __hip_atomic_store(&d.pass_flags[2], 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);  // written, last
    }
    ws.hdr->abort = 0;
    ws.hdr->done = 0;
    ws.hdr->epoch = ep > kPassEpochMask ? 0u : ep;
    if (d.gate_peers) {  // the cross-rank exchange's epoch (every rank's pass bumps its own alike)
      uint32_t *xe = reinterpret_cast<uint32_t *const *>(d.gate_peers)[d.gate_rank];
      __hip_atomic_store(xe, (__hip_atomic_load(xe, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1u) & kPassEpochMask,
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

static int pass_mode_of(const nfdpf_filter_desc &d) {
  return d.force_resample ? kModeForce : d.pass_gate ? kModeGate : kModeSpec;
}
typedef void (*pass_kernel_t)(const nfdpf_filter_desc, PassWs);
static pass_kernel_t pass_kernel_of(const nfdpf_filter_desc &d) {
  const int m = pass_mode_of(d);
  if (m == kModeGate && d.gate_peers) return tiled_pass_kernel<kModeGate, true>;
  return m == kModeForce ? tiled_pass_kernel<kModeForce> : m == kModeGate ? tiled_pass_kernel<kModeGate>
                                                                          : tiled_pass_kernel<kModeSpec>;
}

// The pass applies to this descriptor's configuration (the launcher also needs the speculative
// gate: d.gate given, ess_local) and every workgroup of its grid can be resident at once.
static bool pass_config_ok(const nfdpf_filter_desc &d) {
  const char *e = getenv("NFDPF_PASS");  // read per call: NFDPF_PASS=0 keeps the step-by-step launches
  if (e && e[0] == '0') return false;
  if (!(d.split_nets && d.nf_dyn == NFDPF_DYN_REALNVP && d.nf_cond && d.measurement == NFDPF_MEAS_COS)) return false;
  if (d.rng_mode != NFDPF_RNG_DEVICE || d.phase != 0 || d.E != kE || d.hidden != kH) return false;
  // a forced pass resamples every step inside the launch (soft resampler only); otherwise the
  // caller takes every gate as off and verifies them afterwards
  if (d.force_resample && d.resampler != NFDPF_RESAMPLE_SOFT) return false;
  // the in-launch gate: the whole batch in this launch (unless it follows a plan), the soft resampler
  if (d.pass_gate && !d.force_resample &&
      ((d.B_global != d.B && !d.pass_plan && !(d.gate_peers && d.gate_world >= 1 && d.B_global <= kXgMaxRows)) ||
       d.resampler != NFDPF_RESAMPLE_SOFT))
    return false;
  if (d.N < 2 || n_tiles(d.N) > kPassMaxTiles || d.n_flows < 1 || d.n_flows > 2 || d.T < 1 || d.T > kPassMaxT ||
      d.B < 1 || d.B > 256)  // (the epilogue stages a step's B row sums in LDS)
    return false;
  // every workgroup resident at once; a speculative, forced or plan pass may also run its rows in
  // resident chunks (pass_launch_rows), the gated one not (its rows wait for the batch decision)
  const int rows = pass_resident_rows(pass_kernel_of(d), 4 * kTile, n_tiles(d.N));
  return rows >= d.B || (rows >= 1 && (pass_mode_of(d) != kModeGate || d.pass_plan));
}

}  // namespace nfdpf
