// resample_ot.hip -- entropy-regularised optimal-transport resampling (resamplers.py:62-277).
//
// What the reference does (FP64, dense): centre and scale the particles (transport_function
// :211-227, diameter :72-76), build four B x N x N cost matrices (:183-186), run the
// Sinkhorn loop with epsilon annealing (:113-179) and finally materialise the B x N x N
// transport matrix (:194-210) and multiply it with the particles (:254-264).
//
// What runs here:
//   * only the two potentials that reach the output (a_y, b_x) are iterated: a_x / b_y are
//     computed by the reference but read by nothing (:139-147, :177-178);
//   * costs are recomputed on the fly from the 2-D points, never stored;
//   * potentials, exponents and shifts are fp64 per particle (the reference iterates in fp64;
//     at eps = 0.1 a potential of 100 is an exponent of 1400, whose fp32 ulp would already be a
//     1e-4 relative error of a transport weight); the O(N^2) pair work is fp32 on exponents
//     that are small by construction:
//   * every softmin is a log-sum-exp with a PER-LANE shift m_i predicted from the potentials
//     (no running max per pair).  In base 2, with h_j the softmin's exponent, c_ij = C_ij / e
//     and the row cut into slices s of 256 j with maxima M_s,
//       LSE_j(h_j - c_ij) = m_i + log2 sum_s sum_{j in s} 2^((h_j - M_s) + (M_s - m_i) - c_ij),
//     h_j - M_s <= 0 stored per j (fp32), M_s - m_i formed in fp64 once per slice and lane.
//     m_i = -a_i / (e ln 2) is the lane's current potential (the fixed point of the iteration),
//     so the sum stays near 1; a lane whose sum leaves [2^-60, 2^60] recomputes its softmin
//     exactly with a streamed max-shifted LSE (a diagnostic counter records how often);
//   * the two softmins of an iteration share c_ij, so a slice is summed as
//       2^(M_s - m_i) sum_j alpha_j 2^(-c_ij),   alpha_j = 2^(h_j - M_s)   (stored per j),
//     ONE v_exp_f32 per pair for both softmins -- unless, for some lane of the wave,
//     M_s - m_i > 96 (a heavy particle of the slice far from i: the near terms would underflow
//     in alpha_j K_ij before the factor lifts them); the wave then takes the two-exp form;
//   * the per-j operands form a per-row TABLE of planes written by the launch that produced
//     them (workgroup s writes j in [256 s, 256 s + 256) and its slice maximum: no
//     cross-workgroup hand-off inside a launch);
//   * a workgroup owns 256 i; its 4 waves split the row's slices and every lane carries 4 of
//     the 256 i, so each table word a wave loads (a wave-uniform vector load, software-
//     pipelined one block of 8 j ahead) serves 4 pairs per lane; partial sums meet in LDS in
//     wave order (deterministic);
//   * the transport matrix is never formed: column log-normalisers r_j first, then
//     x'_i = sum_j T_ij x_j with T_ij = 2^(f_i/e + r_j - c_ij) summed directly;
//   * the loop keeps the reference's batch-coupled stop rule -- it ends at the first
//     iteration after which ANY row has converged (torch.all(continue_), :126-129) -- with
//     one launch per iteration that first reads the previous iteration's per-row residuals
//     (identical decision in every workgroup, no atomics).
#include <atomic>
#include <chrono>
#include <mutex>
#include <thread>

#include "common.hpp"

namespace nfdpf {

// i (or j) per workgroup = the table slice length: 256, each lane carrying kR = 4 of the
// workgroup's i.  -DNFDPF_OT_SL=128 builds a layout with twice the waves per launch (kR = 2,
// the 4 waves split the slices four ways; 4 waves per SIMD at C4 instead of 2): measured
// slower on one box (C4 90.4 vs 83.1 ms per pass, C3 forced 27.1 vs 25.5) -- the per-workgroup
// prologue / epilogue doubles with the workgroup count.
#ifndef NFDPF_OT_SL
#define NFDPF_OT_SL 256
#endif
constexpr int kOtThreads = NFDPF_OT_SL;
constexpr int kOtBlock = 256;  // threads per workgroup; threads >= kOtThreads own no i
static_assert(kOtThreads == 128 || kOtThreads == 256, "slice length");
constexpr double kLog2ed = 1.4426950408889634;
constexpr double kLn2d = 0.6931471805599453;
constexpr float kLo = 0x1.0p-60f, kHi = 0x1.0p60f;  // outside: the lane recomputes exactly
// M_s - m_i above: two-exp form.  A term matters when alpha_j K_ij 2^(M_s - m_i) >= 2^-24 (the
// lane's sum is ~1), i.e. c_ij <= 24 + (M_s - m_i): up to 96 every such K_ij = 2^-c_ij and
// alpha_j K_ij stay >= 2^-120, normal fp32 (2^-126); only terms below 2^-24 of the sum can
// underflow.  (60 in r01: late, small-epsilon iterations took the two-exp form on most slices.)
#ifndef NFDPF_OT_RISKY
#define NFDPF_OT_RISKY 96.f
#endif
constexpr float kRisky = NFDPF_OT_RISKY;
// Prescaled coordinates (-DNFDPF_OT_PRESCALE): the iteration / final tables' X, Y planes and the
// lanes' own points are multiplied by s = sqrt(sc) (sc = the base-2 cost scale of the table's
// epsilon), so the pair exponent is -(dx'^2 + dy'^2) with no per-pair scaling multiply.
// Measured (round 2d, one box): C4 +3 %, C3 forced +1 %, but the full-size C3 teacher-forced
// likelihood error grows to 0.14 against the reference's own fp32 error of 0.0098 (the
// difference of two prescaled coordinates rounds ~5x coarser on close pairs): not shipped.
#ifdef NFDPF_OT_PRESCALE
constexpr bool kPrescale = true;
#else
constexpr bool kPrescale = false;
#endif

typedef float f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ f2 sp2(float v) { return f2{v, v}; }
__device__ __forceinline__ f2 pfma2(f2 a, f2 b, f2 c) { return __builtin_elementwise_fma(a, b, c); }

#ifdef NFDPF_OT_RISKSTAT  // experiment builds: share of wave-slices on the two-exp path, per call
__device__ unsigned int g_ot_risky, g_ot_wslices;
#endif
#ifdef NFDPF_EXP_OTTRACE  // experiment builds: per-phase timestamps of every iteration launch, lane 0 of wave 0
__device__ uint64_t g_ot_tr[1024][64][8], g_ot_loopend[1024];
#define OTT_WG (blockIdx.y * gridDim.x + blockIdx.x)
#define OTTRACE(k, slot)                                         \
  if (threadIdx.x == 0 && OTT_WG < 1024)                         \
    g_ot_tr[OTT_WG][(k) & 63][slot] = __builtin_amdgcn_s_memrealtime();
#else
#define OTTRACE(k, slot)
#endif
struct OtState {
  int32_t stopped;    // set by the iteration that observes a converged row
  int32_t K;          // total_iter of the reference
  int32_t fallbacks;  // softmins recomputed exactly (diagnostic, nfdpf_ot_stats)
};

// A table of one row: P planes of Np = splits * 256 floats, plane-major, plus the slice maxima
// (fp64, [splits][NM]).  Exponent planes hold h_j - M_s (fp32, <= 0; -inf on the padding).
struct OtWs {  // carve of the caller's workspace
  OtState *st;
  float *xs;     // [B,N,2] centred / scaled particles x~
  float *logw;   // [B,N]
  double *rowc;  // [B,4]: eps0, logu, max logw, unused
  double *pot;   // [2 buffers][2 (a_y,b_x)][B,N]
  double *res;   // [2 parity][B][splits] max |delta| of the iteration
  double *fg;    // [B,N] final potential f (= a_y after the post-loop softmin)
  float *tabI;   // [2][B][6][Np] X, Y, h_a - M, h_b - M, alpha, beta (iteration consuming a state)
  double *mI;    // [2][B][splits][2]
  float *tabF;   // [B][4][Np] X, Y, h_a - M, h_b - M at the final epsilon (rows still annealing)
  double *mF;    // [B][splits][2]
  float *tabC;   // [B][3][Np] column pass: X, Y, f_i / eps - M
  double *mC;    // [B][splits]
  float *tabA;   // [B][5][Np] apply pass: X, Y, r_j - M, x_j, y_j (x = the input particles)
  double *mA;    // [B][splits]
  double *epsk;  // [B][kEpsTab] running epsilon of iteration k (ot_setup_kernel)
};

static inline int64_t align256(int64_t v) { return (v + 255) / 256 * 256; }
// the running-epsilon table: iterations 0 .. kEpsTab-1 (annealing is over long before: eps0 is
// the squared diameter of the scaled cloud, a few dozen steps of s^2 = 0.5625 above eps)
constexpr int kEpsTab = 128;

static inline int ot_splits(int N) { return (N + kOtThreads - 1) / kOtThreads; }

struct Carver {
  char *p;
  int64_t used = 0;
  template <class T>
  T *take(int64_t n) {
    T *r = (T *)(p ? p + used : nullptr);
    used += align256(n * (int64_t)sizeof(T));
    return r;
  }
};

static OtWs carve(void *ws, int B, int N, int64_t *bytes = nullptr) {
  const int S = ot_splits(N);
  const int64_t Np = (int64_t)S * kOtThreads;
  Carver c{(char *)ws};
  OtWs w;
  w.st = c.take<OtState>(1);
  w.xs = c.take<float>((int64_t)B * N * 2);
  w.logw = c.take<float>((int64_t)B * N);
  w.rowc = c.take<double>((int64_t)B * 4);
  w.pot = c.take<double>((int64_t)4 * B * N);
  w.res = c.take<double>((int64_t)2 * B * S);
  w.fg = c.take<double>((int64_t)B * N);
  // + a padding block: the pair loop prefetches 8 floats past the last plane of the last row
  w.tabI = c.take<float>(2 * B * 6 * Np + 64);
  w.mI = c.take<double>((int64_t)2 * B * S * 2);
  w.tabF = c.take<float>(B * 4 * Np + 64);
  w.mF = c.take<double>((int64_t)B * S * 2);
  w.tabC = c.take<float>(B * 3 * Np + 64);
  w.mC = c.take<double>((int64_t)B * S);
  w.tabA = c.take<float>(B * 5 * Np + 64);
  w.mA = c.take<double>((int64_t)B * S);
  w.epsk = c.take<double>((int64_t)B * kEpsTab);
  if (bytes) *bytes = c.used;
  return w;
}

static int64_t ws_bytes(int B, int N) {
  int64_t n = 0;
  carve(nullptr, B, N, &n);
  return n;
}

struct OtParams {
  int B, N, splits, max_iter;
  double eps, sf, thr;
  const int32_t *gate;     // optional: skip everything when *gate == 0
  const int32_t *stop_at;  // optional: total_iter + 2 to run (sharded batches), else the rule
  int32_t *host;           // optional (poll mode): mapped host flags {stop seq, seq * 4096 + k}
  int32_t seq;             // call sequence number for the host flags
  double *hist;            // optional (sharded batches): every state's potentials [max_iter][2][B][N]
  int64_t x_rs = 0, w_rs = 0;  // row strides (floats) of the input particles / weights
};

// progress of the Sinkhorn loop to the polling host thread (system-scope stores into
// fine-grained host memory; vector stores)
__device__ __forceinline__ void host_flag(int32_t *h, int idx, int32_t v) {
  __hip_atomic_store(h + idx, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ bool ot_off(const OtParams &P) { return P.gate && *P.gate == 0; }

__device__ __forceinline__ int64_t np_of(const OtParams &P) { return (int64_t)P.splits * kOtThreads; }

// potentials of state k: double-buffered by parity, or the state's own slot of the history
// (a sharded call resumes its tail at the batch-global stop, which may lie behind its own)
__device__ __forceinline__ double *pot_ptr(const OtWs &ws, const OtParams &P, int k, int which, int b) {
  if (P.hist) return P.hist + (((int64_t)k * 2 + which) * P.B + b) * P.N;
  return ws.pot + (((int64_t)(k & 1) * 2 + which) * P.B + b) * P.N;
}
__device__ __forceinline__ float *tabI_row(const OtWs &ws, const OtParams &P, int buf, int b) {
  return ws.tabI + ((int64_t)buf * P.B + b) * 6 * np_of(P);
}
__device__ __forceinline__ double *mI_row(const OtWs &ws, const OtParams &P, int buf, int b) {
  return ws.mI + ((int64_t)buf * P.B + b) * P.splits * 2;
}

// running epsilon at iteration k: eps_{k+1} = max(eps_k * s^2, eps) in double (:158)
__device__ __forceinline__ double run_eps(double eps0, int k, double sf, double eps) {
  double e = eps0;
  for (int t = 0; t < k; ++t) e = fmax(e * sf, eps);
  return e;
}

// run_eps of row b from the table (the same fp64 recurrence, evaluated once per call)
__device__ __forceinline__ double eps_at(const OtWs &ws, const OtParams &P, int b, int k) {
  const double *t = ws.epsk + (int64_t)b * kEpsTab;
  return k < kEpsTab ? t[k] : run_eps(t[kEpsTab - 1], k - (kEpsTab - 1), P.sf, P.eps);
}

// sc with sc |dx|^2 = |dx|^2 / (2 e) * log2(e): C_ij / e in base 2
__device__ __forceinline__ float cost_scale(double inv_e) { return (float)(0.5 * inv_e * kLog2ed); }

// ------------------------------------------------------------------------------------------
// Pair loops.  A workgroup owns 256 i (i = 256 s0 + t); its 4 waves split the row's slices
// (wave w takes slices w, w + 4, ...) and every lane carries kR = 4 of the workgroup's i
// (lane + 64 r), so each table word a wave loads serves 4 pairs per lane.  (The table words
// are wave-uniform; a vector load returns them to every lane, and at one i per lane the L1
// return path, not the VALU, bounds the loop.)  Partial sums meet in LDS in wave order.
// ------------------------------------------------------------------------------------------
constexpr int kR = kOtThreads / 64;  // i per lane
constexpr int kWaves = kOtBlock / 64;
constexpr int kLdsPart = kWaves * 3 * kOtThreads;  // floats: wave partials of <= 3 sums per i

template <int NP>
struct TBlock {  // 8 consecutive j of NP planes
  float4 v[NP][2];
};

// load block j of the planes pl[0..NP) of a row table
// The words are wave-uniform.  -DNFDPF_OT_SLOAD reads them through the constant address space
// (scalar loads into SGPRs, one block at a time) instead of the pipelined vector loads that
// return the same 16 B to all 64 lanes: measured SLOWER (C4 iteration 124 vs 118 us, C3 22 vs
// 17 us; the compiler keeps half of the words as vector loads and the scalar waits are not
// overlapped -- profiles/r02_experiments.md).  So was one coalesced load per block handed out by
// v_readlane as SGPR operands (C4 iteration 129-141 vs 117 us).
typedef const float4 __attribute__((address_space(4))) cfloat4;
template <int NP>
__device__ __forceinline__ void tload(TBlock<NP> &B, const float *tab, int64_t Np, int j, const int (&pl)[NP]) {
#pragma unroll
  for (int p = 0; p < NP; ++p) {
#if !defined(NFDPF_OT_SLOAD) || !defined(__HIP_DEVICE_COMPILE__)
    const float4 *X = reinterpret_cast<const float4 *>(tab + pl[p] * Np + j);
#else
    cfloat4 *X = (cfloat4 *)(tab + pl[p] * Np + j);
#endif
    B.v[p][0] = X[0];
    B.v[p][1] = X[1];
  }
}

template <int NP>
__device__ __forceinline__ f2 tpair(const TBlock<NP> &B, int p, int q) {
  const float4 &c = B.v[p][q >> 1];
  return (q & 1) ? f2{c.z, c.w} : f2{c.x, c.y};
}

// Software pipeline over blocks of 8 j in [j0, j1) (a multiple of 16) with vector loads of the
// wave-uniform table words (vmcnt is in order, so a wait covers exactly the block about to be
// used -- scalar loads return out of order and every wait on them is lgkmcnt(0)).  Two named
// buffers; the scheduling barriers keep each block's loads one compute block ahead of their
// use.  Past the end a prefetch reads the next plane / the allocation's padding block and is
// discarded.
template <int NP, class Body>
__device__ __forceinline__ void pipelined(const float *tab, int64_t Np, int j0, int j1, const int (&pl)[NP],
                                          const Body &body) {
#ifdef NFDPF_OT_SLOAD
  // scalar loads: one block at a time (a scalar wait is lgkmcnt(0), so a prefetched block would
  // be waited for with the current one); the other waves of the SIMD cover the latency
  for (int j = j0; j < j1; j += 8) {
    TBlock<NP> A;
    tload(A, tab, Np, j, pl);
    body(A);
  }
  return;
#endif
  TBlock<NP> A, Bk;
  tload(A, tab, Np, j0, pl);
  for (int j = j0; j < j1; j += 16) {
    tload(Bk, tab, Np, j + 8, pl);
    __builtin_amdgcn_sched_barrier(0);
    body(A);
    __builtin_amdgcn_sched_barrier(0);
    tload(A, tab, Np, j + 16, pl);
    __builtin_amdgcn_sched_barrier(0);
    body(Bk);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// LDS-staged slices (default; -DNFDPF_OT_L1 keeps the wave-uniform vector loads above).  A
// wave copies a whole slice (256 j of up to kSlicePl planes) with coalesced loads -- lane l
// holds j0 + 4l .. j0 + 4l + 3 of every plane, 1 KB per plane and load instruction, all of it
// used -- into its own LDS region, and the pair loop reads the wave-uniform words from there
// (ds_read_b128, one address for all lanes).  It replaces wave-uniform 16-B vector loads that
// each returned their 16 B to all 64 lanes through the L1.  Measured (C4 iteration, one box):
// 120 -> 116.5 us -- the L1 return path was not the bound the r01 notes assumed; a register
// prefetch of the next slice was kept in scratch by the compiler and is not used.
constexpr int kSlicePl = 6;                                  // planes of the widest table (iteration)
constexpr int kSliceFloats = kSlicePl * kOtThreads + 16;     // + padding: the loop reads one block ahead
constexpr int kLdsAll = kLdsPart + kWaves * kSliceFloats;    // combine() area + the waves' slices

// one slice (planes 0 .. NPL-1, kOtThreads j each) into the wave's LDS region: float4 f of
// the slice (f = lane + 64 q) is plane f / (kOtThreads / 4), j0 + 4 (f % (kOtThreads / 4))
template <int Q, int NPL>
__device__ __forceinline__ void slice_copy_q(const float *tab, int64_t Np, int j0, float *sl) {
  constexpr int kPer = kOtThreads / 4;  // float4 per plane
  if constexpr (Q * 64 < NPL * kPer) {
    const int f = (threadIdx.x & 63) + 64 * Q;
    const int p = f / kPer, o = 4 * (f % kPer);
    const bool in = p < NPL;  // the last instruction may hold a part plane (NPL odd, 128 j)
    float4 v{};
    if (in) v = *reinterpret_cast<const float4 *>(tab + p * Np + j0 + o);
    slice_copy_q<Q + 1, NPL>(tab, Np, j0, sl);
    if (in) *reinterpret_cast<float4 *>(sl + p * kOtThreads + o) = v;
  }
}
template <int NPL>
__device__ __forceinline__ void slice_copy(const float *tab, int64_t Np, int j0, float *sl) {
  asm volatile("" ::: "memory");
  slice_copy_q<0, NPL>(tab, Np, j0, sl);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}
template <int NP>
__device__ __forceinline__ void lds_tblock(TBlock<NP> &B, const float *sl, int j, const int (&pl)[NP]) {
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const float4 *X = reinterpret_cast<const float4 *>(sl + pl[p] * kOtThreads + j);
    B.v[p][0] = X[0];
    B.v[p][1] = X[1];
  }
}
// the 32 blocks of 8 j of a staged slice, one block read ahead
#ifdef NFDPF_OT_LDS1
constexpr bool kLds1 = true;
#else
constexpr bool kLds1 = false;
#endif
template <int NP, bool ONE = kLds1, class Body>
__device__ __forceinline__ void slice_blocks(const float *sl, const int (&pl)[NP], const Body &body) {
  if constexpr (ONE) {  // one block at a time (32 fewer VGPRs; the SIMD's other waves cover the LDS latency)
    for (int j = 0; j < kOtThreads; j += 8) {
      TBlock<NP> A;
      lds_tblock(A, sl, j, pl);
      body(A);
    }
    return;
  }
  TBlock<NP> A, Bk;
  lds_tblock(A, sl, 0, pl);
  for (int j = 0; j < kOtThreads; j += 16) {
    lds_tblock(Bk, sl, j + 8, pl);
    __builtin_amdgcn_sched_barrier(0);
    body(A);
    __builtin_amdgcn_sched_barrier(0);
    lds_tblock(A, sl, j + 16, pl);  // past the end: the padding / the next plane, discarded
    __builtin_amdgcn_sched_barrier(0);
    body(Bk);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int KR>
struct LaneIK {  // the KR points of a lane, as packed splats
  f2 x[KR], y[KR];
};
using LaneI = LaneIK<kR>;

// Shifted-exponent block (planes X, Y, E_0..E_{NH-1}, V_0..V_{NV-1}; E = h - M_s):
//   acc[r][w] += 2^(E_w[j] + o[r][w] - sc |p_i - p_j|^2),  accv[r][v] += (w = 0 term) V_v[j]
// PS: prescaled points (the lane's and the table's X, Y times sqrt(sc)): the exponent is
// E + o - (dx^2 + dy^2), nsc2 unused.
template <int NH, int NV, int NP, bool PS = false, int KR>
__device__ __forceinline__ void hblock(const TBlock<NP> &B, const LaneIK<KR> &L, f2 nsc2, const f2 (&o)[KR][NH],
                                       f2 (&acc)[KR][NH], f2 (&accv)[KR][NV > 0 ? NV : 1]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      const f2 dx = L.x[r] - tpair(B, 0, q);
      const f2 dy = L.y[r] - tpair(B, 1, q);
      const f2 d2 = (PS && NH == 1) ? f2{} : pfma2(dy, dy, dx * dx);
#pragma unroll
      for (int w = 0; w < NH; ++w) {
        const f2 eo = tpair(B, 2 + w, q) + o[r][w];
        const f2 a = !PS ? pfma2(nsc2, d2, eo) : NH == 1 ? pfma2(-dy, dy, pfma2(-dx, dx, eo)) : eo - d2;
        const f2 t = f2{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
        acc[r][w] += t;
        if (w == 0)
#pragma unroll
          for (int v = 0; v < NV; ++v) accv[r][v] = pfma2(tpair(B, 2 + NH + v, q), t, accv[r][v]);
      }
    }
  }
}

// Shared-kernel block of the two iteration softmins (planes X, Y, alpha, beta): one
// v_exp_f32 per pair, K = 2^(-sc |p_i - p_j|^2);  acc[r][0] += alpha_j K,  acc[r][1] += beta_j K
template <int KR>
__device__ __forceinline__ void kblock(const TBlock<4> &B, const LaneIK<KR> &L, f2 nsc2, f2 (&acc)[KR][2]) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      const f2 dx = L.x[r] - tpair(B, 0, q);
      const f2 dy = L.y[r] - tpair(B, 1, q);
      const f2 a = kPrescale ? -pfma2(dy, dy, dx * dx) : pfma2(dy, dy, dx * dx) * nsc2;
      const f2 k = f2{__builtin_amdgcn_exp2f(a.x), __builtin_amdgcn_exp2f(a.y)};
      acc[r][0] = pfma2(tpair(B, 2, q), k, acc[r][0]);
      acc[r][1] = pfma2(tpair(B, 3, q), k, acc[r][1]);
    }
  }
}

__device__ __forceinline__ float hsum2(f2 a) { return a.x + a.y; }
__device__ __forceinline__ bool risky_any(bool r) { return __builtin_amdgcn_ballot_w64(r) != 0; }

// slice offset M_s - m_i in fp32 (-inf: the slice carries no weight)
__device__ __forceinline__ float slice_off(double Ms, double m) {
  return Ms > -INFINITY ? (float)(Ms - m) : -INFINITY;
}

// The lane's kR points and shifts: pt(i, x, y, m[NH]) for i = 256 s0 + lane + 64 r (i < N).
template <int NH, class Pt, int KR>
__device__ __forceinline__ void lane_points(int N, const Pt &pt, LaneIK<KR> &L, double (&m)[KR][NH], int rbase = 0) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    const int i = blockIdx.x * kOtThreads + lane + 64 * (rbase + r);
    float x = 0.f, y = 0.f;
    double mm[NH];
#pragma unroll
    for (int w = 0; w < NH; ++w) mm[w] = 0.0;
    if (i < N) pt(i, x, y, mm);
    L.x[r] = sp2(x);
    L.y[r] = sp2(y);
#pragma unroll
    for (int w = 0; w < NH; ++w) m[r][w] = mm[w];
  }
}

// Combine the waves' partials through LDS: thread t gets out[k] for its i (wave order).
// (8-wave iteration launches: waves w and w + 4 hold the same slices for the two halves of the
// lanes' i, rbase 0 / 2; both write slot w % 4, so the sums meet in the 4-wave order.)
template <int NK, int KR>
__device__ __forceinline__ void combine(float *lds, const float (&mine)[KR][NK], float (&out)[NK], int rbase = 0) {
  const int lane = threadIdx.x & 63, w = (threadIdx.x >> 6) % kWaves;
#pragma unroll
  for (int r = 0; r < KR; ++r)
#pragma unroll
    for (int k = 0; k < NK; ++k) lds[(w * NK + k) * kOtThreads + lane + 64 * (rbase + r)] = mine[r][k];
  __syncthreads();
  const int t = threadIdx.x % kOtThreads;  // threads >= kOtThreads get a copy (unused)
#pragma unroll
  for (int k = 0; k < NK; ++k) {
    float a = lds[k * kOtThreads + t];
    for (int u = 1; u < kWaves; ++u) a += lds[(u * NK + k) * kOtThreads + t];
    out[k] = a;
  }
}

// the scale of prescaled points (kPrescale): identical in the table writers and the pair loops
__device__ __forceinline__ float pscale(float sc) { return sqrtf(sc); }
template <int KR>
__device__ __forceinline__ void prescale(LaneIK<KR> &L, float sc) {
  const f2 s = sp2(pscale(sc));
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    L.x[r] *= s;
    L.y[r] *= s;
  }
}

// Workgroup sums over the whole row with the shifted-exponent block (table planes 0, 1,
// 2 .. 2+NH+NV, slice maxima msh[s * MS + w]): thread t gets, for i = 256 s0 + t,
//   S[w] = sum_j 2^(h_w[j] - sc |p_i - p_j|^2 - m_i[w]),  SV[v] = sum_j (w = 0 term) V_v[j].
template <int NH, int NV, int MS, bool PS = false, class Pt>
__device__ __forceinline__ void wg_table_sums(const float *tab, const double *msh, int splits, int64_t Np, int N,
                                              float sc, const Pt &pt, float *lds, float (&S)[NH], float *SV) {
  constexpr int NP = 2 + NH + NV;
  int pl[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) pl[p] = p;
  LaneI L;
  double m[kR][NH];
  lane_points<NH>(N, pt, L, m);
  if (PS) prescale(L, sc);
  const f2 nsc2 = sp2(-sc);
  f2 acc[kR][NH], accv[kR][NV > 0 ? NV : 1];
#pragma unroll
  for (int r = 0; r < kR; ++r) {
#pragma unroll
    for (int w = 0; w < NH; ++w) acc[r][w] = sp2(0.f);
#pragma unroll
    for (int v = 0; v < NV; ++v) accv[r][v] = sp2(0.f);
  }
  const int w0 = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
#ifndef NFDPF_OT_L1
  float *sl = lds + kLdsPart + w0 * kSliceFloats;
#endif
  for (int s = w0; s < splits; s += kWaves) {
    f2 o[kR][NH];
#pragma unroll
    for (int r = 0; r < kR; ++r)
#pragma unroll
      for (int w = 0; w < NH; ++w) o[r][w] = sp2(slice_off(msh[s * MS + w], m[r][w]));
#ifndef NFDPF_OT_L1
    slice_copy<NP>(tab, Np, s * kOtThreads, sl);
    slice_blocks<NP>(sl, pl, [&](const TBlock<NP> &B) { hblock<NH, NV, NP, PS>(B, L, nsc2, o, acc, accv); });
#else
    pipelined<NP>(tab, Np, s * kOtThreads, (s + 1) * kOtThreads, pl,
                  [&](const TBlock<NP> &B) { hblock<NH, NV, NP, PS>(B, L, nsc2, o, acc, accv); });
#endif
  }
  float mine[kR][NH + NV], out[NH + NV];
#pragma unroll
  for (int r = 0; r < kR; ++r) {
#pragma unroll
    for (int w = 0; w < NH; ++w) mine[r][w] = hsum2(acc[r][w]);
#pragma unroll
    for (int v = 0; v < NV; ++v) mine[r][NH + v] = hsum2(accv[r][v]);
  }
  combine<NH + NV>(lds, mine, out);
#pragma unroll
  for (int w = 0; w < NH; ++w) S[w] = out[w];
#pragma unroll
  for (int v = 0; v < NV; ++v) SV[v] = out[NH + v];
}

// The two softmins of an iteration over an iteration table (planes X, Y, h_a - M, h_b - M,
// alpha, beta; maxima msh[2 s], msh[2 s + 1]): one exp per pair for both unless some lane of
// the wave is "risky" for the slice (see the file header).
// W = 8 (iteration launches of small grids, ot_iter_waves): waves w and w + 4 take the same
// slices, each for half of the lanes' i (KR = 2), so every (i, slice) sum and the order in
// which they meet are those of the 4-wave launch -- bit-identical, twice the waves per SIMD.
template <int W = kWaves, class Pt>
__device__ __forceinline__ void wg_iter_sums(const float *tab, const double *msh, int splits, int64_t Np, int N,
                                             float sc, const Pt &pt, float *lds, float (&S)[2]) {
  static_assert(W == kWaves || W == 2 * kWaves, "iteration waves");
  constexpr int KR = W == kWaves ? kR : kR / 2;
  const int plk[4] = {0, 1, 4, 5}, plh[4] = {0, 1, 2, 3};
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int rbase = W == kWaves ? 0 : (wv / kWaves) * KR;
  // all kR points' shifts (the two-exp decision is taken over all of them, as in the 4-wave
  // launch); the wave's own KR points (rbase is wave-uniform: selects, no register indexing)
  LaneI La;
  double m[kR][2];
  lane_points<2>(N, pt, La, m);
  LaneIK<KR> L;
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    L.x[r] = rbase ? La.x[(kR - KR + r) % kR] : La.x[r];
    L.y[r] = rbase ? La.y[(kR - KR + r) % kR] : La.y[r];
  }
  if (kPrescale) prescale(L, sc);
  const f2 nsc2 = sp2(-sc);
  float Sk[KR][2];
  f2 hacc[KR][2];
  f2 none[KR][1];
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    Sk[r][0] = Sk[r][1] = 0.f;
    hacc[r][0] = hacc[r][1] = sp2(0.f);
  }
  const int w0 = wv % kWaves;  // the wave's slice set
#ifndef NFDPF_OT_L1
  float *sl = lds + kLdsPart + wv * kSliceFloats;
#endif
  for (int s = w0; s < splits; s += kWaves) {
    const double Ma = msh[2 * s], Mb = msh[2 * s + 1];
    float oa4[kR], ob4[kR], oa[KR], ob[KR];
    bool risky = false;
#pragma unroll
    for (int r = 0; r < kR; ++r) {
      oa4[r] = slice_off(Ma, m[r][0]);
      ob4[r] = slice_off(Mb, m[r][1]);
      risky |= (oa4[r] > kRisky) || (ob4[r] > kRisky);
    }
#pragma unroll
    for (int r = 0; r < KR; ++r) {
      oa[r] = rbase ? oa4[(kR - KR + r) % kR] : oa4[r];
      ob[r] = rbase ? ob4[(kR - KR + r) % kR] : ob4[r];
    }
    const int j0 = s * kOtThreads, j1 = j0 + kOtThreads;
#ifndef NFDPF_OT_L1
    slice_copy<6>(tab, Np, s * kOtThreads, sl);
    (void)j1;
#define OT_SLICE_LOOP(PL, ...) slice_blocks<4, kLds1 || W != kWaves>(sl, PL, __VA_ARGS__)
#else
#define OT_SLICE_LOOP(PL, ...) pipelined<4>(tab, Np, j0, j1, PL, __VA_ARGS__)
#endif
#ifdef NFDPF_OT_RISKSTAT
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(&g_ot_wslices, 1u);
      if (risky_any(risky)) atomicAdd(&g_ot_risky, 1u);
    }
#endif
    if (__builtin_amdgcn_ballot_w64(risky) == 0) {
      f2 acc[KR][2];
#pragma unroll
      for (int r = 0; r < KR; ++r) acc[r][0] = acc[r][1] = sp2(0.f);
      OT_SLICE_LOOP(plk, [&](const TBlock<4> &B) { kblock(B, L, nsc2, acc); });
#pragma unroll
      for (int r = 0; r < KR; ++r) {
        Sk[r][0] = fmaf(exp2f(oa[r]), hsum2(acc[r][0]), Sk[r][0]);
        Sk[r][1] = fmaf(exp2f(ob[r]), hsum2(acc[r][1]), Sk[r][1]);
      }
    } else {
      f2 o[KR][2];
#pragma unroll
      for (int r = 0; r < KR; ++r) {
        o[r][0] = sp2(oa[r]);
        o[r][1] = sp2(ob[r]);
      }
      OT_SLICE_LOOP(plh, [&](const TBlock<4> &B) { hblock<2, 0, 4, kPrescale>(B, L, nsc2, o, hacc, none); });
    }
#undef OT_SLICE_LOOP
  }
#ifdef NFDPF_EXP_OTTRACE
  if (threadIdx.x == 0 && OTT_WG < 1024) g_ot_loopend[OTT_WG] = __builtin_amdgcn_s_memrealtime();
#endif
  float mine[KR][2], out[2];
#pragma unroll
  for (int r = 0; r < KR; ++r) {
    mine[r][0] = Sk[r][0] + hsum2(hacc[r][0]);
    mine[r][1] = Sk[r][1] + hsum2(hacc[r][1]);
  }
  combine<2>(lds, mine, out, rbase);
  S[0] = out[0];
  S[1] = out[1];
}

__device__ __forceinline__ bool sum_ok(float s) { return s >= kLo && s <= kHi; }

// exact base-2 LSE_j(h(j) - sc * |x_i - x_j|^2) over the row (h in fp64, streamed max shift,
// global reads) -- the fallback of a lane whose shifted sum left the safe range
template <class H>
__device__ double lse2_exact(const float *xs, int N, float xi, float yi, float sc, const H &h) {
  double m = -INFINITY, s = 0.0;
  for (int j = 0; j < N; ++j) {
    const float dx = xi - xs[2 * j], dy = yi - xs[2 * j + 1];
    const double v = h(j) - (double)(fmaf(dx, dx, dy * dy) * sc);
    if (v > m) {
      s = s * exp2(m - v) + 1.0;
      m = v;
    } else {
      s += exp2(v - m);
    }
  }
  return m + log2(s);
}

// base-2 LSE from a shifted sum, or exactly when the sum left the safe range
template <class H>
__device__ __forceinline__ double lse2_from(float S, double m, const float *xs, int N, float xi, float yi, float sc,
                                            const H &h, int32_t *fallbacks) {
  if (sum_ok(S)) return m + log2((double)S);
  atomicAdd(fallbacks, 1);
  return lse2_exact(xs, N, xi, yi, sc, h);
}

// Thread's column of a table (j = kOtThreads blockIdx.x + threadIdx.x, threads < kOtThreads): planes X, Y, then NE exponent
// planes stored as h - M_s (slice maxima to msh[blockIdx.x * NE + e]), then NV value planes.
// With ALPHA, planes 2 + NE + e hold 2^(h_e - M_s) (the iteration table's alpha / beta).
// The slice maxima M[e] come from the caller (col_max: one workgroup reduction for all of them).
template <int NE, int NV, bool ALPHA>
__device__ __forceinline__ void write_col_m(float *tab, double *msh, int64_t Np, bool valid, float X, float Y,
                                            const double (&h)[NE], const double *Ms, const float *vals) {
  const int64_t j = (int64_t)blockIdx.x * kOtThreads + threadIdx.x;
  const bool own = threadIdx.x < kOtThreads;  // the slice's columns; other threads only reduce
  valid = valid && own;
  if (own) {
    tab[j] = valid ? X : 0.f;
    tab[Np + j] = valid ? Y : 0.f;
  }
#pragma unroll
  for (int e = 0; e < NE; ++e) {
    const double he = valid ? h[e] : -INFINITY;
    const double M = Ms[e];
    const float E = (he > -INFINITY) ? (float)(he - M) : -INFINITY;
    if (own) tab[(2 + e) * Np + j] = E;
    if (ALPHA && own) tab[(2 + NE + e) * Np + j] = E > -INFINITY ? __builtin_amdgcn_exp2f(E) : 0.f;
    if (threadIdx.x == 0) msh[blockIdx.x * NE + e] = M;
  }
#pragma unroll
  for (int v = 0; v < NV; ++v)
    if (own) tab[(2 + NE + (ALPHA ? NE : 0) + v) * Np + j] = valid ? vals[v] : 0.f;
}
// the column's exponents as the inputs of the slice maxima (-inf outside the slice)
template <int NE>
__device__ __forceinline__ void col_exps(bool valid, const double (&h)[NE], double *out) {
  valid = valid && threadIdx.x < kOtThreads;
#pragma unroll
  for (int e = 0; e < NE; ++e) out[e] = valid ? h[e] : -INFINITY;
}
template <int NE, int NV, bool ALPHA>
__device__ __forceinline__ void write_col(float *tab, double *msh, int64_t Np, bool valid, float X, float Y,
                                          const double (&h)[NE], const float *vals, double *shd) {
  double M[NE];
  col_exps<NE>(valid, h, M);
  block_max_n<NE>(M, shd);
  write_col_m<NE, NV, ALPHA>(tab, msh, Np, valid, X, Y, h, M, vals);
}

// ------------------------------------------------------------------------------------------
// setup + the initial table, one launch of (splits, B) workgroups: every workgroup of row b
// reduces the whole row itself -- centre/scale (transport_function :218-222), eps0 = max_min^2
// (:87-91, :117), the largest log weight -- in the same order as its row's other workgroups
// (identical results), writes the scaled points / log weights of its own slice and, slice 0,
// the row's constants; then its slice of the table of the initial softmins at eps0
// (:120-121): h_a = logw, h_b = logu (base 2).  (Round 1-6: a row launch of up to 1024
// threads, then the table launch: 15 + 5 us at C3.)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(kOtBlock) void ot_setup_kernel(const float *__restrict__ x, const float *__restrict__ w,
                                                            OtParams P, OtWs ws) {
  if (ot_off(P)) return;
  __shared__ double shd[32];
  __shared__ float shf[16];
  const int b = blockIdx.y, N = P.N, s0i = blockIdx.x * kOtThreads, s1i = min(s0i + kOtThreads, N);
  const float *xr = x + (int64_t)b * P.x_rs;
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
  auto sx = [&](int i) { return (float)((double)(xr[2 * i] - m0) / scale); };
  auto sy = [&](int i) { return (float)((double)(xr[2 * i + 1] - m1) / scale); };
  auto lwf = [&](int i) { return logf(w[(int64_t)b * P.w_rs + i]); };
  float mx = -INFINITY, mn = INFINITY, lwmax = -INFINITY;
  for (int i = threadIdx.x; i < N; i += blockDim.x) {
    const float a = sx(i), c = sy(i), lw = lwf(i);
    if (i >= s0i && i < s1i) {  // this workgroup's slice
      ws.xs[((int64_t)b * N + i) * 2] = a;
      ws.xs[((int64_t)b * N + i) * 2 + 1] = c;
      ws.logw[(int64_t)b * N + i] = lw;
    }
    mx = fmaxf(mx, fmaxf(a, c));
    mn = fminf(mn, fminf(a, c));
    lwmax = fmaxf(lwmax, lw);
  }
  mx = block_max(mx, shf);
  mn = -block_max(-mn, shf);
  lwmax = block_max(lwmax, shf);
  const double mm = (double)mx - (double)mn;
  const double eps0 = mm * mm, logu = -(double)logf((float)N);
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    ws.rowc[b * 4 + 0] = eps0;           // epsilon_0 = diameter^2 (:117)
    ws.rowc[b * 4 + 1] = logu;           // uniform log weight (:214-215)
    ws.rowc[b * 4 + 2] = (double)lwmax;  // shift of the first a-softmin
    double e = eps0;                     // eps_k, k = 0 .. kEpsTab-1 (:158)
    for (int k = 0; k < kEpsTab; ++k) {
      ws.epsk[(int64_t)b * kEpsTab + k] = e;
      e = fmax(e * P.sf, P.eps);
    }
    if (b == 0) {
#ifdef NFDPF_OT_RISKSTAT
      g_ot_risky = 0;
      g_ot_wslices = 0;
#endif
      ws.st->stopped = 0;
      ws.st->K = 0;
      ws.st->fallbacks = 0;
    }
  }
  // the slice's table columns (thread t: i = s0i + t), from the same expressions
  const int i = s0i + threadIdx.x;
  const bool v = i < N && threadIdx.x < kOtThreads;
  const double h[2] = {v ? (double)lwf(i) * kLog2ed : 0.0, logu * kLog2ed};
  const float sc = kPrescale ? pscale(cost_scale(1.0 / eps0)) : 1.f;  // ot_init's epsilon
  write_col<2, 0, true>(tabI_row(ws, P, 1, b), mI_row(ws, P, 1, b), np_of(P), v, v ? sx(i) * sc : 0.f,
                        v ? sy(i) * sc : 0.f, h, nullptr, shd);
}

// Table columns of state `ks` (the potentials a_y, b_x of thread i just produced): for the
// iteration that consumes it (epsilon e_ks) and, for a row whose epsilon is still annealing,
// at the final epsilon (the post-loop softmin :173-176, should the batch stop right here).
// All slice maxima of both tables -- and the caller's residual maximum *dmax, if given -- in ONE
// workgroup reduction (shd: 5 doubles per wave).  r02c took two barriers and a shuffle chain
// per maximum (up to 5 per iteration launch).
__device__ __forceinline__ void emit_state_tables(const OtParams &P, const OtWs &ws, int b, int ks, bool v,
                                                  float xi, float yi, float lw, double logu, double ay,
                                                  double bx, double *shd, double *dmax = nullptr) {
  const int64_t Np = np_of(P);
  const double e = eps_at(ws, P, b, ks);
  const bool fin = e != P.eps;  // the row is still annealing: also the final-epsilon table
  const double inv = 1.0 / e, invF = 1.0 / P.eps;
  const double hI[2] = {((double)lw + bx * inv) * kLog2ed, (logu + ay * inv) * kLog2ed};
  const double hF[2] = {((double)lw + bx * invF) * kLog2ed, (logu + ay * invF) * kLog2ed};
  double M[5];
  col_exps<2>(v, hI, M);
  col_exps<2>(v && fin, hF, M + 2);
  M[4] = dmax ? *dmax : 0.0;
  block_max_n<5>(M, shd);
  if (dmax) *dmax = M[4];
  {
    const float s = kPrescale ? pscale(cost_scale(inv)) : 1.f;
    write_col_m<2, 0, true>(tabI_row(ws, P, ks & 1, b), mI_row(ws, P, ks & 1, b), Np, v, xi * s, yi * s, hI, M,
                            nullptr);
  }
  if (fin) {
    const float s = kPrescale ? pscale(cost_scale(invF)) : 1.f;
    write_col_m<2, 0, false>(ws.tabF + (int64_t)b * 4 * Np, ws.mF + (int64_t)b * P.splits * 2, Np, v, xi * s,
                             yi * s, hF, M + 2, nullptr);
  }
}

// the two softmins of an iteration for thread t's i (shifts ma / mb, base 2), from the
// workgroup sums with the lanes' shifts pt(i) -> (x, y, {m_a, m_b}); exact when a sum left
// the safe range.  Returns the softmins -e ln2 LSE2 in fp64.
template <int W = kWaves, class Pt, class HA, class HB>
__device__ __forceinline__ void softmin_pair(const OtParams &P, const float *tab, const double *msh,
                                             const float *xs, bool v, float xi, float yi, double e, double ma,
                                             double mb, const Pt &pt, const HA &ha, const HB &hb, float *lds,
                                             double &A, double &Bv, int32_t *fb) {
  const float sc = cost_scale(1.0 / e);
  float S[2];
  wg_iter_sums<W>(tab, msh, P.splits, np_of(P), P.N, sc, pt, lds, S);
  if (v) {
    A = -e * lse2_from(S[0], ma, xs, P.N, xi, yi, sc, ha, fb) * kLn2d;
    Bv = -e * lse2_from(S[1], mb, xs, P.N, xi, yi, sc, hb, fb) * kLn2d;
  }
}

// initial potentials at eps0 (:120-121): a_y = softmin(eps0, C, logw), b_x = softmin(eps0, C, logu)
__global__ __launch_bounds__(kOtBlock) void ot_init_kernel(OtParams P, OtWs ws) {
  if (ot_off(P)) return;
  __shared__ double shd[32];
  __shared__ __attribute__((aligned(16))) float lds[kLdsAll];
  const int b = blockIdx.y, N = P.N;
  const int i = blockIdx.x * kOtThreads + threadIdx.x;
  const bool v = i < N && threadIdx.x < kOtThreads;
  const float *xs = ws.xs + (int64_t)b * N * 2;
  const float *lw = ws.logw + (int64_t)b * N;
  const double e = ws.rowc[b * 4], logu = ws.rowc[b * 4 + 1];
  const float xi = v ? xs[2 * i] : 0.f, yi = v ? xs[2 * i + 1] : 0.f;
  // shifts: the largest exponent of the row (the costs are <= 1/2 here: eps0 = diameter^2)
  const double ma = ws.rowc[b * 4 + 2] * kLog2ed, mb = logu * kLog2ed;
  double A = 0.0, Bv = 0.0;
  softmin_pair(
      P, tabI_row(ws, P, 1, b), mI_row(ws, P, 1, b), xs, v, xi, yi, e, ma, mb,
      [&](int ii, float &x, float &y, double (&m)[2]) {
        x = xs[2 * ii];
        y = xs[2 * ii + 1];
        m[0] = ma;
        m[1] = mb;
      },
      [&](int j) { return (double)lw[j] * kLog2ed; }, [&](int) { return mb; }, lds, A, Bv, &ws.st->fallbacks);
  if (v) {
    pot_ptr(ws, P, 0, 0, b)[i] = A;
    pot_ptr(ws, P, 0, 1, b)[i] = Bv;
  }
  emit_state_tables(P, ws, b, 0, v, xi, yi, v ? lw[i] : 0.f, logu, A, Bv, shd);
}

// does the loop stop before iteration k?  (stop_condition :126-129) -- every workgroup
// evaluates the same residuals of iteration k-1 (wave 0, lanes over rows; every load of a
// lane independent, one memory latency).  r01 ran this on one lane, row after row with the
// epsilon recurrence re-run per row: a serial chain at the start of every iteration launch.
__device__ __forceinline__ bool ot_stop_before(const OtParams &P, const OtWs &ws, int k) {
  if (k == 0) return false;
  if (P.stop_at) return k >= *P.stop_at - 2;  // the batch-global decision, taken by the caller
  const double *res = ws.res + (int64_t)((k - 1) & 1) * P.B * P.splits;
  bool conv = false;
  for (int b = threadIdx.x & 63; b < P.B; b += 64) {
    const double re = eps_at(ws, P, b, k - 1);
    const double ne = fmax(re * P.sf, P.eps);
    double mx = 0.0;
    for (int s = 0; s < P.splits; ++s) mx = fmax(mx, res[b * P.splits + s]);
    conv |= !(ne < re || mx > P.thr);  // this row converged -> torch.all(continue_) is False
  }
  return __builtin_amdgcn_ballot_w64(conv) != 0;
}

// iteration k: state k (buffer k&1) -> state k+1 (buffer (k+1)&1)  (apply_one :131-153)
#ifndef NFDPF_OT_ITER_WPS
#define NFDPF_OT_ITER_WPS 1
#endif
template <int W>
__global__ __launch_bounds__(64 * W, W == 2 * kWaves ? 4 : NFDPF_OT_ITER_WPS) void ot_iter_kernel(
    OtParams P, OtWs ws, int k) {
  const bool lead = blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0;
  OTTRACE(k, 0)
  if (ot_off(P)) {
    if (lead && P.host) host_flag(P.host, 0, P.seq);  // nothing to iterate: stop enqueueing
    return;
  }
  __shared__ double shd[64];  // block_max_n<5> over up to 8 waves
  __shared__ __attribute__((aligned(16))) float lds[kLdsPart + W * kSliceFloats];
  __shared__ int s_stop;
  if (threadIdx.x < 64) {  // wave 0 (ot_stop_before is a wave-level decision)
    int st = ws.st->stopped;
    if (!st && ot_stop_before(P, ws, k)) {
      st = 1;
      if (lead) {
        ws.st->stopped = 1;
        ws.st->K = k;
      }
    }
    if (threadIdx.x == 0) s_stop = st;
    if (lead && P.host) {
      host_flag(P.host, 1, P.seq * 4096 + k);
      if (st) host_flag(P.host, 0, P.seq);
    }
  }
  __syncthreads();
  if (s_stop) return;
  OTTRACE(k, 1)
  const int b = blockIdx.y, N = P.N;
  const int i = blockIdx.x * kOtThreads + threadIdx.x;
  const bool v = i < N && threadIdx.x < kOtThreads;
  const double re = eps_at(ws, P, b, k), inv = 1.0 / re;
  const float *xs = ws.xs + (int64_t)b * N * 2;
  const float *lw = ws.logw + (int64_t)b * N;
  const double logu = ws.rowc[b * 4 + 1];
  const double *ay = pot_ptr(ws, P, k, 0, b), *bx = pot_ptr(ws, P, k, 1, b);
  const float xi = v ? xs[2 * i] : 0.f, yi = v ? xs[2 * i + 1] : 0.f;
  // at_y = softmin(e, C, logw + b_x/e);  bt_x = softmin(e, C, logu + a_y/e); shifts from the
  // current potentials (softmin = -e ln2 LSE2)
  const double sh = -inv * kLog2ed;
  const double oa = v ? ay[i] : 0.0, ob = v ? bx[i] : 0.0;
  double A = 0.0, Bv = 0.0;
  softmin_pair<W>(
      P, tabI_row(ws, P, k & 1, b), mI_row(ws, P, k & 1, b), xs, v, xi, yi, re, oa * sh, ob * sh,
      [&](int ii, float &x, float &y, double (&m)[2]) {
        x = xs[2 * ii];
        y = xs[2 * ii + 1];
        m[0] = ay[ii] * sh;
        m[1] = bx[ii] * sh;
      },
      [&](int j) { return ((double)lw[j] + bx[j] * inv) * kLog2ed; },
      [&](int j) { return (logu + ay[j] * inv) * kLog2ed; }, lds, A, Bv, &ws.st->fallbacks);
  OTTRACE(k, 3)
#ifdef NFDPF_EXP_OTTRACE
  if (threadIdx.x == 0 && OTT_WG < 1024) g_ot_tr[OTT_WG][k & 63][2] = g_ot_loopend[OTT_WG];
#endif
  double na = 0.0, nb = 0.0, dmax = 0.0;
  if (v) {
    na = 0.5 * (oa + A);
    nb = 0.5 * (ob + Bv);
    pot_ptr(ws, P, k + 1, 0, b)[i] = na;
    pot_ptr(ws, P, k + 1, 1, b)[i] = nb;
    dmax = fmax(fabs(na - oa), fabs(nb - ob));
  }
  OTTRACE(k, 4)
  emit_state_tables(P, ws, b, k + 1, v, xi, yi, v ? lw[i] : 0.f, logu, na, nb, shd, &dmax);
  OTTRACE(k, 5)
#ifdef NFDPF_EXP_OTTRACE
  if (threadIdx.x == 0 && OTT_WG < 1024) {
    g_ot_tr[OTT_WG][k & 63][6] = __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_ID (CU, SIMD, SE)
    g_ot_tr[OTT_WG][k & 63][7] = __builtin_amdgcn_s_getreg(20 | (31 << 11));  // XCC_ID
  }
#endif
  if (threadIdx.x == 0) ws.res[((int64_t)(k & 1) * P.B + b) * P.splits + blockIdx.x] = dmax;
}

__device__ __forceinline__ int ot_total_iter(const OtParams &P, const OtWs &ws) {
  // the caller's count (a sharded batch's global stop, the MIN over ranks of their own)
  if (P.stop_at) return max(min(*P.stop_at - 2, P.max_iter - 1), 0);  // (a stop_at < 2 reads state 0)
  return ws.st->stopped ? ws.st->K : max(P.max_iter - 1, 0);
}

// The tables of state K = the batch-global stop, rebuilt from the potential history: a rank
// whose own rows converged later has since overwritten them (the iteration tables are
// double-buffered, the final-epsilon table is rewritten every annealing iteration).  The same
// workgroup reduction as the iteration epilogue that first wrote them: bit-identical tables.
__global__ __launch_bounds__(kOtBlock) void ot_restore_kernel(OtParams P, OtWs ws) {
  if (ot_off(P)) return;
  __shared__ double shd[32];
  const int b = blockIdx.y, N = P.N;
  const int i = blockIdx.x * kOtThreads + threadIdx.x;
  const bool v = i < N && threadIdx.x < kOtThreads;
  const int K = ot_total_iter(P, ws);
  const float *xs = ws.xs + (int64_t)b * N * 2;
  const float *lw = ws.logw + (int64_t)b * N;
  const double *ay = pot_ptr(ws, P, K, 0, b), *bx = pot_ptr(ws, P, K, 1, b);
  emit_state_tables(P, ws, b, K, v, v ? xs[2 * i] : 0.f, v ? xs[2 * i + 1] : 0.f, v ? lw[i] : 0.f,
                    ws.rowc[b * 4 + 1], v ? ay[i] : 0.0, v ? bx[i] : 0.0, shd);
}

// final potential at eps (:173-176): f = softmin(eps, C, logw + b_x/eps).  (g = softmin(eps,
// C, logu + a_y/eps) cancels in the column normalisation of the transport matrix: not formed.)
// Writes the column table: X, Y, f_i / eps (base 2).
__global__ __launch_bounds__(kOtBlock) void ot_final_kernel(OtParams P, OtWs ws) {
  if (ot_off(P)) return;
  __shared__ double shd[32];
  __shared__ __attribute__((aligned(16))) float lds[kLdsAll];
  const int b = blockIdx.y, N = P.N;
  const int i = blockIdx.x * kOtThreads + threadIdx.x;
  const bool v = i < N && threadIdx.x < kOtThreads;
  const int64_t Np = np_of(P);
  const int K = ot_total_iter(P, ws);
  const double e = P.eps, inv = 1.0 / P.eps;
  const float sc = cost_scale(inv);
  const float *xs = ws.xs + (int64_t)b * N * 2;
  const float *lw = ws.logw + (int64_t)b * N;
  const double *ay = pot_ptr(ws, P, K, 0, b), *bx = pot_ptr(ws, P, K, 1, b);
  // the state's iteration table is at eps unless the row was still annealing at the stop
  const bool annealing = eps_at(ws, P, b, K) != P.eps;
  const float *tab = annealing ? ws.tabF + (int64_t)b * 4 * Np : tabI_row(ws, P, K & 1, b);
  const double *msh = annealing ? ws.mF + (int64_t)b * P.splits * 2 : mI_row(ws, P, K & 1, b);
  const float xi = v ? xs[2 * i] : 0.f, yi = v ? xs[2 * i + 1] : 0.f;
  const double sh = -inv * kLog2ed;  // f is the softmin that a_y converged to
  float S[1];
  wg_table_sums<1, 0, 2, kPrescale>(tab, msh, P.splits, Np, N, sc,
                         [&](int ii, float &x, float &y, double (&m)[1]) {
                           x = xs[2 * ii];
                           y = xs[2 * ii + 1];
                           m[0] = ay[ii] * sh;
                         },
                         lds, S, nullptr);
  double fe = 0.0;
  if (v) {
    const double L = lse2_from(S[0], ay[i] * sh, xs, N, xi, yi, sc,
                               [&](int j) { return ((double)lw[j] + bx[j] * inv) * kLog2ed; }, &ws.st->fallbacks);
    const double f = -e * L * kLn2d;
    ws.fg[(int64_t)b * N + i] = f;
    fe = f * inv * kLog2ed;
  }
  const double h[1] = {fe};
  write_col<1, 0, false>(ws.tabC + (int64_t)b * 3 * Np, ws.mC + (int64_t)b * P.splits, Np, v, xi, yi, h, nullptr,
                         shd);
}

// r_j = log N + logw_j - LSE_i(f_i/eps - C_ij/eps)   (transport_from_potentials :200-207,
// with the column log-normaliser; g_j cancels).  Writes the apply table: X, Y, r_j, x_j, y_j.
__global__ __launch_bounds__(kOtBlock) void ot_col_kernel(OtParams P, OtWs ws, const float *__restrict__ x) {
  if (ot_off(P)) return;
  __shared__ double shd[32];
  __shared__ __attribute__((aligned(16))) float lds[kLdsAll];
  const int b = blockIdx.y, N = P.N;
  const int j = blockIdx.x * kOtThreads + threadIdx.x;
  const bool v = j < N && threadIdx.x < kOtThreads;
  const int64_t Np = np_of(P);
  const int K = ot_total_iter(P, ws);
  const double inv = 1.0 / P.eps;
  const float sc = cost_scale(inv);
  const float *xs = ws.xs + (int64_t)b * N * 2;
  const double *f = ws.fg + (int64_t)b * N;
  const double *bx = pot_ptr(ws, P, K, 1, b);
  const double logu = ws.rowc[b * 4 + 1];
  const float xj = v ? xs[2 * j] : 0.f, yj = v ? xs[2 * j + 1] : 0.f;
  // LSE_i(f_i/eps - C_ij/eps) = -b_x_j/eps - logu at the Sinkhorn fixed point
  auto shift = [&](int jj) { return (-bx[jj] * inv - logu) * kLog2ed; };
  float S[1];
  wg_table_sums<1, 0, 1>(ws.tabC + (int64_t)b * 3 * Np, ws.mC + (int64_t)b * P.splits, P.splits, Np, N, sc,
                         [&](int jj, float &xx, float &yy, double (&m)[1]) {
                           xx = xs[2 * jj];
                           yy = xs[2 * jj + 1];
                           m[0] = shift(jj);
                         },
                         lds, S, nullptr);
  double rj = 0.0;
  if (v) {
    const double L = lse2_from(S[0], shift(j), xs, N, xj, yj, sc, [&](int i) { return f[i] * inv * kLog2ed; },
                               &ws.st->fallbacks);
    rj = -logu + (double)ws.logw[(int64_t)b * N + j] - L * kLn2d;
  }
  const double h[1] = {rj * kLog2ed};
  const float vals[2] = {v ? x[(int64_t)b * P.x_rs + 2 * j] : 0.f, v ? x[(int64_t)b * P.x_rs + 2 * j + 1] : 0.f};
  write_col<1, 2, false>(ws.tabA + (int64_t)b * 5 * Np, ws.mA + (int64_t)b * P.splits, Np, v, xj, yj, h, vals, shd);
}

// x'_i = sum_j T_ij x_j with T_ij = exp(f_i/eps - C_ij/eps + r_j)  (apply_transport_matrix
// :254-264): the terms are the matrix entries themselves (shift -f_i/eps, sum ~ 1)
__global__ __launch_bounds__(kOtBlock) void ot_apply_kernel(OtParams P, OtWs ws,
                                                             const float *__restrict__ x,
                                                             int64_t row_base,
                                                             float *__restrict__ x_out,
                                                             float *__restrict__ w_out,
                                                             int64_t *__restrict__ idx_out,
                                                             int32_t *__restrict__ iters_out) {
  // the call's iteration count (iters_out encoding; 0: the gate was off), from the first lane
  if (iters_out && blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0)
    iters_out[0] = ot_off(P) ? 0 : ot_total_iter(P, ws) + 2;
  if (ot_off(P)) return;
  __shared__ __attribute__((aligned(16))) float lds[kLdsAll];
  const int b = blockIdx.y, N = P.N;
  const int i = blockIdx.x * kOtThreads + threadIdx.x;
  const bool v = i < N && threadIdx.x < kOtThreads;
  const int64_t Np = np_of(P);
  const double inv = 1.0 / P.eps;
  const float sc = cost_scale(inv);
  const float *xs = ws.xs + (int64_t)b * N * 2;
  const double *fg = ws.fg + (int64_t)b * N;
  const double fsh = inv * kLog2ed;
  float S[1], SV[2];
  wg_table_sums<1, 2, 1>(ws.tabA + (int64_t)b * 5 * Np, ws.mA + (int64_t)b * P.splits, P.splits, Np, N, sc,
                         [&](int ii, float &xx, float &yy, double (&m)[1]) {
                           xx = xs[2 * ii];
                           yy = xs[2 * ii + 1];
                           m[0] = -fg[ii] * fsh;
                         },
                         lds, S, SV);
  if (!v) return;
  float ax = SV[0], ay = SV[1];
  if (!sum_ok(S[0])) {  // exact: max shift first, then the weighted sums (fp64 exponents)
    atomicAdd(&ws.st->fallbacks, 1);
    const float xi = xs[2 * i], yi = xs[2 * i + 1];
    const double fi = fg[i] * fsh;
    const float *xr = x + (int64_t)b * P.x_rs;
    const float *E = ws.tabA + (int64_t)b * 5 * Np + 2 * Np;  // r_j - M_s
    const double *ms = ws.mA + (int64_t)b * P.splits;
    auto expo = [&](int j) {
      const float dx = xi - xs[2 * j], dy = yi - xs[2 * j + 1];
      return fi + (double)E[j] + ms[j / kOtThreads] - (double)(fmaf(dx, dx, dy * dy) * sc);
    };
    double mx = -INFINITY;
    for (int j = 0; j < N; ++j) mx = fmax(mx, expo(j));
    double sx = 0.0, sy = 0.0;
    for (int j = 0; j < N; ++j) {
      const double t = exp2(expo(j) - mx);
      sx += t * xr[2 * j];
      sy += t * xr[2 * j + 1];
    }
    const double R = exp2(mx);
    ax = (float)(sx * R);
    ay = (float)(sy * R);
  }
  const int64_t o = (int64_t)b * N + i;
  x_out[2 * o] = ax;
  x_out[2 * o + 1] = ay;
  w_out[o] = 1.0f / (float)N;
  idx_out[o] = (int64_t)N * (row_base + b) + i;
}

// ---- backward (training) ----------------------------------------------
// The reference differentiates x' = bmm(T, x) with T a constant (its transport Function's own
// autograd.grad result is discarded, resamplers.py:234-245), so dL/dx_j = sum_i T_ij g_i.
// Column j:  T_ij = 2^(F_i + R_j - c_ij) (F = f/eps, R = r log2 e as in the apply pass) and
// sum_i T_ij = N w_j exactly (r_j is the column log-normaliser), so with the shift
// L_j = log2 N + log2 w_j - R_j the shifted sum over i is 1 and dL/dx_j = N w_j * SV_j.
// The forward's workspace must be untouched since its call; the iteration tables (free after
// the loop) hold the backward's table: X, Y, F_i - M, g_x, g_y.
__global__ __launch_bounds__(kOtBlock) void ot_bwd_table_kernel(OtParams P, OtWs ws,
                                                                 const float *__restrict__ g) {
  if (ot_off(P)) return;
  __shared__ double shd[32];
  const int b = blockIdx.y, N = P.N;
  const int i = blockIdx.x * kOtThreads + threadIdx.x;
  const bool v = i < N && threadIdx.x < kOtThreads;
  const int64_t Np = np_of(P);
  const float *xs = ws.xs + (int64_t)b * N * 2;
  const double fsh = (1.0 / P.eps) * kLog2ed;
  const double h[1] = {v ? ws.fg[(int64_t)b * N + i] * fsh : 0.0};
  const float vals[2] = {v ? g[((int64_t)b * N + i) * 2] : 0.f, v ? g[((int64_t)b * N + i) * 2 + 1] : 0.f};
  write_col<1, 2, false>(tabI_row(ws, P, 0, b), mI_row(ws, P, 0, b), Np, v, v ? xs[2 * i] : 0.f,
                         v ? xs[2 * i + 1] : 0.f, h, vals, shd);
}

__global__ __launch_bounds__(kOtBlock) void ot_bwd_apply_kernel(OtParams P, OtWs ws,
                                                                 const float *__restrict__ g,
                                                                 float *__restrict__ g_x) {
  const int b = blockIdx.y, N = P.N;
  const int j = blockIdx.x * kOtThreads + threadIdx.x;
  const bool v = j < N && threadIdx.x < kOtThreads;
  const int64_t o = (int64_t)b * N + j;
  if (ot_off(P)) {  // no resampling happened: x' = x
    if (v) {
      g_x[2 * o] = g[2 * o];
      g_x[2 * o + 1] = g[2 * o + 1];
    }
    return;
  }
  __shared__ __attribute__((aligned(16))) float lds[kLdsAll];
  const int64_t Np = np_of(P);
  const float sc = cost_scale(1.0 / P.eps);
  const float *xs = ws.xs + (int64_t)b * N * 2;
  const float *EA = ws.tabA + (int64_t)b * 5 * Np + 2 * Np;  // R_j - M_s
  const double *mA = ws.mA + (int64_t)b * P.splits;
  const double log2N = log2((double)N);
  auto shift = [&](int jj) {  // L_j (0 for a column of zero weight: it carries nothing)
    const double lw = (double)ws.logw[(int64_t)b * N + jj];
    return lw > -INFINITY ? log2N + lw * kLog2ed - ((double)EA[jj] + mA[jj / kOtThreads]) : 0.0;
  };
  const float *tab = tabI_row(ws, P, 0, b);
  const double *msh = mI_row(ws, P, 0, b);
  float S[1], SV[2];
  wg_table_sums<1, 2, 1>(tab, msh, P.splits, Np, N, sc,
                         [&](int jj, float &xx, float &yy, double (&m)[1]) {
                           xx = xs[2 * jj];
                           yy = xs[2 * jj + 1];
                           m[0] = shift(jj);
                         },
                         lds, S, SV);
  if (!v) return;
  const double lw = (double)ws.logw[o];
  if (!(lw > -INFINITY)) {
    g_x[2 * o] = 0.f;
    g_x[2 * o + 1] = 0.f;
    return;
  }
  const double Nw = (double)N * exp(lw);
  double gx = SV[0], gy = SV[1];
  if (!sum_ok(S[0])) {  // exact: max shift first, then the weighted sums (fp64 exponents)
    atomicAdd(&ws.st->fallbacks, 1);
    const float xj = xs[2 * j], yj = xs[2 * j + 1];
    const double Lj = shift(j), fsh = (1.0 / P.eps) * kLog2ed;
    const float *gr = g + (int64_t)b * N * 2;
    auto expo = [&](int i) {
      const float dx = xs[2 * i] - xj, dy = xs[2 * i + 1] - yj;
      return ws.fg[(int64_t)b * N + i] * fsh - Lj - (double)(fmaf(dx, dx, dy * dy) * sc);
    };
    double mx = -INFINITY;
    for (int i = 0; i < N; ++i) mx = fmax(mx, expo(i));
    double sx = 0.0, sy = 0.0;
    for (int i = 0; i < N; ++i) {
      const double t = exp2(expo(i) - mx);
      sx += t * gr[2 * i];
      sy += t * gr[2 * i + 1];
    }
    gx = sx * exp2(mx);
    gy = sy * exp2(mx);
  }
  g_x[2 * o] = (float)(Nw * gx);
  g_x[2 * o + 1] = (float)(Nw * gy);
}

__global__ void ot_iters_kernel(OtParams P, OtWs ws, int32_t *out) {
  out[0] = ot_off(P) ? 0 : ot_total_iter(P, ws) + 2;
}

}  // namespace nfdpf

using namespace nfdpf;

// Waves per iteration workgroup: 4, or 8 with NFDPF_OT_ITER_WAVES=8 (the lanes' i split over
// wave pairs, wg_iter_sums; bit-identical, tests/test_gpu_parity.py).  Measured (round 2d, one
// box): at C3 (64 rows x 4 slices = one 4-wave workgroup per CU, one wave per SIMD) 8 waves did
// not shorten the iteration (18.1-18.3 vs 18.4-20.8 us, pass within noise); forced at C4 they
// cost 8 % (125 vs 117 us); with one LDS block at a time and 126 VGPRs (4 waves per SIMD at C4,
// the build below) still 4 % slower at C4 (122-124 vs 117-120 us) and 6 % at C3 forced -- the
// iteration is throughput-bound, not latency-bound.  So 4 is the default at every grid size.
static int ot_iter_waves(int /*wgs*/) {
  const char *e = getenv("NFDPF_OT_ITER_WAVES");  // read per call (tests switch it)
  return (e && atoi(e) == 2 * kWaves) ? 2 * kWaves : kWaves;
}

#ifdef NFDPF_EXP_OTTRACE
extern "C" __attribute__((visibility("default"))) int nfdpf_exp_ottrace(uint64_t *host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_ot_tr), sizeof(g_ot_tr)) == hipSuccess ? 0 : -1;
}
#endif

extern "C" int64_t nfdpf_ot_workspace_bytes(int B, int N) {
  return (B <= 0 || N <= 0) ? 256 : ws_bytes(B, N);
}

extern "C" int nfdpf_ot_stats(const void *workspace, int32_t *host_out) {
  NFDPF_REQUIRE(workspace && host_out, "nfdpf_ot_stats: null pointer");
  OtState st;
  if (hipMemcpy(&st, workspace, sizeof(st), hipMemcpyDeviceToHost) != hipSuccess)
    return launch_status("nfdpf_ot_stats");
  host_out[0] = st.stopped ? st.K + 2 : -1;
  host_out[1] = st.fallbacks;
#ifdef NFDPF_OT_RISKSTAT  // per-mille of wave-slices on the two-exp path instead
  unsigned int rk = 0, ns = 0;
  if (hipMemcpyFromSymbol(&rk, HIP_SYMBOL(g_ot_risky), sizeof(rk)) != hipSuccess ||
      hipMemcpyFromSymbol(&ns, HIP_SYMBOL(g_ot_wslices), sizeof(ns)) != hipSuccess)
    return launch_status("nfdpf_ot_stats");
  host_out[1] = ns ? (int32_t)((1000ull * rk) / ns) : -1;
#endif
  return NFDPF_OK;
}

// poll mode: library-owned flags in fine-grained (coherent, mapped) host memory, allocated on
// first use and kept for the process; one polled call at a time
static std::mutex g_poll_mu;
static int32_t g_poll_seq = 0;
static bool poll_flags(volatile int32_t **host, int32_t **dev) {
  static int32_t *h = nullptr, *d = nullptr;
  if (!h) {
    void *p = nullptr;
    if (hipHostMalloc(&p, 64, hipHostMallocCoherent | hipHostMallocMapped) != hipSuccess) return false;
    void *dp = nullptr;
    if (hipHostGetDevicePointer(&dp, p, 0) != hipSuccess) return false;
    h = (int32_t *)p;
    d = (int32_t *)dp;
    h[0] = h[1] = -1;
  }
  *host = h;
  *dev = d;
  return true;
}

// The Sinkhorn loop (setup, the initial potentials, the iterations under the batch-coupled stop
// rule or to *stop_at) -- the first half of nfdpf_ot_resample.
static int ot_loop(const float *x, const float *w, OtParams &P, const OtWs &ws, int poll, hipStream_t st) {
  const int B = P.B, max_iter = P.max_iter, splits = P.splits;
  std::unique_lock<std::mutex> lock;
  volatile int32_t *hf = nullptr;
  if (poll) {
    lock = std::unique_lock<std::mutex>(g_poll_mu);
    if (!poll_flags(&hf, &P.host)) return launch_status("nfdpf_ot_resample (poll flags)");
    P.seq = (g_poll_seq = (g_poll_seq + 1) & 0x7ffff);
  }
  const dim3 g(splits, B);
  ot_setup_kernel<<<g, kOtBlock, 0, st>>>(x, w, P, ws);
  ot_init_kernel<<<g, kOtBlock, 0, st>>>(P, ws);
  const bool w8 = ot_iter_waves(B * splits) == 2 * kWaves;
  auto iter = [&](int k) {
    if (w8)
      ot_iter_kernel<2 * kWaves><<<g, 128 * kWaves, 0, st>>>(P, ws, k);
    else
      ot_iter_kernel<kWaves><<<g, kOtBlock, 0, st>>>(P, ws, k);
  };
  if (!poll) {
    for (int k = 0; k < max_iter - 1; ++k) iter(k);
  } else {
    // Keep at most kAhead iterations queued past the one the device has started, and stop
    // enqueueing once an iteration has observed the stop (or the gate is off): the loop then
    // costs (iterations run) + <= kAhead early-exit launches instead of max_iter - 1.  A
    // device that reports nothing for 2 s (should not happen) gets the remaining launches.
    constexpr int kAhead = 2;
    bool blind = false;
    for (int k = 0; k < max_iter - 1; ++k) {
      if (!blind && hf[0] == P.seq) break;
      iter(k);
      if (blind) continue;
      const auto t0 = std::chrono::steady_clock::now();
      for (;;) {
        if (hf[0] == P.seq) break;
        const int32_t pr = hf[1];
        if (pr / 4096 == P.seq && k - pr % 4096 < kAhead) break;
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
          blind = true;
          break;
        }
        std::this_thread::yield();
      }
    }
  }
  P.host = nullptr;
  return NFDPF_OK;
}

// The tail: final potential, column normalisers, transport apply (at *stop_at when given).
static void ot_tail(const float *x, const OtParams &P, const OtWs &ws, int64_t row_base, float *x_out,
                    float *w_out, int64_t *idx_out, int32_t *iters_out, hipStream_t st) {
  const dim3 g(P.splits, P.B);
  if (P.hist) ot_restore_kernel<<<g, kOtBlock, 0, st>>>(P, ws);
  ot_final_kernel<<<g, kOtBlock, 0, st>>>(P, ws);
  ot_col_kernel<<<g, kOtBlock, 0, st>>>(P, ws, x);
  ot_apply_kernel<<<g, kOtBlock, 0, st>>>(P, ws, x, row_base, x_out, w_out, idx_out, iters_out);
}

#define NFDPF_OT_CHECK_ARGS(name)                                                          \
  NFDPF_REQUIRE(B >= 0 && N >= 1 && max_iter >= 1, name ": bad sizes");                   \
  NFDPF_REQUIRE(eps > 0.f && scaling > 0.f, name ": eps and scaling must be > 0");        \
  NFDPF_REQUIRE(((uintptr_t)workspace & 255) == 0, name ": workspace not 256-B aligned"); \
  NFDPF_REQUIRE(max_iter <= 4096, name ": max_iter <= 4096")

extern "C" int nfdpf_ot_resample_rs(const float *x, int64_t x_rs, const float *w, int64_t w_rs, int B, int N,
                                    float eps, float scaling, float threshold, int max_iter, int64_t row_base,
                                    float *x_out, float *w_out, int64_t *idx_out, int32_t *iters_out,
                                    void *workspace, const int32_t *gate, const int32_t *stop_at, int poll,
                                    void *stream) {
  NFDPF_REQUIRE(x && w && x_out && w_out && idx_out && workspace,
                "nfdpf_ot_resample: null pointer");
  NFDPF_OT_CHECK_ARGS("nfdpf_ot_resample");
  NFDPF_REQUIRE(x_rs >= 2 * (int64_t)N && w_rs >= N, "nfdpf_ot_resample: row strides below the row length");
  if (B == 0) return NFDPF_OK;
  hipStream_t st = as_stream(stream);
  OtWs ws = carve(workspace, B, N);
  OtParams P{B, N, ot_splits(N), max_iter, (double)eps, (double)scaling * (double)scaling,
             (double)threshold, gate, stop_at, nullptr, 0, nullptr};
  P.x_rs = x_rs;
  P.w_rs = w_rs;
  const int rc = ot_loop(x, w, P, ws, poll, st);
  if (rc != NFDPF_OK) return rc;
  ot_tail(x, P, ws, row_base, x_out, w_out, idx_out, iters_out, st);
  return launch_status("nfdpf_ot_resample");
}

extern "C" int nfdpf_ot_resample(const float *x, const float *w, int B, int N, float eps,
                                 float scaling, float threshold, int max_iter, int64_t row_base,
                                 float *x_out, float *w_out, int64_t *idx_out, int32_t *iters_out,
                                 void *workspace, const int32_t *gate, const int32_t *stop_at,
                                 int poll, void *stream) {
  return nfdpf_ot_resample_rs(x, 2 * (int64_t)N, w, N, B, N, eps, scaling, threshold, max_iter, row_base, x_out,
                              w_out, idx_out, iters_out, workspace, gate, stop_at, poll, stream);
}

extern "C" int64_t nfdpf_ot_history_bytes(int B, int N, int max_iter) {
  return (B <= 0 || N <= 0 || max_iter <= 0) ? 256 : align256((int64_t)max_iter * 2 * B * N * sizeof(double));
}

extern "C" int nfdpf_ot_sinkhorn_local(const float *x, const float *w, int B, int N, float eps, float scaling,
                                       float threshold, int max_iter, int32_t *iters_out, void *workspace,
                                       void *history, const int32_t *gate, int poll, void *stream) {
  NFDPF_REQUIRE(x && w && iters_out && workspace && history, "nfdpf_ot_sinkhorn_local: null pointer");
  NFDPF_OT_CHECK_ARGS("nfdpf_ot_sinkhorn_local");
  if (B == 0) return NFDPF_OK;
  hipStream_t st = as_stream(stream);
  OtWs ws = carve(workspace, B, N);
  OtParams P{B, N, ot_splits(N), max_iter, (double)eps, (double)scaling * (double)scaling,
             (double)threshold, gate, nullptr, nullptr, 0, (double *)history};
  P.x_rs = 2 * (int64_t)N;
  P.w_rs = N;
  const int rc = ot_loop(x, w, P, ws, poll, st);
  if (rc != NFDPF_OK) return rc;
  ot_iters_kernel<<<1, 1, 0, st>>>(P, ws, iters_out);
  return launch_status("nfdpf_ot_sinkhorn_local");
}

extern "C" int nfdpf_ot_sinkhorn_finish(const float *x, int B, int N, float eps, float scaling, float threshold,
                                        int max_iter, int64_t row_base, float *x_out, float *w_out,
                                        int64_t *idx_out, int32_t *iters_out, void *workspace, void *history,
                                        const int32_t *gate, const int32_t *stop_at, void *stream) {
  NFDPF_REQUIRE(x && x_out && w_out && idx_out && workspace && history && stop_at,
                "nfdpf_ot_sinkhorn_finish: null pointer");
  NFDPF_OT_CHECK_ARGS("nfdpf_ot_sinkhorn_finish");
  if (B == 0) return NFDPF_OK;
  hipStream_t st = as_stream(stream);
  OtWs ws = carve(workspace, B, N);
  OtParams P{B, N, ot_splits(N), max_iter, (double)eps, (double)scaling * (double)scaling,
             (double)threshold, gate, stop_at, nullptr, 0, (double *)history};
  P.x_rs = 2 * (int64_t)N;
  P.w_rs = N;
  ot_tail(x, P, ws, row_base, x_out, w_out, idx_out, iters_out, st);
  return launch_status("nfdpf_ot_sinkhorn_finish");
}

extern "C" int nfdpf_ot_transport_backward(const float *g_out, int B, int N, float eps, float *g_x,
                                           void *workspace, const int32_t *gate, void *stream) {
  NFDPF_REQUIRE(g_out && g_x && workspace, "nfdpf_ot_transport_backward: null pointer");
  NFDPF_REQUIRE(B >= 0 && N >= 1, "nfdpf_ot_transport_backward: bad sizes");
  NFDPF_REQUIRE(eps > 0.f, "nfdpf_ot_transport_backward: eps must be > 0");
  NFDPF_REQUIRE(((uintptr_t)workspace & 255) == 0, "nfdpf_ot_transport_backward: workspace not 256-B aligned");
  if (B == 0) return NFDPF_OK;
  hipStream_t st = as_stream(stream);
  const int splits = ot_splits(N);
  OtWs ws = carve(workspace, B, N);
  OtParams P{B, N, splits, 1, (double)eps, 1.0, 0.0, gate, nullptr, nullptr, 0, nullptr};
  const dim3 g(splits, B);
  ot_bwd_table_kernel<<<g, kOtBlock, 0, st>>>(P, ws, g_out);
  ot_bwd_apply_kernel<<<g, kOtBlock, 0, st>>>(P, ws, g_out, g_x);
  return launch_status("nfdpf_ot_transport_backward");
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
