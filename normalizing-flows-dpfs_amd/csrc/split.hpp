// split.hpp -- a coupling flow on two waves per particle group: the t-net of every particle
// runs on one wave, its s-net on a partner wave, and the two exchange their single output
// through LDS once per coupling half.
//
// Why: at the C2 workload (64 rows x 1000 particles) one particle per lane is ONE wave per
// SIMD across the chip, where a VALU instruction issues at half rate and nothing hides the
// scalar weight loads or the exp/rcp latencies of the tanh chains.  Splitting the nets
// halves each wave's chain and doubles the waves in flight without adding arithmetic (the
// only duplicated work is the coupling update itself, a handful of VALU ops).
//
// Weight layout (the "split suffix" of a dynamic / proposal flow blob, nfdpf.pack
// split_flow_tensors, include/nfdpf.h): for each flow, coupling half n (t1/s1, t2/s2) and
// net r (t, s), kSplitNet floats
//   [ W1[:, 0] as hidden pairs (4) | W2 rows as hidden pairs [4][8] | b2 pairs (4) |
//     W3 pairs (4) | {b3, 0} ]
// so one v_pk_fma_f32 advances hidden units 2m and 2m+1 of ONE net (HALF = 1, H = 8: the
// 2-D particle flows of the filter).  The folded first-layer biases are re-ordered the same
// way in LDS: [flow][half][net][j] (split_cb_index).
#pragma once

#include "stages.hpp"

namespace nfdpf {

constexpr int kSplitNet = 90;              // floats per net (45 pairs)
constexpr int kSplitFlow = 4 * kSplitNet;  // t1, s1, t2, s2
static_assert(kH == 8, "split nets are laid out for hidden width 8");

// offset (floats) of the split suffix behind the pair layout of an n_flows stack of
// RealNVP_cond(2, O) flows
__host__ __device__ constexpr int split_suffix_offset(int n_flows, int O) {
  return n_flows * 2 * net_size<1, kH>(O) * 2;
}

// position of float `tid` of a pair-order fold table ([flow][half][j][t|s], fold_ref) in the
// split order [flow][half][net][j]
__device__ __forceinline__ int split_cb_index(int tid) {
  const int f = tid / (4 * kH), r = tid % (4 * kH);
  const int n = r / (2 * kH), j = (r >> 1) % kH, w = r & 1;
  return ((f * 2 + n) * 2 + w) * kH + j;
}

__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// Pairwise hand-off between the t-wave and the s-wave of one particle group, through LDS,
// with no workgroup barrier: each side writes its value, publishes a per-wave counter and
// spins (s_sleep) until the partner's counter reaches the same exchange.  Values are double
// buffered by exchange parity, so a fast side never overwrites one its partner has not read
// (it would first need the partner's NEXT counter, published only after that read).  Both
// waves of a pair cover the same particles, so they execute the same exchanges.
typedef __attribute__((address_space(3))) float lds_float;
typedef volatile __attribute__((address_space(3))) int lds_vint;

struct PairX {
  lds_float *buf;  // pair_swap: [2 parities][2 nets][kTile] x {value, tag} (2 floats each)
  lds_vint *mine;  // this wave's counter
  lds_vint *theirs;
  int role, slot, k;
};

// Wave roles of a split workgroup: waves 2g and 2g + 1 are the t-net and the s-net of
// particle group g (adjacent waves sit on different SIMDs, so a pair computes side by side
// rather than taking turns on one SIMD); waves from `flow_waves` on take role 2.
struct SplitLane {
  int role, slot;
};
__device__ __forceinline__ SplitLane split_lane(int flow_waves) {
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;
  if (w < flow_waves) return SplitLane{w & 1, (w >> 1) * 64 + l};
  return SplitLane{2, (w - flow_waves) * 64 + l};
}

// the PairX of a flow wave (role 0 / 1): its partner is the adjacent wave
__device__ __forceinline__ PairX pair_of(float *buf, int *flags, int role, int slot) {
  const int w = (threadIdx.x >> 6) & 15;
  return PairX{(lds_float *)buf, (lds_vint *)(flags + w), (lds_vint *)(flags + (w ^ 1)), role, slot, 0};
}

constexpr int kSpinCap = 1 << 22;  // ~0.1 s of s_sleep: a safety exit, never reached in a correct run

// Count of hand-offs that gave up at kSpinCap (the partner never arrived: a broken pairing).
// The kernel then proceeds on stale data, so the host must treat any count as a failed
// launch: nfdpf_split_fault (filter_tiled.hip) reads and clears it, FilterEngine.run raises.
static __device__ int g_split_fault = 0;

// publish this wave's exchange counter (after its values have landed) and wait for the
// partner's; both waves of a pair execute the same sequence of exchanges
__device__ __forceinline__ void pair_wait(PairX &x) {
  const int k = ++x.k;
#ifndef NFDPF_EXP_NOWAIT
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the values land before the counter
  *x.mine = k;
  int it = 0;
  for (; __builtin_amdgcn_readfirstlane(*x.theirs) < k && it < kSpinCap; ++it) __builtin_amdgcn_s_sleep(1);
  if (it == kSpinCap && (threadIdx.x & 63) == 0) atomicAdd(&g_split_fault, 1);
#endif
  asm volatile("" ::: "memory");
}

// One value each way, tagged: every lane writes {value, exchange number} with ONE 64-bit LDS
// store and polls its partner lane's {value, tag} until the tag is this exchange's -- one LDS
// round trip per side instead of value store, counter store, counter poll and value load.
// Buffers alternate by exchange parity (a side cannot be two exchanges ahead: it needs the
// partner's value of the previous one first).  buf = [2 parities][2 roles][tile_len] x 2 words.
typedef volatile __attribute__((address_space(3))) unsigned long long lds_vu64;
// LDS is not cleared between workgroups: a previous workgroup's tags would satisfy a poll, so
// every kernel zeroes its pair_swap buffer (4 tile_len words) before its first barrier
__device__ __forceinline__ void pair_clear(float *buf, int tile_len) {
  for (int j = threadIdx.x; j < 4 * tile_len; j += blockDim.x) ((lds_vu64 *)buf)[j] = 0ull;
}
__device__ __forceinline__ float pair_swap(PairX &x, float v, int tile_len) {
  const int k = ++x.k;
  lds_vu64 *tb = (lds_vu64 *)x.buf + (k & 1) * 2 * tile_len;
  tb[x.role * tile_len + x.slot] = ((unsigned long long)(unsigned)k << 32) | (unsigned)__float_as_uint(v);
  unsigned long long r;
  int it = 0;
  for (;;) {
    r = tb[(1 - x.role) * tile_len + x.slot];
    if (__all((int)(r >> 32) == k) || ++it >= kSpinCap) break;
    __builtin_amdgcn_s_sleep(1);
  }
  if (it >= kSpinCap && (threadIdx.x & 63) == 0) atomicAdd(&g_split_fault, 1);
  asm volatile("" ::: "memory");
  return __uint_as_float((unsigned)r);
}

// Cosine pieces (|e|^2, <e, v> over this role's output pairs) with the particle encoder's
// second layer split over the wave pair as well (model/models.py:130-139): role r computes
// hidden pairs [8 r, 8 r + 8) of Linear(16, 32), the pair exchanges them through `hbuf`
// ([2 roles][16 floats][tile_len], used once per launch), and each role then computes its 8
// output pairs from all 32 hidden units -- the fma sequence of pe_hidden / pe_out per output.
template <int E>
__device__ __forceinline__ void encode_dot_pair(cfloat *pe, float x0, float x1, const float *v, double &ss,
                                                double &dot, PairX &x, float *hbuf, int tile_len) {
  constexpr int M = kPeH2 / 2, MH = M / 2;  // 16 hidden pairs, 8 per role
  cf2 *w1 = (cf2 *)pe, *b1 = (cf2 *)(pe + kPeB1);
  f2 h1[kPeH1 / 2];
#pragma unroll
  for (int m = 0; m < kPeH1 / 2; ++m)
    h1[m] = relu2(pfma(w1[2 * m + 1], splat(x1), pfma(w1[2 * m], splat(x0), b1[m])));
  const int m0 = x.role * MH;
  cf2 *w2 = (cf2 *)(pe + kPeW2) + m0, *b2 = (cf2 *)(pe + kPeB2) + m0;
  f2 mine[MH];
#pragma unroll
  for (int m = 0; m < MH; ++m) mine[m] = b2[m];
#pragma unroll
  for (int k = 0; k < kPeH1; ++k) {
    const float hk = pick(h1, k);
#pragma unroll
    for (int m = 0; m < MH; ++m) mine[m] = pfma(w2[k * M + m], splat(hk), mine[m]);
  }
#pragma unroll
  for (int m = 0; m < MH; ++m) mine[m] = relu2(mine[m]);
  // exchange the halves (the pair_swap protocol: values, then the counter, then spin)
  lds_float *hb = (lds_float *)hbuf;
#pragma unroll
  for (int m = 0; m < MH; ++m) {
    hb[(x.role * 2 * MH + 2 * m) * tile_len + x.slot] = mine[m].x;
    hb[(x.role * 2 * MH + 2 * m + 1) * tile_len + x.slot] = mine[m].y;
  }
  pair_wait(x);
  f2 h2[M];
  const int other = 1 - x.role;
#pragma unroll
  for (int m = 0; m < MH; ++m) {
    const f2 o{hb[(other * 2 * MH + 2 * m) * tile_len + x.slot], hb[(other * 2 * MH + 2 * m + 1) * tile_len + x.slot]};
    h2[x.role ? m : MH + m] = o;
    h2[x.role ? MH + m : m] = mine[m];
  }
  f2 a[E / 4];
  pe_out<E, E / 4>(pe, h2, x.role * (E / 4), a);
  ss = 0.0;  // fp64 partials: see encode_dot (flows.hpp)
  dot = 0.0;
  const int o0 = x.role * (E / 4);
#pragma unroll
  for (int m = 0; m < E / 4; ++m) {
    const double ax = a[m].x, ay = a[m].y;
    ss = fma(ax, ax, ss);
    dot = fma(ax, (double)v[2 * (o0 + m)], dot);
    ss = fma(ay, ay, ss);
    dot = fma(ay, (double)v[2 * (o0 + m) + 1], dot);
  }
}

// ---- the cosine encoder's dense layers on f32 MFMA (v_mfma_f32_16x16x4_f32) ----------------
typedef float f4v __attribute__((ext_vector_type(4)));

// The cosine measurement's encoder on MFMA with the pair split by PARTICLES instead of outputs:
// wave r of the pair takes particle blocks {2r, 2r + 1} (particles [32 r, 32 r + 32) of the
// group) through all three layers, so the pair never hands off (no layer-3 operand exchange,
// no partial-sum exchange).  Layer 1 as encode_dot_pair_mfma; layers 2 / 3 per block as two
// 16-column output tiles (bias-initialised exact k-ordered MFMA chains); the 32 outputs of a
// particle come back through Hw to lane l = particle - 32 r, which accumulates |e|^2 and <e, v>
// in fp64 in output order (particle_encode + encode_dot's arithmetic).  Lanes >= 32 return 0.
struct EncFrag2 {
  float w10[4], w11[4], b1[4];  // layer 1 for k = 4 s + (lane >> 4)
  float b2[2][4], b3[2][8];     // B fragments of output tiles n = 0, 1 (columns 16 n + (lane & 15))
  float bias2[2], bias3[2];
};
__device__ __forceinline__ EncFrag2 enc_frag2_load(const float *pe) {
  EncFrag2 f;
  const int l = threadIdx.x & 63, kk = l >> 4;
#pragma unroll
  for (int st = 0; st < 4; ++st) {
    const int k = 4 * st + kk;
    f.w10[st] = pe[4 * (k >> 1) + (k & 1)];
    f.w11[st] = pe[4 * (k >> 1) + 2 + (k & 1)];
    f.b1[st] = pe[kPeB1 + k];
  }
#pragma unroll
  for (int n = 0; n < 2; ++n) {
    const int c = 16 * n + (l & 15);
#pragma unroll
    for (int st = 0; st < 4; ++st) f.b2[n][st] = pe[kPeW2 + kPeH2 * (4 * st + kk) + c];
#pragma unroll
    for (int st = 0; st < 8; ++st) f.b3[n][st] = pe[kPeW3 + kE * (4 * st + kk) + c];
    f.bias2[n] = pe[kPeB2 + c];
    f.bias3[n] = pe[kPeW3 + kE * kPeH2 + c];
  }
  return f;
}
constexpr int kHPitch = 36;  // [32 particles][32 units] LDS rows (bank spread of the A reads)

// q0 / q1: the group's proposals (64 each); Hw: [32][kHPitch] this wave's own (layer-2 outputs,
// then layer-3 outputs).  Every lane takes part (MFMA operands).
template <int E>
__device__ __forceinline__ void encode_dot_mfma_half(const EncFrag2 &f, int role, const float *q0, const float *q1,
                                                     const float *v, double &ss, double &dot, float *Hw) {
  static_assert(E == kE && kPeH1 == 16 && kPeH2 == 32, "MFMA encoder: 2 -> 16 -> 32 -> 32");
  const int l = threadIdx.x & 63, r16 = l & 15, kk = l >> 4;
  lds_float *hw = (lds_float *)Hw;
  f4v acc[2][2];
#pragma unroll
  for (int bb = 0; bb < 2; ++bb) {  // layer 1 in A order, layer 2
    const int p = 32 * role + 16 * bb + r16;
    const float x0 = q0[p], x1 = q1[p];
    float h[4];
#pragma unroll
    for (int st = 0; st < 4; ++st) h[st] = relu(fmaf(f.w11[st], x1, fmaf(f.w10[st], x0, f.b1[st])));
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      acc[bb][n] = f4v{f.bias2[n], f.bias2[n], f.bias2[n], f.bias2[n]};
#pragma unroll
      for (int st = 0; st < 4; ++st) acc[bb][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(h[st], f.b2[n][st], acc[bb][n], 0, 0, 0);
    }
  }
#pragma unroll
  for (int bb = 0; bb < 2; ++bb)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) hw[(16 * bb + 4 * kk + i) * kHPitch + 16 * n + r16] = relu(acc[bb][n][i]);
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  QTRACE(8)
#pragma unroll
  for (int bb = 0; bb < 2; ++bb) {  // layer 3
    float a[8];
#pragma unroll
    for (int st = 0; st < 8; ++st) a[st] = hw[(16 * bb + r16) * kHPitch + 4 * st + kk];
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      acc[bb][n] = f4v{f.bias3[n], f.bias3[n], f.bias3[n], f.bias3[n]};
#pragma unroll
      for (int st = 0; st < 8; ++st) acc[bb][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[st], f.b3[n][st], acc[bb][n], 0, 0, 0);
    }
  }
  __builtin_amdgcn_wave_barrier();  // every lane's layer-3 A reads are done before Hw is reused
#pragma unroll
  for (int bb = 0; bb < 2; ++bb)
#pragma unroll
    for (int n = 0; n < 2; ++n)
#pragma unroll
      for (int i = 0; i < 4; ++i) hw[(16 * bb + 4 * kk + i) * kHPitch + 16 * n + r16] = acc[bb][n][i];
  __builtin_amdgcn_wave_barrier();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  QTRACE(9)
  // lane l < 32: |e|^2 and <e, v> of particle 32 r + l, in output order.  (Splitting the two
  // sums over the lane halves in interleaved chains measured 3.8 us SLOWER per launch --
  // profiles/r02_experiments.md, QUAD8.)
  ss = 0.0;
  dot = 0.0;
  if (l < 32) {
#pragma unroll
    for (int c = 0; c < 32; ++c) {
      const double a = hw[l * kHPitch + c];
      ss = fma(a, a, ss);
      dot = fma(a, (double)v[c], dot);
    }
  }
}

// One exchange of two doubles between the waves of a pair through a buffer used once per
// launch ([2 roles][4 floats][tile_len]; single use, so no parity is needed -- cf. pair_swap).
__device__ __forceinline__ void pair_swap_once2(PairX &x, double a, double b, float *dbuf, int tile_len,
                                                double &ao, double &bo) {
  lds_float *db = (lds_float *)dbuf;
  const long long ia = __double_as_longlong(a), ib = __double_as_longlong(b);
  db[(x.role * 4 + 0) * tile_len + x.slot] = __int_as_float((int)ia);
  db[(x.role * 4 + 1) * tile_len + x.slot] = __int_as_float((int)(ia >> 32));
  db[(x.role * 4 + 2) * tile_len + x.slot] = __int_as_float((int)ib);
  db[(x.role * 4 + 3) * tile_len + x.slot] = __int_as_float((int)(ib >> 32));
  pair_wait(x);
  const int o = 1 - x.role;
  auto get = [&](int j) { return (unsigned int)__float_as_int(db[(o * 4 + j) * tile_len + x.slot]); };
  ao = __longlong_as_double((long long)(((unsigned long long)get(1) << 32) | get(0)));
  bo = __longlong_as_double((long long)(((unsigned long long)get(3) << 32) | get(2)));
}

// One net (t or s) of a coupling half on input u; cb = this net's 4 folded bias pairs.
__device__ __forceinline__ float net_split(cf2 *w, float u, const f2 *cb) {
  constexpr int P = kH / 2;
  f2 h[P];
#pragma unroll
  for (int m = 0; m < P; ++m) h[m] = tanh2(pfma(w[m], splat(u), cb[m]));
  cf2 *w2 = w + P;
  f2 g[P];
#pragma unroll
  for (int m = 0; m < P; ++m) {
    f2 a = w2[P * kH + m];
#pragma unroll
    for (int k = 0; k < kH; ++k) a = pfma(w2[m * kH + k], splat((k & 1) ? h[k >> 1].y : h[k >> 1].x), a);
    g[m] = tanh2(a);
  }
  cf2 *w3 = w2 + P * kH + P;
  f2 a = w3[0] * g[0];
#pragma unroll
  for (int m = 1; m < P; ++m) a = pfma(w3[m], g[m], a);
  return (a.x + a.y) + w3[P].x;
}

// RealNVP_cond flow, forward (nf/flows.py:215-226) / inverse (:228-239), split over a wave
// pair.  fw = the flow's split block (kSplitFlow floats, wave-uniform), cbs = its folded
// biases in split order (16 pairs).  Both waves end with identical lo, up and log-det.
// NFDPF_EXP_SAMEW (experiment builds only, scripts/archive/exp_build.sh; wrong results): every net of
// a stack reads the first net's weights -- the scalar-cache footprint of the coupling nets
// shrinks from 16 nets to 2, which prices their weight misses.
#ifdef NFDPF_EXP_SAMEW
#define EXP_NET(k) 0
#else
#define EXP_NET(k) (k)
#endif

__device__ __forceinline__ float coupling_forward_split(const float *fw, float &lo, float &up, const f2 *cbs,
                                                        PairX &x, int tile_len) {
  const int r = x.role;
  float v = net_split(wptr2(fw + EXP_NET(r) * kSplitNet), lo, cbs + r * 4);
  float o = pair_swap(x, v, tile_len);
  float t = r ? o : v, s = r ? v : o;
  up = t + up * expf(s);
  const float l1 = s;
  v = net_split(wptr2(fw + EXP_NET(2 + r) * kSplitNet), up, cbs + (2 + r) * 4);
  o = pair_swap(x, v, tile_len);
  t = r ? o : v;
  s = r ? v : o;
  lo = t + lo * expf(s);
  return l1 + s;
}

__device__ __forceinline__ float coupling_inverse_split(const float *fw, float &lo, float &up, const f2 *cbs,
                                                        PairX &x, int tile_len) {
  const int r = x.role;
  float v = net_split(wptr2(fw + EXP_NET(2 + r) * kSplitNet), up, cbs + (2 + r) * 4);
  float o = pair_swap(x, v, tile_len);
  float t = r ? o : v, s = r ? v : o;
  lo = (lo - t) * expf(-s);
  const float l2 = -s;
  v = net_split(wptr2(fw + EXP_NET(r) * kSplitNet), lo, cbs + r * 4);
  o = pair_swap(x, v, tile_len);
  t = r ? o : v;
  s = r ? v : o;
  up = (up - t) * expf(-s);
  return -s + l2;
}

// ---- the filter stages on a wave pair (stages.hpp restated for the split nets) ----

// nf_dyn inverse (model/models.py:305-332) of x_phys; role 0 writes scr x_dyn and hjac.
__device__ __forceinline__ void stage_dyn_inverse_split(const nfdpf_filter_desc &d, const RowSlot &S, int i,
                                                        float x0, float x1, const f2 *cbs, PairX &x, int tile_len,
                                                        float &xd0, float &xd1) {
  const float *base = d.dyn_params + split_suffix_offset(d.n_flows, kOctxDyn);
  float lo = x0, up = x1, ld = 0.f;
  for (int f = d.n_flows - 1; f >= 0; --f)
    ld += coupling_inverse_split(base + EXP_NET(f) * kSplitFlow, lo, up, cbs + f * 16, x, tile_len);
  if (x.role == 0) {
    S.scr[4 * i] = lo;
    S.scr[4 * i + 1] = up;
    if (S.hjac) S.hjac[i] = -ld;
  }
  xd0 = lo;
  xd1 = up;
}

// NF proposal inverse (model/models.py:334-356): returns jac_prop = -log_det.
__device__ __forceinline__ float stage_propose_inverse_split(const nfdpf_filter_desc &d, const PropIn &in,
                                                             const f2 *cbs, PairX &x, int tile_len, float &q0x,
                                                             float &q1x) {
  const float *base = d.cond_params + split_suffix_offset(d.n_flows, d.E + 4);
  float lo = in.xd0, up = in.xd1, ld = 0.f;
  for (int f = d.n_flows - 1; f >= 0; --f)
    ld += coupling_inverse_split(base + EXP_NET(f) * kSplitFlow, lo, up, cbs + f * 16, x, tile_len);
  q0x = lo;
  q1x = up;
  return -ld;
}

// nf_dyn forward of the proposal + densities (model/models.py:358-377) with --NF-dyn and
// --NF-cond; role 0 writes hx = proposal, scr propose/prior and hprior.
__device__ __forceinline__ void stage_prior_split(const nfdpf_filter_desc &d, const RowSlot &S, int i,
                                                  const PropIn &in, const f2 *cbs, float q0x, float q1x,
                                                  float jac_prop, PairX &x, int tile_len, float &propose,
                                                  float &prior) {
  const float K = d.dens_const;
  const float two_var = 2.0f * (d.pos_noise * d.pos_noise);
  const float de = density(in.e0, in.e1, K, two_var);
  const float r0 = in.p0 - in.e0, r1 = in.p1 - in.e1;
  const float *base = d.dyn_params + split_suffix_offset(d.n_flows, kOctxDyn);
  float lo = q0x, up = q1x, ld2 = 0.f;
  for (int f = 0; f < d.n_flows; ++f)
    ld2 += coupling_forward_split(base + EXP_NET(f) * kSplitFlow, lo, up, cbs + f * 16, x, tile_len);
  prior = density(lo - r0, up - r1, K, two_var) - (-ld2);
  propose = (de + in.jac) + jac_prop;
  if (x.role == 0) {
    S.hx[2 * i] = q0x;
    S.hx[2 * i + 1] = q1x;
    S.scr[4 * i + 2] = propose;
    S.scr[4 * i + 3] = prior;
    if (S.hprior) S.hprior[i] = prior;
  }
}

}  // namespace nfdpf
