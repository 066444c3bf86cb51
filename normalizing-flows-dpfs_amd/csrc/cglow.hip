// cglow.hip -- the conditional-GLOW measurement (model/models.py:280-303 over
// nf/cglow/CGlowModel.py:123-176 and nf/cglow/modules.py), BASELINE config 5.
//
// Per particle: x = particle_encoder(pos) reshaped (3,8,8); y = this row's frame encoding
// (3,8,8), squeezed to (12,4,4); one CondGlowStep (K = 1, L = 1):
//   cond-actnorm : (logs, bias) = tanh(MLP(convs(x)))          y = (y + bias) e^logs
//   cond-1x1conv : W (12x12)    = tanh(MLP(convs(x)))          y = W y,  + 16 log|det W|
//   cond-affine  : h = convs(x) (3->16->6->6 at 4x4); f([h, z1]) -> (shift, scale)
//                  z2 = (z2 + shift) sigmoid(scale + 2)
// then nll = -(logdet + Gaussian logp) / (192 log 2) and lik = -nll (raw; the row-max
// shift of :301-302 is applied by the caller -- the filter's EXTERNAL-measurement phase or
// measurement_model_cglow).
//
// Mapping (one workgroup = 4 waves = a tile of 16 particles, persistent over tiles):
//   * layers whose outputs are per particle and wide (encoder 32->192, the conditioning
//     MLPs, their 2x2-stride convs) run as f32 MFMA 16x16x4 GEMMs with the 16 particles as
//     M; v_mfma_f32_16x16x4_f32 is an exact k-ordered fmaf chain;
//   * layers over the 4x4 / 8x8 grids (the coupling's convolutions, actnorm, 1x1 conv,
//     log-det) run on VALU with lane = (particle, 4x4 position): 16 lanes per particle, the
//     same output channel in every lane, so weights are wave-uniform scalar loads; 3x3
//     neighbourhoods are exchanged through LDS;
//   * log|det W| of each particle's 12x12 matrix: Gaussian elimination with partial
//     pivoting across the particle's 16 lanes (row r in lane r), rows exchanged by shuffles.
#include <type_traits>

#include "cglow.hpp"

namespace nfdpf {
namespace cg {
#ifdef NFDPF_EXP_CGDUMP
__device__ float g_cgdump[256];
#endif

constexpr int kTileP = 16;    // particles per workgroup tile
constexpr int kThreads = 256;


// ---- workgroup LDS ----
// Stage-local buffers share storage (anonymous union): the encoder's hidden layers, the
// conditioning nets' activations and the y / coupling stage's grids are never live together
// (every hand-over is separated by a SYNC, the tile loop ends with one), which brings the
// workgroup from 80 KB to 50 KB of LDS: 3 workgroups per CU instead of 2.
struct Lds {
  float pxy[kTileP][2];
  float xs[kTileP][kE + 1];            // particle encoding, [c][8][8]
  float an[kTileP][2 * kC + 1];        // actnorm (logs | bias)
  float wm[kTileP][kC * kC + 4];       // 1x1 conv weight, row-major [out][in] (rows 16-B aligned)
  float ld[kTileP];                    // per-particle log-det of actnorm + 1x1 conv
#ifdef NFDPF_EXP_CGDUMP
  float ldw_dbg[kTileP];
#endif
  int row[kTileP];
  float escale[2 * kYH + kC];          // exp of the coupling net's log-scales (once per launch)
  float zrow[kC + 1];                  // zeros: the 3x3 convolutions' out-of-grid neighbour
  union {
    struct {  // particle encoder
      float h1[kTileP][kPeH1 + 1];
      float h2[kTileP][kPeH2 + 1];
    };
    struct {  // conditioning nets (actnorm A | 1x1 conv I)
      float cv1[kTileP][16][2 * kXH + 1];  // cond conv1 (A | I) at the 4x4 positions
      float cv2[kTileP][4][2 * kXH + 1];   // cond conv2 at 2x2
      float cv3[kTileP][2 * kXH + 1];
      float v0[kTileP][2 * kXS + 1];
      float v1[kTileP][2 * kXS + 1];
    };
    struct {  // y after actnorm + 1x1 conv, the coupling's convolutions
      float ex[kTileP][16][kC + 1];  // 4x4-grid exchange
      float yv[kTileP][16][kC + 1];  // y after actnorm + 1x1 conv, per position
    };
  };
};

typedef float f4 __attribute__((ext_vector_type(4)));

__shared__ Lds S;  // one instance per workgroup, shared by the phase functions below

#ifdef NFDPF_EXP_CGTRACE  // experiment: per-phase timestamps of one tile per workgroup
__device__ uint64_t g_cgtrace[1024][16];
#define CGTRACE(k)                                                                  \
  if (trace_it && threadIdx.x == 0 && blockIdx.x < 1024)                           \
    g_cgtrace[blockIdx.x][k] = __builtin_amdgcn_s_memrealtime();
#else
#define CGTRACE(k)
#endif

// One 16x16 output tile of C = A B over K (zero-padded to 4*KSTEPS): lane l feeds A[l&15][k]
// and B[k][l&15] for k = 4s + (l>>4), and gets C rows 4(l>>4)+i, column l&15.
template <int KSTEPS, class FA, class FB>
__device__ __forceinline__ f4 mfma_tile(const FA &fa, const FB &fb) {
  const int l = threadIdx.x & 63, r = l & 15, kk = l >> 4;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KSTEPS; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa(r, 4 * s + kk), fb(4 * s + kk, r), acc, 0, 0, 0);
  return acc;
}
// the same with this lane's B operands already in registers: b[s] = B[4 s + l / 16][l % 16]
template <int KSTEPS, class FA>
__device__ __forceinline__ f4 mfma_tile_b(const FA &fa, const float (&b)[KSTEPS]) {
  const int l = threadIdx.x & 63, r = l & 15, kk = l >> 4;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < KSTEPS; ++s) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(fa(r, 4 * s + kk), b[s], acc, 0, 0, 0);
  return acc;
}
template <class FE>
__device__ __forceinline__ void mfma_store(const f4 &acc, const FE &epi) {
  const int l = threadIdx.x & 63;
#pragma unroll
  for (int i = 0; i < 4; ++i) epi(4 * (l >> 4) + i, l & 15, acc[i]);
}

__device__ __forceinline__ float sigmoidf_(float v) { return 1.0f / (1.0f + expf(-v)); }

// tanh of the conditioning nets' outputs and of the coupling's shift / scale: libm tanhf.
// (-DNFDPF_CG_FAST_TANH: tanh_fast, common.hpp -- 2 % faster per launch, but the golden
// error grows from 1.8e-6 to 5.5e-6 against the reference's own 2.1e-6: not shipped.  Round 3:
// libm's two regimes evaluated branch-free and selected, ~2 ulp -- 2.03 ms either way, removed.)
__device__ __forceinline__ float cg_tanh(float x) {
#if defined(NFDPF_CG_FAST_TANH)
  return tanh_fast(x);
#else
  return tanhf(x);
#endif
}

// A lane-dependent weight load through a GLOBAL pointer (a generic one compiles to flat_load,
// which also counts on lgkmcnt: every LDS wait would then wait for it too), unconditional --
// the callers clamp the index and select afterwards (a guarded load became an exec-mask branch
// per element).
typedef const float __attribute__((address_space(1))) gfloat;
__device__ __forceinline__ float gld(const float *p, int i) { return ((gfloat *)p)[i]; }

// A pointer argument of a non-inlined function arrives in VGPRs; it is wave-uniform, so move
// it to SGPRs (readfirstlane) before making it a scalar-load weight pointer.
__device__ __forceinline__ const float *sgpr_ptr(const float *p) {
  const uint64_t v = (uint64_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (const float *)(((uint64_t)hi << 32) | lo);
}

// log|det W| of the 12x12 matrix held one row per lane (lanes g*16 + r, r < 12), partial
// pivoting by |value|; every lane of the group returns the same value.  The pivot search is a
// 16-lane (|v|, lane) max on DPP (ties to the lowest lane); the pivot row goes through LDS
// (the pivot lane writes it to prow_lds, the group reads it back: same wave, in order).
#ifdef NFDPF_CG_SHFL_LU
__device__ float logabsdet12(float (&a)[kC], int q, float *) {
  const int base = (threadIdx.x & 63) & ~15;  // first lane of this particle's group
  float ld = 0.f;
  bool done = q >= kC;                        // lanes 12..15 hold no row
#pragma unroll
  for (int k = 0; k < kC; ++k) {
    float v = done ? -1.f : fabsf(a[k]);
    int who = q;
#pragma unroll
    for (int o = 8; o > 0; o >>= 1) {
      const float v2 = __shfl_xor(v, o, 16);
      const int w2 = __shfl_xor(who, o, 16);
      if (v2 > v || (v2 == v && w2 < who)) {
        v = v2;
        who = w2;
      }
    }
    float prow[kC];
#pragma unroll
    for (int j = 0; j < kC; ++j) prow[j] = __shfl(a[j], base + who, 64);
    const float piv = prow[k];
    ld += logf(fabsf(piv));
    if (q == who) done = true;
    if (!done) {
      const float f = a[k] / piv;
#pragma unroll
      for (int j = 0; j < kC; ++j)
        if (j > k) a[j] = fmaf(-f, prow[j], a[j]);
    }
  }
  return ld;
}
#elif !defined(NFDPF_CG_EXACT_LU)
// The pivot search as ONE unsigned max per DPP step: the key of a lane is |a[k]|'s bit pattern
// (monotonic in the value for non-negative floats) with its low 4 mantissa bits replaced by
// 15 - lane, so the 16-lane max picks the largest |value| -- to 2^-19 relative; among values
// that equal to that precision, the lowest lane -- and names its lane.  Lanes whose row was a
// pivot already (and lanes 12..15) hold key 0 and never win: a live lane's key is >= 4.  The
// multiplier is a[k] times the pivot's reciprocal (v_rcp_f32, 1 ulp).  Round 2's search (an
// exact compare-and-select argmax, branchy after compilation: ~70 instructions per pivot) and
// IEEE division (11) stay behind -DNFDPF_CG_EXACT_LU.
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_max_u(uint32_t v) {
  return max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float logabsdet12(float (&a)[kC], int q, float *prow_lds) {
  float ld = 0.f;
  bool done = q >= kC;  // lanes 12..15 hold no row
  const uint32_t tag = 15u - (uint32_t)q;
#pragma unroll
  for (int k = 0; k < kC; ++k) {
    uint32_t key = done ? 0u : ((__float_as_uint(fabsf(a[k])) & ~0xFu) | tag);
    key = dpp_max_u<kDppXor1>(key);
    key = dpp_max_u<kDppXor2>(key);
    key = dpp_max_u<kDppHalfMirror>(key);
    key = dpp_max_u<kDppMirror>(key);
    const int who = 15 - (int)(key & 0xFu);
    if (q == who)
#pragma unroll
      for (int j = k; j < kC; ++j) prow_lds[j] = a[j];
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float prow[kC];
#pragma unroll
    for (int j = k; j < kC; ++j) prow[j] = prow_lds[j];
    const float piv = prow[k];
    ld += logf(fabsf(piv));
    if (q == who) done = true;
    if (!done) {
      const float f = a[k] * __builtin_amdgcn_rcpf(piv);
#pragma unroll
      for (int j = k + 1; j < kC; ++j) a[j] = fmaf(-f, prow[j], a[j]);
    }
    __builtin_amdgcn_wave_barrier();  // every lane has read the row before the next is written
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  return ld;
}
#else
template <int CTRL>
__device__ __forceinline__ void argmax_step(float &v, int &who) {
  const float v2 = dpp_f<CTRL>(v);
  const int w2 = __builtin_amdgcn_update_dpp(who, who, CTRL, 0xf, 0xf, false);
  if (v2 > v || (v2 == v && w2 < who)) {
    v = v2;
    who = w2;
  }
}
__device__ __forceinline__ float logabsdet12(float (&a)[kC], int q, float *prow_lds) {
  float ld = 0.f;
  bool done = q >= kC;  // lanes 12..15 hold no row
#pragma unroll
  for (int k = 0; k < kC; ++k) {
    float v = done ? -1.f : fabsf(a[k]);
    int who = q;
    argmax_step<kDppXor1>(v, who);
    argmax_step<kDppXor2>(v, who);
    argmax_step<kDppHalfMirror>(v, who);
    argmax_step<kDppMirror>(v, who);
    if (q == who)
#pragma unroll
      for (int j = k; j < kC; ++j) prow_lds[j] = a[j];
    __builtin_amdgcn_wave_barrier();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    float prow[kC];
#pragma unroll
    for (int j = k; j < kC; ++j) prow[j] = prow_lds[j];
    const float piv = prow[k];
    ld += logf(fabsf(piv));
    if (q == who) done = true;
    if (!done) {
      const float f = a[k] / piv;
#pragma unroll
      for (int j = k + 1; j < kC; ++j) a[j] = fmaf(-f, prow[j], a[j]);
    }
    __builtin_amdgcn_wave_barrier();  // every lane has read the row before the next is written
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  return ld;
}
#endif

}  // namespace cg

using namespace cg;

// phase_resize / phase_f as calls (default) or inlined (-DNFDPF_CG_PHASE_INLINE=__forceinline__:
// 156 B of scratch, not run)
#ifndef NFDPF_CG_PHASE_INLINE
#define NFDPF_CG_PHASE_INLINE __noinline__
#endif

// workgroup barrier that is also a scheduling fence
#define SYNC()                            \
  do {                                    \
    __builtin_amdgcn_sched_barrier(0);    \
    __syncthreads();                      \
    __builtin_amdgcn_sched_barrier(0);    \
  } while (0)
// From phase_y to the tile's end every LDS hand-off stays inside one particle's 16 lanes (lane
// = (particle tid / 16, position tid % 16): the 3x3 neighbourhoods, S.yv, S.ex, S.ld), i.e.
// inside one wave, whose LDS accesses execute in order: a compiler fence suffices, and the
// waves run those phases without waiting for each other.  (-DNFDPF_CG_BARRIERS: workgroup
// barriers there, as in r01.)
#ifdef NFDPF_CG_BARRIERS
#define WSYNC() SYNC()
#else
#define WSYNC()                                          \
  do {                                                   \
    __builtin_amdgcn_sched_barrier(0);                   \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   \
    __builtin_amdgcn_wave_barrier();                     \
    __builtin_amdgcn_sched_barrier(0);                   \
  } while (0)
#endif

// squeeze(y) at position q (y prefetched at the tile's start: yq = y_fetch(...)),
// cond-actnorm, cond-1x1 conv (-> S.yv), their log-dets (-> S.ld)
__device__ __forceinline__ void y_fetch(const float *__restrict__ enc, int64_t enc_rs, int row, int q,
                                        float (&y)[kC]) {
  const int qi = q >> 2, qj = q & 3;
  const float *er = enc + (int64_t)row * enc_rs;
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int f = 0; f < 4; ++f) y[c * 4 + f] = gld(er, c * 64 + (2 * qi + (f >> 1)) * 8 + 2 * qj + (f & 1));
}
__device__ __forceinline__ void phase_y(float (&y)[kC], int p, int q) {
  float sl = 0.f;
#pragma unroll
  for (int c = 0; c < kC; ++c) {
    const float ls = S.an[p][c];
    y[c] = (y[c] + S.an[p][kC + c]) * expf(ls);
    sl += ls;
  }
  const f4 *wrow = reinterpret_cast<const f4 *>(&S.wm[p][0]);
#pragma unroll
  for (int o = 0; o < kC; ++o) {
    float a = 0.f;
#pragma unroll
    for (int c4 = 0; c4 < kC / 4; ++c4) {
      const f4 w4 = wrow[o * (kC / 4) + c4];
#pragma unroll
      for (int e = 0; e < 4; ++e) a = fmaf(w4[e], y[4 * c4 + e], a);
    }
    S.yv[p][q][o] = a;
  }
  float wr[kC];
  const int qr = q < kC ? q : 0;
#pragma unroll
  for (int c4 = 0; c4 < kC / 4; ++c4) {
    const f4 w4 = wrow[qr * (kC / 4) + c4];
#pragma unroll
    for (int e = 0; e < 4; ++e) wr[4 * c4 + e] = q < kC ? w4[e] : 0.f;
  }
  // the pivot rows go through this particle's S.ex[p][0] (free until phase_resize writes it)
  const float ldw = logabsdet12(wr, q, &S.ex[p][0][0]);
  if (q == 0) S.ld[p] = 16.0f * sl + 16.0f * ldw;  // dimensions (4x4) x (sum logs, log|det W|)
#ifdef NFDPF_EXP_CGDUMP
  if (q == 0) S.ldw_dbg[p] = ldw;
#endif
}

// resize_x = conv3x3(3->16, pad 1) ReLU, conv2x2/2(16->6) ReLU, fused per 4x4 position (the
// 2x2 block of 8x8 conv1 outputs stays in registers) -> S.ex[p][q][0:6].  Weights are stored
// tap-major, output channel fastest (nfdpf.pack.cglow_tensors), so each input value feeds a
// contiguous run of output-channel pairs (v_pk_fma_f32 with an SGPR pair).
__device__ NFDPF_CG_PHASE_INLINE void phase_resize(const float *glow_, int p, int q) {
  const float *glow = sgpr_ptr(glow_);
  const int qi = q >> 2, qj = q & 3;
  // The 4x4 window (rows 2qi-1 .. 2qi+2, cols 2qj-1 .. 2qj+2, zero outside) is read from LDS per
  // tap, and the tap loop is OUTERMOST: each tap's 16 weights (one s_load_dwordx16) feed the
  // four 8x8 outputs of this position's 2x2 block -- 32 independent v_pk_fma per tap.  (r01: a
  // 48-value register window indexed by the partly unrolled tap loop lived in scratch, and the
  // weights were loaded once per block.)  Out-of-window reads stay inside the LDS struct and
  // are discarded by the select.
  const float *xrow = &S.xs[p][(2 * qi - 1) * 8 + 2 * qj - 1];
  const bool r0 = qi > 0, r3 = qi < 3, c0 = qj > 0, c3 = qj < 3;
  cf2 *F2 = (cf2 *)wptr(glow + kOffF);
  f2 hb[4][8];
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const f2 bias = F2[Aff::r0b / 2 + m];
#pragma unroll
    for (int ab = 0; ab < 4; ++ab) hb[ab][m] = bias;
  }
// tap loop unrolled by 9 (one (dr) row of taps: its weight loads issue ahead of the fmas):
// 2.33 -> 2.28 ms per C5 launch against unroll 3; unroll 1 2.43 ms; 27 spills to scratch
#ifndef NFDPF_CG_RESIZE_UNROLL
#define NFDPF_CG_RESIZE_UNROLL 9
#endif
#pragma unroll NFDPF_CG_RESIZE_UNROLL
  for (int t = 0; t < 27; ++t) {  // taps (dr, ds, c) of the 3x3x3 window
    F2 = (cf2 *)wptr(glow + kOffF);
    const int dr = t / 9, ds = (t / 3) % 3, c = t % 3;
    float v[4];
#pragma unroll
    for (int ab = 0; ab < 4; ++ab) {
      const int r = (ab >> 1) + dr, s2 = (ab & 1) + ds;
      const bool in = (r > 0 || r0) && (r < 3 || r3) && (s2 > 0 || c0) && (s2 < 3 || c3);
      const float x = xrow[c * 64 + r * 8 + s2];
      v[ab] = in ? x : 0.f;
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const f2 wgt = F2[(Aff::r0w + t * 16) / 2 + m];
#pragma unroll
      for (int ab = 0; ab < 4; ++ab) hb[ab][m] = pfma(wgt, splat(v[ab]), hb[ab][m]);
    }
  }
  f2 h62[kCh / 2];
  F2 = (cf2 *)wptr(glow + kOffF);
#pragma unroll
  for (int m = 0; m < kCh / 2; ++m) h62[m] = F2[Aff::r2b / 2 + m];
#pragma unroll
  for (int ab = 0; ab < 4; ++ab) {
    F2 = (cf2 *)wptr(glow + kOffF);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const f2 hv = relu2(hb[ab][m]);
#pragma unroll
      for (int n = 0; n < kCh / 2; ++n) {
        h62[n] = pfma(F2[(Aff::r2w + (ab * 16 + 2 * m) * kCh) / 2 + n], splat(hv.x), h62[n]);
        h62[n] = pfma(F2[(Aff::r2w + (ab * 16 + 2 * m + 1) * kCh) / 2 + n], splat(hv.y), h62[n]);
      }
    }
  }
#pragma unroll
  for (int m = 0; m < kCh / 2; ++m) {
    S.ex[p][q][2 * m] = relu(h62[m].x);
    S.ex[p][q][2 * m + 1] = relu(h62[m].y);
  }
}

// 3x3 'same' conv on the 4x4 grid from the neighbours' channel vectors in S.ex; weights
// [tap][c][o] with o fastest; acc holds NP output pairs.  Per tap the neighbour's CIN channels
// are read together and the tap's weights in chunks of 4 channels (one scalar-load batch per
// chunk), so a tap is 3-12 x NP independent v_pk_fma instead of NP per loop trip.  Same
// (tap, channel) order of the fma chain as the per-(tap, channel) loop it replaces.
template <int CIN, int NP>
__device__ __forceinline__ void conv3x3(const float *glow, int wofs, int p, int q, f2 (&acc)[NP]) {
  const int qi = q >> 2, qj = q & 3;
#ifdef NFDPF_CG_CONV_TC
#pragma unroll 2
  for (int tc = 0; tc < 9 * CIN; ++tc) {  // (tap, input channel), tap-major
    const int t9 = tc / CIN, c = tc - CIN * (tc / CIN);
    const int dr = t9 / 3, ds = t9 - 3 * (t9 / 3);
    cf2 *F2 = (cf2 *)wptr(glow + kOffF);  // a few weights live at a time
    const int rr = qi + dr - 1, ss = qj + ds - 1;
    const bool in = rr >= 0 && rr < 4 && ss >= 0 && ss < 4;
    const float v = in ? S.ex[p][rr * 4 + ss][c] : 0.f;
#pragma unroll
    for (int n = 0; n < NP; ++n) acc[n] = pfma(F2[(wofs + tc * (2 * NP)) / 2 + n], splat(v), acc[n]);
  }
#else
  constexpr int kChunk = CIN % 4 == 0 ? 4 : (CIN % 3 == 0 ? 3 : 2);
// (unrolled by 3: 2.71 vs 2.33 ms per C5 launch, 32 B of scratch; by 9: 724 B of scratch)
#ifndef NFDPF_CG_CONV_UNROLL
#define NFDPF_CG_CONV_UNROLL 1
#endif
#pragma unroll NFDPF_CG_CONV_UNROLL
  for (int t9 = 0; t9 < 9; ++t9) {
    const int dr = t9 / 3, ds = t9 - 3 * (t9 / 3);
    const int rr = qi + dr - 1, ss = qj + ds - 1;
    const bool in = rr >= 0 && rr < 4 && ss >= 0 && ss < 4;
    // an out-of-grid neighbour reads the zero row (one address select per tap instead of a
    // select per channel; written as `in ? src[c] : 0` the compiler had also guarded every load
    // with an exec-mask branch)
    const float *src = in ? S.ex[p][rr * 4 + ss] : S.zrow;
    float v[CIN];
#pragma unroll
    for (int c = 0; c < CIN; ++c) v[c] = src[c];
#pragma unroll
    for (int c0 = 0; c0 < CIN; c0 += kChunk) {
      cf2 *F2 = (cf2 *)wptr(glow + kOffF);
#pragma unroll
      for (int c = c0; c < c0 + kChunk; ++c)
#pragma unroll
        for (int n = 0; n < NP; ++n)
          acc[n] = pfma(F2[(wofs + (t9 * CIN + c) * (2 * NP)) / 2 + n], splat(v[c]), acc[n]);
    }
  }
#endif
}

// resize conv3, the coupling net f, the affine update of z2 and the Gaussian log-prob;
// returns this particle's sum (over its 16 positions) of log scale + logp
__device__ NFDPF_CG_PHASE_INLINE float phase_f(const float *glow_, int p, int q, float *zrow) {
  const float *glow = sgpr_ptr(glow_);
  cfloat *F = wptr(glow + kOffF);
  float fin[kC];  // cat(resize_x(x), z1)
  {
    f2 a3[kCh / 2];
#pragma unroll
    for (int m = 0; m < kCh / 2; ++m) a3[m] = ((cf2 *)F)[Aff::r4b / 2 + m];
    conv3x3<kCh>(glow, Aff::r4w, p, q, a3);
#pragma unroll
    for (int m = 0; m < kCh / 2; ++m) {
      fin[2 * m] = relu(a3[m].x);
      fin[2 * m + 1] = relu(a3[m].y);
    }
  }
#pragma unroll
  for (int c = 0; c < kCh; ++c) fin[kCh + c] = S.yv[p][q][c];
  WSYNC();
#pragma unroll
  for (int c = 0; c < kC; ++c) S.ex[p][q][c] = fin[c];
  WSYNC();
  // f: Conv2dNormy(12->8, 3x3) ReLU, Conv2dNormy(8->8, 1x1) ReLU, Conv2dZerosy(8->12) Tanh
  float g8b[kYH];
  {
    f2 a0[kYH / 2];
#pragma unroll
    for (int m = 0; m < kYH / 2; ++m) a0[m] = splat(0.f);
    conv3x3<kC>(glow, Aff::f0w, p, q, a0);
    F = wptr(glow + kOffF);
    float g8[kYH];
#pragma unroll
    for (int m = 0; m < kYH / 2; ++m) {
      g8[2 * m] = relu((a0[m].x + F[Aff::f0ab + 2 * m]) * S.escale[2 * m]);
      g8[2 * m + 1] = relu((a0[m].y + F[Aff::f0ab + 2 * m + 1]) * S.escale[2 * m + 1]);
    }
    f2 a1[kYH / 2];
#pragma unroll
    for (int m = 0; m < kYH / 2; ++m) a1[m] = splat(0.f);
#pragma unroll
    for (int c = 0; c < kYH; ++c)
#pragma unroll
      for (int m = 0; m < kYH / 2; ++m) a1[m] = pfma(((cf2 *)F)[(Aff::f2w + c * kYH) / 2 + m], splat(g8[c]), a1[m]);
#pragma unroll
    for (int m = 0; m < kYH / 2; ++m) {
      g8b[2 * m] = relu((a1[m].x + F[Aff::f2ab + 2 * m]) * S.escale[kYH + 2 * m]);
      g8b[2 * m + 1] = relu((a1[m].y + F[Aff::f2ab + 2 * m + 1]) * S.escale[kYH + 2 * m + 1]);
    }
  }
  WSYNC();
#pragma unroll
  for (int c = 0; c < kYH; ++c) S.ex[p][q][c] = g8b[c];
  WSYNC();
  f2 a4[kC / 2];  // pair m = (shift_m, scale_m): channels 2m, 2m+1 (split_feature "cross")
#pragma unroll
  for (int m = 0; m < kC / 2; ++m) a4[m] = splat(0.f);
  conv3x3<kYH>(glow, Aff::f4w, p, q, a4);
  F = wptr(glow + kOffF);
  float lsum = 0.f, lp = 0.f;
#pragma unroll
  for (int c = 0; c < kCh; ++c) {
    const float hs = cg_tanh((a4[c].x + F[Aff::f4b + 2 * c] + F[Aff::f4nb + 2 * c]) * S.escale[2 * kYH + 2 * c]);
    const float hc =
        cg_tanh((a4[c].y + F[Aff::f4b + 2 * c + 1] + F[Aff::f4nb + 2 * c + 1]) * S.escale[2 * kYH + 2 * c + 1]);
    const float sc = sigmoidf_(hc + 2.0f);
    const float z1 = S.yv[p][q][c];
    const float z2 = (S.yv[p][q][kCh + c] + hs) * sc;
    if (zrow) {  // z = cat(z1, z2) as (12, 4, 4) (CondAffineCoupling.forward, modules.py:288-303)
      zrow[c * 16 + q] = z1;
      zrow[(kCh + c) * 16 + q] = z2;
    }
    lsum += logf(sc);
    lp += z2 * z2;
    lp += z1 * z1;
  }
  // Gaussian logp over the 12 channels at this position, plus this position's log scale,
  // summed over the particle's 16 positions (one DPP row)
  float part = lsum - 0.5f * (lp + (float)kC * 1.8378770664093453f);
  part += dpp_f<kDppXor1>(part);
  part += dpp_f<kDppXor2>(part);
  part += dpp_f<kDppHalfMirror>(part);
  part += dpp_f<kDppMirror>(part);
  return part;
}



// x: particle (b, i) at x + b * x_rs + 2 i;  enc: row b at enc + b * enc_rs (192 floats);
// lik: (b, i) at lik + b * lik_rs + i.  Raw likelihood (no row-max shift).
// 3 workgroups per CU: 50 KB of LDS each (the stage union of Lds) and <= 168 VGPRs (162) for
// 3 waves per SIMD.  (r01f: min-blocks 2 with 80 KB of LDS spilled 182 SGPRs and ran 5.24 ms
// at C5; min-blocks 1, same occupancy, 5.09 ms; the union + min-blocks 3 4.72 ms -- A/B, 3 runs.)
#ifndef NFDPF_CG_WGS
#define NFDPF_CG_WGS 3  // resident workgroups per CU (LDS 50 KB, <= 168 VGPRs); 2: 2.52 vs 2.12 ms
#endif
__global__ __launch_bounds__(kThreads, NFDPF_CG_WGS) void cglow_kernel(const float *__restrict__ pe,
                                                            const float *__restrict__ glow,
                                                            const float *__restrict__ enc,
                                                            int64_t enc_rs, const float *__restrict__ x,
                                                            int64_t x_rs, int B, int N,
                                                            float *__restrict__ lik, int64_t lik_rs,
                                                            const float *__restrict__ xin,
                                                            float *__restrict__ zout, float out_sign) {
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const int64_t total = (int64_t)B * N;
  const int64_t ntiles = (total + kTileP - 1) / kTileP;
  auto PW = [](const float *w, int o, int i, int K) { return gld(w, ((o >> 1) * K + i) * 2 + (o & 1)); };
  // the coupling net's per-channel scales exp(logs) (Conv2dNormy, nf/cglow/modules.py:214) and exp(3 logs)
  // (Conv2dZerosy, :233), once per launch (ordered before use by the tile's first SYNC)
  if (tid <= kC) S.zrow[tid] = 0.f;  // read-only from here (ordered by the tile's first SYNC)
  if (tid < 2 * kYH + kC) {
    const float *F = glow + kOffF;
    S.escale[tid] = tid < kYH ? expf(F[Aff::f0al + tid])
                    : tid < 2 * kYH ? expf(F[Aff::f2al + tid - kYH])
                                    : expf(F[Aff::f4l + tid - 2 * kYH] * 3.0f);
  }

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
#ifdef NFDPF_EXP_CGTRACE
    const bool trace_it = tile == blockIdx.x + 2 * (int64_t)gridDim.x;
#endif
    CGTRACE(0)
    // this lane's squeezed y (phase_y), fetched now so its latency hides behind the encoder
    // and the conditioning nets (lane = (particle w * 4 + l / 16, position l % 16))
    float yq[kC];
    {
      const int64_t gy = tile * kTileP + (tid >> 4);
      const int rowy = gy < total ? (int)(gy / N) : 0;
      y_fetch(enc, enc_rs, xin ? (int)(gy < total ? gy : 0) : rowy, tid & 15, yq);
    }
    // weight pointers re-derived per tile behind an asm barrier, so the compiler re-reads
    // weights from the caches instead of hoisting every one of them out of the tile loop
    const float *gw = glow, *pe_ = pe;
    asm volatile("" : "+s"(gw), "+s"(pe_));
    const float *gA = gw + kOffA, *gI = gw + kOffI;
    // encoder weights (nfdpf.pack.encoder_tensors)
    const float *pw1 = pe_, *pb1 = pe_ + kPeB1, *pw2 = pe_ + kPeW2, *pb2 = pe_ + kPeB2, *pw3 = pe_ + kPeW3,
                *pb3 = pe_ + kPeW3 + kE * kPeH2;
    // W2 / W3 in col_pairs order (nfdpf.pack.encoder_tensors): {W[2m, k], W[2m+1, k]} at [k][m]
    auto W3 = [&](int n, int k) { return gld(pw3, (k * (kE / 2) + (n >> 1)) * 2 + (n & 1)); };
    const int64_t g0 = tile * kTileP;
    if (xin) {
      // CondGlowModel.forward(x, y): the condition x (3 x 8 x 8) is given per sample and y is
      // per sample too (N = 1: row = sample), no particle encoder
      for (int k = tid; k < kTileP * kE; k += kThreads) {
        const int p = k / kE, c = k - p * kE;
        const int64_t gi = g0 + p;
        S.xs[p][c] = gi < total ? xin[gi * kE + c] : 0.f;
      }
      if (tid < kTileP) S.row[tid] = (int)(g0 + tid < total ? g0 + tid : 0);
      SYNC();
    } else {
      // ---- particles of the tile
      if (tid < kTileP) {
        const int64_t gi = g0 + tid;
        float a = 0.f, c = 0.f;
        int rb = 0;
        if (gi < total) {
          rb = (int)(gi / N);
          const int i = (int)(gi - (int64_t)rb * N);
          a = gld(x, rb * x_rs + 2 * i);
          c = gld(x, rb * x_rs + 2 * i + 1);
        }
        S.pxy[tid][0] = a;
        S.pxy[tid][1] = c;
        S.row[tid] = rb;
      }
      SYNC();
      // ---- particle encoder (model/models.py:141-150): 2 -> 16 -> 32 (ReLU), then 32 -> 192
      {
        const int p = tid >> 4, j = tid & 15;
        const float h = fmaf(PW(pw1, j, 1, 2), S.pxy[p][1], fmaf(PW(pw1, j, 0, 2), S.pxy[p][0], gld(pb1, j)));
        S.h1[p][j] = relu(h);
      }
      SYNC();
      {
        const int p = tid >> 4, j = tid & 15;
  #pragma unroll
        for (int hh = 0; hh < 2; ++hh) {
          const int o = j + 16 * hh;
          float a = gld(pb2, o);
  #pragma unroll
          for (int k = 0; k < kPeH1; ++k) a = fmaf(gld(pw2, (k * (kPeH2 / 2) + (o >> 1)) * 2 + (o & 1)), S.h1[p][k], a);
          S.h2[p][o] = relu(a);
        }
      }
      SYNC();
#pragma unroll
      for (int j = 0; j < 3; ++j) {  // N tiles w, w + 4, w + 8 of kE / 16 = 12
        const int n0 = (w + 4 * j) * 16;
        const f4 acc = mfma_tile<kPeH2 / 4>([&](int r, int k) { return S.h2[r][k]; },
                                            [&](int k, int c) { return W3(n0 + c, k); });
        mfma_store(acc, [&](int r, int c, float v) { S.xs[r][n0 + c] = v + gld(pb3, n0 + c); });
      }
      SYNC();
    }
    CGTRACE(1)
    // ---- conditioning nets, conv1 (3 -> 8, 2x2 stride 2, 8x8 -> 4x4) for actnorm (A) and
    //      1x1-conv (I) nets: VALU, lane = (particle, 4x4 position)
    // This wave's B operands (weights) and epilogue biases of the conditioning nets' MFMA
    // layers are lane-dependent vector loads; in place each layer paid a global round trip for
    // them (and another for its bias) between two barriers.  Each is issued one phase ahead.
    // (lane l: column c = l % 16, k = 4 s + l / 16 -- mfma_tile's operand order)
    const int fc = l & 15, fk = l >> 4;
    float bC2[2][8], bbC2[2];              // cond conv2 of net 0 (A) and 1 (I), row tile w
#pragma unroll
    for (int net = 0; net < 2; ++net) {
      const float *G = net ? gI : gA;
#pragma unroll
      for (int s2 = 0; s2 < 8; ++s2) bC2[net][s2] = gld(G, CondA::c2w + (fc & 7) * 32 + 4 * s2 + fk);
#pragma unroll
      for (int s2 = 0; s2 < 8; ++s2) bC2[net][s2] = fc < kXH ? bC2[net][s2] : 0.f;
      bbC2[net] = gld(G, CondA::c2b + (fc & 7));
    }
    const int p = w * 4 + (l >> 4), q = l & 15, qi = q >> 2, qj = q & 3;
    {
      float in[12];
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b2 = 0; b2 < 2; ++b2) in[c * 4 + a * 2 + b2] = S.xs[p][c * 64 + (2 * qi + a) * 8 + 2 * qj + b2];
#pragma unroll
      for (int net = 0; net < 2; ++net) {
        cfloat *G = wptr(net ? gI : gA);
#pragma unroll
        for (int o = 0; o < kXH; ++o) {
          float acc = G[CondA::c0b + o];
#pragma unroll
          for (int k = 0; k < 12; ++k) acc = fmaf(G[CondA::c0w + k * kXH + o], in[k], acc);
          S.cv1[p][q][net * kXH + o] = relu(acc);
        }
      }
    }
    SYNC();
    CGTRACE(2)
    float bC3[8], bbC3, bL0[2], bbL0, bL2[4], bbL2;  // cond conv3, x_Linear of net w (w < 2)
    {
      const float *G = w ? gI : gA;
#pragma unroll
      for (int s2 = 0; s2 < 8; ++s2) bC3[s2] = gld(G, CondA::c4w + (fc & 7) * 32 + 4 * s2 + fk);
#pragma unroll
      for (int s2 = 0; s2 < 8; ++s2) bC3[s2] = fc < kXH ? bC3[s2] : 0.f;
      bbC3 = gld(G, CondA::c4b + (fc & 7));
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) bL0[s2] = gld(G, CondA::l0w + fc * kXH + 4 * s2 + fk);
      bbL0 = gld(G, CondA::l0b + fc);
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) bL2[s2] = gld(G, CondA::l2w + fc * kXS + 4 * s2 + fk);
      bbL2 = gld(G, CondA::l2b + fc);
    }
    // conv2 (8 -> 8, 2x2 stride 2, 4x4 -> 2x2): GEMM, rows (particle, 2x2 pos), k (ci, a, b)
#pragma unroll
    for (int net = 0; net < 2; ++net) {  // jobs w (net 0) and w + 4 (net 1), row tile mt = w
      const int mt = w;  // 4 row tiles of 16 = 64 rows
      const f4 acc = mfma_tile_b<8>(
          [&](int r, int k) {
            const int row = mt * 16 + r, pp = row >> 2, pos = row & 3;
            const int ci = k >> 2, a = (k >> 1) & 1, b2 = k & 1;
            return S.cv1[pp][(2 * (pos >> 1) + a) * 4 + 2 * (pos & 1) + b2][net * kXH + ci];
          },
          bC2[net]);
      mfma_store(acc, [&](int r, int c, float v) {
        if (c < kXH) {
          const int row = mt * 16 + r;
          S.cv2[row >> 2][row & 3][net * kXH + c] = relu(v + bbC2[net]);
        }
      });
    }
    SYNC();
    CGTRACE(3)
    float bL4[3][4], bbL4[3];  // last layer: jobs w, w + 4, w + 8 (< 11)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int job = w + 4 * j;
      const bool isI = job >= 2;
      const int n = (isI ? job - 2 : job) * 16 + fc, nout = isI ? kC * kC : 2 * kC;
      const float *G = isI ? gI : gA;
      const int lw = isI ? CondI::l4w : CondA::l4w, lb = isI ? CondI::l4b : CondA::l4b;
      const bool ok = job < 11 && n < nout;
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) bL4[j][s2] = gld(G, lw + (ok ? n : 0) * kXS + 4 * s2 + fk);
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) bL4[j][s2] = ok ? bL4[j][s2] : 0.f;
      bbL4[j] = gld(G, lb + (ok ? n : 0));
      bbL4[j] = ok ? bbL4[j] : 0.f;
    }
    // conv3 (8 -> 8, 2x2 stride 2, 2x2 -> 1x1): rows = particles, k = (ci, a, b)
    if (w < 2) {
      const int net = w;
      const f4 acc = mfma_tile_b<8>([&](int r, int k) { return S.cv2[r][k & 3][net * kXH + (k >> 2)]; }, bC3);
      mfma_store(acc, [&](int r, int c, float v) {
        if (c < kXH) S.cv3[r][net * kXH + c] = relu(v + bbC3);
      });
    }
    SYNC();
    CGTRACE(4)
    // x_Linear: 8 -> 16 -> 16 (ReLU)
    if (w < 2) {
      const int net = w;
      const f4 acc = mfma_tile_b<2>([&](int r, int k) { return S.cv3[r][net * kXH + k]; }, bL0);
      mfma_store(acc, [&](int r, int c, float v) { S.v0[r][net * kXS + c] = relu(v + bbL0); });
    }
    SYNC();
    if (w < 2) {
      const int net = w;
      const f4 acc = mfma_tile_b<4>([&](int r, int k) { return S.v0[r][net * kXS + k]; }, bL2);
      mfma_store(acc, [&](int r, int c, float v) { S.v1[r][net * kXS + c] = relu(v + bbL2); });
    }
    SYNC();
    CGTRACE(5)
    // last layer + tanh: actnorm (24 = 2 tiles) and 1x1 conv (144 = 9 tiles)
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int job = w + 4 * j;
      if (job >= 11) break;
      const bool isI = job >= 2;
      const int n0 = (isI ? job - 2 : job) * 16, nout = isI ? kC * kC : 2 * kC;
      const f4 acc = mfma_tile_b<4>([&](int r, int k) { return S.v1[r][(isI ? kXS : 0) + k]; }, bL4[j]);
      mfma_store(acc, [&](int r, int c, float v) {
        const int n = n0 + c;
        if (n < nout) {
          const float t = cg_tanh(v + bbL4[j]);
          if (isI)
            S.wm[r][n] = t;
          else
            S.an[r][n] = t;
        }
      });
    }
    SYNC();
    CGTRACE(6)

    // ---- squeeze(y) at position q, cond-actnorm, cond-1x1 conv, log|det W|
    phase_y(yq, p, q);
    WSYNC();
    CGTRACE(7)
    phase_resize(gw, p, q);
    WSYNC();
    CGTRACE(8)
    const int64_t gi = g0 + p;
    const float part = phase_f(gw, p, q, zout && gi < total ? zout + gi * kE : nullptr);
#ifdef NFDPF_EXP_CGDUMP
    // experiment only: one particle's 1x1-conv W, its log|det W| (the LU's), actnorm outputs
    if (gi == (int64_t)NFDPF_CG_TARGET && q < 16) {
      for (int k = q; k < kC * kC; k += 16) g_cgdump[k] = S.wm[p][k];
      for (int k = q; k < 2 * kC; k += 16) g_cgdump[160 + k] = S.an[p][k];
      if (q == 0) {
        g_cgdump[200] = S.ldw_dbg[p];
        g_cgdump[201] = S.ld[p];
        g_cgdump[202] = part;
      }
    }
#endif
    if (q == 0 && gi < total) {
      // logdet0 = -log(256) * 192, plus actnorm / 1x1-conv log-dets, plus this particle's sum
      const float obj = (-5.545177444479562f * (float)kE + S.ld[p]) + part;
      const int rb = S.row[p];
      const int i = (int)(gi - (int64_t)rb * N);
      lik[rb * lik_rs + i] = out_sign * (obj / (0.6931471805599453f * (float)kE));
    }
    SYNC();
    CGTRACE(9)
  }
}

}  // namespace nfdpf

using namespace nfdpf;

#ifdef NFDPF_EXP_CGDUMP
extern "C" NFDPF_API int nfdpf_exp_cgdump_read(void *host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_cgdump), sizeof(g_cgdump)) == hipSuccess ? 0 : 1;
}
#endif
#ifdef NFDPF_EXP_CGTRACE
extern "C" NFDPF_API int nfdpf_exp_cgtrace_read(void *host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_cgtrace), sizeof(g_cgtrace)) == hipSuccess ? 0 : 1;
}
#endif

extern "C" int64_t nfdpf_cglow_params_size(int K) { return K == 1 ? (int64_t)kStep : -1; }

extern "C" int nfdpf_cglow_measurement(const float *pe_params, const float *glow_params, int K,
                                       const float *enc, int64_t enc_rs, const float *x, int64_t x_rs,
                                       int B, int N, float *lik, int64_t lik_rs, void *stream) {
  NFDPF_REQUIRE(pe_params && glow_params && enc && x && lik, "nfdpf_cglow_measurement: null pointer");
  NFDPF_REQUIRE(K == 1, "nfdpf_cglow_measurement: built for flow_depth K = 1 (got %d)", K);
  NFDPF_REQUIRE(B >= 0 && N >= 1, "nfdpf_cglow_measurement: bad sizes");
  if (B == 0) return NFDPF_OK;
  const int64_t tiles = ((int64_t)B * N + kTileP - 1) / kTileP;
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) cus = v;
  }
  // a persistent grid of exactly the resident workgroups (3 per CU: LDS 50 KB, 162 VGPRs):
  // more would start a second, late round of workgroups and leave the tail unbalanced
  const int grid = (int)std::min<int64_t>(tiles, (int64_t)cus * NFDPF_CG_WGS);
  cglow_kernel<<<grid, kThreads, 0, as_stream(stream)>>>(pe_params, glow_params, enc, enc_rs, x, x_rs, B, N,
                                                        lik, lik_rs, nullptr, nullptr, 1.0f);
  return launch_status("nfdpf_cglow_measurement");
}

static int cglow_grid(int64_t tiles) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) {
    int v = 0;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) cus = v;
  }
  return (int)std::min<int64_t>(tiles, (int64_t)cus * NFDPF_CG_WGS);
}

extern "C" int nfdpf_cglow_flow(const float *glow_params, int K, const float *x, const float *y, int64_t M,
                                float *z, float *nll, void *stream) {
  NFDPF_REQUIRE(glow_params && x && y && nll, "nfdpf_cglow_flow: null pointer");
  NFDPF_REQUIRE(K == 1, "nfdpf_cglow_flow: built for flow_depth K = 1 (got %d)", K);
  NFDPF_REQUIRE(M >= 0 && M <= (int64_t)INT32_MAX, "nfdpf_cglow_flow: bad size");
  if (M == 0) return NFDPF_OK;
  // B = M rows of N = 1 (y row m is sample m), the condition x given, out_sign -1: nll
  cglow_kernel<<<cglow_grid((M + kTileP - 1) / kTileP), kThreads, 0, as_stream(stream)>>>(
      glow_params, glow_params, y, kE, nullptr, 0, (int)M, 1, nll, 1, x, z, -1.0f);
  return launch_status("nfdpf_cglow_flow");
}
