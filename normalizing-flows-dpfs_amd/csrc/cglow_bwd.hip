// cglow_bwd.hip -- backward of the conditional-GLOW measurement (training):
// the autograd gradient of model/models.py:280-303 over nf/cglow/CGlowModel.py:123-176 and
// nf/cglow/modules.py (CondActNorm :76-132, Cond1x1Conv :136-211 with the slogdet of :165,
// CondAffineCoupling :258-303, Conv2dResize / Zeros / Normy / Zerosy :38-253, LinearZeros /
// Norm, GaussianDiag :377-403) and of the particle encoder (model/models.py:141-150), for the
// configuration cglow.hip is built for (K = 1, L = 1, 3x8x8 x and y, learn_top off).
//
// One workgroup = 4 waves = a tile of 16 particles (persistent over tiles), lane = (particle
// tid / 16, 4x4 position tid % 16) as in the forward.  Per tile:
//   1. forward recompute (encoder, both conditioning nets, actnorm, 1x1 conv, the resize and f
//      convolutions), activations in LDS; W^-1 of every particle's 12x12 matrix by Gauss-Jordan
//      with partial pivoting on the particle's 16 lanes (d log|det W| / dW = W^-T);
//   2. the backward chain per lane: Gaussian log-prob and log-scale -> affine coupling -> f
//      (3x3, 1x1, 3x3) -> resize_x (3x3, 2x2/2, 3x3) -> 1x1 conv / actnorm -> the two
//      conditioning nets -> the encodings (and the particle encoder).  Transposed 3x3
//      convolutions read the neighbours' output gradients through LDS.
//   3. parameter gradients: every parameter of the blob has ONE owner thread (blob index
//      mod 256 within its layer), which contracts the tile's (gradient x input) terms from LDS
//      in a fixed order into a register accumulator.  The workgroup's accumulators go to its
//      row of the workspace at the end, and cglow_param_reduce_kernel sums the rows in a fixed
//      order: deterministic, no atomics.
// The resize_x first layer (16 channels on the 8x8 grid: 1 024 values per particle) is staged
// four particles (one wave) at a time.
#include "cglow.hpp"

namespace nfdpf {
namespace cgb {

using namespace cg;

constexpr int kTP = 16;  // particles per tile
constexpr int kThreads = 256;
constexpr int kPeE = pe_size(kE);  // particle encoder 2 -> 16 -> 32 -> 192

// ---- parameter layers of the two blobs (glow, then the particle encoder at kStep) ----
// mf: the layer's gradient is a GEMM over the tile's (particle, position) terms, accumulated on
// f32 MFMA (v_mfma_f32_16x16x4f32, an exact k-ordered fmaf chain) in registers that persist
// across tiles; the others have owner threads (contract below).
struct LayerDef {
  int off, n;
  bool mf;
};
#define COND_LAYERS(O, C)                                                                          \
  {O + C::c0w, C::c0b - C::c0w, true}, {O + C::c0b, C::c2w - C::c0b}, {O + C::c2w, C::c2b - C::c2w, true}, \
      {O + C::c2b, C::c4w - C::c2b}, {O + C::c4w, C::c4b - C::c4w}, {O + C::c4b, C::l0w - C::c4b}, \
      {O + C::l0w, C::l0b - C::l0w}, {O + C::l0b, C::l2w - C::l0b}, {O + C::l2w, C::l2b - C::l2w}, \
      {O + C::l2b, C::l4w - C::l2b}, {O + C::l4w, C::l4b - C::l4w, true}, {O + C::l4b, C::size - C::l4b}
constexpr LayerDef kLayers[] = {
    COND_LAYERS(kOffA, CondA),
    COND_LAYERS(kOffI, CondI),
    {kOffF + Aff::r0w, Aff::r0b - Aff::r0w, true},
    {kOffF + Aff::r0b, Aff::r2w - Aff::r0b},
    {kOffF + Aff::r2w, Aff::r2b - Aff::r2w, true},
    {kOffF + Aff::r2b, Aff::r4w - Aff::r2b},
    {kOffF + Aff::r4w, Aff::r4b - Aff::r4w, true},
    {kOffF + Aff::r4b, Aff::f0w - Aff::r4b},
    {kOffF + Aff::f0w, Aff::f0ab - Aff::f0w, true},
    {kOffF + Aff::f0ab, kYH},
    {kOffF + Aff::f0al, kYH},
    {kOffF + Aff::f2w, kYH * kYH, true},
    {kOffF + Aff::f2ab, kYH},
    {kOffF + Aff::f2al, kYH},
    {kOffF + Aff::f4w, Aff::f4b - Aff::f4w, true},
    {kOffF + Aff::f4b, kC},
    {kOffF + Aff::f4l, kC},
    {kOffF + Aff::f4nb, kC},
    {kStep + 0, kPeB1},
    {kStep + kPeB1, kPeW2 - kPeB1},
    {kStep + kPeW2, kPeB2 - kPeW2},
    {kStep + kPeB2, kPeW3 - kPeB2},
    {kStep + kPeW3, kE * kPeH2, true},
    {kStep + kPeW3 + kE * kPeH2, kE},
};
#undef COND_LAYERS
constexpr int kNumLayers = sizeof(kLayers) / sizeof(kLayers[0]);
constexpr int kTotParams = kStep + kPeE;  // one workspace row

constexpr int slots_of(int n) { return (n + kThreads - 1) / kThreads; }
constexpr int layer_slots(int i) { return kLayers[i].mf ? 0 : slots_of(kLayers[i].n); }
constexpr int slot_base(int off) {
  int s = 0;
  for (int i = 0; i < kNumLayers; ++i) {
    if (kLayers[i].off == off) return kLayers[i].mf ? -1 : s;
    s += layer_slots(i);
  }
  return -1;
}
constexpr int layer_n(int off) {
  for (int i = 0; i < kNumLayers; ++i)
    if (kLayers[i].off == off) return kLayers[i].n;
  return -1;
}
constexpr int count_slots() {
  int s = 0;
  for (int i = 0; i < kNumLayers; ++i) s += layer_slots(i);
  return s;
}
constexpr bool layers_tile() {  // the layers cover both blobs exactly, in order
  int o = 0;
  for (int i = 0; i < kNumLayers; ++i) {
    if (kLayers[i].off != o || kLayers[i].n <= 0) return false;
    o += kLayers[i].n;
  }
  return o == kTotParams;
}
static_assert(layers_tile(), "cglow_bwd: layer table does not tile the parameter blobs");
constexpr int kSlots = count_slots();

typedef float Acc[kSlots];

// the owner threads of layer OFF add f(j) (this tile's sum of parameter j's terms, j local to
// the layer) to their register accumulators
template <int OFF, class F>
__device__ __forceinline__ void contract(Acc &acc, const F &f) {
  constexpr int base = slot_base(OFF), n = layer_n(OFF);
  static_assert(base >= 0 && n > 0, "unknown layer");
#pragma unroll
  for (int i = 0; i < slots_of(n); ++i) {
    const int j = (int)threadIdx.x + kThreads * i;
    if (n % kThreads == 0 || j < n) acc[base + i] += f(j);
  }
}

// the accumulators of layers L.. to the workgroup's row (compile-time slots: registers)
template <int L>
__device__ __forceinline__ void store_acc(const Acc &acc, float *row) {
  if constexpr (L < kNumLayers) {
    constexpr int off = kLayers[L].off, n = kLayers[L].n, base = slot_base(off);
#pragma unroll
    for (int i = 0; i < layer_slots(L); ++i) {
      const int j = (int)threadIdx.x + kThreads * i;
      if (n % kThreads == 0 || j < n) row[off + j] = acc[base + i];
    }
    store_acc<L + 1>(acc, row);
  }
}

typedef float f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
// C (16 x 16 tile, this lane: rows 4 (l / 16) + i, column l % 16) into the workgroup's row:
// row[idx(m, n)] for m < M, n = n0 + l % 16 < NC
template <class IDX>
__device__ __forceinline__ void store_tile(const f4 &c, float *row, int M, int n0, int NC, const IDX &idx) {
  const int l = threadIdx.x & 63, n = n0 + (l & 15);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int m = 4 * (l >> 4) + i;
    if (m < M && n < NC) row[idx(m, n)] = c[i];
  }
}

// ---- workgroup LDS (dynamic: ~146 KB) ----
struct BLds {
  float X[kTP][kE];        // the condition x (3,8,8): c * 64 + r * 8 + s
  float gX[kTP][kE];       // dL/dx
  float pxy[kTP][2];
  float h1[kTP][kPeH1];    // particle encoder hidden layers (ReLU outputs)
  float h2[kTP][kPeH2];
  float c1[kTP][16][2 * kXH];  // conditioning nets A | I: conv1 (4x4), conv2 (2x2), conv3, linears
  float c2[kTP][4][2 * kXH];
  float c3[kTP][2 * kXH];
  float l0[kTP][2 * kXS];
  float l1[kTP][2 * kXS];
  float an[kTP][2 * kC];   // tanh outputs: logs | bias
  float wm[kTP][kC * kC];  // W [o][c]
  float wi[kTP][kC * kC];  // W^-1 [r][c]
  float gw[kTP][kC * kC];  // dL/dW, then dL/d(pre-tanh)
  float gan[kTP][2 * kC];
  float prow[kTP][2 * kC];  // Gauss-Jordan pivot row
  float sm[kTP][48];        // per-particle sums of the small (per-channel) parameters
  float ya[kTP][16][kC];    // y after actnorm
  float r2[kTP][16][kCh];   // resize_x conv2 output (ReLU)
  float fin[kTP][16][kC];   // cat(resize_x(x), z1)
  union {
    struct {
      float g1[kTP][16][kYH];  // f conv0 / conv1 outputs (ReLU)
      float g2[kTP][16][kYH];
    };
    float R1[4][16][4][16];          // resize_x conv1 values / gradients of one wave's particles
    float G1c[kTP][16][2 * kXH];     // conditioning conv1 output gradients
  };
  float D[kTP][16][kC];  // output gradients of the layer being differentiated (exchange)
  float esc[2 * kYH + kC];                     // exp(f0 logs), exp(f2 logs), exp(3 f4 logs)
  float w4A[2 * kC * kXS], w4I[kC * kC * kXS];  // the nets' last layers [n][k] (lane-indexed reads)
  float b4[2 * kC + kC * kC];                   // ... their biases (A then I)
  float wc2[2][kXH * kXH * 4], wc4[2][kXH * kXH * 4];  // conv2 / conv3 of nets A, I [o][ci][a][b]
};
static_assert(sizeof(BLds) <= 160 * 1024, "cglow_bwd: LDS above 160 KB");

#ifdef NFDPF_EXP_CBTRACE  // experiment: per-phase timestamps of one tile per workgroup
__device__ uint64_t g_cbtrace[256][24];
#define CBT(k)                                                                        \
  do {                                                                                \
    if (cbt_on && threadIdx.x == 0) g_cbtrace[blockIdx.x & 255][k] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
#else
#define CBT(k) \
  do {         \
  } while (0)
#endif

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_max_u(uint32_t v) {
  return max(v, (uint32_t)__builtin_amdgcn_update_dpp((int)v, (int)v, CTRL, 0xf, 0xf, false));
}
// sum over the particle's 16 lanes (one DPP row), in every lane
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<kDppXor1>(v);
  v += dpp_f<kDppXor2>(v);
  v += dpp_f<kDppHalfMirror>(v);
  v += dpp_f<kDppMirror>(v);
  return v;
}
#define WFENCE()                                       \
  do {                                                 \
    __builtin_amdgcn_sched_barrier(0);                 \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); \
    __builtin_amdgcn_wave_barrier();                   \
    __builtin_amdgcn_sched_barrier(0);                 \
  } while (0)

__device__ __forceinline__ float sigm(float v) { return 1.0f / (1.0f + expf(-v)); }
__device__ __forceinline__ bool in4(int r, int s) { return r >= 0 && r < 4 && s >= 0 && s < 4; }

// PART: particles (b, i) at x + b * x_rs + 2 i through the particle encoder, y = row b's frame
// encoding (enc + b * enc_rs), upstream g_lik (b, i) at g_lik + b * glik_rs + i (lik = -nll, raw).
// !PART (CondGlowModel.forward): x = xin [M, 192], y [M, 192] per sample, upstream g_nll [M] and
// optionally g_z [M, 192].  Outputs: g_y [M, 192] per sample / particle, g_x (PART: [M, 2]
// particles; else [M, 192]), and this workgroup's parameter-gradient row of `partial`.
template <bool PART>
__global__ __launch_bounds__(kThreads, 1) void cglow_bwd_kernel(
    const float *__restrict__ pe_, const float *__restrict__ glow, const float *__restrict__ enc, int64_t enc_rs,
    const float *__restrict__ x, int64_t x_rs, int B, int N, const float *__restrict__ g_up, int64_t gup_rs,
    const float *__restrict__ g_z, float *__restrict__ g_y, float *__restrict__ g_x, float *__restrict__ partial) {
  extern __shared__ __attribute__((aligned(16))) char lds_raw[];
  BLds &S = *reinterpret_cast<BLds *>(lds_raw);
  const int tid = threadIdx.x, p = tid >> 4, q = tid & 15, qi = q >> 2, qj = q & 3;
  const int w = tid >> 6;
  const int64_t M = (int64_t)B * N;
  const int64_t ntiles = (M + kTP - 1) / kTP;
  Acc acc;
#pragma unroll
  for (int s = 0; s < kSlots; ++s) acc[s] = 0.f;
  // this wave's MFMA jobs (column tiles of the mf layers), persistent across tiles
  const int lr = tid & 15, lk = (tid >> 4) & 3;  // MFMA lane: row / column l % 16, k offset l / 16
  f4 cF4a = {}, cF4b = {}, cF0a = {}, cF0b = {}, cR4 = {}, cR2 = {}, cR0 = {}, cF2 = {}, cC0 = {}, cC2 = {};
  f4 cW3[6] = {}, cL4[3] = {};
  // per-channel scales of f (Conv2dNormy exp(logs), Conv2dZerosy exp(3 logs)) and the
  // conditioning nets' last layers, once per workgroup (ordered by the tile's first barrier)
  {
    const float *F = glow + kOffF;
    if (tid < 2 * kYH + kC)
      S.esc[tid] = tid < kYH ? expf(F[Aff::f0al + tid])
                   : tid < 2 * kYH ? expf(F[Aff::f2al + tid - kYH]) : expf(F[Aff::f4l + tid - 2 * kYH] * 3.0f);
    for (int k = tid; k < 2 * kC * kXS; k += kThreads) S.w4A[k] = glow[kOffA + CondA::l4w + k];
    for (int k = tid; k < kC * kC * kXS; k += kThreads) S.w4I[k] = glow[kOffI + CondI::l4w + k];
    if (tid < 2 * kC + kC * kC)
      S.b4[tid] = tid < 2 * kC ? glow[kOffA + CondA::l4b + tid] : glow[kOffI + CondI::l4b + tid - 2 * kC];
    for (int k = tid; k < 2 * kXH * kXH * 4; k += kThreads) {
      const int net = k >> 8, j = k & 255;
      S.wc2[net][j] = glow[(net ? kOffI : kOffA) + CondA::c2w + j];
      S.wc4[net][j] = glow[(net ? kOffI : kOffA) + CondA::c4w + j];
    }
  }
  const float *es0 = S.esc, *es2 = S.esc + kYH, *e3 = S.esc + 2 * kYH;

  for (int64_t tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    // weight pointers laundered per tile: the compiler re-reads the weights from the caches in
    // each tile instead of hoisting thousands of scalar loads out of the tile loop (SGPR spills)
    const float *gw_ = glow, *pe = pe_;
    asm volatile("" : "+s"(gw_), "+s"(pe));
    const float *gA = gw_ + kOffA, *gI = gw_ + kOffI, *F = gw_ + kOffF;
#ifdef NFDPF_EXP_CBTRACE
    const bool cbt_on = tile == blockIdx.x + 2 * (int64_t)gridDim.x;
#endif
    const int64_t m_raw = tile * kTP + p;
    const bool valid = m_raw < M;
    const int64_t m = valid ? m_raw : M - 1;  // invalid lanes recompute a real particle, upstream 0
    const int rowb = PART ? (int)(m / N) : (int)m;
    CBT(0);
    // ---------------- forward recompute ----------------
    float yq[kC];  // squeezed y at position q: channel c * 4 + f
    {
      const float *yr = PART ? enc + (int64_t)rowb * enc_rs : enc + m * kE;
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int f = 0; f < 4; ++f) yq[c * 4 + f] = yr[c * 64 + (2 * qi + (f >> 1)) * 8 + 2 * qj + (f & 1)];
    }
#pragma unroll
    for (int k = 0; k < kE / 16; ++k) S.gX[p][q + 16 * k] = 0.f;
    if (PART) {
      const int i = (int)(m - (int64_t)rowb * N);
      if (q < 2) S.pxy[p][q] = x[(int64_t)rowb * x_rs + 2 * i + q];
      __syncthreads();
      {  // h1: lane = hidden unit (W1 row_pairs: W1[j][k] at ((j >> 1) * 2 + k) * 2 + (j & 1))
        const int j = q;
        float a = pe[kPeB1 + j];
        a = fmaf(pe[((j >> 1) * 2 + 0) * 2 + (j & 1)], S.pxy[p][0], a);
        a = fmaf(pe[((j >> 1) * 2 + 1) * 2 + (j & 1)], S.pxy[p][1], a);
        S.h1[p][j] = relu(a);
      }
      __syncthreads();
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {  // h2 (W2 col_pairs: W2[o][k] at (k * 16 + (o >> 1)) * 2 + (o & 1))
        const int o = q + 16 * hh;
        float a = pe[kPeB2 + o];
#pragma unroll
        for (int k = 0; k < kPeH1; ++k) a = fmaf(pe[kPeW2 + (k * (kPeH2 / 2) + (o >> 1)) * 2 + (o & 1)], S.h1[p][k], a);
        S.h2[p][o] = relu(a);
      }
      __syncthreads();
      {  // xs = W3 h2 + b3 on MFMA (the forward kernel's arithmetic): C[p][n], A = h2, B[k][n] =
         // W3[n][k] (col_pairs: (k * 96 + n / 2) * 2 + n % 2); wave w: column tiles w, w + 4, w + 8
        float bw[3][8];
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int n = (w + 4 * j) * 16 + lr;
#pragma unroll
          for (int s2 = 0; s2 < 8; ++s2) bw[j][s2] = pe[kPeW3 + ((4 * s2 + lk) * (kE / 2) + (n >> 1)) * 2 + (n & 1)];
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          const int n0 = (w + 4 * j) * 16;
          f4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
          for (int s2 = 0; s2 < 8; ++s2) c = mfma4(S.h2[lr][4 * s2 + lk], bw[j][s2], c);
          const float bias = pe[kPeW3 + kE * kPeH2 + n0 + lr];
#pragma unroll
          for (int i = 0; i < 4; ++i) S.X[4 * lk + i][n0 + lr] = c[i] + bias;
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < kE / 16; ++k) S.X[p][q + 16 * k] = x[m * kE + q + 16 * k];
    }
    __syncthreads();
    CBT(1);
    // conditioning nets: conv1 (3 -> 8, 2x2 stride 2, 8x8 -> 4x4) at position q
    {
      float in[12];
#pragma unroll
      for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b2 = 0; b2 < 2; ++b2) in[c * 4 + a * 2 + b2] = S.X[p][c * 64 + (2 * qi + a) * 8 + 2 * qj + b2];
#pragma unroll
      for (int net = 0; net < 2; ++net) {
        const float *G = net ? gI : gA;
#pragma unroll
        for (int o = 0; o < kXH; ++o) {
          float a = G[CondA::c0b + o];
#pragma unroll
          for (int k = 0; k < 12; ++k) a = fmaf(G[CondA::c0w + k * kXH + o], in[k], a);
          S.c1[p][q][net * kXH + o] = relu(a);
        }
      }
    }
    __syncthreads();
    {  // conv2 (8 -> 8, 4x4 -> 2x2): lane q = (net, output channel), the four positions
      const int net = q >> 3, o = q & 7;
      const float *G = net ? gI : gA;
      _Pragma("unroll 1") for (int pos = 0; pos < 4; ++pos) {
        float a = G[CondA::c2b + o];
#pragma unroll
        for (int ci = 0; ci < kXH; ++ci)
#pragma unroll
          for (int ab = 0; ab < 4; ++ab)
            a = fmaf(S.wc2[net][o * 32 + ci * 4 + ab],
                     S.c1[p][(2 * (pos >> 1) + (ab >> 1)) * 4 + 2 * (pos & 1) + (ab & 1)][net * kXH + ci], a);
        S.c2[p][pos][net * kXH + o] = relu(a);
      }
    }
    __syncthreads();
    {  // conv3 (2x2 -> 1x1)
      const int net = q >> 3, o = q & 7;
      const float *G = net ? gI : gA;
      float a = G[CondA::c4b + o];
#pragma unroll
      for (int ci = 0; ci < kXH; ++ci)
#pragma unroll
        for (int ab = 0; ab < 4; ++ab) a = fmaf(S.wc4[net][o * 32 + ci * 4 + ab], S.c2[p][ab][net * kXH + ci], a);
      S.c3[p][net * kXH + o] = relu(a);
    }
    __syncthreads();
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {  // x_Linear 8 -> 16
      const int net = hh, o = q;
      const float *G = net ? gI : gA;
      float a = G[CondA::l0b + o];
#pragma unroll
      for (int k = 0; k < kXH; ++k) a = fmaf(G[CondA::l0w + o * kXH + k], S.c3[p][net * kXH + k], a);
      S.l0[p][net * kXS + o] = relu(a);
    }
    __syncthreads();
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {  // 16 -> 16
      const int net = hh, o = q;
      const float *G = net ? gI : gA;
      float a = G[CondA::l2b + o];
#pragma unroll
      for (int k = 0; k < kXS; ++k) a = fmaf(G[CondA::l2w + o * kXS + k], S.l0[p][net * kXS + k], a);
      S.l1[p][net * kXS + o] = relu(a);
    }
    __syncthreads();
    for (int idx = q; idx < 2 * kC + kC * kC; idx += 16) {  // last layer + tanh: A (24) then I (144)
      const bool isI = idx >= 2 * kC;
      const int n = isI ? idx - 2 * kC : idx;
      const float *W = isI ? S.w4I : S.w4A;
      float a = S.b4[idx];
#pragma unroll
      for (int k = 0; k < kXS; ++k) a = fmaf(W[n * kXS + k], S.l1[p][(isI ? kXS : 0) + k], a);
      const float t = tanhf(a);
      if (isI)
        S.wm[p][n] = t;
      else
        S.an[p][n] = t;
    }
    __syncthreads();
    CBT(2);
    // actnorm, 1x1 conv at position q
    float yw[kC];
    {
      float ya[kC];
#pragma unroll
      for (int c = 0; c < kC; ++c) {
        ya[c] = (yq[c] + S.an[p][kC + c]) * expf(S.an[p][c]);
        S.ya[p][q][c] = ya[c];
      }
      const f4 *wr = reinterpret_cast<const f4 *>(S.wm[p]);
#pragma unroll
      for (int o = 0; o < kC; ++o) {
        float a = 0.f;
#pragma unroll
        for (int c4 = 0; c4 < kC / 4; ++c4) {
          const f4 wv = wr[o * (kC / 4) + c4];
#pragma unroll
          for (int e = 0; e < 4; ++e) a = fmaf(wv[e], ya[4 * c4 + e], a);
        }
        yw[o] = a;
      }
    }
    CBT(16);
    // W^-1: Gauss-Jordan with partial pivoting, lane q < 12 holding row q of [W | I]
    {
      float a[2 * kC];
      const int qr = q < kC ? q : 0;
#pragma unroll
      for (int j = 0; j < kC; ++j) {
        a[j] = q < kC ? S.wm[p][qr * kC + j] : 0.f;
        a[kC + j] = (q == j) ? 1.f : 0.f;
      }
      bool done = q >= kC;
      int mycol = 0;
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
          for (int j = 0; j < 2 * kC; ++j) S.prow[p][j] = a[j];
        WFENCE();
        float pr[2 * kC];
        {
          const f4 *pv = reinterpret_cast<const f4 *>(S.prow[p]);
#pragma unroll
          for (int j4 = 0; j4 < 2 * kC / 4; ++j4) {
            const f4 v = pv[j4];
#pragma unroll
            for (int e = 0; e < 4; ++e) pr[4 * j4 + e] = v[e];
          }
        }
        const float inv = 1.0f / pr[k];
        if (q == who) {
          done = true;
          mycol = k;
#pragma unroll
          for (int j = 0; j < 2 * kC; ++j) a[j] = pr[j] * inv;
        } else if (q < kC) {
          const float f = a[k];
#pragma unroll
          for (int j = 0; j < 2 * kC; ++j) a[j] = fmaf(-f, pr[j] * inv, a[j]);
        }
        WFENCE();
      }
      if (q < kC)
#pragma unroll
        for (int j = 0; j < kC; ++j) S.wi[p][mycol * kC + j] = a[kC + j];
    }
    CBT(17);
    // resize_x: conv3x3 (3 -> 16) at this position's 2x2 block of the 8x8 grid, ReLU, conv 2x2/2
    // (16 -> 6), ReLU
    auto resize1 = [&](float (&h)[4][16]) {
#pragma unroll
      for (int ab = 0; ab < 4; ++ab)
#pragma unroll
        for (int o = 0; o < 16; ++o) h[ab][o] = F[Aff::r0b + o];
      _Pragma("unroll 3") for (int t = 0; t < 27; ++t) {
        const int dr = t / 9, ds = (t / 3) % 3, c = t % 3;
        float v[4];
#pragma unroll
        for (int ab = 0; ab < 4; ++ab) {
          const int r = 2 * qi + (ab >> 1) + dr - 1, s = 2 * qj + (ab & 1) + ds - 1;
          v[ab] = (r >= 0 && r < 8 && s >= 0 && s < 8) ? S.X[p][c * 64 + r * 8 + s] : 0.f;
        }
#pragma unroll
        for (int o = 0; o < 16; ++o) {
          const float wt = F[Aff::r0w + t * 16 + o];
#pragma unroll
          for (int ab = 0; ab < 4; ++ab) h[ab][o] = fmaf(wt, v[ab], h[ab][o]);
        }
      }
#pragma unroll
      for (int ab = 0; ab < 4; ++ab)
#pragma unroll
        for (int o = 0; o < 16; ++o) h[ab][o] = relu(h[ab][o]);
    };
    float r2v[kCh];
    {
      float r1[4][16];
      resize1(r1);
#pragma unroll
      for (int o = 0; o < kCh; ++o) {
      float a = F[Aff::r2b + o];
#pragma unroll
      for (int ab = 0; ab < 4; ++ab)
#pragma unroll
        for (int c = 0; c < 16; ++c) a = fmaf(F[Aff::r2w + (ab * 16 + c) * kCh + o], r1[ab][c], a);
      r2v[o] = relu(a);
      S.r2[p][q][o] = r2v[o];
      }
    }
    __syncthreads();
    CBT(3);
    float fin[kC];
    {  // conv3x3 (6 -> 6), ReLU
      float a[kCh];
#pragma unroll
      for (int o = 0; o < kCh; ++o) a[o] = F[Aff::r4b + o];
      _Pragma("unroll 1") for (int t9 = 0; t9 < 9; ++t9) {
        const int rr = qi + t9 / 3 - 1, ss = qj + t9 % 3 - 1;
        if (!in4(rr, ss)) continue;
        float v[kCh];
#pragma unroll
        for (int c = 0; c < kCh; ++c) v[c] = S.r2[p][rr * 4 + ss][c];
#pragma unroll
        for (int c = 0; c < kCh; ++c)
#pragma unroll
          for (int o = 0; o < kCh; ++o) a[o] = fmaf(F[Aff::r4w + (t9 * kCh + c) * kCh + o], v[c], a[o]);
      }
#pragma unroll
      for (int o = 0; o < kCh; ++o) fin[o] = relu(a[o]);
    }
#pragma unroll
    for (int c = 0; c < kCh; ++c) fin[kCh + c] = yw[c];
#pragma unroll
    for (int c = 0; c < kC; ++c) S.fin[p][q][c] = fin[c];
    __syncthreads();
    CBT(4);
    // f: Conv2dNormy(12 -> 8, 3x3) ReLU, Conv2dNormy(8 -> 8, 1x1) ReLU, Conv2dZerosy(8 -> 12) tanh
    float g1[kYH], g2[kYH], u[kC], h[kC];
    {
      float a[kYH] = {};
      _Pragma("unroll 1") for (int t9 = 0; t9 < 9; ++t9) {
        const int rr = qi + t9 / 3 - 1, ss = qj + t9 % 3 - 1;
        if (!in4(rr, ss)) continue;
        float v[kC];
#pragma unroll
        for (int c = 0; c < kC; ++c) v[c] = S.fin[p][rr * 4 + ss][c];
#pragma unroll
        for (int c = 0; c < kC; ++c)
#pragma unroll
          for (int o = 0; o < kYH; ++o) a[o] = fmaf(F[Aff::f0w + (t9 * kC + c) * kYH + o], v[c], a[o]);
      }
#pragma unroll
      for (int o = 0; o < kYH; ++o) {
        g1[o] = relu((a[o] + F[Aff::f0ab + o]) * es0[o]);
        S.g1[p][q][o] = g1[o];
      }
    }
#pragma unroll
    for (int o = 0; o < kYH; ++o) {
      float a = 0.f;
#pragma unroll
      for (int c = 0; c < kYH; ++c) a = fmaf(F[Aff::f2w + c * kYH + o], g1[c], a);
      g2[o] = relu((a + F[Aff::f2ab + o]) * es2[o]);
      S.g2[p][q][o] = g2[o];
    }
    __syncthreads();
    {
      float a[kC] = {};
      _Pragma("unroll 1") for (int t9 = 0; t9 < 9; ++t9) {
        const int rr = qi + t9 / 3 - 1, ss = qj + t9 % 3 - 1;
        if (!in4(rr, ss)) continue;
        float v[kYH];
#pragma unroll
        for (int c = 0; c < kYH; ++c) v[c] = S.g2[p][rr * 4 + ss][c];
#pragma unroll
        for (int c = 0; c < kYH; ++c)
#pragma unroll
          for (int o = 0; o < kC; ++o) a[o] = fmaf(F[Aff::f4w + (t9 * kYH + c) * kC + o], v[c], a[o]);
      }
#pragma unroll
      for (int o = 0; o < kC; ++o) {
        u[o] = (a[o] + F[Aff::f4b + o] + F[Aff::f4nb + o]) * e3[o];
        h[o] = tanhf(u[o]);
      }
    }

    // ---------------- backward ----------------
    // obj = -log(256) 192 + 16 sum logs + 16 log|det W| + sum log sc + Gaussian logp;
    // lik = obj / (192 ln 2) (PART), nll = -lik
    const float scale = 1.0f / (0.6931471805599453f * (float)kE);
    float gobj = 0.f;
    if (valid) {
      if (PART) {
        const int i = (int)(m - (int64_t)rowb * N);
        gobj = g_up[(int64_t)rowb * gup_rs + i] * scale;
      } else {
        gobj = -g_up[m * gup_rs] * scale;
      }
    }
    float gz1[kCh], gz2[kCh], gu[kC];
    float sb[kC], sl4[kC];  // this lane's terms of the f4 bias / log-scale gradients
#pragma unroll
    for (int c = 0; c < kCh; ++c) {
      const float shift = h[2 * c], sc = sigm(h[2 * c + 1] + 2.0f);
      const float z1 = yw[c], z2 = yw[kCh + c], z2p = (z2 + shift) * sc;
      float ez1 = 0.f, ez2 = 0.f;
      if (!PART && g_z && valid) {
        ez1 = g_z[m * kE + c * 16 + q];
        ez2 = g_z[m * kE + (kCh + c) * 16 + q];
      }
      gz1[c] = fmaf(-z1, gobj, ez1);
      const float gz2p = fmaf(-z2p, gobj, ez2);
      gz2[c] = gz2p * sc;
      const float gsh = gz2p * sc;
      const float gsp = gz2p * (z2 + shift) * sc * (1.0f - sc) + gobj * (1.0f - sc);
      gu[2 * c] = gsh * (1.0f - h[2 * c] * h[2 * c]);
      gu[2 * c + 1] = gsp * (1.0f - h[2 * c + 1] * h[2 * c + 1]);
    }
#pragma unroll
    for (int o = 0; o < kC; ++o) {
      const float d = gu[o] * e3[o];  // dL/d(conv output), = dL/d(bias) = dL/d(newbias)
      S.D[p][q][o] = d;
      sb[o] = d;
      sl4[o] = 3.0f * gu[o] * u[o];
    }
    // per-particle sums of the small parameters: sm[p][0..11] f4 bias, [12..23] f4 logs
#pragma unroll
    for (int o = 0; o < kC; ++o) {
      const float a = row16_sum(sb[o]), b2 = row16_sum(sl4[o]);
      if (q == 0) {
        S.sm[p][o] = a;
        S.sm[p][kC + o] = b2;
      }
    }
    __syncthreads();
    CBT(5);
    {  // f4w: dW[o][n = (t9, c)] = sum_(p,q) D[p][q][o] g2[p][q + tap][c] (K = 256): column
       // tiles w, and 4 in wave 0
      auto job = [&](f4 &cc, int nt) {
        const int n = nt * 16 + lr, t9 = n >> 3, ch = n & 7, dr = t9 / 3 - 1, ds = t9 % 3 - 1;
        const bool nok = n < 9 * kYH, mok = lr < kC;
        const int orow = mok ? lr : 0;
#pragma unroll 4
        for (int s2 = 0; s2 < 64; ++s2) {
          const int k = 4 * s2 + lk, pp = k >> 4, q2 = k & 15;
          const int rr = (q2 >> 2) + dr, ss = (q2 & 3) + ds;
          const bool ok = nok && in4(rr, ss);
          const float bv = S.g2[pp][ok ? rr * 4 + ss : 0][ch];
          const float av = S.D[pp][q2][orow];
          cc = mfma4(mok ? av : 0.f, ok ? bv : 0.f, cc);
        }
      };
      job(cF4a, w);
      if (w == 0) job(cF4b, 4);
    }
    contract<kOffF + Aff::f4b>(acc, [&](int j) {
      float a = 0.f;
      _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.sm[pp][j];
      return a;
    });
    contract<kOffF + Aff::f4nb>(acc, [&](int j) {
      float a = 0.f;
      _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.sm[pp][j];
      return a;
    });
    contract<kOffF + Aff::f4l>(acc, [&](int j) {
      float a = 0.f;
      _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.sm[pp][kC + j];
      return a;
    });
    // transposed conv -> dL/dg2 at q; ReLU; Conv2dNormy(1x1) with actnorm scale es2
    float d2[kYH];
    float tg2[kYH] = {};
    _Pragma("unroll 1") for (int t9 = 0; t9 < 9; ++t9) {
      const int rr = qi - (t9 / 3 - 1), ss = qj - (t9 % 3 - 1);  // the output whose tap t9 reads q
      if (!in4(rr, ss)) continue;
      float dd[kC];
#pragma unroll
      for (int o = 0; o < kC; ++o) dd[o] = S.D[p][rr * 4 + ss][o];
#pragma unroll
      for (int c = 0; c < kYH; ++c)
#pragma unroll
        for (int o = 0; o < kC; ++o) tg2[c] = fmaf(F[Aff::f4w + (t9 * kYH + c) * kC + o], dd[o], tg2[c]);
    }
#pragma unroll
    for (int c = 0; c < kYH; ++c) {
      const float a = tg2[c];
      const float gv = g2[c] > 0.f ? a : 0.f;  // dL/d(v2), v2 = (conv + ab) es2
      d2[c] = gv * es2[c];
      sb[c] = d2[c];          // ab2
      sl4[c] = gv * g2[c];    // al2: dL/dv2 * v2 (v2 = g2 where the ReLU passes)
    }
#pragma unroll
    for (int o = 0; o < kYH; ++o) {
      const float a = row16_sum(sb[o]), b2 = row16_sum(sl4[o]);
      if (q == 0) {
        S.sm[p][24 + o] = a;
        S.sm[p][32 + o] = b2;
      }
    }
    __syncthreads();  // D (f4) fully read
#pragma unroll
    for (int o = 0; o < kYH; ++o) S.D[p][q][o] = d2[o];
    __syncthreads();
    CBT(6);
    if (w == 1) {  // f2w: dW[o][c] = sum_(p,q) D[p][q][o] g1[p][q][c]
      const bool ok = lr < kYH;
      const int o = ok ? lr : 0;
#pragma unroll 4
      for (int s2 = 0; s2 < 64; ++s2) {
        const int k = 4 * s2 + lk, pp = k >> 4, q2 = k & 15;
        const float av = S.D[pp][q2][o], bv = S.g1[pp][q2][o];
        cF2 = mfma4(ok ? av : 0.f, ok ? bv : 0.f, cF2);
      }
    }
    contract<kOffF + Aff::f2ab>(acc, [&](int j) {
      float a = 0.f;
      _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.sm[pp][24 + j];
      return a;
    });
    contract<kOffF + Aff::f2al>(acc, [&](int j) {
      float a = 0.f;
      _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.sm[pp][32 + j];
      return a;
    });
    float d0[kYH];
#pragma unroll
    for (int c = 0; c < kYH; ++c) {
      float a = 0.f;
#pragma unroll
      for (int o = 0; o < kYH; ++o) a = fmaf(F[Aff::f2w + c * kYH + o], d2[o], a);
      const float gv = g1[c] > 0.f ? a : 0.f;
      d0[c] = gv * es0[c];
      sb[c] = d0[c];
      sl4[c] = gv * g1[c];
    }
#pragma unroll
    for (int o = 0; o < kYH; ++o) {
      const float a = row16_sum(sb[o]), b2 = row16_sum(sl4[o]);
      if (q == 0) {
        S.sm[p][o] = a;
        S.sm[p][8 + o] = b2;
      }
    }
    __syncthreads();
#pragma unroll
    for (int o = 0; o < kYH; ++o) S.D[p][q][o] = d0[o];
    __syncthreads();
    {  // f0w: dW[o][n = (t9, c)] = sum D[p][q][o] fin[p][q + tap][c]: column tiles w, w + 4 (< 7)
      auto job = [&](f4 &cc, int nt) {
        const int n = nt * 16 + lr, t9 = n / kC, ch = n % kC, dr = t9 / 3 - 1, ds = t9 % 3 - 1;
        const bool nok = n < 9 * kC, mok = lr < kYH;
        const int orow = mok ? lr : 0;
#pragma unroll 4
        for (int s2 = 0; s2 < 64; ++s2) {
          const int k = 4 * s2 + lk, pp = k >> 4, q2 = k & 15;
          const int rr = (q2 >> 2) + dr, ss = (q2 & 3) + ds;
          const bool ok = nok && in4(rr, ss);
          const float bv = S.fin[pp][ok ? rr * 4 + ss : 0][ok ? ch : 0];
          const float av = S.D[pp][q2][orow];
          cc = mfma4(mok ? av : 0.f, ok ? bv : 0.f, cc);
        }
      };
      job(cF0a, w);
      if (w + 4 < 7) job(cF0b, w + 4);
    }
    contract<kOffF + Aff::f0ab>(acc, [&](int j) {
      float a = 0.f;
      _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.sm[pp][j];
      return a;
    });
    contract<kOffF + Aff::f0al>(acc, [&](int j) {
      float a = 0.f;
      _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.sm[pp][8 + j];
      return a;
    });
    float gfin[kC] = {};
    _Pragma("unroll 1") for (int t9 = 0; t9 < 9; ++t9) {
      const int rr = qi - (t9 / 3 - 1), ss = qj - (t9 % 3 - 1);
      if (!in4(rr, ss)) continue;
      float dd[kYH];
#pragma unroll
      for (int o = 0; o < kYH; ++o) dd[o] = S.D[p][rr * 4 + ss][o];
#pragma unroll
      for (int c = 0; c < kC; ++c)
#pragma unroll
        for (int o = 0; o < kYH; ++o) gfin[c] = fmaf(F[Aff::f0w + (t9 * kC + c) * kYH + o], dd[o], gfin[c]);
    }
#pragma unroll
    for (int c = 0; c < kCh; ++c) gz1[c] += gfin[kCh + c];
    // resize_x conv3 (6 -> 6): ReLU output fin[0..5]
    float d4[kCh];
#pragma unroll
    for (int o = 0; o < kCh; ++o) {
      d4[o] = fin[o] > 0.f ? gfin[o] : 0.f;
      sb[o] = d4[o];
    }
#pragma unroll
    for (int o = 0; o < kCh; ++o) {
      const float a = row16_sum(sb[o]);
      if (q == 0) S.sm[p][16 + o] = a;
    }
    __syncthreads();
#pragma unroll
    for (int o = 0; o < kCh; ++o) S.D[p][q][o] = d4[o];
    __syncthreads();
    CBT(7);
    {  // r4w: dW[o][n = (t9, c)] = sum D[p][q][o] r2[p][q + tap][c]: column tile w (54 columns)
      const int n = w * 16 + lr, t9 = n / kCh, ch = n % kCh, dr = t9 / 3 - 1, ds = t9 % 3 - 1;
      const bool nok = n < 9 * kCh, mok = lr < kCh;
      const int orow = mok ? lr : 0;
#pragma unroll 4
      for (int s2 = 0; s2 < 64; ++s2) {
        const int k = 4 * s2 + lk, pp = k >> 4, q2 = k & 15;
        const int rr = (q2 >> 2) + dr, ss = (q2 & 3) + ds;
        const bool ok = nok && in4(rr, ss);
        const float bv = S.r2[pp][ok ? rr * 4 + ss : 0][ok ? ch : 0];
        const float av = S.D[pp][q2][orow];
        cR4 = mfma4(mok ? av : 0.f, ok ? bv : 0.f, cR4);
      }
    }
    contract<kOffF + Aff::r4b>(acc, [&](int j) {
      float a = 0.f;
      _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.sm[pp][16 + j];
      return a;
    });
    float dr2[kCh];  // dL/d(resize conv2 pre-activation)
    float tr2[kCh] = {};
    _Pragma("unroll 1") for (int t9 = 0; t9 < 9; ++t9) {
      const int rr = qi - (t9 / 3 - 1), ss = qj - (t9 % 3 - 1);
      if (!in4(rr, ss)) continue;
      float dd[kCh];
#pragma unroll
      for (int o = 0; o < kCh; ++o) dd[o] = S.D[p][rr * 4 + ss][o];
#pragma unroll
      for (int c = 0; c < kCh; ++c)
#pragma unroll
        for (int o = 0; o < kCh; ++o) tr2[c] = fmaf(F[Aff::r4w + (t9 * kCh + c) * kCh + o], dd[o], tr2[c]);
    }
#pragma unroll
    for (int c = 0; c < kCh; ++c) {
      const float a = tr2[c];
      dr2[c] = r2v[c] > 0.f ? a : 0.f;
      sb[c] = dr2[c];
    }
#pragma unroll
    for (int o = 0; o < kCh; ++o) {
      const float a = row16_sum(sb[o]);
      if (q == 0) S.sm[p][24 + o] = a;
    }
    __syncthreads();  // D (r4), g1 / g2 (aliased by R1) no longer read; sm complete
    CBT(8);
    contract<kOffF + Aff::r2b>(acc, [&](int j) {
      float a = 0.f;
      _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.sm[pp][24 + j];
      return a;
    });
#pragma unroll
    for (int o = 0; o < kCh; ++o) S.D[p][q][o] = dr2[o];
    // Four rounds of four particles (the resize stage's 8x8 grids do not fit LDS for the whole
    // tile).  In round rw every wave works on particles 4 rw + l / 16 (lane l of the wave) at
    // block q = l % 16, wave w on the channel group 4w .. 4w + 3: r1 recomputed (ReLU outputs)
    // and staged -> r2w (MFMA); d r1 in its place -> r0w (MFMA) and dL/dx (wave w: the block's
    // position w).
    for (int rw = 0; rw < 4; ++rw) {
      const int p4 = (tid & 63) >> 4, pp = 4 * rw + p4;
      float hv[4][4];  // [ab][c4]: channel 4 w + c4
#pragma unroll
      for (int ab = 0; ab < 4; ++ab)
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) hv[ab][c4] = F[Aff::r0b + 4 * w + c4];
      _Pragma("unroll 3") for (int t = 0; t < 27; ++t) {
        const int dr = t / 9, ds = (t / 3) % 3, c = t % 3;
        float v[4];
#pragma unroll
        for (int ab = 0; ab < 4; ++ab) {
          const int r = 2 * qi + (ab >> 1) + dr - 1, s8 = 2 * qj + (ab & 1) + ds - 1;
          const bool in = r >= 0 && r < 8 && s8 >= 0 && s8 < 8;
          const float xv = S.X[pp][in ? c * 64 + r * 8 + s8 : 0];
          v[ab] = in ? xv : 0.f;
        }
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          const float wt = F[Aff::r0w + t * 16 + 4 * w + c4];
#pragma unroll
          for (int ab = 0; ab < 4; ++ab) hv[ab][c4] = fmaf(wt, v[ab], hv[ab][c4]);
        }
      }
#pragma unroll
      for (int ab = 0; ab < 4; ++ab) {
        f4 v;
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) v[c4] = relu(hv[ab][c4]);
        *reinterpret_cast<f4 *>(&S.R1[p4][q][ab][4 * w]) = v;
      }
      __syncthreads();
      if (rw == 0) CBT(13);
      {  // r2w: dW[o][n = (ab, c)] = sum_(p4,q) D[4 rw + p4][q][o] r1[p4][q][ab][c]: tile ab = w
        const bool mok = lr < kCh;
        const int orow = mok ? lr : 0;
#pragma unroll 4
        for (int s2 = 0; s2 < 16; ++s2) {
          const int k = 4 * s2 + lk, k4 = k >> 4, q2 = k & 15;
          const float av = S.D[4 * rw + k4][q2][orow], bv = S.R1[k4][q2][w][lr];
          cR2 = mfma4(mok ? av : 0.f, bv, cR2);
        }
      }
      __syncthreads();
      if (rw == 0) CBT(14);
      {  // d r1 of this lane's entries (read, then overwritten in place), per-particle sums (r0b)
        float dd[kCh];
#pragma unroll
        for (int o = 0; o < kCh; ++o) dd[o] = S.D[pp][q][o];
        float sum4[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ab = 0; ab < 4; ++ab) {
          f4 *slot = reinterpret_cast<f4 *>(&S.R1[p4][q][ab][4 * w]);
          const f4 rv = *slot;
          f4 dv;
#pragma unroll
          for (int c4 = 0; c4 < 4; ++c4) {
            float a = 0.f;
#pragma unroll
            for (int o = 0; o < kCh; ++o) a = fmaf(F[Aff::r2w + (ab * 16 + 4 * w + c4) * kCh + o], dd[o], a);
            dv[c4] = rv[c4] > 0.f ? a : 0.f;
            sum4[c4] += dv[c4];
          }
          *slot = dv;
        }
#pragma unroll
        for (int c4 = 0; c4 < 4; ++c4) {
          const float s1 = row16_sum(sum4[c4]);
          if (q == 0) S.sm[pp][32 + 4 * w + c4] = s1;
        }
      }
      __syncthreads();
      if (rw == 0) CBT(15);
      {  // r0w: dW[o][t] = sum_(p4, 8x8 pos) d1[p4][pos][o] x[p4][c][pos + tap]; wave w: column
         // tile w & 1, particles 2 (w >> 1) .. +1 of the round (the halves are added at the end)
        const int n = (w & 1) * 16 + lr, dr = n / 9 - 1, ds = (n / 3) % 3 - 1, c = n % 3;
        const bool nok = n < 27;
#pragma unroll 4
        for (int s2 = 0; s2 < 32; ++s2) {
          const int k = 4 * s2 + lk, k4 = 2 * (w >> 1) + (k >> 6), pos = k & 63, r = pos >> 3, s8 = pos & 7;
          const int rr = r + dr, ss = s8 + ds;
          const bool ok = nok && rr >= 0 && rr < 8 && ss >= 0 && ss < 8;
          const float bv = S.X[4 * rw + k4][ok ? c * 64 + rr * 8 + ss : 0];
          const float av = S.R1[k4][(r >> 1) * 4 + (s8 >> 1)][(r & 1) * 2 + (s8 & 1)][lr];
          cR0 = mfma4(av, ok ? bv : 0.f, cR0);
        }
      }
      {  // dL/dx from resize conv1 at position w of this lane's 2x2 block, 3 channels
        const int r = 2 * qi + (w >> 1), s8 = 2 * qj + (w & 1);
        float a[3] = {0.f, 0.f, 0.f};
        _Pragma("unroll 1") for (int t9 = 0; t9 < 9; ++t9) {
          const int ro = r - (t9 / 3 - 1), so = s8 - (t9 % 3 - 1);  // output reading (r, s) by tap t9
          if (ro < 0 || ro >= 8 || so < 0 || so >= 8) continue;
          const f4 *dd4 = reinterpret_cast<const f4 *>(S.R1[p4][(ro >> 1) * 4 + (so >> 1)][(ro & 1) * 2 + (so & 1)]);
          float dd[16];
#pragma unroll
          for (int o4 = 0; o4 < 4; ++o4) {
            const f4 v = dd4[o4];
#pragma unroll
            for (int e = 0; e < 4; ++e) dd[4 * o4 + e] = v[e];
          }
#pragma unroll
          for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int o = 0; o < 16; ++o) a[c] = fmaf(F[Aff::r0w + ((t9 * 3) + c) * 16 + o], dd[o], a[c]);
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) S.gX[pp][c * 64 + r * 8 + s8] += a[c];
      }
      __syncthreads();
      CBT(9);
    }
    contract<kOffF + Aff::r0b>(acc, [&](int j) {
      float a = 0.f;
      _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.sm[pp][32 + j];
      return a;
    });
    // 1x1 conv and actnorm: dL/dyw = (g_z1, g_z2)
    float gyw[kC];
#pragma unroll
    for (int c = 0; c < kCh; ++c) {
      gyw[c] = gz1[c];
      gyw[kCh + c] = gz2[c];
    }
#pragma unroll
    for (int o = 0; o < kC; ++o) S.D[p][q][o] = gyw[o];
    float gya[kC];
#pragma unroll
    for (int c = 0; c < kC; ++c) {
      float a = 0.f;
#pragma unroll
      for (int o = 0; o < kC; ++o) a = fmaf(S.wm[p][o * kC + c], gyw[o], a);
      gya[c] = a;
    }
    __syncthreads();
    // dL/dW[o][c] = sum_q gyw[o] ya[c] + 16 gobj W^-1[c][o]; lane q: entries q + 16 k
    for (int e = q; e < kC * kC; e += 16) {
      const int o = e / kC, c = e % kC;
      float a = 0.f;
      for (int qq = 0; qq < 16; ++qq) a = fmaf(S.D[p][qq][o], S.ya[p][qq][c], a);
      a = fmaf(16.0f * gobj, S.wi[p][c * kC + o], a);
      S.gw[p][e] = a;
    }
    {  // dL/dy (squeezed back to 3x8x8); dL/dlogs, dL/dbias summed over the positions
      float *gyr = g_y + m * kE;
#pragma unroll
      for (int c = 0; c < kC; ++c) {
        const float gy0 = gya[c] * expf(S.an[p][c]);
        if (valid) gyr[(c >> 2) * 64 + (2 * qi + ((c & 3) >> 1)) * 8 + 2 * qj + (c & 1)] = gy0;
        const float gls = row16_sum(gya[c] * S.ya[p][q][c]), gb = row16_sum(gy0);
        if (q == 0) {
          S.gan[p][c] = fmaf(16.0f, gobj, gls);
          S.gan[p][kC + c] = gb;
        }
      }
    }
    __syncthreads();
    CBT(10);
    // ---------------- conditioning nets backward (A: actnorm, I: 1x1 conv) ----------------
    for (int idx = q; idx < 2 * kC + kC * kC; idx += 16) {  // through the tanh
      const bool isI = idx >= 2 * kC;
      const int n = isI ? idx - 2 * kC : idx;
      if (isI) {
        const float t = S.wm[p][n];
        S.gw[p][n] *= 1.0f - t * t;
      } else {
        const float t = S.an[p][n];
        S.gan[p][n] *= 1.0f - t * t;
      }
    }
    __syncthreads();
    // last layers: dW[n][k] = sum_p g[p][n] l1[p][k] (K = 16 particles) on MFMA: row tiles
    // A 0-1, I 0-8 as jobs w, w + 4, w + 8 (< 11)
#pragma unroll
    for (int jj = 0; jj < 3; ++jj) {
      const int job = w + 4 * jj;
      if (job >= 11) break;
      const bool isI = job >= 2;
      const int n = (isI ? job - 2 : job) * 16 + lr, nout = isI ? kC * kC : 2 * kC;
      const bool ok = n < nout;
#pragma unroll
      for (int s2 = 0; s2 < 4; ++s2) {
        const int k = 4 * s2 + lk;
        const float av = isI ? S.gw[k][ok ? n : 0] : S.gan[k][ok ? n : 0];
        cL4[jj] = mfma4(ok ? av : 0.f, S.l1[k][(isI ? kXS : 0) + lr], cL4[jj]);
      }
    }
    contract<kOffA + CondA::l4b>(acc, [&](int j) {
      float a = 0.f;
      _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.gan[pp][j];
      return a;
    });
    contract<kOffI + CondI::l4b>(acc, [&](int j) {
      float a = 0.f;
      _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.gw[pp][j];
      return a;
    });
    // the small gradient buffers of the nets reuse D: per particle [0, 32) l1, [32, 64) l0,
    // [64, 80) c3, [80, 144) c2 (pos, net * 8 + ci)
    float *Gp = &S.D[p][0][0];
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {  // dL/dl1, lane q = hidden unit, net hh
      const int net = hh, k = q;
      float a = 0.f;
      if (net == 0) {
        _Pragma("unroll 8") for (int n = 0; n < 2 * kC; ++n) a = fmaf(S.w4A[n * kXS + k], S.gan[p][n], a);
      } else {
        _Pragma("unroll 8") for (int n = 0; n < kC * kC; ++n) a = fmaf(S.w4I[n * kXS + k], S.gw[p][n], a);
      }
      Gp[net * kXS + k] = S.l1[p][net * kXS + k] > 0.f ? a : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int net = 0; net < 2; ++net) {
      auto l2w = [&](int j) {
        const int o = j / kXS, k = j % kXS;
        float a = 0.f;
        _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a = fmaf(S.D[pp][0][net * kXS + o], S.l0[pp][net * kXS + k], a);
        return a;
      };
      auto l2b = [&](int j) {
        float a = 0.f;
        _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.D[pp][0][net * kXS + j];
        return a;
      };
      if (net == 0) {
        contract<kOffA + CondA::l2w>(acc, l2w);
        contract<kOffA + CondA::l2b>(acc, l2b);
      } else {
        contract<kOffI + CondI::l2w>(acc, l2w);
        contract<kOffI + CondI::l2b>(acc, l2b);
      }
    }
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {  // dL/dl0
      const int net = hh, k = q;
      const float *G = net ? gI : gA;
      float a = 0.f;
#pragma unroll
      for (int o = 0; o < kXS; ++o) a = fmaf(G[CondA::l2w + o * kXS + k], Gp[net * kXS + o], a);
      Gp[32 + net * kXS + k] = S.l0[p][net * kXS + k] > 0.f ? a : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int net = 0; net < 2; ++net) {
      auto l0w = [&](int j) {
        const int o = j / kXH, k = j % kXH;
        float a = 0.f;
        _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a = fmaf(S.D[pp][0][32 + net * kXS + o], S.c3[pp][net * kXH + k], a);
        return a;
      };
      auto l0b = [&](int j) {
        float a = 0.f;
        _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.D[pp][0][32 + net * kXS + j];
        return a;
      };
      if (net == 0) {
        contract<kOffA + CondA::l0w>(acc, l0w);
        contract<kOffA + CondA::l0b>(acc, l0b);
      } else {
        contract<kOffI + CondI::l0w>(acc, l0w);
        contract<kOffI + CondI::l0b>(acc, l0b);
      }
    }
    {  // dL/dc3: lane q = (net, channel)
      const int net = q >> 3, k = q & 7;
      const float *G = net ? gI : gA;
      float a = 0.f;
#pragma unroll
      for (int o = 0; o < kXS; ++o) a = fmaf(G[CondA::l0w + o * kXH + k], Gp[32 + net * kXS + o], a);
      Gp[64 + net * kXH + k] = S.c3[p][net * kXH + k] > 0.f ? a : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int net = 0; net < 2; ++net) {
      auto c4w = [&](int j) {  // [o][ci][a][b]
        const int o = j / 32, ci = (j / 4) % kXH, ab = j % 4;
        float a = 0.f;
        _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a = fmaf(S.D[pp][0][64 + net * kXH + o], S.c2[pp][ab][net * kXH + ci], a);
        return a;
      };
      auto c4b = [&](int j) {
        float a = 0.f;
        _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.D[pp][0][64 + net * kXH + j];
        return a;
      };
      if (net == 0) {
        contract<kOffA + CondA::c4w>(acc, c4w);
        contract<kOffA + CondA::c4b>(acc, c4b);
      } else {
        contract<kOffI + CondI::c4w>(acc, c4w);
        contract<kOffI + CondI::c4b>(acc, c4b);
      }
    }
    {  // dL/dc2: lane q = (net, ci), the four positions
      const int net = q >> 3, ci = q & 7;
#pragma unroll
      for (int ab = 0; ab < 4; ++ab) {
        float a = 0.f;
#pragma unroll
        for (int o = 0; o < kXH; ++o) a = fmaf(S.wc4[net][o * 32 + ci * 4 + ab], Gp[64 + net * kXH + o], a);
        Gp[80 + ab * 16 + net * kXH + ci] = S.c2[p][ab][net * kXH + ci] > 0.f ? a : 0.f;
      }
    }
    __syncthreads();
#pragma unroll
    for (int net = 0; net < 2; ++net) {
      auto c2b = [&](int j) {
        float a = 0.f;
        _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp)
#pragma unroll
          for (int pos = 0; pos < 4; ++pos) a += S.D[pp][0][80 + pos * 16 + net * kXH + j];
        return a;
      };
      if (net == 0)
        contract<kOffA + CondA::c2b>(acc, c2b);
      else
        contract<kOffI + CondI::c2b>(acc, c2b);
    }
    {  // c2w of net w >> 1, column tile w & 1: dW[o][n = (ci, ab)] = sum_(p, pos) g[p][pos][o] c1[p][..][ci]
      const int net = w >> 1, n = (w & 1) * 16 + lr, ci = n >> 2, ab = n & 3;
      const bool mok = lr < kXH;
#pragma unroll 4
      for (int s2 = 0; s2 < 16; ++s2) {
        const int k = 4 * s2 + lk, pp = k >> 2, pos = k & 3;
        const float av = S.D[pp][0][80 + pos * 16 + net * kXH + (mok ? lr : 0)];
        const float bv = S.c1[pp][(2 * (pos >> 1) + (ab >> 1)) * 4 + 2 * (pos & 1) + (ab & 1)][net * kXH + ci];
        cC2 = mfma4(mok ? av : 0.f, bv, cC2);
      }
    }
    {  // dL/dc1 at position q (both nets)
      const int pos = (qi >> 1) * 2 + (qj >> 1), ab = (qi & 1) * 2 + (qj & 1);
#pragma unroll
      for (int net = 0; net < 2; ++net) {
#pragma unroll
        for (int ci = 0; ci < kXH; ++ci) {
          float a = 0.f;
#pragma unroll
          for (int o = 0; o < kXH; ++o) a = fmaf(S.wc2[net][o * 32 + ci * 4 + ab], Gp[80 + pos * 16 + net * kXH + o], a);
          S.G1c[p][q][net * kXH + ci] = S.c1[p][q][net * kXH + ci] > 0.f ? a : 0.f;
        }
      }
    }
    __syncthreads();
    if (w == 2) {  // c0w of both nets (rows net * 8 + o): dW[k = (ci, a, b)][o] = sum_(p,q) g1c x
      const int n = lr < 12 ? lr : 0, ci = n >> 2, a2 = (n >> 1) & 1, b2 = n & 1;
#pragma unroll 4
      for (int s2 = 0; s2 < 64; ++s2) {
        const int k = 4 * s2 + lk, pp = k >> 4, q2 = k & 15;
        const float av = S.G1c[pp][q2][lr];
        const float bv = S.X[pp][ci * 64 + (2 * (q2 >> 2) + a2) * 8 + 2 * (q2 & 3) + b2];
        cC0 = mfma4(av, lr < 12 ? bv : 0.f, cC0);
      }
    }
#pragma unroll
    for (int net = 0; net < 2; ++net) {
      auto c0b = [&](int j) {
        float a = 0.f;
        _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp)
          for (int qq = 0; qq < 16; ++qq) a += S.G1c[pp][qq][net * kXH + j];
        return a;
      };
      if (net == 0)
        contract<kOffA + CondA::c0b>(acc, c0b);
      else
        contract<kOffI + CondI::c0b>(acc, c0b);
    }
    // dL/dx from both conditioning conv1s at this lane's 2x2 block
#pragma unroll
    for (int k = 0; k < 12; ++k) {
      const int ci = k >> 2, a2 = (k >> 1) & 1, b2 = k & 1;
      float a = 0.f;
#pragma unroll
      for (int net = 0; net < 2; ++net) {
        const float *G = net ? gI : gA;
#pragma unroll
        for (int o = 0; o < kXH; ++o) a = fmaf(G[CondA::c0w + k * kXH + o], S.G1c[p][q][net * kXH + o], a);
      }
      S.gX[p][ci * 64 + (2 * qi + a2) * 8 + 2 * qj + b2] += a;
    }
    __syncthreads();
    CBT(11);
    // ---------------- the condition's gradient: out, or through the particle encoder ----------------
    if (!PART) {
      if (valid)
#pragma unroll
        for (int k = 0; k < kE / 16; ++k) g_x[m * kE + q + 16 * k] = S.gX[p][q + 16 * k];
    } else {
#pragma unroll
      for (int jj = 0; jj < 6; ++jj) {  // W3: dW[n][k] = sum_p gX[p][n] h2[p][k]; job w + 4 jj = (n tile, k tile)
        const int j = w + 4 * jj, mt = j >> 1, kt = j & 1;
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          const int k = 4 * s2 + lk;
          cW3[jj] = mfma4(S.gX[k][mt * 16 + lr], S.h2[k][kt * 16 + lr], cW3[jj]);
        }
      }
      contract<kStep + kPeW3 + kE * kPeH2>(acc, [&](int j) {
        float a = 0.f;
        _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.gX[pp][j];
        return a;
      });
      {  // dL/dh2[p][k] = sum_n gX[p][n] W3[n][k] on MFMA -> D[p][0][0..31]: wave w: k tile w & 1,
         // n half w >> 1 (the halves added in a fixed order through LDS)
        const int kt = w & 1, nh = w >> 1, kk = kt * 16 + lr;
        float bw[24];
#pragma unroll
        for (int s2 = 0; s2 < 24; ++s2) {
          const int n = nh * 96 + 4 * s2 + lk;
          bw[s2] = pe[kPeW3 + (kk * (kE / 2) + (n >> 1)) * 2 + (n & 1)];
        }
        f4 c = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s2 = 0; s2 < 24; ++s2) c = mfma4(S.gX[lr][nh * 96 + 4 * s2 + lk], bw[s2], c);
        float *cmb = &S.R1[0][0][0][0];
        if (nh == 1)
#pragma unroll
          for (int i = 0; i < 4; ++i) cmb[(kt * 64 + (tid & 63)) * 4 + i] = c[i];
        __syncthreads();
        if (nh == 0)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int pp = 4 * lk + i;
            const float v = c[i] + cmb[(kt * 64 + (tid & 63)) * 4 + i];
            S.D[pp][0][kk] = S.h2[pp][kk] > 0.f ? v : 0.f;
          }
      }
      __syncthreads();
      contract<kStep + kPeW2>(acc, [&](int j) {
        const int pr = j >> 1, k = pr / (kPeH2 / 2), o = (pr % (kPeH2 / 2)) * 2 + (j & 1);
        float a = 0.f;
        _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a = fmaf(S.D[pp][0][o], S.h1[pp][k], a);
        return a;
      });
      contract<kStep + kPeB2>(acc, [&](int j) {
        float a = 0.f;
        _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.D[pp][0][j];
        return a;
      });
      {  // dL/dh1 -> D[p][0][32 + k]
        const int k = q;
        float a = 0.f;
#pragma unroll
        for (int o = 0; o < kPeH2; ++o) a = fmaf(pe[kPeW2 + (k * (kPeH2 / 2) + (o >> 1)) * 2 + (o & 1)], Gp[o], a);
        Gp[32 + k] = S.h1[p][k] > 0.f ? a : 0.f;
      }
      __syncthreads();
      contract<kStep + 0>(acc, [&](int j) {  // row_pairs: W1[jj][i] at ((jj >> 1) * 2 + i) * 2 + (jj & 1)
        const int t = j >> 1, i = t & 1, jj = (t >> 1) * 2 + (j & 1);
        float a = 0.f;
        _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a = fmaf(S.D[pp][0][32 + jj], S.pxy[pp][i], a);
        return a;
      });
      contract<kStep + kPeB1>(acc, [&](int j) {
        float a = 0.f;
        _Pragma("unroll 1") for (int pp = 0; pp < kTP; ++pp) a += S.D[pp][0][32 + j];
        return a;
      });
      if (q < 2 && valid) {
        const int i = q;
        float a = 0.f;
#pragma unroll
        for (int jj = 0; jj < kPeH1; ++jj) a = fmaf(pe[((jj >> 1) * 2 + i) * 2 + (jj & 1)], Gp[32 + jj], a);
        g_x[m * 2 + i] = a;
      }
    }
    __syncthreads();
    CBT(12);
  }
  // this workgroup's parameter-gradient row
  float *row = partial + (int64_t)blockIdx.x * kTotParams;
  store_acc<0>(acc, row);
  store_tile(cF4a, row, kC, w * 16, 9 * kYH, [](int m, int n) { return kOffF + Aff::f4w + n * kC + m; });
  if (w == 0) store_tile(cF4b, row, kC, 64, 9 * kYH, [](int m, int n) { return kOffF + Aff::f4w + n * kC + m; });
  store_tile(cF0a, row, kYH, w * 16, 9 * kC, [](int m, int n) { return kOffF + Aff::f0w + n * kYH + m; });
  if (w + 4 < 7)
    store_tile(cF0b, row, kYH, (w + 4) * 16, 9 * kC, [](int m, int n) { return kOffF + Aff::f0w + n * kYH + m; });
  store_tile(cR4, row, kCh, w * 16, 9 * kCh, [](int m, int n) { return kOffF + Aff::r4w + n * kCh + m; });
  store_tile(cR2, row, kCh, 0, 16, [w](int m, int n) { return kOffF + Aff::r2w + (w * 16 + n) * kCh + m; });
  if (w == 1) store_tile(cF2, row, kYH, 0, kYH, [](int m, int n) { return kOffF + Aff::f2w + n * kYH + m; });
  if (w == 2)
    store_tile(cC0, row, 16, 0, 12, [](int m, int n) { return ((m >> 3) ? kOffI : kOffA) + CondA::c0w + n * kXH + (m & 7); });
  {
    const int net = w >> 1;
    store_tile(cC2, row, kXH, (w & 1) * 16, 32,
               [net](int m, int n) { return (net ? kOffI : kOffA) + CondA::c2w + m * 32 + n; });
  }
#pragma unroll
  for (int jj = 0; jj < 3; ++jj) {
    const int job = w + 4 * jj;
    if (job < 11) {
      const bool isI = job >= 2;
      const int m0 = (isI ? job - 2 : job) * 16;
      const int rows = min(16, (isI ? kC * kC : 2 * kC) - m0);
      store_tile(cL4[jj], row, rows, 0, kXS,
                 [=](int m, int n) { return (isI ? kOffI + CondI::l4w : kOffA + CondA::l4w) + (m0 + m) * kXS + n; });
    }
  }
  if (PART)
#pragma unroll
    for (int jj = 0; jj < 6; ++jj) {
      const int j = w + 4 * jj, mt = j >> 1, kt = j & 1;
      store_tile(cW3[jj], row, 16, kt * 16, 32, [mt](int m, int n) {
        const int nx = mt * 16 + m;
        return kStep + kPeW3 + (n * (kE / 2) + (nx >> 1)) * 2 + (nx & 1);
      });
    }
  // r0w: the two particle halves (waves w and w + 2) added in a fixed order
  float *cmb = &S.D[0][0][0];
  const int l = tid & 63;
  if (w >= 2)
#pragma unroll
    for (int i = 0; i < 4; ++i) cmb[((w - 2) * 64 + l) * 4 + i] = cR0[i];
  __syncthreads();
  if (w < 2) {
    f4 t = cR0;
#pragma unroll
    for (int i = 0; i < 4; ++i) t[i] += cmb[(w * 64 + l) * 4 + i];
    store_tile(t, row, 16, w * 16, 27, [](int m, int n) { return kOffF + Aff::r0w + n * 16 + m; });
  }
}

// out[j] = sum over the workgroup rows, in row order
__global__ __launch_bounds__(256) void cglow_param_reduce_kernel(const float *__restrict__ partial, int rows,
                                                                 float *__restrict__ g_glow, float *__restrict__ g_pe) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= kTotParams) return;
  float a = 0.f;
  for (int r = 0; r < rows; ++r) a += partial[(int64_t)r * kTotParams + j];
  if (j < kStep)
    g_glow[j] = a;
  else if (g_pe)
    g_pe[j - kStep] = a;
}

// One resident workgroup per CU (160 KB of LDS each), persistent over tiles.  A fixed cap (the
// MI355X's 256 CUs), not the current device's CU count: the workspace the caller sized with
// nfdpf_cglow_backward_workspace holds exactly this many partial rows, whichever device is
// current at either call.
constexpr int kBwdGrid = 256;
static int bwd_grid(int64_t M) {
  const int64_t tiles = (M + kTP - 1) / kTP;
  return (int)std::max<int64_t>(1, std::min<int64_t>(tiles, kBwdGrid));
}

template <bool PART>
static int launch_bwd(const float *pe, const float *glow, const float *enc, int64_t enc_rs, const float *x,
                      int64_t x_rs, int B, int N, const float *g_up, int64_t gup_rs, const float *g_z, float *g_y,
                      float *g_x, float *g_glow, float *g_pe, void *ws, hipStream_t st) {
  const int64_t M = (int64_t)B * N;
  const int grid = bwd_grid(M);
  const size_t lds = sizeof(BLds);
  ensure_max_dynamic_lds((const void *)cglow_bwd_kernel<PART>, (int)lds);
  float *partial = (float *)ws;
  cglow_bwd_kernel<PART><<<grid, kThreads, lds, st>>>(pe, glow, enc, enc_rs, x, x_rs, B, N, g_up, gup_rs, g_z, g_y,
                                                      g_x, partial);
  cglow_param_reduce_kernel<<<(kTotParams + 255) / 256, 256, 0, st>>>(partial, grid, g_glow, g_pe);
  return launch_status("cglow_backward");
}

}  // namespace cgb
}  // namespace nfdpf

using namespace nfdpf;

#ifdef NFDPF_EXP_CBTRACE
extern "C" NFDPF_API int nfdpf_exp_cbtrace_read(void *host) {
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(cgb::g_cbtrace), sizeof(cgb::g_cbtrace)) == hipSuccess ? 0 : 1;
}
#endif

extern "C" int64_t nfdpf_cglow_backward_workspace(int64_t M) {
  if (M < 0) return -1;
  return (int64_t)cgb::bwd_grid(M) * cgb::kTotParams * (int64_t)sizeof(float);
}

extern "C" int nfdpf_cglow_measurement_backward(const float *pe_params, const float *glow_params, int K,
                                                const float *enc, int64_t enc_rs, const float *x, int64_t x_rs,
                                                int B, int N, const float *g_lik, int64_t glik_rs, float *g_x,
                                                float *g_y, float *g_glow, float *g_pe, void *workspace,
                                                void *stream) {
  NFDPF_REQUIRE(K == 1, "nfdpf_cglow_measurement_backward: built for flow_depth K = 1 (got %d)", K);
  NFDPF_REQUIRE(B >= 0 && N >= 1, "nfdpf_cglow_measurement_backward: bad sizes");
  NFDPF_REQUIRE(g_glow && g_pe, "nfdpf_cglow_measurement_backward: null pointer");
  hipStream_t st = as_stream(stream);
  if (B == 0) {
    (void)hipMemsetAsync(g_glow, 0, sizeof(float) * cg::kStep, st);
    (void)hipMemsetAsync(g_pe, 0, sizeof(float) * cgb::kPeE, st);
    return launch_status("nfdpf_cglow_measurement_backward");
  }
  NFDPF_REQUIRE(pe_params && glow_params && enc && x && g_lik && g_x && g_y && workspace,
                "nfdpf_cglow_measurement_backward: null pointer");
  return cgb::launch_bwd<true>(pe_params, glow_params, enc, enc_rs, x, x_rs, B, N, g_lik, glik_rs, nullptr, g_y,
                               g_x, g_glow, g_pe, workspace, as_stream(stream));
}

extern "C" int nfdpf_cglow_flow_backward(const float *glow_params, int K, const float *x, const float *y, int64_t M,
                                         const float *g_z, const float *g_nll, float *g_x, float *g_y,
                                         float *g_glow, void *workspace, void *stream) {
  NFDPF_REQUIRE(K == 1, "nfdpf_cglow_flow_backward: built for flow_depth K = 1 (got %d)", K);
  NFDPF_REQUIRE(M >= 0 && M <= (int64_t)INT32_MAX, "nfdpf_cglow_flow_backward: bad size");
  NFDPF_REQUIRE(g_glow, "nfdpf_cglow_flow_backward: null pointer");
  hipStream_t st = as_stream(stream);
  if (M == 0) {
    (void)hipMemsetAsync(g_glow, 0, sizeof(float) * cg::kStep, st);
    return launch_status("nfdpf_cglow_flow_backward");
  }
  NFDPF_REQUIRE(glow_params && x && y && g_nll && g_x && g_y && workspace, "nfdpf_cglow_flow_backward: null pointer");
  return cgb::launch_bwd<false>(nullptr, glow_params, y, cg::kE, x, 0, (int)M, 1, g_nll, 1, g_z, g_y, g_x, g_glow,
                                nullptr, workspace, st);
}
