// common.hpp -- device utilities shared by the libnfdpf kernels (gfx950 / CDNA4).
//
// * error plumbing for the C ABI (include/nfdpf.h)
// * Philox4x32-10 counter RNG + Box-Muller (shard-invariant device RNG mode)
// * tanh with Cephes-style small-argument polynomial (FCNN activations, nf/flows.py:105-111)
// * wave64 / workgroup reductions with a fixed, thread-count-independent combine order
// * the ATen-CPU cascade row sum (oracle/cascade.py) for bit-exact soft resampling
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdio>
#include <string>

#include "../../include/nfdpf.h"

namespace nfdpf {

// ----------------------------------------------------------------------------------------
// host-side error plumbing
// ----------------------------------------------------------------------------------------
void set_error(const char *fmt, ...);
int launch_status(const char *what);
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (kernel, current device), thread-safe
void ensure_max_dynamic_lds(const void *fn, int bytes);

#define NFDPF_REQUIRE(cond, ...)            \
  do {                                      \
    if (!(cond)) {                          \
      ::nfdpf::set_error(__VA_ARGS__);      \
      return NFDPF_EINVAL;                  \
    }                                       \
  } while (0)

inline hipStream_t as_stream(void *s) { return reinterpret_cast<hipStream_t>(s); }

constexpr int kWave = 64;

// ----------------------------------------------------------------------------------------
// RNG: Philox4x32-10 (Salmon et al., SC'11).  Counter = (particle, global row, step, tag),
// key = seed.  Streams (tag): see RngTag.
// ----------------------------------------------------------------------------------------
enum RngTag : uint32_t { kTagMotion = 0, kTagOffset = 1, kTagInitPos = 2, kTagInitNormal = 3 };

struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox4x32_10(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = c.x * 0xD2511F53u, hi0 = __umulhi(c.x, 0xD2511F53u);
    const uint32_t lo1 = c.z * 0xCD9E8D57u, hi1 = __umulhi(c.z, 0xCD9E8D57u);
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ U4 rng_draw(uint64_t seed, uint32_t tag, uint32_t step, int64_t row,
                                       uint32_t idx) {
  U4 c{idx, (uint32_t)row, (uint32_t)(row >> 32) ^ (step << 8), tag};
  return philox4x32_10(c, (uint32_t)seed, (uint32_t)(seed >> 32));
}

// [0,1) with 24 random bits
__device__ __forceinline__ float u01(uint32_t u) { return (float)(u >> 8) * 0x1.0p-24f; }
// (0,1]
__device__ __forceinline__ float u01_open0(uint32_t u) { return ((float)(u >> 8) + 1.0f) * 0x1.0p-24f; }

// two standard normals from two uniforms (Box-Muller)
__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float &z0, float &z1) {
  const float r = sqrtf(-2.0f * logf(u01_open0(a)));
  float s, c;
  sincospif(2.0f * u01(b), &s, &c);
  z0 = r * c;
  z1 = r * s;
}

// ----------------------------------------------------------------------------------------
// activations
// ----------------------------------------------------------------------------------------
// tanh(x) = 1 - 2 / (1 + e^{2x}): one v_exp_f32 + one v_rcp_f32 + 2 VALU.  Absolute error
// ~1e-7 over the whole range (relative accuracy near 0 is not needed: every tanh feeds a
// Linear layer, so absolute error is what propagates into t, s and the log-det).
__device__ __forceinline__ float tanh_fast(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);  // 2^(2x log2 e)
  return fmaf(-2.0f, __builtin_amdgcn_rcpf(e + 1.0f), 1.0f);
}

__device__ __forceinline__ float relu(float x) { return fmaxf(x, 0.0f); }

// ----------------------------------------------------------------------------------------
// reductions (fixed combine order: lanes by xor-butterfly, then waves in index order)
// ----------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}

// Row-local wave reductions on DPP (no LDS traffic): butterflies inside quads, then the
// half-row and row mirrors give every lane its 16-lane row's total; the four row totals are
// read with v_readlane and added in a fixed order ((r0 + r1) + (r2 + r3)).  The result is
// wave-uniform.  Fixed order, so deterministic; values are combined commutatively.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(__float_as_int(v), __float_as_int(v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ double dpp_d(double v) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp((int)x, (int)x, CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp((int)(x >> 32), (int)(x >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
constexpr int kDppXor1 = 0xB1, kDppXor2 = 0x4E, kDppHalfMirror = 0x141, kDppMirror = 0x140;

// a double moved by DPP with 0 where the source lane is out of the row (or the row masked off)
template <int CTRL, int ROWMASK = 0xf>
__device__ __forceinline__ double dpp_d0(double v) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)x, CTRL, ROWMASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(x >> 32), CTRL, ROWMASK, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
// Inclusive prefix sum over the wave's 64 lanes on DPP (row_shr 1, 2, 4, 8 inside each 16-lane
// row, then row_bcast15 / row_bcast31 across rows): six steps without an LDS permute.  Its
// addition order differs from a shfl_up scan: callers rely on it only where every partial sum
// is exact (e.g. f64 sums of ~1e3 fp32 terms of a bounded exponent range).
__device__ __forceinline__ double wave_incl_scan_dpp_d(double v) {
  v += dpp_d0<0x111>(v);
  v += dpp_d0<0x112>(v);
  v += dpp_d0<0x114>(v);
  v += dpp_d0<0x118>(v);
  v += dpp_d0<0x142, 0xa>(v);
  v += dpp_d0<0x143, 0xc>(v);
  return v;
}

__device__ __forceinline__ float readlane_f(float v, int l) {
  return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l));
}
__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long x = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)x, l), hi = __builtin_amdgcn_readlane((int)(x >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_d<kDppXor1>(v);
  v += dpp_d<kDppXor2>(v);
  v += dpp_d<kDppHalfMirror>(v);
  v += dpp_d<kDppMirror>(v);
  return (readlane_d(v, 0) + readlane_d(v, 16)) + (readlane_d(v, 32) + readlane_d(v, 48));
}
// wave_sum_dpp of K values at once, step by step across the values: the K butterfly chains
// are independent, so their DPP / fp64-add latencies overlap (same arithmetic per value).
template <int K>
__device__ __forceinline__ void wave_sum_dpp_n(double (&v)[K]) {
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_d<kDppXor1>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_d<kDppXor2>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_d<kDppHalfMirror>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] += dpp_d<kDppMirror>(v[k]);
#pragma unroll
  for (int k = 0; k < K; ++k)
    v[k] = (readlane_d(v[k], 0) + readlane_d(v[k], 16)) + (readlane_d(v[k], 32) + readlane_d(v[k], 48));
}
__device__ __forceinline__ float wave_max_dpp(float v) {
  v = fmaxf(v, dpp_f<kDppXor1>(v));
  v = fmaxf(v, dpp_f<kDppXor2>(v));
  v = fmaxf(v, dpp_f<kDppHalfMirror>(v));
  v = fmaxf(v, dpp_f<kDppMirror>(v));
  return fmaxf(fmaxf(readlane_f(v, 0), readlane_f(v, 16)), fmaxf(readlane_f(v, 32), readlane_f(v, 48)));
}

__device__ __forceinline__ double wave_max_dpp_d(double v) {
  v = fmax(v, dpp_d<kDppXor1>(v));
  v = fmax(v, dpp_d<kDppXor2>(v));
  v = fmax(v, dpp_d<kDppHalfMirror>(v));
  v = fmax(v, dpp_d<kDppMirror>(v));
  return fmax(fmax(readlane_d(v, 0), readlane_d(v, 16)), fmax(readlane_d(v, 32), readlane_d(v, 48)));
}
// block_max of a float with the wave step on DPP (block_max: six shuffle rounds); same result
__device__ __forceinline__ float block_max_dpp(float v, float *sh) {
  v = wave_max_dpp(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  const int nw = (blockDim.x + 63) >> 6;
  float r = sh[0];
  for (int i = 1; i < nw; ++i) r = fmaxf(r, sh[i]);
  return r;
}
// K workgroup maxima with one LDS exchange (DPP inside each wave); every thread gets all K.
// `sh` holds K doubles per wave.  (block_max below: shuffles and two barriers per value.)
template <int K>
__device__ __forceinline__ void block_max_n(double (&v)[K], double *sh) {
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = wave_max_dpp_d(v[k]);
  __syncthreads();  // sh may still be read by a previous reduction
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < K; ++k) sh[K * (threadIdx.x >> 6) + k] = v[k];
  __syncthreads();
  const int nw = (blockDim.x + 63) >> 6;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    double r = sh[k];
    for (int i = 1; i < nw; ++i) r = fmax(r, sh[K * i + k]);
    v[k] = r;
  }
}

// Four workgroup sums with ONE barrier; thread q < 4 stores sum q to dst[q].  `sh` holds
// 4 doubles per wave and must not be in use by a concurrent reduction.
__device__ __forceinline__ void block_sum4_store(double a, double b, double c, double e, double *sh,
                                                 double *dst) {
  a = wave_sum_dpp(a);
  b = wave_sum_dpp(b);
  c = wave_sum_dpp(c);
  e = wave_sum_dpp(e);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[4 * w] = a;
    sh[4 * w + 1] = b;
    sh[4 * w + 2] = c;
    sh[4 * w + 3] = e;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const int nw = (blockDim.x + 63) >> 6;
    double r = sh[threadIdx.x];
    for (int i = 1; i < nw; ++i) r += sh[4 * i + threadIdx.x];
    dst[threadIdx.x] = r;
  }
}

// Eight workgroup sums with ONE barrier: (a0..a3) -> dst0[0..3], (b0..b3) -> dst1[0..3];
// `sh` holds 8 doubles per wave.
__device__ __forceinline__ void block_sum8_store(const double (&a)[4], double *dst0, const double (&c)[4],
                                                 double *dst1, double *sh) {
  double v[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[k] = wave_sum_dpp(a[k]);
    v[4 + k] = wave_sum_dpp(c[k]);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0)
#pragma unroll
    for (int k = 0; k < 8; ++k) sh[8 * w + k] = v[k];
  __syncthreads();
  if (threadIdx.x < 8) {
    const int nw = (blockDim.x + 63) >> 6;
    double r = sh[threadIdx.x];
    for (int i = 1; i < nw; ++i) r += sh[8 * i + threadIdx.x];
    if (threadIdx.x < 4)
      dst0[threadIdx.x] = r;
    else
      dst1[threadIdx.x - 4] = r;
  }
}

// Workgroup reductions.  `sh` is LDS scratch of >= 16 elements of T, reused across calls
// (the leading barrier protects the previous use).  Every thread gets the result.
template <typename T>
__device__ T block_sum(T v, T *sh) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  const int nw = (blockDim.x + 63) >> 6;
  T r = sh[0];
  for (int i = 1; i < nw; ++i) r += sh[i];
  return r;
}
template <typename T>
__device__ T block_max(T v, T *sh) {
  v = wave_max(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
  __syncthreads();
  const int nw = (blockDim.x + 63) >> 6;
  T r = sh[0];
  for (int i = 1; i < nw; ++i) r = fmax(r, sh[i]);
  return r;
}

// Exclusive prefix over the workgroup of one value per thread (thread order).
template <typename T>
__device__ T block_exclusive_scan(T v, T *sh, T *total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  T inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    T u = __shfl_up(inc, o);
    if (lane >= o) inc += u;
  }
  __syncthreads();
  if (lane == 63) sh[w] = inc;
  __syncthreads();
  const int nw = (blockDim.x + 63) >> 6;
  T base = 0, all = 0;
  for (int i = 0; i < nw; ++i) {
    if (i < w) base += sh[i];
    all += sh[i];
  }
  if (total) *total = all;
  return base + inc - v;
}

__device__ __forceinline__ int ceil_log2_i(int n) { return n <= 1 ? 0 : 32 - __clz(n - 1); }

// ----------------------------------------------------------------------------------------
// ATen CPU cascade sum of a contiguous float row (torch.sum(x, -1) on CPU), bit-exact.
// Order (oracle/cascade.py): 8-wide vectors, 4 ILP slots, 4-level cascade with level step
// 2^max(4, ceil_log2(nvec/4)/4); leftover vectors into slot 0; fold slots 0+1+2+3; scalar
// tail first, then the 8 lanes in order.  Rows shorter than 8 use width-1 vectors.
// Must be called by all 64 lanes of ONE wave; returns the sum in every lane.
// ----------------------------------------------------------------------------------------
template <class Get>
__device__ float cascade_row_sum(const Get &v, int n) {
#pragma clang fp contract(off)
  const int lane = threadIdx.x & 63;
  const int W = (n < 8) ? 1 : 8;
  const int nv = n / W;
  const int n4 = nv / 4;
  const int k = lane / W, j = lane - (lane / W) * W;
  const bool act = lane < 4 * W;
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  if (act) {
    const int power = max(4, ceil_log2_i(n4) / 4);
    const int step = 1 << power, mask = step - 1;
    int i = 0;
    while (i + step <= n4) {
      for (int jj = 0; jj < step; ++jj) a0 += v(((i + jj) * 4 + k) * W + j);
      i += step;
      a1 += a0;
      a0 = 0.f;
      if ((i & (mask << power)) == 0) {
        a2 += a1;
        a1 = 0.f;
        if ((i & (mask << (2 * power))) == 0) {
          a3 += a2;
          a2 = 0.f;
        }
      }
    }
    for (; i < n4; ++i) a0 += v((i * 4 + k) * W + j);
    a0 += a1;
    a0 += a2;
    a0 += a3;
    if (k == 0)
      for (int r = n4 * 4; r < nv; ++r) a0 += v(r * W + j);
  }
  const float s1 = __shfl(a0, j + W), s2 = __shfl(a0, j + 2 * W), s3 = __shfl(a0, j + 3 * W);
  float ps = a0;
  ps += s1;
  ps += s2;
  ps += s3;
  if (W == 1) return __shfl(ps, 0);
  float tot = 0.f;
  for (int r = nv * 8; r < n; ++r) tot += v(r);
#pragma unroll  // lanes 0..7 in order; v_readlane (SGPR broadcast) instead of an LDS permute each
  for (int q = 0; q < 8; ++q) tot += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ps), q));
  return tot;
}

// cascade_row_sum for 8 <= n <= 1024 (n4 <= 32 per lane, so the cascade's block size is 16 and
// no higher level ever flushes): the same additions in the same order, with each lane's up to
// 32 values loaded before the first add (the generic loop waits for every load in turn).
// CAP >= 1024: v(j) may be read for any j < 1024 (an LDS array of that size; the values past n are
// loaded and discarded -- selected away, never added), so no index needs the clamp to n - 1
template <int CAP = 0, class Get>
__device__ float cascade_row_sum_1k(const Get &v, int n) {
#pragma clang fp contract(off)
  // (an opaque lane: inside a persistent step loop the compiler would otherwise hoist the 32
  // loads' lane addresses out of the loop and, out of VGPRs, spill them to scratch -- 32 scratch
  // reloads per call on the forced pass's critical path)
  int lane = threadIdx.x & 63;
  asm volatile("" : "+v"(lane));
  const int nv = n / 8, n4 = nv / 4;
  const int k = lane / 8, j = lane - (lane / 8) * 8;
  const bool act = lane < 32;
  float vals[32];
#pragma unroll
  for (int ii = 0; ii < 32; ++ii) {  // unconditional (clamped) reads: no branch per value
    const float x = v(CAP >= 1024 ? (ii * 4 + k) * 8 + j : min((ii * 4 + k) * 8 + j, n - 1));
    vals[ii] = (act && ii < n4) ? x : 0.f;
  }
  // The cascade's slots, with the values past n4 zeroed (x + 0 = x exactly, the sums are of
  // non-negative terms): a full first block of 16 leaves a1 = S0 and the rest sums into a0 = S1
  // (or, n4 = 32, a second full block makes a1 = S0 + S1 and a0 = 0); with n4 < 16 a0 = S0 and
  // S1 = 0.  In every case the slot is S1 + S0 (IEEE addition commutes): two independent chains
  // of 16 adds instead of one predicated chain of 32.
  float a0 = 0.f;
  if (act) {
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) {
      s0 += vals[jj];
      s1 += vals[16 + jj];
    }
    a0 = s1 + s0;
    if (k == 0)
      for (int r = n4 * 4; r < nv; ++r) a0 += v(r * 8 + j);
  }
  const float s1 = __shfl(a0, j + 8), s2 = __shfl(a0, j + 16), s3 = __shfl(a0, j + 24);
  float ps = a0;
  ps += s1;
  ps += s2;
  ps += s3;
  float tot = 0.f;
  for (int r = nv * 8; r < n; ++r) tot += v(r);
#pragma unroll
  for (int q = 0; q < 8; ++q) tot += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(ps), q));
  return tot;
}

// ----------------------------------------------------------------------------------------
// misc
// ----------------------------------------------------------------------------------------
// Weights are read through the CONSTANT address space: wave-uniform addresses with
// compile-time offsets become s_load_dwordx16 into SGPRs (operands of v_fma_f32 directly),
// instead of one flat/global vector load per weight.
typedef const float __attribute__((address_space(4))) cfloat;

// Hide a wave-uniform pointer from loop-invariant code motion (so a particle loop re-reads
// weights from the scalar cache instead of hoisting hundreds into SGPRs that then spill),
// and re-type it as a constant-address-space pointer.
__device__ __forceinline__ cfloat *wptr(const float *p) {
  asm volatile("" : "+s"(p));
  return (cfloat *)p;
}

inline int round_up(int a, int b) { return (a + b - 1) / b * b; }

// threads per workgroup for a one-row-per-workgroup kernel over n particles
inline int row_threads(int n) {
  int t = round_up(n < 64 ? 64 : n, 64);
  return t > 1024 ? 1024 : t;
}

}  // namespace nfdpf
