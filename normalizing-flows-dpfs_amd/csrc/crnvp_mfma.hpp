// crnvp_mfma.hpp -- the conditional-RealNVP measurement (model/models.py:256-278; nf/flows.py:
// 183-226, nf/models.py:38-51) for the 64 particles of a wave on f32 MFMA
// (v_mfma_f32_16x16x4_f32), with FEATURES as the MFMA rows (M) and PARTICLES as its columns (N).
//
// Every dense layer of the measurement is a GEMM over the wave's particles:
//   encoder   2 -> 16 (VALU, relu) -> 32 (relu) -> 32 = e, the condition
//   per flow f and coupling half n (nets t, s stacked as 16 hidden rows: t 0-7, s 8-15):
//     fold    W1[:, HALF:] e + b1          (16 x 32)  -- the per-particle condition columns
//     layer 1 + W1[:, :HALF] u             (16 x 16)  -- u = lo (half 1) or up (half 2)
//     layer 2 block-diag(W2t, W2s)         (16 x 16)
//     layer 3 block-diag(W3t, W3s) -> [t; s] (32 x 16; t units in registers 0-1, s in 2-3,
//             so each output tile reads only its net's two K-steps)
//     up = t + up exp(s)  (half 1) / lo = t + lo exp(s)  (half 2);  log-det += sum(s)
//   prior     N(0, prior_std^2 I) log-density of [lo, up] (fp64)
// so one particle's 12.7 kFLOP run as 400 MFMAs per wave (layer 2's block-diagonal tile at half
// occupancy) instead of ~3,100 packed VALU FMAs with their weights streamed through the scalar
// cache (26 KB per particle pass: SMEM 2.2e7 per launch).
//
// Layout.  A 16x16 D tile holds rows 4 g + r (g = lane >> 4, register r) of column (lane & 15),
// so chained layers need no data movement: K-step s of the next layer takes, in lane group g,
// feature k(s, g) = 16 (s >> 2) + 4 g + (s & 3) -- register (s & 3) of the previous layer's M
// tile (s >> 2) -- and its A operand is W[16 MT + (lane & 15)][k(s, lane >> 4)].  The host
// packs every matrix in that fragment order (nfdpf.pack.crnvp_mfma_tensors): [M tile][lane]
// [K step], so a lane's operands of one M tile are contiguous (ds_read_b128) once the blob is
// staged in LDS.  The particle of column c of N tile q is particle 16 q + c of the wave.
//
// tanh in the "r form" (as the C2 pass, nfdpf.pack.pass_coupling_tensors): every hidden unit is
// r = 1 / (1 + 2^y) of a pre-scaled argument, the -2 and the next layer's 2 log2(e) folded into
// the weights, so a unit costs exp2 + add + rcp.  MFMA f32 is an exact k-ordered fmaf chain; the
// sums run in another order than the reference's MKL GEMMs (rounding-level differences, the
// float32 envelope of tests/test_gpu_pass_cm.py).
#pragma once

#include "flows.hpp"

namespace nfdpf {

typedef float f4v __attribute__((ext_vector_type(4)));

// the fragment blob (floats), include/nfdpf.h nfdpf_filter_pass_tiled
constexpr int kCmfEW1 = 0;                     // encoder layer 1: W1 [16][2], then b1 [16] (plain)
constexpr int kCmfEW2 = 48;                    // layer 2: [2 MT][64][4]
constexpr int kCmfEB2 = kCmfEW2 + 2 * 64 * 4;  // [32]
constexpr int kCmfEW3 = kCmfEB2 + 32;          // layer 3: [2 MT][64][8]
constexpr int kCmfEB3 = kCmfEW3 + 2 * 64 * 8;  // [32]
constexpr int kCmfEnc = kCmfEB3 + 32;          // encoder floats (1648)
// per coupling half (flow f, half n at kCmfEnc + (2 f + n) kCmfHalf):
constexpr int kCmfWc = 0;                      // fold over e: [64][8]
constexpr int kCmfW1 = kCmfWc + 64 * 8;        // layer 1 over u: [64][4]
constexpr int kCmfW2 = kCmfW1 + 64 * 4;        // [64][4]
constexpr int kCmfW3 = kCmfW2 + 64 * 4;        // [2 MT][64][4]
constexpr int kCmfB1 = kCmfW3 + 2 * 64 * 4;    // [16]
constexpr int kCmfB2 = kCmfB1 + 16;            // [16]
constexpr int kCmfB3 = kCmfB2 + 16;            // [32]
constexpr int kCmfHalf = kCmfB3 + 32;          // 1600
__host__ __device__ constexpr int crnvp_mfma_floats(int n_flows) { return kCmfEnc + 2 * n_flows * kCmfHalf; }

__device__ __forceinline__ f4v mfma4(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f4v ld4(const float *p) { return *reinterpret_cast<const f4v *>(p); }
// relu as one v_max_i32 on the bit pattern (a negative float, -0 included, is a negative int):
// fmaxf(x, 0) of an MFMA result compiles to a canonicalising v_max(x, x) plus the max
__device__ __forceinline__ float relu_i(float x) { return __int_as_float(max(__float_as_int(x), 0)); }
__device__ __forceinline__ float sig_r(float y) { return __builtin_amdgcn_rcpf(__builtin_amdgcn_exp2f(y) + 1.0f); }
__device__ __forceinline__ double shfl_xor_d(double v, int m) {
  const long long x = __double_as_longlong(v);
  const int lo = __shfl_xor((int)x, m), hi = __shfl_xor((int)(x >> 32), m);
  return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// the raw CRNVP likelihood of the wave's particle `lane` (crnvp_lik's value): W = the fragment
// blob in LDS, xr = the wave's 64 particles [64][2] in LDS, encv = the row's frame encoding (32,
// LDS).  Every lane of the wave takes part (MFMA operands); lanes of invalid particles return
// a value nobody reads.
__device__ __forceinline__ float crnvp_lik_mfma(const float *W, int n_flows, float prior_std, const float *encv,
                                                const float *xr) {
  const int l = threadIdx.x & 63, col = l & 15, g = l >> 4;
  // ---- encoder layer 1 (VALU) straight into the B layout: h1[q][r] = feature 4 g + r of particle 16 q + col
  float h1[4][4];
  {
    float w0[4], w1[4], b1[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      w0[r] = W[kCmfEW1 + 2 * (4 * g + r)];
      w1[r] = W[kCmfEW1 + 2 * (4 * g + r) + 1];
      b1[r] = W[kCmfEW1 + 32 + 4 * g + r];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const float x0 = xr[2 * (16 * q + col)], x1 = xr[2 * (16 * q + col) + 1];
#pragma unroll
      for (int r = 0; r < 4; ++r) h1[q][r] = relu_i(fmaf(w1[r], x1, fmaf(w0[r], x0, b1[r])));
    }
  }
  // ---- layers 2 (16 -> 32, relu) and 3 (32 -> 32): e, the condition; one N tile at a time (its
  // layer-2 output is all layer 3 needs: 8 live registers instead of 32)
  f4v e[2][4];
  {
    const f4v a2[2] = {ld4(W + kCmfEW2 + l * 4), ld4(W + kCmfEW2 + (64 + l) * 4)};
    const f4v bias2[2] = {ld4(W + kCmfEB2 + 4 * g), ld4(W + kCmfEB2 + 16 + 4 * g)};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      f4v h2[2];
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        f4v acc = bias2[mt];
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(a2[mt][s], h1[q][s], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = relu_i(acc[r]);
        h2[mt] = acc;
      }
#pragma unroll
      for (int mt = 0; mt < 2; ++mt) {
        const f4v a0 = ld4(W + kCmfEW3 + (mt * 64 + l) * 8), a1 = ld4(W + kCmfEW3 + (mt * 64 + l) * 8 + 4);
        f4v acc = ld4(W + kCmfEB3 + 16 * mt + 4 * g);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(a0[s], h2[0][s], acc);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(a1[s], h2[1][s], acc);
        e[mt][q] = acc;
      }
    }
  }
  // ---- the flows: lo = encv[0:16], up = encv[16:32] (the same for every particle at the start)
  f4v lo[4], up[4];
  {
    const f4v lo0 = ld4(encv + 4 * g), up0 = ld4(encv + 16 + 4 * g);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      lo[q] = lo0;
      up[q] = up0;
    }
  }
  float lds[4] = {0.f, 0.f, 0.f, 0.f};  // per N tile: this lane's share of sum(s) over every half
  for (int f = 0; f < n_flows; ++f) {
#pragma unroll
    for (int n = 0; n < 2; ++n) {
      const float *H = W + kCmfEnc + (2 * f + n) * kCmfHalf;
      f4v (&u)[4] = n == 0 ? lo : up;
      f4v (&v)[4] = n == 0 ? up : lo;
      // fold + layer 1
      const f4v c0 = ld4(H + kCmfWc + l * 8), c1 = ld4(H + kCmfWc + l * 8 + 4), a1 = ld4(H + kCmfW1 + l * 4);
      const f4v b1 = ld4(H + kCmfB1 + 4 * g);
      f4v hh[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f4v acc = b1;
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(c0[s], e[0][q][s], acc);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(c1[s], e[1][q][s], acc);
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(a1[s], u[q][s], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = sig_r(acc[r]);
        hh[q] = acc;
      }
      // layer 2
      const f4v a2 = ld4(H + kCmfW2 + l * 4), b2 = ld4(H + kCmfB2 + 4 * g);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f4v acc = b2;
#pragma unroll
        for (int s = 0; s < 4; ++s) acc = mfma4(a2[s], hh[q][s], acc);
#pragma unroll
        for (int r = 0; r < 4; ++r) acc[r] = sig_r(acc[r]);
        hh[q] = acc;
      }
      // layer 3: t (M tile 0) and s (M tile 1), then the coupling update.  The t units sit in
      // registers 0-1 of every lane group, the s units in 2-3 (the packer's hidden row order), so
      // t reads K-steps 0-1 and s K-steps 2-3: the block-diagonal zeros are never multiplied
      const f4v a3t = ld4(H + kCmfW3 + l * 4), a3s = ld4(H + kCmfW3 + (64 + l) * 4);
      const f4v b3t = ld4(H + kCmfB3 + 4 * g), b3s = ld4(H + kCmfB3 + 16 + 4 * g);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        f4v t = b3t, s = b3s;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          t = mfma4(a3t[k], hh[q][k], t);
          s = mfma4(a3s[2 + k], hh[q][2 + k], s);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {  // exp(s) as one v_exp_f32 of s log2(e): |s| is O(1) here, where
                                       // expf's range reduction (~10 VALU) buys nothing
          v[q][r] = t[r] + v[q][r] * __builtin_amdgcn_exp2f(s[r] * 1.4426950408889634f);
        }
        lds[q] += (s[0] + s[1]) + (s[2] + s[3]);
      }
    }
  }
  // ---- log N(z; 0, prior_std^2 I) in fp64 + the log-det: this lane's 8 features of each
  // column, then the column's 4 lane groups (xor 16, 32); lane l keeps column (l & 15) of its
  // own tile q = l >> 4 -- particle l
  const double is = 1.0 / (double)prior_std;
  double mq[4];
  float ldq[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    double m = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double a = lo[q][r] * is, c = up[q][r] * is;
      m = fma(a, a, m);
      m = fma(c, c, m);
    }
    m += shfl_xor_d(m, 16);
    mq[q] = m + shfl_xor_d(m, 32);
    float ls = lds[q];
    ls += __shfl_xor(ls, 16);
    ldq[q] = ls + __shfl_xor(ls, 32);
  }
  const double m = g == 0 ? mq[0] : g == 1 ? mq[1] : g == 2 ? mq[2] : mq[3];
  const float ld = g == 0 ? ldq[0] : g == 1 ? ldq[1] : g == 2 ? ldq[2] : ldq[3];
  const double lp = -0.5 * (kE * 1.8378770664093453 + m) - kE * log((double)prior_std);
  return (float)(lp + (double)ld);
}

}  // namespace nfdpf
