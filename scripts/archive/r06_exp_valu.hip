// Experiment: issue cost per wave64 instruction on one SIMD for the Sinkhorn pair loop's mix --
// v_pk_fma_f32 / v_pk_add_f32 / v_pk_mul_f32 streams, v_exp_f32, and the loop's 7 packed : 2 exp
// pattern -- at one and two waves per SIMD (256 / 512 workgroups of 256 threads).  Cycles from
// s_memtime (shader clock) around the loop, wall from s_memrealtime (100 MHz).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void k(float *out, int iters, unsigned long long *cyc, float seed) {
  f2 a[8], b = f2{seed, seed * 0.5f}, c = f2{0.999f, 1.001f};
#pragma unroll
  for (int u = 0; u < 8; ++u) a[u] = f2{(float)threadIdx.x * 1e-3f + u, -(float)u};
  float e[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) e[u] = -(float)(threadIdx.x & 7) * 0.01f - u * 0.1f;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
  for (int it = 0; it < iters; ++it) {
    if (MODE == 0) {  // packed fma stream: 8 independent
#pragma unroll
      for (int u = 0; u < 8; ++u) a[u] = __builtin_elementwise_fma(a[u], c, b);
    } else if (MODE == 1) {  // exp stream: 8 independent
#pragma unroll
      for (int u = 0; u < 8; ++u) e[u] = __builtin_amdgcn_exp2f(e[u]) - 1.0f;
    } else {  // the shared-kernel block per two pairs: dx, dy, dx^2, fma, scale, 2 exps, 2 fma-acc
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const f2 dx = a[u] - b, dy = a[u + 4] - c;
        const f2 q = __builtin_elementwise_fma(dy, dy, dx * dx) * f2{-0.01f, -0.01f};
        const f2 kk = f2{__builtin_amdgcn_exp2f(q.x), __builtin_amdgcn_exp2f(q.y)};
        a[u] = __builtin_elementwise_fma(b, kk, a[u]);
        a[u + 4] = __builtin_elementwise_fma(c, kk, a[u + 4]);
      }
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 8; ++u) s += a[u].x + a[u].y + e[u];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    cyc[0] = t1 - t0;
    cyc[1] = r1 - r0;
  }
}

int main() {
  float *out;
  unsigned long long *cyc, h[2];
  hipMalloc(&out, 1024 * 256 * 4);
  hipMalloc(&cyc, 16);
  const int iters = 20000;
  const char *names[3] = {"pk_fma x8", "exp x8", "pair block (4 x {7 pk, 2 exp})"};
  const double per_it[3] = {8, 8, 4};  // instructions of the named kind / pair-groups per iteration
  for (int mode = 0; mode < 3; ++mode) {
    for (int wgs : {256, 512}) {
      for (int rep = 0; rep < 2; ++rep) {
        if (mode == 0) k<0><<<wgs, 256>>>(out, iters, cyc, 1.f);
        if (mode == 1) k<1><<<wgs, 256>>>(out, iters, cyc, 1.f);
        if (mode == 2) k<2><<<wgs, 256>>>(out, iters, cyc, 1.f);
        hipDeviceSynchronize();
      }
      hipMemcpy(h, cyc, 16, hipMemcpyDeviceToHost);
      const double n = (double)iters * per_it[mode];
      printf("%-34s waves/SIMD %d: %.2f shader cycles per unit (clock %.2f GHz)\n", names[mode], wgs / 256,
             (double)h[0] / n, (double)h[0] / ((double)h[1] * 10.0));
    }
  }
  return 0;
}
