// Issue-cost microbenchmark (experiment only): cycles per instruction of one wave's stream of
// independent / dependent v_pk_fma_f32, v_fma_f32, v_exp_f32, v_rcp_f32 on gfx950, with W waves
// per SIMD.  Built by hand: hipcc --offload-arch=gfx950 -O3 scripts/archive/exp_issue.hip -o exp/issue_bench
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2 __attribute__((ext_vector_type(2)));

template <int KIND>
__global__ void kern(float *out, long long *cyc, float s0, float s1, int iters) {
  float a[16];
  f2 p[8];
  for (int k = 0; k < 16; ++k) a[k] = threadIdx.x * 0.001f + k;
  for (int k = 0; k < 8; ++k) p[k] = f2{a[2 * k], a[2 * k + 1]};
  const f2 w = f2{s0, s1};
  __syncthreads();
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      if constexpr (KIND == 0) {  // 8 independent pk_fma
#pragma unroll
        for (int k = 0; k < 8; ++k) p[k] = __builtin_elementwise_fma(w, p[k], w);
      } else if constexpr (KIND == 1) {  // 16 independent fma
#pragma unroll
        for (int k = 0; k < 16; ++k) a[k] = __builtin_fmaf(s0, a[k], s1);
      } else if constexpr (KIND == 2) {  // 16 independent exp
#pragma unroll
        for (int k = 0; k < 16; ++k) a[k] = __builtin_amdgcn_exp2f(a[k]);
      } else if constexpr (KIND == 3) {  // 16 independent rcp
#pragma unroll
        for (int k = 0; k < 16; ++k) a[k] = __builtin_amdgcn_rcpf(a[k]);
      } else if constexpr (KIND == 4) {  // 1 dependent pk_fma chain (x8)
#pragma unroll
        for (int k = 0; k < 8; ++k) p[0] = __builtin_elementwise_fma(w, p[0], w);
      } else if constexpr (KIND == 5) {  // 1 dependent fma chain (x16)
#pragma unroll
        for (int k = 0; k < 16; ++k) a[0] = __builtin_fmaf(s0, a[0], s1);
      } else if constexpr (KIND == 6) {  // dependent exp chain (x16)
#pragma unroll
        for (int k = 0; k < 16; ++k) a[0] = __builtin_amdgcn_exp2f(a[0]);
      } else if constexpr (KIND == 7) {  // 4 independent pk_fma chains
#pragma unroll
        for (int k = 0; k < 8; ++k) p[k & 3] = __builtin_elementwise_fma(w, p[k & 3], w);
      }
    }
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  float acc = 0.f;
  for (int k = 0; k < 16; ++k) acc += a[k];
  for (int k = 0; k < 8; ++k) acc += p[k].x + p[k].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int KIND>
void run(const char *name, int ninstr_per_round, int waves_per_simd) {
  const int threads = 256 * waves_per_simd, iters = 2000;
  float *out;
  long long *cyc;
  hipMalloc(&out, threads * 4 * 256);
  hipMalloc(&cyc, 8 * 16 * 256);
  for (int rep = 0; rep < 2; ++rep) kern<KIND><<<256, threads>>>(out, cyc, 0.999f, 0.001f, iters);
  hipDeviceSynchronize();
  long long h[16];
  hipMemcpy(h, cyc, 8 * (threads / 64), hipMemcpyDeviceToHost);
  double n = (double)iters * 8 * ninstr_per_round;
  printf("%-28s waves/SIMD %d: %.2f cycles per instruction per wave (memtime clk)\n", name, waves_per_simd, h[0] / n);
  hipFree(out);
  hipFree(cyc);
}

int main() {
  for (int w = 1; w <= 2; ++w) {
    run<0>("pk_fma independent x8", 8, w);
    run<1>("fma independent x16", 16, w);
    run<2>("exp independent x16", 16, w);
    run<3>("rcp independent x16", 16, w);
    run<4>("pk_fma dependent", 8, w);
    run<5>("fma dependent", 16, w);
    run<6>("exp dependent", 16, w);
    run<7>("pk_fma 4 chains", 8, w);
  }
  return 0;
}
