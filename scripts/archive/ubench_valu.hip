// Experiment: issue cost per wave-instruction of the VALU ops the coupling nets use
// (v_exp_f32, v_rcp_f32, v_fma_f32, v_pk_fma_f32, v_pk_mul_f32) at 1, 2, 4 waves per SIMD.
// Build: hipcc -O3 -w --offload-arch=gfx950 scripts/archive/ubench_valu.hip -o exp/ubench
#include <hip/hip_runtime.h>
#include <stdio.h>

typedef float f2 __attribute__((ext_vector_type(2)));

constexpr int kIters = 2048;
constexpr int kChains = 8;

template <int OP>
__global__ void ubench(float *out, long long *cyc, float seed) {
  float v[kChains];
  f2 p[kChains];
#pragma unroll
  for (int c = 0; c < kChains; ++c) {
    v[c] = seed * (threadIdx.x + c) * 1e-3f;
    p[c] = f2{v[c], v[c] + 1.f};
  }
  const f2 m = f2{seed, seed * 0.5f}, a = f2{0.25f, 0.125f};
  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < kIters; ++it) {
#pragma unroll
    for (int c = 0; c < kChains; ++c) {
      if (OP == 0) v[c] = __builtin_amdgcn_exp2f(v[c]);
      if (OP == 1) v[c] = __builtin_amdgcn_rcpf(v[c]);
      if (OP == 2) v[c] = fmaf(v[c], seed, 0.5f);
      if (OP == 3) p[c] = __builtin_elementwise_fma(p[c], m, a);
      if (OP == 4) p[c] = p[c] * m;
      if (OP == 5) {  // the tanh2 sequence of flows.hpp on a pair
        const f2 y = p[c] * m;
        const f2 d = f2{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)} + a;
        p[c] = __builtin_elementwise_fma(f2{-2.f, -2.f}, f2{__builtin_amdgcn_rcpf(d.x), __builtin_amdgcn_rcpf(d.y)}, a);
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < kChains; ++c) s += v[c] + p[c].x + p[c].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int OP>
void run(const char *name, int insts_per_chain_step) {
  for (int wps = 1; wps <= 4; wps *= 2) {
    const int threads = 64 * 4 * wps, blocks = 256;
    float *out;
    long long *cyc;
    hipMalloc(&out, sizeof(float) * threads * blocks);
    hipMalloc(&cyc, sizeof(long long) * blocks * threads / 64);
    ubench<OP><<<blocks, threads>>>(out, cyc, 0.999f);
    ubench<OP><<<blocks, threads>>>(out, cyc, 0.999f);
    hipDeviceSynchronize();
    const int nw = blocks * threads / 64;
    long long *h = new long long[nw];
    hipMemcpy(h, cyc, sizeof(long long) * nw, hipMemcpyDeviceToHost);
    double mean = 0;
    for (int i = 0; i < nw; ++i) mean += h[i];
    mean /= nw;
    const double per = mean / ((double)kIters * kChains * insts_per_chain_step);
    printf("%-10s waves/SIMD %d : %.2f cycles per wave-instruction (per SIMD: %.2f)\n", name, wps, per, per / wps);
    delete[] h;
    hipFree(out);
    hipFree(cyc);
  }
}

int main() {
  run<0>("v_exp", 1);
  run<1>("v_rcp", 1);
  run<2>("v_fma", 1);
  run<3>("v_pk_fma", 1);
  run<4>("v_pk_mul", 1);
  run<5>("tanh2", 7);
  return 0;
}
