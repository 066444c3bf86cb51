// Experiment: cost of a kernel boundary vs an in-kernel grid barrier (agent-scope fences + one
// device counter) for grids of 256 / 512 workgroups of 256 threads.  Each "iteration" every
// workgroup writes 4 KB and, after the boundary / barrier, reads the 4 KB another workgroup
// (on another XCD) wrote and checks it.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      exit(1);                                                                 \
    }                                                                          \
  } while (0)

constexpr int kWords = 1024;  // 4 KB per workgroup per iteration

__device__ __forceinline__ void work(float *buf, int wg, int nwg, int it, int *bad) {
  // check the partner's words of the previous iteration, then write this iteration's
  if (it > 0) {
    const int p = (wg + 1) % nwg;
    const float *src = buf + ((int64_t)((it - 1) & 1) * nwg + p) * kWords;
    for (int k = threadIdx.x; k < kWords; k += blockDim.x)
      if (src[k] != (float)(p * 7 + (it - 1) * 13 + k)) atomicAdd(bad, 1);
  }
  float *dst = buf + ((int64_t)(it & 1) * nwg + wg) * kWords;
  for (int k = threadIdx.x; k < kWords; k += blockDim.x) dst[k] = (float)(wg * 7 + it * 13 + k);
}

__global__ __launch_bounds__(256) void step_kernel(float *buf, int it, int *bad) {
  work(buf, blockIdx.x, gridDim.x, it, bad);
}

__global__ __launch_bounds__(256) void persist_kernel(float *buf, int iters, unsigned *cnt, int *bad, int *tmo) {
  const int nwg = gridDim.x;
  for (int it = 0; it < iters; ++it) {
    work(buf, blockIdx.x, nwg, it, bad);
    __syncthreads();
    if (threadIdx.x == 0) {
      __threadfence();
      __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const unsigned target = (unsigned)nwg * (it + 1);
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
        __builtin_amdgcn_s_sleep(1);
        if (__hip_atomic_load(tmo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) break;
        if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {  // 1 s at 100 MHz
          atomicAdd(tmo, 1);
          break;
        }
      }
      __threadfence();
    }
    __syncthreads();
  }
}

// V: bit0 = fences, bit1 = flag array (else one atomic counter)
template <int V>
__global__ __launch_bounds__(256) void persist_v(float *buf, int iters, unsigned *cnt, unsigned *flags, int *bad, int *tmo) {
  const int nwg = gridDim.x;
  for (int it = 0; it < iters; ++it) {
    work(buf, blockIdx.x, nwg, it, bad);
    __syncthreads();
    if (threadIdx.x < 64) {
      if ((V & 1) && threadIdx.x == 0) __threadfence();
      if (V & 2) {
        if (threadIdx.x == 0) __hip_atomic_store(flags + blockIdx.x, (unsigned)(it + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        for (;;) {
          bool ok = true;
          for (int w = threadIdx.x; w < nwg; w += 64)
            ok = ok && __hip_atomic_load(flags + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= (unsigned)(it + 1);
          if (__all(ok)) break;
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {
            if (threadIdx.x == 0) atomicAdd(tmo, 1);
            break;
          }
        }
      } else if (threadIdx.x == 0) {
        __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned target = (unsigned)nwg * (it + 1);
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
        while (__hip_atomic_load(cnt, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
          __builtin_amdgcn_s_sleep(1);
          if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {
            atomicAdd(tmo, 1);
            break;
          }
        }
      }
      if ((V & 1) && threadIdx.x == 0) __threadfence();
    }
    __syncthreads();
  }
}

template <int V>
static void run_v(int nwg, int iters, float *buf, unsigned *cnt, unsigned *flags, int *bad, int *tmo) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  CK(hipMemset(bad, 0, 64));
  CK(hipMemset(cnt, 0, 64));
  CK(hipMemset(tmo, 0, 64));
  CK(hipMemset(flags, 0, 4096));
  CK(hipEventRecord(a, 0));
  persist_v<V><<<nwg, 256>>>(buf, iters, cnt, flags, bad, tmo);
  CK(hipEventRecord(b, 0));
  CK(hipEventSynchronize(b));
  float ms = 0;
  CK(hipEventElapsedTime(&ms, a, b));
  int pb = 0, pt = 0;
  CK(hipMemcpy(&pb, bad, 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(&pt, tmo, 4, hipMemcpyDeviceToHost));
  printf("  nwg %d variant fences=%d flags=%d: %.2f us/iter (bad %d, timeouts %d)\n", nwg, V & 1, (V >> 1) & 1,
         1000.0 * ms / iters, pb, pt);
}

int main() {
  const int iters = 200;
  for (int nwg : {256, 512}) {
    float *buf;
    unsigned *cnt;
    int *bad, *tmo;
    CK(hipMalloc(&buf, (size_t)2 * nwg * kWords * 4));
    CK(hipMalloc(&cnt, 64));
    CK(hipMalloc(&bad, 64));
    CK(hipMalloc(&tmo, 64));
    int occ = 0;
    CK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, persist_kernel, 256, 0));
    hipDeviceProp_t pr;
    CK(hipGetDeviceProperties(&pr, 0));
    if (occ * pr.multiProcessorCount < nwg) {
      printf("nwg %d: not co-resident (%d x %d)\n", nwg, occ, pr.multiProcessorCount);
      continue;
    }
    hipEvent_t a, b;
    CK(hipEventCreate(&a));
    CK(hipEventCreate(&b));
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipMemset(bad, 0, 64));
      CK(hipEventRecord(a, 0));
      for (int it = 0; it < iters; ++it) step_kernel<<<nwg, 256>>>(buf, it, bad);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms_l = 0;
      CK(hipEventElapsedTime(&ms_l, a, b));
      int hb = 0;
      CK(hipMemcpy(&hb, bad, 4, hipMemcpyDeviceToHost));
      CK(hipMemset(bad, 0, 64));
      CK(hipMemset(cnt, 0, 64));
      CK(hipMemset(tmo, 0, 64));
      CK(hipEventRecord(a, 0));
      persist_kernel<<<nwg, 256>>>(buf, iters, cnt, bad, tmo);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms_p = 0;
      CK(hipEventElapsedTime(&ms_p, a, b));
      int pb = 0, pt = 0;
      CK(hipMemcpy(&pb, bad, 4, hipMemcpyDeviceToHost));
      CK(hipMemcpy(&pt, tmo, 4, hipMemcpyDeviceToHost));
      printf("nwg %d occ %d: launches %.2f us/iter (bad %d) | grid barrier %.2f us/iter (bad %d, timeouts %d)\n",
             nwg, occ, 1000.0 * ms_l / iters, hb, 1000.0 * ms_p / iters, pb, pt);
    }
    unsigned *flags;
    CK(hipMalloc(&flags, 4096));
    for (int rep = 0; rep < 2; ++rep) {
      run_v<0>(nwg, iters, buf, cnt, flags, bad, tmo);
      run_v<1>(nwg, iters, buf, cnt, flags, bad, tmo);
      run_v<2>(nwg, iters, buf, cnt, flags, bad, tmo);
      run_v<3>(nwg, iters, buf, cnt, flags, bad, tmo);
    }
    CK(hipFree(flags));
    CK(hipFree(buf));
    CK(hipFree(cnt));
    CK(hipFree(bad));
    CK(hipFree(tmo));
  }
  return 0;
}
