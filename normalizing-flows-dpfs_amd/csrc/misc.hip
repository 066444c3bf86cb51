// misc.hip -- particle_initialization (utils.py:46-62) in DEVICE rng mode.
#include <cstring>

#include "common.hpp"

namespace nfdpf {

__global__ void particle_init_kernel(const float *__restrict__ start_xy, int B, int N, float width,
                                     int true_state, uint64_t seed, int64_t row_base,
                                     float *__restrict__ x, float *__restrict__ logw) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= (int64_t)B * N) return;
  const int b = (int)(o / N), i = (int)(o - (int64_t)b * N);
  const int64_t grow = row_base + b;
  float a0, a1;
  if (true_state) {
    const U4 r = rng_draw(seed, kTagInitNormal, 0u, grow, (uint32_t)i);
    box_muller(r.x, r.y, a0, a1);
    a0 += start_xy[2 * b];
    a1 += start_xy[2 * b + 1];
  } else {
    // (hi - lo) * U[0,1) + lo, hi = width/2, lo = -width/2 (utils.py:53-56)
    const U4 r = rng_draw(seed, kTagInitPos, 0u, grow, (uint32_t)i);
    const float hi = width / 2.0f, lo = -width / 2.0f;
    a0 = (hi - lo) * u01(r.x) + lo;
    a1 = (hi - lo) * u01(r.y) + lo;
  }
  x[2 * o] = a0;
  x[2 * o + 1] = a1;
  logw[o] = logf(1.0f / (float)N);  // torch.log(ones / N) (:60)
}

// torch.sum(x, -1) of each row in ATen's CPU cascade order, one wave per row: variant 0 =
// cascade_row_sum (any n), 1 = cascade_row_sum_1k (8 <= n <= 1024, the one-launch pass's forced
// resampling) -- the same additions in the same order, so the same bits
__global__ __launch_bounds__(64) void cascade_row_sum_kernel(const float *__restrict__ x, int N, int variant,
                                                             float *__restrict__ out) {
  const float *row = x + (int64_t)blockIdx.x * N;
  const float s = variant ? cascade_row_sum_1k([&](int j) { return row[j]; }, N)
                          : cascade_row_sum([&](int j) { return row[j]; }, N);
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

}  // namespace nfdpf

using namespace nfdpf;

extern "C" int nfdpf_cascade_row_sum(const float *x, int B, int N, int variant, float *out, void *stream) {
  NFDPF_REQUIRE(x && out && B >= 0 && N >= 1, "nfdpf_cascade_row_sum: bad arguments");
  NFDPF_REQUIRE(!variant || (N >= 8 && N <= 1024), "nfdpf_cascade_row_sum: variant 1 needs 8 <= N <= 1024");
  if (B == 0) return NFDPF_OK;
  cascade_row_sum_kernel<<<B, 64, 0, as_stream(stream)>>>(x, N, variant, out);
  return launch_status("nfdpf_cascade_row_sum");
}

extern "C" int nfdpf_particle_init(const float *start_xy, int B, int N, float width, int true_state,
                                   uint64_t seed, int64_t row_base, float *x, float *logw,
                                   void *stream) {
  NFDPF_REQUIRE(x && logw && (!true_state || start_xy), "nfdpf_particle_init: null pointer");
  NFDPF_REQUIRE(B >= 0 && N >= 1, "nfdpf_particle_init: bad sizes");
  const int64_t M = (int64_t)B * N;
  if (M == 0) return NFDPF_OK;
  particle_init_kernel<<<(unsigned)((M + 255) / 256), 256, 0, as_stream(stream)>>>(
      start_xy, B, N, width, true_state, seed, row_base, x, logw);
  return launch_status("nfdpf_particle_init");
}

// Pinned, device-mapped, coherent host memory (the zero-copy path of hipHostMalloc): a kernel's
// small result words (the one-launch pass's flags) land in host memory with the kernel, and the
// host reads them once an event behind the kernel has completed -- no copy launch.
extern "C" int nfdpf_host_mapped_alloc(int64_t bytes, void **host, void **dev) {
  NFDPF_REQUIRE(bytes > 0 && host && dev, "nfdpf_host_mapped_alloc: bad arguments");
  *host = *dev = nullptr;
  if (hipHostMalloc(host, (size_t)bytes, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    *host = nullptr;
    return launch_status("nfdpf_host_mapped_alloc (hipHostMalloc)");
  }
  memset(*host, 0, (size_t)bytes);
  if (hipHostGetDevicePointer(dev, *host, 0) != hipSuccess) {
    (void)hipHostFree(*host);
    *host = *dev = nullptr;
    return launch_status("nfdpf_host_mapped_alloc (hipHostGetDevicePointer)");
  }
  return NFDPF_OK;
}

extern "C" int nfdpf_host_mapped_free(void *host) {
  if (host) NFDPF_REQUIRE(hipHostFree(host) == hipSuccess, "nfdpf_host_mapped_free: hipHostFree failed");
  return NFDPF_OK;
}


// The sharded gated pass's cross-rank gate exchange (include/nfdpf.h, filter_pass.hpp pass_gate):
// uncached device memory, so that granules a peer GPU stores over xGMI are read from memory by
// this GPU's polling loads, never from a stale L2 line.
static int xchg_fail(const char *what, hipError_t e) {
  (void)hipGetLastError();
  set_error("%s: %s", what, hipGetErrorString(e));
  return NFDPF_ELAUNCH;
}

extern "C" int64_t nfdpf_gate_xchg_bytes(int B_global) {
  return B_global <= 0 ? 0 : 256 + 2 * (int64_t)B_global * 8;
}

extern "C" int nfdpf_gate_xchg_alloc(int64_t bytes, void **dev, void *ipc_handle) {
  NFDPF_REQUIRE(bytes > 0 && dev && ipc_handle, "nfdpf_gate_xchg_alloc: bad arguments");
  *dev = nullptr;
  hipError_t e = hipExtMallocWithFlags(dev, (size_t)bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) {
    *dev = nullptr;
    return xchg_fail("nfdpf_gate_xchg_alloc (hipExtMallocWithFlags)", e);
  }
  hipIpcMemHandle_t h;
  if ((e = hipMemset(*dev, 0, (size_t)bytes)) != hipSuccess || (e = hipDeviceSynchronize()) != hipSuccess ||
      (e = hipIpcGetMemHandle(&h, *dev)) != hipSuccess) {
    (void)hipFree(*dev);
    *dev = nullptr;
    return xchg_fail("nfdpf_gate_xchg_alloc (hipIpcGetMemHandle)", e);
  }
  static_assert(sizeof(h) == 64, "hipIpcMemHandle_t is 64 bytes");
  memcpy(ipc_handle, &h, sizeof(h));
  return NFDPF_OK;
}

extern "C" int nfdpf_gate_xchg_open(const void *ipc_handle, void **dev) {
  NFDPF_REQUIRE(ipc_handle && dev, "nfdpf_gate_xchg_open: bad arguments");
  hipIpcMemHandle_t h;
  memcpy(&h, ipc_handle, sizeof(h));
  *dev = nullptr;
  const hipError_t e = hipIpcOpenMemHandle(dev, h, hipIpcMemLazyEnablePeerAccess);
  if (e != hipSuccess) {
    *dev = nullptr;
    return xchg_fail("nfdpf_gate_xchg_open (hipIpcOpenMemHandle)", e);
  }
  return NFDPF_OK;
}

extern "C" int nfdpf_gate_xchg_close(void *dev) {
  if (dev) NFDPF_REQUIRE(hipIpcCloseMemHandle(dev) == hipSuccess, "nfdpf_gate_xchg_close: hipIpcCloseMemHandle failed");
  return NFDPF_OK;
}

extern "C" int nfdpf_gate_xchg_free(void *dev) {
  if (dev) NFDPF_REQUIRE(hipFree(dev) == hipSuccess, "nfdpf_gate_xchg_free: hipFree failed");
  return NFDPF_OK;
}
