// measure.hip -- standalone measurement models behind nfdpf_measurement:
// cos (model/models.py:206-219), CRNVP (:256-278), NN (:221-235), gaussian (:237-254).
// One workgroup per batch row (the row max of CRNVP / gaussian is a row reduction).
#include "measure.hpp"

namespace nfdpf {

template <int BLK, int MEAS>
__global__ __launch_bounds__(BLK) void measurement_kernel(MeasArgs a, const float *__restrict__ enc,
                                                          const float *__restrict__ x, int N,
                                                          float *__restrict__ lik) {
  __shared__ StepShared L;
  const int b = blockIdx.x;
  measure_row_setup<MEAS>(enc + (int64_t)b * kE, a.meas_params, L);
  __syncthreads();
  float m = -INFINITY;
  for (int i = threadIdx.x; i < N; i += BLK) {
    const int64_t o = (int64_t)b * N + i;
    const float v = measure<MEAS>(a, L, x[2 * o], x[2 * o + 1]);
    lik[o] = v;
    m = fmaxf(m, v);
  }
  if (MEAS == NFDPF_MEAS_CRNVP || MEAS == NFDPF_MEAS_GAUSSIAN) {
    m = block_max(m, L.f);
    for (int i = threadIdx.x; i < N; i += BLK) lik[(int64_t)b * N + i] -= m;
  }
}

}  // namespace nfdpf

using namespace nfdpf;

extern "C" int nfdpf_measurement(int kind, const float *pe_params, const float *meas_params,
                                 int n_flows, const float *enc, const float *x, int B, int N,
                                 int E, float prior_std, float *lik, void *stream) {
  NFDPF_REQUIRE(pe_params && enc && x && lik, "nfdpf_measurement: null pointer");
  NFDPF_REQUIRE(B >= 0 && N >= 1, "nfdpf_measurement: bad sizes");
  NFDPF_REQUIRE(E == kE, "nfdpf_measurement: built for E = %d (got %d)", kE, E);
  NFDPF_REQUIRE(!(kind == NFDPF_MEAS_CRNVP || kind == NFDPF_MEAS_NN) || meas_params,
                "nfdpf_measurement: meas_params missing");
  NFDPF_REQUIRE(kind != NFDPF_MEAS_CRNVP || (n_flows >= 0 && prior_std > 0.f),
                "nfdpf_measurement: bad CRNVP arguments");
  if (B == 0) return NFDPF_OK;
  hipStream_t st = as_stream(stream);
  MeasArgs a{pe_params, meas_params, n_flows, prior_std};
  switch (kind) {
    case NFDPF_MEAS_COS:
      measurement_kernel<256, NFDPF_MEAS_COS><<<B, 256, 0, st>>>(a, enc, x, N, lik);
      break;
    case NFDPF_MEAS_CRNVP:
      measurement_kernel<256, NFDPF_MEAS_CRNVP><<<B, 256, 0, st>>>(a, enc, x, N, lik);
      break;
    case NFDPF_MEAS_NN:
      measurement_kernel<256, NFDPF_MEAS_NN><<<B, 256, 0, st>>>(a, enc, x, N, lik);
      break;
    case NFDPF_MEAS_GAUSSIAN:
      measurement_kernel<256, NFDPF_MEAS_GAUSSIAN><<<B, 256, 0, st>>>(a, enc, x, N, lik);
      break;
    default:
      set_error("nfdpf_measurement: unsupported kind %d", kind);
      return NFDPF_EINVAL;
  }
  return launch_status("nfdpf_measurement");
}
