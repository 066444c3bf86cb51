// Experiment: tiled_finalize_kernel variants against a host reference (hand-built:
// hipcc --offload-arch=gfx950 -O3 scripts/exp_finalize.hip -o exp/fin_bench)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>
#include <vector>
__global__ void fin_naive(const double *__restrict__ fin, int BT, int tiles, float *__restrict__ pred,
                          float *__restrict__ lw_sum) {
  const int bt = blockIdx.x * blockDim.x + threadIdx.x;
  if (bt >= BT) return;
  double px = 0, py = 0, sw = 0;
  for (int k = 0; k < tiles; ++k) {
    const double *f = fin + ((int64_t)bt * tiles + k) * 4;
    px += f[1];
    py += f[2];
    sw += f[3];
  }
  pred[2 * bt] = (float)px;
  pred[2 * bt + 1] = (float)py;
  lw_sum[bt] = (float)sw;
}
__global__ void fin_unroll(const double *__restrict__ fin, int BT, int tiles, float *__restrict__ pred,
                           float *__restrict__ lw_sum) {
  const int bt = blockIdx.x * blockDim.x + threadIdx.x;
  if (bt >= BT) return;
  double px = 0, py = 0, sw = 0;
  for (int k0 = 0; k0 < tiles; k0 += 8) {
    double a[8][3];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const double *f = fin + ((int64_t)bt * tiles + k0 + j) * 4;
      a[j][0] = f[1];
      a[j][1] = f[2];
      a[j][2] = f[3];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      px += a[j][0];
      py += a[j][1];
      sw += a[j][2];
    }
  }
  pred[2 * bt] = (float)px;
  pred[2 * bt + 1] = (float)py;
  lw_sum[bt] = (float)sw;
}
int main() {
  const int BT = 48, tiles = 32;
  std::vector<double> h(BT * tiles * 4);
  for (size_t i = 0; i < h.size(); ++i) h[i] = std::sin(0.37 * i) * 10;
  double *d;
  float *p1, *p2, *l1, *l2;
  hipMalloc(&d, h.size() * 8);
  hipMalloc(&p1, BT * 8); hipMalloc(&p2, BT * 8); hipMalloc(&l1, BT * 4); hipMalloc(&l2, BT * 4);
  hipMemcpy(d, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  fin_naive<<<1, 256>>>(d, BT, tiles, p1, l1);
  fin_unroll<<<1, 256>>>(d, BT, tiles, p2, l2);
  std::vector<float> a(BT * 2), b(BT * 2);
  hipMemcpy(a.data(), p1, BT * 8, hipMemcpyDeviceToHost);
  hipMemcpy(b.data(), p2, BT * 8, hipMemcpyDeviceToHost);
  double md = 0;
  for (int i = 0; i < BT * 2; ++i) md = fmax(md, fabs(a[i] - b[i]));
  double ref = 0;
  for (int k = 0; k < tiles; ++k) ref += h[(0 * tiles + k) * 4 + 1];
  printf("naive %f unroll %f host %f maxdiff %g\n", a[0], b[0], ref, md);
  return 0;
}
