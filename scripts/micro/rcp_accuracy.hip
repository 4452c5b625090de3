// Accuracy of v_rcp_f64 (+ Newton steps) vs IEEE 1/x on gfx950: max error in ulps over random
// inputs spanning the pivot range of the solver.  hipcc --offload-arch=gfx950 -O3 rcp_accuracy.hip
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

__global__ void k(const double* x, double* r0, double* r1, double* r2, double* ref, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double a = x[i];
  double y = __builtin_amdgcn_rcp(a);
  r0[i] = y;
  double e = __builtin_fma(-a, y, 1.0);
  double y1 = __builtin_fma(y, e, y);
  r1[i] = y1;
  e = __builtin_fma(-a, y1, 1.0);
  r2[i] = __builtin_fma(y1, e, y1);
  ref[i] = 1.0 / a;
}

static double ulps(double a, double b) {
  int64_t ia, ib;
  memcpy(&ia, &a, 8);
  memcpy(&ib, &b, 8);
  return fabs((double)(ia - ib));
}

int main() {
  const int n = 1 << 22;
  double* h = (double*)malloc(n * sizeof(double) * 5);
  srand(1);
  for (int i = 0; i < n; ++i) {
    double m = 1.0 + (double)rand() / RAND_MAX;
    int e = rand() % 120 - 60;
    h[i] = ldexp(m, e) * ((rand() & 1) ? 1 : -1);
  }
  double* d;
  hipMalloc(&d, n * sizeof(double) * 5);
  hipMemcpy(d, h, n * sizeof(double), hipMemcpyHostToDevice);
  k<<<(n + 255) / 256, 256>>>(d, d + n, d + 2 * n, d + 3 * n, d + 4 * n, n);
  hipMemcpy(h, d, n * sizeof(double) * 5, hipMemcpyDeviceToHost);
  double m0 = 0, m1 = 0, m2 = 0, n2 = 0;
  for (int i = 0; i < n; ++i) {
    double ref = h[4 * n + i];
    m0 = fmax(m0, ulps(h[n + i], ref));
    m1 = fmax(m1, ulps(h[2 * n + i], ref));
    m2 = fmax(m2, ulps(h[3 * n + i], ref));
    n2 += h[3 * n + i] != ref;
  }
  printf("v_rcp_f64 max %.0f ulp | 1 Newton max %.0f ulp | 2 Newton max %.0f ulp (%.0f of %d differ from 1/x)\n",
         m0, m1, m2, n2, n);
  return 0;
}
