// Dependent-chain latency on gfx950 (cycles per link, s_memtime): v_add_f64 alone, and the
// evaluateRange clock step (compare + select + add).  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>
#include <stdio.h>

__global__ void k_add(double* out, double dt, int n, long long* cyc) {
  double t = threadIdx.x * 1e-3;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    t += dt;
    asm volatile("" : "+v"(t));
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = t;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

__global__ void k_step(double* out, double dt, double Ti, int n, long long* cyc) {
  double t = threadIdx.x * 1e-3, a = 0.0;
  long long c = 0;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
    const bool go = !(t > Ti);
    c += go;
    t = go ? t + dt : t - Ti;
    a = go ? a + dt : a;
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = t + a + c;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  double* o;
  long long* c;
  hipMalloc(&o, 64 * sizeof(double));
  hipMalloc(&c, sizeof(long long));
  const int n = 1 << 16;
  long long h;
  for (int rep = 0; rep < 2; ++rep) {
    k_add<<<1, 64>>>(o, 0.01, n, c);
    hipMemcpy(&h, c, sizeof(h), hipMemcpyDeviceToHost);
    if (rep) printf("dependent v_add_f64: %.2f cycles/link\n", (double)h / n);
    k_step<<<1, 64>>>(o, 0.01, 7.5, n, c);
    hipMemcpy(&h, c, sizeof(h), hipMemcpyDeviceToHost);
    if (rep) printf("clock step (cmp+select+add): %.2f cycles/step\n", (double)h / n);
  }
  return 0;
}
