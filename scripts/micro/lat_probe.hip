// Latency probes on gfx950 (s_memtime cycles per dependent link, one wave alone):
//   fma   : v_fma_f64 chain
//   rcp   : v_rcp_f64 chain
//   lds   : ds_write_b64 -> s_waitcnt -> ds_read_b64 of another lane's slot (exchange round trip)
//   bar   : the same with __syncthreads (one-wave block)
//   bcast : ds_read_b64 of one address by all lanes -> dependent add (broadcast read latency)
// hipcc --offload-arch=gfx950 -O3 -o lat_probe lat_probe.hip
#include <hip/hip_runtime.h>
#include <stdio.h>

#define N_IT 256

__global__ void k_fma(double* out, double a, long long* cyc) {
  double x = threadIdx.x * 1e-3;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N_IT; ++i) {
    x = __builtin_fma(x, a, 0.5);
    asm volatile("" : "+v"(x));
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

__global__ void k_fma4(double* out, double a, long long* cyc) {  // 4 independent chains
  double x0 = threadIdx.x * 1e-3, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N_IT; ++i) {
    x0 = __builtin_fma(x0, a, 0.5);
    x1 = __builtin_fma(x1, a, 0.5);
    x2 = __builtin_fma(x2, a, 0.5);
    x3 = __builtin_fma(x3, a, 0.5);
    asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x0 + x1 + x2 + x3;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

__global__ void k_rcp(double* out, long long* cyc) {
  double x = 1.0 + threadIdx.x * 1e-3;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N_IT; ++i) {
    x = __builtin_amdgcn_rcp(x);
    asm volatile("" : "+v"(x));
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

__global__ void k_lds(double* out, int bar, long long* cyc) {
  __shared__ double s[64];
  double x = threadIdx.x * 1e-3;
  const int o = (threadIdx.x + 1) & 63;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N_IT; ++i) {
    s[threadIdx.x] = x;
    if (bar)
      __syncthreads();
    else
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    x = s[o] + 1.0;
    if (bar)
      __syncthreads();
    else
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

__global__ void k_bcast(double* out, long long* cyc) {
  __shared__ double s[64];
  s[threadIdx.x] = threadIdx.x;
  __syncthreads();
  double x = 0.0;
  int idx = 0;
  long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < N_IT; ++i) {
    x += s[idx];
    idx = ((int)x) & 7;  // address depends on the loaded value
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[threadIdx.x] = x;
  if (threadIdx.x == 0) *cyc = t1 - t0;
}

int main() {
  double* out;
  long long* cyc;
  hipMalloc(&out, 64 * sizeof(double));
  hipMallocManaged(&cyc, sizeof(long long));
  long long c;
  auto run = [&](const char* name, auto launch) {
    for (int r = 0; r < 3; ++r) launch();
    hipDeviceSynchronize();
    c = *cyc;
    printf("{\"probe\": \"%s\", \"cycles_per_link\": %.1f}\n", name, (double)c / N_IT);
  };
  run("fma_f64_chain", [&] { k_fma<<<1, 64>>>(out, 0.999, cyc); });
  run("fma_f64_4chains_per_iter", [&] { k_fma4<<<1, 64>>>(out, 0.999, cyc); });
  run("rcp_f64_chain", [&] { k_rcp<<<1, 64>>>(out, cyc); });
  run("lds_exchange_waitcnt", [&] { k_lds<<<1, 64>>>(out, 0, cyc); });
  run("lds_exchange_syncthreads", [&] { k_lds<<<1, 64>>>(out, 1, cyc); });
  run("lds_read_dependent", [&] { k_bcast<<<1, 64>>>(out, cyc); });
  return 0;
}
