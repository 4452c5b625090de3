// HBM write ceiling for evaluateRange's output (2.38 GB for 1e4 config-2 trajectories at dt = 0.01):
// how fast can MI355X write a buffer of that size with the store shapes the range kernel can use?
//   gs8 / gs16     grid-stride 8-B / 16-B stores, 2048 x 256 threads
//   wave8 / wave16 one 64-lane block per "trajectory" of 238 KB, coalesced 8-B / 16-B stores
//   wave16x4       the same, four independent 16-B stores per lane per iteration
//   memset         hipMemsetAsync
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/micro/write_bw scripts/micro/write_bw.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>

constexpr size_t kBytes = size_t(2380) << 20;
constexpr int kTraj = 10000;
constexpr size_t kPer = kBytes / kTraj / 64 * 64;  // bytes per trajectory, 64-B multiple

__global__ void gs8(double* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = 1.0;
}
__global__ void gs16(double2* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_double2(1.0, 2.0);
}
__global__ __launch_bounds__(64) void wave8(double* __restrict__ a, size_t per) {
  double* p = a + blockIdx.x * (per / 8);
  for (size_t i = threadIdx.x; i < per / 8; i += 64) p[i] = 1.0;
}
__global__ __launch_bounds__(64) void wave16(double2* __restrict__ a, size_t per) {
  double2* p = a + blockIdx.x * (per / 16);
  for (size_t i = threadIdx.x; i < per / 16; i += 64) p[i] = make_double2(1.0, 2.0);
}
__global__ __launch_bounds__(64) void wave16x4(double2* __restrict__ a, size_t per) {
  double2* p = a + blockIdx.x * (per / 16);
  const size_t n = per / 16;
  size_t i = threadIdx.x;
  for (; i + 192 < n; i += 256) {
    p[i] = make_double2(1.0, 2.0);
    p[i + 64] = make_double2(1.0, 2.0);
    p[i + 128] = make_double2(1.0, 2.0);
    p[i + 192] = make_double2(1.0, 2.0);
  }
  for (; i < n; i += 64) p[i] = make_double2(1.0, 2.0);
}
// 1024-thread blocks of contiguous trajectories: 16 waves per block share a CU
__global__ __launch_bounds__(256) void blk16(double2* __restrict__ a, size_t per) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  double2* p = a + (blockIdx.x * 4 + w) * (per / 16);
  for (size_t i = l; i < per / 16; i += 64) p[i] = make_double2(1.0, 2.0);
}

// evaluateRange's store pattern: per wave ("trajectory") 7448 samples in 128-sample blocks, each
// block 3 KB of rows (3 x 16-B pieces per lane) and 1 KB of sample times (2 x 8 B per lane), two
// streams per wave; FLOPS: plus 6 interleaved 18-deep f64 multiply-add chains per lane per block
// (the D = 3 Horner work, 108 f64 instructions)
constexpr int kSamples = 7448;
template <int FLOPS>
__global__ __launch_bounds__(64) void pat2(double* __restrict__ rows, double* __restrict__ st, double x0) {
  const int l = threadIdx.x;
  double2* rp = reinterpret_cast<double2*>(rows + (size_t)blockIdx.x * kSamples * 3);
  double* sp = st + (size_t)blockIdx.x * kSamples;
  for (int nb = 0; nb + 128 <= kSamples; nb += 128) {
    double v[6];
    const double t0 = x0 + nb + l, t1 = t0 + 64.0;
#pragma unroll
    for (int c = 0; c < 6; ++c) v[c] = (c < 3 ? t0 : t1) * 0.5;
    if (FLOPS) {
#pragma unroll
      for (int j = 0; j < 9; ++j)
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          v[c] = v[c] * (c < 3 ? t0 : t1);
          v[c] = v[c] + 0.25;
        }
    }
    sp[nb + l] = t0;
    sp[nb + 64 + l] = t1;
#pragma unroll
    for (int u = 0; u < 3; ++u) rp[nb * 3 / 2 + u * 64 + l] = make_double2(v[2 * u], v[2 * u + 1]);
  }
}

// the same with evaluateRange's spread of samples per trajectory (3300..11596, mean 7448, like the
// 1e4 config-2 batch's 3289..12229): trajectory b = order[block] has cnt[b] samples at offset off[b]
template <int FLOPS>
__global__ __launch_bounds__(64) void pat2v(double* __restrict__ rows, double* __restrict__ st, const int* __restrict__ cnt,
                                            const long long* __restrict__ off, const int* __restrict__ order, double x0) {
  const int l = threadIdx.x;
  const int b = order[blockIdx.x];
  const int n = cnt[b];
  const long long o = off[b] & ~1ll;  // (rows 16-B aligned)
  double2* rp = reinterpret_cast<double2*>(rows + o * 3);
  double* sp = st + o;
  for (int nb = 0; nb + 128 <= n; nb += 128) {
    double v[6];
    const double t0 = x0 + nb + l, t1 = t0 + 64.0;
#pragma unroll
    for (int c = 0; c < 6; ++c) v[c] = (c < 3 ? t0 : t1) * 0.5;
    if (FLOPS) {
#pragma unroll
      for (int j = 0; j < 9; ++j)
#pragma unroll
        for (int c = 0; c < 6; ++c) {
          v[c] = v[c] * (c < 3 ? t0 : t1);
          v[c] = v[c] + 0.25;
        }
    }
    sp[nb + l] = t0;
    sp[nb + 64 + l] = t1;
#pragma unroll
    for (int u = 0; u < 3; ++u) rp[nb * 3 / 2 + u * 64 + l] = make_double2(v[2 * u], v[2 * u + 1]);
  }
}

template <class F>
static float timeit(F f) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  f();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) f();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / 5;
}

int main() {
  double* a;
  if (hipMalloc(&a, kBytes) != hipSuccess) return 1;
  const size_t tot = kPer * kTraj;
  auto rep = [&](const char* name, float ms) {
    std::printf("%-10s %8.1f us  %6.2f TB/s\n", name, ms * 1e3, tot / (ms * 1e-3) / 1e12);
  };
  rep("gs8", timeit([&] { hipLaunchKernelGGL(gs8, dim3(2048), dim3(256), 0, 0, a, tot / 8); }));
  rep("gs16", timeit([&] { hipLaunchKernelGGL(gs16, dim3(2048), dim3(256), 0, 0, (double2*)a, tot / 16); }));
  rep("gs16_8k", timeit([&] { hipLaunchKernelGGL(gs16, dim3(8192), dim3(256), 0, 0, (double2*)a, tot / 16); }));
  rep("wave8", timeit([&] { hipLaunchKernelGGL(wave8, dim3(kTraj), dim3(64), 0, 0, a, kPer); }));
  rep("wave16", timeit([&] { hipLaunchKernelGGL(wave16, dim3(kTraj), dim3(64), 0, 0, (double2*)a, kPer); }));
  rep("wave16x4", timeit([&] { hipLaunchKernelGGL(wave16x4, dim3(kTraj), dim3(64), 0, 0, (double2*)a, kPer); }));
  rep("blk16", timeit([&] { hipLaunchKernelGGL(blk16, dim3(kTraj / 4), dim3(256), 0, 0, (double2*)a, kPer); }));
  {
    const size_t rows = (size_t)kTraj * kSamples * 3 * 8, sts = (size_t)kTraj * kSamples * 8;
    auto rep2 = [&](const char* name, float ms) {
      std::printf("%-10s %8.1f us  %6.2f TB/s\n", name, ms * 1e3, (rows + sts) / (ms * 1e-3) / 1e12);
    };
    if (rows + sts <= kBytes) {
      double* st = a + (size_t)kTraj * kSamples * 3;
      rep2("pat2", timeit([&] { hipLaunchKernelGGL(pat2<0>, dim3(kTraj), dim3(64), 0, 0, a, st, 1.0); }));
      rep2("pat2_flop", timeit([&] { hipLaunchKernelGGL(pat2<1>, dim3(kTraj), dim3(64), 0, 0, a, st, 1.0); }));
    }
  }
  {
    // variable samples per trajectory: index order, and longest first
    int h_cnt[kTraj], h_ord[kTraj], h_srt[kTraj];
    long long h_off[kTraj], acc = 0;
    for (int b = 0; b < kTraj; ++b) {
      h_cnt[b] = 3300 + (int)(((unsigned)b * 2654435761u >> 8) % 8296u);
      h_off[b] = acc;
      acc += h_cnt[b];
      h_ord[b] = b;
      h_srt[b] = b;
    }
    std::sort(h_srt, h_srt + kTraj, [&](int x, int y) { return h_cnt[x] > h_cnt[y]; });
    const size_t rows = (size_t)acc * 3 * 8, sts = (size_t)acc * 8;
    if (rows + sts + 64 <= kBytes) {
      int *d_cnt, *d_ord, *d_srt;
      long long* d_off;
      hipMalloc(&d_cnt, sizeof(h_cnt));
      hipMalloc(&d_ord, sizeof(h_ord));
      hipMalloc(&d_srt, sizeof(h_srt));
      hipMalloc(&d_off, sizeof(h_off));
      hipMemcpy(d_cnt, h_cnt, sizeof(h_cnt), hipMemcpyHostToDevice);
      hipMemcpy(d_ord, h_ord, sizeof(h_ord), hipMemcpyHostToDevice);
      hipMemcpy(d_srt, h_srt, sizeof(h_srt), hipMemcpyHostToDevice);
      hipMemcpy(d_off, h_off, sizeof(h_off), hipMemcpyHostToDevice);
      double* st = a + (size_t)acc * 3 + 2;
      auto rep3 = [&](const char* name, float ms) {
        std::printf("%-10s %8.1f us  %6.2f TB/s\n", name, ms * 1e3, (rows + sts) / (ms * 1e-3) / 1e12);
      };
      rep3("pat2v", timeit([&] { hipLaunchKernelGGL(pat2v<1>, dim3(kTraj), dim3(64), 0, 0, a, st, d_cnt, d_off, d_ord, 1.0); }));
      rep3("pat2v_lpt", timeit([&] { hipLaunchKernelGGL(pat2v<1>, dim3(kTraj), dim3(64), 0, 0, a, st, d_cnt, d_off, d_srt, 1.0); }));
    }
  }
  rep("memset", timeit([&] { hipMemsetAsync(a, 0, tot); }));
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  return 0;
}
