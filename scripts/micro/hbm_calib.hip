// HBM counter calibration: kernels that move a known number of bytes with the
// access widths of the solve kernels, for rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE.  The guide
// calibrates FETCH_SIZE only for 16-B-per-lane streaming reads (it reports half the bytes); the
// split path's workspace is 8 B per lane (ws[(v NE + e) B + b], trajectory index fastest).
//   read8   one double per lane, coalesced        (the split kernels' workspace reads)
//   read16  one double2 per lane, coalesced       (reference: the guide's calibrated case)
//   write8  one double per lane                   (the split kernels' workspace writes)
//   write16 one double2 per lane                  (the solve kernels' coefficient stores)
// Each kernel touches BYTES = 512 MiB (past the 256 MiB Infinity Cache), once per launch.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/micro/hbm_calib scripts/micro/hbm_calib.hip
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr size_t kBytes = size_t(512) << 20;

__global__ void read8(const double* __restrict__ a, double* __restrict__ out, size_t n) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) s += a[i];
  if (s == 1.2345) out[0] = s;  // never true for the zero-filled input: keeps the loads
}
__global__ void read16(const double2* __restrict__ a, double* __restrict__ out, size_t n) {
  double s = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 1.2345) out[0] = s;
}
__global__ void write8(double* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) a[i] = 1.0;
}
__global__ void write16(double2* __restrict__ a, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    a[i] = make_double2(1.0, 2.0);
}

int main() {
  double *a, *out;
  if (hipMalloc(&a, kBytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  if (hipMemset(a, 0, kBytes) != hipSuccess) return 1;
  const dim3 grid(256 * 8), block(256);
  for (int rep = 0; rep < 3; ++rep) {
    hipLaunchKernelGGL(read8, grid, block, 0, 0, a, out, kBytes / 8);
    hipLaunchKernelGGL(read16, grid, block, 0, 0, reinterpret_cast<const double2*>(a), out, kBytes / 16);
    hipLaunchKernelGGL(write8, grid, block, 0, 0, a, kBytes / 8);
    hipLaunchKernelGGL(write16, grid, block, 0, 0, reinterpret_cast<double2*>(a), kBytes / 16);
  }
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  std::printf("hbm_calib: %zu bytes per kernel launch\n", kBytes);
  return 0;
}
