// Calibrates rocprofv3 FETCH_SIZE / WRITE_SIZE for the access width track_kernel uses
// (MI355X_MICROARCH.md, HBM section: "other access widths are uncalibrated").
//
// track_kernel moves its inputs/outputs as coalesced 8-byte-per-lane global loads/stores,
// one 64-lane wave per workgroup.  This program runs the same pattern over known byte counts:
//   read8   : 1 GiB read, 8 B/lane  (plus 8 B per wave written)
//   write8  : 1 GiB written, 8 B/lane
//   read16  : 1 GiB read, 16 B/lane (the guide's calibrated case, as a control)
// Buffers are 4x the 256 MiB Infinity Cache, so nothing is served on-die.
// Usage: rocprofv3 --pmc FETCH_SIZE --kernel-trace -d DIR -o calib --output-format csv -- ./calib_fetch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

constexpr size_t kBytes = size_t(1) << 30;

__global__ __launch_bounds__(64) void read8(const double* __restrict__ a, double* __restrict__ out, size_t n) {
  double s = 0.0;
  for (size_t i = size_t(blockIdx.x) * 64 + threadIdx.x; i < n; i += size_t(gridDim.x) * 64) s += a[i];
  if (s == 12345.678) out[blockIdx.x * 64 + threadIdx.x] = s;  // never true for the zero fill
}

__global__ __launch_bounds__(64) void write8(double* __restrict__ a, size_t n) {
  for (size_t i = size_t(blockIdx.x) * 64 + threadIdx.x; i < n; i += size_t(gridDim.x) * 64) a[i] = double(i);
}

__global__ __launch_bounds__(64) void read16(const double2* __restrict__ a, double* __restrict__ out, size_t n) {
  double s = 0.0;
  for (size_t i = size_t(blockIdx.x) * 64 + threadIdx.x; i < n; i += size_t(gridDim.x) * 64) {
    double2 v = a[i];
    s += v.x + v.y;
  }
  if (s == 12345.678) out[blockIdx.x * 64 + threadIdx.x] = s;
}

int main() {
  double *a = nullptr, *out = nullptr;
  CHECK(hipMalloc(&a, kBytes));
  CHECK(hipMalloc(&out, size_t(1) << 24));
  CHECK(hipMemset(a, 0, kBytes));
  const int grid = 256 * 32;
  const size_t n = kBytes / 8;
  for (int r = 0; r < 3; ++r) {
    read8<<<grid, 64>>>(a, out, n);
    write8<<<grid, 64>>>(a, n);
    CHECK(hipMemset(a, 0, kBytes));
    read16<<<grid, 64>>>(reinterpret_cast<const double2*>(a), out, n / 2);
  }
  CHECK(hipDeviceSynchronize());
  std::printf("known bytes per dispatch: %zu (%.1f KB)\n", kBytes, kBytes / 1024.0);
  CHECK(hipFree(a));
  CHECK(hipFree(out));
  return 0;
}
