// Semantics check of the 64-bit DPP broadcast used by the OBCA correction sweep (riccati_vec): lane t of the
// output holds the value of lane rowbc_src(t) of the input.  usage: ./ubench_dpp64  (prints the source lane per lane)
#include <hip/hip_runtime.h>
#include <cstdio>
template <int L_>
__device__ __forceinline__ double rowbc(double v) {
    const long long b = __double_as_longlong(v);
    return __longlong_as_double(__builtin_amdgcn_update_dpp(b, b, 0x150 + L_, 0xF, 0xF, false));
}
__global__ void k(double* out) {
    const double v = 1000.0 + threadIdx.x;
    out[threadIdx.x] = rowbc<0>(v);
    out[64 + threadIdx.x] = rowbc<3>(v);
    out[128 + threadIdx.x] = rowbc<5>(v);
}
int main() {
    double* d;
    double h[192];
    if (hipMalloc(&d, sizeof(h)) != hipSuccess) return 1;
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
    if (hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost) != hipSuccess) return 1;
    for (int r = 0; r < 3; ++r) {
        printf("rowbc<%d>:", r == 0 ? 0 : r == 1 ? 3 : 5);
        for (int t = 0; t < 64; ++t) printf(" %d", (int)(h[64 * r + t] - 1000.0));
        printf("\n");
    }
    return 0;
}
