// Bitwise check of tt_trig.hpp's straight-line sincos and tan / cos against the device library's on gfx950 (diagnostic, GPU
// box): random arguments over several magnitude ranges, arguments next to multiples of pi/4, and special values.
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -I car-trailer-mpc_amd/csrc tools/trig_check.hip -o tools/trig_check
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include "tt_trig.hpp"

__device__ unsigned long long mix(unsigned long long z) {
    z += 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

__global__ void check(unsigned long long n, unsigned long long* bad, double* first) {
    const unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const unsigned long long r = mix(i);
    const int kind = (int)(i % 6);
    const double u = (double)(r >> 11) * 0x1.0p-53;  // [0, 1)
    double x;
    if (kind == 0) x = (2.0 * u - 1.0) * 4.0;                  // the kernels' angles
    else if (kind == 1) x = (2.0 * u - 1.0) * 100.0;
    else if (kind == 2) x = (2.0 * u - 1.0) * 1.0e6;
    else if (kind == 3) x = (2.0 * u - 1.0) * 1073741823.0;    // up to the fast path's bound
    else if (kind == 4) {                                      // next to k pi/4
        const double k = (double)((long long)(r % 2000001ull) - 1000000);
        x = k * 0.78539816339744830962 + (double)((long long)((r >> 24) % 2001) - 1000) * 1e-16 * fmax(1.0, fabs(k));
    } else {                                                   // tiny and subnormal magnitudes
        x = ldexp(2.0 * u - 1.0, -(int)((r >> 40) % 1070));
    }
    double s0, c0, s1, c1, t1, c2;
    sincos(x, &s0, &c0);
    ttmpc::sincos_small(x, s1, c1);
    const double t0 = tan(x), c3 = cos(x);
    ttmpc::tancos_small(x, t1, c2);
    if (__double_as_longlong(s0) != __double_as_longlong(s1) || __double_as_longlong(c0) != __double_as_longlong(c1)) {
        if (atomicAdd(bad, 1ull) == 0ull) { first[0] = x; first[1] = s0; first[2] = s1; first[3] = c0; first[4] = c1; }
    }
    if (__double_as_longlong(t0) != __double_as_longlong(t1) || __double_as_longlong(c3) != __double_as_longlong(c2)) {
        if (atomicAdd(bad + 1, 1ull) == 0ull) { first[5] = x; first[6] = t0; first[7] = t1; first[8] = c3; first[9] = c2; }
    }
}

int main(int argc, char** argv) {
    const unsigned long long n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (1ull << 28);
    unsigned long long* bad;
    double* first;
    if (hipMalloc(&bad, 16) != hipSuccess || hipMalloc(&first, 10 * 8) != hipSuccess) return 2;
    if (hipMemset(bad, 0, 16) != hipSuccess || hipMemset(first, 0, 80) != hipSuccess) return 2;
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(check, dim3(blocks), dim3(256), 0, 0, n, bad, first);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 2; }
    unsigned long long hb[2] = {0, 0};
    double hf[10];
    if (hipMemcpy(hb, bad, 16, hipMemcpyDeviceToHost) != hipSuccess || hipMemcpy(hf, first, 80, hipMemcpyDeviceToHost) != hipSuccess)
        return 2;
    printf("sincos_small vs library sincos: %llu arguments, %llu bitwise mismatches\n", n, hb[0]);
    printf("tancos_small vs library tan, cos: %llu arguments, %llu bitwise mismatches\n", n, hb[1]);
    if (hb[0]) printf("first: x=%.17g sin %.17g vs %.17g, cos %.17g vs %.17g\n", hf[0], hf[1], hf[2], hf[3], hf[4]);
    if (hb[1]) printf("first: x=%.17g tan %.17g vs %.17g, cos %.17g vs %.17g\n", hf[5], hf[6], hf[7], hf[8], hf[9]);
    return hb[0] || hb[1] ? 1 : 0;
}
