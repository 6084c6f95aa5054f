// Accuracy of v_rcp_f64 + k Newton steps against IEEE 1/x (gfx950), over log-uniform x in [1e-12, 1e12].
//   build: hipcc --offload-arch=gfx950 -O3 tools/ubench_rcp.hip -o tools/build/ubench_rcp
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

__global__ void rcp_test(const double* x, double* r0, double* r1, double* r2, double* q, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    double r = __builtin_amdgcn_rcp(v);
    r0[i] = r;
    double e = fma(-v, r, 1.0);
    r = fma(r, e, r);
    r1[i] = r;
    e = fma(-v, r, 1.0);
    r = fma(r, e, r);
    r2[i] = r;
    q[i] = 1.0 / v;
}

static long long ulps(double a, double b) {
    long long ia, ib;
    std::memcpy(&ia, &a, 8);
    std::memcpy(&ib, &b, 8);
    return ia > ib ? ia - ib : ib - ia;
}

int main() {
    const int n = 1 << 22;
    double* h = (double*)std::malloc(n * 8);
    unsigned long long s = 0x9E3779B97F4A7C15ull;
    for (int i = 0; i < n; ++i) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        const double u = (double)(s >> 11) / 9007199254740992.0;
        h[i] = std::pow(10.0, -12.0 + 24.0 * u) * ((s & 1) ? -1.0 : 1.0);
    }
    double *dx, *a, *b, *c, *d;
    hipMalloc(&dx, n * 8); hipMalloc(&a, n * 8); hipMalloc(&b, n * 8); hipMalloc(&c, n * 8); hipMalloc(&d, n * 8);
    hipMemcpy(dx, h, n * 8, hipMemcpyHostToDevice);
    rcp_test<<<n / 256, 256>>>(dx, a, b, c, d, n);
    hipDeviceSynchronize();
    double *ha = (double*)std::malloc(n * 8), *hb = (double*)std::malloc(n * 8), *hc = (double*)std::malloc(n * 8);
    hipMemcpy(ha, a, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(hb, b, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(hc, c, n * 8, hipMemcpyDeviceToHost);
    long long m0 = 0, m1 = 0, m2 = 0, e1 = 0, e2 = 0;
    for (int i = 0; i < n; ++i) {
        const double ref = 1.0 / h[i];
        const long long u0 = ulps(ha[i], ref), u1 = ulps(hb[i], ref), u2 = ulps(hc[i], ref);
        m0 = u0 > m0 ? u0 : m0; m1 = u1 > m1 ? u1 : m1; m2 = u2 > m2 ? u2 : m2;
        e1 += u1 != 0; e2 += u2 != 0;
    }
    std::printf("v_rcp_f64 alone: max %lld ulp\n+1 Newton: max %lld ulp, inexact %lld / %d\n+2 Newton: max %lld ulp, inexact %lld / %d\n",
                m0, m1, e1, n, m2, e2, n);
    return 0;
}
