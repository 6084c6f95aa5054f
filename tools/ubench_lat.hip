// Single-wave latency microbenchmarks for the f64 instruction mix of track_kernel (gfx950).
// Each test runs a dependent chain of R links inside one wave and reports s_memtime cycles per link.
//   build: hipcc --offload-arch=gfx950 -O3 tools/ubench_lat.hip -o tools/build/ubench_lat
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int R = 256;
enum { T_MFMA_C, T_MFMA_AB, T_MFMA_IND4, T_FMA, T_FMA_IND4, T_RCP, T_READLANE, T_PERM, T_DS, T_MFMA_READLANE,
       T_DPP, T_SINCOS, T_BPERM, T_LOG, T_DIV, NT };
static const char* names[NT] = {
    "mfma_f64_16x16x4 dependent via srcC (accumulate chain)",
    "mfma_f64_16x16x4 result -> next srcA/srcB (operand chain)",
    "mfma_f64_16x16x4 4 independent accumulators (throughput / link)",
    "v_fma_f64 dependent chain",
    "v_fma_f64 4 independent chains (per link of each)",
    "v_rcp_f64 dependent chain",
    "v_fma_f64 -> v_readlane -> s-operand v_fma_f64 (per link)",
    "v_permlane16_swap x2 (b64) -> v_add_f64 (per link)",
    "ds_write_b64 -> ds_read_b64 -> v_add_f64 (per link)",
    "mfma -> accvgpr/readlane -> v_fma as next srcA (per link)",
    "DPP row op (b64 as 2x32) -> v_add_f64 (per link)",
    "sincos(double) -> v_fma_f64 (per link)",
    "ds_bpermute_b32 x2 (b64, lane+3) -> v_add_f64 (per link)",
    "log(double) -> v_add_f64 (per link)",
    "IEEE 1.0 / x (double) (per link)",
};

__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

__global__ __launch_bounds__(64) void lat(int test, double seed, double* out, unsigned long long* cyc) {
    __shared__ double sm[64 * 4];
    const int lane = threadIdx.x;
    double x = seed + lane * 1e-3, y = x * 0.5, z = x * 0.25, w = x * 0.125;
    d4 acc = {x, y, z, w}, a1 = acc, a2 = acc, a3 = acc;
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    switch (test) {
        case T_MFMA_C:
            for (int r = 0; r < R; ++r) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
            x = acc[0] + acc[3];
            break;
        case T_MFMA_AB:
            for (int r = 0; r < R; ++r) {
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
                x = acc[1];
            }
            x += acc[0];
            break;
        case T_MFMA_IND4:
            for (int r = 0; r < R; ++r) {
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
                a1 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, z, a1, 0, 0, 0);
                a2 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, z, a2, 0, 0, 0);
                a3 = __builtin_amdgcn_mfma_f64_16x16x4f64(w, z, a3, 0, 0, 0);
            }
            x = acc[0] + a1[1] + a2[2] + a3[3];
            break;
        case T_FMA:
            for (int r = 0; r < R; ++r) x = fma(x, y, z);
            break;
        case T_FMA_IND4:
            for (int r = 0; r < R; ++r) { x = fma(x, y, z); w = fma(w, y, z); a1[0] = fma(a1[0], y, z); a2[0] = fma(a2[0], y, z); }
            x += w + a1[0] + a2[0];
            break;
        case T_RCP:
            for (int r = 0; r < R; ++r) x = __builtin_amdgcn_rcp(x);
            break;
        case T_READLANE:
            for (int r = 0; r < R; ++r) { const double s = readlane_d(x, 5); x = fma(s, y, z); }
            break;
        case T_PERM:
            for (int r = 0; r < R; ++r) {
                const long long b = __double_as_longlong(x);
                const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)(b & 0xffffffffll), (unsigned)(b & 0xffffffffll), false, false);
                const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(b >> 32), (unsigned)(b >> 32), false, false);
                x = __longlong_as_double(((long long)hi[0] << 32) | lo[0]) + y;
            }
            break;
        case T_DS:
            for (int r = 0; r < R; ++r) {
                sm[lane + 64 * (r & 3)] = x;
                __builtin_amdgcn_wave_barrier();
                x = sm[(lane ^ 1) + 64 * (r & 3)] + y;
            }
            break;
        case T_MFMA_READLANE:
            for (int r = 0; r < R; ++r) {
                acc = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, acc, 0, 0, 0);
                x = fma(readlane_d(acc[1], 21), z, acc[0]);
            }
            break;
        case T_DPP:
            for (int r = 0; r < R; ++r) {
                const long long b = __double_as_longlong(x);
                const int lo = __builtin_amdgcn_update_dpp((int)(b & 0xffffffffll), (int)(b & 0xffffffffll), 0x141, 0xF, 0xF, false);
                const int hi = __builtin_amdgcn_update_dpp((int)(b >> 32), (int)(b >> 32), 0x141, 0xF, 0xF, false);
                x = __longlong_as_double(((long long)hi << 32) | (unsigned int)lo) + y;
            }
            break;
        case T_SINCOS:
            for (int r = 0; r < R; ++r) { double sn, cs; sincos(x, &sn, &cs); x = fma(cs, 1e-3, sn) + y; }
            break;
        case T_BPERM:
            for (int r = 0; r < R; ++r) {
                const long long b = __double_as_longlong(x);
                const int src = ((lane + 3) & 63) << 2;
                const int lo = __builtin_amdgcn_ds_bpermute(src, (int)(b & 0xffffffffll));
                const int hi = __builtin_amdgcn_ds_bpermute(src, (int)(b >> 32));
                x = __longlong_as_double(((long long)hi << 32) | (unsigned int)lo) + y;
            }
            break;
        case T_LOG:
            for (int r = 0; r < R; ++r) x = log(x) + 1.5;
            break;
        case T_DIV:
            for (int r = 0; r < R; ++r) x = 1.0 / x + y;
            break;
    }
    __builtin_amdgcn_s_waitcnt(0);
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + lane] = x;
    if (lane == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
    double* out;
    unsigned long long* cyc;
    CHECK(hipMalloc(&out, 64 * sizeof(double) * 1024));
    CHECK(hipMalloc(&cyc, 1024 * sizeof(unsigned long long)));
    for (int t = 0; t < NT; ++t) {
        unsigned long long h[1];
        double best = 1e30;
        for (int rep = 0; rep < 5; ++rep) {
            lat<<<1, 64>>>(t, 1.0001, out, cyc);
            CHECK(hipDeviceSynchronize());
            CHECK(hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost));
            const double per = (double)h[0] / R;
            if (per < best) best = per;
        }
        std::printf("%-66s %8.1f cyc/link\n", names[t], best);
    }
    // the same MFMA chain with one wave on every SIMD of the chip (1024 waves): does it stay latency-bound?
    unsigned long long hs[1024];
    lat<<<1024, 64>>>(T_MFMA_C, 1.0001, out, cyc);
    CHECK(hipDeviceSynchronize());
    CHECK(hipMemcpy(hs, cyc, sizeof(hs), hipMemcpyDeviceToHost));
    double s = 0;
    for (int i = 0; i < 1024; ++i) s += hs[i];
    std::printf("%-66s %8.1f cyc/link\n", "mfma srcC chain, 1024 waves (mean)", s / 1024 / R);
    return 0;
}
