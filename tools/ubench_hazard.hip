// Correctness probe for v_mfma_f64_16x16x4_f64 result hazards on gfx950.
// Each pattern is computed twice in one wave: "fast" = only the wait states the compiler inserts,
// "safe" = an s_sleep between the MFMA and its consumer.  Any mismatch means the consumer read a
// register before the MFMA wrote it (missing interlock / too few wait states).
// Result on MI355X (round 1): 0 mismatching lanes in every pattern -- reads of f64 MFMA results are safe
// with the compiler's wait states.  (Write-after-read on MFMA sources cannot be probed this way: an
// MFMA inside inline asm is invisible to the compiler's hazard recognizer, which breaks the probe.)
//   build: hipcc --offload-arch=gfx950 -O3 tools/ubench_hazard.hip -o tools/build/ubench_hazard
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); std::exit(1); } } while (0)

typedef double d4 __attribute__((ext_vector_type(4)));
constexpr int NP = 6;
static const char* names[NP] = {
    "mfma(srcC=0) -> VALU add of result",
    "mfma(srcC=0) -> v_readlane of result",
    "mfma(srcC=0) -> next mfma srcA",
    "2 independent mfma -> VALU add (the Riccati PA pattern)",
    "mfma(srcC=VALU value) -> VALU add",
    "mfma -> permlane16_swap of result",
};

__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

template <int P, bool SAFE>
__device__ __forceinline__ double pattern(double x, double y, double z) {
    const d4 Z = {0.0, 0.0, 0.0, 0.0};
    double r = 0.0;
    for (int it = 0; it < 8; ++it) {
        if constexpr (P == 0) {
            const d4 a = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, Z, 0, 0, 0);
            if (SAFE) __builtin_amdgcn_s_sleep(127);
            x = a[0] + a[1] + z;
        } else if constexpr (P == 1) {
            const d4 a = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, Z, 0, 0, 0);
            if (SAFE) __builtin_amdgcn_s_sleep(127);
            x = readlane_d(a[1], 21) * 1e-3 + x;
        } else if constexpr (P == 2) {
            const d4 a = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, Z, 0, 0, 0);
            if (SAFE) __builtin_amdgcn_s_sleep(127);
            const d4 b = __builtin_amdgcn_mfma_f64_16x16x4f64(a[0], z, Z, 0, 0, 0);
            if (SAFE) __builtin_amdgcn_s_sleep(127);
            x = b[0] * 1e-2 + b[1] * 1e-2 + x;
        } else if constexpr (P == 3) {
            const d4 a = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, Z, 0, 0, 0);
            const d4 b = __builtin_amdgcn_mfma_f64_16x16x4f64(z, y, Z, 0, 0, 0);
            if (SAFE) __builtin_amdgcn_s_sleep(127);
            x = (a[0] + b[0]) * 0.5 + (a[1] + b[1]) * 0.25;
        } else if constexpr (P == 4) {
            const d4 C = {x * z, y * z, 0.0, 0.0};
            const d4 a = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, C, 0, 0, 0);
            if (SAFE) __builtin_amdgcn_s_sleep(127);
            x = (a[0] - a[1]) * 0.5 + z;
        } else {
            const d4 a = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, Z, 0, 0, 0);
            if (SAFE) __builtin_amdgcn_s_sleep(127);
            const long long bb = __double_as_longlong(a[1]);
            const auto lo = __builtin_amdgcn_permlane16_swap((unsigned)(bb & 0xffffffffll), (unsigned)(bb & 0xffffffffll), false, false);
            const auto hi = __builtin_amdgcn_permlane16_swap((unsigned)(bb >> 32), (unsigned)(bb >> 32), false, false);
            x = __longlong_as_double(((long long)hi[0] << 32) | lo[0]) * 1e-2 + x;
        }
        x = x - floor(x);  // keep the values bounded
        r += x;
    }
    return r;
}

template <int P>
__global__ __launch_bounds__(64) void probe(const double* in, double* fast, double* safe) {
    const int l = threadIdx.x, b = blockIdx.x;
    const double x = in[b * 64 + l], y = in[(b * 64 + l + 7) % (gridDim.x * 64)] + 0.5, z = 0.25 + 0.01 * l;
    fast[b * 64 + l] = pattern<P, false>(x, y, z);
    safe[b * 64 + l] = pattern<P, true>(x, y, z);
}

typedef void (*KFn)(const double*, double*, double*);
static const KFn kernels[NP] = {probe<0>, probe<1>, probe<2>, probe<3>, probe<4>, probe<5>};

int main() {
    const int G = 1024, n = G * 64;
    double *in, *f, *s;
    CHECK(hipMalloc(&in, n * sizeof(double)));
    CHECK(hipMalloc(&f, n * sizeof(double)));
    CHECK(hipMalloc(&s, n * sizeof(double)));
    double* h = (double*)std::malloc(n * sizeof(double));
    double* hf = (double*)std::malloc(n * sizeof(double));
    double* hs = (double*)std::malloc(n * sizeof(double));
    unsigned long long st = 88172645463325252ull;
    for (int i = 0; i < n; ++i) {
        st ^= st << 13; st ^= st >> 7; st ^= st << 17;
        h[i] = (double)(st >> 11) / 9007199254740992.0;
    }
    CHECK(hipMemcpy(in, h, n * sizeof(double), hipMemcpyHostToDevice));
    int bad_total = 0;
    for (int p = 0; p < NP; ++p) {
        kernels[p]<<<G, 64>>>(in, f, s);
        CHECK(hipDeviceSynchronize());
        CHECK(hipMemcpy(hf, f, n * sizeof(double), hipMemcpyDeviceToHost));
        CHECK(hipMemcpy(hs, s, n * sizeof(double), hipMemcpyDeviceToHost));
        int bad = 0;
        for (int i = 0; i < n; ++i) bad += std::memcmp(&hf[i], &hs[i], sizeof(double)) != 0;
        bad_total += bad;
        std::printf("%-58s mismatching lanes %6d / %d\n", names[p], bad, n);
    }
    std::printf("TOTAL_MISMATCH %d\n", bad_total);
    return 0;
}
