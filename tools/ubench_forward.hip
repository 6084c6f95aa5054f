// Microbenchmark (diagnostic, never shipped): cycles per stage of the tracking kernel's Newton forward sweep
// (tt_track.hip phase_forward, N = 20 unrolled) and of variants that change how x^_{k+1} reaches the lanes of the
// next stage.  One wave per workgroup (one wave per SIMD, as C2).  Every variant must write the stage records bit for
// bit as phase_forward does (the checksum column).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Icar-trailer-mpc_amd/csrc \
//         tools/ubench_forward.hip -o tools/bin/ubench_forward && tools/bin/ubench_forward
//
// V = 0  phase_forward as shipped: lane 8g + m holds Phi[g][m] x[m]; the group sum by three DPP adds; x^_{k+1}[m]
//        to lane (g, m) by one ds_bpermute from group m.
// V = 1  row per lane: lane g (g = lane & 7, eight copies) forms row g of [Phi; K^] itself and sums its seven
//        products in the DPP tree's order; x^_{k+1} becomes wave-uniform by v_readlane (SGPR operands next stage).
// V = 4  V = 1 with the next stage's operand loads issued first and their arithmetic after the exchange
//        (scheduling barriers), so that no wait for them sits on the chain.
// V = 2  V = 0's products and DPP sums, x^_{k+1} by v_readlane and a per-lane select instead of the ds_bpermute.
// V = 3  V = 0 without the exchange (x stays put): the floor of the products, sums, stores and prefetch.
#include "../car-trailer-mpc_amd/csrc/tt_track.hip"

#include <cstdio>
#include <vector>

namespace ttmpc {
namespace {

constexpr int UB_BM = kMaskMPC | kDiagBit;
constexpr int UB_N = 20;

template <int V>
__device__ __forceinline__ void ub_forward(const Ctx<UB_BM>& c, int crow, int bhrow, int orow) {
    constexpr int NS = UB_N;
    if constexpr (V == 0) {
        phase_forward<UB_BM, NS>(c, crow, bhrow, orow);
    } else if constexpr (V == 1 || V == 4) {
        const int g = c.lane & 7;
        const int u = (g == 5 || g == 6) ? 0 : (g == 4 || g == 7) ? 1 : -1;
        const double fkc = u >= 0 ? (g < 6 ? c.dt : 1.0) : 0.0;
        int fas[7], fk[7];
        double fone[7], fsg[7];
#pragma unroll
        for (int m = 0; m < 7; ++m) {
            fas[m] = (g < 6 && m < 6 && d_idx(g, m) >= 0) ? rAJ + d_idx(g, m)
                   : (m == 6 && (g == 4 || g == 5)) ? PAD
                   : (m == 6 && g == 6) ? SR + crow + 5 : (m == 6 && g == 7) ? SR + crow + 4
                   : (g < 6 && m == 6) ? bhrow + g : PAD;
            fsg[m] = (m == 6 && g >= 6) ? 1.0 / c.dt : 1.0;
            fk[m] = (u >= 0 && m < 6) ? rK + 6 * u + m : (u >= 0 && m == 6) ? rKF + u : PAD;
            fone[m] = (g < 6 && m == g) ? 1.0 : 0.0;
        }
        double x[6];
#pragma unroll
        for (int m = 0; m < 6; ++m) x[m] = -c.r(crow + m, 0);
        if (c.lane < 6) c.r(orow + c.lane, 0) = -c.r(crow + c.lane, 0);
        const int fst = c.lane < 8 ? (g < 6 ? SR + orow + g : orow + g) : rHD + (g % 6);
        double ph[7];
#pragma unroll
        for (int m = 0; m < 7; ++m) ph[m] = fma(fkc, c.r(fk[m], 0), fma(fsg[m], c.r(fas[m], 0), fone[m]));
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            double cur[7];
#pragma unroll
            for (int m = 0; m < 7; ++m) cur[m] = ph[m];
            const int kn = k + 1 < NS ? k + 1 : k;
            double la[7], lb[7];
#pragma unroll
            for (int m = 0; m < 7; ++m) { la[m] = c.r(fas[m], kn); lb[m] = c.r(fk[m], kn); }
            if constexpr (V == 4) __builtin_amdgcn_sched_barrier(0);
            double y;
            {
#pragma clang fp contract(off)
                const double y0 = cur[0] * x[0], y1 = cur[1] * x[1], y2 = cur[2] * x[2], y3 = cur[3] * x[3];
                const double y4 = cur[4] * x[4], y5 = cur[5] * x[5];
                y = ((y0 + y1) + (y2 + y3)) + ((y4 + y5) + (cur[6] + 0.0));
            }
            c.sm[HEAD + k * SR + fst] = y;
#pragma unroll
            for (int m = 0; m < 6; ++m) x[m] = readlane_d(y, m);
            if constexpr (V == 4) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int m = 0; m < 7; ++m) ph[m] = fma(fkc, lb[m], fma(fsg[m], la[m], fone[m]));
        }
        __syncthreads();
    } else {
        // V = 2 / 3: phase_forward's body with the exchange replaced (2) or dropped (3)
        const int N = c.N, g = c.lane >> 3, mm = c.lane & 7;
        const int u = (g == 5 || g == 6) ? 0 : (g == 4 || g == 7) ? 1 : -1;
        const double fone = (g < 6 && mm == g) ? 1.0 : 0.0;
        const bool shf = mm == 6;
        const int fas = (g < 6 && mm < 6 && d_idx(g, mm) >= 0) ? rAJ + d_idx(g, mm)
                      : (shf && (g == 4 || g == 5)) ? PAD
                      : (shf && g == 6) ? SR + crow + 5 : (shf && g == 7) ? SR + crow + 4
                      : (g < 6 && mm == 6) ? bhrow + g : PAD;
        const double fsg = (shf && g >= 6) ? 1.0 / c.dt : 1.0;
        const int fk = (u >= 0 && mm < 6) ? rK + 6 * u + mm : (u >= 0 && mm == 6) ? rKF + u : PAD;
        const double fkc = u >= 0 ? (g < 6 ? c.dt : 1.0) : 0.0;
        double x = mm < 6 ? -c.r(crow + mm, 0) : (mm == 6 ? 1.0 : 0.0);
        if (c.lane < 6) c.r(orow + c.lane, 0) = -c.r(crow + c.lane, 0);
        double nph = fone + fsg * c.r(fas, 0) + fkc * c.r(fk, 0);
        const int fst = mm == 0 ? (g < 6 ? SR + orow + g : orow + g) : rHD + (g % 6);
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            const double ph = nph;
            const int kn = k + 1 < N ? k + 1 : k;
            nph = fone + fsg * c.r(fas, kn) + fkc * c.r(fk, kn);
            double y = ph * x;
            y += dppd<0xB1>(y);
            y += dppd<0x4E>(y);
            y += dppd<0x141>(y);
            c.sm[HEAD + k * SR + fst] = y;
            if constexpr (V == 2) {
                const double x0 = readlane_d(y, 0), x1 = readlane_d(y, 8), x2 = readlane_d(y, 16);
                const double x3 = readlane_d(y, 24), x4 = readlane_d(y, 32), x5 = readlane_d(y, 40);
                double xn = x0;
                xn = mm == 1 ? x1 : xn;
                xn = mm == 2 ? x2 : xn;
                xn = mm == 3 ? x3 : xn;
                xn = mm == 4 ? x4 : xn;
                xn = mm == 5 ? x5 : xn;
                x = mm < 6 ? xn : (mm == 6 ? 1.0 : 0.0);
            } else {
                x = mm < 6 ? y : (mm == 6 ? 1.0 : 0.0);
            }
        }
        __syncthreads();
    }
}

template <int V>
__global__ __launch_bounds__(64) void ub_kernel(int reps, unsigned long long* out) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    Ctx<UB_BM> c;
    c.sm = sm;
    c.N = UB_N;
    c.lane = threadIdx.x;
    c.dt = 0.05;
    const int total = SR * (UB_N + 1) + kScratch;
    for (int t = c.lane; t < total; t += 64) sm[t] = 1e-2 * (double)((t * 37 + blockIdx.x) % 97) - 0.4;
    __syncthreads();
    for (int k = 0; k <= UB_N; ++k)
        if (c.lane == 0) sm[HEAD + k * SR + PAD] = 0.0;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        ub_forward<V>(c, rCC, rBH, rDX);
        // the sweep's output feeds the next repetition's residual rows, so no repetition is dead code
        if (c.lane < 6) sm[HEAD + rCC + c.lane] = 0.5 * sm[HEAD + UB_N * SR + rDX + c.lane];
        __syncthreads();
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (c.lane == 0) out[blockIdx.x] = t1 - t0;
    // checksum of the rows the sweeps wrote (V = 3 differs by construction)
    double cs = 0.0;
    for (int k = 0; k <= UB_N; ++k)
        for (int q = c.lane; q < 8; q += 64) cs += sm[HEAD + k * SR + rDX + q] * (double)(1 + (k * 8 + q) % 13);
    cs = wsum(cs);
    if (c.lane == 0) out[gridDim.x + blockIdx.x] = (unsigned long long)__double_as_longlong(cs);
}

std::vector<unsigned long long> g_ref;  // the shipped phase's checksums (set by its run)

template <int V>
void run(const char* name, int B = 1024) {
    const int reps = 200;
    unsigned long long* d_out;
    (void)hipMalloc(&d_out, 2 * B * sizeof(unsigned long long));
    const int bytes = 8 * (SR * (UB_N + 1) + kScratch);
    hipLaunchKernelGGL(ub_kernel<V>, dim3(B), dim3(64), bytes, 0, reps, d_out);  // warm-up
    hipLaunchKernelGGL(ub_kernel<V>, dim3(B), dim3(64), bytes, 0, reps, d_out);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(2 * B);
    (void)hipMemcpy(h.data(), d_out, 2 * B * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double s = 0;
    for (int b = 0; b < B; ++b) s += (double)h[b];
    std::vector<unsigned long long>& ref = g_ref;  // one reference for every instantiation of run<V>
    if (V == 0) ref.assign(h.begin() + B, h.end());
    int diff = 0;
    for (int b = 0; b < B && b < (int)ref.size(); ++b) diff += h[B + b] != ref[b];
    printf("[records vs phase_forward: %4d of %d instances differ] %-52s B=%5d %8.2f ticks/stage\n", diff, B, name, B,
           s / B / reps / UB_N);
    (void)hipFree(d_out);
}

}  // namespace
}  // namespace ttmpc

int main() {
    using namespace ttmpc;
    for (int rep = 0; rep < 2; ++rep) {
        run<0>("phase_forward<N=20> (DPP sums, ds_bpermute)");
        run<1>("row per lane, uniform x by v_readlane");
        run<2>("DPP sums, v_readlane + select");
        run<3>("DPP sums, no exchange (floor)");
        run<4>("row per lane, loads first, arithmetic last");
    }
    run<0>("phase_forward<N=20> B=256", 256);
    run<1>("row per lane B=256", 256);
    run<4>("row per lane, loads first B=256", 256);
    return 0;
}
