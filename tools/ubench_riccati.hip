// Microbenchmark (diagnostic, never shipped): cycles per stage of the tracking kernel's Riccati stage
// loop (tt_track.hip phase_riccati, N = 20 unrolled) and of variants that drop one ingredient, to find
// what sets the per-stage latency.  One wave per workgroup, 1024 workgroups (one wave per SIMD, as C2).
//
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Iinclude -Icar-trailer-mpc_amd/csrc \
//         tools/ubench_riccati.hip -o tools/ubench_riccati && tools/ubench_riccati
#include "../car-trailer-mpc_amd/csrc/tt_track.hip"

#include <cstdio>
#include <vector>

namespace ttmpc {
namespace {

constexpr int UB_BM = kMaskMPC | kDiagBit;
constexpr int UB_N = 20;

// V: 0 = as shipped; 1 = no next-stage prefetch (operands reused); 2 = no factor-row stores;
//    3 = no PA tile round trip (column from the lane's own PA); 4 = no P tile round trip (row from
//    registers); 5 = 1 + 2; 6 = no reciprocal of det
template <int V>
__device__ __forceinline__ bool ub_riccati(const Ctx<UB_BM>& c, double dw) {
    constexpr int NS = UB_N;
    const int N = c.N, i = c.lane >> 3, j = c.lane & 7;
    EpMap m;
    m.init(i, j, c.sm + hQW);
    const double dt = c.dt, dt2 = dt * dt;
    const double r00 = 2.0 * c.h(hRW), r01 = 2.0 * c.h(hRW + 1), r11 = 2.0 * c.h(hRW + 3);
    double* PF = c.sm + hPF;
    double* PT = c.sm + hPT;
    double Pij = m.q2 + m.dg * dw + c.r(m.hs, N);
    PF[c.lane] = Pij;
    asm volatile("" ::: "memory");
    bool pd = true;
    // V7 store map: one row per lane; every lane without an entry of its own rewrites the (uniform) i11
    const bool own_p = i < 6 && j < 7 && (j == 6 || i <= j);
    const bool stv_ih = i < 6 && !own_p;
    const int st_row = own_p ? (j < 6 ? rPS + sym_idx(i, j) : rPV + i)
                     : stv_ih ? rIH + 2
                     : j < 6 ? rK + 6 * (i - 6) + j : j == 6 ? rKF + (i - 6) : rIH + (i - 6);
    auto stage = [&](int k, const EpOps& o, EpOps& nx, int kn) {
        double2 r01v, r23v, r45v, p5;
        double p44;
        if constexpr (V == 4) {
            r01v = make_double2(Pij, Pij * 0.5); r23v = make_double2(Pij * 0.25, Pij); r45v = r01v; p5 = r23v; p44 = Pij;
        } else {
            r01v = ld2(PF + 8 * i); r23v = ld2(PF + 8 * i + 2); r45v = ld2(PF + 8 * i + 4);
            p5 = ld2(PF + 44); p44 = PF[36];
        }
        const double h00 = r00 + o.sgu0 + dw + dt2 * p5.y, h01 = r01 + dt2 * p5.x, h11 = r11 + o.sgu1 + dw + dt2 * p44;
        const double det = h00 * h11 - h01 * h01;
        pd = pd & (h00 > 0.0) & (h11 > 0.0) & (det > 1e-13 * h00 * h11);
        const double id = V == 6 ? det * 1e-3 : frcp(det), i00 = h11 * id, i01 = -h01 * id, i11 = h00 * id;
        double pa = fma(r01v.x, o.dj[0], Pij), pb = r01v.y * o.dj[1];
        pa = fma(r23v.x, o.dj[2], pa);
        pb = fma(r23v.y, o.dj[3], pb);
        pa = fma(r45v.x, o.dj[4], pa);
        pb = fma(r45v.y, o.dj[5], pb);
        const double PAij = pa + pb;
        double2 c01, c23, c45, gi;
        if constexpr (V == 3) {
            c01 = make_double2(PAij, PAij * 0.5); c23 = c01; c45 = make_double2(PAij * 0.25, PAij); gi = c45;
        } else {
            PT[8 * j + i] = PAij;
            asm volatile("" ::: "memory");
            c01 = ld2(PT + 8 * j); c23 = ld2(PT + 8 * j + 2); c45 = ld2(PT + 8 * j + 4);
            gi = ld2(PT + 8 * i + 4);
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (V != 1 && V != 5) nx = ep_ops(c, m, kn, dw);
        else nx = o;
        double fa = fma(o.di[0], c01.x, PAij + o.h), fb = o.di[1] * c01.y;
        fa = fma(o.di[2], c23.x, fa);
        fb = fma(o.di[3], c23.y, fb);
        fa = fma(o.di[4], c45.x, fa);
        fb = fma(o.di[5], c45.y, fb);
        const double F = fa + fb;
        const double g0j = fma(dt, c45.y, o.gj0), g1j = fma(dt, c45.x, o.gj1);
        const double g0i = fma(dt, gi.y, o.gi0), g1i = fma(dt, gi.x, o.gi1);
        const double m0 = fma(i00, g0j, i01 * g1j), m1 = fma(i01, g0j, i11 * g1j);
        Pij = F - fma(g0i, m0, g1i * m1);
        if constexpr (V != 4) {
            PF[c.lane] = Pij;
            asm volatile("" ::: "memory");
        }
        if constexpr (V == 7) {
            // one unmasked store per lane: P entries on rows i < 6 (the lower triangle rewrites its
            // bitwise-equal mirror), K rows on lanes i = 6, 7 (j < 7), the 2x2 inverse on (6,7), (7,7), (1,0)
            const double v = i < 6 ? (stv_ih ? i11 : Pij) : j < 7 ? (i == 6 ? -m0 : -m1) : (i == 6 ? i00 : i01);
            c.sm[HEAD + k * SR + st_row] = v;
        } else if constexpr (V != 2 && V != 5) {
            mstore(c, i < 2 && j < 7, j < 6 ? rK + 6 * i + j : rKF + i, k, i == 0 ? -m0 : -m1);
            mstore(c, c.lane < 3, rIH + c.lane, k, c.lane == 0 ? i00 : c.lane == 1 ? i01 : i11);
            mstore(c, m.ps >= 0, m.ps, k, Pij);
        }
    };
    EpOps oa = ep_ops(c, m, N - 1, dw), ob;
#pragma unroll
    for (int k = NS - 1; k >= 1; k -= 2) {
        stage(k, oa, ob, k - 1);
        stage(k - 1, ob, oa, k >= 2 ? k - 2 : 0);
    }
    if (V == 4) c.sm[hDUMP + (c.lane & 31)] = Pij;  // keep the chain alive
    return pd;
}

template <int V>
__global__ __launch_bounds__(64) void ub_kernel(int reps, unsigned long long* out, int* bad) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    Ctx<UB_BM> c;
    c.sm = sm;
    c.N = UB_N;
    c.lane = threadIdx.x;
    c.dt = 0.05;
    c.iL1 = 1.0 / 7.05;
    c.iL2 = 1.0 / 12.45;
    c.Mh = 0.15;
    c.mu = 0.1;
    c.tau = 0.99;
    const int total = kRowsPerStage * (UB_N + 1) + kScratch;
    for (int t = c.lane; t < total; t += 64) sm[t] = 1e-3 * (double)((t * 37 + blockIdx.x) % 97);
    __syncthreads();
    if (c.lane < 36) sm[hQW + c.lane] = (c.lane % 7 == 0) ? 1.0 : 0.0;
    if (c.lane < 4) sm[hRW + c.lane] = (c.lane == 0 || c.lane == 3) ? 10.0 : 0.0;
    for (int k = 0; k <= UB_N; ++k)
        for (int q = c.lane; q < 6; q += 64) sm[HEAD + k * SR + rHD + q] = 2.0;  // diagonal Hessian rows
    if (c.lane < 32) sm[HEAD + c.lane % SR] = sm[HEAD + c.lane % SR];
    __syncthreads();
    bool ok = true;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) ok = ub_riccati<V>(c, 1e-4 + 1e-12 * r) && ok;
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (c.lane == 0) out[blockIdx.x] = t1 - t0;
    if (!ok && c.lane == 0) atomicAdd(bad, 1);
}

template <int V>
void run(const char* name, int B = 1024) {
    const int reps = 200;
    unsigned long long* d_out;
    int* d_bad;
    (void)hipMalloc(&d_out, B * sizeof(unsigned long long));
    (void)hipMalloc(&d_bad, sizeof(int));
    (void)hipMemset(d_bad, 0, sizeof(int));
    const int bytes = lds_bytes(UB_N);
    hipLaunchKernelGGL(ub_kernel<V>, dim3(B), dim3(64), bytes, 0, reps, d_out, d_bad);  // warm-up
    hipLaunchKernelGGL(ub_kernel<V>, dim3(B), dim3(64), bytes, 0, reps, d_out, d_bad);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(B);
    (void)hipMemcpy(h.data(), d_out, B * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double s = 0;
    for (auto v : h) s += (double)v;
    printf("%-44s B=%5d %8.1f cycles/stage\n", name, B, s / B / reps / UB_N);
    (void)hipFree(d_out);
    (void)hipFree(d_bad);
}

}  // namespace
}  // namespace ttmpc

int main() {
    using namespace ttmpc;
    run<0>("as shipped");
    run<1>("no next-stage prefetch");
    run<2>("no factor-row stores");
    run<3>("no PA tile round trip");
    run<4>("no P tile round trip");
    run<5>("no prefetch, no stores");
    run<6>("no reciprocal");
    run<7>("one unmasked store per lane");
    run<0>("as shipped", 256);
    run<5>("no prefetch, no stores", 256);
    run<7>("one unmasked store per lane", 256);
    return 0;
}
