// Prototype cost of a stage-parallel (associative-scan) Riccati sweep on gfx950 (diagnostic, GPU box).
//
// The parallel-in-time LQR form (Saerkkae & Garcia-Fernandez, "Temporal parallelisation of dynamic programming and
// linear quadratic control", 2023) writes each stage as an element e = (A, b, C, eta, J) of the conditional value
// function and combines two adjacent elements by
//   T   = (I + C_i J_j)^-1                (J_j C_i + I = (I + C_i J_j)^T for symmetric C, J, so one inverse serves both)
//   A_ij = A_j T A_i                      b_ij = A_j T (b_i + C_i eta_j) + b_j
//   C_ij = A_j T C_i A_j^T + C_j          eta_ij = (T A_i)^T (eta_j - J_j b_i) + eta_i
//   J_ij = (T A_i)^T J_j A_i + J_i
// i.e. one 6x6 inverse and eight 6x6 products per combination (the input block B enters only through C = B R^-1 B^T
// per stage, formed once).  An N = 20 sweep needs log2(21) ~ 5 levels: 74 combinations as a Hillis-Steele scan, ~40 as a
// work-efficient (Blelloch) scan in ~9 levels, plus the per-stage gain extraction.
//
// This kernel runs the combination the way the tracking kernel runs its Riccati stage: one wave per instance, lane
// 6i + j owning entry (i, j) of every 6x6 block (36 lanes busy), blocks in LDS, the inverse by Gauss-Jordan on the
// augmented [M | I] (two entries per lane).  It times `reps` dependent combinations (each one's output feeds the next)
// with s_memtime, one wave per SIMD (grid = 4 x CUs of 64-lane workgroups), and prints cycles per combination, next
// to the tracking kernel's measured serial stage (~745 cycles per stage, 14.9 k per N = 20 sweep: tools/phase_stamps.py).
// build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/ubench_scan.hip -o tools/ubench_scan
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

namespace {

constexpr int NX = 6, NN = NX * NX;
// LDS layout (doubles): element i (A C J b eta) | element j (same) | work blocks
enum { oA = 0, oC = 36, oJ = 72, ob = 108, oe = 114, EL = 120 };
enum { EI = 0, EJ = EL, W0 = 2 * EL, W1 = W0 + NN, W2 = W1 + NN, W3 = W2 + NN, W4 = W3 + NN, AUG = W4 + NN,
       LDS_DOUBLES = AUG + 2 * NN + 16 };

// Z = X Y (or X^T Y, X Y^T) for 6x6 blocks in LDS; lanes 0..35 own entry (i, j)
template <bool TX, bool TY>
__device__ __forceinline__ void mm(double* s, int z, int x, int y, int lane) {
    double acc = 0.0;
    if (lane < NN) {
        const int i = lane / NX, j = lane % NX;
#pragma unroll
        for (int m = 0; m < NX; ++m) {
            const double xv = TX ? s[x + m * NX + i] : s[x + i * NX + m];
            const double yv = TY ? s[y + j * NX + m] : s[y + m * NX + j];
            acc = fma(xv, yv, acc);
        }
    }
    __builtin_amdgcn_s_waitcnt(0);  // (one wave: LDS requests complete in order)
    if (lane < NN) s[z + lane] = acc;
}
// Z = X + Y
__device__ __forceinline__ void madd(double* s, int z, int x, int y, int lane) {
    if (lane < NN) s[z + lane] = s[x + lane] + s[y + lane];
}
// inverse of M (6x6 at m) into t by Gauss-Jordan on [M | I] without pivoting (I + C J with C, J PSD: well conditioned)
__device__ __forceinline__ void inv6(double* s, int m, int t, int lane) {
    double* a = s + AUG;  // 6 x 12, row-major
    if (lane < NN) {
        const int i = lane / NX, j = lane % NX;
        a[i * 12 + j] = s[m + lane];
        a[i * 12 + 6 + j] = i == j ? 1.0 : 0.0;
    }
    for (int p = 0; p < NX; ++p) {
        double v0 = 0.0, v1 = 0.0;
        if (lane < NN) {
            const int i = lane / NX, j = lane % NX;
            const double piv = a[p * 12 + p];
            const double f = a[i * 12 + p];
            const double rp0 = a[p * 12 + j], rp1 = a[p * 12 + 6 + j];
            const double ip = 1.0 / piv;
            if (i == p) { v0 = rp0 * ip; v1 = rp1 * ip; }
            else { v0 = fma(-f * ip, rp0, a[i * 12 + j]); v1 = fma(-f * ip, rp1, a[i * 12 + 6 + j]); }
        }
        __builtin_amdgcn_s_waitcnt(0);
        if (lane < NN) {
            const int i = lane / NX, j = lane % NX;
            a[i * 12 + j] = v0;
            a[i * 12 + 6 + j] = v1;
        }
    }
    if (lane < NN) s[t + lane] = a[(lane / NX) * 12 + 6 + lane % NX];
}

// one combination e_i (x) e_j -> written back into e_i (so repeated combinations form one dependent chain)
__device__ __forceinline__ void combine(double* s, int lane) {
    // M = I + C_i J_j ; T = M^-1
    mm<false, false>(s, W0, EI + oC, EJ + oJ, lane);
    if (lane < NN) s[W0 + lane] += (lane / NX == lane % NX) ? 1.0 : 0.0;
    inv6(s, W0, W1, lane);                         // W1 = T
    mm<false, false>(s, W2, W1, EI + oA, lane);    // W2 = T A_i
    mm<false, false>(s, W3, EJ + oA, W1, lane);    // W3 = A_j T
    mm<false, false>(s, W0, W3, EI + oC, lane);    // W0 = A_j T C_i
    mm<false, true>(s, W4, W0, EJ + oA, lane);     // W4 = A_j T C_i A_j^T
    madd(s, EI + oC, W4, EJ + oC, lane);           // C_ij
    mm<false, false>(s, W0, EJ + oJ, EI + oA, lane);  // W0 = J_j A_i
    mm<true, false>(s, W4, W2, W0, lane);          // W4 = (T A_i)^T J_j A_i
    madd(s, EI + oJ, W4, EI + oJ, lane);           // J_ij
    // vectors (lanes 0..5): b_ij = A_j T (b_i + C_i eta_j) + b_j, eta_ij = (T A_i)^T (eta_j - J_j b_i) + eta_i
    double bn = 0.0, en = 0.0;
    if (lane < NX) {
        double v[NX], w[NX];
#pragma unroll
        for (int r = 0; r < NX; ++r) {
            double t1 = s[EI + ob + r], t2 = s[EJ + oe + r];
#pragma unroll
            for (int m = 0; m < NX; ++m) {
                t1 = fma(s[EI + oC + r * NX + m], s[EJ + oe + m], t1);
                t2 = fma(-s[EJ + oJ + r * NX + m], s[EI + ob + m], t2);
            }
            v[r] = t1;
            w[r] = t2;
        }
        bn = s[EJ + ob + lane];
        en = s[EI + oe + lane];
#pragma unroll
        for (int m = 0; m < NX; ++m) {
            bn = fma(s[W3 + lane * NX + m], v[m], bn);
            en = fma(s[W2 + m * NX + lane], w[m], en);
        }
    }
    mm<false, false>(s, W4, W3, EI + oA, lane);    // W4 = A_j T A_i
    __builtin_amdgcn_s_waitcnt(0);
    if (lane < NN) s[EI + oA + lane] = s[W4 + lane];
    if (lane < NX) { s[EI + ob + lane] = bn; s[EI + oe + lane] = en; }
}

__global__ __launch_bounds__(64) void scan_kernel(int reps, unsigned long long* cyc, double* sink) {
    __shared__ double s[LDS_DOUBLES];
    const int lane = threadIdx.x;
    // a well-conditioned pair: A = I + 0.05 R, C and J = 0.1 I + 0.01 R R^T (PSD), small vectors
    for (int t = lane; t < 2 * EL; t += 64) {
        const int e = t % EL;
        const double r = 0.01 * (double)((t * 7919 + blockIdx.x * 31) % 97) / 97.0;
        double v;
        if (e < oC) v = ((e / NX) == (e % NX) ? 1.0 : 0.0) + 0.05 * r;
        else if (e < ob) { const int q = (e - (e < oJ ? oC : oJ)); v = ((q / NX) == (q % NX) ? 0.1 : 0.0) + 0.01 * r; }
        else v = r;
        s[t] = v;
    }
    // symmetrise C and J
    if (lane < NN) {
        const int i = lane / NX, j = lane % NX;
        for (int base : {EI + oC, EI + oJ, EJ + oC, EJ + oJ}) {
            const double a = s[base + i * NX + j], b = s[base + j * NX + i];
            __builtin_amdgcn_s_waitcnt(0);
            s[base + i * NX + j] = 0.5 * (a + b);
        }
    }
    __builtin_amdgcn_s_waitcnt(0);
    combine(s, lane);  // warm-up
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int r = 0; r < reps; ++r) {
        // keep the chain bounded: rescale A_i back towards the identity (the repeated product would blow up)
        if (lane < NN) s[EI + oA + lane] = 0.5 * s[EI + oA + lane] + ((lane / NX == lane % NX) ? 0.5 : 0.0);
        if (lane < NN) s[EI + oC + lane] *= 0.5;
        if (lane < NN) s[EI + oJ + lane] *= 0.5;
        combine(s, lane);
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    if (lane == 0) {
        cyc[blockIdx.x] = t1 - t0;
        sink[blockIdx.x] = s[EI + oA] + s[EI + oJ] + s[EI + ob];
    }
}

}  // namespace

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 200;
    int dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
        return 2;
    const int grid = 4 * cus;  // one wave per SIMD, as the C2 launch (B = 1024)
    unsigned long long* cyc;
    double* sink;
    if (hipMalloc(&cyc, grid * 8) != hipSuccess || hipMalloc(&sink, grid * 8) != hipSuccess) return 2;
    hipLaunchKernelGGL(scan_kernel, dim3(grid), dim3(64), 0, 0, reps, cyc, sink);
    if (hipDeviceSynchronize() != hipSuccess) { printf("kernel failed\n"); return 2; }
    unsigned long long* h = (unsigned long long*)malloc(grid * 8);
    double* hs = (double*)malloc(grid * 8);
    if (hipMemcpy(h, cyc, grid * 8, hipMemcpyDeviceToHost) != hipSuccess || hipMemcpy(hs, sink, grid * 8, hipMemcpyDeviceToHost) != hipSuccess)
        return 2;
    double mean = 0.0;
    for (int b = 0; b < grid; ++b) mean += (double)h[b];
    mean /= grid;
    const double per = mean / reps;
    printf("associative-scan Riccati combination (6x6 blocks, one wave, 36 entry lanes, %d workgroups = one wave per SIMD): "
           "%.0f cycles per combination (%d dependent reps; sink %.3g)\n", grid, per, reps, hs[0]);
    printf("N = 20 sweep by this operator, one combination at a time per wave: Hillis-Steele 74 combinations ~ %.0f k cycles, "
           "work-efficient ~40 combinations ~ %.0f k cycles, against the serial entry-parallel sweep's measured 14.9 k\n",
           74.0 * per / 1000.0, 40.0 * per / 1000.0);
    printf("  lower bound with the 5-level Hillis-Steele depth and unlimited lanes: %.1f k cycles (5 dependent combinations)\n",
           5.0 * per / 1000.0);
    return 0;
}
