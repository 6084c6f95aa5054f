// Batched LQR terminal score on gfx950: python-files/LQR_cost.py:7-41.
//
//   A = I + dt df/dx(x_goal, u_goal),  B = dt df/du      (forward-Euler map, LQR_cost.py:13-30)
//   P = DARE(A, B, Q, R), symmetrised                     (scipy.linalg.solve_discrete_are, 32-34)
//   score = (x - x_goal)' P (x - x_goal)                  (lqr_distance, 37-41)
//
// The reference solves the DARE with scipy's generalized-Schur method.  Here each instance runs the
// structure-preserving doubling algorithm (SDA; Chu, Fan & Lin 2005), which needs only 6x6 products and
// one 6x18 Gauss-Jordan per doubling and converges quadratically:
//   A0 = A, G0 = B R^-1 B', H0 = Q;  W = I + G H;  V1 = W^-1 A, V2 = W^-1 G
//   A+ = A V1,  G+ = G + A V2 A',  H+ = H + A' H V1    ->  H -> P
// One 64-lane workgroup per instance; matrices live in LDS, lane (i, j) < 36 owns entry (i, j) of every
// 6x6 product, and all 64 lanes share the row operations of the Gauss-Jordan sweep.
#include <errno.h>
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>

#include "ttmpc.h"

namespace {

constexpr int kMaxDoublings = 64;

struct LqrArgs {
    tt_plant p;
    double Q[36], R[4];
    const double* xc;
    const double* xg;
    const double* ug;
    double* P;
    double* score;
    int* iters;
    int B;
};

__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}

// out = X Y (+ Z) over 6x6 row-major LDS matrices; lanes < 36
__device__ __forceinline__ double mm(const double* X, const double* Y, int i, int j) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < 6; ++k) s += X[i * 6 + k] * Y[k * 6 + j];
    return s;
}

__global__ void __launch_bounds__(64) lqr_kernel(LqrArgs a) {
    __shared__ double sA[36], sG[36], sH[36], sT[36], sAug[6 * 18], sPiv[2];
    const int b = blockIdx.x, lane = threadIdx.x;
    if (b >= a.B) return;
    const int i = lane / 6, j = lane % 6;
    const bool own = lane < 36;
    const double dt = a.p.dt, L1 = a.p.L1, L2 = a.p.L2, Mh = a.p.Mh;
    const double* xg = a.xg + (size_t)b * 6;
    // A = I + dt J(x_goal) (truck_trailer_model.py:8-24 differentiated; u enters f linearly)
    if (own) {
        const double th = xg[2], ps = xg[3], ph = xg[4], v = xg[5];
        const double c2 = 1.0 / (cos(ph) * cos(ph)), t = tan(ph);
        double J = 0.0;
        if (i == 0 && j == 2) J = -v * sin(th);
        if (i == 0 && j == 5) J = cos(th);
        if (i == 1 && j == 2) J = v * cos(th);
        if (i == 1 && j == 5) J = sin(th);
        if (i == 2 && j == 4) J = v * c2 / L1;
        if (i == 2 && j == 5) J = t / L1;
        if (i == 3 && j == 3) J = v * t * Mh * sin(ps) / (L1 * L2) - v * cos(ps) / L2;
        if (i == 3 && j == 4) J = -v * c2 / L1 * (1 + Mh / L2 * cos(ps));
        if (i == 3 && j == 5) J = -t / L1 * (1 + Mh / L2 * cos(ps)) - sin(ps) / L2;
        sA[lane] = (i == j ? 1.0 : 0.0) + dt * J;
        // G = B R^-1 B' with B = dt [e5 e4] (a -> v row 5, omega -> phi row 4)
        const double det = a.R[0] * a.R[3] - a.R[1] * a.R[2];
        const double Ri00 = a.R[3] / det, Ri01 = -a.R[1] / det, Ri10 = -a.R[2] / det, Ri11 = a.R[0] / det;
        double g = 0.0;
        if (i == 5 && j == 5) g = Ri00;
        if (i == 5 && j == 4) g = Ri01;
        if (i == 4 && j == 5) g = Ri10;
        if (i == 4 && j == 4) g = Ri11;
        sG[lane] = dt * dt * g;
        sH[lane] = a.Q[lane];
    }
    __syncthreads();
    int it = 0;
    bool done = false;
    for (; it < kMaxDoublings && !done; ++it) {
        // [W | A | G], W = I + G H
        if (own) {
            sAug[i * 18 + j] = (i == j ? 1.0 : 0.0) + mm(sG, sH, i, j);
            sAug[i * 18 + 6 + j] = sA[lane];
            sAug[i * 18 + 12 + j] = sG[lane];
        }
        __syncthreads();
        // Gauss-Jordan with partial pivoting
        for (int c = 0; c < 6; ++c) {
            if (lane == 0) {
                int r = c;
                double best = fabs(sAug[c * 18 + c]);
                for (int q = c + 1; q < 6; ++q)
                    if (fabs(sAug[q * 18 + c]) > best) { best = fabs(sAug[q * 18 + c]); r = q; }
                sPiv[0] = (double)r;
            }
            __syncthreads();
            const int r = (int)sPiv[0];
            if (r != c && lane < 18) {
                const double t0 = sAug[c * 18 + lane];
                sAug[c * 18 + lane] = sAug[r * 18 + lane];
                sAug[r * 18 + lane] = t0;
            }
            __syncthreads();
            const double inv = 1.0 / sAug[c * 18 + c];
            __syncthreads();
            if (lane < 18) sAug[c * 18 + lane] *= inv;
            __syncthreads();
            for (int e = lane; e < 6 * 18; e += 64) {
                const int q = e / 18, col = e % 18;
                if (q != c && col != c) sAug[e] -= sAug[q * 18 + c] * sAug[c * 18 + col];
            }
            __syncthreads();
            if (lane < 6 && lane != c) sAug[lane * 18 + c] = 0.0;
            __syncthreads();
        }
        // V1 = sAug[:, 6:12], V2 = sAug[:, 12:18]
        double An = 0.0, Gt = 0.0, Ht = 0.0;
        if (own) {
            double s1 = 0.0, s2 = 0.0;
#pragma unroll
            for (int k = 0; k < 6; ++k) {
                s1 += sA[i * 6 + k] * sAug[k * 18 + 6 + j];    // A V1
                s2 += sH[i * 6 + k] * sAug[k * 18 + 6 + j];    // H V1
            }
            An = s1;
            sT[lane] = s2;
        }
        __syncthreads();
        if (own) {
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < 6; ++k) s += sA[k * 6 + i] * sT[k * 6 + j];   // A' (H V1)
            Ht = sH[lane] + s;
        }
        __syncthreads();
        if (own) {
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < 6; ++k) s += sAug[i * 18 + 12 + k] * sA[j * 6 + k];   // V2 A'
            sT[lane] = s;
        }
        __syncthreads();
        if (own) {
            double s = 0.0;
#pragma unroll
            for (int k = 0; k < 6; ++k) s += sA[i * 6 + k] * sT[k * 6 + j];   // A (V2 A')
            Gt = sG[lane] + s;
        }
        const double dH = wave_max(own ? fabs(Ht - sH[lane]) : 0.0);
        const double nH = wave_max(own ? fabs(Ht) : 0.0);
        __syncthreads();
        if (own) {
            sA[lane] = An;
            sG[lane] = Gt;
            sH[lane] = Ht;
        }
        __syncthreads();
        done = !(dH > 1e-14 * nH) || !isfinite(nH);
    }
    // P = (H + H') / 2 (LQR_cost.py:34); score = dx' P dx
    double Pij = 0.0, term = 0.0;
    if (own) {
        Pij = 0.5 * (sH[lane] + sH[j * 6 + i]);
        const double* xc = a.xc + (size_t)b * 6;
        term = (xc[i] - xg[i]) * Pij * (xc[j] - xg[j]);
        if (a.P) a.P[(size_t)b * 36 + lane] = Pij;
    }
    // fixed-order sum of the 36 terms (lane 0 gathers through LDS)
    __syncthreads();
    if (own) sT[lane] = term;
    __syncthreads();
    if (lane == 0) {
        double s = 0.0;
        for (int q = 0; q < 36; ++q) s += sT[q];
        a.score[b] = s;
        if (a.iters) a.iters[b] = done ? it : -1;
    }
}

}  // namespace

extern "C" int tt_lqr_score_device(int B, const tt_plant* p, const double* Q, const double* R, const double* x_cur,
                                   const double* x_goal, const double* u_goal, double* P_out, double* score,
                                   int* iters, void* stream) {
    if (B < 0 || !p || !Q || !R || !x_cur || !x_goal || !score) return -EINVAL;
    if (B == 0) return 0;
    LqrArgs a;
    a.p = *p;
    for (int k = 0; k < 36; ++k) a.Q[k] = Q[k];
    for (int k = 0; k < 4; ++k) a.R[k] = R[k];
    if (a.R[0] * a.R[3] - a.R[1] * a.R[2] == 0.0) return -EINVAL;
    a.xc = x_cur;
    a.xg = x_goal;
    a.ug = u_goal;   // the Euler map is linear in u: A and B do not depend on u_goal (kept for the signature)
    a.P = P_out;
    a.score = score;
    a.iters = iters;
    a.B = B;
    hipLaunchKernelGGL(lqr_kernel, dim3(B), dim3(64), 0, (hipStream_t)stream, a);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        fprintf(stderr, "ttmpc: lqr_kernel launch failed: %s\n", hipGetErrorString(e));
        return -EIO;
    }
    return 0;
}
