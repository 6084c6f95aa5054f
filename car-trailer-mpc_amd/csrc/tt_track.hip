// Batched truck-trailer tracking NMPC on gfx950 (MI355X / CDNA4).
//
// One 64-lane wavefront solves one NLP instance end to end; all per-stage state lives in LDS.
//
// NLP (reference python-files/, restated):
//   min  sum_k |x_k - xr_k|^2_Qw + |u_k - ur_k|^2_Rw + |x_N - xr_N|^2_Qw     mpc_control.py:17-25
//   s.t. x_0 = x_init; x_{k+1} = x_k + dt f(x_k, u_k)                       trajectory_planning.py:28-36
//        box bounds on every x_k (k = 0..N) and u_k                          trajectory_planning.py:38-60
//   f = truck_trailer_model.py:8-24 (Euler: 26-29); fuzzy Qw = D Q D         mpc_control_fuzzy.py:23-24
//
// Solver: the primal-dual barrier method IPOPT runs for these NLPs (mpc_control.py:53 nlpsol
// 'ipopt'), restated with the same constants (tol/acc, mu_init 0.1, kappa_eps 10, kappa_mu 0.2,
// theta_mu 1.5, tau = max(.99, 1-mu), bound_relax 1e-8, bound_push/frac 1e-2, kappa_sigma 1e10,
// exact Lagrangian Hessian) and an l1-merit line search with one second-order correction.  The
// Newton system is never assembled: it is the KKT system of an equality-constrained LQ problem and
// is solved by a stage-wise Riccati recursion (inertia test = 2x2 Cholesky of each reduced input
// Hessian), O(N) per iteration instead of IPOPT's sparse LDL^T.
//
// Lane mapping (wave-uniform control flow everywhere):
//   * stage-parallel phases (model + Jacobian + curvature, residuals, barrier terms, merit
//     evaluations, multiplier updates): lane k owns stage k (loop k += 64 for N >= 64);
//   * Riccati backward sweep (serial in k): lanes 0..35 build PA = P A (one entry each), lanes
//     36..41 w = P b + p; then lanes 0..20 the upper triangle of P_k, 21..26 p_k, 27..38 the gain
//     K_k, 39 the feed-forward / inverse Hessian -- two barriers per stage, P ping-ponged in LDS;
//   * forward sweep: lane 0 (~40 dependent FMAs per stage, operands read from LDS).
//
// LDS map (doubles; row r of stage k at sm[k*149 + r]; the odd stride keeps lane-per-stage
// ds_read_b64 accesses bank-conflict-free and turns every row offset into an immediate):
//   0-5 X | 6-7 U | 8-13 Y (eq. multipliers, IPOPT sign) | 14-21 zL | 22-29 zU | 30-35 Xref
//   36-37 Uref | 38-43 dX | 44-45 dU | 46-51 Y+ | 52-60 dt*J (9 nnz) | 61-67 curvature (7 nnz)
//   68-75 Sigma | 76-83 barrier gradient | 84-89 c | 90-95 c(trial)/c_soc | 96-107 K | 108-109 k_ff
//   110-112 inv(H_uu) | 113-133 P_k (upper) | 134-139 p_k | 140-145 dX_soc | 146-147 dU_soc | 148 pad
//   tail: Qw(36) Rw(4) P ping/pong (2x36) p ping/pong (2x6) PA(36) w(6) x_init(6) lb(8) ub(8)
#include <math.h>

#include "tt_kernel.hpp"

namespace ttmpc {
namespace {

constexpr int W = 64;
constexpr int SR = kRowsPerStage;

// rows
constexpr int rX = 0, rY = 8, rZL = 14, rZU = 22, rXR = 30, rUR = 36, rDX = 38, rYP = 46, rAJ = 52, rWC = 61;
constexpr int rSG = 68, rGR = 76, rCC = 84, rCT = 90, rK = 96, rKF = 108, rIH = 110, rPS = 113, rPV = 134;
constexpr int rDXS = 140;

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, W);
    return v;
}
__device__ __forceinline__ double wmax(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fmax(v, __shfl_xor(v, m, W));
    return v;
}
__device__ __forceinline__ double wmin(double v) {
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = fmin(v, __shfl_xor(v, m, W));
    return v;
}

// upper-triangle enumeration of a symmetric 6x6
__device__ __forceinline__ void ut_ij(int e, int& i, int& j) {
    i = e < 6 ? 0 : e < 11 ? 1 : e < 15 ? 2 : e < 18 ? 3 : e < 20 ? 4 : 5;
    const int start = i == 0 ? 0 : i == 1 ? 6 : i == 2 ? 11 : i == 3 ? 15 : i == 4 ? 18 : 20;
    j = i + (e - start);
}
__host__ __device__ constexpr int sym_idx(int i, int j) {
    return i <= j ? i * 6 - (i * (i - 1)) / 2 + (j - i) : j * 6 - (j * (j - 1)) / 2 + (i - j);
}

// dt*J nonzeros: 0:J02 1:J05 2:J12 3:J15 4:J24 5:J25 6:J33 7:J34 8:J35   (A = I + dt*J)
// sum_l dtJ[l][v] * y[l*st]   (column v of dtJ)
__device__ __forceinline__ double colJ(const double* aj, int v, const double* y, int st) {
    switch (v) {
        case 2: return aj[0] * y[0] + aj[2] * y[st];
        case 3: return aj[6] * y[3 * st];
        case 4: return aj[4] * y[2 * st] + aj[7] * y[3 * st];
        case 5: return aj[1] * y[0] + aj[3] * y[st] + aj[5] * y[2 * st] + aj[8] * y[3 * st];
        default: return 0.0;
    }
}
// sum_l dtJ[r][l] * x[l]   (row r of dtJ)
__device__ __forceinline__ double rowJ(const double* aj, int r, const double* x) {
    switch (r) {
        case 0: return aj[0] * x[2] + aj[1] * x[5];
        case 1: return aj[2] * x[2] + aj[3] * x[5];
        case 2: return aj[4] * x[4] + aj[5] * x[5];
        case 3: return aj[6] * x[3] + aj[7] * x[4] + aj[8] * x[5];
        default: return 0.0;
    }
}
// curvature nonzeros: 0:(2,2) 1:(2,5) 2:(3,3) 3:(3,4) 4:(3,5) 5:(4,4) 6:(4,5); -1 = structural zero
__device__ __forceinline__ int wc_idx(int i, int j) {
    if (i > j) { int t = i; i = j; j = t; }
    switch (i * 6 + j) {
        case 14: return 0;
        case 17: return 1;
        case 21: return 2;
        case 22: return 3;
        case 23: return 4;
        case 28: return 5;
        case 29: return 6;
        default: return -1;
    }
}

// Diagnostic phase stamps (MI355X_MICROARCH: s_memtime counts shader cycles).  Compiled out unless
// -DTT_STAMPS; never in the shipped library.
#ifdef TT_STAMPS
struct Stamps {
    unsigned long long acc[kNumPhases] = {};
    unsigned long long t0 = 0, tstart = 0;
    __device__ __forceinline__ void begin() { t0 = tstart = __builtin_amdgcn_s_memtime(); }
    __device__ __forceinline__ void mark(int ph) {
        const unsigned long long t = __builtin_amdgcn_s_memtime();
        acc[ph] += t - t0;
        t0 = t;
    }
    __device__ __forceinline__ void store(unsigned long long* out, int lane) {
        acc[PH_TOTAL] = __builtin_amdgcn_s_memtime() - tstart;
        if (out && lane == 0)
            for (int i = 0; i < kNumPhases; ++i) out[i] = acc[i];
    }
};
#define STAMP(ph) stamps.mark(ph)
#else
#define STAMP(ph) ((void)0)
#endif

// Armijo test with IPOPT's round-off allowance (Compare_le: lhs - rhs <= 10 eps |reference|)
__device__ __forceinline__ bool armijo(double trial, double ref, double alpha, double D) {
    return trial - (ref + 1e-4 * alpha * D) <= 10.0 * 2.220446049250313e-16 * fabs(ref);
}

// fraction-to-boundary helper: largest a with s + a*d >= (1-tau) s
__device__ __forceinline__ void ftb(double s, double d, double tau, double& a) {
    if (d < 0.0) a = fmin(a, -tau * s / d);
}

// Per-wave solver context (registers: a handful of scalars; data: LDS)
struct Ctx {
    double* sm;
    double *QW, *RW, *PW0, *PW1, *PV0, *PV1, *PA, *WV, *XI, *LB, *UB;
    int N, lane;
    double dt, L1, L2, Mh;
    double mu, tau, nu;
    __device__ __forceinline__ double& r(int row, int k) const { return sm[k * SR + row]; }
    __device__ __forceinline__ bool hl(int v) const { return LB[v] > -INFINITY; }
    __device__ __forceinline__ bool hu(int v) const { return UB[v] < INFINITY; }
};

// ---------------- model: truck_trailer_model.py:8-24 ----------------
__device__ __forceinline__ void model_f(const Ctx& c, const double* x, const double* u, double* fo) {
    double sth, cth, sps, cps;
    sincos(x[2], &sth, &cth);
    sincos(x[3], &sps, &cps);
    const double t = tan(x[4]), v = x[5];
    fo[0] = v * cth;
    fo[1] = v * sth;
    fo[2] = v * t / c.L1;
    fo[3] = -v * t / c.L1 * (1.0 + c.Mh / c.L2 * cps) - v * sps / c.L2;
    fo[4] = u[1];
    fo[5] = u[0];
}

// f, dt*J and the curvature -dt * sum_i y_i d2f_i/dx2 in one pass (5 transcendentals)
__device__ __forceinline__ void model_lin(const Ctx& c, const double* x, const double* u, const double* y, double* fo,
                                          double* aj, double* wc) {
    double sth, cth, sps, cps;
    sincos(x[2], &sth, &cth);
    sincos(x[3], &sps, &cps);
    const double phi = x[4], v = x[5], dt = c.dt, Mh = c.Mh, L2 = c.L2;
    const double t = tan(phi), cph = cos(phi), c2 = 1.0 / (cph * cph);
    const double k = 1.0 + Mh / L2 * cps, iL1 = 1.0 / c.L1, iL1L2 = 1.0 / (c.L1 * L2);
    fo[0] = v * cth;
    fo[1] = v * sth;
    fo[2] = v * t * iL1;
    fo[3] = -v * t * iL1 * k - v * sps / L2;
    fo[4] = u[1];
    fo[5] = u[0];
    aj[0] = dt * (-v * sth);
    aj[1] = dt * cth;
    aj[2] = dt * (v * cth);
    aj[3] = dt * sth;
    aj[4] = dt * (v * c2 * iL1);
    aj[5] = dt * (t * iL1);
    aj[6] = dt * (v * t * Mh * sps * iL1L2 - v * cps / L2);
    aj[7] = dt * (-v * c2 * iL1 * k);
    aj[8] = dt * (-t * iL1 * k - sps / L2);
    const double s = -dt;
    wc[0] = s * (y[0] * (-v * cth) + y[1] * (-v * sth));
    wc[1] = s * (y[0] * (-sth) + y[1] * cth);
    wc[2] = s * (y[3] * (v * t * Mh * cps * iL1L2 + v * sps / L2));
    wc[3] = s * (y[3] * (v * c2 * Mh * sps * iL1L2));
    wc[4] = s * (y[3] * (t * Mh * sps * iL1L2 - cps / L2));
    wc[5] = s * (y[2] * (2.0 * v * t * c2 * iL1) + y[3] * (-2.0 * v * t * c2 * k * iL1));
    wc[6] = s * (y[2] * (c2 * iL1) + y[3] * (-c2 * k * iL1));
}

struct Err {
    double dinf, pinf, c0, cmu, sy, sz;
};

// ============ linearise at the current point + optimality-error pieces (stage-parallel) ============
__device__ __forceinline__ Err phase_linearize(const Ctx& c) {
    const int N = c.N;
    double dinf = 0.0, pinf = 0.0, c0 = 0.0, cmu = 0.0, sy = 0.0, sz = 0.0;
    bool fin = true;
    for (int k = c.lane; k <= N; k += W) {
        double x[6], u[2] = {0.0, 0.0}, yk[6], y1[6] = {0, 0, 0, 0, 0, 0}, aj[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 6; ++i) { x[i] = c.r(rX + i, k); yk[i] = c.r(rY + i, k); sy += fabs(yk[i]); }
        if (k == 0) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double cc = x[i] - c.XI[i];
                c.r(rCC + i, 0) = cc;
                pinf = fmax(pinf, fabs(cc));
            }
        }
        if (k < N) {
            double fo[6], wc[7];
            u[0] = c.r(rX + 6, k);
            u[1] = c.r(rX + 7, k);
#pragma unroll
            for (int i = 0; i < 6; ++i) y1[i] = c.r(rY + i, k + 1);
            model_lin(c, x, u, y1, fo, aj, wc);
#pragma unroll
            for (int i = 0; i < 9; ++i) c.r(rAJ + i, k) = aj[i];
#pragma unroll
            for (int i = 0; i < 7; ++i) c.r(rWC + i, k) = wc[i];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double cc = c.r(rX + i, k + 1) - (x[i] + c.dt * fo[i]);
                c.r(rCC + i, k + 1) = cc;
                pinf = fmax(pinf, fabs(cc));
            }
        }
        double dxr[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) dxr[i] = x[i] - c.r(rXR + i, k);
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            if (v >= 6 && k == N) break;
            double g;  // d/dz of the Lagrangian: 2 Qw dx + y_k - A'y_{k+1} - zL + zU
            if (v < 6) {
                g = 0.0;
#pragma unroll
                for (int j = 0; j < 6; ++j) g += c.QW[v * 6 + j] * dxr[j];
                g = 2.0 * g + yk[v];
                if (k < N) g -= y1[v] + colJ(aj, v, y1, 1);
            } else {
                const int rr = v - 6;
                g = 2.0 * (c.RW[rr * 2] * (u[0] - c.r(rUR, k)) + c.RW[rr * 2 + 1] * (u[1] - c.r(rUR + 1, k)));
                g -= c.dt * y1[rr == 0 ? 5 : 4];
            }
            const double xv = v < 6 ? x[v] : u[v - 6];
            if (c.hl(v)) {
                const double zl = c.r(rZL + v, k), s = xv - c.LB[v];
                g -= zl;
                c0 = fmax(c0, fabs(zl * s));
                cmu = fmax(cmu, fabs(zl * s - c.mu));
                sz += zl;
            }
            if (c.hu(v)) {
                const double zu = c.r(rZU + v, k), s = c.UB[v] - xv;
                g += zu;
                c0 = fmax(c0, fabs(zu * s));
                cmu = fmax(cmu, fabs(zu * s - c.mu));
                sz += zu;
            }
            if (!isfinite(g)) fin = false;
            dinf = fmax(dinf, fabs(g));
        }
    }
    Err e;
    e.dinf = wmax(fin ? dinf : INFINITY);
    e.pinf = wmax(pinf);
    e.c0 = wmax(c0);
    e.cmu = wmax(cmu);
    e.sy = wsum(sy);
    e.sz = wsum(sz);
    return e;
}

__device__ __forceinline__ double phase_compl_mu(const Ctx& c) {
    double cm = 0.0;
    for (int k = c.lane; k <= c.N; k += W) {
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            if (v >= 6 && k == c.N) break;
            const double xv = c.r(rX + v, k);
            if (c.hl(v)) cm = fmax(cm, fabs(c.r(rZL + v, k) * (xv - c.LB[v]) - c.mu));
            if (c.hu(v)) cm = fmax(cm, fabs(c.r(rZU + v, k) * (c.UB[v] - xv) - c.mu));
        }
    }
    return wmax(cm);
}

// ============ barrier Hessian diagonal Sigma and barrier gradient (stage-parallel) ============
__device__ __forceinline__ void phase_barrier(const Ctx& c) {
    const int N = c.N;
    for (int k = c.lane; k <= N; k += W) {
        double dxr[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) dxr[i] = c.r(rX + i, k) - c.r(rXR + i, k);
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            if (v >= 6 && k == N) break;
            double g;
            if (v < 6) {
                g = 0.0;
#pragma unroll
                for (int j = 0; j < 6; ++j) g += c.QW[v * 6 + j] * dxr[j];
                g *= 2.0;
            } else {
                const int rr = v - 6;
                g = 2.0 * (c.RW[rr * 2] * (c.r(rX + 6, k) - c.r(rUR, k)) + c.RW[rr * 2 + 1] * (c.r(rX + 7, k) - c.r(rUR + 1, k)));
            }
            const double xv = c.r(rX + v, k);
            double sg = 0.0;
            if (c.hl(v)) { const double s = xv - c.LB[v]; sg += c.r(rZL + v, k) / s; g -= c.mu / s; }
            if (c.hu(v)) { const double s = c.UB[v] - xv; sg += c.r(rZU + v, k) / s; g += c.mu / s; }
            c.r(rSG + v, k) = sg;
            c.r(rGR + v, k) = g;
        }
    }
    __syncthreads();
}

// ============ Riccati backward sweep; returns false if a reduced input Hessian is not PD ============
__device__ __forceinline__ bool phase_riccati(const Ctx& c, double dw) {
    const int N = c.N, lane = c.lane;
    const double dt = c.dt, dt2 = dt * dt;
    double* Pc = c.PW0;
    double* Pn = c.PW1;
    double* pc = c.PV0;
    double* pn = c.PV1;
    double* PA = c.PA;
    double* WV = c.WV;
    if (lane < 21) {
        int i, j;
        ut_ij(lane, i, j);
        const double v = 2.0 * c.QW[i * 6 + j] + (i == j ? c.r(rSG + i, N) + dw : 0.0);
        Pc[i * 6 + j] = v;
        Pc[j * 6 + i] = v;
        c.r(rPS + lane, N) = v;
    } else if (lane < 27) {
        const int rr = lane - 21;
        const double v = c.r(rGR + rr, N);
        pc[rr] = v;
        c.r(rPV + rr, N) = v;
    }
    __syncthreads();
    for (int k = N - 1; k >= 0; --k) {
        double aj[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) aj[i] = c.r(rAJ + i, k);
        // --- step 1: PA = P A ; w = P b + p  (b = -c_{k+1})
        if (lane < 36) {
            const int i = lane / 6, j = lane % 6;
            PA[lane] = Pc[lane] + colJ(aj, j, Pc + i * 6, 1);
        } else if (lane < 42) {
            const int rr = lane - 36;
            double s = pc[rr];
#pragma unroll
            for (int l = 0; l < 6; ++l) s -= Pc[rr * 6 + l] * c.r(rCC + l, k + 1);
            WV[rr] = s;
        }
        __syncthreads();
        // --- step 2: reduced input Hessian H = 2R + Sigma_u + B'PB (every lane, wave-uniform)
        const double h00 = 2.0 * c.RW[0] + c.r(rSG + 6, k) + dw + dt2 * Pc[35];
        const double h01 = 2.0 * c.RW[1] + dt2 * Pc[34];
        const double h11 = 2.0 * c.RW[3] + c.r(rSG + 7, k) + dw + dt2 * Pc[28];
        const double det = h00 * h11 - h01 * h01;
        if (!(h00 > 0.0 && h11 > 0.0 && det > 1e-13 * h00 * h11)) {
            __syncthreads();
            return false;
        }
        const double id = 1.0 / det, i00 = h11 * id, i01 = -h01 * id, i11 = h00 * id;
        const double hv0 = c.r(rGR + 6, k) + dt * WV[5];
        const double hv1 = c.r(rGR + 7, k) + dt * WV[4];
        const double kf0 = -(i00 * hv0 + i01 * hv1), kf1 = -(i01 * hv0 + i11 * hv1);
        if (lane < 21) {  // P_k = A'PA + H_xx - G' H^-1 G, G = B'PA (rows 5, 4 of PA scaled by dt)
            int i, j;
            ut_ij(lane, i, j);
            const int wi = wc_idx(i, j);
            double F = PA[i * 6 + j] + colJ(aj, i, PA + j, 6) + 2.0 * c.QW[i * 6 + j] + (wi >= 0 ? c.r(rWC + wi, k) : 0.0);
            if (i == j) F += c.r(rSG + i, k) + dw;
            const double g0i = dt * PA[30 + i], g1i = dt * PA[24 + i];
            const double g0j = dt * PA[30 + j], g1j = dt * PA[24 + j];
            const double v = F - (g0i * (i00 * g0j + i01 * g1j) + g1i * (i01 * g0j + i11 * g1j));
            Pn[i * 6 + j] = v;
            Pn[j * 6 + i] = v;
            c.r(rPS + lane, k) = v;
        } else if (lane < 27) {  // p_k = g_x + A'w + G' k_ff
            const int rr = lane - 21;
            const double v = c.r(rGR + rr, k) + WV[rr] + colJ(aj, rr, WV, 1) + dt * PA[30 + rr] * kf0 + dt * PA[24 + rr] * kf1;
            pn[rr] = v;
            c.r(rPV + rr, k) = v;
        } else if (lane < 39) {  // K = -H^-1 G
            const int e = lane - 27, rr = e / 6, cc = e % 6;
            const double g0c = dt * PA[30 + cc], g1c = dt * PA[24 + cc];
            c.r(rK + e, k) = rr == 0 ? -(i00 * g0c + i01 * g1c) : -(i01 * g0c + i11 * g1c);
        } else if (lane == 39) {
            c.r(rKF, k) = kf0;
            c.r(rKF + 1, k) = kf1;
            c.r(rIH, k) = i00;
            c.r(rIH + 1, k) = i01;
            c.r(rIH + 2, k) = i11;
        }
        double* t = Pc; Pc = Pn; Pn = t;
        t = pc; pc = pn; pn = t;
        __syncthreads();
    }
    return true;
}

// ============ forward sweep (lane 0): dx_0 = -c_0; du = K dx + k_ff; dx' = A dx + B du - c ============
__device__ __forceinline__ void phase_forward(const Ctx& c, int crow, int orow) {
    if (c.lane == 0) {
        const double dt = c.dt;
        double dx[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) { dx[i] = -c.r(crow + i, 0); c.r(orow + i, 0) = dx[i]; }
        for (int k = 0; k < c.N; ++k) {
            double aj[9], K[12], cc[6];
#pragma unroll
            for (int i = 0; i < 9; ++i) aj[i] = c.r(rAJ + i, k);
#pragma unroll
            for (int i = 0; i < 12; ++i) K[i] = c.r(rK + i, k);
#pragma unroll
            for (int i = 0; i < 6; ++i) cc[i] = c.r(crow + i, k + 1);
            double du0 = c.r(rKF, k), du1 = c.r(rKF + 1, k);
#pragma unroll
            for (int j = 0; j < 6; ++j) { du0 += K[j] * dx[j]; du1 += K[6 + j] * dx[j]; }
            c.r(orow + 6, k) = du0;
            c.r(orow + 7, k) = du1;
            double nx[6];
#pragma unroll
            for (int rr = 0; rr < 6; ++rr) nx[rr] = dx[rr] + rowJ(aj, rr, dx) - cc[rr];
            nx[5] += dt * du0;
            nx[4] += dt * du1;
#pragma unroll
            for (int rr = 0; rr < 6; ++rr) { dx[rr] = nx[rr]; c.r(orow + rr, k + 1) = nx[rr]; }
        }
    }
    __syncthreads();
}

// ============ SOC: backward vector pass with the stored factorisation, rhs c_soc in rCT ============
__device__ __forceinline__ void phase_soc_backward(const Ctx& c) {
    if (c.lane == 0) {
        const int N = c.N;
        const double dt = c.dt;
        double p[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) p[i] = c.r(rGR + i, N);
        for (int k = N - 1; k >= 0; --k) {
            double aj[9], w[6], cn[6];
#pragma unroll
            for (int i = 0; i < 9; ++i) aj[i] = c.r(rAJ + i, k);
#pragma unroll
            for (int i = 0; i < 6; ++i) cn[i] = c.r(rCT + i, k + 1);
#pragma unroll
            for (int rr = 0; rr < 6; ++rr) {
                double s = p[rr];
#pragma unroll
                for (int l = 0; l < 6; ++l) s -= c.r(rPS + sym_idx(rr, l), k + 1) * cn[l];
                w[rr] = s;
            }
            const double h0 = c.r(rGR + 6, k) + dt * w[5], h1 = c.r(rGR + 7, k) + dt * w[4];
            const double i00 = c.r(rIH, k), i01 = c.r(rIH + 1, k), i11 = c.r(rIH + 2, k);
            c.r(rKF, k) = -(i00 * h0 + i01 * h1);
            c.r(rKF + 1, k) = -(i01 * h0 + i11 * h1);
#pragma unroll
            for (int rr = 0; rr < 6; ++rr) {
                p[rr] = c.r(rGR + rr, k) + w[rr] + colJ(aj, rr, w, 1) + c.r(rK + rr, k) * h0 + c.r(rK + 6 + rr, k) * h1;
                c.r(rPV + rr, k) = p[rr];
            }
        }
    }
    __syncthreads();
}

struct StepInfo {
    double ap, az, ymax, Dg, th0, rel;
};

// ============ new multipliers y+ = -(P dx + p), step bounds, merit slope (stage-parallel) ============
__device__ __forceinline__ StepInfo phase_step(const Ctx& c, int dzr, bool primal_pieces) {
    const int N = c.N;
    double ap = 1.0, az = 1.0, ymax = 0.0, Dg = 0.0, th0 = 0.0, rel = 0.0;
    for (int k = c.lane; k <= N; k += W) {
        double dx[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) dx[i] = c.r(dzr + i, k);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            double s = c.r(rPV + i, k);
#pragma unroll
            for (int j = 0; j < 6; ++j) s += c.r(rPS + sym_idx(i, j), k) * dx[j];
            c.r(rYP + i, k) = -s;
            ymax = fmax(ymax, fabs(s));
            th0 += fabs(c.r(rCC + i, k));
        }
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            if (v >= 6 && k == N) break;
            const double d = c.r(dzr + v, k), xv = c.r(rX + v, k);
            Dg += c.r(rGR + v, k) * d;
            rel = fmax(rel, fabs(d) / (1.0 + fabs(xv)));
            if (c.hl(v)) {
                const double s = xv - c.LB[v], zl = c.r(rZL + v, k);
                ftb(s, d, c.tau, ap);
                ftb(zl, c.mu / s - zl - zl / s * d, c.tau, az);
            }
            if (c.hu(v)) {
                const double s = c.UB[v] - xv, zu = c.r(rZU + v, k);
                ftb(s, -d, c.tau, ap);
                ftb(zu, c.mu / s - zu + zu / s * d, c.tau, az);
            }
        }
    }
    StepInfo r;
    r.az = wmin(az);
    r.ap = wmin(ap);
    if (primal_pieces) {
        r.ymax = wmax(ymax);
        r.Dg = wsum(Dg);
        r.th0 = wsum(th0);
        r.rel = wmax(rel);
    } else {
        r.ymax = r.Dg = r.th0 = r.rel = 0.0;
    }
    __syncthreads();
    return r;
}

// ============ merit value at z + alpha*dz (rows dzr): F - mu*sum(log s) + nu*||c||_1 ============
__device__ __forceinline__ double phase_merit(const Ctx& c, double alpha, int dzr, bool storeC) {
    const int N = c.N;
    double cost = 0.0, bar = 0.0, th = 0.0;
    bool bad = false;
    for (int k = c.lane; k <= N; k += W) {
        double x[6], u[2] = {0.0, 0.0};
#pragma unroll
        for (int i = 0; i < 6; ++i) x[i] = c.r(rX + i, k) + alpha * c.r(dzr + i, k);
        if (k < N) {
            u[0] = c.r(rX + 6, k) + alpha * c.r(dzr + 6, k);
            u[1] = c.r(rX + 7, k) + alpha * c.r(dzr + 7, k);
        }
        double dxr[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) dxr[i] = x[i] - c.r(rXR + i, k);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            double s = 0.0;
#pragma unroll
            for (int j = 0; j < 6; ++j) s += c.QW[i * 6 + j] * dxr[j];
            cost += dxr[i] * s;
        }
        if (k < N) {
            const double e0 = u[0] - c.r(rUR, k), e1 = u[1] - c.r(rUR + 1, k);
            cost += e0 * (c.RW[0] * e0 + c.RW[1] * e1) + e1 * (c.RW[2] * e0 + c.RW[3] * e1);
        }
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            if (v >= 6 && k == N) break;
            const double xv = v < 6 ? x[v] : u[v - 6];
            if (c.hl(v)) { const double s = xv - c.LB[v]; if (s <= 0.0) bad = true; else bar -= c.mu * log(s); }
            if (c.hu(v)) { const double s = c.UB[v] - xv; if (s <= 0.0) bad = true; else bar -= c.mu * log(s); }
        }
        if (k == 0) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double cc = x[i] - c.XI[i];
                th += fabs(cc);
                if (storeC) c.r(rCT + i, 0) = cc;
            }
        }
        if (k < N) {
            double fo[6];
            model_f(c, x, u, fo);
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double xn = c.r(rX + i, k + 1) + alpha * c.r(dzr + i, k + 1);
                const double cc = xn - (x[i] + c.dt * fo[i]);
                th += fabs(cc);
                if (storeC) c.r(rCT + i, k + 1) = cc;
            }
        }
    }
    const double badv = wmax(bad ? 1.0 : 0.0);
    cost = wsum(cost);
    bar = wsum(bar);
    th = wsum(th);
    __syncthreads();
    return badv > 0.0 ? INFINITY : cost + bar + c.nu * th;
}

// ============ accept the step (stage-parallel) ============
__device__ __forceinline__ void phase_update(const Ctx& c, int dzr, double alpha, double az) {
    const int N = c.N;
    for (int k = c.lane; k <= N; k += W) {
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            if (v >= 6 && k == N) break;
            const double d = c.r(dzr + v, k), xo = c.r(rX + v, k), xn = xo + alpha * d;
            if (c.hl(v)) {
                const double s = xo - c.LB[v], zl = c.r(rZL + v, k);
                const double znew = zl + az * (c.mu / s - zl - zl / s * d), sn = xn - c.LB[v];
                c.r(rZL + v, k) = fmax(fmin(znew, 1e10 * c.mu / sn), c.mu / (1e10 * sn));  // kappa_sigma
            }
            if (c.hu(v)) {
                const double s = c.UB[v] - xo, zu = c.r(rZU + v, k);
                const double znew = zu + az * (c.mu / s - zu + zu / s * d), sn = c.UB[v] - xn;
                c.r(rZU + v, k) = fmax(fmin(znew, 1e10 * c.mu / sn), c.mu / (1e10 * sn));
            }
            c.r(rX + v, k) = xn;
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) c.r(rY + i, k) += alpha * (c.r(rYP + i, k) - c.r(rY + i, k));
    }
    __syncthreads();
}

// ============ c_soc = alpha c(z) + c(z + alpha dz), in place in rCT ============
__device__ __forceinline__ void phase_soc_rhs(const Ctx& c, double alpha) {
    for (int k = c.lane; k <= c.N; k += W) {
#pragma unroll
        for (int i = 0; i < 6; ++i) c.r(rCT + i, k) = alpha * c.r(rCC + i, k) + c.r(rCT + i, k);
    }
    __syncthreads();
}

__device__ __forceinline__ double phase_soc_alpha(const Ctx& c) {
    double as = 1.0;
    for (int k = c.lane; k <= c.N; k += W) {
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            if (v >= 6 && k == c.N) break;
            const double d = c.r(rDXS + v, k), xv = c.r(rX + v, k);
            if (c.hl(v)) ftb(xv - c.LB[v], d, c.tau, as);
            if (c.hu(v)) ftb(c.UB[v] - xv, -d, c.tau, as);
        }
    }
    return wmin(as);
}

// ---------------- load one instance into LDS (coalesced flat copies) ----------------
__device__ __forceinline__ void phase_load(const Ctx& c, const TrackArgs& a, int b) {
    const int lane = c.lane, N = c.N, S = N + 1, n = 8 * N + 6;
    if (lane < 8) {  // relaxed bounds (bound_relax_factor 1e-8), -inf/+inf = free
        const int v = lane;
        const double l = v < 6 ? a.xlb[v] : a.ulb[v - 6];
        const double u = v < 6 ? a.xub[v] : a.uub[v - 6];
        const bool hl = isfinite(l) && l > -1e19, hu = isfinite(u) && u < 1e19;
        c.LB[v] = hl ? l - 1e-8 * fmax(1.0, fabs(l)) : -INFINITY;
        c.UB[v] = hu ? u + 1e-8 * fmax(1.0, fabs(u)) : INFINITY;
    }
    const double* wq = a.wqwr ? a.wqwr + (size_t)b * 8 : nullptr;
    if (lane < 36) {  // Qw = diag(wq) sym(Q) diag(wq)   (mpc_control_fuzzy.py:23-24)
        const int i = lane / 6, j = lane % 6;
        const double q = 0.5 * (a.Q[i * 6 + j] + a.Q[j * 6 + i]);
        c.QW[lane] = wq ? q * wq[i] * wq[j] : q;
    } else if (lane < 40) {
        const int e = lane - 36, i = e / 2, j = e % 2;
        const double r = 0.5 * (a.R[i * 2 + j] + a.R[j * 2 + i]);
        c.RW[e] = wq ? r * wq[6 + i] * wq[6 + j] : r;
    } else if (lane < 46) {
        c.XI[lane - 40] = a.x0[(size_t)b * 6 + (lane - 40)];
    }
    const double* xr = a.xref + (size_t)b * S * 6;
    for (int t = lane; t < S * 6; t += W) c.r(rXR + t % 6, t / 6) = xr[t];
    const double* ur = a.uref + (size_t)b * N * 2;
    for (int t = lane; t < N * 2; t += W) c.r(rUR + t % 2, t / 2) = ur[t];
    if (a.zg) {
        const double* zg = a.zg + (size_t)b * n;
        for (int t = lane; t < n; t += W) c.r(t % 8, t / 8) = zg[t];
    }
    __syncthreads();
    if (!a.zg) {  // reference-copy guess, mpc_control.py:58-65 (the x_0 guess is Xref[:,0])
        for (int k = lane; k <= N; k += W)
#pragma unroll
            for (int v = 0; v < 8; ++v) {
                if (v >= 6 && k == N) break;
                c.r(rX + v, k) = c.r(rXR + v, k);
            }
    }
    __syncthreads();
}

// bound push (IPOPT bound_push / bound_frac = 1e-2), z_L = z_U = 1, y = 0
__device__ __forceinline__ void phase_init(const Ctx& c) {
    const int N = c.N;
    for (int k = c.lane; k <= N; k += W) {
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            if (v >= 6 && k == N) break;
            double z = c.r(rX + v, k);
            const double l = c.LB[v], u = c.UB[v];
            if (c.hl(v) && c.hu(v)) {
                const double pl = fmin(1e-2 * fmax(1.0, fabs(l)), 1e-2 * (u - l));
                const double pu = fmin(1e-2 * fmax(1.0, fabs(u)), 1e-2 * (u - l));
                z = fmin(fmax(z, l + pl), u - pu);
            } else if (c.hl(v)) {
                z = fmax(z, l + 1e-2 * fmax(1.0, fabs(l)));
            } else if (c.hu(v)) {
                z = fmin(z, u - 1e-2 * fmax(1.0, fabs(u)));
            }
            c.r(rX + v, k) = z;
            c.r(rZL + v, k) = c.hl(v) ? 1.0 : 0.0;
            c.r(rZU + v, k) = c.hu(v) ? 1.0 : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) c.r(rY + i, k) = 0.0;
    }
    __syncthreads();
}

__global__ __launch_bounds__(W) void track_kernel(TrackArgs a) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    const int b = blockIdx.x;
    const int N = a.N, S = N + 1;
    Ctx c;
    c.sm = sm;
    c.QW = sm + SR * S;
    c.RW = c.QW + 36;
    c.PW0 = c.RW + 4;
    c.PW1 = c.PW0 + 36;
    c.PV0 = c.PW1 + 36;
    c.PV1 = c.PV0 + 6;
    c.PA = c.PV1 + 6;
    c.WV = c.PA + 36;
    c.XI = c.WV + 6;
    c.LB = c.XI + 6;
    c.UB = c.LB + 8;
    c.N = N;
    c.lane = threadIdx.x;
    c.dt = a.dt;
    c.L1 = a.L1;
    c.L2 = a.L2;
    c.Mh = a.Mh;
    c.mu = 0.1;
    c.tau = fmax(0.99, 1.0 - c.mu);
    c.nu = 1.0;

#ifdef TT_STAMPS
    Stamps stamps;
    stamps.begin();
#endif
    phase_load(c, a, b);
    int nbx = 0, nbu = 0;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
        if (v < 6) nbx += (int)c.hl(v) + (int)c.hu(v);
        else nbu += (int)c.hl(v) + (int)c.hu(v);
    }
    const int nb = (N + 1) * nbx + N * nbu;
    // infeasible: x_0 = x_init cannot hold inside the (relaxed) box of x_0
    bool infeas = false;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const double xi = c.XI[i];
        if (!isfinite(xi) || (c.hl(i) && xi < c.LB[i]) || (c.hu(i) && xi > c.UB[i])) infeas = true;
    }
    int status = infeas ? 3 : 2, iter = 0;
    double E0 = INFINITY;
    if (!infeas) {
        phase_init(c);
        STAMP(PH_LOAD);
        double dw_last = 0.0;
        int acc_count = 0;
        for (iter = 0;; ++iter) {
            const Err e = phase_linearize(c);
            __syncthreads();
            STAMP(PH_LIN);
            if (!isfinite(e.dinf) || !isfinite(e.pinf)) { status = 4; break; }
            const double sd = fmax(100.0, (e.sy + e.sz) / (double)(6 * (N + 1) + nb)) / 100.0;
            const double sc = nb ? fmax(100.0, e.sz / (double)nb) / 100.0 : 1.0;
            E0 = fmax(fmax(e.dinf / sd, e.pinf), e.c0 / sc);
            if (E0 <= a.tol) { status = 0; break; }
            if (E0 <= a.acc_tol) {
                if (++acc_count >= a.acc_iter) { status = 1; break; }
            } else {
                acc_count = 0;
            }
            if (iter >= a.max_iter) { status = E0 <= a.acc_tol ? 1 : 2; break; }
            // barrier parameter (monotone Fiacco-McCormick)
            double cmu = e.cmu;
            for (;;) {
                const double Emu = fmax(fmax(e.dinf / sd, e.pinf), cmu / sc);
                if (!(Emu <= 10.0 * c.mu && c.mu > a.tol / 10.0 * 1.0000001)) break;
                c.mu = fmax(a.tol / 10.0, fmin(0.2 * c.mu, pow(c.mu, 1.5)));
                c.tau = fmax(0.99, 1.0 - c.mu);
                cmu = phase_compl_mu(c);
            }
            phase_barrier(c);
            STAMP(PH_MU_BAR);
            // Newton step: Riccati with inertia correction
            double dw = 0.0;
            bool ok = false;
            for (int attempt = 0; attempt < 30; ++attempt) {
                if (phase_riccati(c, dw)) { ok = true; break; }
                dw = (dw == 0.0) ? (dw_last == 0.0 ? 1e-4 : fmax(1e-20, dw_last / 3.0))
                                 : (dw_last == 0.0 ? 100.0 * dw : 8.0 * dw);
                if (dw > 1e40) break;
            }
            if (!ok) { status = 4; break; }
            if (dw > 0.0) dw_last = dw;
            STAMP(PH_RIC);
            phase_forward(c, rCC, rDX);
            STAMP(PH_FWD);
            const StepInfo si = phase_step(c, rDX, true);
            STAMP(PH_STEP);
            if (c.nu < si.ymax + 1.0) c.nu = fmax(1.1 * si.ymax + 1.0, c.nu);
            // l1-merit backtracking line search with one second-order correction
            const double phi0 = phase_merit(c, 0.0, rDX, false);
            STAMP(PH_MERIT);
            const double D = si.Dg - c.nu * si.th0;
            double alpha = si.ap, az = si.az;
            int accepted = si.rel < 1e-15 ? 1 : 0;
            bool soc = false;
            for (int ls = 0; ls < 40 && !accepted; ++ls) {
                const double phit = phase_merit(c, alpha, rDX, ls == 0);
                STAMP(PH_MERIT);
                if (armijo(phit, phi0, alpha, D)) { accepted = 1; break; }
                if (ls == 0 && isfinite(phit)) {
                    phase_soc_rhs(c, alpha);
                    phase_soc_backward(c);
                    phase_forward(c, rCT, rDXS);
                    const double as = phase_soc_alpha(c);
                    const double phis = phase_merit(c, as, rDXS, false);
                    if (armijo(phis, phi0, alpha, D)) {
                        accepted = 2;
                        soc = true;
                        alpha = as;
                        az = phase_step(c, rDXS, false).az;  // y+ and dual step bound of the corrected step
                        STAMP(PH_SOC);
                        break;
                    }
                    STAMP(PH_SOC);
                }
                alpha *= 0.5;
            }
            if (!accepted) alpha *= 2.0;
            phase_update(c, soc ? rDXS : rDX, alpha, az);
            STAMP(PH_UPDATE);
        }
    }
    __syncthreads();
    {
        const int lane = c.lane;
        double* xo = a.xout + (size_t)b * S * 6;
        for (int t = lane; t < S * 6; t += W) xo[t] = c.r(rX + t % 6, t / 6);
        double* uo = a.uout + (size_t)b * N * 2;
        for (int t = lane; t < N * 2; t += W) uo[t] = c.r(rX + 6 + t % 2, t / 2);
#ifdef TT_STAMPS
        stamps.store(a.stamps ? a.stamps + (size_t)b * kNumPhases : nullptr, lane);
#endif
        if (lane == 0) {
            a.status[b] = status;
            if (a.iters) a.iters[b] = iter;
            if (a.kkt) a.kkt[b] = E0;
        }
    }
}

}  // namespace

hipError_t launch_track(const TrackArgs& a, hipStream_t stream) {
    const int bytes = lds_bytes(a.N);
    static int configured = 0;
    if (bytes > 64 * 1024 && configured < bytes) {
        hipError_t e = hipFuncSetAttribute((const void*)track_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        if (e != hipSuccess) return e;
        configured = bytes;
    }
    hipLaunchKernelGGL(track_kernel, dim3(a.B), dim3(W), bytes, stream, a);
    return hipGetLastError();
}

}  // namespace ttmpc
