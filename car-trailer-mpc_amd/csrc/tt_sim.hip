// Closed-loop simulation step on gfx950: the per-timestep glue of python-files/simulation.py around
// the NLP solve, batched over B independent Monte-Carlo instances and kept resident in HBM between
// steps.  All kernels here are tiny and HBM/launch bound (a few hundred bytes
// per instance per step); they exist so that a closed loop never leaves the device.
//
//   sim_window_kernel   reference window with end padding       simulation.py:486-501
//                       + noisy state measurement               simulation.py:509-513, 151-165
//   collision_kernel    SAT OBB-vs-AABB over a trajectory       simulation.py:224-385
//   plant_kernel        disturbed plant update                  simulation.py:167-199 (+50-149)
//                       (zero control after an NMPC failure     simulation_nmpc.py:204-218)
//   warm_kernel         shifted warm start for NMPC / fuzzy     mpc_control_nmpc.py:69-100
//   record_kernel       keep the last successful optimum        mpc_control_nmpc.py:107-111
//   interp_kernel       OBCA plan -> MPC rate (dt 0.1 -> 0.05)  simulation.py:201-218
#include <errno.h>
#include <math.h>
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "ttmpc.h"

namespace {

constexpr int kThreads = 256;

__host__ __device__ inline int grid_for(long long n) { return (int)((n + kThreads - 1) / kThreads); }

// ---- reference window + measured state, one thread per (instance, stage) --------------------------
// xr[j] = plan_x[min(k+j, Np)] in all three branches of simulation.py:486-501; ur[j] = plan_u[min(k+j,
// Np-1)] while k < Np, else 0 (the k >= N branch zeroes the inputs).
__global__ void __launch_bounds__(kThreads) sim_window_kernel(int B, int N, int k, int Np, const double* __restrict__ px,
                                                              const double* __restrict__ pu, int per_instance,
                                                              const double* __restrict__ state,
                                                              const double* __restrict__ noise,
                                                              double* __restrict__ xmeas, double* __restrict__ xr,
                                                              double* __restrict__ ur) {
    const long long t = (long long)blockIdx.x * kThreads + threadIdx.x;
    const long long total = (long long)B * (N + 1);
    if (t >= total) return;
    const int b = (int)(t / (N + 1)), j = (int)(t % (N + 1));
    const size_t pb = per_instance ? (size_t)b : 0;
    const int sx = min(k + j, Np);
    const double* src = px + (pb * (Np + 1) + sx) * 6;
    double* dst = xr + ((size_t)b * (N + 1) + j) * 6;
#pragma unroll
    for (int i = 0; i < 6; ++i) dst[i] = src[i];
    if (j < N) {
        double* du = ur + ((size_t)b * N + j) * 2;
        if (k < Np) {
            const double* su = pu + (pb * Np + min(k + j, Np - 1)) * 2;
            du[0] = su[0];
            du[1] = su[1];
        } else {
            du[0] = 0.0;
            du[1] = 0.0;
        }
    } else if (xmeas) {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const double s = state[(size_t)b * 6 + i];
            xmeas[(size_t)b * 6 + i] = noise ? s + noise[(size_t)b * 6 + i] : s;
        }
    }
}

// ---- the same window for a step index read from the device (hipGraph replay of a closed-loop step):
// k = ks[*step] (the reference's float-accumulated clock, precomputed), noise = noise_all[*step]
__global__ void __launch_bounds__(kThreads) sim_window_indexed_kernel(int B, int N, const int* __restrict__ ks,
                                                                      const int* __restrict__ step, int Np,
                                                                      const double* __restrict__ px,
                                                                      const double* __restrict__ pu, int per_instance,
                                                                      const double* __restrict__ state,
                                                                      const double* __restrict__ noise_all,
                                                                      double* __restrict__ xmeas,
                                                                      double* __restrict__ xr, double* __restrict__ ur) {
    const int j = *step;
    const int k = ks[j];
    const double* noise = noise_all ? noise_all + (size_t)j * B * 6 : nullptr;
    const long long t = (long long)blockIdx.x * kThreads + threadIdx.x;
    if (t >= (long long)B * (N + 1)) return;
    const int b = (int)(t / (N + 1)), jj = (int)(t % (N + 1));
    const size_t pb = per_instance ? (size_t)b : 0;
    const double* src = px + (pb * (Np + 1) + min(k + jj, Np)) * 6;
    double* dst = xr + ((size_t)b * (N + 1) + jj) * 6;
#pragma unroll
    for (int i = 0; i < 6; ++i) dst[i] = src[i];
    if (jj < N) {
        double* du = ur + ((size_t)b * N + jj) * 2;
        if (k < Np) {
            const double* su = pu + (pb * Np + min(k + jj, Np - 1)) * 2;
            du[0] = su[0];
            du[1] = su[1];
        } else {
            du[0] = 0.0;
            du[1] = 0.0;
        }
    } else {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const double v = state[(size_t)b * 6 + i];
            xmeas[(size_t)b * 6 + i] = noise ? v + noise[(size_t)b * 6 + i] : v;
        }
    }
}

// closed-loop logs at the device step index: S[step+1] = state, Ua[step] = applied control, status /
// iterations / collision flag of the step
__global__ void __launch_bounds__(kThreads) sim_log_kernel(int B, const int* __restrict__ step,
                                                           const double* __restrict__ state,
                                                           const double* __restrict__ ua, const int* __restrict__ st,
                                                           const int* __restrict__ it, const int* __restrict__ fl,
                                                           double* __restrict__ S, double* __restrict__ Ua,
                                                           int* __restrict__ Ss, int* __restrict__ Si,
                                                           int* __restrict__ Sc) {
    const int b = blockIdx.x * kThreads + threadIdx.x;
    if (b >= B) return;
    const size_t j = (size_t)*step;
#pragma unroll
    for (int i = 0; i < 6; ++i) S[((j + 1) * B + b) * 6 + i] = state[(size_t)b * 6 + i];
    Ua[(j * B + b) * 2] = ua[(size_t)b * 2];
    Ua[(j * B + b) * 2 + 1] = ua[(size_t)b * 2 + 1];
    Ss[j * B + b] = st[b];
    Si[j * B + b] = it ? it[b] : 0;
    Sc[j * B + b] = fl ? fl[b] : 0;
}
__global__ void sim_advance_kernel(int* step) { *step += 1; }

// ---- SAT collision: check_obb_aabb_collision for truck and trailer, every pose, every obstacle ------
// Evaluated literally as the reference does (corners = R local + c, projections min/max of corners . axis,
// strict '<' gap test, touching = collision), without FMA contraction so the arithmetic is numpy's.
struct Poly {
    double x[4], y[4];
};

__device__ __forceinline__ void rect_corners(double cx, double cy, double hl, double hw, double ang, Poly& p) {
#pragma clang fp contract(off)
    const double c = cos(ang), s = sin(ang);
    const double lx[4] = {hl, hl, -hl, -hl}, ly[4] = {hw, -hw, -hw, hw};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        p.x[i] = (c * lx[i] + (-s) * ly[i]) + cx;
        p.y[i] = (s * lx[i] + c * ly[i]) + cy;
    }
}

__device__ __forceinline__ void proj(const Poly& p, double ax, double ay, double& lo, double& hi) {
#pragma clang fp contract(off)
    lo = hi = p.x[0] * ax + p.y[0] * ay;
#pragma unroll
    for (int i = 1; i < 4; ++i) {
        const double v = p.x[i] * ax + p.y[i] * ay;
        lo = fmin(lo, v);
        hi = fmax(hi, v);
    }
}

// The oriented body's half of the separating-axis test: its axes (the AABB's two, then its own edge normals) and its
// projections on them.  Independent of the obstacle, so a pose computes them once per body instead of once per
// (obstacle, body) pair as check_obb_aabb_collision does; the arithmetic of every value is the reference's.
struct ObbAxes {
    double ax[4], ay[4], omin[4], omax[4];
    int na;
};

__device__ __forceinline__ void obb_axes(const Poly& o, ObbAxes& r) {
#pragma clang fp contract(off)
    r.ax[0] = 1.0; r.ay[0] = 0.0;
    r.ax[1] = 0.0; r.ay[1] = 1.0;
    r.ax[2] = r.ax[3] = r.ay[2] = r.ay[3] = 0.0;
    int na = 2;
    const double e1x = o.x[1] - o.x[0], e1y = o.y[1] - o.y[0];
    const double e2x = o.x[3] - o.x[0], e2y = o.y[3] - o.y[0];
    const double n1 = sqrt(e1x * e1x + e1y * e1y), n2 = sqrt(e2x * e2x + e2y * e2y);
    if (n1 > 1e-9) { r.ax[na] = -e1y / n1; r.ay[na] = e1x / n1; ++na; }
    if (n2 > 1e-9) { r.ax[na] = -e2y / n2; r.ay[na] = e2x / n2; ++na; }
    r.na = na;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (i < na) proj(o, r.ax[i], r.ay[i], r.omin[i], r.omax[i]);
}

// check_obb_aabb_collision (simulation.py:224-300) with the body's half precomputed (obb_axes)
__device__ bool obb_aabb(const ObbAxes& o, double cx, double cy, double hw, double hh) {
#pragma clang fp contract(off)
    Poly a;
    a.x[0] = cx + hw; a.y[0] = cy + hh;
    a.x[1] = cx + hw; a.y[1] = cy - hh;
    a.x[2] = cx - hw; a.y[2] = cy - hh;
    a.x[3] = cx - hw; a.y[3] = cy + hh;
    for (int i = 0; i < o.na; ++i) {
        double amin, amax;
        proj(a, o.ax[i], o.ay[i], amin, amax);
        if (o.omax[i] < amin || amax < o.omin[i]) return false;
    }
    return true;
}

__device__ bool pose_collides(const double* q, const double* obs, int M, double L1, double L2, double Mh, double W1,
                              double W2) {
#pragma clang fp contract(off)
    const double x = q[0], y = q[1], th = q[2], ps = q[3];
    Poly v, t;
    rect_corners(x + cos(th) * L1 / 2, y + sin(th) * L1 / 2, L1 / 2, W1 / 2, th, v);          // 318-326
    const double hx = x - cos(th) * Mh, hy = y - sin(th) * Mh;                                    // 328-335
    rect_corners(hx - cos(th + ps) * L2 / 2, hy - sin(th + ps) * L2 / 2, L2 / 2, W2 / 2, th + ps, t);
    ObbAxes va, ta;
    obb_axes(v, va);
    obb_axes(t, ta);
    for (int m = 0; m < M; ++m) {
        const double* o = obs + 4 * m;
        if (obb_aabb(va, o[0], o[1], o[2] / 2, o[3] / 2)) return true;
        if (obb_aabb(ta, o[0], o[1], o[2] / 2, o[3] / 2)) return true;
    }
    return false;
}

// one wave per instance, lanes over the K poses; flag = any pose collides (check_trajectory_collision)
__global__ void __launch_bounds__(64) collision_kernel(int B, int K, long long stride_b, int stride_k,
                                                      const double* __restrict__ poses, const double* __restrict__ obs,
                                                      int M, double L1, double L2, double Mh, double W1, double W2,
                                                      int* __restrict__ flag) {
    const int b = blockIdx.x, lane = threadIdx.x;
    if (b >= B) return;
    bool hit = false;
    for (int j = lane; j < K; j += 64)
        hit = hit || pose_collides(poses + b * stride_b + (long long)j * stride_k, obs, M, L1, L2, Mh, W1, W2);
    const unsigned long long any = __ballot(hit);
    if (lane == 0) flag[b] = any != 0ull ? 1 : 0;
}

// ---- disturbed plant: update(q, u, params, DISTURBANCE_PARAMS), simulation.py:167-199 ------------------
// one instance in place: q (6) <- update(q, (a, om)); (a, om) before friction/slippage scaling.  sn: the NMPC /
// fuzzy drivers' in-plant process noise (simulation_nmpc.py:94-105, simulation_fuzzy.py: q_ += state_noise * dt
// after the Euler step), or nullptr (simulation.py's update has none)
__device__ __forceinline__ void plant_apply(const tt_plant& p, double* q, double a, double om, const double* sn) {
#pragma clang fp contract(off)
    if (p.enable) { a *= p.friction_coeff; om *= p.slippage_coeff; }                     // apply_disturbances 66-80
    const double th = q[2], ps = q[3], ph = q[4], v = q[5];
    double qd[6];                                                                        // f_dyn 34-48
    qd[0] = v * cos(th);
    qd[1] = v * sin(th);
    qd[2] = v * tan(ph) / p.L1;
    qd[3] = -v * tan(ph) / p.L1 * (1 + p.Mh / p.L2 * cos(ps)) - v * sin(ps) / p.L2;
    qd[4] = om;
    qd[5] = a;
    if (p.enable) {                                                                      // slippage 89-115
        const double slip = 1.0 - fmin(fabs(ph) * fabs(v) * p.slip_angle_max, 0.3);
        qd[2] *= slip;
        qd[3] *= slip;
    }
#pragma unroll
    for (int i = 0; i < 6; ++i) q[i] = q[i] + qd[i] * p.dt;
    if (sn)
#pragma unroll
        for (int i = 0; i < 6; ++i) q[i] = q[i] + sn[i] * p.dt;
    if (p.enable) {                                                                      // lateral slip 117-149
        const double mag = p.lateral_slip_gain * fabs(v) * fabs(ph);
        q[0] += mag * cos(th + M_PI / 2) * p.dt;
        q[1] += mag * sin(th + M_PI / 2) * p.dt;
    }
}

__global__ void __launch_bounds__(kThreads) plant_kernel(int B, tt_plant p, double* __restrict__ state,
                                                         const double* __restrict__ u, long long u_stride,
                                                         const int* __restrict__ status, int zero_on_fail,
                                                         const double* __restrict__ noise, double* __restrict__ u_applied) {
    const int b = blockIdx.x * kThreads + threadIdx.x;
    if (b >= B) return;
    double q[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) q[i] = state[(size_t)b * 6 + i];
    double a = u[b * u_stride], om = u[b * u_stride + 1];
    if (zero_on_fail && status && status[b] > TT_ACCEPTABLE) { a = 0.0; om = 0.0; }   // simulation_nmpc.py:208-214
    if (u_applied) { u_applied[(size_t)b * 2] = a; u_applied[(size_t)b * 2 + 1] = om; }
    plant_apply(p, q, a, om, noise ? noise + (size_t)b * 6 : nullptr);
#pragma unroll
    for (int i = 0; i < 6; ++i) state[(size_t)b * 6 + i] = q[i];
}

// ---- closed-loop failure policies of the three drivers, fused with the plant update ----------------------
// success (status <= acceptable): u = inputs[:, 0], last = u, consecutive = 0.  On failure (failure_count++,
// consecutive++):
//   TT_POLICY_TRACK  simulation.py:519-527        u = inputs[:, 0] as returned (no failure branch)
//   TT_POLICY_NMPC   simulation_nmpc.py:206-216   u = 0, last = 0; consecutive > 20: stop
//   TT_POLICY_FUZZY  simulation_fuzzy.py:207-221  u = last; consecutive > 15: u = 0; consecutive > 30: stop
// A stopped instance (the reference's `break`, before update) keeps its state and applies nothing from then on.
__global__ void __launch_bounds__(kThreads) policy_plant_kernel(int B, tt_plant p, int policy, double* __restrict__ state,
                                                                const double* __restrict__ u, long long u_stride,
                                                                const int* __restrict__ status, double* __restrict__ u_last,
                                                                int* __restrict__ consec, int* __restrict__ fails,
                                                                int* __restrict__ active, const double* __restrict__ noise,
                                                                double* __restrict__ u_applied) {
    const int b = blockIdx.x * kThreads + threadIdx.x;
    if (b >= B) return;
    double a = 0.0, om = 0.0;
    bool go = active[b] != 0;
    if (go) {
        if (status[b] <= TT_ACCEPTABLE) {
            a = u[b * u_stride];
            om = u[b * u_stride + 1];
            u_last[(size_t)b * 2] = a;
            u_last[(size_t)b * 2 + 1] = om;
            consec[b] = 0;
        } else {
            fails[b] += 1;
            const int cf = consec[b] + 1;
            consec[b] = cf;
            if (policy == TT_POLICY_NMPC) {
                u_last[(size_t)b * 2] = u_last[(size_t)b * 2 + 1] = 0.0;
                if (cf > 20) go = false;
            } else if (policy == TT_POLICY_FUZZY) {
                a = u_last[(size_t)b * 2];
                om = u_last[(size_t)b * 2 + 1];
                if (cf > 15) { a = 0.0; om = 0.0; }
                if (cf > 30) go = false;
            } else {
                a = u[b * u_stride];
                om = u[b * u_stride + 1];
            }
        }
        if (!go) { a = 0.0; om = 0.0; active[b] = 0; }
    }
    if (u_applied) { u_applied[(size_t)b * 2] = a; u_applied[(size_t)b * 2 + 1] = om; }
    if (!go) return;
    double q[6];
#pragma unroll
    for (int i = 0; i < 6; ++i) q[i] = state[(size_t)b * 6 + i];
    plant_apply(p, q, a, om, noise ? noise + (size_t)b * 6 : nullptr);
#pragma unroll
    for (int i = 0; i < 6; ++i) state[(size_t)b * 6 + i] = q[i];
}

// ---- fuzzy weights (mpc_control_fuzzy.py:90-119) from the measured state and the window's first reference
// speed: hitch-angle severity h = min(|psi| / 0.35, 1), reversing (ref v or v < -0.1) scales by 1.1 / 1.2,
// weights clipped to [1, 3.5].  w[b] = (q0..q5, r0, r1).
__global__ void __launch_bounds__(kThreads) fuzzy_kernel(int B, int N, const double* __restrict__ x,
                                                         const double* __restrict__ xref, double* __restrict__ w) {
    const int b = blockIdx.x * kThreads + threadIdx.x;
    if (b >= B) return;
    const double psi = x[(size_t)b * 6 + 3], v = x[(size_t)b * 6 + 5];
    const double ref_v = xref[(size_t)b * (N + 1) * 6 + 5];
    const double h = fmin(fabs(psi) / 0.35, 1.0);
    const bool reversing = (ref_v < -0.1) || (v < -0.1);
    double hitch = 1.0 + 2.0 * h, steer = 1.0 + 1.2 * h, steer_rate = 1.0 + 1.5 * h;
    if (reversing) { hitch *= 1.1; steer *= 1.1; steer_rate *= 1.2; }
    auto clip = [](double t) { return fmin(fmax(t, 1.0), 3.5); };
    double* o = w + (size_t)b * 8;
    o[0] = 1.0; o[1] = 1.0;
    o[2] = clip(fmax(1.0, steer));
    o[3] = clip(fmax(1.0, hitch));
    o[4] = clip(fmax(1.0, steer));
    o[5] = 1.0;
    o[6] = 1.0;
    o[7] = clip(fmax(1.0, steer_rate));
}

// ---- NMPC warm start: z_guess = have ? shift(last) : [xr_0, ur_0, ..., xr_N] ----------------------------
// shift (mpc_control_nmpc.py:69-88): stages 1..N-1 move to 0..N-2; the last stage is built from
// last[-8:-2] / last[-2:] (bug_compatible: [u_{N-1}, x_N[0:4]] and x_N[4:6]) or the intended x_N / u_{N-1}.
__global__ void __launch_bounds__(kThreads) warm_kernel(int B, int N, const double* __restrict__ last,
                                                        const int* __restrict__ have, const double* __restrict__ xr,
                                                        const double* __restrict__ ur, int bug_compatible,
                                                        double* __restrict__ zg) {
    const int n = 8 * N + 6;
    const long long t = (long long)blockIdx.x * kThreads + threadIdx.x;
    if (t >= (long long)B * n) return;
    const int b = (int)(t / n), e = (int)(t % n);
    const double* L = last + (size_t)b * n;
    double v;
    if (!have[b]) {
        const int k = e / 8, r = e % 8;   // reference-copy guess (mpc_control_nmpc.py:60-67)
        v = k == N ? xr[((size_t)b * (N + 1) + N) * 6 + r]
                   : (r < 6 ? xr[((size_t)b * (N + 1) + k) * 6 + r] : ur[((size_t)b * N + k) * 2 + (r - 6)]);
    } else if (e < 8 * (N - 1)) {
        v = L[e + 8];
    } else {
        const int r = e - 8 * (N - 1);    // 0..13: last_state(6), last_input(2), last_state(6)
        const int rs = r < 6 ? r : (r < 8 ? 6 + (r - 6) : r - 8);
        if (bug_compatible) {
            v = rs < 6 ? L[n - 8 + rs] : L[n - 2 + (rs - 6)];
        } else {
            v = rs < 6 ? L[8 * N + rs] : L[8 * (N - 1) + 6 + (rs - 6)];
        }
    }
    zg[t] = v;
}

// last <- pack(X, U) where the solve succeeded (status <= acceptable); have[b] |= success
__global__ void __launch_bounds__(kThreads) record_kernel(int B, int N, const double* __restrict__ X,
                                                          const double* __restrict__ U, const int* __restrict__ status,
                                                          double* __restrict__ last, int* __restrict__ have) {
    const int n = 8 * N + 6;
    const long long t = (long long)blockIdx.x * kThreads + threadIdx.x;
    if (t >= (long long)B * n) return;
    const int b = (int)(t / n), e = (int)(t % n);
    if (status[b] > TT_ACCEPTABLE) return;
    const int k = e / 8, r = e % 8;
    last[t] = k == N ? X[((size_t)b * (N + 1) + N) * 6 + r]
                     : (r < 6 ? X[((size_t)b * (N + 1) + k) * 6 + r] : U[((size_t)b * N + k) * 2 + (r - 6)]);
    if (e == 0) have[b] = 1;
}

// ---- do_interpolation (simulation.py:201-218): linear states, zero-order-hold inputs, factor n --------
__global__ void __launch_bounds__(kThreads) interp_kernel(int B, int Np, int n, const double* __restrict__ sx,
                                                          const double* __restrict__ su, double* __restrict__ dx,
                                                          double* __restrict__ du) {
#pragma clang fp contract(off)
    const int Nn = n * Np;
    const long long t = (long long)blockIdx.x * kThreads + threadIdx.x;
    if (t >= (long long)B * (Nn + 1)) return;
    const int b = (int)(t / (Nn + 1)), c = (int)(t % (Nn + 1));
    const double* S = sx + (size_t)b * (Np + 1) * 6;
    double* D = dx + ((size_t)b * (Nn + 1) + c) * 6;
    if (c == Nn) {
#pragma unroll
        for (int i = 0; i < 6; ++i) D[i] = S[(size_t)Np * 6 + i];
        return;
    }
    const int k = c / n, m = c % n;
    const double tt = (double)m / (double)n;
#pragma unroll
    for (int i = 0; i < 6; ++i) D[i] = (1 - tt) * S[(size_t)k * 6 + i] + tt * S[(size_t)(k + 1) * 6 + i];
    const double* Su = su + ((size_t)b * Np + k) * 2;
    double* Du = du + ((size_t)b * Nn + c) * 2;
    Du[0] = Su[0];
    Du[1] = Su[1];
}

int launched(const char* where) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        fprintf(stderr, "ttmpc: %s launch failed: %s\n", where, hipGetErrorString(e));
        return -EIO;
    }
    return 0;
}

}  // namespace

extern "C" {

int tt_sim_window_device(int B, int N, int k, int Np, const double* plan_x, const double* plan_u, int per_instance,
                         const double* state, const double* meas_noise, double* x_meas, double* xref, double* uref,
                         void* stream) {
    if (B < 0 || N < 1 || Np < 1 || k < 0 || !plan_x || !plan_u || !xref || !uref || (x_meas && !state))
        return -EINVAL;
    if (B == 0) return 0;
    const long long tot = (long long)B * (N + 1);
    hipLaunchKernelGGL(sim_window_kernel, dim3(grid_for(tot)), dim3(kThreads), 0, (hipStream_t)stream, B, N, k, Np,
                       plan_x, plan_u, per_instance, state, meas_noise, x_meas, xref, uref);
    return launched("sim_window_kernel");
}

int tt_sim_window_indexed_device(int B, int N, const int* ks, const int* step, int Np, const double* plan_x,
                                 const double* plan_u, int per_instance, const double* state, const double* noise_all,
                                 double* x_meas, double* xref, double* uref, void* stream) {
    if (B < 0 || N < 1 || Np < 1 || !ks || !step || !plan_x || !plan_u || !state || !x_meas || !xref || !uref)
        return -EINVAL;
    if (B == 0) return 0;
    const long long tot = (long long)B * (N + 1);
    hipLaunchKernelGGL(sim_window_indexed_kernel, dim3(grid_for(tot)), dim3(kThreads), 0, (hipStream_t)stream, B, N,
                       ks, step, Np, plan_x, plan_u, per_instance, state, noise_all, x_meas, xref, uref);
    return launched("sim_window_indexed_kernel");
}

int tt_sim_log_advance_device(int B, int* step, const double* state, const double* u_applied, const int* status,
                              const int* iters, const int* flag, double* S, double* Ua, int* Ss, int* Si, int* Sc,
                              void* stream) {
    if (B < 0 || !step || !state || !u_applied || !status || !S || !Ua || !Ss || !Si || !Sc) return -EINVAL;
    if (B > 0) {
        hipLaunchKernelGGL(sim_log_kernel, dim3(grid_for(B)), dim3(kThreads), 0, (hipStream_t)stream, B, step, state,
                           u_applied, status, iters, flag, S, Ua, Ss, Si, Sc);
        const int rc = launched("sim_log_kernel");
        if (rc) return rc;
    }
    hipLaunchKernelGGL(sim_advance_kernel, dim3(1), dim3(1), 0, (hipStream_t)stream, step);
    return launched("sim_advance_kernel");
}

int tt_collision_device(int B, int K, const double* poses, long long stride_b, int stride_k, const double* obstacles,
                        int M, const tt_plant* p, int* flag, void* stream) {
    if (B < 0 || K < 1 || !poses || !p || !flag || M < 0 || (M > 0 && !obstacles) || stride_k < 4) return -EINVAL;
    if (B == 0) return 0;
    hipLaunchKernelGGL(collision_kernel, dim3(B), dim3(64), 0, (hipStream_t)stream, B, K, stride_b, stride_k, poses,
                       obstacles, M, p->L1, p->L2, p->Mh, p->W1, p->W2, flag);
    return launched("collision_kernel");
}

int tt_plant_update_noise_device(int B, const tt_plant* p, double* state, const double* u, long long u_stride,
                                 const int* status, int zero_on_fail, const double* state_noise, double* u_applied,
                                 void* stream) {
    if (B < 0 || !p || !state || !u || u_stride < 2) return -EINVAL;
    if (B == 0) return 0;
    hipLaunchKernelGGL(plant_kernel, dim3(grid_for(B)), dim3(kThreads), 0, (hipStream_t)stream, B, *p, state, u,
                       u_stride, status, zero_on_fail, state_noise, u_applied);
    return launched("plant_kernel");
}

int tt_plant_update_device(int B, const tt_plant* p, double* state, const double* u, long long u_stride,
                           const int* status, int zero_on_fail, double* u_applied, void* stream) {
    return tt_plant_update_noise_device(B, p, state, u, u_stride, status, zero_on_fail, nullptr, u_applied, stream);
}

int tt_policy_plant_noise_device(int B, const tt_plant* p, int policy, double* state, const double* u,
                                 long long u_stride, const int* status, double* u_last, int* consecutive, int* failures,
                                 int* active, const double* state_noise, double* u_applied, void* stream) {
    if (B < 0 || !p || !state || !u || u_stride < 2 || !status || !u_last || !consecutive || !failures || !active ||
        policy < TT_POLICY_TRACK || policy > TT_POLICY_FUZZY)
        return -EINVAL;
    if (B == 0) return 0;
    hipLaunchKernelGGL(policy_plant_kernel, dim3(grid_for(B)), dim3(kThreads), 0, (hipStream_t)stream, B, *p, policy,
                       state, u, u_stride, status, u_last, consecutive, failures, active, state_noise, u_applied);
    return launched("policy_plant_kernel");
}

int tt_policy_plant_device(int B, const tt_plant* p, int policy, double* state, const double* u, long long u_stride,
                           const int* status, double* u_last, int* consecutive, int* failures, int* active,
                           double* u_applied, void* stream) {
    return tt_policy_plant_noise_device(B, p, policy, state, u, u_stride, status, u_last, consecutive, failures, active,
                                        nullptr, u_applied, stream);
}

int tt_fuzzy_weights_device(int B, int N, const double* x, const double* xref, double* wq_wr, void* stream) {
    if (B < 0 || N < 1 || !x || !xref || !wq_wr) return -EINVAL;
    if (B == 0) return 0;
    hipLaunchKernelGGL(fuzzy_kernel, dim3(grid_for(B)), dim3(kThreads), 0, (hipStream_t)stream, B, N, x, xref, wq_wr);
    return launched("fuzzy_kernel");
}

int tt_warm_start_device(int B, int N, const double* last, const int* have, const double* xref, const double* uref,
                         int bug_compatible, double* z_guess, void* stream) {
    if (B < 0 || N < 1 || !last || !have || !xref || !uref || !z_guess) return -EINVAL;
    if (B == 0) return 0;
    hipLaunchKernelGGL(warm_kernel, dim3(grid_for((long long)B * (8 * N + 6))), dim3(kThreads), 0,
                       (hipStream_t)stream, B, N, last, have, xref, uref, bug_compatible, z_guess);
    return launched("warm_kernel");
}

int tt_record_solution_device(int B, int N, const double* x_out, const double* u_out, const int* status, double* last,
                              int* have, void* stream) {
    if (B < 0 || N < 1 || !x_out || !u_out || !status || !last || !have) return -EINVAL;
    if (B == 0) return 0;
    hipLaunchKernelGGL(record_kernel, dim3(grid_for((long long)B * (8 * N + 6))), dim3(kThreads), 0,
                       (hipStream_t)stream, B, N, x_out, u_out, status, last, have);
    return launched("record_kernel");
}

int tt_interpolate_device(int B, int Np, int factor, const double* state_traj, const double* input_traj,
                          double* state_out, double* input_out, void* stream) {
    if (B < 0 || Np < 1 || factor < 1 || !state_traj || !input_traj || !state_out || !input_out) return -EINVAL;
    if (B == 0) return 0;
    hipLaunchKernelGGL(interp_kernel, dim3(grid_for((long long)B * (factor * Np + 1))), dim3(kThreads), 0,
                       (hipStream_t)stream, B, Np, factor, state_traj, input_traj, state_out, input_out);
    return launched("interp_kernel");
}

}  // extern "C"
