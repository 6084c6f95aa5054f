// Batched OBCA trajectory optimisation / MPC+OBCA on gfx950 (MI355X / CDNA4).
//
// NLP (reference python-files/, restated; see oracle/c/tt_obca.c for the CPU statement):
//   variables   x_k, u_k, mu_k (8M), lam_k (8M) >= 0             trajectory_optimization.py:55-91
//   dynamics    x_0 = x_init, x_{k+1} = x_k + dt f(x_k, u_k)         trajectory_planning.py:28-36
//   OBCA rows   per stage k, obstacle i, body b (truck/trailer):     trajectory_optimization.py:93-166
//     d1 = g'mu - (A p(x) - b)'lam + d_min <= 0,  d2,d3 = G'mu + R(x)'A'lam in [-1e-5, 1e-5],
//     d4 = ||A'lam|| - 1 <= 0                       (bodies: truck_trailer_model.py:31-72)
//   plan  : goal cost, terminal 100 Q, |x_N - g| <= 1e-2               trajectory_optimization.py:168-183
//   track : reference tracking cost, Q_f = Q                           mpc_control_obs.py:31-41
//
// Solver: the IPOPT restatement of the oracle (IPOPT defaults, trajectory_optimization.py:195-205):
// slack-form barrier method (tol 1e-8, acceptable 1e-6 x 15, monotone mu, bound_relax 1e-8, bound_push
// 1e-2, kappa_sigma 1e10, exact Hessian), least-squares constraint multipliers at the start
// (constr_mult_init_max 1000), delta_w inertia correction, filter line search with up to 4 second-order
// corrections, the soft restoration phase and the MinC_1Nrm feasibility restoration phase (elastic
// p/n per constraint row, rho 1000, proximity sqrt(mu_R) ||D_R (xbar - xbar_R)||^2; the dynamics rows
// become soft, so its Riccati sweep eliminates P~ = P - P Y P with Y = S (I + S P S)^-1 S).
//
// One workgroup (4 waves) per instance.  Work split:
//   * stage-parallel phases (linearisation, optimality error, block elimination + stage Hessians,
//     block step recovery, fraction-to-boundary, trial evaluation, updates, restoration entry/exit):
//     thread k owns stage k, its 6 dynamics rows and its 2M OBCA blocks (obstacle x body).  Each block
//     (8 duals, 4 rows) couples only to (X, Y, theta, psi) of its stage; its mu part is diagonal and its
//     lam part a 4x4 SPD block, so the elimination is a 4x4 Cholesky + a 4x4 Schur complement
//     T = E + Y'Y (never C'DC: D reaches 1e10 on the +-1e-5 range rows and that product cancels).
//   * serial phases (Riccati backward sweep over the 6x6 stage blocks, forward sweep): wave 0, lane
//     (i,j) owns entry (i,j) of the 6x6 products; P and PA tiles in LDS.
//   * the factor and residual passes' block parts run over the flat block index f = j (N + 1) + k in chunks of T blocks
//     (factor_block / nres_block, each writing a contribution record its stage adds in block order), and helper
//     workgroups -- one per CU, launched after the B instances' -- run chunks of the instances still solving once
//     CUs are idle (run_pass / helper_main): the C4 tail's handful of max_iter instances spread over the idle GPU.
// Workspace: per instance in HBM, stage fields [f][k] and block fields [f][j][k] so that the lanes of a
// stage-parallel phase (consecutive k) read consecutive addresses.
#include <math.h>

#include "tt_kernel.hpp"
#include "tt_trig.hpp"

// FMA contraction within a source expression only (the C rule), never across statements: the backend's
// cross-statement fusion depends on how many uses a product has in the inlined context, so the same block
// elimination could round differently in phase_factor and in the recovery passes that recompute it
// (block_refactor); with contraction fixed by the source they are bitwise the same computation.
#pragma clang fp contract(on)


namespace ttmpc {
namespace {

constexpr int T = kObcaThreads;
constexpr double RELAX = 1e-8;
constexpr double EPS = 2.220446049250313e-16;
constexpr double RHO = 1000.0;                 // resto_penalty_parameter
constexpr double KAPPA_RESTO = 0.9;            // required_infeasibility_reduction
constexpr double BOUND_MULT_RESET = 1000.0;    // bound_mult_reset_threshold
constexpr double CONSTR_MULT_INIT_MAX = 1000.0;
constexpr double SOFT_RESTO_FACTOR = 0.9999;   // soft_resto_pderror_reduction_factor
constexpr int MAX_SOFT_RESTO = 10;             // max_soft_resto_iters

enum : int {
    S_X = 0, S_U = 6, S_ZLX = 8, S_ZUX = 14, S_ZLU = 20, S_ZUU = 22, S_YC = 24,
    S_GX = 30, S_GU = 36, S_C = 38, S_AJ = 44, S_WD = 53, S_QT = 60, S_QV = 81, S_RT = 87, S_RV = 90,
    S_P = 92, S_PV = 113, S_K = 119, S_KF = 131, S_GI = 133,
    // iterative refinement: the elastic-pair constants of the correction solve (dynamics rows; restoration phase)
    S_OP = 136, S_ON = 142,
    // step buffers: 0 the Newton step, 1 the second-order correction, 2 (dx, du, y+ only) a refinement correction
    S_DX = 148, S_DU = 166, S_YCP = 172,
    S_CT = 190, S_CR = 196,
    // restoration phase: elastic pairs of the 6 dynamics rows of the stage (and their steps, 2 buffers),
    // S = sqrt(E) of those rows, Y = S M^-1 S of the soft Riccati, the effective row residual, the
    // reference point and D_R^2, the saved original bound multipliers, the stored acceptable point and the
    // soft-restoration snapshot (x u zLx zUx zLu zUu yc)
    S_PR = 202, S_NR = 208, S_ZP = 214, S_ZN = 220, S_DP = 226, S_DN = 238, S_SD = 250, S_Y = 256,
    S_CE = 277, S_XR = 283, S_UR = 289, S_DRX = 291, S_DRU = 297, S_SZ = 299, S_XACC = 315, S_UACC = 321,
    S_SNAP = 323, S_END = 353
};
static_assert(S_END == kObcaStageFields, "stage field count");
enum : int {
    B_W = 0, B_ZW = 8, B_S = 16, B_VL = 20, B_VU = 24, B_YD = 28, B_D = 32, B_DW = 36, B_DS = 52, B_YP = 60,
    B_DT = 68, B_DR = 72,
    // restoration phase: elastic pairs of the 4 rows (+ steps, 2 buffers), reference duals / slacks and
    // D_R^2, saved multipliers, acceptable point, soft-restoration snapshot (w zw s vL vU yd)
    B_PR = 76, B_NR = 80, B_ZP = 84, B_ZN = 88, B_DP = 92, B_DN = 100, B_WR = 108, B_DRW = 116, B_SR = 124,
    B_SZW = 128, B_SVL = 136, B_SVU = 140, B_WACC = 144, B_SNAP = 152,
    // iterative refinement: slack and elastic-pair constants of the correction solve (read by its recovery)
    B_OS = 184, B_OP = 188, B_ON = 192,
    // the right-hand side of a correction solve (phase_nres prep -> NR_CORR): fw 8 | zf_lam 4 | t 4.  The elimination
    // itself is recomputed by every pass that needs it (block_refactor), not stored.
    B_FR = 196,
    // phase_nres: a block's contribution record (nres_block -> the stage part)
    B_CB = 212, B_END = 229
};
enum : int { FR_FW = 0, FR_ZFL = 8, FR_T = 12, FR_END = 16 };
static_assert(B_FR + FR_END == B_CB, "factor record");
static_assert(B_END == kObcaBlockFields, "block field count");

// packed symmetric 6x6 (upper) index
__host__ __device__ constexpr int sy6(int i, int j) {
    return i <= j ? i * 6 - (i * (i - 1)) / 2 + (j - i) : j * 6 - (j * (j - 1)) / 2 + (i - j);
}
// packed lower 4x4 index
__host__ __device__ constexpr int lo4(int i, int j) { return i * (i + 1) / 2 + j; }

// dt*J nonzeros: 0:(0,2) 1:(0,5) 2:(1,2) 3:(1,5) 4:(2,4) 5:(2,5) 6:(3,3) 7:(3,4) 8:(3,5)   (A = I + dt J)
// dynamics curvature nonzeros (symmetric): 0:(2,2) 1:(2,5) 2:(3,3) 3:(3,4) 4:(3,5) 5:(4,4) 6:(4,5)

// ---------------- wave / workgroup reductions (DPP inside 16-lane rows, readlane across rows) ----------
template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_update_dpp((int)(b & 0xffffffffll), (int)(b & 0xffffffffll), CTRL, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp((int)(b >> 32), (int)(b >> 32), CTRL, 0xF, 0xF, false);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
__device__ __forceinline__ double readlane_d(double v, int l) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}
enum { R_SUM = 0, R_MAX = 1, R_MIN = 2 };
__device__ __forceinline__ double rop(int op, double a, double b) {
    return op == R_SUM ? a + b : op == R_MAX ? fmax(a, b) : fmin(a, b);
}
__device__ __forceinline__ double wave_red(double v, int op) {
    v = rop(op, v, dppd<0xB1>(v));
    v = rop(op, v, dppd<0x4E>(v));
    v = rop(op, v, dppd<0x141>(v));
    v = rop(op, v, dppd<0x140>(v));
    return rop(op, rop(op, readlane_d(v, 0), readlane_d(v, 16)), rop(op, readlane_d(v, 32), readlane_d(v, 48)));
}

__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
}

struct Shared {
    double red[4][16];
    // final-row (plan mode) state, owned by the thread of stage N
    double sf[6], vLf[6], vUf[6], ydf[6], df[6], dsf[2][6], ydpf[2][6], dft[6], dfr[6], Dsf[6], Dfe[6], rf[6];
    // their restoration-phase elastic pairs, saved multipliers and the soft-restoration snapshot
    double pf[6], nf[6], zpf[6], znf[6], dpf[2][6], dnf[2][6], sfR[6], svLf[6], svUf[6], snapf[24];
    // iterative refinement: the final rows' slack / elastic-pair constants of the correction solve
    double osf[6], opf[6], onf[6];
    // filters: [0] original problem, [1] restoration problem
    double fth[2][kObcaMaxFilter], fph[2][kObcaMaxFilter];
    int nfl[2];
    int R;       // 1 while in the restoration phase
    int lsq;     // 1 while assembling the least-squares multiplier system
    double zeta; // restoration proximity weight sqrt(mu_R)
    double dc;   // delta_c (= delta_d) of the current factorisation: -dc on every constraint row's diagonal
    int flag;    // the Riccati sweep's factorisation code (F_OK / F_MANY / F_ZERO)
    unsigned long long stamp[kObcaPhases];
    unsigned long long t0;
    // helper workgroups (run_pass / helper_main): passes published, the claimed chunk / instance, exit and failure flags,
    // and a helper's copy of the pass parameters
    unsigned hep;
    int hcur, hb, hexit, hfail, hp_pk;
    double hp_mu, hp_dw, hp_tau;
};
typedef __attribute__((address_space(3))) Shared LShared;  // the kernel's Shared block, LDS-addressed


// diagnostic phase clock (thread 0, shader cycles); a no-op unless the caller passed a stamps buffer
__device__ __forceinline__ void stamp(LShared& sh, bool on, int ph) {
    if (on && threadIdx.x == 0) {
        const unsigned long long t = clock64();
        sh.stamp[ph] += t - sh.t0;
        sh.t0 = t;
    }
}
// diagnostic event counter (thread 0)
__device__ __forceinline__ void count(LShared& sh, bool on, int ev) {
    if (on && threadIdx.x == 0) sh.stamp[ev] += 1;
}

// workgroup reduction of NV values with per-value op; result uniform in every thread, fixed order
template <int NV>
__device__ __forceinline__ void wg_reduce(LShared& sh, double (&v)[NV], const int (&op)[NV]) {
    static_assert(NV <= 16, "Shared::red holds 16 values per wave");
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double r[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) r[i] = wave_red(v[i], op[i]);
    __syncthreads();
    if (lane == 0) {
#pragma unroll
        for (int i = 0; i < NV; ++i) sh.red[wave][i] = r[i];
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < NV; ++i) v[i] = rop(op[i], rop(op[i], sh.red[0][i], sh.red[1][i]), rop(op[i], sh.red[2][i], sh.red[3][i]));
}

// 1/x by v_rcp_f64 + two Newton steps
__device__ __forceinline__ double frcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}

// 1/x for the barrier terms: IEEE division (the oracle divides; round 3's shared reciprocals cost the GPU-vs-oracle
// agreement and were removed in round 4)
__device__ __forceinline__ double inv(double x) {
    return 1.0 / x;
}


// a if p else b by bit masks, both operands computed in every lane (the empty asm): no divergent branch, whatever the
// backend would make of a select on a lane-dependent condition
__device__ __forceinline__ double bsel(bool p, double a, double b) {
    asm("" : "+v"(a), "+v"(b));
    const unsigned long long m = 0ull - (unsigned long long)p;
    return __longlong_as_double((long long)(((unsigned long long)__double_as_longlong(a) & m) |
                                            ((unsigned long long)__double_as_longlong(b) & ~m)));
}
// v_q of six values computed in every lane, as v_cndmask selects: the empty asm makes each operand a value computed before
// the select, so the backend cannot sink the arithmetic into lane-divergent branches (a serial sweep paid an exec-masked
// branch per operand and stage for that)
__device__ __forceinline__ double sel6(int q, double v0, double v1, double v2, double v3, double v4, double v5) {
    asm("" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5));
    // bit masks instead of a select chain (which the backend turns into a cascade of divergent branches on q)
    unsigned long long r = (unsigned long long)__double_as_longlong(v0);
    const double v[5] = {v1, v2, v3, v4, v5};
#pragma unroll
    for (int i = 0; i < 5; ++i) {
        const unsigned long long m = 0ull - (unsigned long long)(q == i + 1);
        r = ((unsigned long long)__double_as_longlong(v[i]) & m) | (r & ~m);
    }
    return __longlong_as_double((long long)r);
}

// row_newbcast:l (gfx90a+ DPP on a 64-bit move): every lane of a 16-lane row receives lane l of that row
template <int L_>
__device__ __forceinline__ double rowbc(double v) {
    const long long b = __double_as_longlong(v);
    return __longlong_as_double(__builtin_amdgcn_update_dpp(b, b, 0x150 + L_, 0xF, 0xF, false));
}

// sum of logs as log(prod of mantissas) + (sum of exponents) ln 2
struct LogSum {
    double m = 1.0;
    int e = 0;
    int n = 0;
    __device__ __forceinline__ void add(double s) {
        int ex;
        m *= frexp(s, &ex);
        e += ex;
        if (++n == 24) {  // renormalise before the mantissa product can underflow (0.5^24 >> DBL_MIN)
            int e2;
            m = frexp(m, &e2);
            e += e2;
            n = 0;
        }
    }
    __device__ __forceinline__ double value() const { return log(m) + (double)e * 0.69314718055994530942; }
};

// ---------------- per-instance context ----------------
typedef __attribute__((address_space(1))) double gdouble;  // global-qualified: global_load / global_store
// the launch arguments, copied once into LDS: the phases read Q, R, bounds and obstacles with ds_read
// broadcasts instead of flat loads from the kernel's private copy of the by-value argument
typedef __attribute__((address_space(3))) const ObcaArgs LArgs;
struct Ctx {
    LArgs* a;
    gdouble* ws;
    double* lds;  // dynamic LDS for the staged sweeps, or nullptr (sweeps read the HBM workspace)
    __attribute__((address_space(3))) double* slab;  // block-phase slabs (dynamic LDS, kSlab x T; thread t at slab + t)
    int N, NP, nbk, tid, b;
    bool pd;                // round 2's positive-definite block test instead of the exact block inertia (A/B)
    bool refine;            // IPOPT's iterative refinement of every step solve
    double dt;
    double xl[6], xu[6], ul[2], uu[2];
    int hx, hu;             // bit i: finite lower (i) / upper (8+i) bound
    double rlo, rhi;        // relaxed bounds of the range rows d2, d3
    double fL, fU;          // final box
    const double* tgt_x;    // plan: x_goal; track: xref of this instance
    const double* tgt_u;    // track: uref
    // Field rows are uniform (scalar) offsets of the instance's workspace and k only ever adds a 32-bit lane offset,
    // so every access is one global_load / global_store with an SGPR base and a VGPR byte offset (the "saddr" form)
    // instead of 64-bit address arithmetic on the VALU per access.
    __device__ __forceinline__ gdouble& at(size_t row, int k) const {
        typedef __attribute__((address_space(1))) char gchar;
        // the phases are separate (noinline) functions that receive the context in VGPRs: readfirstlane tells the
        // compiler that the base and the stride are wave-uniform again
        const unsigned long long wsu = (unsigned long long)ws;
        const unsigned lo = __builtin_amdgcn_readfirstlane((unsigned)wsu), hi = __builtin_amdgcn_readfirstlane((unsigned)(wsu >> 32));
        gdouble* const base = (gdouble*)(((unsigned long long)hi << 32) | lo);
        const size_t np = (size_t)(unsigned)__builtin_amdgcn_readfirstlane(NP);
        return *(gdouble*)((gchar*)(base + row * np) + (unsigned)k * 8u);
    }
    __device__ __forceinline__ gdouble& S(int f, int k) const { return at((size_t)f, k); }
    __device__ __forceinline__ gdouble& B(int f, int j, int k) const {
        return at((size_t)S_END + (size_t)f * (size_t)(unsigned)__builtin_amdgcn_readfirstlane(nbk) + j, k);
    }
    __device__ __forceinline__ bool hlx(int i) const { return (hx >> i) & 1; }
    __device__ __forceinline__ bool hux(int i) const { return (hx >> (8 + i)) & 1; }
    __device__ __forceinline__ bool hlu(int i) const { return (hu >> i) & 1; }
    __device__ __forceinline__ bool huu(int i) const { return (hu >> (8 + i)) & 1; }
    __device__ __forceinline__ bool plan() const { return a->mode == OBCA_PLAN; }
    // row r of a block: lower bound finite only for the range rows 1, 2
    __device__ __forceinline__ bool hrl(int r) const { return r == 1 || r == 2; }
    __device__ __forceinline__ double rL(int r) const { return (r == 1 || r == 2) ? rlo : -INFINITY; }
    __device__ __forceinline__ double rU(int r) const { return (r == 1 || r == 2) ? rhi : RELAX; }
};

// The workspace as one phase sees it: base and strides read once per phase through readfirstlane, so they sit in
// SGPRs (a noinline phase receives the context through memory, i.e. in VGPRs) and every field access is an SGPR base
// plus this lane's 32-bit byte offset -- one global_load / global_store, no per-access VALU address arithmetic.
struct WsView {
    gdouble* base;
    size_t np, bstart, nbk;
    __device__ __forceinline__ gdouble& at(size_t row, int k) const {
        typedef __attribute__((address_space(1))) char gchar;
        return *(gdouble*)((gchar*)(base + row * np) + (unsigned)k * 8u);
    }
    __device__ __forceinline__ gdouble& S(int f, int k) const { return at((size_t)f, k); }
    __device__ __forceinline__ gdouble& B(int f, int j, int k) const { return at(bstart + (size_t)f * nbk + j, k); }
};
__device__ __forceinline__ WsView ws_view(const Ctx& c) {
    const unsigned long long w = (unsigned long long)c.ws;
    WsView v;
    v.base = (gdouble*)(((unsigned long long)__builtin_amdgcn_readfirstlane((unsigned)(w >> 32)) << 32) |
                        (unsigned)__builtin_amdgcn_readfirstlane((unsigned)w));
    v.np = (size_t)(unsigned)__builtin_amdgcn_readfirstlane(c.NP);
    v.nbk = (size_t)(unsigned)__builtin_amdgcn_readfirstlane(c.nbk);
    v.bstart = (size_t)S_END;
    return v;
}

// ---------------- model: truck_trailer_model.py:8-24 ----------------
__device__ __forceinline__ void model_f(LArgs& a, const double* x, const double* u, double* fo) {
    const double th = x[2], psi = x[3], phi = x[4], v = x[5];
    double sth, cth, sps, cps, t, cphi;
    sincos2_tancos(th, sth, cth, psi, sps, cps, phi, t, cphi);
    (void)cphi;
    fo[0] = v * cth;
    fo[1] = v * sth;
    fo[2] = v * t / a.L1;
    fo[3] = -v * t / a.L1 * (1.0 + a.Mh / a.L2 * cps) - v * sps / a.L2;
    fo[4] = u[1];
    fo[5] = u[0];
}

// dt*J nonzeros (9) and the dynamics curvature -dt sum_i y_i d2 f_i (7 nonzeros)
__device__ __forceinline__ void model_lin(LArgs& a, const double* x, const double* y, double* dj, double* wd) {
    const double th = x[2], psi = x[3], phi = x[4], v = x[5];
    const double L1 = a.L1, L2 = a.L2, M = a.Mh, dt = a.dt;
    double sn, cs, sp, cp, t, cphi;
    sincos2_tancos(th, sn, cs, psi, sp, cp, phi, t, cphi);
    const double c2 = 1.0 / (cphi * cphi), k = 1.0 + M / L2 * cp;
    dj[0] = dt * (-v * sn);
    dj[1] = dt * cs;
    dj[2] = dt * (v * cs);
    dj[3] = dt * sn;
    dj[4] = dt * (v * c2 / L1);
    dj[5] = dt * (t / L1);
    dj[6] = dt * (v * t * M * sp / (L1 * L2) - v * cp / L2);
    dj[7] = dt * (-v * c2 / L1 * k);
    dj[8] = dt * (-t / L1 * k - sp / L2);
    const double s = -dt;
    wd[0] = s * (y[0] * (-v * cs) + y[1] * (-v * sn));
    wd[1] = s * (y[0] * (-sn) + y[1] * cs);
    wd[2] = s * (y[3] * (v * t * M * cp / (L1 * L2) + v * sp / L2));
    wd[3] = s * (y[3] * (v * c2 * M * sp / (L1 * L2)));
    wd[4] = s * (y[3] * (t * M * sp / (L1 * L2) - cp / L2));
    wd[5] = s * (y[2] * (2 * v * t * c2 / L1) + y[3] * (-2 * v * t * c2 * k / L1));
    wd[6] = s * (y[2] * (c2 / L1) + y[3] * (-c2 * k / L1));
}

// ---------------- OBCA block geometry (truck_trailer_model.py:31-72, trajectory_optimization.py:32-53) --------
struct Geom {
    double p0, p1, dpt0, dpt1, dpp0, dpp1, ppt0, ppt1, ptp0, ptp1, ppp0, ppp1, ca, sa, angp, hl, hw;
};
// the stage's two body angles (theta, theta + psi): computed once per stage, shared by its 2M blocks
struct Trig {
    double st, ct, sa, ca;
};
__device__ __forceinline__ Trig stage_trig(const double* xk) {
    Trig t;
    sincos2(xk[2], t.st, t.ct, xk[2] + xk[3], t.sa, t.ca);
    return t;
}
__device__ __forceinline__ void body_geom(LArgs& a, const double* xk, int body, const Trig& tr, Geom& g) {
    const double st = tr.st, ct = tr.ct;
    if (body == 0) {
        const double h1 = 0.5 * a.L1;
        g.ca = ct; g.sa = st; g.angp = 0.0; g.hl = 0.5 * a.L1; g.hw = 0.5 * a.W1;
        g.p0 = xk[0] + h1 * ct; g.p1 = xk[1] + h1 * st;
        g.dpt0 = -h1 * st; g.dpt1 = h1 * ct;
        g.dpp0 = 0.0; g.dpp1 = 0.0;
        g.ppt0 = -h1 * ct; g.ppt1 = -h1 * st;
        g.ptp0 = g.ptp1 = g.ppp0 = g.ppp1 = 0.0;
    } else {
        const double h2 = 0.5 * a.L2, M = a.Mh;
        const double sa = tr.sa, ca = tr.ca;
        g.ca = ca; g.sa = sa; g.angp = 1.0; g.hl = 0.5 * a.L2; g.hw = 0.5 * a.W2;
        g.p0 = xk[0] - M * ct - h2 * ca; g.p1 = xk[1] - M * st - h2 * sa;
        g.dpt0 = M * st + h2 * sa; g.dpt1 = -M * ct - h2 * ca;
        g.dpp0 = h2 * sa; g.dpp1 = -h2 * ca;
        g.ppt0 = M * ct + h2 * ca; g.ppt1 = M * st + h2 * sa;
        g.ptp0 = h2 * ca; g.ptp1 = h2 * sa;
        g.ppp0 = h2 * ca; g.ppp1 = h2 * sa;
    }
}

// constraint values of block j (obstacle j>>1, body j&1)
__device__ __forceinline__ void blk_vals(LArgs& a, const double* xk, const Trig& tr, int j, const double* w, double* d) {
    Geom g;
    body_geom(a, xk, j & 1, tr, g);
    const auto* ob = a.obs + 4 * (j >> 1);
    const double ex = g.p0 - ob[0], ey = g.p1 - ob[1], hwo = 0.5 * ob[2], hho = 0.5 * ob[3];
    const double aa = w[4] - w[6], cc = w[5] - w[7];
    d[0] = g.hl * (w[0] + w[2]) + g.hw * (w[1] + w[3]) -
           ((ex - hwo) * w[4] + (ey - hho) * w[5] + (-ex - hwo) * w[6] + (-ey - hho) * w[7]) + a.dmin;
    d[1] = (w[0] - w[2]) + g.ca * aa + g.sa * cc;
    d[2] = (w[1] - w[3]) - g.sa * aa + g.ca * cc;
    d[3] = sqrt(aa * aa + cc * cc) - 1.0;
}

// Full block linearisation + elimination.  See the header comment and oracle/c/tt_obca.c:block_factor.
typedef __attribute__((address_space(3))) double lds_double;  // LDS-qualified: ds_read / ds_write

// per-thread LDS slab of the block phases: the 48 doubles of Yl, Zl, G (field stride T, conflict-free).  Kept in
// registers they were what the block elimination spilled to scratch, and every scratch reload waited behind
// the factor-record stores (one in-order vmcnt); ds_ reads wait on lgkmcnt only.
// W_{x lam} of the block (16 doubles) lives in the slab too (rows 48-63)
constexpr int kSlab = 64;
struct Blk {
    lds_double* m;                   // this thread's slab (Yl 0-15 | Zl 16-31 | G 32-47)
    __device__ __forceinline__ lds_double& Yl(int a, int r) const { return m[(a * 4 + r) * T]; }  // L^-1 Jw_lam'  [a][r]
    __device__ __forceinline__ lds_double& Zl(int a, int q) const { return m[(16 + a * 4 + q) * T]; }  // L^-1 W_lam x  [a][q]
    __device__ __forceinline__ lds_double& G(int r, int q) const { return m[(32 + r * 4 + q) * T]; }  // Y_lam' Z - Jx  [r][q]
    // linearisation
    double d[4];
    double jx0[4], e2, e3, angp;     // Jx rows 0..2 (row 3 = 0)
    double jw0[8], ca, sa, an, cn;   // Jw row 0 + the rotation/normal data of rows 1..3
    double hl, hw;
    double hxx22, hxx23, hxx33;
    __device__ __forceinline__ lds_double& H(int q, int a) const { return m[(48 + q * 4 + a) * T]; }  // W_{x lam} [q][a]
    double haa, hac, hcc;            // the lam-lam Hessian y4 T'H4T (LL before the elimination), see hll
    // elimination
    double idm[4];                   // 1 / (Sigma_mu + dw) (mu block is diagonal)
    double LL[10];                   // chol of the lam block (1/L_ii on the diagonal)
    double LT[10];                   // chol of T (1/L_ii on the diagonal)
    double D[4];                     // Sigma_s + dw of the 4 slacks
    double E[4];                     // E of the 4 rows: 1/D (+ 1/D_p + 1/D_n in the restoration phase)
};

// Factorisation outcomes (oracle/c/tt_obca.c: factor): F_MANY a negative pivot where IPOPT's inertia (n, m, 0) wants a
// positive one (PerturbForWrongInertia), F_ZERO a numerically zero pivot, F_FEW too few negative eigenvalues (both
// PerturbForSingularity: IPOPT's PDFullSpaceSolver treats the second as singular once IncreaseQuality fails, and the
// elimination here has no pivot tolerance to raise).
enum { F_OK = 0, F_MANY = 1, F_ZERO = 2, F_FEW = 3 };
// a failed Cholesky pivot s of a positive-definiteness test (diagonal entry ajj): negative, or numerically zero
__device__ __forceinline__ int pivot_fail(double s, double ajj) { return s < -1e-14 * fabs(ajj) ? F_MANY : F_ZERO; }
// the 2x2 reduced input Hessian G of a Riccati stage: F_OK when positive definite, else how its Cholesky fails
// (first pivot G00, second G11 - G01^2 / G00 = det / G00)
__device__ __forceinline__ int g2_code(double G00, double G11, double det) {
    if (!(G00 >= 2.2250738585072014e-308)) return pivot_fail(G00, G00);
    if (!(det >= 2.2250738585072014e-308 * G00)) return pivot_fail(det, G11 * G00);
    return F_OK;
}

// Signed LDL' of a packed lower 4x4, A = L S L' (S = diag(+-1), |L_jj| = sqrt|d_j|, no pivoting; the oracle's
// schol).  The diagonal keeps S_j / L_jj: the solves multiply by its magnitude and read S_j from its sign.  Returns
// the number of negative pivots, -1 on a (numerically) zero pivot (|s| <= 1e-14 |a_jj|; a subnormal positive pivot
// counts as zero, since 1/sqrt of it overflows), or -2 on a negative pivot with pd (round 2's positive-definite test).
// On a positive definite matrix every operation is the plain Cholesky's (S = 1 exactly).
__device__ __forceinline__ double sgn(double d) { return copysign(1.0, d); }
__device__ __forceinline__ int schol4(double* L, bool pd) {
    int neg = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const double ajj = L[lo4(j, j)];
        double s = ajj;
#pragma unroll
        for (int k = 0; k < j; ++k) s = fma(-(L[lo4(j, k)] * sgn(L[lo4(k, k)])), L[lo4(j, k)], s);
        if (!(s >= 2.2250738585072014e-308)) {  // s < DBL_MIN, or NaN
            if (!(s < -1e-14 * fabs(ajj))) return -1;
            if (pd) return -2;
        }
        const double sj = s > 0.0 ? 1.0 : -1.0;
        neg += s < 0.0 ? 1 : 0;
        const double ir = frcp(sqrt(fabs(s)));
        L[lo4(j, j)] = sj * ir;
#pragma unroll
        for (int i = j + 1; i < 4; ++i) {
            double t = L[lo4(i, j)];
#pragma unroll
            for (int k = 0; k < j; ++k) t = fma(-(L[lo4(i, k)] * sgn(L[lo4(k, k)])), L[lo4(j, k)], t);
            L[lo4(i, j)] = (t * ir) * sj;
        }
    }
    return neg;
}
// b <- L^-1 b
__device__ __forceinline__ void fsub4(const double* L, double* b) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        double t = b[i];
#pragma unroll
        for (int k = 0; k < i; ++k) t -= L[lo4(i, k)] * b[k];
        b[i] = t * fabs(L[lo4(i, i)]);
    }
}
// b <- L^-T b
__device__ __forceinline__ void bsub4(const double* L, double* b) {
#pragma unroll
    for (int i = 3; i >= 0; --i) {
        double t = b[i];
#pragma unroll
        for (int k = i + 1; k < 4; ++k) t -= L[lo4(k, i)] * b[k];
        b[i] = t * fabs(L[lo4(i, i)]);
    }
}
// b <- (L S L')^-1 b
__device__ __forceinline__ void ssolve4(const double* L, double* b) {
    fsub4(L, b);
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] *= sgn(L[lo4(i, i)]);
    bsub4(L, b);
}

// entry (i, q), i >= q, of the lam-lam Hessian: T = [[1,0,-1,0],[0,1,0,-1]], H[i][q] = T0i(haa T0q + hac T1q) +
// T1i(hac T0q + hcc T1q)
__device__ __forceinline__ double hll(const Blk& k, int i, int q) {
    const double T0[4] = {1, 0, -1, 0}, T1[4] = {0, 1, 0, -1};
    return T0[i] * (k.haa * T0[q] + k.hac * T1[q]) + T1[i] * (k.hac * T0[q] + k.hcc * T1[q]);
}

__device__ __forceinline__ void blk_lin(LArgs& a, const double* xk, const Trig& tr, int j, const double* w, const double* y,
                                        Blk& k) {
    Geom g;
    body_geom(a, xk, j & 1, tr, g);
    const auto* ob = a.obs + 4 * (j >> 1);
    const double ex = g.p0 - ob[0], ey = g.p1 - ob[1], hwo = 0.5 * ob[2], hho = 0.5 * ob[3];
    const double aa = w[4] - w[6], cc = w[5] - w[7];
    double nr = sqrt(aa * aa + cc * cc);
    k.d[0] = g.hl * (w[0] + w[2]) + g.hw * (w[1] + w[3]) -
             ((ex - hwo) * w[4] + (ey - hho) * w[5] + (-ex - hwo) * w[6] + (-ey - hho) * w[7]) + a.dmin;
    k.d[1] = (w[0] - w[2]) + g.ca * aa + g.sa * cc;
    k.d[2] = (w[1] - w[3]) - g.sa * aa + g.ca * cc;
    k.d[3] = nr - 1.0;
    nr = fmax(nr, 1e-12);
    const double inr = 1.0 / nr;
    k.e2 = -g.sa * aa + g.ca * cc;
    k.e3 = -g.ca * aa - g.sa * cc;
    k.angp = g.angp;
    k.jx0[0] = -aa; k.jx0[1] = -cc;
    k.jx0[2] = -(aa * g.dpt0 + cc * g.dpt1);
    k.jx0[3] = -(aa * g.dpp0 + cc * g.dpp1);
    k.hl = g.hl; k.hw = g.hw;
    k.jw0[0] = g.hl; k.jw0[1] = g.hw; k.jw0[2] = g.hl; k.jw0[3] = g.hw;
    k.jw0[4] = -(ex - hwo); k.jw0[5] = -(ey - hho); k.jw0[6] = ex + hwo; k.jw0[7] = ey + hho;
    k.ca = g.ca; k.sa = g.sa; k.an = aa * inr; k.cn = cc * inr;
    const double y1 = y[0], y2 = y[1], y3 = y[2], y4 = y[3];
    const double rot = y2 * (-g.ca * aa - g.sa * cc) + y3 * (g.sa * aa - g.ca * cc);
    k.hxx22 = -y1 * (aa * g.ppt0 + cc * g.ppt1) + rot;
    k.hxx23 = -y1 * (aa * g.ptp0 + cc * g.ptp1) + rot * g.angp;
    k.hxx33 = -y1 * (aa * g.ppp0 + cc * g.ppp1) + rot * g.angp;
    const double r0 = -y2 * g.sa - y3 * g.ca, r1 = y2 * g.ca - y3 * g.sa;
    k.H(0, 0) = -y1; k.H(0, 1) = 0.0; k.H(0, 2) = y1; k.H(0, 3) = 0.0;
    k.H(1, 0) = 0.0; k.H(1, 1) = -y1; k.H(1, 2) = 0.0; k.H(1, 3) = y1;
    k.H(2, 0) = -y1 * g.dpt0 + r0; k.H(2, 1) = -y1 * g.dpt1 + r1;
    k.H(2, 2) = y1 * g.dpt0 - r0;  k.H(2, 3) = y1 * g.dpt1 - r1;
    k.H(3, 0) = -y1 * g.dpp0 + g.angp * r0; k.H(3, 1) = -y1 * g.dpp1 + g.angp * r1;
    k.H(3, 2) = y1 * g.dpp0 - g.angp * r0;  k.H(3, 3) = y1 * g.dpp1 - g.angp * r1;
    // lam-lam block y4 T'H4T (into LL, before the diagonal is added)
    const double n3 = nr * nr * nr;
    k.haa = y4 * cc * cc / n3;
    k.hac = -y4 * aa * cc / n3;
    k.hcc = y4 * aa * aa / n3;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int q = 0; q <= i; ++q) k.LL[lo4(i, q)] = hll(k, i, q);
}

// Jx[r][q] (rows 0..3, cols X,Y,theta,psi)
__device__ __forceinline__ double jx(const Blk& k, int r, int q) {
    if (r == 0) return q == 0 ? k.jx0[0] : q == 1 ? k.jx0[1] : q == 2 ? k.jx0[2] : k.jx0[3];
    if (r == 1) return q == 2 ? k.e2 : q == 3 ? k.e2 * k.angp : 0.0;
    if (r == 2) return q == 2 ? k.e3 : q == 3 ? k.e3 * k.angp : 0.0;
    return 0.0;
}
// Jw[r][4 + a] (lam columns)
__device__ __forceinline__ double jwl(const Blk& k, int r, int a) {
    if (r == 0) return a == 0 ? k.jw0[4] : a == 1 ? k.jw0[5] : a == 2 ? k.jw0[6] : k.jw0[7];
    if (r == 1) return a == 0 ? k.ca : a == 1 ? k.sa : a == 2 ? -k.ca : -k.sa;
    if (r == 2) return a == 0 ? -k.sa : a == 1 ? k.ca : a == 2 ? k.sa : -k.ca;
    return a == 0 ? k.an : a == 1 ? k.cn : a == 2 ? -k.an : -k.cn;
}
// Jw[r][a] (mu columns)
__device__ __forceinline__ double jwm(const Blk& k, int r, int a) {
    if (r == 0) return a == 0 ? k.jw0[0] : a == 1 ? k.jw0[1] : a == 2 ? k.jw0[2] : k.jw0[3];
    if (r == 1) return a == 0 ? 1.0 : a == 2 ? -1.0 : 0.0;
    if (r == 2) return a == 1 ? 1.0 : a == 3 ? -1.0 : 0.0;
    return 0.0;
}

// elimination of a linearised block.  Inertia (IPOPT tests the whole KKT matrix; oracle/c/tt_obca.c:block_factor):
// by Haynsworth the block [[A, Jw'], [Jw, -E]] has the inertia (8, 4, 0) iff T = E + Jw A^-1 Jw' has as many
// negative pivots as A; the mu part of A is a positive diagonal, so A's negative pivots are those of the lam block
// LL.  Returns false when the test fails (with pd: when LL or T is not positive definite, round 2's test).
// sig_w: diagonal Hessian of the 8 duals (Sigma_w, plus zeta D_R^2 in the restoration phase); E: the rows'
// dual regularisation (1/D, plus 1/D_p + 1/D_n in the restoration phase).  Adds the Schur complement
// W_xx - Z' S_A Z + G' T^-1 G into the stage Hessian contribution C (10 packed lower entries over X,Y,theta,psi).
__device__ __forceinline__ int blk_factor(Blk& k, const double* sig_w, double dw, double* C, bool pd) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        k.idm[i] = frcp(sig_w[i] + dw);
        k.LL[lo4(i, i)] += sig_w[4 + i] + dw;
    }
    const int negA = schol4(k.LL, pd);
    if (negA < 0) return negA == -1 ? F_ZERO : F_MANY;
    double SA[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) SA[a] = sgn(k.LL[lo4(a, a)]);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        double col[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) col[a] = jwl(k, r, a);
        fsub4(k.LL, col);
#pragma unroll
        for (int a = 0; a < 4; ++a) k.Yl(a, r) = col[a];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        double col[4];
#pragma unroll
        for (int a = 0; a < 4; ++a) col[a] = k.H(q, a);
        fsub4(k.LL, col);
#pragma unroll
        for (int a = 0; a < 4; ++a) k.Zl(a, q) = col[a];
    }
    const double* idm = k.idm;
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int s = 0; s <= r; ++s) {
            double t = (r == s) ? k.E[r] : 0.0;
#pragma unroll
            for (int a = 0; a < 4; ++a) t += jwm(k, r, a) * jwm(k, s, a) * idm[a] + (k.Yl(a, r) * SA[a]) * k.Yl(a, s);
            k.LT[lo4(r, s)] = t;
        }
#pragma unroll
    for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            double g = -jx(k, r, q);
#pragma unroll
            for (int a = 0; a < 4; ++a) g += (k.Yl(a, r) * SA[a]) * k.Zl(a, q);
            k.G(r, q) = g;
        }
    const int negT = schol4(k.LT, pd);
    // Haynsworth: the block has IPOPT's inertia (8, 4, 0) iff negT == negA; negT > negA leaves it with too few negative
    // eigenvalues (its rows need delta_c), negT < negA with too many (negative curvature: delta_x)
    // (pd mode: A was positive definite, so a negative T pivot, -2, means too few negative eigenvalues)
    if (negT < 0) return negT == -1 ? F_ZERO : F_FEW;
    if (negT != negA) return negT > negA ? F_FEW : F_MANY;
    double Wm[4][4];  // LT^-1 G
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        double col[4] = {k.G(0, q), k.G(1, q), k.G(2, q), k.G(3, q)};
        fsub4(k.LT, col);
#pragma unroll
        for (int r = 0; r < 4; ++r) Wm[r][q] = col[r];
    }
    const double hxx[4][4] = {{0, 0, 0, 0}, {0, 0, 0, 0}, {0, 0, k.hxx22, k.hxx23}, {0, 0, k.hxx23, k.hxx33}};
#pragma unroll
    for (int p = 0; p < 4; ++p)
#pragma unroll
        for (int q = 0; q <= p; ++q) {
            double t = hxx[p][q];
#pragma unroll
            for (int a = 0; a < 4; ++a)
                t += (Wm[a][p] * sgn(k.LT[lo4(a, a)])) * Wm[a][q] - (k.Zl(a, p) * SA[a]) * k.Zl(a, q);
            C[lo4(p, q)] += t;
        }
    return F_OK;
}

// right-hand side of a factored block.  fw: gradient constants of the 8 duals; rd: row constant
// (d - s) + D^-1 grad phi_s.  Returns zf (mu part fw/dm, lam part LL^-1 fw), t = T^-1 h, and adds the gradient
// contribution -(Z' S_A zl + G' t) into q4.
__device__ __forceinline__ void blk_rhs(const Blk& k, const double* fw, const double* rd, double* zf, double* t, double* q4) {
#pragma unroll
    for (int a = 0; a < 4; ++a) zf[a] = fw[a] * k.idm[a];
    double zl[4] = {fw[4], fw[5], fw[6], fw[7]};
    fsub4(k.LL, zl);
#pragma unroll
    for (int a = 0; a < 4; ++a) zf[4 + a] = zl[a];
    double szl[4];  // S_A zl
#pragma unroll
    for (int a = 0; a < 4; ++a) szl[a] = zl[a] * sgn(k.LL[lo4(a, a)]);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        double h = rd[r];
#pragma unroll
        for (int a = 0; a < 4; ++a) h -= jwm(k, r, a) * zf[a] + k.Yl(a, r) * szl[a];
        t[r] = h;
    }
    ssolve4(k.LT, t);
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        double g = 0.0;
#pragma unroll
        for (int a = 0; a < 4; ++a) g -= k.Zl(a, p) * szl[a];
#pragma unroll
        for (int r = 0; r < 4; ++r) g -= k.G(r, p) * t[r];
        q4[p] += g;
    }
}

// recovery: y+ = t - T^-1 G dx^, dw_mu = -(fw_mu + Jw_mu' y+)/dm, dw_lam = -L^-T S_A (zl + Z dx^ + Y y+)
__device__ __forceinline__ void blk_recover(const Blk& k, const double* fw, const double* zf, const double* t,
                                            const double* dxh, double* yp, double* dwv) {
    double g4[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        double s = 0.0;
#pragma unroll
        for (int q = 0; q < 4; ++q) s += k.G(r, q) * dxh[q];
        g4[r] = s;
    }
    ssolve4(k.LT, g4);
#pragma unroll
    for (int r = 0; r < 4; ++r) yp[r] = t[r] - g4[r];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        double s = fw[a];
#pragma unroll
        for (int r = 0; r < 4; ++r) s += jwm(k, r, a) * yp[r];
        dwv[a] = -s * k.idm[a];
    }
    double v[4];
#pragma unroll
    for (int a = 0; a < 4; ++a) {
        double s = zf[4 + a];
#pragma unroll
        for (int q = 0; q < 4; ++q) s += k.Zl(a, q) * dxh[q];
#pragma unroll
        for (int r = 0; r < 4; ++r) s += k.Yl(a, r) * yp[r];
        v[a] = s * sgn(k.LL[lo4(a, a)]);
    }
    bsub4(k.LL, v);
#pragma unroll
    for (int a = 0; a < 4; ++a) dwv[4 + a] = -v[a];
}

// separating-axis dual certificate (see oracle/c/tt_obca.c:dual_certificate)
__device__ __forceinline__ void dual_certificate(LArgs& a, const double* xk, int j, double* w) {
    Geom g;
    body_geom(a, xk, j & 1, stage_trig(xk), g);
    const auto* ob = a.obs + 4 * (j >> 1);
    double best = -INFINITY, b0 = 1.0, b1 = 0.0;
#pragma unroll
    for (int c = 0; c < 8; ++c) {
        const double s = (c & 1) ? -1.0 : 1.0;
        double n0, n1;
        if (c < 4) { n0 = (c < 2) ? s : 0.0; n1 = (c < 2) ? 0.0 : s; }
        else if (c < 6) { n0 = s * g.ca; n1 = s * g.sa; }
        else { n0 = -s * g.sa; n1 = s * g.ca; }
        const double mx = -(g.ca * n0 + g.sa * n1), my = -(-g.sa * n0 + g.ca * n1);
        const double hB = g.hl * fabs(mx) + g.hw * fabs(my);
        const double hO = n0 * ob[0] + n1 * ob[1] + 0.5 * ob[2] * fabs(n0) + 0.5 * ob[3] * fabs(n1);
        const double gap = n0 * g.p0 + n1 * g.p1 - hB - hO;
        if (gap > best) { best = gap; b0 = n0; b1 = n1; }
    }
    const double sc = 0.99;
    const double mx = -(g.ca * b0 + g.sa * b1), my = -(-g.sa * b0 + g.ca * b1);
    w[0] = sc * fmax(mx, 0.0); w[1] = sc * fmax(my, 0.0); w[2] = sc * fmax(-mx, 0.0); w[3] = sc * fmax(-my, 0.0);
    w[4] = sc * fmax(b0, 0.0); w[5] = sc * fmax(b1, 0.0); w[6] = sc * fmax(-b0, 0.0); w[7] = sc * fmax(-b1, 0.0);
}

__device__ __forceinline__ double push_into(double v, double lo, double hi, bool hl, bool hu) {
    const double k1 = 1e-2, k2 = 1e-2;
    if (hl && hu) {
        const double pl = fmin(k1 * fmax(1.0, fabs(lo)), k2 * (hi - lo));
        const double pu = fmin(k1 * fmax(1.0, fabs(hi)), k2 * (hi - lo));
        return fmin(fmax(v, lo + pl), hi - pu);
    }
    if (hl) return fmax(v, lo + k1 * fmax(1.0, fabs(lo)));
    if (hu) return fmin(v, hi - k1 * fmax(1.0, fabs(hi)));
    return v;
}

__device__ __forceinline__ void clamp_mult(double& z, double sl, double mu) {
    const double ks = 1e10, t = mu * inv(sl);
    z = fmax(fmin(z, ks * t), t * (1.0 / ks));
}

// fraction to the boundary helpers
__device__ __forceinline__ void ftb_lo(double v, double lo, double d, double tau, double& a) {
    if (d < 0.0) a = fmin(a, -tau * (v - lo) * inv(d));
}
__device__ __forceinline__ void ftb_hi(double v, double hi, double d, double tau, double& a) {
    if (d > 0.0) a = fmin(a, tau * (hi - v) * inv(d));
}

// ---------------- restoration-phase elastic pairs (IPOPT MinC_1NrmRestorationPhase) ----------------
// closed-form start: argmin rho (p + n) - mu (ln p + ln n) subject to p - n = r
__device__ __forceinline__ void pn_closed_form(double r, double mu, double& p, double& n) {
    const double S = sqrt(mu * mu + RHO * RHO * r * r);
    const double am = mu - RHO * r, bp = mu + RHO * r;
    n = am >= 0.0 ? (am + S) / (2.0 * RHO) : mu * r / (S - am);
    p = bp >= 0.0 ? (bp + S) / (2.0 * RHO) : -mu * r / (S - bp);
}
// Newton terms of a pair: D_p dp - y+ = -g_p, D_n dn + y+ = -g_n (least-squares system: unit Hessian,
// gradient rho - z)
struct PN {
    double Dp, Dn, gp, gn;
};
__device__ __forceinline__ PN pn_terms(bool lsq, double p, double n, double zp, double zn, double mu, double dw) {
    PN t;
    t.Dp = lsq ? 1.0 : zp / p + dw;
    t.Dn = lsq ? 1.0 : zn / n + dw;
    t.gp = RHO - (lsq ? zp : mu / p);
    t.gn = RHO - (lsq ? zn : mu / n);
    return t;
}

// ---------------- stage pieces ----------------
__device__ __forceinline__ void load_x(const Ctx& c, int k, double* x) {
#pragma unroll
    for (int i = 0; i < 6; ++i) x[i] = c.S(S_X + i, k);
}
__device__ __forceinline__ double stage_cost(const Ctx& c, int k, const double* x, const double* u) {
    LArgs& a = *c.a;
    const double* tg = c.plan() ? c.tgt_x : c.tgt_x + 6 * k;
    const double sc = (k == c.N && c.plan()) ? a.tfac : 1.0;
    double e[6], F = 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) e[i] = x[i] - tg[i];
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        double t = 0.0;
#pragma unroll
        for (int j2 = 0; j2 < 6; ++j2) t += 0.5 * (a.Q[i * 6 + j2] + a.Q[j2 * 6 + i]) * e[j2];
        F += sc * e[i] * t;
    }
    if (k < c.N) {
        double r0 = u[0] - (c.plan() ? 0.0 : c.tgt_u[2 * k]), r1 = u[1] - (c.plan() ? 0.0 : c.tgt_u[2 * k + 1]);
        const double R01 = 0.5 * (a.R[1] + a.R[2]);
        F += r0 * (a.R[0] * r0 + R01 * r1) + r1 * (R01 * r0 + a.R[3] * r1);
    }
    return F;
}

// barrier gradients of the block rows
__device__ __forceinline__ double sig_row(const Ctx& c, int r, double s, double vl, double vu) {
    double sg = vu / (c.rU(r) - s);
    if (c.hrl(r)) sg += vl / (s - c.rL(r));
    return sg;
}
__device__ __forceinline__ double grad_row(const Ctx& c, int r, double s, double mu) {
    double g = mu / (c.rU(r) - s);
    if (c.hrl(r)) g -= mu / (s - c.rL(r));
    return g;
}

// the workspace inputs of one block's factor step (restoration fields only when rs)
struct BlkIn {
    double w[8], zw[8], y[4], s[4], vl[4], vu[4], dr[4];
    double drw[8], wr[8], pr[4], nr[4], zp[4], zn[4];
};
__device__ __forceinline__ void load_blk_in(const Ctx& c, bool rs, int j, int k, BlkIn& in) {
#pragma unroll
    for (int e = 0; e < 8; ++e) { in.w[e] = c.B(B_W + e, j, k); in.zw[e] = c.B(B_ZW + e, j, k); }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        in.y[r] = c.B(B_YD + r, j, k);
        in.s[r] = c.B(B_S + r, j, k); in.vl[r] = c.B(B_VL + r, j, k); in.vu[r] = c.B(B_VU + r, j, k);
        in.dr[r] = c.B(B_DR + r, j, k);
    }
    if (rs) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { in.drw[e] = c.B(B_DRW + e, j, k); in.wr[e] = c.B(B_WR + e, j, k); }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            in.pr[r] = c.B(B_PR + r, j, k); in.nr[r] = c.B(B_NR + r, j, k);
            in.zp[r] = c.B(B_ZP + r, j, k); in.zn[r] = c.B(B_ZN + r, j, k);
        }
    }
}

// linearise + factor + rhs of one block at the current iterate (inputs preloaded); returns the factorisation outcome
// (F_OK ...).  Outputs D (Sigma_s + dw), E (row regularisation: 1/D + delta_c, plus 1/D_p + 1/D_n in the restoration
// phase), the elimination and the block's Hessian / gradient contribution to its stage.  With delta_c the row
// constant carries + delta_c y (IPOPT perturbs dy; the unknown here is y+ = y + dy).
template <bool RHS = true>
__device__ __forceinline__ int block_setup(const Ctx& c, const LShared& sh, const BlkIn& in, int j, const double* x,
                                            const Trig& tr, double mu, double dw, Blk& bk, double* fw, double* zf,
                                            double* t4, double* C4, double* q4) {
    const bool rs = sh.R != 0, lsq = sh.lsq != 0;
    const double dc = sh.dc;
    double sw[8], rd[4];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const double sl = in.w[e] + RELAX, zw = in.zw[e];
        double gw = 0.0, hw = 0.0;
        if (rs) {
            hw = sh.zeta * in.drw[e];
            gw = hw * (in.w[e] - in.wr[e]);
        }
        sw[e] = lsq ? 1.0 : zw / sl + hw;
        fw[e] = lsq ? gw - zw : gw - mu / sl;
    }
    blk_lin(*c.a, x, tr, j, in.w, in.y, bk);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const double s = in.s[r], vl = in.vl[r], vu = in.vu[r];
        bk.D[r] = lsq ? 1.0 : sig_row(c, r, s, vl, vu) + dw;
        bk.E[r] = 1.0 / bk.D[r] + dc;
        const double gs = lsq ? (c.hrl(r) ? -vl : 0.0) + vu : grad_row(c, r, s, mu);
        rd[r] = (dc > 0.0 ? fma(dc, in.y[r], in.dr[r]) : in.dr[r]) + gs / bk.D[r];
        if (rs) {
            const PN t = pn_terms(lsq, in.pr[r], in.nr[r], in.zp[r], in.zn[r], mu, dw);
            bk.E[r] += 1.0 / t.Dp + 1.0 / t.Dn;
            rd[r] += t.gp / t.Dp - t.gn / t.Dn;
        }
    }
    const int f = blk_factor(bk, sw, dw, C4, c.pd);
    if (f != F_OK) return f;
    if constexpr (RHS) blk_rhs(bk, fw, rd, zf, t4, q4);
    return F_OK;
}

// The block's elimination recomputed where a recovery pass needs it, from the same workspace inputs through the same
// code as phase_factor (whose stage contributions C4 / q4 are dropped here).  Round 2 stored it as a 92-double record
// on every inertia attempt (~2.5 per iteration) and read it back in every recovery pass: 30 % of the OBCA kernel's
// HBM traffic for arithmetic the FP64 pipes redo at a fraction of the cost.  RHS: also the main solve's right-hand
// side fw, zf, t (the correction solves read theirs from B_FR).
template <bool RHS>
__device__ __forceinline__ void block_refactor(const Ctx& c, const LShared& sh, const BlkIn& in, int j, const double* x,
                                               const Trig& tr, double mu, double dw, Blk& bk, double* fw, double* zf,
                                               double* t4) {
    double C4[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, q4[4] = {0, 0, 0, 0};
    block_setup<RHS>(c, sh, in, j, x, tr, mu, dw, bk, fw, zf, t4, C4, q4);
}

// ---------------- helper workgroups: the block passes of the instances still solving ----------------
// The launch has nhelp workgroups after the B instances' (blockIdx >= B).  They start once instance workgroups have
// finished and CUs are free -- in the C4 tail a handful of instances run thousands of iterations on an otherwise idle
// GPU -- and run chunks (T consecutive blocks of the flat block index) of those instances' factor and residual passes.
// A chunk's arithmetic does not depend on which workgroup runs it, so the results are bitwise those of the instance
// running every chunk itself (the local path, taken while no helper has started: the whole busy phase of a large batch).
// Board (HBM, zeroed before every launch), one 128-B line per instance:
//   [0] claim = epoch << 40 | chunks << 20 | next chunk (odd epoch: open; kClaimChunkShift), [1] done = epoch << 32 | chunks done by
//   helpers, [2..6] mu dw tau zeta dc (bits), [7] pass | buf << 4 | prep << 8 | mode << 12 | R << 16 | lsq << 20;
// header line (index B): [0] instances finished, [1] helpers started, [2] instances started.
// Hand-off (agent scope; MI355X_MICROARCH.md, inter-workgroup visibility): the instance's waves drain their stores, one
// lane releases (L2 write-back) and stores the claim word; a helper's claim is followed by one acquire before any load
// of the instance's data; a helper's chunk ends with drained stores, a release and the done add; the instance acquires
// once the done count is complete.  Every spin is bounded: an instance that waits longer than the spin limit for its
// helpers' chunks (kSpinTicks, 5 s) sets hfail, runs every later pass of the iteration itself and ends the solve with
// status TT_HANDOFF_TIMEOUT (6); helpers leave after 12 spin limits (60 s) of wall clock whatever the board says.
// Memory model: a helper's chunk stores are agent-scope write-through (sc1) stores drained by s_waitcnt vmcnt(0) in
// every wave before the workgroup barrier, and lane 0 then publishes with a RELEASE done add; the instance's acquire
// after the done count pairs with that release.
typedef __attribute__((address_space(1))) unsigned long long gu64;
enum { PASS_FACTOR = 1, PASS_NRES = 2, PASS_UPDATE = 4 };
struct ChunkPass {
    double mu, dw, tau;
    int pass, buf, prep, mode;
};
__device__ void do_chunks(const Ctx& c, const LShared& sh, ChunkPass p, int c0, int c1, bool helper);

__device__ __forceinline__ gu64* board_line(LArgs& a, int b) { return (gu64*)(a.board + (size_t)b * kObcaBoardStride); }
__device__ __forceinline__ unsigned long long ld_rlx(gu64* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_rlx(gu64* p, unsigned long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long add_rlx(gu64* p, unsigned long long v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ unsigned long long dbits(double v) { return (unsigned long long)__double_as_longlong(v); }
__device__ __forceinline__ double bitsd(unsigned long long v) { return __longlong_as_double((long long)v); }
constexpr unsigned long long kSpinTicks = 500000000ull;  // 5 s of the 100 MHz s_memrealtime clock
constexpr unsigned long long kStartTicks = 2000ull;  // 20 us: how long a helper waits for the batch to have started
constexpr int kStatusHandoffTimeout = 6;  // TT_HANDOFF_TIMEOUT (include/ttmpc.h)
#ifndef OBCA_HELPER_RELEASE
#define OBCA_HELPER_RELEASE 1
#endif

// one block pass of this instance (every thread of its workgroup), ending with a workgroup barrier
__device__ void run_pass(const Ctx& c, LShared& sh, const ChunkPass& p) {
    LArgs& a = *c.a;
    const int nch = (c.nbk * c.NP + T - 1) / T;
    if (threadIdx.x == 0) {
        // shared mode once there is a helper for every instance still solving (before that the hand-off costs the
        // instances more than the few helpers return: profiles/r05/helpers/stamps_h.txt); never again after a hand-off
        // timed out (the solve ends with TT_HANDOFF_TIMEOUT at the next convergence test)
        int on = 0;
        if (a.board && a.nhelp > 0 && !sh.hfail) {
            gu64* hdr = board_line(a, a.B);
            const unsigned long long fin = ld_rlx(hdr), hlp = ld_rlx(hdr + 1), started = ld_rlx(hdr + 2);
            on = hlp > 0 && hlp + fin >= started;
        }
        on |= c.b == a.fail_b && !sh.hfail;  // the forced-timeout instance publishes whether or not helpers came
        sh.hcur = on;
    }
    __syncthreads();
    const bool shared = sh.hcur != 0;
    __syncthreads();
    if (!shared) {
        do_chunks(c, sh, p, 0, nch, false);
        __syncthreads();
        return;
    }
    gu64* ln = board_line(a, c.b);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every wave's workspace stores complete
    __syncthreads();
    unsigned long long ep = 0;
    if (threadIdx.x == 0) {
        ep = 2ull * sh.hep + 1ull;
        sh.hep += 1;
        ln[2] = dbits(p.mu); ln[3] = dbits(p.dw); ln[4] = dbits(p.tau); ln[5] = dbits(sh.zeta); ln[6] = dbits(sh.dc);
        ln[7] = (unsigned long long)(p.pass | p.buf << 4 | p.prep << 8 | p.mode << 12 | sh.R << 16 | sh.lsq << 20);
        st_rlx(ln + 1, ep << 32);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        st_rlx(ln, ep << 40 | (unsigned long long)nch << kClaimChunkShift);
    }
    // the debug instance (ObcaArgs::fail_b) leaves every chunk to the helpers and waits for a count that never comes
    const bool forced = c.b == a.fail_b;
    int own = 0;
    for (;;) {
        if (threadIdx.x == 0) sh.hcur = forced ? nch : (int)(add_rlx(ln, 1) & kClaimFieldMask);
        __syncthreads();
        const int ci = sh.hcur;
        __syncthreads();
        if (ci >= nch) break;
        do_chunks(c, sh, p, ci, ci + 1, false);
        ++own;
    }
    if (threadIdx.x == 0) {
        const unsigned long long want = forced ? ~0ull : ep << 32 | (unsigned long long)(nch - own);
        const unsigned long long lim = a.spin_ticks ? a.spin_ticks : kSpinTicks, t0 = __builtin_amdgcn_s_memrealtime();
        while (ld_rlx(ln + 1) != want) {
            if (__builtin_amdgcn_s_memrealtime() - t0 > lim) { sh.hfail = 1; break; }
            __builtin_amdgcn_s_sleep(2);
        }
        st_rlx(ln, (ep + 1ull) << 40);  // closed
        if (own < nch) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    }
    __syncthreads();
}

// a block part's store: plain (the instance's own chunks), or write-through (sc1) when a helper workgroup runs the chunk,
// so that its hand-off needs no L2 write-back (MI355X guide, R1: every payload byte stored sc1 and drained, then the done
// count; the instance still acquires before reading)
template <bool SC1>
__device__ __forceinline__ void bst(gdouble& ref, double v) {
    if constexpr (SC1) __hip_atomic_store((gu64*)&ref, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT);
    else ref = v;
}
// ---- the factor pass's block part: linearise + factor + right-hand side of block (j, k) of the flat block index ----
// Only the block's contributions to its stage leave it (the recovery passes recompute the elimination, block_refactor):
// the Schur complement C4, the gradient q4 and the factorisation outcome, in its record B_CB; phase_factor's stage part
// adds a stage's records in block order (the arithmetic of the block loop inside the stage loop).
enum : int { CF_C4 = 0, CF_Q4 = 10, CF_FAIL = 14, CF_END = 15 };
static_assert(CF_END <= B_END - B_CB, "factor contribution record");
template <bool SC1>
__device__ __forceinline__ void factor_block(const Ctx& c, const LShared& sh, const WsView& vw, int j, int k, double mu,
                                             double dw) {
    double x[6];
    load_x(c, k, x);
    const Trig tr = stage_trig(x);
    Blk bk;
    bk.m = c.slab + threadIdx.x;
    double fw[8], zf[8], t4[4];
    double cf[CF_END] = {};
    BlkIn cur;
    load_blk_in(c, sh.R != 0, j, k, cur);
    cf[CF_FAIL] = (double)block_setup(c, sh, cur, j, x, tr, mu, dw, bk, fw, zf, t4, cf + CF_C4, cf + CF_Q4);
#pragma unroll
    for (int i = 0; i < CF_END; ++i) bst<SC1>(vw.B(B_CB + i, j, k), cf[i]);
}

// ======== phase: stage Hessians + gradients (all threads) -> factorisation outcome (uniform) ========
// Also the effective dynamics-row residuals S_CE (= S_CR + delta_c y outside the restoration phase) and the soft-row
// scales S_SD = sqrt(E) (E = 1/D_p + 1/D_n in the restoration phase, + delta_c).
__device__ __noinline__ int phase_factor(const Ctx& c, LShared& sh, double mu, double dw) {
    const WsView vw = ws_view(c);
    LArgs& a = *c.a;
    const int N = c.N;
    const bool plan = c.plan(), rs = sh.R != 0, lsq = sh.lsq != 0;
    const double dc = sh.dc;
    const bool soft = rs || dc > 0.0;
    double fail[3] = {0.0, 0.0, 0.0};  // F_ZERO, F_MANY, F_FEW seen
    // the block part over the flat block index (factor_block), by this workgroup and any helpers
    run_pass(c, sh, ChunkPass{mu, dw, 0.0, PASS_FACTOR, 0, 0, 0});
    for (int k = (int)threadIdx.x; k <= N; k += T) {
        double x[6];
        load_x(c, k, x);
        // the blocks' stage contributions, in block order
        double C4[10] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, q4[4] = {0, 0, 0, 0};
        for (int j = 0; j < c.nbk; ++j) {
            double cf[CF_END];
#pragma unroll
            for (int i = 0; i < CF_END; ++i) cf[i] = vw.B(B_CB + i, j, k);
#pragma unroll
            for (int i = 0; i < 10; ++i) C4[i] += cf[CF_C4 + i];
#pragma unroll
            for (int i = 0; i < 4; ++i) q4[i] += cf[CF_Q4 + i];
            const int f = (int)cf[CF_FAIL];
            if (f == F_ZERO) fail[0] = 1.0;
            if (f == F_MANY) fail[1] = 1.0;
            if (f == F_FEW) fail[2] = 1.0;
        }
        double Qs[21], qv[6];
        const double sc = (k == N && plan) ? a.tfac : 1.0;
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j2 = i; j2 < 6; ++j2)
                Qs[sy6(i, j2)] = lsq ? (i == j2 ? 1.0 : 0.0) : rs ? 0.0 : sc * (a.Q[i * 6 + j2] + a.Q[j2 * 6 + i]);
        if (k < N && !lsq) {
            Qs[sy6(2, 2)] += vw.S(S_WD + 0, k);
            Qs[sy6(2, 5)] += vw.S(S_WD + 1, k);
            Qs[sy6(3, 3)] += vw.S(S_WD + 2, k);
            Qs[sy6(3, 4)] += vw.S(S_WD + 3, k);
            Qs[sy6(3, 5)] += vw.S(S_WD + 4, k);
            Qs[sy6(4, 4)] += vw.S(S_WD + 5, k);
            Qs[sy6(4, 5)] += vw.S(S_WD + 6, k);
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const double xv = x[i];
            double sg = dw + (rs && !lsq ? sh.zeta * vw.S(S_DRX + i, k) : 0.0), g = vw.S(S_GX + i, k);
            if (c.hlx(i)) {
                const double zl = vw.S(S_ZLX + i, k), il = inv(xv - c.xl[i]);
                sg += zl * il;
                g -= lsq ? zl : mu * il;
            }
            if (c.hux(i)) {
                const double zu = vw.S(S_ZUX + i, k), iu = inv(c.xu[i] - xv);
                sg += zu * iu;
                g += lsq ? zu : mu * iu;
            }
            if (!lsq) Qs[sy6(i, i)] += sg;
            qv[i] = g;
        }
#pragma unroll
        for (int p = 0; p < 4; ++p) {
#pragma unroll
            for (int q = 0; q <= p; ++q) Qs[sy6(q, p)] += C4[lo4(p, q)];
            qv[p] += q4[p];
        }
        if (k == N && plan)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double sl = sh.sf[i] - c.fL, su = c.fU - sh.sf[i];
                const double Ds = lsq ? 1.0 : sh.vLf[i] / sl + sh.vUf[i] / su + dw;
                const double gs = lsq ? -sh.vLf[i] + sh.vUf[i] : -mu / sl + mu / su;
                double E = 1.0 / Ds + dc, rf = (dc > 0.0 ? fma(dc, sh.ydf[i], sh.dfr[i]) : sh.dfr[i]) + gs / Ds;
                if (rs) {
                    const PN t = pn_terms(lsq, sh.pf[i], sh.nf[i], sh.zpf[i], sh.znf[i], mu, dw);
                    E += 1.0 / t.Dp + 1.0 / t.Dn;
                    rf += t.gp / t.Dp - t.gn / t.Dn;
                }
                const double Dfe = 1.0 / E;
                sh.Dsf[i] = Ds;
                sh.Dfe[i] = Dfe;
                sh.rf[i] = rf;
                Qs[sy6(i, i)] += Dfe;
                qv[i] += Dfe * rf;
            }
#pragma unroll
        for (int i = 0; i < 21; ++i) vw.S(S_QT + i, k) = Qs[i];
#pragma unroll
        for (int i = 0; i < 6; ++i) vw.S(S_QV + i, k) = qv[i];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            double ce = vw.S(S_CR + i, k), sd = 0.0, e = dc;
            if (dc > 0.0) ce = fma(dc, (double)vw.S(S_YC + i, k), ce);
            if (rs) {
                const PN t = pn_terms(lsq, vw.S(S_PR + i, k), vw.S(S_NR + i, k), vw.S(S_ZP + i, k), vw.S(S_ZN + i, k), mu, dw);
                const double ip = inv(t.Dp), in_ = inv(t.Dn);
                ce += t.gp * ip - t.gn * in_;
                e = (ip + in_) + dc;
            }
            if (soft) sd = sqrt(e);
            vw.S(S_CE + i, k) = ce;
            vw.S(S_SD + i, k) = sd;
        }
        if (k < N) {
            const double u0 = vw.S(S_U, k), u1 = vw.S(S_U + 1, k);
            double R0, R1, R3, g0 = vw.S(S_GU, k), g1 = vw.S(S_GU + 1, k);
            if (lsq) {
                R0 = 1.0; R1 = 0.0; R3 = 1.0;
                if (c.hlu(0)) g0 -= vw.S(S_ZLU, k);
                if (c.huu(0)) g0 += vw.S(S_ZUU, k);
                if (c.hlu(1)) g1 -= vw.S(S_ZLU + 1, k);
                if (c.huu(1)) g1 += vw.S(S_ZUU + 1, k);
            } else {
                R0 = (rs ? sh.zeta * vw.S(S_DRU, k) : 2.0 * a.R[0]) + dw;
                R1 = rs ? 0.0 : a.R[1] + a.R[2];
                R3 = (rs ? sh.zeta * vw.S(S_DRU + 1, k) : 2.0 * a.R[3]) + dw;
                if (c.hlu(0)) { const double t = inv(u0 - c.ul[0]); R0 += vw.S(S_ZLU, k) * t; g0 -= mu * t; }
                if (c.huu(0)) { const double t = inv(c.uu[0] - u0); R0 += vw.S(S_ZUU, k) * t; g0 += mu * t; }
                if (c.hlu(1)) { const double t = inv(u1 - c.ul[1]); R3 += vw.S(S_ZLU + 1, k) * t; g1 -= mu * t; }
                if (c.huu(1)) { const double t = inv(c.uu[1] - u1); R3 += vw.S(S_ZUU + 1, k) * t; g1 += mu * t; }
            }
            vw.S(S_RT, k) = R0;
            vw.S(S_RT + 1, k) = R1;
            vw.S(S_RT + 2, k) = R3;
            vw.S(S_RV, k) = g0;
            vw.S(S_RV + 1, k) = g1;
        }
    }
    const int ops[3] = {R_MAX, R_MAX, R_MAX};
    wg_reduce(sh, fail, ops);
    return fail[0] != 0.0 ? F_ZERO : fail[1] != 0.0 ? F_MANY : fail[2] != 0.0 ? F_FEW : F_OK;
}

// Stage data of the serial sweeps, either straight from the HBM workspace (GSrc) or from LDS copies
// staged by all four waves before the sweep (LSrc: region A = sweep inputs, region B = its outputs).
// CR is the effective dynamics-row residual S_CE.
struct GSrc {
    const Ctx& c;
    __device__ double QT(int i, int k) const { return c.S(S_QT + i, k); }
    __device__ double QV(int i, int k) const { return c.S(S_QV + i, k); }
    __device__ double RT(int i, int k) const { return c.S(S_RT + i, k); }
    __device__ double RV(int i, int k) const { return c.S(S_RV + i, k); }
    __device__ double AJ(int i, int k) const { return c.S(S_AJ + i, k); }
    __device__ double CR(int i, int k) const { return c.S(S_CE + i, k); }
    __device__ double P(int i, int k) const { return c.S(S_P + i, k); }
    __device__ double PV(int i, int k) const { return c.S(S_PV + i, k); }
    __device__ double K(int i, int k) const { return c.S(S_K + i, k); }
    __device__ double KF(int i, int k) const { return c.S(S_KF + i, k); }
    __device__ void setP(int i, int k, double v) const { c.S(S_P + i, k) = v; }
    __device__ void setPV(int i, int k, double v) const { c.S(S_PV + i, k) = v; }
    __device__ void setK(int i, int k, double v) const { c.S(S_K + i, k) = v; }
    __device__ void setKF(int i, int k, double v) const { c.S(S_KF + i, k) = v; }
    __device__ void setGI(int i, int k, double v) const { c.S(S_GI + i, k) = v; }
};
// region A per stage: QT 21 | QV 6 | RT 3 | RV 2 | AJ 9 | CR 6  (47);  region B: P 21 | PV 6 | K 12 | KF 2 | G^-1 3 (44)
constexpr int LA = 47, LB = 44;
struct LSrc {
    const lds_double* A;
    lds_double* B;
    __device__ double QT(int i, int k) const { return A[k * LA + i]; }
    __device__ double QV(int i, int k) const { return A[k * LA + 21 + i]; }
    __device__ double RT(int i, int k) const { return A[k * LA + 27 + i]; }
    __device__ double RV(int i, int k) const { return A[k * LA + 30 + i]; }
    __device__ double AJ(int i, int k) const { return A[k * LA + 32 + i]; }
    __device__ double CR(int i, int k) const { return A[k * LA + 41 + i]; }
    __device__ double P(int i, int k) const { return B[k * LB + i]; }
    __device__ double PV(int i, int k) const { return B[k * LB + 21 + i]; }
    __device__ double K(int i, int k) const { return B[k * LB + 27 + i]; }
    __device__ double KF(int i, int k) const { return B[k * LB + 39 + i]; }
    __device__ void setP(int i, int k, double v) const { B[k * LB + i] = v; }
    __device__ void setPV(int i, int k, double v) const { B[k * LB + 21 + i] = v; }
    __device__ void setK(int i, int k, double v) const { B[k * LB + 27 + i] = v; }
    __device__ void setKF(int i, int k, double v) const { B[k * LB + 39 + i] = v; }
    __device__ double GI(int i, int k) const { return B[k * LB + 41 + i]; }
    __device__ void setGI(int i, int k, double v) const { B[k * LB + 41 + i] = v; }
};
__host__ __device__ inline size_t obca_lds_bytes(int N) { return (size_t)(LA + LB) * (N + 1) * 8; }  // >= the soft records (53, 77)
constexpr size_t kObcaLdsMax = 150 * 1024;  // dynamic LDS budget for the staged sweeps (+ static Shared)

// all threads: copy the sweep inputs of every stage into region A (field-major reads: coalesced in k)
// Copy F stage fields of every stage into an LDS record array A[k * F + f] (value(f, k) reads the workspace):
// eight loads per thread are in flight before their LDS stores, instead of one load waited for per element.
template <int F, class Val>
__device__ __forceinline__ void stage_copy(const Ctx& c, double* A, Val value) {
    const int NP = c.NP, tot = F * NP;
    for (int base = threadIdx.x; base < tot; base += 8 * T) {
        double v[8];
        int d[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int idx = base + u * T;
            d[u] = -1;
            v[u] = 0.0;
            if (idx < tot) {
                const int f = idx / NP, k = idx - f * NP;
                d[u] = k * F + f;
                v[u] = value(f, k);
            }
        }
        lds_double* L = (lds_double*)A;  // ds_write, not flat stores (which would also queue on vmcnt)
#pragma unroll
        for (int u = 0; u < 8; ++u)
            if (d[u] >= 0) L[d[u]] = v[u];
    }
}
__device__ __noinline__ void stage_inputs(const Ctx& c, double* A) {
    const WsView vw = ws_view(c);
    stage_copy<LA>(c, A, [&](int f, int k) -> double {
        int g;
        if (f < 21) g = S_QT + f;
        else if (f < 27) g = S_QV + f - 21;
        else if (f < 30) g = S_RT + f - 27;
        else if (f < 32) g = S_RV + f - 30;
        else if (f < 41) g = S_AJ + f - 32;
        else g = S_CE + f - 41;
        return (k < c.N || (f < 27 || f >= 41)) ? (double)vw.S(g, k) : 0.0;
    });
}

// ======== phase: Riccati backward sweep (wave 0).  Sets sh.flag = 1 if an input block is not PD ========
// P_N = Q~_N; G = R~ + B'PB, H = B'PA, K = -G^-1 H, P_k = Q~_k + A'PA + H'K   (B = dt [e5 e4])
// vector: p' = p_{k+1} - P_{k+1} c_{k+1}, kff = -G^-1 (r~ + B'p'), p_k = q~_k + A'p' + H'kff
//
// Entry-parallel, branch-free: lane (i, j) < 36 forms PA[i][j] from row i of the P tile, then P_k at the
// symmetric position (min, max) from column max of the PA tile, so both halves of the P tile are bitwise
// equal.  Lanes 48..53 carry the vector recursion (row r = lane - 48).  A = I + D with D the 9 dt*J
// nonzeros; the lane's D coefficients are selects on its column index, not branches.  One wave: LDS
// operations complete in program order, so the two tiles need only compiler ordering, and the next
// stage's operands are loaded behind the tile reads.
struct RicOps {
    double dj[9], e[6], R0, R1, R3, rv0, rv1, qt, qv;
};
template <class Src>
__device__ __forceinline__ void ric_ops(const Src& src, int k, int sij, int r, bool vec, RicOps& o) {
#pragma unroll
    for (int q = 0; q < 9; ++q) o.dj[q] = src.AJ(q, k);
#pragma unroll
    for (int q = 0; q < 6; ++q) o.e[q] = src.CR(q, k + 1);
    o.R0 = src.RT(0, k);
    o.R1 = src.RT(1, k);
    o.R3 = src.RT(2, k);
    o.rv0 = src.RV(0, k);
    o.rv1 = src.RV(1, k);
    o.qt = src.QT(sij, k);
    o.qv = vec ? src.QV(r, k) : 0.0;
}
// D[q][col] for q = 0..3 (rows 4, 5 of D are zero), as products with 0/1 column indicators so that the
// coefficients stay in registers (a select of array elements would become a load of a selected address)
struct ColMask {
    double m2, m3, m4, m5;
    __device__ explicit ColMask(int col)
        : m2(col == 2 ? 1.0 : 0.0), m3(col == 3 ? 1.0 : 0.0), m4(col == 4 ? 1.0 : 0.0), m5(col == 5 ? 1.0 : 0.0) {}
};
__device__ __forceinline__ void dcol(const double* dj, const ColMask& m, double& c0, double& c1, double& c2,
                                     double& c3) {
    c0 = fma(m.m2, dj[0], m.m5 * dj[1]);
    c1 = fma(m.m2, dj[2], m.m5 * dj[3]);
    c2 = fma(m.m4, dj[4], m.m5 * dj[5]);
    c3 = fma(m.m3, dj[6], fma(m.m4, dj[7], m.m5 * dj[8]));
}
__device__ __forceinline__ double2 ldd2(const double* p) { return *reinterpret_cast<const double2*>(p); }

template <class Src>
__device__ __noinline__ void riccati(const Ctx& c, LShared& sh, const Src src) {
    const int lane = threadIdx.x, N = c.N;
    const double dt = c.dt, dt2 = dt * dt;
    const bool act = lane < 36, vec = lane >= 48 && lane < 54;
    const int i = act ? lane / 6 : 0, j = act ? lane % 6 : 0, r = vec ? lane - 48 : 0;
    const int ii = min(i, j), jj = max(i, j), sij = sy6(ii, jj);
    const int row = vec ? r : i;  // row of P this lane reads
    const ColMask mj(j), mi(ii), mr(r);
    // the two tiles as LDS-addressed arrays (ds_read / ds_write, not flat accesses through `sh`)
    __shared__ __attribute__((aligned(16))) double P[48];   // P_{k+1}, row-major, row stride 8
    __shared__ __attribute__((aligned(16))) double PT[48];  // PA transposed: PT[8 j + r] = PA[r][j]
    // with refinement the factorisation (P, K, G^-1) also goes to the HBM workspace for the correction solves: from the
    // LDS record by keep_factors (waves 1-3, during the forward sweep), so the serial sweep issues no HBM stores
    if (act) {
        const double q = src.QT(sij, N);
        P[8 * i + j] = q;
        if (i <= j) src.setP(sij, N, q);
    }
    double pv = vec ? src.QV(r, N) : 0.0;
    if (vec) src.setPV(r, N, pv);
    bool fail = false;
    int fcode = F_OK;  // the first failed pivot's outcome (the oracle stops there)
    // one stage; `cur` = this stage's operands, `nx` receives stage k-1's (ping-pong, no struct copies)
    auto stage = [&](int k, const RicOps& cur, RicOps& nx) __attribute__((always_inline)) {
        // ---- row `row` of P_{k+1}: PA[i][j] (act lanes) and p' = p - P c (vector lanes)
        const double2 p01 = ldd2(P + 8 * row), p23 = ldd2(P + 8 * row + 2), p45 = ldd2(P + 8 * row + 4);
        const double pij = P[8 * row + j];
        const double2 g44 = ldd2(P + 8 * 4 + 4);  // P[4][4], P[4][5]
        const double p55 = P[8 * 5 + 5];
        double cj0, cj1, cj2, cj3;
        dcol(cur.dj, mj, cj0, cj1, cj2, cj3);
        const double pa = fma(p01.x, cj0, fma(p01.y, cj1, fma(p23.x, cj2, fma(p23.y, cj3, pij))));
        if (act) PT[8 * j + i] = pa;
        double pp = pv;
        pp = fma(-p01.x, cur.e[0], pp);
        pp = fma(-p01.y, cur.e[1], pp);
        pp = fma(-p23.x, cur.e[2], pp);
        pp = fma(-p23.y, cur.e[3], pp);
        pp = fma(-p45.x, cur.e[4], pp);
        pp = fma(-p45.y, cur.e[5], pp);
        asm volatile("" ::: "memory");
        // ---- reduced input Hessian G = R~ + B'PB and its inverse
        const double G00 = cur.R0 + dt2 * p55, G01 = cur.R1 + dt2 * g44.y, G11 = cur.R3 + dt2 * g44.x;
        const double det = G00 * G11 - G01 * G01;
        const int gc = g2_code(G00, G11, det);
        if (!fail) fcode = gc;
        fail = fail || gc != F_OK;
        const double idet = frcp(det);
        const double Gi00 = G11 * idet, Gi01 = -G01 * idet, Gi11 = G00 * idet;
        // ---- column jj of PA, and PA[4..5][ii] (H at ii); vector lanes: PA[4..5][r]
        const double2 a01 = ldd2(PT + 8 * jj), a23 = ldd2(PT + 8 * jj + 2), a45 = ldd2(PT + 8 * jj + 4);
        const double aij = PT[8 * jj + ii];
        const double2 hi = ldd2(PT + 8 * (vec ? r : ii) + 4);  // PA[4][.], PA[5][.]
        if (k > 0) ric_ops(src, k - 1, sij, r, vec, nx);  // next stage's operands, behind the tile reads
        double ci0, ci1, ci2, ci3;
        dcol(cur.dj, mi, ci0, ci1, ci2, ci3);
        const double atpa = fma(ci0, a01.x, fma(ci1, a01.y, fma(ci2, a23.x, fma(ci3, a23.y, aij))));
        const double H0i = dt * hi.y, H1i = dt * hi.x, H0j = dt * a45.y, H1j = dt * a45.x;
        const double K0j = -fma(Gi00, H0j, Gi01 * H1j), K1j = -fma(Gi01, H0j, Gi11 * H1j);
        const double Pk = cur.qt + atpa + fma(H0i, K0j, H1i * K1j);
        // ---- vector recursion: p' from lanes 48..53 to the lanes of their 16-lane row (DPP row_newbcast; lanes 48..53
        // and lane 48's KF / G^-1 stores are its only readers)
        double ppl[6];
        ppl[0] = rowbc<0>(pp); ppl[1] = rowbc<1>(pp); ppl[2] = rowbc<2>(pp);
        ppl[3] = rowbc<3>(pp); ppl[4] = rowbc<4>(pp); ppl[5] = rowbc<5>(pp);
        const double g0 = fma(dt, ppl[5], cur.rv0), g1 = fma(dt, ppl[4], cur.rv1);
        const double kf0 = -fma(Gi00, g0, Gi01 * g1), kf1 = -fma(Gi01, g0, Gi11 * g1);
        double cr0, cr1, cr2, cr3;
        dcol(cur.dj, mr, cr0, cr1, cr2, cr3);
        double ppr = ppl[0];
        ppr = r == 1 ? ppl[1] : ppr;
        ppr = r == 2 ? ppl[2] : ppr;
        ppr = r == 3 ? ppl[3] : ppr;
        ppr = r == 4 ? ppl[4] : ppr;
        ppr = r == 5 ? ppl[5] : ppr;
        const double atp = fma(cr0, ppl[0], fma(cr1, ppl[1], fma(cr2, ppl[2], fma(cr3, ppl[3], ppr))));
        const double pnew = cur.qv + atp + fma(dt * hi.y, kf0, dt * hi.x * kf1);
        // ---- outputs; the P tile is overwritten after every lane's reads of it were issued
        if (act) {
            P[8 * i + j] = Pk;
            if (i <= j) src.setP(sij, k, Pk);
        }
        if (vec) {
            const double H0 = dt * hi.y, H1 = dt * hi.x;
            const double K0 = -fma(Gi00, H0, Gi01 * H1), K1 = -fma(Gi01, H0, Gi11 * H1);
            src.setK(r, k, K0);
            src.setK(6 + r, k, K1);
            src.setPV(r, k, pnew);
        }
        if (lane == 48) {
            src.setKF(0, k, kf0);
            src.setKF(1, k, kf1);
            if (c.refine) { src.setGI(0, k, Gi00); src.setGI(1, k, Gi01); src.setGI(2, k, Gi11); }
        }
        pv = pnew;
        asm volatile("" ::: "memory");
    };
    RicOps oa, ob;
    ric_ops(src, N - 1, sij, r, vec, oa);
    asm volatile("" ::: "memory");
    int k = N - 1;
    for (; k >= 1; k -= 2) {
        stage(k, oa, ob);
        stage(k - 1, ob, oa);
        // a failed inertia attempt is discarded (the caller raises delta_w): stop at the first failed pivot
        // instead of finishing the sweep (fail is wave-uniform: every lane evaluates the same G)
        if (__builtin_amdgcn_readfirstlane((int)fail)) break;
    }
    if (k == 0 && !fail) stage(0, oa, ob);
    // the failure code (all lanes evaluate the same uniform G; keep it explicit)
    if (lane == 0) sh.flag = fcode;
    wave_sync();
}

// ======== phase: forward sweep (wave 0) into step buffer buf ========
// dx_0 = -c_0; du_k = K_k dx_k + kff_k; dx_{k+1} = A_k dx_k + B du_k - c_{k+1}; y+_k = -(P_k dx_k + p_k).
// The 6-vector recursion is carried redundantly by every lane (wave-uniform registers: no readlane /
// broadcast on the serial chain); lanes 0..5 then write row r of the stage outputs off the chain.  The chain's
// operands of stage k+1 (K, kff, the D nonzeros, c_{k+2}: broadcast LDS reads) are loaded during stage k, so no
// stage waits for its own LDS reads (the same operations on the same values as loading them in place).
struct FwdOps {
    double kf0, kf1, K[12], aj[9], e[6];
};
template <class Src>
__device__ __forceinline__ void fwd_ops(const Src& src, int k, FwdOps& o) {
    o.kf0 = src.KF(0, k);
    o.kf1 = src.KF(1, k);
#pragma unroll
    for (int q = 0; q < 12; ++q) o.K[q] = src.K(q, k);
#pragma unroll
    for (int q = 0; q < 9; ++q) o.aj[q] = src.AJ(q, k);
#pragma unroll
    for (int q = 0; q < 6; ++q) o.e[q] = src.CR(q, k + 1);
}
template <class Src>
__device__ __noinline__ void forward(const Ctx& c, const Src src, int buf) {
    const WsView vw = ws_view(c);
    const int lane = threadIdx.x, N = c.N;
    const double dt = c.dt;
    const int r = lane < 6 ? lane : 0;
    double dx[6];
#pragma unroll
    for (int q = 0; q < 6; ++q) dx[q] = -src.CR(q, 0);
    auto out = [&](int k) __attribute__((always_inline)) {
        if (lane < 6) {
            double t = src.PV(r, k), dxr = dx[0];
#pragma unroll
            for (int q = 0; q < 6; ++q) t = fma(src.P(sy6(r, q), k), dx[q], t);
#pragma unroll
            for (int q = 1; q < 6; ++q) dxr = r == q ? dx[q] : dxr;
            vw.S(S_YCP + 6 * buf + r, k) = -t;
            vw.S(S_DX + 6 * buf + r, k) = dxr;
        }
    };
    auto chain = [&](int k, const FwdOps& o) __attribute__((always_inline)) {
        double du0 = o.kf0, du1 = o.kf1;
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            du0 = fma(o.K[q], dx[q], du0);
            du1 = fma(o.K[6 + q], dx[q], du1);
        }
        if (lane == 0) {
            vw.S(S_DU + 2 * buf, k) = du0;
            vw.S(S_DU + 2 * buf + 1, k) = du1;
        }
        const double* aj = o.aj;
        const double* e = o.e;
        double nx[6];
        nx[0] = (dx[0] - e[0]) + fma(aj[0], dx[2], aj[1] * dx[5]);
        nx[1] = (dx[1] - e[1]) + fma(aj[2], dx[2], aj[3] * dx[5]);
        nx[2] = (dx[2] - e[2]) + fma(aj[4], dx[4], aj[5] * dx[5]);
        nx[3] = (dx[3] - e[3]) + fma(aj[6], dx[3], fma(aj[7], dx[4], aj[8] * dx[5]));
        nx[4] = (dx[4] - e[4]) + dt * du1;
        nx[5] = (dx[5] - e[5]) + dt * du0;
#pragma unroll
        for (int q = 0; q < 6; ++q) dx[q] = nx[q];
    };
    // two stages per trip, ping-pong operand sets (no register copies between stages)
    FwdOps oa, ob;
    int k = 0;
    if (N > 0) fwd_ops(src, 0, oa);
    for (; k + 1 < N; k += 2) {
        fwd_ops(src, k + 1, ob);
        out(k);
        chain(k, oa);
        if (k + 2 < N) fwd_ops(src, k + 2, oa);
        out(k + 1);
        chain(k + 1, ob);
    }
    if (k < N) {
        out(k);
        chain(k, oa);
        ++k;
    }
    out(N);
}

// ======== restoration phase: Riccati sweep with soft dynamics rows (wave 0) ========
// Row k reads x_k - F(x_{k-1}) - p + n = c: eliminating the elastic pair leaves J dx - E y+ = -r~ with
// E = 1/D_p + 1/D_n, so x_k = yhat_k + E y+_k.  Before stage k-1 the cost-to-go of stage k is softened:
// M = I + S P_k S (S = E^1/2; positive definite or the inertia is wrong), Y_k = S M^-1 S,
// P~_k = P_k - P_k Y_k P_k, p~_k = p_k - P_k Y_k p_k; stage k-1 then runs the hard recursion on P~, p~.
// M^-1 by in-place Gauss-Jordan (lane (i, j) owns entry (i, j); the pivots are M's LDL' pivots).  Y_k
// is kept (S_Y) for the forward sweep.
// One wave: its LDS operations complete in program order, so the tiles need only compiler ordering
// (lds_order), never a memory fence (a fence would also wait for the HBM stores of P, K, Y).  The
// inputs come from LDS copies staged by all four waves (SoftA) when the dynamic LDS holds them, else
// straight from HBM (GSrc); either way the next stage's operands are loaded one stage ahead.
__device__ __forceinline__ void lds_order() { asm volatile("" ::: "memory"); }

// region of the soft sweep's inputs, per stage: QT 21 | QV 6 | RT 3 | RV 2 | AJ 9 | CE 6 | SD 6  (53)
constexpr int LAS = 53;
struct SoftA {
    const lds_double* A;
    __device__ double QT(int i, int k) const { return A[k * LAS + i]; }
    __device__ double QV(int i, int k) const { return A[k * LAS + 21 + i]; }
    __device__ double RT(int i, int k) const { return A[k * LAS + 27 + i]; }
    __device__ double RV(int i, int k) const { return A[k * LAS + 30 + i]; }
    __device__ double AJ(int i, int k) const { return A[k * LAS + 32 + i]; }
    __device__ double CR(int i, int k) const { return A[k * LAS + 41 + i]; }
    __device__ double SD(int i, int k) const { return A[k * LAS + 47 + i]; }
};
struct SoftG {
    const Ctx& c;
    __device__ double QT(int i, int k) const { return c.S(S_QT + i, k); }
    __device__ double QV(int i, int k) const { return c.S(S_QV + i, k); }
    __device__ double RT(int i, int k) const { return c.S(S_RT + i, k); }
    __device__ double RV(int i, int k) const { return c.S(S_RV + i, k); }
    __device__ double AJ(int i, int k) const { return c.S(S_AJ + i, k); }
    __device__ double CR(int i, int k) const { return c.S(S_CE + i, k); }
    __device__ double SD(int i, int k) const { return c.S(S_SD + i, k); }
};
__device__ __noinline__ void stage_soft_inputs(const Ctx& c, double* A) {
    const WsView vw = ws_view(c);
    stage_copy<LAS>(c, A, [&](int f, int k) -> double {
        int g;
        if (f < 21) g = S_QT + f;
        else if (f < 27) g = S_QV + f - 21;
        else if (f < 30) g = S_RT + f - 27;
        else if (f < 32) g = S_RV + f - 30;
        else if (f < 41) g = S_AJ + f - 32;
        else if (f < 47) g = S_CE + f - 41;
        else g = S_SD + f - 47;
        return (k < c.N || f < 27 || f >= 41) ? (double)vw.S(g, k) : 0.0;
    });
}
// operands of one soft stage: the softening of stage k (S entries of the lane) and the hard step k-1
struct SoftOps {
    double si, sj;
    RicOps r;
};
template <class Src>
__device__ __forceinline__ void soft_ops(const Src& src, int k, int i, int j, int sij, int r, bool vec, SoftOps& o) {
    o.si = src.SD(i, k);
    o.sj = src.SD(j, k);
    if (k > 0) ric_ops(src, k - 1, sij, r, vec, o.r);
}

template <class Src>
__device__ __noinline__ void riccati_soft(const Ctx& c, LShared& sh, const Src src) {
    const WsView vw = ws_view(c);
    const GSrc out{c};
    const int lane = threadIdx.x, N = c.N;
    const double dt = c.dt, dt2 = dt * dt;
    const bool act = lane < 36, vec = lane >= 48 && lane < 54;
    const int i = act ? lane / 6 : 0, j = act ? lane % 6 : 0, r = vec ? lane - 48 : 0;
    const int ii = min(i, j), jj = max(i, j), sij = sy6(ii, jj);
    const ColMask mj(j), mi(ii), mr(r);
    __shared__ double Pt[48], Yt[48], Tt[48];
    constexpr int DT = 47;                   // dead tile slot (no reader: entries are 8 i + j, i, j < 6)
    const int tij = act ? 8 * i + j : DT;    // this lane's tile entry, or the dead slot
    if (act) {
        const double q = src.QT(sij, N);
        Pt[8 * i + j] = q;
        if (i <= j) out.setP(sij, N, q);
    }
    double pv = vec ? src.QV(r, N) : 0.0;
    if (vec) out.setPV(r, N, pv);
    bool fail = false;
    int fcode = F_OK;
    lds_order();
    auto stage = [&](int k, const SoftOps& cur, SoftOps& nx) __attribute__((always_inline)) {
        if (k > 0) soft_ops(src, k - 1, i, j, sij, r, vec, nx);  // next stage's operands, one stage ahead
        // ---- soften stage k: M = I + S P S inverted by Gauss-Jordan in registers (lane 6i + j holds M[i][j]);
        // each pivot arrives by v_readlane, its row and column entries by ds_bpermute, so no LDS write / read
        // round trip sits on the six-pivot chain (same arithmetic as an LDS tile)
        double mv = act ? (i == j ? 1.0 : 0.0) + cur.si * Pt[8 * ii + jj] * cur.sj : 0.0;
        const double m0 = mv;  // M before elimination (its diagonal classifies a failed pivot)
#pragma unroll
        for (int p = 0; p < 6; ++p) {
            const double piv = readlane_d(mv, 7 * p);
            // (wave-uniform scalars: selected, not branched on)
            const int fc = pivot_fail(piv, readlane_d(m0, 7 * p));
            fcode = (!fail && !(piv >= 2.2250738585072014e-308)) ? fc : fcode;
            const double aip = __shfl(mv, 6 * i + p), apj = __shfl(mv, 6 * p + j);
            const double ip = 1.0 / piv;
            const double nv = bsel(i == p && j == p, ip, bsel(i == p, apj * ip, bsel(j == p, -aip * ip, mv - aip * apj * ip)));
            fail = fail || !(piv >= 2.2250738585072014e-308);
            mv = act ? nv : 0.0;
        }
        // Branch-free from here on: every lane evaluates the entry expressions at its clamped (i, j) / r and only the
        // stores are predicated -- tile stores of idle lanes go to the dead slot DT (no exec-mask branch around each
        // expression; the HBM stores keep theirs)
        const double mji = __shfl(mv, 6 * j + i);
        // Y = S M^-1 S from the upper entry (symmetric by construction)
        const double y = bsel(i <= j, cur.si * mv * cur.sj, cur.sj * mji * cur.si);
        Yt[tij] = y;
        if (act && i <= j) vw.S(S_Y + sij, k) = y;
        lds_order();
        {
            double t = 0.0;
#pragma unroll
            for (int l = 0; l < 6; ++l) t = fma(Pt[8 * i + l], Yt[8 * l + j], t);
            Tt[tij] = t;  // P Y
        }
        // p of lanes 48..53 to the lanes of their row (DPP row_newbcast: the vector lanes are its only readers)
        double pl[6];
        pl[0] = rowbc<0>(pv); pl[1] = rowbc<1>(pv); pl[2] = rowbc<2>(pv);
        pl[3] = rowbc<3>(pv); pl[4] = rowbc<4>(pv); pl[5] = rowbc<5>(pv);
        lds_order();
        double nP, npv = pv;
        {
            double t = Pt[8 * ii + jj];
#pragma unroll
            for (int l = 0; l < 6; ++l) t = fma(-Tt[8 * ii + l], Pt[8 * l + jj], t);
            nP = t;
        }
#pragma unroll
        for (int l = 0; l < 6; ++l) npv = fma(-Tt[8 * r + l], pl[l], npv);
        lds_order();
        Pt[tij] = nP;
        pv = npv;
        lds_order();
        if (k == 0) return;
        // ---- stage kk = k-1 on P~_k, p~_k
        const int kk = k - 1;
        const RicOps& o = cur.r;
        {  // PA[i][j] = P[i][j] + sum_{l<4} P[i][l] D[l][j]
            double c0, c1, c2, c3;
            dcol(o.dj, mj, c0, c1, c2, c3);
            Tt[tij] = fma(Pt[8 * i + 0], c0, fma(Pt[8 * i + 1], c1, fma(Pt[8 * i + 2], c2, fma(Pt[8 * i + 3], c3, Pt[8 * i + j]))));
        }
        double pp = pv;
#pragma unroll
        for (int q = 0; q < 6; ++q) pp = fma(-Pt[8 * r + q], o.e[q], pp);
        lds_order();
        const double G00 = o.R0 + dt2 * Pt[8 * 5 + 5], G01 = o.R1 + dt2 * Pt[8 * 5 + 4];
        const double G11 = o.R3 + dt2 * Pt[8 * 4 + 4];
        const double det = G00 * G11 - G01 * G01;
        const int gc = g2_code(G00, G11, det);
        if (!fail) fcode = gc;
        fail = fail || gc != F_OK;
        const double idet = 1.0 / det;
        const double Gi00 = G11 * idet, Gi01 = -G01 * idet, Gi11 = G00 * idet;
        double Pk;
        {  // P_kk[ii][jj] = Q~ + (A'PA)[ii][jj] + H'K
            double c0, c1, c2, c3;
            dcol(o.dj, mi, c0, c1, c2, c3);
            const double atpa = fma(c0, Tt[8 * 0 + jj], fma(c1, Tt[8 * 1 + jj], fma(c2, Tt[8 * 2 + jj], fma(c3, Tt[8 * 3 + jj], Tt[8 * ii + jj]))));
            const double H0i = dt * Tt[8 * 5 + ii], H1i = dt * Tt[8 * 4 + ii], H0j = dt * Tt[8 * 5 + jj], H1j = dt * Tt[8 * 4 + jj];
            const double K0j = -fma(Gi00, H0j, Gi01 * H1j), K1j = -fma(Gi01, H0j, Gi11 * H1j);
            Pk = o.qt + atpa + fma(H0i, K0j, H1i * K1j);
        }
        double ppl[6];
        ppl[0] = rowbc<0>(pp); ppl[1] = rowbc<1>(pp); ppl[2] = rowbc<2>(pp);
        ppl[3] = rowbc<3>(pp); ppl[4] = rowbc<4>(pp); ppl[5] = rowbc<5>(pp);
        const double g0 = fma(dt, ppl[5], o.rv0), g1 = fma(dt, ppl[4], o.rv1);
        const double kf0 = -fma(Gi00, g0, Gi01 * g1), kf1 = -fma(Gi01, g0, Gi11 * g1);
        double pnew;
        {
            double c0, c1, c2, c3;
            dcol(o.dj, mr, c0, c1, c2, c3);
            double ppr = ppl[0];
#pragma unroll
            for (int q = 1; q < 6; ++q) ppr = bsel(r == q, ppl[q], ppr);
            const double H0 = dt * Tt[8 * 5 + r], H1 = dt * Tt[8 * 4 + r];
            pnew = o.qv + fma(c0, ppl[0], fma(c1, ppl[1], fma(c2, ppl[2], fma(c3, ppl[3], ppr)))) + fma(H0, kf0, H1 * kf1);
            const double K0 = -fma(Gi00, H0, Gi01 * H1), K1 = -fma(Gi01, H0, Gi11 * H1);
            if (vec) {
                out.setK(r, kk, K0);
                out.setK(6 + r, kk, K1);
                out.setPV(r, kk, pnew);
            }
        }
        if (lane == 48) {
            out.setKF(0, kk, kf0);
            out.setKF(1, kk, kf1);
            if (c.refine) { vw.S(S_GI, kk) = Gi00; vw.S(S_GI + 1, kk) = Gi01; vw.S(S_GI + 2, kk) = Gi11; }
        }
        if (act && i <= j) out.setP(sij, kk, Pk);
        lds_order();
        Pt[tij] = Pk;
        pv = pnew;
        lds_order();
    };
    SoftOps oa, ob;
    soft_ops(src, N, i, j, sij, r, vec, oa);
    int k = N;
    for (; k >= 1; k -= 2) {
        stage(k, oa, ob);
        stage(k - 1, ob, oa);
        // stop at the first failed pivot (M or G): the attempt is discarded (fail is wave-uniform -- pivots by
        // v_readlane, G from tile broadcasts)
        if (__builtin_amdgcn_readfirstlane((int)fail)) break;
    }
    if (k == 0 && !fail) stage(0, oa, ob);
    if (lane == 0) sh.flag = fcode;
    wave_sync();
}

// forward sweep with soft rows: yhat = A dx + B du - r~; dx = yhat - Y (P yhat + p).  Operands from LDS
// copies staged by all four waves (SoftF) or from HBM (GSrc + S_Y); the 6-vector chain is carried by
// every lane (wave-uniform), lanes 0..5 write row r of the stage outputs.
// staged record per stage: P 21 | PV 6 | K 12 | KF 2 | Y 21 | AJ 9 | CE 6  (77)
constexpr int LFS = 77;
struct SoftF {
    const lds_double* A;
    __device__ double P(int i, int k) const { return A[k * LFS + i]; }
    __device__ double PV(int i, int k) const { return A[k * LFS + 21 + i]; }
    __device__ double K(int i, int k) const { return A[k * LFS + 27 + i]; }
    __device__ double KF(int i, int k) const { return A[k * LFS + 39 + i]; }
    __device__ double Y(int i, int k) const { return A[k * LFS + 41 + i]; }
    __device__ double AJ(int i, int k) const { return A[k * LFS + 62 + i]; }
    __device__ double CR(int i, int k) const { return A[k * LFS + 71 + i]; }
};
struct SoftFG {
    const Ctx& c;
    __device__ double P(int i, int k) const { return c.S(S_P + i, k); }
    __device__ double PV(int i, int k) const { return c.S(S_PV + i, k); }
    __device__ double K(int i, int k) const { return c.S(S_K + i, k); }
    __device__ double KF(int i, int k) const { return c.S(S_KF + i, k); }
    __device__ double Y(int i, int k) const { return c.S(S_Y + i, k); }
    __device__ double AJ(int i, int k) const { return c.S(S_AJ + i, k); }
    __device__ double CR(int i, int k) const { return c.S(S_CE + i, k); }
};
__device__ __noinline__ void stage_soft_forward(const Ctx& c, double* A, bool soft = true) {
    const WsView vw = ws_view(c);
    stage_copy<LFS>(c, A, [&](int f, int k) -> double {
        if (!soft && f >= 41 && f < 62) return 0.0;  // hard rows: Y unused
        int g;
        if (f < 21) g = S_P + f;
        else if (f < 27) g = S_PV + f - 21;
        else if (f < 39) g = S_K + f - 27;
        else if (f < 41) g = S_KF + f - 39;
        else if (f < 62) g = S_Y + f - 41;
        else if (f < 71) g = S_AJ + f - 62;
        else g = S_CE + f - 71;
        return (k < c.N || f < 27 || (f >= 41 && f < 62) || f >= 71) ? (double)vw.S(g, k) : 0.0;
    });
}
template <class Src>
__device__ __noinline__ void forward_soft(const Ctx& c, const Src src, int buf) {
    const WsView vw = ws_view(c);
    const int lane = threadIdx.x, N = c.N;
    const double dt = c.dt;
    // lanes 0..5 own dx[q] (q = lane); the 6-vectors the rows need (dx, P dx + p) arrive by DPP row_newbcast, so each
    // lane reads only its own rows of P and Y.  Same operations in the same order as the redundant form (bitwise).
    // The stage's operands are read one stage ahead of their use (ping-pong operand sets).
    const int q = lane < 6 ? lane : 0;
    struct Ops {
        double pv, p[6], y[6], kf0, kf1, K[12], aj[9], e;
    };
    auto load = [&](int k, Ops& o) __attribute__((always_inline)) {
        o.pv = src.PV(q, k);
#pragma unroll
        for (int l = 0; l < 6; ++l) { o.p[l] = src.P(sy6(q, l), k); o.y[l] = src.Y(sy6(q, l), k); }
        if (k < N) {
            o.kf0 = src.KF(0, k);
            o.kf1 = src.KF(1, k);
#pragma unroll
            for (int l = 0; l < 12; ++l) o.K[l] = src.K(l, k);
#pragma unroll
            for (int l = 0; l < 9; ++l) o.aj[l] = src.AJ(l, k);
            o.e = src.CR(q, k + 1);
        }
    };
    double dq = -src.CR(q, 0);
    // one stage; returns false after the terminal stage
    auto stage = [&](int k, const Ops& o) __attribute__((always_inline)) -> bool {
        double d[6];
        d[0] = rowbc<0>(dq); d[1] = rowbc<1>(dq); d[2] = rowbc<2>(dq);
        d[3] = rowbc<3>(dq); d[4] = rowbc<4>(dq); d[5] = rowbc<5>(dq);
        double bq = o.pv;
#pragma unroll
        for (int l = 0; l < 6; ++l) bq = fma(o.p[l], d[l], bq);
        double bv[6];
        bv[0] = rowbc<0>(bq); bv[1] = rowbc<1>(bq); bv[2] = rowbc<2>(bq);
        bv[3] = rowbc<3>(bq); bv[4] = rowbc<4>(bq); bv[5] = rowbc<5>(bq);
        {
            double t = 0.0;
#pragma unroll
            for (int l = 0; l < 6; ++l) t = fma(o.y[l], bv[l], t);
            dq -= t;
        }
        d[0] = rowbc<0>(dq); d[1] = rowbc<1>(dq); d[2] = rowbc<2>(dq);
        d[3] = rowbc<3>(dq); d[4] = rowbc<4>(dq); d[5] = rowbc<5>(dq);
        {
            double t = o.pv;
#pragma unroll
            for (int l = 0; l < 6; ++l) t = fma(o.p[l], d[l], t);
            if (lane < 6) {
                vw.S(S_YCP + 6 * buf + q, k) = -t;
                vw.S(S_DX + 6 * buf + q, k) = dq;
            }
        }
        if (k == N) return false;
        double du0 = o.kf0, du1 = o.kf1;
#pragma unroll
        for (int l = 0; l < 6; ++l) {
            du0 = fma(o.K[l], d[l], du0);
            du1 = fma(o.K[6 + l], d[l], du1);
        }
        if (lane == 0) {
            vw.S(S_DU + 2 * buf, k) = du0;
            vw.S(S_DU + 2 * buf + 1, k) = du1;
        }
        const double* aj = o.aj;
        const double eq = o.e;
        const double n0 = (d[0] - eq) + fma(aj[0], d[2], aj[1] * d[5]);
        const double n1 = (d[1] - eq) + fma(aj[2], d[2], aj[3] * d[5]);
        const double n2 = (d[2] - eq) + fma(aj[4], d[4], aj[5] * d[5]);
        const double n3 = (d[3] - eq) + fma(aj[6], d[3], fma(aj[7], d[4], aj[8] * d[5]));
        const double n4 = (d[4] - eq) + dt * du1;
        const double n5 = (d[5] - eq) + dt * du0;
        dq = sel6(q, n0, n1, n2, n3, n4, n5);
        return true;
    };
    Ops oa, ob;
    load(0, oa);
    for (int k = 0;; k += 2) {
        if (k + 1 <= N) load(k + 1, ob);
        if (!stage(k, oa)) break;
        if (k + 2 <= N) load(k + 2, oa);
        if (!stage(k + 1, ob)) break;
    }
}

// elastic-pair step of one row from its new multiplier: dp = (y+ - g_p)/D_p, dn = (-y+ - g_n)/D_n, plus
// fraction to the boundary (p, n >= 0; z_p, z_n >= 0), directional derivative and relative step size
__device__ __forceinline__ void pn_step(double p, double n, double zp, double zn, double yp, double mu, double dw,
                                        double tau, double& dp, double& dn, double& ap, double& az, double& Dm,
                                        double& rel) {
    const PN t = pn_terms(false, p, n, zp, zn, mu, dw);
    dp = (yp - t.gp) / t.Dp;
    dn = (-yp - t.gn) / t.Dn;
    ftb_lo(p, 0.0, dp, tau, ap);
    ftb_lo(n, 0.0, dn, tau, ap);
    const double dzp = mu / p - zp - zp / p * dp, dzn = mu / n - zn - zn / n * dn;
    if (dzp < 0.0) az = fmin(az, -tau * zp / dzp);
    if (dzn < 0.0) az = fmin(az, -tau * zn / dzn);
    Dm += t.gp * dp + t.gn * dn;
    rel = fmax(rel, fmax(fabs(dp) / (1.0 + fabs(p)), fabs(dn) / (1.0 + fabs(n))));
}

// ======== phase: block step recovery + fraction to boundary + directional derivative ========
// out: [0] alpha_primal (min), [1] alpha_dual (min), [2] grad phi' d (sum), [3] max relative step,
//      [4] max |y+| (least-squares multiplier test)
__device__ __noinline__ void phase_recover(const Ctx& c, LShared& sh, double mu, double dw, double tau, int buf,
                                           double (&out)[5]) {
    const WsView vw = ws_view(c);
    const int N = c.N;
    const bool plan = c.plan(), rs = sh.R != 0 && !sh.lsq, lsq = sh.lsq != 0;
    double ap = 1.0, az = 1.0, Dm = 0.0, rel = 0.0, ymax = 0.0;
    for (int k = (int)threadIdx.x; k <= N; k += T) {
        double x[6], dx[6];
        load_x(c, k, x);
#pragma unroll
        for (int i = 0; i < 6; ++i) dx[i] = vw.S(S_DX + 6 * buf + i, k);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const double xv = x[i], d = dx[i];
            double g = vw.S(S_GX + i, k);
            rel = fmax(rel, fabs(d) / (1.0 + fabs(xv)));
            if (c.hlx(i)) {
                const double sl = xv - c.xl[i], z = vw.S(S_ZLX + i, k);
                g -= mu / sl;
                ftb_lo(xv, c.xl[i], d, tau, ap);
                const double dz = mu / sl - z - z / sl * d;
                if (dz < 0.0) az = fmin(az, -tau * z / dz);
            }
            if (c.hux(i)) {
                const double sl = c.xu[i] - xv, z = vw.S(S_ZUX + i, k);
                g += mu / sl;
                ftb_hi(xv, c.xu[i], d, tau, ap);
                const double dz = mu / sl - z + z / sl * d;
                if (dz < 0.0) az = fmin(az, -tau * z / dz);
            }
            Dm += g * d;
            const double yp = vw.S(S_YCP + 6 * buf + i, k);
            ymax = fmax(ymax, fabs(yp));
            if (rs) {
                double dp, dn;
                pn_step(vw.S(S_PR + i, k), vw.S(S_NR + i, k), vw.S(S_ZP + i, k), vw.S(S_ZN + i, k), yp, mu, dw, tau, dp, dn,
                        ap, az, Dm, rel);
                vw.S(S_DP + 6 * buf + i, k) = dp;
                vw.S(S_DN + 6 * buf + i, k) = dn;
            }
        }
        if (k < N)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const double uv = vw.S(S_U + i, k), d = vw.S(S_DU + 2 * buf + i, k);
                double g = vw.S(S_GU + i, k);
                rel = fmax(rel, fabs(d) / (1.0 + fabs(uv)));
                if (c.hlu(i)) {
                    const double sl = uv - c.ul[i], z = vw.S(S_ZLU + i, k);
                    g -= mu / sl;
                    ftb_lo(uv, c.ul[i], d, tau, ap);
                    const double dz = mu / sl - z - z / sl * d;
                    if (dz < 0.0) az = fmin(az, -tau * z / dz);
                }
                if (c.huu(i)) {
                    const double sl = c.uu[i] - uv, z = vw.S(S_ZUU + i, k);
                    g += mu / sl;
                    ftb_hi(uv, c.uu[i], d, tau, ap);
                    const double dz = mu / sl - z + z / sl * d;
                    if (dz < 0.0) az = fmin(az, -tau * z / dz);
                }
                Dm += g * d;
            }
        const Trig tr = stage_trig(x);
        for (int j = 0; j < c.nbk; ++j) {
            Blk bk;
            bk.m = c.slab + threadIdx.x;
            double fw[8], zf[8], t4[4], yp[4], dwv[8];
            BlkIn in;
            load_blk_in(c, sh.R != 0, j, k, in);
            block_refactor<true>(c, sh, in, j, x, tr, mu, dw, bk, fw, zf, t4);
            blk_recover(bk, fw, zf, t4, dx, yp, dwv);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const double wv = in.w[e], z = in.zw[e], sl = wv + RELAX, d = dwv[e];
                vw.B(B_DW + 8 * buf + e, j, k) = d;
                rel = fmax(rel, fabs(d) / (1.0 + fabs(wv)));
                Dm += fw[e] * d;
                ftb_lo(wv, -RELAX, d, tau, ap);
                const double dz = mu / sl - z - z / sl * d;
                if (dz < 0.0) az = fmin(az, -tau * z / dz);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double s = in.s[r], vl = in.vl[r], vu = in.vu[r];
                const double gs = lsq ? (c.hrl(r) ? -vl : 0.0) + vu : grad_row(c, r, s, mu);
                const double ds = (yp[r] - gs) / bk.D[r];
                vw.B(B_YP + 4 * buf + r, j, k) = yp[r];
                vw.B(B_DS + 4 * buf + r, j, k) = ds;
                ymax = fmax(ymax, fabs(yp[r]));
                rel = fmax(rel, fabs(ds) / (1.0 + fabs(s)));
                Dm += gs * ds;
                const double slu = c.rU(r) - s;
                ftb_hi(s, c.rU(r), ds, tau, ap);
                const double dvu = mu / slu - vu + vu / slu * ds;
                if (dvu < 0.0) az = fmin(az, -tau * vu / dvu);
                if (c.hrl(r)) {
                    const double sll = s - c.rL(r);
                    ftb_lo(s, c.rL(r), ds, tau, ap);
                    const double dvl = mu / sll - vl - vl / sll * ds;
                    if (dvl < 0.0) az = fmin(az, -tau * vl / dvl);
                }
                if (rs) {
                    double dp, dn;
                    pn_step(in.pr[r], in.nr[r], in.zp[r], in.zn[r], yp[r], mu, dw, tau, dp, dn, ap, az, Dm, rel);
                    vw.B(B_DP + 4 * buf + r, j, k) = dp;
                    vw.B(B_DN + 4 * buf + r, j, k) = dn;
                }
            }
        }
        if (k == N && plan)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double sl = sh.sf[i] - c.fL, su = c.fU - sh.sf[i];
                const double gs = lsq ? -sh.vLf[i] + sh.vUf[i] : -mu / sl + mu / su;
                const double yp = sh.Dfe[i] * (dx[i] + sh.rf[i]);
                const double ds = (yp - gs) / sh.Dsf[i];
                sh.ydpf[buf][i] = yp;
                sh.dsf[buf][i] = ds;
                ymax = fmax(ymax, fabs(yp));
                rel = fmax(rel, fabs(ds) / (1.0 + fabs(sh.sf[i])));
                Dm += gs * ds;
                ftb_lo(sh.sf[i], c.fL, ds, tau, ap);
                ftb_hi(sh.sf[i], c.fU, ds, tau, ap);
                const double dvl = mu / sl - sh.vLf[i] - sh.vLf[i] / sl * ds;
                const double dvu = mu / su - sh.vUf[i] + sh.vUf[i] / su * ds;
                if (dvl < 0.0) az = fmin(az, -tau * sh.vLf[i] / dvl);
                if (dvu < 0.0) az = fmin(az, -tau * sh.vUf[i] / dvu);
                if (rs) {
                    double dp, dn;
                    pn_step(sh.pf[i], sh.nf[i], sh.zpf[i], sh.znf[i], yp, mu, dw, tau, dp, dn, ap, az, Dm, rel);
                    sh.dpf[buf][i] = dp;
                    sh.dnf[buf][i] = dn;
                }
            }
    }
    if (!isfinite(ymax)) ymax = INFINITY;
    out[0] = ap; out[1] = az; out[2] = Dm; out[3] = rel; out[4] = ymax;
    const int ops[5] = {R_MIN, R_MIN, R_SUM, R_MAX, R_MAX};
    wg_reduce(sh, out, ops);
}

// ======== phase: trial point x + alpha d (step buffer buf) -> theta, phi (barrier objective), bad ========
// of the current NLP; also stores the trial residual rows (for second-order corrections)
template <bool RS_>
__device__ __noinline__ void phase_trial_t(const Ctx& c, LShared& sh, double mu, double alpha, int buf, double (&out)[3]) {
    LArgs& a = *c.a;
    const int N = c.N;
    const bool plan = c.plan();
    constexpr bool rs = RS_;
    double th = 0.0, F = 0.0, logs = 0.0, bad = 0.0;
    for (int k = (int)threadIdx.x; k <= N; k += T) {
        double x[6], u[2] = {0.0, 0.0};
#pragma unroll
        for (int i = 0; i < 6; ++i) x[i] = c.S(S_X + i, k) + alpha * c.S(S_DX + 6 * buf + i, k);
        if (k < N)
#pragma unroll
            for (int i = 0; i < 2; ++i) u[i] = c.S(S_U + i, k) + alpha * c.S(S_DU + 2 * buf + i, k);
        // the tracking / plan cost first: its target loads are issued before any of the pass's stores (a load behind a
        // store waits for it)
        const double scost = rs ? 0.0 : stage_cost(c, k, x, u);
        LogSum ls;
        bool ok = true;
        double Fr = 0.0, prox = 0.0;  // restoration objective of this stage: rho sum(p + n), D_R-weighted distances
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            if (c.hlx(i)) { const double sl = x[i] - c.xl[i]; ok &= sl > 0.0; ls.add(sl); }
            if (c.hux(i)) { const double sl = c.xu[i] - x[i]; ok &= sl > 0.0; ls.add(sl); }
            if (rs) { const double e = x[i] - c.S(S_XR + i, k); prox += c.S(S_DRX + i, k) * e * e; }
        }
        if (k < N)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                if (c.hlu(i)) { const double sl = u[i] - c.ul[i]; ok &= sl > 0.0; ls.add(sl); }
                if (c.huu(i)) { const double sl = c.uu[i] - u[i]; ok &= sl > 0.0; ls.add(sl); }
                if (rs) { const double e = u[i] - c.S(S_UR + i, k); prox += c.S(S_DRU + i, k) * e * e; }
            }
        // dynamics residual c_{k+1} = x_{k+1} - F(x_k, u_k) (thread k), c_0 = x_0 - x_init; stored after the
        // block loop (and each block's trial residual after the next block's loads): a store ahead of a load
        // in the in-order vmcnt queue makes the load's wait include it
        double ck[6] = {0, 0, 0, 0, 0, 0}, cn[6] = {0, 0, 0, 0, 0, 0};
        if (k == 0) {
#pragma unroll
            for (int i = 0; i < 6; ++i) ck[i] = x[i] - a.x0[6 * (size_t)c.b + i];
        }
        if (k < N) {
            double fo[6];
            model_f(a, x, u, fo);
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double xn = c.S(S_X + i, k + 1) + alpha * c.S(S_DX + 6 * buf + i, k + 1);
                double cv = xn - (x[i] + a.dt * fo[i]);
                if (rs) {  // row of stage k+1 (owned there: read its elastic pair)
                    const double p = c.S(S_PR + i, k + 1) + alpha * c.S(S_DP + 6 * buf + i, k + 1);
                    const double n = c.S(S_NR + i, k + 1) + alpha * c.S(S_DN + 6 * buf + i, k + 1);
                    cv -= p - n;
                }
                cn[i] = cv;
                th += fabs(cv);
            }
        }
        if (rs)  // elastic pairs of this stage's own dynamics rows: barrier + objective (+ row 0's residual)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double p = c.S(S_PR + i, k) + alpha * c.S(S_DP + 6 * buf + i, k);
                const double n = c.S(S_NR + i, k) + alpha * c.S(S_DN + 6 * buf + i, k);
                ok &= p > 0.0 && n > 0.0;
                ls.add(p);
                ls.add(n);
                Fr += p + n;
                if (k == 0) ck[i] -= p - n;
            }
        if (k == 0)
#pragma unroll
            for (int i = 0; i < 6; ++i) th += fabs(ck[i]);
        const Trig tr = stage_trig(x);
        double pdt[4] = {0, 0, 0, 0};
        int pj = -1;
        for (int j = 0; j < c.nbk; ++j) {
            double w[8], d[4], wr[8], drw[8], sv[4], pv[4], nv[4];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                w[e] = c.B(B_W + e, j, k) + alpha * c.B(B_DW + 8 * buf + e, j, k);
                if (rs) { wr[e] = c.B(B_WR + e, j, k); drw[e] = c.B(B_DRW + e, j, k); }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                sv[r] = c.B(B_S + r, j, k) + alpha * c.B(B_DS + 4 * buf + r, j, k);
                if (rs) {
                    pv[r] = c.B(B_PR + r, j, k) + alpha * c.B(B_DP + 4 * buf + r, j, k);
                    nv[r] = c.B(B_NR + r, j, k) + alpha * c.B(B_DN + 4 * buf + r, j, k);
                }
            }
            if (pj >= 0)
#pragma unroll
                for (int r = 0; r < 4; ++r) c.B(B_DT + r, pj, k) = pdt[r];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const double sl = w[e] + RELAX;
                ok &= sl > 0.0;
                ls.add(sl);
                if (rs) { const double ew = w[e] - wr[e]; prox += drw[e] * ew * ew; }
            }
            blk_vals(a, x, tr, j, w, d);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double s = sv[r];
                double res = d[r] - s;
                if (rs) {
                    const double p = pv[r];
                    const double n = nv[r];
                    ok &= p > 0.0 && n > 0.0;
                    ls.add(p);
                    ls.add(n);
                    Fr += p + n;
                    res -= p - n;
                }
                pdt[r] = res;
                th += fabs(res);
                const double su = c.rU(r) - s;
                ok &= su > 0.0;
                ls.add(su);
                if (c.hrl(r)) { const double sl = s - c.rL(r); ok &= sl > 0.0; ls.add(sl); }
            }
            pj = j;
        }
        if (pj >= 0)
#pragma unroll
            for (int r = 0; r < 4; ++r) c.B(B_DT + r, pj, k) = pdt[r];
        if (k < N)
#pragma unroll
            for (int i = 0; i < 6; ++i) c.S(S_CT + i, k + 1) = cn[i];
        if (k == 0)
#pragma unroll
            for (int i = 0; i < 6; ++i) c.S(S_CT + i, 0) = ck[i];
        if (k == N && plan)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double s = sh.sf[i] + alpha * sh.dsf[buf][i];
                double res = (x[i] - c.tgt_x[i]) - s;
                if (rs) {
                    const double p = sh.pf[i] + alpha * sh.dpf[buf][i], n = sh.nf[i] + alpha * sh.dnf[buf][i];
                    ok &= p > 0.0 && n > 0.0;
                    ls.add(p);
                    ls.add(n);
                    Fr += p + n;
                    res -= p - n;
                }
                sh.dft[i] = res;
                th += fabs(res);
                const double sl = s - c.fL, su = c.fU - s;
                ok &= sl > 0.0 && su > 0.0;
                ls.add(sl);
                ls.add(su);
            }
        F += rs ? RHO * Fr + 0.5 * sh.zeta * prox : scost;
        if (!ok) bad = 1.0;
        else logs += ls.value();
    }
    double v[4] = {th, F, logs, bad};
    const int ops[4] = {R_SUM, R_SUM, R_SUM, R_MAX};
    wg_reduce(sh, v, ops);
    out[0] = v[3] > 0.0 ? INFINITY : v[0];
    out[1] = v[3] > 0.0 ? INFINITY : v[1] - mu * v[2];
    out[2] = v[3];
}

// one instantiation per problem (original / restoration phase): the original problem's skips every restoration
// branch and its loads (bitwise the same results, profiles/r03/ab_one/)
__device__ __forceinline__ void phase_trial(const Ctx& c, LShared& sh, double mu, double alpha, int buf, double (&out)[3]) {
    sh.R ? phase_trial_t<true>(c, sh, mu, alpha, buf, out) : phase_trial_t<false>(c, sh, mu, alpha, buf, out);
}


// ======== phase: NA line-search trial points in one pass (the backtracking trials after the first) ========
// The filter line search tries alpha, alpha/2, ... one after the other (8.8 trial points per iteration in the C4 tail,
// profiles/r05/session_o/tail.txt), and each trial is a full pass over the trajectory whose time is its memory latency,
// not its arithmetic.  This pass loads the iterate and the step once and evaluates NA step lengths: for each the same
// expressions as phase_trial_t in the same order, so out[a] is bitwise phase_trial_t's result for alphas[a].  No
// trial residual rows are stored: only the first trial of an iteration feeds a second-order correction.
template <bool RS_, int NA>
__device__ __noinline__ void phase_trial_multi_t(const Ctx& c, LShared& sh, double mu, const double (&al)[NA], int buf,
                                                 double (&out)[NA][3]) {
    LArgs& a = *c.a;
    const int N = c.N;
    const bool plan = c.plan();
    constexpr bool rs = RS_;
    double th[NA], F[NA], logs[NA], bad[NA];
#pragma unroll
    for (int q = 0; q < NA; ++q) { th[q] = 0.0; F[q] = 0.0; logs[q] = 0.0; bad[q] = 0.0; }
    for (int k = (int)threadIdx.x; k <= N; k += T) {
        double X[6], DX[6], U[2] = {0.0, 0.0}, DU[2] = {0.0, 0.0};
#pragma unroll
        for (int i = 0; i < 6; ++i) { X[i] = c.S(S_X + i, k); DX[i] = c.S(S_DX + 6 * buf + i, k); }
        if (k < N)
#pragma unroll
            for (int i = 0; i < 2; ++i) { U[i] = c.S(S_U + i, k); DU[i] = c.S(S_DU + 2 * buf + i, k); }
        double x[NA][6], u[NA][2];
#pragma unroll
        for (int q = 0; q < NA; ++q) {
#pragma unroll
            for (int i = 0; i < 6; ++i) x[q][i] = X[i] + al[q] * DX[i];
#pragma unroll
            for (int i = 0; i < 2; ++i) u[q][i] = k < N ? U[i] + al[q] * DU[i] : 0.0;
        }
        double scost[NA];
#pragma unroll
        for (int q = 0; q < NA; ++q) scost[q] = rs ? 0.0 : stage_cost(c, k, x[q], u[q]);
        LogSum ls[NA];
        bool ok[NA];
        double Fr[NA], prox[NA];
#pragma unroll
        for (int q = 0; q < NA; ++q) { ok[q] = true; Fr[q] = 0.0; prox[q] = 0.0; }
        double xr[6], drx[6];
        if (rs)
#pragma unroll
            for (int i = 0; i < 6; ++i) { xr[i] = c.S(S_XR + i, k); drx[i] = c.S(S_DRX + i, k); }
#pragma unroll
        for (int q = 0; q < NA; ++q)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                if (c.hlx(i)) { const double sl = x[q][i] - c.xl[i]; ok[q] &= sl > 0.0; ls[q].add(sl); }
                if (c.hux(i)) { const double sl = c.xu[i] - x[q][i]; ok[q] &= sl > 0.0; ls[q].add(sl); }
                if (rs) { const double e = x[q][i] - xr[i]; prox[q] += drx[i] * e * e; }
            }
        if (k < N) {
            double ur[2], dru[2];
            if (rs)
#pragma unroll
                for (int i = 0; i < 2; ++i) { ur[i] = c.S(S_UR + i, k); dru[i] = c.S(S_DRU + i, k); }
#pragma unroll
            for (int q = 0; q < NA; ++q)
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    if (c.hlu(i)) { const double sl = u[q][i] - c.ul[i]; ok[q] &= sl > 0.0; ls[q].add(sl); }
                    if (c.huu(i)) { const double sl = c.uu[i] - u[q][i]; ok[q] &= sl > 0.0; ls[q].add(sl); }
                    if (rs) { const double e = u[q][i] - ur[i]; prox[q] += dru[i] * e * e; }
                }
        }
        double ck[NA][6];
#pragma unroll
        for (int q = 0; q < NA; ++q)
#pragma unroll
            for (int i = 0; i < 6; ++i) ck[q][i] = k == 0 ? x[q][i] - a.x0[6 * (size_t)c.b + i] : 0.0;
        if (k < N) {
            double XN[6], DXN[6], PN[6], DPN[6], NN[6], DNN[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                XN[i] = c.S(S_X + i, k + 1); DXN[i] = c.S(S_DX + 6 * buf + i, k + 1);
                if (rs) {
                    PN[i] = c.S(S_PR + i, k + 1); DPN[i] = c.S(S_DP + 6 * buf + i, k + 1);
                    NN[i] = c.S(S_NR + i, k + 1); DNN[i] = c.S(S_DN + 6 * buf + i, k + 1);
                }
            }
#pragma unroll
            for (int q = 0; q < NA; ++q) {
                double fo[6];
                model_f(a, x[q], u[q], fo);
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    const double xn = XN[i] + al[q] * DXN[i];
                    double cv = xn - (x[q][i] + a.dt * fo[i]);
                    if (rs) {
                        const double p = PN[i] + al[q] * DPN[i];
                        const double n = NN[i] + al[q] * DNN[i];
                        cv -= p - n;
                    }
                    th[q] += fabs(cv);
                }
            }
        }
        if (rs) {
            double P0[6], DP0[6], N0[6], DN0[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                P0[i] = c.S(S_PR + i, k); DP0[i] = c.S(S_DP + 6 * buf + i, k);
                N0[i] = c.S(S_NR + i, k); DN0[i] = c.S(S_DN + 6 * buf + i, k);
            }
#pragma unroll
            for (int q = 0; q < NA; ++q)
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    const double p = P0[i] + al[q] * DP0[i];
                    const double n = N0[i] + al[q] * DN0[i];
                    ok[q] &= p > 0.0 && n > 0.0;
                    ls[q].add(p);
                    ls[q].add(n);
                    Fr[q] += p + n;
                    if (k == 0) ck[q][i] -= p - n;
                }
        }
        if (k == 0)
#pragma unroll
            for (int q = 0; q < NA; ++q)
#pragma unroll
                for (int i = 0; i < 6; ++i) th[q] += fabs(ck[q][i]);
        Trig tr[NA];
#pragma unroll
        for (int q = 0; q < NA; ++q) tr[q] = stage_trig(x[q]);
        for (int j = 0; j < c.nbk; ++j) {
            double W[8], DW[8], wr[8], drw[8], S[4], DS[4], PV[4], DPV[4], NV[4], DNV[4];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                W[e] = c.B(B_W + e, j, k); DW[e] = c.B(B_DW + 8 * buf + e, j, k);
                if (rs) { wr[e] = c.B(B_WR + e, j, k); drw[e] = c.B(B_DRW + e, j, k); }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                S[r] = c.B(B_S + r, j, k); DS[r] = c.B(B_DS + 4 * buf + r, j, k);
                if (rs) {
                    PV[r] = c.B(B_PR + r, j, k); DPV[r] = c.B(B_DP + 4 * buf + r, j, k);
                    NV[r] = c.B(B_NR + r, j, k); DNV[r] = c.B(B_DN + 4 * buf + r, j, k);
                }
            }
#pragma unroll
            for (int q = 0; q < NA; ++q) {
                double w[8], d[4];
#pragma unroll
                for (int e = 0; e < 8; ++e) w[e] = W[e] + al[q] * DW[e];
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const double sl = w[e] + RELAX;
                    ok[q] &= sl > 0.0;
                    ls[q].add(sl);
                    if (rs) { const double ew = w[e] - wr[e]; prox[q] += drw[e] * ew * ew; }
                }
                blk_vals(a, x[q], tr[q], j, w, d);
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const double s = S[r] + al[q] * DS[r];
                    double res = d[r] - s;
                    if (rs) {
                        const double p = PV[r] + al[q] * DPV[r];
                        const double n = NV[r] + al[q] * DNV[r];
                        ok[q] &= p > 0.0 && n > 0.0;
                        ls[q].add(p);
                        ls[q].add(n);
                        Fr[q] += p + n;
                        res -= p - n;
                    }
                    th[q] += fabs(res);
                    const double su = c.rU(r) - s;
                    ok[q] &= su > 0.0;
                    ls[q].add(su);
                    if (c.hrl(r)) { const double sl = s - c.rL(r); ok[q] &= sl > 0.0; ls[q].add(sl); }
                }
            }
        }
        if (k == N && plan)
#pragma unroll
            for (int q = 0; q < NA; ++q)
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    const double s = sh.sf[i] + al[q] * sh.dsf[buf][i];
                    double res = (x[q][i] - c.tgt_x[i]) - s;
                    if (rs) {
                        const double p = sh.pf[i] + al[q] * sh.dpf[buf][i], n = sh.nf[i] + al[q] * sh.dnf[buf][i];
                        ok[q] &= p > 0.0 && n > 0.0;
                        ls[q].add(p);
                        ls[q].add(n);
                        Fr[q] += p + n;
                        res -= p - n;
                    }
                    th[q] += fabs(res);
                    const double sl = s - c.fL, su = c.fU - s;
                    ok[q] &= sl > 0.0 && su > 0.0;
                    ls[q].add(sl);
                    ls[q].add(su);
                }
#pragma unroll
        for (int q = 0; q < NA; ++q) {
            F[q] += rs ? RHO * Fr[q] + 0.5 * sh.zeta * prox[q] : scost[q];
            if (!ok[q]) bad[q] = 1.0;
            else logs[q] += ls[q].value();
        }
    }
    double v[4 * NA];
    int ops[4 * NA];
#pragma unroll
    for (int q = 0; q < NA; ++q) {
        v[4 * q] = th[q]; v[4 * q + 1] = F[q]; v[4 * q + 2] = logs[q]; v[4 * q + 3] = bad[q];
        ops[4 * q] = R_SUM; ops[4 * q + 1] = R_SUM; ops[4 * q + 2] = R_SUM; ops[4 * q + 3] = R_MAX;
    }
    wg_reduce(sh, v, ops);
#pragma unroll
    for (int q = 0; q < NA; ++q) {
        out[q][0] = v[4 * q + 3] > 0.0 ? INFINITY : v[4 * q];
        out[q][1] = v[4 * q + 3] > 0.0 ? INFINITY : v[4 * q + 1] - mu * v[4 * q + 2];
        out[q][2] = v[4 * q + 3];
    }
}
#ifndef OBCA_TRIAL_BATCH
#define OBCA_TRIAL_BATCH 4
#endif
constexpr int kTrialBatch = OBCA_TRIAL_BATCH;  // trials per batched pass (A/B builds: -DOBCA_TRIAL_BATCH=n)
__device__ __forceinline__ void phase_trial_multi(const Ctx& c, LShared& sh, double mu, const double (&al)[kTrialBatch],
                                                  int buf, double (&out)[kTrialBatch][3]) {
    sh.R ? phase_trial_multi_t<true, kTrialBatch>(c, sh, mu, al, buf, out)
         : phase_trial_multi_t<false, kTrialBatch>(c, sh, mu, al, buf, out);
}

// ======== phase: second-order-correction residual r <- a_soc r + r(trial) ========
// (both residual phases load every value before the stores that would precede it in program order -- their
// waits would include those stores, one in-order vmcnt queue -- so a block's results are stored after the
// next block's loads)
__device__ __noinline__ void phase_soc_resid(const Ctx& c, LShared& sh, double a_soc) {
    const WsView vw = ws_view(c);
    for (int k = (int)threadIdx.x; k <= c.N; k += T) {
        double cr[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) cr[i] = a_soc * vw.S(S_CR + i, k) + vw.S(S_CT + i, k);
        double dr[4], nx[4];
        auto blk = [&](int j, double* v) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] = a_soc * vw.B(B_DR + r, j, k) + vw.B(B_DT + r, j, k);
        };
        if (c.nbk > 0) blk(0, dr);
#pragma unroll
        for (int i = 0; i < 6; ++i) vw.S(S_CR + i, k) = cr[i];
        for (int j = 0; j < c.nbk; ++j) {
            if (j + 1 < c.nbk) blk(j + 1, nx);
#pragma unroll
            for (int r = 0; r < 4; ++r) { vw.B(B_DR + r, j, k) = dr[r]; dr[r] = nx[r]; }
        }
        if (k == c.N && c.plan())
#pragma unroll
            for (int i = 0; i < 6; ++i) sh.dfr[i] = a_soc * sh.dfr[i] + sh.dft[i];
    }
}

// ======== phase: residual rows of the Newton right-hand side at the iterate (zero: least squares) ========
__device__ __noinline__ void phase_resid(const Ctx& c, LShared& sh, bool zero) {
    const bool rs = sh.R != 0;
    for (int k = (int)threadIdx.x; k <= c.N; k += T) {
        double cr[6];
#pragma unroll
        for (int i = 0; i < 6; ++i)
            cr[i] = zero ? 0.0 : c.S(S_C + i, k) - (rs ? c.S(S_PR + i, k) - c.S(S_NR + i, k) : 0.0);
        double dr[4], nx[4];
        auto blk = [&](int j, double* v) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
                v[r] = zero ? 0.0 : c.B(B_D + r, j, k) - c.B(B_S + r, j, k) - (rs ? c.B(B_PR + r, j, k) - c.B(B_NR + r, j, k) : 0.0);
        };
        if (c.nbk > 0) blk(0, dr);
#pragma unroll
        for (int i = 0; i < 6; ++i) c.S(S_CR + i, k) = cr[i];
        for (int j = 0; j < c.nbk; ++j) {
            if (j + 1 < c.nbk) blk(j + 1, nx);
#pragma unroll
            for (int r = 0; r < 4; ++r) { c.B(B_DR + r, j, k) = dr[r]; dr[r] = nx[r]; }
        }
        if (k == c.N && c.plan())
#pragma unroll
            for (int i = 0; i < 6; ++i) sh.dfr[i] = zero ? 0.0 : sh.df[i] - sh.sf[i] - (rs ? sh.pf[i] - sh.nf[i] : 0.0);
    }
}

// inputs of one block's update (restoration pairs only when rs)
struct UpdIn {
    double w[8], dw[8], zw[8], s[4], ds[4], vu[4], vl[4], yd[4], yp[4];
    double pr[4], nr[4], zp[4], zn[4], dp[4], dn[4];
};
__device__ __forceinline__ void load_upd_in(const Ctx& c, bool rs, int buf, int j, int k, UpdIn& in) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        in.w[e] = c.B(B_W + e, j, k); in.dw[e] = c.B(B_DW + 8 * buf + e, j, k); in.zw[e] = c.B(B_ZW + e, j, k);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        in.s[r] = c.B(B_S + r, j, k); in.ds[r] = c.B(B_DS + 4 * buf + r, j, k);
        in.vu[r] = c.B(B_VU + r, j, k); in.vl[r] = c.hrl(r) ? (double)c.B(B_VL + r, j, k) : 0.0;
        in.yd[r] = c.B(B_YD + r, j, k); in.yp[r] = c.B(B_YP + 4 * buf + r, j, k);
        if (rs) {
            in.pr[r] = c.B(B_PR + r, j, k); in.nr[r] = c.B(B_NR + r, j, k);
            in.zp[r] = c.B(B_ZP + r, j, k); in.zn[r] = c.B(B_ZN + r, j, k);
            in.dp[r] = c.B(B_DP + 4 * buf + r, j, k); in.dn[r] = c.B(B_DN + 4 * buf + r, j, k);
        }
    }
}

// ---- the update pass's block part: block (j, k) of the flat block index (no reduction: any workgroup can run it) ----
template <bool RS_, bool SC1>
__device__ __forceinline__ void update_block(const Ctx& c, const WsView& vw, int j, int k, double mu, double alpha,
                                             double az, int buf) {
    constexpr bool rs = RS_;
    UpdIn cur;
    load_upd_in(c, rs, buf, j, k, cur);
    double wn[8], zwn[8], sn[4], vun[4], vln[4], ydn[4], prn[4], nrn[4], zpn[4], znn[4];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const double w = cur.w[e], dv = cur.dw[e], z = cur.zw[e];
        const double sl = w + RELAX;
        wn[e] = w + alpha * dv;
        double zn2 = z + az * (mu * inv(sl) - z - z * inv(sl) * dv);
        clamp_mult(zn2, wn[e] + RELAX, mu);
        zwn[e] = zn2;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const double sv = cur.s[r], dv = cur.ds[r];
        sn[r] = sv + alpha * dv;
        const double vu = cur.vu[r], slu = c.rU(r) - sv;
        double vu2 = vu + az * (mu * inv(slu) - vu + vu * inv(slu) * dv);
        clamp_mult(vu2, c.rU(r) - sn[r], mu);
        vun[r] = vu2;
        if (c.hrl(r)) {
            const double vl = cur.vl[r], sll = sv - c.rL(r);
            double vl2 = vl + az * (mu * inv(sll) - vl - vl * inv(sll) * dv);
            clamp_mult(vl2, sn[r] - c.rL(r), mu);
            vln[r] = vl2;
        }
        ydn[r] = cur.yd[r] + alpha * (cur.yp[r] - cur.yd[r]);
        if (rs) {
            const double p = cur.pr[r], n = cur.nr[r], zpv = cur.zp[r], znv = cur.zn[r];
            prn[r] = p + alpha * cur.dp[r];
            nrn[r] = n + alpha * cur.dn[r];
            double a1 = zpv + az * (mu * inv(p) - zpv - zpv * inv(p) * cur.dp[r]);
            double a2 = znv + az * (mu * inv(n) - znv - znv * inv(n) * cur.dn[r]);
            clamp_mult(a1, prn[r], mu);
            clamp_mult(a2, nrn[r], mu);
            zpn[r] = a1;
            znn[r] = a2;
        }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) { bst<SC1>(vw.B(B_W + e, j, k), wn[e]); bst<SC1>(vw.B(B_ZW + e, j, k), zwn[e]); }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        bst<SC1>(vw.B(B_VU + r, j, k), vun[r]);
        if (c.hrl(r)) bst<SC1>(vw.B(B_VL + r, j, k), vln[r]);
        bst<SC1>(vw.B(B_S + r, j, k), sn[r]);
        bst<SC1>(vw.B(B_YD + r, j, k), ydn[r]);
        if (rs) {
            bst<SC1>(vw.B(B_PR + r, j, k), prn[r]);
            bst<SC1>(vw.B(B_NR + r, j, k), nrn[r]);
            bst<SC1>(vw.B(B_ZP + r, j, k), zpn[r]);
            bst<SC1>(vw.B(B_ZN + r, j, k), znn[r]);
        }
    }
}

// ======== phase: accept the step (primal alpha, duals az, kappa_sigma safeguard) ========
// All loads of a stage are issued before its stores, and block j+1's loads before block j's stores: the
// workspace fields may alias as far as the compiler knows, so interleaved load / store pairs would each wait
// for the previous stores (one in-order vmcnt queue).
template <bool RS_>
__device__ __noinline__ void phase_update_t(const Ctx& c, LShared& sh, double mu, double alpha, double az, int buf) {
    const int N = c.N;
    constexpr bool rs = RS_;
    // the blocks over the flat block index (update_block), by this workgroup and any helpers (alpha and az travel as
    // the pass's second and third parameters); the stage fields below
    run_pass(c, sh, ChunkPass{mu, alpha, az, PASS_UPDATE, buf, 0, 0});
    for (int k = (int)threadIdx.x; k <= N; k += T) {
        double x[6], d[6], zl[6], zu[6], y[6], yp[6], pr[6], nr[6], zp[6], zn[6], dp[6], dn[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            x[i] = c.S(S_X + i, k); d[i] = c.S(S_DX + 6 * buf + i, k);
            zl[i] = c.hlx(i) ? (double)c.S(S_ZLX + i, k) : 0.0;
            zu[i] = c.hux(i) ? (double)c.S(S_ZUX + i, k) : 0.0;
            y[i] = c.S(S_YC + i, k); yp[i] = c.S(S_YCP + 6 * buf + i, k);
            if (rs) {
                pr[i] = c.S(S_PR + i, k); nr[i] = c.S(S_NR + i, k); zp[i] = c.S(S_ZP + i, k); zn[i] = c.S(S_ZN + i, k);
                dp[i] = c.S(S_DP + 6 * buf + i, k); dn[i] = c.S(S_DN + 6 * buf + i, k);
            }
        }
        double u[2] = {0.0, 0.0}, du[2] = {0.0, 0.0}, zlu[2] = {0.0, 0.0}, zuu[2] = {0.0, 0.0};
        if (k < N)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                u[i] = c.S(S_U + i, k); du[i] = c.S(S_DU + 2 * buf + i, k);
                if (c.hlu(i)) zlu[i] = c.S(S_ZLU + i, k);
                if (c.huu(i)) zuu[i] = c.S(S_ZUU + i, k);
            }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const double xv = x[i], dv = d[i];
            const double xn = xv + alpha * dv;
            if (c.hlx(i)) {
                const double sl = xv - c.xl[i], z = zl[i];
                double zn2 = z + az * (mu * inv(sl) - z - z * inv(sl) * dv);
                clamp_mult(zn2, xn - c.xl[i], mu);
                c.S(S_ZLX + i, k) = zn2;
            }
            if (c.hux(i)) {
                const double sl = c.xu[i] - xv, z = zu[i];
                double zn2 = z + az * (mu * inv(sl) - z + z * inv(sl) * dv);
                clamp_mult(zn2, c.xu[i] - xn, mu);
                c.S(S_ZUX + i, k) = zn2;
            }
            c.S(S_X + i, k) = xn;
            c.S(S_YC + i, k) = y[i] + alpha * (yp[i] - y[i]);
            if (rs) {
                const double p = pr[i], n = nr[i], zpv = zp[i], znv = zn[i];
                const double pn = p + alpha * dp[i], nn = n + alpha * dn[i];
                double zpn = zpv + az * (mu * inv(p) - zpv - zpv * inv(p) * dp[i]), znn = znv + az * (mu * inv(n) - znv - znv * inv(n) * dn[i]);
                clamp_mult(zpn, pn, mu);
                clamp_mult(znn, nn, mu);
                c.S(S_PR + i, k) = pn;
                c.S(S_NR + i, k) = nn;
                c.S(S_ZP + i, k) = zpn;
                c.S(S_ZN + i, k) = znn;
            }
        }
        if (k < N)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const double uv = u[i], dv = du[i];
                const double un = uv + alpha * dv;
                if (c.hlu(i)) {
                    const double sl = uv - c.ul[i], z = zlu[i];
                    double zn2 = z + az * (mu * inv(sl) - z - z * inv(sl) * dv);
                    clamp_mult(zn2, un - c.ul[i], mu);
                    c.S(S_ZLU + i, k) = zn2;
                }
                if (c.huu(i)) {
                    const double sl = c.uu[i] - uv, z = zuu[i];
                    double zn2 = z + az * (mu * inv(sl) - z + z * inv(sl) * dv);
                    clamp_mult(zn2, c.uu[i] - un, mu);
                    c.S(S_ZUU + i, k) = zn2;
                }
                c.S(S_U + i, k) = un;
            }
        if (k == N && c.plan())
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double s = sh.sf[i], d = sh.dsf[buf][i], sn = s + alpha * d;
                const double sl = s - c.fL, su = c.fU - s;
                double vl = sh.vLf[i] + az * (mu * inv(sl) - sh.vLf[i] - sh.vLf[i] * inv(sl) * d);
                double vu = sh.vUf[i] + az * (mu * inv(su) - sh.vUf[i] + sh.vUf[i] * inv(su) * d);
                clamp_mult(vl, sn - c.fL, mu);
                clamp_mult(vu, c.fU - sn, mu);
                sh.vLf[i] = vl;
                sh.vUf[i] = vu;
                sh.sf[i] = sn;
                sh.ydf[i] += alpha * (sh.ydpf[buf][i] - sh.ydf[i]);
                if (rs) {
                    const double p = sh.pf[i], n = sh.nf[i], zp = sh.zpf[i], zn = sh.znf[i];
                    const double dp = sh.dpf[buf][i], dn = sh.dnf[buf][i];
                    const double pn = p + alpha * dp, nn = n + alpha * dn;
                    double zpn = zp + az * (mu * inv(p) - zp - zp * inv(p) * dp), znn = zn + az * (mu * inv(n) - zn - zn * inv(n) * dn);
                    clamp_mult(zpn, pn, mu);
                    clamp_mult(znn, nn, mu);
                    sh.pf[i] = pn;
                    sh.nf[i] = nn;
                    sh.zpf[i] = zpn;
                    sh.znf[i] = znn;
                }
            }
    }
}

// one instantiation per problem (original / restoration phase): the original problem's skips every restoration
// branch and its loads (bitwise the same results, profiles/r03/ab_one/)
__device__ __forceinline__ void phase_update(const Ctx& c, LShared& sh, double mu, double alpha, double az, int buf) {
    sh.R ? phase_update_t<true>(c, sh, mu, alpha, az, buf) : phase_update_t<false>(c, sh, mu, alpha, az, buf);
}


// filters: [0] original problem, [1] restoration problem
__device__ __forceinline__ bool in_filter(const LShared& sh, int f, double th, double ph) {
    for (int i = 0; i < sh.nfl[f]; ++i)
        if (th >= sh.fth[f][i] && ph >= sh.fph[f][i]) return true;
    return false;
}
__device__ __forceinline__ void add_filter(LShared& sh, int f, double th, double ph) {  // thread 0 only
    int j = 0;
    for (int i = 0; i < sh.nfl[f]; ++i)
        if (!(sh.fth[f][i] >= th && sh.fph[f][i] >= ph)) { sh.fth[f][j] = sh.fth[f][i]; sh.fph[f][j] = sh.fph[f][i]; ++j; }
    if (j == kObcaMaxFilter) {
        for (int i = 0; i + 1 < kObcaMaxFilter; ++i) { sh.fth[f][i] = sh.fth[f][i + 1]; sh.fph[f][i] = sh.fph[f][i + 1]; }
        --j;
    }
    sh.fth[f][j] = th;
    sh.fph[f][j] = ph;
    sh.nfl[f] = j + 1;
}

// ======== phase: linearisation at the iterate + optimality-error ingredients of the current NLP ========
// out: [0] dual inf (max) [1] primal inf (max) [2] complementarity (max) [3] sum |y| + sum z [4] sum z
//      [5] theta (l1 of the residual rows) [6] objective [7] sum log slacks [8] sum |dual residuals|
//      [9] original theta [10] original cost [11] original sum log slacks [12] original primal inf (max)
//      (restoration: the original problem's rows without p, n)
// |z s - mu| over every bound and elastic pair of stage k (its blocks and, at k = N in plan mode, the final rows):
// max into cm[0], sum into cm[1].  (Evaluated inside phase_lin as well it measured slower than this pass of its own:
// profiles/r03/ab_cfold/.)
__device__ __forceinline__ void compl_stage(const Ctx& c, const LShared& sh, int k, double mu, bool rs, double (&cm)[2]) {
    const int N = c.N;
    auto acc = [&](double v) { cm[0] = fmax(cm[0], v); cm[1] += v; };
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const double xv = c.S(S_X + i, k);
        if (c.hlx(i)) acc(fabs(c.S(S_ZLX + i, k) * (xv - c.xl[i]) - mu));
        if (c.hux(i)) acc(fabs(c.S(S_ZUX + i, k) * (c.xu[i] - xv) - mu));
        if (rs) {
            acc(fabs(c.S(S_ZP + i, k) * c.S(S_PR + i, k) - mu));
            acc(fabs(c.S(S_ZN + i, k) * c.S(S_NR + i, k) - mu));
        }
    }
    if (k < N)
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const double uv = c.S(S_U + i, k);
            if (c.hlu(i)) acc(fabs(c.S(S_ZLU + i, k) * (uv - c.ul[i]) - mu));
            if (c.huu(i)) acc(fabs(c.S(S_ZUU + i, k) * (c.uu[i] - uv) - mu));
        }
    for (int j = 0; j < c.nbk; ++j) {
#pragma unroll
        for (int e = 0; e < 8; ++e) acc(fabs(c.B(B_ZW + e, j, k) * (c.B(B_W + e, j, k) + RELAX) - mu));
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const double s = c.B(B_S + r, j, k);
            acc(fabs(c.B(B_VU + r, j, k) * (c.rU(r) - s) - mu));
            if (c.hrl(r)) acc(fabs(c.B(B_VL + r, j, k) * (s - c.rL(r)) - mu));
            if (rs) {
                acc(fabs(c.B(B_ZP + r, j, k) * c.B(B_PR + r, j, k) - mu));
                acc(fabs(c.B(B_ZN + r, j, k) * c.B(B_NR + r, j, k) - mu));
            }
        }
    }
    if (k == N && c.plan())
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            acc(fabs(sh.vLf[i] * (sh.sf[i] - c.fL) - mu));
            acc(fabs(sh.vUf[i] * (c.fU - sh.sf[i]) - mu));
            if (rs) {
                acc(fabs(sh.zpf[i] * sh.pf[i] - mu));
                acc(fabs(sh.znf[i] * sh.nf[i] - mu));
            }
        }
}

template <bool RS_>
__device__ __noinline__ void phase_lin_t(const Ctx& c, LShared& sh, double (&red_out)[13]) {
    LArgs& a = *c.a;
    const int N = c.N;
    const bool plan = c.plan();
    constexpr bool rs = RS_;
    const double zeta = sh.zeta;
    // the sums accumulate in registers (the caller's array is memory that every workspace store may alias: kept there,
    // each update was a flat load and store behind the pass's workspace stores)
    double red[13];
#pragma unroll
    for (int i = 0; i < 13; ++i) red[i] = 0.0;

    const double* xinit = a.x0 + 6 * (size_t)c.b;
    for (int k = (int)threadIdx.x; k <= N; k += T) {
        double x[6], u[2] = {0.0, 0.0}, gl[6];
        // this stage's outputs stay in registers until every load of the stage has been issued (a store ahead
        // of a load in the in-order vmcnt queue makes the load's wait include it); block j's row values are
        // stored after block j+1's loads
        double gxs[6], gus[2] = {0.0, 0.0}, dj[9], wd[7];
        double objR = 0.0;  // restoration objective of this stage
        load_x(c, k, x);
        if (k < N) { u[0] = c.S(S_U, k); u[1] = c.S(S_U + 1, k); }
        // the stage cost before any of the pass's stores (its target loads would wait for them)
        const double cost = stage_cost(c, k, x, u);
        if (rs) {
            double prox = 0.0;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double dr = c.S(S_DRX + i, k), e = x[i] - c.S(S_XR + i, k);
                gl[i] = zeta * dr * e;
                gxs[i] = gl[i];
                prox += dr * e * e;
            }
            if (k < N)
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const double dr = c.S(S_DRU + i, k), e = u[i] - c.S(S_UR + i, k);
                    gus[i] = zeta * dr * e;
                    prox += dr * e * e;
                }
            objR += 0.5 * zeta * prox;
        } else {
            const double* tg = plan ? c.tgt_x : c.tgt_x + 6 * k;
            const double sc = (k == N && plan) ? a.tfac : 1.0;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                double g = 0.0;
#pragma unroll
                for (int j2 = 0; j2 < 6; ++j2) g += 0.5 * (a.Q[i * 6 + j2] + a.Q[j2 * 6 + i]) * (x[j2] - tg[j2]);
                gl[i] = 2.0 * sc * g;
                gxs[i] = gl[i];
            }
            if (k < N) {
                const double r0 = u[0] - (plan ? 0.0 : c.tgt_u[2 * k]), r1 = u[1] - (plan ? 0.0 : c.tgt_u[2 * k + 1]);
                const double R01 = 0.5 * (a.R[1] + a.R[2]);
                gus[0] = 2.0 * (a.R[0] * r0 + R01 * r1);
                gus[1] = 2.0 * (R01 * r0 + a.R[3] * r1);
            }
        }
        double ck[6];
        if (k == 0) {
#pragma unroll
            for (int i = 0; i < 6; ++i) ck[i] = x[i] - xinit[i];
        } else {
            double xp[6], up[2] = {c.S(S_U, k - 1), c.S(S_U + 1, k - 1)}, fo[6];
            load_x(c, k - 1, xp);
            model_f(a, xp, up, fo);
#pragma unroll
            for (int i = 0; i < 6; ++i) ck[i] = x[i] - (xp[i] + a.dt * fo[i]);
        }
        LogSum lsum, lorig;
        double crs[6];  // the Newton right-hand side's dynamics rows (phase_resid's S_CR), stored with the stage
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            double res = ck[i];
            if (rs) {
                const double p = c.S(S_PR + i, k), n = c.S(S_NR + i, k), zp = c.S(S_ZP + i, k), zn = c.S(S_ZN + i, k);
                const double y = c.S(S_YC + i, k);
                res -= p - n;
                const double t1 = RHO - y - zp, t2 = RHO + y - zn;
                red[0] = fmax(red[0], fmax(fabs(t1), fabs(t2)));
                red[8] += fabs(t1) + fabs(t2);
                red[2] = fmax(red[2], fmax(fabs(p * zp), fabs(n * zn)));
                red[3] += zp + zn;
                red[4] += zp + zn;
                lsum.add(p);
                lsum.add(n);
                objR += RHO * (p + n);
            }
            red[1] = fmax(red[1], fabs(res));
            red[5] += fabs(res);
            red[9] += fabs(ck[i]);
            red[12] = fmax(red[12], fabs(ck[i]));
            crs[i] = res;
        }
        double yk[6], yn[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 6; ++i) yk[i] = c.S(S_YC + i, k);
        if (k < N) {
#pragma unroll
            for (int i = 0; i < 6; ++i) yn[i] = c.S(S_YC + i, k + 1);
            model_lin(a, x, yn, dj, wd);
#pragma unroll
            for (int i = 0; i < 6; ++i) gl[i] += yk[i] - yn[i];
            gl[2] -= dj[0] * yn[0] + dj[2] * yn[1];
            gl[3] -= dj[6] * yn[3];
            gl[4] -= dj[4] * yn[2] + dj[7] * yn[3];
            gl[5] -= dj[1] * yn[0] + dj[3] * yn[1] + dj[5] * yn[2] + dj[8] * yn[3];
        } else {
#pragma unroll
            for (int i = 0; i < 6; ++i) gl[i] += yk[i];
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) red[3] += fabs(yk[i]);
        const Trig tr = stage_trig(x);
        double pdv[4] = {0, 0, 0, 0}, pdr[4] = {0, 0, 0, 0};  // the previous block's row values and residual rows
        int pj = -1;
        for (int j = 0; j < c.nbk; ++j) {
            double w[8], y[4], zw[8], drw[8], wrv[8], sv[4], vlv[4], vuv[4], prv[4], nrv[4], zpv[4], znv[4];
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                w[e] = c.B(B_W + e, j, k); zw[e] = c.B(B_ZW + e, j, k);
                if (rs) { drw[e] = c.B(B_DRW + e, j, k); wrv[e] = c.B(B_WR + e, j, k); }
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                y[r] = c.B(B_YD + r, j, k);
                sv[r] = c.B(B_S + r, j, k); vlv[r] = c.B(B_VL + r, j, k); vuv[r] = c.B(B_VU + r, j, k);
                if (rs) {
                    prv[r] = c.B(B_PR + r, j, k); nrv[r] = c.B(B_NR + r, j, k);
                    zpv[r] = c.B(B_ZP + r, j, k); znv[r] = c.B(B_ZN + r, j, k);
                }
            }
            if (pj >= 0)
#pragma unroll
                for (int r = 0; r < 4; ++r) { c.B(B_D + r, pj, k) = pdv[r]; c.B(B_DR + r, pj, k) = pdr[r]; }
            Blk bk;
            bk.m = c.slab + threadIdx.x;
            blk_lin(a, x, tr, j, w, y, bk);
#pragma unroll
            for (int r = 0; r < 4; ++r) pdv[r] = bk.d[r];
            pj = j;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                double s = 0.0;
#pragma unroll
                for (int r = 0; r < 3; ++r) s += jx(bk, r, q) * y[r];
                gl[q] += s;
            }
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                double t = -zw[e];
                if (rs) {
                    const double dr = drw[e], ew = w[e] - wrv[e];
                    t += zeta * dr * ew;
                    objR += 0.5 * zeta * dr * ew * ew;
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) t += (e < 4 ? jwm(bk, r, e) : jwl(bk, r, e - 4)) * y[r];
                red[0] = fmax(red[0], fabs(t));
                red[8] += fabs(t);
                const double sl = w[e] + RELAX;
                red[2] = fmax(red[2], fabs(zw[e] * sl));
                red[3] += zw[e];
                red[4] += zw[e];
                lsum.add(sl);
                lorig.add(sl);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double s = sv[r], vl = vlv[r], vu = vuv[r];
                const double td = -y[r] - vl + vu;
                red[0] = fmax(red[0], fabs(td));
                red[8] += fabs(td);
                double res = bk.d[r] - s;
                red[9] += fabs(res);
                red[12] = fmax(red[12], fabs(res));
                if (rs) {
                    const double p = prv[r], n = nrv[r], zp = zpv[r], zn = znv[r];
                    res -= p - n;
                    const double t1 = RHO - y[r] - zp, t2 = RHO + y[r] - zn;
                    red[0] = fmax(red[0], fmax(fabs(t1), fabs(t2)));
                    red[8] += fabs(t1) + fabs(t2);
                    red[2] = fmax(red[2], fmax(fabs(p * zp), fabs(n * zn)));
                    red[3] += zp + zn;
                    red[4] += zp + zn;
                    lsum.add(p);
                    lsum.add(n);
                    objR += RHO * (p + n);
                }
                red[1] = fmax(red[1], fabs(res));
                red[5] += fabs(res);
                pdr[r] = res;
                red[3] += fabs(y[r]) + vu;
                red[4] += vu;
                red[2] = fmax(red[2], fabs(vu * (c.rU(r) - s)));
                lsum.add(c.rU(r) - s);
                lorig.add(c.rU(r) - s);
                if (c.hrl(r)) {
                    red[2] = fmax(red[2], fabs(vl * (s - c.rL(r))));
                    red[3] += vl;
                    red[4] += vl;
                    lsum.add(s - c.rL(r));
                    lorig.add(s - c.rL(r));
                }
            }
        }
        if (k == N && plan)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                gl[i] += sh.ydf[i];
                const double dfi = x[i] - c.tgt_x[i];
                sh.df[i] = dfi;
                const double td = -sh.ydf[i] - sh.vLf[i] + sh.vUf[i];
                red[0] = fmax(red[0], fabs(td));
                red[8] += fabs(td);
                double res = dfi - sh.sf[i];
                red[9] += fabs(res);
                red[12] = fmax(red[12], fabs(res));
                if (rs) {
                    const double p = sh.pf[i], n = sh.nf[i], zp = sh.zpf[i], zn = sh.znf[i];
                    res -= p - n;
                    const double t1 = RHO - sh.ydf[i] - zp, t2 = RHO + sh.ydf[i] - zn;
                    red[0] = fmax(red[0], fmax(fabs(t1), fabs(t2)));
                    red[8] += fabs(t1) + fabs(t2);
                    red[2] = fmax(red[2], fmax(fabs(p * zp), fabs(n * zn)));
                    red[3] += zp + zn;
                    red[4] += zp + zn;
                    lsum.add(p);
                    lsum.add(n);
                    objR += RHO * (p + n);
                }
                red[1] = fmax(red[1], fabs(res));
                red[5] += fabs(res);
                sh.dfr[i] = res;
                const double sl = sh.sf[i] - c.fL, su = c.fU - sh.sf[i];
                red[2] = fmax(red[2], fmax(fabs(sh.vLf[i] * sl), fabs(sh.vUf[i] * su)));
                red[3] += fabs(sh.ydf[i]) + sh.vLf[i] + sh.vUf[i];
                red[4] += sh.vLf[i] + sh.vUf[i];
                lsum.add(sl);
                lsum.add(su);
                lorig.add(sl);
                lorig.add(su);
            }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const double zl = c.S(S_ZLX + i, k), zu = c.S(S_ZUX + i, k);
            gl[i] += -zl + zu;
            red[0] = fmax(red[0], fabs(gl[i]));
            red[8] += fabs(gl[i]);
            if (c.hlx(i)) { const double sl = x[i] - c.xl[i]; red[2] = fmax(red[2], fabs(zl * sl)); red[3] += zl; red[4] += zl; lsum.add(sl); lorig.add(sl); }
            if (c.hux(i)) { const double sl = c.xu[i] - x[i]; red[2] = fmax(red[2], fabs(zu * sl)); red[3] += zu; red[4] += zu; lsum.add(sl); lorig.add(sl); }
        }
        if (k < N)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const double zl = c.S(S_ZLU + i, k), zu = c.S(S_ZUU + i, k);
                const double t = gus[i] - a.dt * yn[i == 0 ? 5 : 4] - zl + zu;
                red[0] = fmax(red[0], fabs(t));
                red[8] += fabs(t);
                if (c.hlu(i)) { const double sl = u[i] - c.ul[i]; red[2] = fmax(red[2], fabs(zl * sl)); red[3] += zl; red[4] += zl; lsum.add(sl); lorig.add(sl); }
                if (c.huu(i)) { const double sl = c.uu[i] - u[i]; red[2] = fmax(red[2], fabs(zu * sl)); red[3] += zu; red[4] += zu; lsum.add(sl); lorig.add(sl); }
            }
        if (pj >= 0)
#pragma unroll
            for (int r = 0; r < 4; ++r) { c.B(B_D + r, pj, k) = pdv[r]; c.B(B_DR + r, pj, k) = pdr[r]; }
#pragma unroll
        for (int i = 0; i < 6; ++i) { c.S(S_GX + i, k) = gxs[i]; c.S(S_C + i, k) = ck[i]; c.S(S_CR + i, k) = crs[i]; }
        if (k < N) {
#pragma unroll
            for (int i = 0; i < 2; ++i) c.S(S_GU + i, k) = gus[i];
#pragma unroll
            for (int i = 0; i < 9; ++i) c.S(S_AJ + i, k) = dj[i];
#pragma unroll
            for (int i = 0; i < 7; ++i) c.S(S_WD + i, k) = wd[i];
        }
        red[6] += rs ? objR : cost;
        red[7] += lsum.value();
        red[10] += cost;
        red[11] += lorig.value();
        if (!isfinite(red[0]) || !isfinite(red[1])) red[0] = INFINITY;
    }
    const int ops[13] = {R_MAX, R_MAX, R_MAX, R_SUM, R_SUM, R_SUM, R_SUM, R_SUM, R_SUM, R_SUM, R_SUM, R_SUM, R_MAX};
    wg_reduce(sh, red, ops);
#pragma unroll
    for (int i = 0; i < 13; ++i) red_out[i] = red[i];
}

// one instantiation per problem (original / restoration phase): the original problem's skips every restoration
// branch and its loads (bitwise the same results, profiles/r03/ab_one/)
__device__ __forceinline__ void phase_lin(const Ctx& c, LShared& sh, double (&red)[13]) {
    sh.R ? phase_lin_t<true>(c, sh, red) : phase_lin_t<false>(c, sh, red);
}


// ======== phase: complementarity vs mu: max and sum of |z s - mu| (elastic pairs included) ========
__device__ __noinline__ double2 phase_compl(const Ctx& c, LShared& sh, double mu) {
    const int N = c.N;
    const bool rs = sh.R != 0;
    double cm[2] = {0.0, 0.0};
    for (int k = (int)threadIdx.x; k <= N; k += T) compl_stage(c, sh, k, mu, rs, cm);
    const int ops[2] = {R_MAX, R_SUM};
    wg_reduce(sh, cm, ops);
    return make_double2(cm[0], cm[1]);
}

// Newton solve for the current residual arrays (S_CR / B_DR / sh.dfr) with the given dw into buffer buf.
// Returns false when the Riccati/blocks are not positive definite.
// One factorisation + condensed solve with the perturbations (dw, dc) into step buffer buf: F_OK, or the outcome of the
// failed factorisation (F_MANY / F_ZERO / F_FEW) for the perturbation handler.
// the Riccati factors of the LDS record (region B) to the HBM workspace (S_P, S_K, S_GI) for the refinement's correction
// solves: threads 64..255, field-major (consecutive k on consecutive lanes: coalesced stores), while wave 0 runs the
// forward sweep on the same (read-only) record
__device__ __noinline__ void keep_factors(const Ctx& c, const LSrc src) {
    const WsView vw = ws_view(c);
    const int NP = c.NP, N = c.N, nt = T - 64;
    constexpr int NF = 21 + 12 + 3;
    for (int idx = (int)threadIdx.x - 64; idx < NF * NP; idx += nt) {
        const int f = idx / NP, k = idx - f * NP;
        if (f < 21) vw.S(S_P + f, k) = src.P(f, k);
        else if (k < N) {
            if (f < 33) vw.S(S_K + f - 21, k) = src.K(f - 21, k);
            else vw.S(S_GI + f - 33, k) = src.GI(f - 33, k);
        }
    }
}

__device__ __noinline__ int newton_solve(const Ctx& c, LShared& sh, double mu, double dw, double dc, int buf) {
    const bool on = c.a->stamps != nullptr;
    stamp(sh, on, OPH_UPD);
    __syncthreads();
    if (threadIdx.x == 0) sh.dc = dc;
    count(sh, on, OCNT_FACTOR);
    __syncthreads();
    const int f = phase_factor(c, sh, mu, dw);
    stamp(sh, on, OPH_FACTOR);
    if (f != F_OK) return f;
    if (sh.R || dc > 0.0) {  // soft dynamics rows (restoration phase, delta_c)
        if (c.lds) {
            stage_soft_inputs(c, c.lds);
            __syncthreads();
            if (threadIdx.x < 64) riccati_soft(c, sh, SoftA{(const lds_double*)c.lds});
        } else if (threadIdx.x < 64) {
            riccati_soft(c, sh, SoftG{c});
        }
        __syncthreads();
        stamp(sh, on, OPH_RIC_SOFT);
        if (sh.flag) return sh.flag;
        if (c.lds) {
            stage_soft_forward(c, c.lds);
            __syncthreads();
            if (threadIdx.x < 64) forward_soft(c, SoftF{(const lds_double*)c.lds}, buf);
        } else if (threadIdx.x < 64) {
            forward_soft(c, SoftFG{c}, buf);
        }
        __syncthreads();
        stamp(sh, on, OPH_FWD_SOFT);
        return F_OK;
    } else if (c.lds) {
        stage_inputs(c, c.lds);
        __syncthreads();
        stamp(sh, on, OPH_COMPL);  // (diagnostic: staging cost booked under 'compl')
        const LSrc src{(const lds_double*)c.lds, (lds_double*)(c.lds + (size_t)LA * c.NP)};
        if (threadIdx.x < 64) riccati(c, sh, src);
        __syncthreads();
        stamp(sh, on, OPH_RIC);
        if (sh.flag) return sh.flag;
        if (threadIdx.x < 64) forward(c, src, buf);
        else if (c.refine) keep_factors(c, src);
    } else {
        const GSrc src{c};
        if (threadIdx.x < 64) riccati(c, sh, src);
        __syncthreads();
        stamp(sh, on, OPH_RIC);
        if (sh.flag) return sh.flag;
        if (threadIdx.x < 64) forward(c, src, buf);
    }
    __syncthreads();
    stamp(sh, on, OPH_FWD);
    return F_OK;
}

// ================= IPOPT's iterative refinement (PDFullSpaceSolver; oracle/c/tt_obca.c:refined_solve) =================
// Every step solve is followed by at least one refinement step on the un-condensed primal-dual system: the residual
// r of every Newton row at the computed step (phase_nres), a correction solve K e = -r through the same
// factorisation (the block record, P, K, G^-1, Y), step += e; stop when max|r| <= 1e-10 (min(|sol|, 1e6) + |rhs|)
// after the first step, when r stops decreasing (residual_improvement_factor 1) or after 10 steps.

// ---- correction solve, backward: vector-only Riccati sweep over the stored factorisation (wave 0) ----
// Per stage k = N..1 (A = I + D, B = dt [e5 e4]):
//   s = p_k - P_k c_k,  p' = s - P_k Y_k s  (= p~_k - P~_k c_k of the soft sweep; Y = 0 outside the restoration phase),
//   g = r_{k-1} + B'p',  kf_{k-1} = -G^-1 g,  p_{k-1} = q_{k-1} + A'p' + K'g   (K'g = H' kf)
// P_k c_k and P_k Y_k do not depend on the recursion: all four waves stage them per stage (record LV) before the
// sweep, so the serial chain is one 6x6 product (restoration only) plus the sparse A' and K' products, carried
// redundantly by every lane; lanes 0..5 / lane 0 store p / kf for the forward sweep.
constexpr int LV = 74;  // W = P c 6 | PY 36 | QV 6 | RV 2 | GI 3 | K 12 | AJ 9
struct VecL {
    const lds_double* A;
    __device__ double W(int i, int k) const { return A[k * LV + i]; }
    __device__ double PY(int i, int j, int k) const { return A[k * LV + 6 + 6 * i + j]; }
    __device__ double QV(int i, int k) const { return A[k * LV + 42 + i]; }
    __device__ double RV(int i, int k) const { return A[k * LV + 48 + i]; }
    __device__ double GI(int i, int k) const { return A[k * LV + 50 + i]; }
    __device__ double K(int i, int k) const { return A[k * LV + 53 + i]; }
    __device__ double AJ(int i, int k) const { return A[k * LV + 65 + i]; }
};
// the same operands straight from the HBM workspace (horizons whose records do not fit the LDS budget)
struct VecG {
    const Ctx& c;
    __device__ double W(int i, int k) const {
        double t = 0.0;
#pragma unroll
        for (int l = 0; l < 6; ++l) t = fma((double)c.S(S_P + sy6(i, l), k), (double)c.S(S_CE + l, k), t);
        return t;
    }
    __device__ double PY(int i, int j, int k) const {
        double t = 0.0;
#pragma unroll
        for (int l = 0; l < 6; ++l) t = fma((double)c.S(S_P + sy6(i, l), k), (double)c.S(S_Y + sy6(l, j), k), t);
        return t;
    }
    __device__ double QV(int i, int k) const { return c.S(S_QV + i, k); }
    __device__ double RV(int i, int k) const { return c.S(S_RV + i, k); }
    __device__ double GI(int i, int k) const { return c.S(S_GI + i, k); }
    __device__ double K(int i, int k) const { return c.S(S_K + i, k); }
    __device__ double AJ(int i, int k) const { return c.S(S_AJ + i, k); }
};
template <bool SOFT>
__device__ __noinline__ void stage_vec_inputs_t(const Ctx& c, double* A) {
    constexpr bool soft = SOFT;
    for (int k = (int)threadIdx.x; k <= c.N; k += T) {
        lds_double* r = (lds_double*)A + (size_t)k * LV;
        double P[21], e[6];
#pragma unroll
        for (int i = 0; i < 21; ++i) P[i] = c.S(S_P + i, k);
#pragma unroll
        for (int i = 0; i < 6; ++i) e[i] = c.S(S_CE + i, k);
        double q[6], rv[2] = {0.0, 0.0}, gi[3] = {0.0, 0.0, 0.0}, kk[12], aj[9];
#pragma unroll
        for (int i = 0; i < 6; ++i) q[i] = c.S(S_QV + i, k);
        // (stage N's K, AJ, RV, GI rows are never read by the sweep -- it reads them at k - 1 -- so every stage loads them:
        // no exec-masked branch per field)
#pragma unroll
        for (int i = 0; i < 12; ++i) kk[i] = c.S(S_K + i, k);
#pragma unroll
        for (int i = 0; i < 9; ++i) aj[i] = c.S(S_AJ + i, k);
        rv[0] = c.S(S_RV, k); rv[1] = c.S(S_RV + 1, k);
        gi[0] = c.S(S_GI, k); gi[1] = c.S(S_GI + 1, k); gi[2] = c.S(S_GI + 2, k);
        double Y[21];
#pragma unroll
        for (int i = 0; i < 21; ++i) Y[i] = soft ? (double)c.S(S_Y + i, k) : 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            double t = 0.0;
#pragma unroll
            for (int l = 0; l < 6; ++l) t = fma(P[sy6(i, l)], e[l], t);
            r[i] = t;
        }
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j = 0; j < 6; ++j) {
                double t = 0.0;
                if (soft)
#pragma unroll
                    for (int l = 0; l < 6; ++l) t = fma(P[sy6(i, l)], Y[sy6(l, j)], t);
                r[6 + 6 * i + j] = t;
            }
#pragma unroll
        for (int i = 0; i < 6; ++i) r[42 + i] = q[i];
        r[48] = rv[0]; r[49] = rv[1];
        r[50] = gi[0]; r[51] = gi[1]; r[52] = gi[2];
#pragma unroll
        for (int i = 0; i < 12; ++i) r[53 + i] = kk[i];
#pragma unroll
        for (int i = 0; i < 9; ++i) r[65 + i] = aj[i];
    }
}
__device__ __forceinline__ void stage_vec_inputs(const Ctx& c, double* A, bool soft) {
    soft ? stage_vec_inputs_t<true>(c, A) : stage_vec_inputs_t<false>(c, A);
}
// operands of one stage of the vector sweep (lane q's row), loaded one stage ahead of its use
struct VecOps {
    double w, py[6], rv0, rv1, gi0, gi1, gi2, qv, k0, k1, dj[9];
};
template <class Src>
__device__ __forceinline__ void vec_ops(const Src& src, int k, int q, bool soft, VecOps& o) {
    const int km = k - 1;
    o.w = src.W(q, k);
#pragma unroll
    for (int l = 0; l < 6; ++l) o.py[l] = soft ? src.PY(q, l, k) : 0.0;
    o.rv0 = src.RV(0, km);
    o.rv1 = src.RV(1, km);
    o.gi0 = src.GI(0, km);
    o.gi1 = src.GI(1, km);
    o.gi2 = src.GI(2, km);
    o.qv = src.QV(q, km);
    o.k0 = src.K(q, km);
    o.k1 = src.K(6 + q, km);
#pragma unroll
    for (int e = 0; e < 9; ++e) o.dj[e] = src.AJ(e, km);
}
// lanes 0..5 hold p[q] (q = lane); the serial chain per stage is sv -> (soft: 6 broadcasts, 6 FMAs) -> 6 broadcasts of
// p' -> np, with only the lane's own row of PY, K, QV and W read from LDS, one stage ahead (ping-pong operand sets)
template <class Src, bool SOFT>
__device__ __noinline__ void riccati_vec_t(const Ctx& c, const Src src) {
    constexpr bool soft = SOFT;  // one instantiation per row type: no exec-masked branches on the flag in the chain
    const WsView vw = ws_view(c);
    const int lane = threadIdx.x, N = c.N;
    const double dt = c.dt;
    const int q = lane < 6 ? lane : 0;
    double pq = src.QV(q, N);
    if (lane < 6) vw.S(S_PV + q, N) = pq;
    auto stage = [&](int k, const VecOps& o) __attribute__((always_inline)) {
        const int km = k - 1;
        const double sv = pq - o.w;
        double pp = sv;
        if (soft) {
            double t = sv;
            t = fma(-o.py[0], rowbc<0>(sv), t);
            t = fma(-o.py[1], rowbc<1>(sv), t);
            t = fma(-o.py[2], rowbc<2>(sv), t);
            t = fma(-o.py[3], rowbc<3>(sv), t);
            t = fma(-o.py[4], rowbc<4>(sv), t);
            t = fma(-o.py[5], rowbc<5>(sv), t);
            pp = t;
        }
        const double pp0 = rowbc<0>(pp), pp1 = rowbc<1>(pp), pp2 = rowbc<2>(pp), pp3 = rowbc<3>(pp);
        const double pp4 = rowbc<4>(pp), pp5 = rowbc<5>(pp);
        const double g0 = fma(dt, pp5, o.rv0), g1 = fma(dt, pp4, o.rv1);
        const double kf0 = -fma(o.gi0, g0, o.gi1 * g1), kf1 = -fma(o.gi1, g0, o.gi2 * g1);
        double np = o.qv + pp + fma(o.k0, g0, o.k1 * g1);
        // D' p' (D: 0:(0,2) 1:(0,5) 2:(1,2) 3:(1,5) 4:(2,4) 5:(2,5) 6:(3,3) 7:(3,4) 8:(3,5)): the lane's own row
        // (row 3 as the contracted np[3] += dj[6] * pp[3] of the redundant version: bitwise the same)
        const double* dj = o.dj;
        const double t2 = fma(dj[0], pp0, dj[2] * pp1), t4 = fma(dj[4], pp2, dj[7] * pp3);
        const double t5 = fma(dj[1], pp0, fma(dj[3], pp1, fma(dj[5], pp2, dj[8] * pp3)));
        np = sel6(q, np, np, np + t2, fma(dj[6], pp3, np), np + t4, np + t5);
        if (lane < 6) vw.S(S_PV + q, km) = np;
        if (lane == 0) { vw.S(S_KF, km) = kf0; vw.S(S_KF + 1, km) = kf1; }
        pq = np;
    };
    VecOps oa, ob;
    int k = N;
    if (k >= 1) vec_ops(src, k, q, soft, oa);
    for (; k - 1 >= 1; k -= 2) {
        vec_ops(src, k - 1, q, soft, ob);
        stage(k, oa);
        if (k - 2 >= 1) vec_ops(src, k - 2, q, soft, oa);
        stage(k - 1, ob);
    }
    if (k >= 1) stage(k, oa);
}
template <class Src>
__device__ __forceinline__ void riccati_vec(const Ctx& c, const Src src, bool soft) {
    soft ? riccati_vec_t<Src, true>(c, src) : riccati_vec_t<Src, false>(c, src);
}

// ---- residuals of the un-condensed Newton rows at the step in buffer buf (+ the correction's right-hand side) ----
// (oracle/c/tt_obca.c:newton_resid, and solve_rhs in override mode)  Rows and their constants: the stationarity of
// x, u, the duals w, the slacks s, sf and the elastic pairs p, n (the barrier gradients), the linearised dynamics /
// OBCA / final rows (the row residuals S_CR / B_DR / dfr of the solve).  With prep, the right-hand side of the
// correction solve (phase_factor's rhs with the residuals as the constants): QV, RV, CE, the factor record's
// fw / zf_lam / t, and the constants the recovery needs (B_OS, B_OP / B_ON, S_OP / S_ON, osf / opf / onf).
// out: [0] max |residual| [1] max |constant| [2] max |dx, y+_c, dw| (the oracle's solution norm)
//      [3] alpha_primal [4] alpha_dual [5] grad phi' d [6] max relative step  (of the step in buf: the line search's)
// mode: NR_STEP the step in buf is complete; NR_MAIN the forward sweep's dx, du, y+_c are in buf and the blocks' and
// elastic pairs' parts are recovered here first from the factor record (phase_recover's work, fused: one pass over
// the blocks instead of two); NR_CORR a correction's dx is in buffer 2, the stage parts are already added into buf
// (phase_stage_add), and the blocks' correction is recovered here (with the constants prep left) and added.
enum { NR_STEP = 0, NR_MAIN = 1, NR_CORR = 2 };
// ---- the residual pass's block part: block (j, k) of the flat block index f = j (N + 1) + k ----
// Everything one OBCA block contributes to phase_nres, from the workspace alone (the stage's x, its step dx and the
// block's own fields): the block's step / correction (NR_MAIN, NR_CORR) and the next correction's right-hand side (prep)
// go to the block's fields; its contributions to the stage rows and to the pass's reductions go to its record B_CB --
// the x rows' adds (W_xx dx, W_x lam dw_lam + Jx' y+), the gradient adds of the correction's right-hand side, its part of
// grad phi' d as one term, and its maxima / minima.  The stage part (phase_nres) adds a stage's records in block order:
// the arithmetic of the pass with the block loop inside the stage loop.  No block reads another block's output, so any
// thread of any workgroup can run any block.
enum : int { CB_DM = 0, CB_RMAX = 1, CB_BMAX = 2, CB_SN = 3, CB_REL = 4, CB_AP = 5, CB_AZ = 6, CB_RX = 7, CB_Q4 = 13,
             CB_END = 17 };
static_assert(B_CB + CB_END == B_END, "contribution record");
template <bool SC1>
__device__ __forceinline__ void nres_block(const Ctx& c, const LShared& sh, const WsView& vw, int j, int k, double mu,
                                           double dw, double tau, int buf, bool prep, int mode) {
    LArgs& a = *c.a;
    const bool rs = sh.R != 0;
    const double zeta = sh.zeta, dc = sh.dc;
    double x[6], dx[6];
    load_x(c, k, x);
#pragma unroll
    for (int i = 0; i < 6; ++i) dx[i] = vw.S(S_DX + 6 * buf + i, k);
    const Trig tr = stage_trig(x);
    double rmax = 0.0, bmax = 0.0, snorm = 0.0, ap = 1.0, az = 1.0, rel = 0.0, Dmb = 0.0;
    double cb[CB_END] = {};
    auto R = [&](double v) { rmax = fmax(rmax, fabs(v)); return v; };
    auto Bc = [&](double v) { bmax = fmax(bmax, fabs(v)); return v; };
    auto dual = [&](double z, double dz) { if (dz < 0.0) az = fmin(az, -tau * z * inv(dz)); };
    BlkIn in;
    load_blk_in(c, rs, j, k, in);
    const double *w = in.w, *zw = in.zw, *sv = in.s, *vl = in.vl, *vu = in.vu, *dres = in.dr;
    double dwv[8], ds[4], ydp[4];
    Blk bk;
    bk.m = c.slab + threadIdx.x;
    // the elimination (block_refactor, which linearises too) where the pass recovers a step or prepares a
    // correction's right-hand side; the linearisation alone otherwise
    if (mode == NR_MAIN || mode == NR_CORR || prep) {
        double fw[8], zf[8], t4[4];
        if (mode == NR_MAIN) {
            block_refactor<true>(c, sh, in, j, x, tr, mu, dw, bk, fw, zf, t4);
        } else {
            block_refactor<false>(c, sh, in, j, x, tr, mu, dw, bk, fw, zf, t4);
            if (mode == NR_CORR) {  // the correction's right-hand side, as the previous prep pass left it
#pragma unroll
                for (int e = 0; e < 8; ++e) fw[e] = vw.B(B_FR + FR_FW + e, j, k);
#pragma unroll
                for (int e = 0; e < 4; ++e) { zf[4 + e] = vw.B(B_FR + FR_ZFL + e, j, k); t4[e] = vw.B(B_FR + FR_T + e, j, k); }
            }
        }
        if (mode != NR_STEP) {
            // ---- the block's part of the step (NR_MAIN) or of the correction (NR_CORR) ----
            double ypr[4], dwr[8], dxr[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) dxr[i] = mode == NR_MAIN ? dx[i] : (double)vw.S(S_DX + 12 + i, k);
            blk_recover(bk, fw, zf, t4, dxr, ypr, dwr);
            const bool add = mode == NR_CORR;
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                dwv[e] = add ? (double)vw.B(B_DW + 8 * buf + e, j, k) + dwr[e] : dwr[e];
                bst<SC1>(vw.B(B_DW + 8 * buf + e, j, k), dwv[e]);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const double gs = add ? (double)vw.B(B_OS + r, j, k) : grad_row(c, r, sv[r], mu);
                const double dsr = (ypr[r] - gs) / bk.D[r];
                ydp[r] = add ? (double)vw.B(B_YP + 4 * buf + r, j, k) + ypr[r] : ypr[r];
                ds[r] = add ? (double)vw.B(B_DS + 4 * buf + r, j, k) + dsr : dsr;
                bst<SC1>(vw.B(B_YP + 4 * buf + r, j, k), ydp[r]);
                bst<SC1>(vw.B(B_DS + 4 * buf + r, j, k), ds[r]);
                if (rs) {
                    const double p = in.pr[r], n = in.nr[r], zp = in.zp[r], zn = in.zn[r];
                    const double gp = add ? (double)vw.B(B_OP + r, j, k) : RHO - mu / p;
                    const double gn = add ? (double)vw.B(B_ON + r, j, k) : RHO - mu / n;
                    const double dpr = (ypr[r] - gp) / (zp / p + dw), dnr = (-ypr[r] - gn) / (zn / n + dw);
                    bst<SC1>(vw.B(B_DP + 4 * buf + r, j, k), add ? (double)vw.B(B_DP + 4 * buf + r, j, k) + dpr : dpr);
                    bst<SC1>(vw.B(B_DN + 4 * buf + r, j, k), add ? (double)vw.B(B_DN + 4 * buf + r, j, k) + dnr : dnr);
                }
            }
        }
    } else {
        blk_lin(a, x, tr, j, w, in.y, bk);
    }
    if (mode == NR_STEP) {
#pragma unroll
        for (int e = 0; e < 8; ++e) dwv[e] = vw.B(B_DW + 8 * buf + e, j, k);
#pragma unroll
        for (int r = 0; r < 4; ++r) { ds[r] = vw.B(B_DS + 4 * buf + r, j, k); ydp[r] = vw.B(B_YP + 4 * buf + r, j, k); }
    }
    // x rows: W_xx dx + W_x lam dw_lam + Jx' y+
    cb[CB_RX] = bk.hxx22 * dx[2] + bk.hxx23 * dx[3];
    cb[CB_RX + 1] = bk.hxx23 * dx[2] + bk.hxx33 * dx[3];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        double t = 0.0;
#pragma unroll
        for (int e = 0; e < 4; ++e) t += bk.H(q, e) * dwv[4 + e];
#pragma unroll
        for (int r = 0; r < 3; ++r) t += jx(bk, r, q) * ydp[r];
        cb[CB_RX + 2 + q] = t;
    }
    // w rows
    double rw[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
        const double sl = w[e] + RELAX, isl = inv(sl), d = dwv[e];
        double hw = 0.0, gw = -mu * isl;
        if (rs) {
            hw = zeta * in.drw[e];
            gw += hw * (w[e] - in.wr[e]);
        }
        double t = Bc(gw) + (zw[e] * isl + dw + hw) * d;
#pragma unroll
        for (int r = 0; r < 4; ++r) t += (e < 4 ? jwm(bk, r, e) : jwl(bk, r, e - 4)) * ydp[r];
        if (e >= 4) {
#pragma unroll
            for (int q = 0; q < 4; ++q) t += bk.H(q, e - 4) * dx[q];
#pragma unroll
            for (int b2 = 0; b2 < 4; ++b2) t += hll(bk, max(e - 4, b2), min(e - 4, b2)) * dwv[4 + b2];
        }
        rw[e] = R(t);
        Dmb += gw * d;
        rel = fmax(rel, fabs(d) * inv(1.0 + fabs(w[e])));
        snorm = fmax(snorm, fabs(d));
        ftb_lo(w[e], -RELAX, d, tau, ap);
        dual(zw[e], mu * isl - zw[e] - zw[e] * isl * d);
    }
    // slack, row and elastic-pair rows
    double rsl[4], rdv[4], rpv[4] = {0, 0, 0, 0}, rnv[4] = {0, 0, 0, 0}, Dpv[4] = {1, 1, 1, 1}, Dnv[4] = {1, 1, 1, 1};
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const double s = sv[r], d = ds[r];
        const double iu = inv(c.rU(r) - s), il = c.hrl(r) ? inv(s - c.rL(r)) : 0.0;
        const double gs = c.hrl(r) ? mu * iu - mu * il : mu * iu;
        const double sgr = c.hrl(r) ? vu[r] * iu + vl[r] * il : vu[r] * iu;
        rsl[r] = R(Bc(gs) + (sgr + dw) * d - ydp[r]);
        double t = Bc(dc > 0.0 ? fma(dc, in.y[r], dres[r]) : dres[r]) - d;
#pragma unroll
        for (int q = 0; q < 4; ++q) t += jx(bk, r, q) * dx[q];
#pragma unroll
        for (int e = 0; e < 4; ++e) t += jwm(bk, r, e) * dwv[e] + jwl(bk, r, e) * dwv[4 + e];
        if (rs) {
            const double p = in.pr[r], n = in.nr[r], zp = in.zp[r], zn = in.zn[r];
            const double dp = vw.B(B_DP + 4 * buf + r, j, k), dn = vw.B(B_DN + 4 * buf + r, j, k);
            t += -dp + dn;
            const double ip = inv(p), in_ = inv(n);
            Dpv[r] = zp * ip + dw;
            Dnv[r] = zn * in_ + dw;
            const double gp = RHO - mu * ip, gn = RHO - mu * in_;
            rpv[r] = R(Bc(gp) + Dpv[r] * dp - ydp[r]);
            rnv[r] = R(Bc(gn) + Dnv[r] * dn + ydp[r]);
            ftb_lo(p, 0.0, dp, tau, ap);
            ftb_lo(n, 0.0, dn, tau, ap);
            dual(zp, mu * ip - zp - zp * ip * dp);
            dual(zn, mu * in_ - zn - zn * in_ * dn);
            Dmb += gp * dp + gn * dn;
            rel = fmax(rel, fmax(fabs(dp) * inv(1.0 + fabs(p)), fabs(dn) * inv(1.0 + fabs(n))));
        }
        if (dc > 0.0) t -= dc * ydp[r];
        rdv[r] = R(t);
        Dmb += gs * d;
        rel = fmax(rel, fabs(d) * inv(1.0 + fabs(s)));
        ftb_hi(s, c.rU(r), d, tau, ap);
        dual(vu[r], mu * iu - vu[r] + vu[r] * iu * d);
        if (c.hrl(r)) {
            ftb_lo(s, c.rL(r), d, tau, ap);
            dual(vl[r], mu * il - vl[r] - vl[r] * il * d);
        }
    }
    if (prep) {  // bk holds the elimination (block_refactor above)
        double rdc[4], zf[8], t4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) rdc[r] = rdv[r] + rsl[r] / bk.D[r] + (rs ? rpv[r] / Dpv[r] - rnv[r] / Dnv[r] : 0.0);
        blk_rhs(bk, rw, rdc, zf, t4, cb + CB_Q4);
        auto stf = [&](int f, double v) { bst<SC1>(vw.B(B_FR + f, j, k), v); };
#pragma unroll
        for (int e = 0; e < 8; ++e) stf(FR_FW + e, rw[e]);
#pragma unroll
        for (int e = 0; e < 4; ++e) { stf(FR_ZFL + e, zf[4 + e]); stf(FR_T + e, t4[e]); }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            bst<SC1>(vw.B(B_OS + r, j, k), rsl[r]);
            if (rs) { bst<SC1>(vw.B(B_OP + r, j, k), rpv[r]); bst<SC1>(vw.B(B_ON + r, j, k), rnv[r]); }
        }
    }
    cb[CB_DM] = Dmb; cb[CB_RMAX] = rmax; cb[CB_BMAX] = bmax; cb[CB_SN] = snorm; cb[CB_REL] = rel; cb[CB_AP] = ap;
    cb[CB_AZ] = az;
#pragma unroll
    for (int i = 0; i < CB_END; ++i) bst<SC1>(vw.B(B_CB + i, j, k), cb[i]);
}

// chunks [c0, c1) of a block pass: thread t runs block f = ci T + t of the flat block index (one function per pass, so
// that neither block part's registers constrain the other's).  The helpers' write-through instances (SC1) are inlined
// into the helper path of the kernel entry, which saves no registers: as calls, every chunk paid the callee-saved
// register saves and restores of a ~270-register frame.
template <bool SC1>
__device__ __forceinline__ void nres_chunks_body(const Ctx& c, const LShared& sh, ChunkPass p, int c0, int c1) {
    const WsView vw = ws_view(c);
    const int nblk = c.nbk * c.NP, np = c.NP;
    for (int ci = c0; ci < c1; ++ci) {
        const int f = ci * T + (int)threadIdx.x;
        if (f >= nblk) break;
        const int j = f / np;
        nres_block<SC1>(c, sh, vw, j, f - j * np, p.mu, p.dw, p.tau, p.buf, p.prep != 0, p.mode);
    }
}
template <bool SC1>
__device__ __forceinline__ void factor_chunks_body(const Ctx& c, const LShared& sh, ChunkPass p, int c0, int c1) {
    const WsView vw = ws_view(c);
    const int nblk = c.nbk * c.NP, np = c.NP;
    for (int ci = c0; ci < c1; ++ci) {
        const int f = ci * T + (int)threadIdx.x;
        if (f >= nblk) break;
        const int j = f / np;
        factor_block<SC1>(c, sh, vw, j, f - j * np, p.mu, p.dw);
    }
}
template <bool RS_, bool SC1>
__device__ __forceinline__ void update_chunks_body(const Ctx& c, ChunkPass p, int c0, int c1) {
    const WsView vw = ws_view(c);
    const int nblk = c.nbk * c.NP, np = c.NP;
    for (int ci = c0; ci < c1; ++ci) {
        const int f = ci * T + (int)threadIdx.x;
        if (f >= nblk) break;
        const int j = f / np;
        update_block<RS_, SC1>(c, vw, j, f - j * np, p.mu, p.dw, p.tau, p.buf);
    }
}
__device__ __noinline__ void nres_chunks(const Ctx& c, const LShared& sh, ChunkPass p, int c0, int c1) {
    nres_chunks_body<false>(c, sh, p, c0, c1);
}
__device__ __noinline__ void factor_chunks(const Ctx& c, const LShared& sh, ChunkPass p, int c0, int c1) {
    factor_chunks_body<false>(c, sh, p, c0, c1);
}
template <bool RS_>
__device__ __noinline__ void update_chunks(const Ctx& c, ChunkPass p, int c0, int c1) {
    update_chunks_body<RS_, false>(c, p, c0, c1);
}
// the instance's own chunks (plain stores, calls)
__device__ void do_chunks(const Ctx& c, const LShared& sh, ChunkPass p, int c0, int c1, bool helper) {
    (void)helper;
    if (p.pass == PASS_NRES) nres_chunks(c, sh, p, c0, c1);
    else if (p.pass == PASS_FACTOR) factor_chunks(c, sh, p, c0, c1);
    else if (sh.R) update_chunks<true>(c, p, c0, c1);
    else update_chunks<false>(c, p, c0, c1);
}
// a helper's chunk (write-through stores, inlined)
__device__ __forceinline__ void do_chunks_helper(const Ctx& c, const LShared& sh, ChunkPass p, int c0, int c1) {
    if (p.pass == PASS_NRES) nres_chunks_body<true>(c, sh, p, c0, c1);
    else if (p.pass == PASS_FACTOR) factor_chunks_body<true>(c, sh, p, c0, c1);
    else if (sh.R) update_chunks_body<true, true>(c, p, c0, c1);
    else update_chunks_body<false, true>(c, p, c0, c1);
}

// a helper workgroup: serve open chunks of any instance until every instance has finished
__device__ __forceinline__ void helper_main(LArgs& a, Ctx& cw, LShared& sh) {
    const int B = a.B, lane = (int)threadIdx.x;
    gu64* hdr = board_line(a, B);
    if (lane == 0) {
        // a helper that finds an instance not yet started leaves: a workgroup that waits for the batch to finish must
        // never hold a CU an instance still needs (dispatch order is not promised).  The instances count themselves at
        // kernel entry; a helper dispatched right behind them waits up to kStartTicks (20 us) for that count before it
        // decides -- round 5 decided at the first look, so with a small batch the helpers could all leave while the
        // instances were still in their first instructions (a flaky 2x on the B = 1 plan).
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        unsigned long long st = ld_rlx(hdr + 2);
        while (st < (unsigned long long)B && __builtin_amdgcn_s_memrealtime() - t0 < kStartTicks) {
            __builtin_amdgcn_s_sleep(4);
            st = ld_rlx(hdr + 2);
        }
        sh.hexit = st < (unsigned long long)B ? 1 : 0;
        if (!sh.hexit) add_rlx(hdr + 1, 1);
    }
    __syncthreads();
    if (sh.hexit) return;
    int pos = (((int)blockIdx.x - B) * 7) % B;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
        if (lane < 64) {  // wave 0 looks at 64 instances per round
            int ex = 0;
            if (lane == 0)
                ex = ld_rlx(hdr) >= (unsigned long long)B || __builtin_amdgcn_s_memrealtime() - t0 > 12ull * kSpinTicks;
            ex = __builtin_amdgcn_readfirstlane(ex);
            int gb = -1, gc = -1;
            if (!ex) {
                const int b = (pos + lane) % B;
                const unsigned long long w = lane < B ? ld_rlx(board_line(a, b)) : 0ull;
                auto claimable = [](unsigned long long v) {  // open pass, next chunk below the chunk count
                    return ((v >> 40) & 1ull) && (v & kClaimFieldMask) < ((v >> kClaimChunkShift) & kClaimFieldMask);
                };
                const bool open = claimable(w);
                const unsigned long long m = __ballot(open);
                if (m) {
                    const int l = __ffsll((long long)m) - 1;
                    int cb = -1, cc = -1;
                    if (lane == l) {
                        const unsigned long long o = add_rlx(board_line(a, b), 1);
                        if (claimable(o)) { cb = b; cc = (int)(o & kClaimFieldMask); }
                    }
                    gb = __builtin_amdgcn_readlane(cb, l);
                    gc = __builtin_amdgcn_readlane(cc, l);
                    pos = (pos + l) % B;  // the next round starts at the instance just served
                } else {
                    pos = (pos + 64) % B;
                }
            }
            if (lane == 0) { sh.hexit = ex; sh.hb = gb; sh.hcur = gc; }
        }
        __syncthreads();
        const int b = sh.hb, ci = sh.hcur, ex = sh.hexit;
        __syncthreads();
        if (ex) break;
        if (b < 0) {
            __builtin_amdgcn_s_sleep(32);
            continue;
        }
        if (lane == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            gu64* ln = board_line(a, b);
            const unsigned long long pk = ld_rlx(ln + 7);
            sh.hp_mu = bitsd(ld_rlx(ln + 2)); sh.hp_dw = bitsd(ld_rlx(ln + 3)); sh.hp_tau = bitsd(ld_rlx(ln + 4));
            sh.zeta = bitsd(ld_rlx(ln + 5)); sh.dc = bitsd(ld_rlx(ln + 6));
            sh.hp_pk = (int)pk;
            sh.R = (int)(pk >> 16) & 15;
            sh.lsq = (int)(pk >> 20) & 15;
            cw.ws = (gdouble*)(a.ws + (size_t)b * obca_ws_doubles(a.N, a.M));
            cw.b = b;
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        ChunkPass p;
        p.mu = sh.hp_mu; p.dw = sh.hp_dw; p.tau = sh.hp_tau;
        const int pk = sh.hp_pk;
        p.pass = pk & 15; p.buf = (pk >> 4) & 15; p.prep = (pk >> 8) & 15; p.mode = (pk >> 12) & 15;
        do_chunks_helper(cw, sh, p, ci, ci + 1);  // write-through (sc1) stores
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        // the done count publishes the chunk: a release add (advisor r5), so the instance's acquire synchronizes with
        // it under the HIP memory model and not only by the sc1 + vmcnt(0) drain above (OBCA_HELPER_RELEASE 0: relaxed)
        if (lane == 0) {
            if constexpr (OBCA_HELPER_RELEASE)
                __hip_atomic_fetch_add(board_line(a, b) + 1, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            else
                add_rlx(board_line(a, b) + 1, 1);
        }
    }
}

__device__ __noinline__ void phase_nres(const Ctx& c, LShared& sh, double mu, double dw, double tau, int buf, bool prep,
                                        int mode, double (&out)[7]) {
    const WsView vw = ws_view(c);
    LArgs& a = *c.a;
    const int N = c.N;
    const bool plan = c.plan(), rs = sh.R != 0;
    const double zeta = sh.zeta, dt = c.dt, dc = sh.dc;
    double rmax = 0.0, bmax = 0.0, snorm = 0.0, ap = 1.0, az = 1.0, Dm = 0.0, rel = 0.0;
    auto R = [&](double v) { rmax = fmax(rmax, fabs(v)); return v; };
    auto Bc = [&](double v) { bmax = fmax(bmax, fabs(v)); return v; };
    auto dual = [&](double z, double dz) { if (dz < 0.0) az = fmin(az, -tau * z * inv(dz)); };
    // the block part over the flat block index (all threads busy: 2M (N + 1) blocks in ceil(2M (N + 1) / T) rounds), by
    // this workgroup and any helpers
    run_pass(c, sh, ChunkPass{mu, dw, tau, PASS_NRES, buf, prep ? 1 : 0, mode});
    for (int k = (int)threadIdx.x; k <= N; k += T) {
        const bool st = k < N;
        double x[6], dx[6], yp[6], ypn[6] = {0, 0, 0, 0, 0, 0}, dj[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0}, wd[7] = {0, 0, 0, 0, 0, 0, 0};
        load_x(c, k, x);
#pragma unroll
        for (int i = 0; i < 6; ++i) { dx[i] = vw.S(S_DX + 6 * buf + i, k); yp[i] = vw.S(S_YCP + 6 * buf + i, k); }
        if (st) {
#pragma unroll
            for (int i = 0; i < 6; ++i) ypn[i] = vw.S(S_YCP + 6 * buf + i, k + 1);
#pragma unroll
            for (int i = 0; i < 9; ++i) dj[i] = vw.S(S_AJ + i, k);
#pragma unroll
            for (int i = 0; i < 7; ++i) wd[i] = vw.S(S_WD + i, k);
        }
        // ---- x rows (without the block terms, added below) ----
        double rx[6];
        const double sc = (k == N && plan) ? a.tfac : 1.0;
        double Hd[21];
#pragma unroll
        for (int i = 0; i < 6; ++i)
#pragma unroll
            for (int j2 = i; j2 < 6; ++j2) Hd[sy6(i, j2)] = rs ? 0.0 : sc * (a.Q[i * 6 + j2] + a.Q[j2 * 6 + i]);
        Hd[sy6(2, 2)] += wd[0]; Hd[sy6(2, 5)] += wd[1]; Hd[sy6(3, 3)] += wd[2]; Hd[sy6(3, 4)] += wd[3];
        Hd[sy6(3, 5)] += wd[4]; Hd[sy6(4, 4)] += wd[5]; Hd[sy6(4, 5)] += wd[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const double xv = x[i], d = dx[i];
            double g = vw.S(S_GX + i, k), sg = dw + (rs ? zeta * vw.S(S_DRX + i, k) : 0.0);
            rel = fmax(rel, fabs(d) * inv(1.0 + fabs(xv)));
            if (c.hlx(i)) {
                const double is = inv(xv - c.xl[i]), z = vw.S(S_ZLX + i, k);
                g -= mu * is;
                sg += z * is;
                ftb_lo(xv, c.xl[i], d, tau, ap);
                dual(z, mu * is - z - z * is * d);
            }
            if (c.hux(i)) {
                const double is = inv(c.xu[i] - xv), z = vw.S(S_ZUX + i, k);
                g += mu * is;
                sg += z * is;
                ftb_hi(xv, c.xu[i], d, tau, ap);
                dual(z, mu * is - z + z * is * d);
            }
            Dm += g * d;
            double t = Bc(g) + sg * d + yp[i] - ypn[i];
#pragma unroll
            for (int j2 = 0; j2 < 6; ++j2) t += Hd[sy6(i, j2)] * dx[j2];
            rx[i] = t;
            snorm = fmax(snorm, fmax(fabs(d), fabs(yp[i])));
        }
        // -A'y+_{k+1}: the D' part
        rx[2] -= dj[0] * ypn[0] + dj[2] * ypn[1];
        rx[3] -= dj[6] * ypn[3];
        rx[4] -= dj[4] * ypn[2] + dj[7] * ypn[3];
        rx[5] -= dj[1] * ypn[0] + dj[3] * ypn[1] + dj[5] * ypn[2] + dj[8] * ypn[3];
        // ---- OBCA blocks: their records (nres_block), in block order ----
        double q4[4] = {0, 0, 0, 0};
        for (int j = 0; j < c.nbk; ++j) {
            double cb[CB_END];
#pragma unroll
            for (int i = 0; i < CB_END; ++i) cb[i] = vw.B(B_CB + i, j, k);
            rx[2] += cb[CB_RX];
            rx[3] += cb[CB_RX + 1];
#pragma unroll
            for (int q = 0; q < 4; ++q) rx[q] += cb[CB_RX + 2 + q];
            if (prep)
#pragma unroll
                for (int q = 0; q < 4; ++q) q4[q] += cb[CB_Q4 + q];
            rmax = fmax(rmax, cb[CB_RMAX]);
            bmax = fmax(bmax, cb[CB_BMAX]);
            snorm = fmax(snorm, cb[CB_SN]);
            rel = fmax(rel, cb[CB_REL]);
            ap = fmin(ap, cb[CB_AP]);
            az = fmin(az, cb[CB_AZ]);
            Dm += cb[CB_DM];
        }
        // ---- u rows (after the blocks: their operands are re-read rather than kept live across the block loop) ----
        double yq[6], yn4 = 0.0, yn5 = 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) yq[i] = vw.S(S_YCP + 6 * buf + i, k);
        if (st) { yn4 = vw.S(S_YCP + 6 * buf + 4, k + 1); yn5 = vw.S(S_YCP + 6 * buf + 5, k + 1); }
        double ru[2] = {0.0, 0.0}, u[2] = {0.0, 0.0}, du[2] = {0.0, 0.0};
        if (st)
#pragma unroll
            for (int i = 0; i < 2; ++i) { u[i] = vw.S(S_U + i, k); du[i] = vw.S(S_DU + 2 * buf + i, k); }
        if (st)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const double uv = u[i], d = du[i];
                double g = vw.S(S_GU + i, k), sg = dw + (rs ? zeta * vw.S(S_DRU + i, k) : 0.0);
                rel = fmax(rel, fabs(d) * inv(1.0 + fabs(uv)));
                if (c.hlu(i)) {
                    const double is = inv(uv - c.ul[i]), z = vw.S(S_ZLU + i, k);
                    g -= mu * is;
                    sg += z * is;
                    ftb_lo(uv, c.ul[i], d, tau, ap);
                    dual(z, mu * is - z - z * is * d);
                }
                if (c.huu(i)) {
                    const double is = inv(c.uu[i] - uv), z = vw.S(S_ZUU + i, k);
                    g += mu * is;
                    sg += z * is;
                    ftb_hi(uv, c.uu[i], d, tau, ap);
                    dual(z, mu * is - z + z * is * d);
                }
                Dm += g * d;
                double t = Bc(g) + sg * d - dt * (i == 0 ? yn5 : yn4);
                if (!rs) t += (i == 0 ? 2.0 * a.R[0] * du[0] + (a.R[1] + a.R[2]) * du[1]
                                      : (a.R[1] + a.R[2]) * du[0] + 2.0 * a.R[3] * du[1]);
                ru[i] = R(t);
            }
        // ---- dynamics rows of stage k: c_k (+ delta_c y_k) + dx_k - A_{k-1} dx_{k-1} - B du_{k-1} (- dp + dn)
        // (- delta_c y+_k) ----
        double rc[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const double cr = vw.S(S_CR + i, k);
            rc[i] = Bc(dc > 0.0 ? fma(dc, (double)vw.S(S_YC + i, k), cr) : cr) + dx[i];
        }
        if (k > 0) {
            double dxp[6], ajp[9];
#pragma unroll
            for (int i = 0; i < 6; ++i) dxp[i] = vw.S(S_DX + 6 * buf + i, k - 1);
#pragma unroll
            for (int i = 0; i < 9; ++i) ajp[i] = vw.S(S_AJ + i, k - 1);
            const double dup0 = vw.S(S_DU + 2 * buf, k - 1), dup1 = vw.S(S_DU + 2 * buf + 1, k - 1);
            rc[0] -= dxp[0] + fma(ajp[0], dxp[2], ajp[1] * dxp[5]);
            rc[1] -= dxp[1] + fma(ajp[2], dxp[2], ajp[3] * dxp[5]);
            rc[2] -= dxp[2] + fma(ajp[4], dxp[4], ajp[5] * dxp[5]);
            rc[3] -= dxp[3] + fma(ajp[6], dxp[3], fma(ajp[7], dxp[4], ajp[8] * dxp[5]));
            rc[4] -= dxp[4] + dt * dup1;
            rc[5] -= dxp[5] + dt * dup0;
        }
        double rpc[6] = {0, 0, 0, 0, 0, 0}, rnc[6] = {0, 0, 0, 0, 0, 0}, gpnc[6] = {0, 0, 0, 0, 0, 0};
        if (rs)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double p = vw.S(S_PR + i, k), n = vw.S(S_NR + i, k), zp = vw.S(S_ZP + i, k), zn = vw.S(S_ZN + i, k);
                const double ip = inv(p), in_ = inv(n);
                const double Dp = zp * ip + dw, Dn = zn * in_ + dw, gp = RHO - mu * ip, gn = RHO - mu * in_;
                double dp, dn;
                if (mode == NR_MAIN) {  // the pair's step from the new multiplier (phase_recover's pn_step)
                    dp = (yq[i] - gp) / Dp;
                    dn = (-yq[i] - gn) / Dn;
                    vw.S(S_DP + 6 * buf + i, k) = dp;
                    vw.S(S_DN + 6 * buf + i, k) = dn;
                } else {
                    dp = vw.S(S_DP + 6 * buf + i, k);
                    dn = vw.S(S_DN + 6 * buf + i, k);
                }
                rc[i] += -dp + dn;
                rpc[i] = R(Bc(gp) + Dp * dp - yq[i]);
                rnc[i] = R(Bc(gn) + Dn * dn + yq[i]);
                gpnc[i] = rpc[i] / Dp - rnc[i] / Dn;
                ftb_lo(p, 0.0, dp, tau, ap);
                ftb_lo(n, 0.0, dn, tau, ap);
                dual(zp, mu * ip - zp - zp * ip * dp);
                dual(zn, mu * in_ - zn - zn * in_ * dn);
                Dm += gp * dp + gn * dn;
                rel = fmax(rel, fmax(fabs(dp) * inv(1.0 + fabs(p)), fabs(dn) * inv(1.0 + fabs(n))));
            }
        if (dc > 0.0)
#pragma unroll
            for (int i = 0; i < 6; ++i) rc[i] -= dc * yq[i];
#pragma unroll
        for (int i = 0; i < 6; ++i) R(rc[i]);
        // ---- final rows (plan mode, stage N) ----
        double qf[6] = {0, 0, 0, 0, 0, 0};
        if (k == N && plan)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                if (mode == NR_MAIN) {  // the final rows' part of the step (phase_recover's)
                    const double sl = sh.sf[i] - c.fL, su = c.fU - sh.sf[i];
                    const double ypm = sh.Dfe[i] * (dx[i] + sh.rf[i]);
                    sh.ydpf[buf][i] = ypm;
                    sh.dsf[buf][i] = (ypm - (-mu / sl + mu / su)) / sh.Dsf[i];
                    if (rs) {
                        sh.dpf[buf][i] = (ypm - (RHO - mu / sh.pf[i])) / (sh.zpf[i] / sh.pf[i] + dw);
                        sh.dnf[buf][i] = (-ypm - (RHO - mu / sh.nf[i])) / (sh.znf[i] / sh.nf[i] + dw);
                    }
                }
                const double s = sh.sf[i], d = sh.dsf[buf][i], ypf = sh.ydpf[buf][i];
                rx[i] += ypf;
                const double sl = s - c.fL, su = c.fU - s;
                const double gs = -mu / sl + mu / su;
                double rf = Bc(dc > 0.0 ? fma(dc, sh.ydf[i], sh.dfr[i]) : sh.dfr[i]) + dx[i] - d;
                const double rsf = R(Bc(gs) + (sh.vLf[i] / sl + sh.vUf[i] / su + dw) * d - ypf);
                double gpn = 0.0;
                if (rs) {
                    const double p = sh.pf[i], n = sh.nf[i], zp = sh.zpf[i], zn = sh.znf[i];
                    const double dp = sh.dpf[buf][i], dn = sh.dnf[buf][i];
                    rf += -dp + dn;
                    const double Dp = zp / p + dw, Dn = zn / n + dw, gp = RHO - mu / p, gn = RHO - mu / n;
                    const double rp = R(Bc(gp) + Dp * dp - ypf), rn = R(Bc(gn) + Dn * dn + ypf);
                    gpn = rp / Dp - rn / Dn;
                    if (prep) { sh.opf[i] = rp; sh.onf[i] = rn; }
                    ftb_lo(p, 0.0, dp, tau, ap);
                    ftb_lo(n, 0.0, dn, tau, ap);
                    dual(zp, mu / p - zp - zp / p * dp);
                    dual(zn, mu / n - zn - zn / n * dn);
                    Dm += gp * dp + gn * dn;
                    rel = fmax(rel, fmax(fabs(dp) * inv(1.0 + fabs(p)), fabs(dn) * inv(1.0 + fabs(n))));
                }
                if (dc > 0.0) rf -= dc * ypf;
                R(rf);
                Dm += gs * d;
                rel = fmax(rel, fabs(d) * inv(1.0 + fabs(s)));
                ftb_lo(s, c.fL, d, tau, ap);
                ftb_hi(s, c.fU, d, tau, ap);
                dual(sh.vLf[i], mu / sl - sh.vLf[i] - sh.vLf[i] / sl * d);
                dual(sh.vUf[i], mu / su - sh.vUf[i] + sh.vUf[i] / su * d);
                if (prep) {
                    const double rfp = rf + rsf / sh.Dsf[i] + gpn;
                    sh.rf[i] = rfp;
                    sh.osf[i] = rsf;
                    qf[i] = sh.Dfe[i] * rfp;
                }
            }
#pragma unroll
        for (int i = 0; i < 6; ++i) R(rx[i]);
        if (prep) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                vw.S(S_QV + i, k) = rx[i] + (i < 4 ? q4[i] : 0.0) + qf[i];
                vw.S(S_CE + i, k) = rc[i] + (rs ? gpnc[i] : 0.0);
                if (rs) { vw.S(S_OP + i, k) = rpc[i]; vw.S(S_ON + i, k) = rnc[i]; }
            }
            if (st) { vw.S(S_RV, k) = ru[0]; vw.S(S_RV + 1, k) = ru[1]; }
        }
    }
    out[0] = rmax; out[1] = bmax; out[2] = snorm; out[3] = ap; out[4] = az; out[5] = Dm; out[6] = rel;
    const int ops[7] = {R_MAX, R_MAX, R_MAX, R_MIN, R_MIN, R_SUM, R_MAX};
    wg_reduce(sh, out, ops);
}

// ---- correction solve: its stage parts (dx, du, y+_c, the dynamics rows' elastic-pair steps, the final rows)
// added into the step in buffer buf; the blocks' parts follow in phase_nres (NR_CORR), which reads the summed
// stage fields of neighbouring stages (hence a pass of its own) ----
__device__ __noinline__ void phase_stage_add(const Ctx& c, LShared& sh, double dw, int buf) {
    const WsView vw = ws_view(c);
    const int N = c.N;
    const bool plan = c.plan(), rs = sh.R != 0;
    for (int k = (int)threadIdx.x; k <= N; k += T) {
        double dxc[6], ypc[6], sdx[6], syp[6], sdp[6] = {0, 0, 0, 0, 0, 0}, sdn[6] = {0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            dxc[i] = vw.S(S_DX + 12 + i, k); ypc[i] = vw.S(S_YCP + 12 + i, k);
            sdx[i] = vw.S(S_DX + 6 * buf + i, k); syp[i] = vw.S(S_YCP + 6 * buf + i, k);
        }
        if (rs)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double p = vw.S(S_PR + i, k), n = vw.S(S_NR + i, k), zp = vw.S(S_ZP + i, k), zn = vw.S(S_ZN + i, k);
                sdp[i] = vw.S(S_DP + 6 * buf + i, k) + (ypc[i] - vw.S(S_OP + i, k)) / (zp / p + dw);
                sdn[i] = vw.S(S_DN + 6 * buf + i, k) + (-ypc[i] - vw.S(S_ON + i, k)) / (zn / n + dw);
            }
        double du0 = 0.0, du1 = 0.0;
        if (k < N) {
            du0 = vw.S(S_DU + 2 * buf, k) + vw.S(S_DU + 4, k);
            du1 = vw.S(S_DU + 2 * buf + 1, k) + vw.S(S_DU + 5, k);
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            vw.S(S_DX + 6 * buf + i, k) = sdx[i] + dxc[i];
            vw.S(S_YCP + 6 * buf + i, k) = syp[i] + ypc[i];
            if (rs) { vw.S(S_DP + 6 * buf + i, k) = sdp[i]; vw.S(S_DN + 6 * buf + i, k) = sdn[i]; }
        }
        if (k < N) { vw.S(S_DU + 2 * buf, k) = du0; vw.S(S_DU + 2 * buf + 1, k) = du1; }
        if (k == N && plan)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double ypf = sh.Dfe[i] * (dxc[i] + sh.rf[i]);
                sh.ydpf[buf][i] += ypf;
                sh.dsf[buf][i] += (ypf - sh.osf[i]) / sh.Dsf[i];
                if (rs) {
                    sh.dpf[buf][i] += (ypf - sh.opf[i]) / (sh.zpf[i] / sh.pf[i] + dw);
                    sh.dnf[buf][i] += (-ypf - sh.onf[i]) / (sh.znf[i] / sh.nf[i] + dw);
                }
            }
    }
}

// the correction solve of one refinement step: right-hand side prepared by phase_nres (prep), vector-only sweeps
// through the stored factorisation into buffer 2, its stage parts added into buffer buf (the blocks' parts: the
// next phase_nres, NR_CORR)
__device__ __noinline__ void correction_solve(const Ctx& c, LShared& sh, double mu, double dw, int buf) {
    const bool soft = sh.R != 0 || sh.dc > 0.0, on = c.a->stamps != nullptr;
    if (c.lds) {
        stage_vec_inputs(c, c.lds, soft);
        __syncthreads();
        stamp(sh, on, OPH_REF_STAGE);
        if (threadIdx.x < 64) riccati_vec(c, VecL{(const lds_double*)c.lds}, soft);
        __syncthreads();
        stamp(sh, on, OPH_REF_SWEEP);
        stage_soft_forward(c, c.lds, soft);
        __syncthreads();
        stamp(sh, on, OPH_REF_STAGE);
        if (threadIdx.x < 64) {
            if (soft) forward_soft(c, SoftF{(const lds_double*)c.lds}, 2);
            else forward(c, SoftF{(const lds_double*)c.lds}, 2);
        }
    } else {
        if (threadIdx.x < 64) riccati_vec(c, VecG{c}, soft);
        __syncthreads();
        if (threadIdx.x < 64) {
            if (soft) forward_soft(c, SoftFG{c}, 2);
            else forward(c, SoftFG{c}, 2);
        }
    }
    __syncthreads();
    stamp(sh, on, OPH_REF_SWEEP);
    phase_stage_add(c, sh, dw, buf);
    __syncthreads();
}

// the step solve's recovery + IPOPT's iterative refinement for the step in buffer buf (factorisation, sweeps and
// forward sweep done; the blocks' recovery is fused into the first residual pass).  rec: the line-search quantities
// of the refined step (alpha_primal, alpha_dual, grad phi' d, max relative step), as phase_recover's.
// PDFullSpaceSolver::Solve: at least min_refinement_steps 1 correction; continue while the residual ratio
// max|r| / (min(max|sol|, 1e6) + max|rhs|) exceeds residual_ratio_max 1e-10; give up ("quit", returned true) after more
// than one correction when the ratio did not improve (residual_improvement_factor 1) or after max_refinement_steps 10.
// *ratio: the final residual ratio (the caller's pretend-singular test, oracle/c/tt_obca.c: pd_solve).
__device__ __noinline__ bool refine(const Ctx& c, LShared& sh, double mu, double dw, double tau, int buf, double (&rec)[5],
                                    double* ratio_out) {
    const bool on = c.a->stamps != nullptr;
    double q[7];
    phase_nres(c, sh, mu, dw, tau, buf, true, NR_MAIN, q);
    stamp(sh, on, OPH_REC);
    const double bnorm = q[1];
    double ratio = q[0] / (fmin(q[2], 1e6) + bnorm);
    bool quit = false, prepped = true;  // the NR_MAIN pass prepared the first correction's right-hand side
    for (int it = 0; !quit && (it < 1 || ratio > 1e-10); ++it) {
        // One correction is the rule away from the degenerate tail, so the residual pass after the first runs without
        // the next correction's right-hand side (the prep part); once a second correction was needed, more follow (C4
        // tail: ~3.8 per solve, profiles/r04/tail/) and every residual pass prepares the next one, instead of a
        // separate NR_STEP pass per correction (the same expressions on the same inputs: bitwise the same step)
        if (!prepped) {
            phase_nres(c, sh, mu, dw, tau, buf, true, NR_STEP, q);
            stamp(sh, on, OPH_REF_REC);
        }
        __syncthreads();
        count(sh, on, OCNT_CORR);
        correction_solve(c, sh, mu, dw, buf);
        prepped = it >= 1;
        phase_nres(c, sh, mu, dw, tau, buf, prepped, NR_CORR, q);
        stamp(sh, on, OPH_REF_REC);
        const double ratio2 = q[0] / (fmin(q[2], 1e6) + bnorm);
        if (ratio2 > 1e-10 && it + 1 > 1 && (it + 1 > 10 || ratio2 > ratio)) quit = true;
        ratio = ratio2;
    }
    __syncthreads();
    rec[0] = q[3]; rec[1] = q[4]; rec[2] = q[5]; rec[3] = q[6];
    *ratio_out = ratio;
    return quit;
}

// ======== restoration / soft-restoration / acceptable-point bookkeeping (all stage-parallel) ========
// snapshot of the iterate (save = true) or its restore (soft restoration trial)
__device__ __noinline__ void phase_snapshot(const Ctx& c, LShared& sh, bool save) {
    const int N = c.N;
    auto mv = [&](gdouble& live, gdouble& snap) { if (save) snap = live; else live = snap; };
    for (int k = (int)threadIdx.x; k <= N; k += T) {
        int o = S_SNAP;
#pragma unroll
        for (int i = 0; i < 6; ++i) { mv(c.S(S_X + i, k), c.S(o + i, k)); mv(c.S(S_ZLX + i, k), c.S(o + 6 + i, k)); mv(c.S(S_ZUX + i, k), c.S(o + 12 + i, k)); mv(c.S(S_YC + i, k), c.S(o + 18 + i, k)); }
#pragma unroll
        for (int i = 0; i < 2; ++i) { mv(c.S(S_U + i, k), c.S(o + 24 + i, k)); mv(c.S(S_ZLU + i, k), c.S(o + 26 + i, k)); mv(c.S(S_ZUU + i, k), c.S(o + 28 + i, k)); }
        for (int j = 0; j < c.nbk; ++j) {
#pragma unroll
            for (int e = 0; e < 8; ++e) { mv(c.B(B_W + e, j, k), c.B(B_SNAP + e, j, k)); mv(c.B(B_ZW + e, j, k), c.B(B_SNAP + 8 + e, j, k)); }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                mv(c.B(B_S + r, j, k), c.B(B_SNAP + 16 + r, j, k));
                mv(c.B(B_VL + r, j, k), c.B(B_SNAP + 20 + r, j, k));
                mv(c.B(B_VU + r, j, k), c.B(B_SNAP + 24 + r, j, k));
                mv(c.B(B_YD + r, j, k), c.B(B_SNAP + 28 + r, j, k));
            }
        }
        if (k == N && c.plan())
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                if (save) { sh.snapf[i] = sh.sf[i]; sh.snapf[6 + i] = sh.vLf[i]; sh.snapf[12 + i] = sh.vUf[i]; sh.snapf[18 + i] = sh.ydf[i]; }
                else { sh.sf[i] = sh.snapf[i]; sh.vLf[i] = sh.snapf[6 + i]; sh.vUf[i] = sh.snapf[12 + i]; sh.ydf[i] = sh.snapf[18 + i]; }
            }
    }
}

// last acceptable iterate (IPOPT's stored acceptable point): store (x, u, w) or restore it
__device__ __noinline__ void phase_acc(const Ctx& c, bool restore) {
    const WsView vw = ws_view(c);
    for (int k = (int)threadIdx.x; k <= c.N; k += T) {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            if (restore) vw.S(S_X + i, k) = vw.S(S_XACC + i, k); else vw.S(S_XACC + i, k) = vw.S(S_X + i, k);
        }
        if (k < c.N)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                if (restore) vw.S(S_U + i, k) = vw.S(S_UACC + i, k); else vw.S(S_UACC + i, k) = vw.S(S_U + i, k);
            }
        for (int j = 0; j < c.nbk; ++j)
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                if (restore) vw.B(B_W + e, j, k) = vw.B(B_WACC + e, j, k); else vw.B(B_WACC + e, j, k) = vw.B(B_W + e, j, k);
            }
    }
}

__device__ __forceinline__ double dr2(double v) { const double d = fmin(1.0, 1.0 / fabs(v)); return d * d; }

// elastic pairs at their closed form for the raw rows at the iterate (entry; restoration of the restoration)
__device__ __noinline__ void phase_setpn(const Ctx& c, LShared& sh, double mu) {
    const int N = c.N;
    for (int k = (int)threadIdx.x; k <= N; k += T) {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            double p, n;
            pn_closed_form(c.S(S_C + i, k), mu, p, n);
            c.S(S_PR + i, k) = p;
            c.S(S_NR + i, k) = n;
            c.S(S_ZP + i, k) = mu / p;
            c.S(S_ZN + i, k) = mu / n;
        }
        for (int j = 0; j < c.nbk; ++j)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                double p, n;
                pn_closed_form(c.B(B_D + r, j, k) - c.B(B_S + r, j, k), mu, p, n);
                c.B(B_PR + r, j, k) = p;
                c.B(B_NR + r, j, k) = n;
                c.B(B_ZP + r, j, k) = mu / p;
                c.B(B_ZN + r, j, k) = mu / n;
            }
        if (k == N && c.plan())
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                double p, n;
                pn_closed_form(sh.df[i] - sh.sf[i], mu, p, n);
                sh.pf[i] = p;
                sh.nf[i] = n;
                sh.zpf[i] = mu / p;
                sh.znf[i] = mu / n;
            }
    }
}

// enter the restoration phase at the (linearised, original) iterate: reference point and D_R^2, saved
// bound multipliers, elastic pairs, bound multipliers clipped to rho, constraint multipliers 0
__device__ __noinline__ void phase_enter_resto(const Ctx& c, LShared& sh, double muR) {
    const int N = c.N;
    for (int k = (int)threadIdx.x; k <= N; k += T) {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const double x = c.S(S_X + i, k);
            c.S(S_XR + i, k) = x;
            c.S(S_DRX + i, k) = dr2(x);
            const double zl = c.S(S_ZLX + i, k), zu = c.S(S_ZUX + i, k);
            c.S(S_SZ + i, k) = zl;
            c.S(S_SZ + 6 + i, k) = zu;
            c.S(S_ZLX + i, k) = fmin(zl, RHO);
            c.S(S_ZUX + i, k) = fmin(zu, RHO);
            c.S(S_YC + i, k) = 0.0;
        }
        if (k < N)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const double u = c.S(S_U + i, k);
                c.S(S_UR + i, k) = u;
                c.S(S_DRU + i, k) = dr2(u);
                const double zl = c.S(S_ZLU + i, k), zu = c.S(S_ZUU + i, k);
                c.S(S_SZ + 12 + i, k) = zl;
                c.S(S_SZ + 14 + i, k) = zu;
                c.S(S_ZLU + i, k) = fmin(zl, RHO);
                c.S(S_ZUU + i, k) = fmin(zu, RHO);
            }
        for (int j = 0; j < c.nbk; ++j) {
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                const double w = c.B(B_W + e, j, k), z = c.B(B_ZW + e, j, k);
                c.B(B_WR + e, j, k) = w;
                c.B(B_DRW + e, j, k) = dr2(w);
                c.B(B_SZW + e, j, k) = z;
                c.B(B_ZW + e, j, k) = fmin(z, RHO);
            }
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                c.B(B_SR + r, j, k) = c.B(B_S + r, j, k);
                const double vl = c.B(B_VL + r, j, k), vu = c.B(B_VU + r, j, k);
                c.B(B_SVL + r, j, k) = vl;
                c.B(B_SVU + r, j, k) = vu;
                c.B(B_VL + r, j, k) = fmin(vl, RHO);
                c.B(B_VU + r, j, k) = fmin(vu, RHO);
                c.B(B_YD + r, j, k) = 0.0;
            }
        }
        if (k == N && c.plan())
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                sh.sfR[i] = sh.sf[i];
                sh.svLf[i] = sh.vLf[i];
                sh.svUf[i] = sh.vUf[i];
                sh.vLf[i] = fmin(sh.vLf[i], RHO);
                sh.vUf[i] = fmin(sh.vUf[i], RHO);
                sh.ydf[i] = 0.0;
            }
    }
    phase_setpn(c, sh, muR);
    __syncthreads();
    if (threadIdx.x == 0) {
        sh.R = 1;
        sh.zeta = sqrt(muR);
    }
    __syncthreads();
}

// leave the restoration phase: original bound multipliers advanced by the complementarity Newton step of
// the whole restoration change (fraction to the boundary tau), kappa_sigma safeguard, all reset to 1 when
// one exceeds 1000; constraint multipliers 0
__device__ __noinline__ void phase_leave_resto(const Ctx& c, LShared& sh, double mu, double tau) {
    const int N = c.N;
    double red[1] = {1.0};
    // dz of a lower-bound multiplier z0 whose slack moved from sl0 by d
    auto dzl = [&](double z0, double sl0, double d) { return mu / sl0 - z0 - z0 / sl0 * d; };
    for (int pass = 0; pass < 2; ++pass) {
        double acc = pass == 0 ? 1.0 : 0.0;  // pass 0: fraction to the boundary; pass 1: max multiplier
        const double al = red[0];
        auto use = [&](double z0, double dz, gdouble& z, double slnew) {
            if (pass == 0) { if (dz < 0.0) acc = fmin(acc, -tau * z0 / dz); }
            else { double zn = z0 + al * dz; clamp_mult(zn, slnew, mu); z = zn; acc = fmax(acc, zn); }
        };
        for (int k = (int)threadIdx.x; k <= N; k += T) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double x = c.S(S_X + i, k), xr = c.S(S_XR + i, k), d = x - xr;
                if (c.hlx(i)) { const double z0 = c.S(S_SZ + i, k); use(z0, dzl(z0, xr - c.xl[i], d), c.S(S_ZLX + i, k), x - c.xl[i]); }
                if (c.hux(i)) { const double z0 = c.S(S_SZ + 6 + i, k); use(z0, dzl(z0, c.xu[i] - xr, -d), c.S(S_ZUX + i, k), c.xu[i] - x); }
            }
            if (k < N)
#pragma unroll
                for (int i = 0; i < 2; ++i) {
                    const double u = c.S(S_U + i, k), ur = c.S(S_UR + i, k), d = u - ur;
                    if (c.hlu(i)) { const double z0 = c.S(S_SZ + 12 + i, k); use(z0, dzl(z0, ur - c.ul[i], d), c.S(S_ZLU + i, k), u - c.ul[i]); }
                    if (c.huu(i)) { const double z0 = c.S(S_SZ + 14 + i, k); use(z0, dzl(z0, c.uu[i] - ur, -d), c.S(S_ZUU + i, k), c.uu[i] - u); }
                }
            for (int j = 0; j < c.nbk; ++j) {
#pragma unroll
                for (int e = 0; e < 8; ++e) {
                    const double w = c.B(B_W + e, j, k), wr = c.B(B_WR + e, j, k), z0 = c.B(B_SZW + e, j, k);
                    use(z0, dzl(z0, wr + RELAX, w - wr), c.B(B_ZW + e, j, k), w + RELAX);
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const double s = c.B(B_S + r, j, k), sr = c.B(B_SR + r, j, k), d = s - sr;
                    if (c.hrl(r)) { const double z0 = c.B(B_SVL + r, j, k); use(z0, dzl(z0, sr - c.rL(r), d), c.B(B_VL + r, j, k), s - c.rL(r)); }
                    const double z0 = c.B(B_SVU + r, j, k);
                    use(z0, dzl(z0, c.rU(r) - sr, -d), c.B(B_VU + r, j, k), c.rU(r) - s);
                }
            }
            if (k == N && c.plan())
#pragma unroll
                for (int i = 0; i < 6; ++i) {
                    const double s = sh.sf[i], sr = sh.sfR[i], d = s - sr;
                    const double dl = dzl(sh.svLf[i], sr - c.fL, d), du = dzl(sh.svUf[i], c.fU - sr, -d);
                    if (pass == 0) {
                        if (dl < 0.0) acc = fmin(acc, -tau * sh.svLf[i] / dl);
                        if (du < 0.0) acc = fmin(acc, -tau * sh.svUf[i] / du);
                    } else {
                        double vl = sh.svLf[i] + al * dl, vu = sh.svUf[i] + al * du;
                        clamp_mult(vl, s - c.fL, mu);
                        clamp_mult(vu, c.fU - s, mu);
                        sh.vLf[i] = vl;
                        sh.vUf[i] = vu;
                        acc = fmax(acc, fmax(vl, vu));
                    }
                }
        }
        red[0] = acc;
        const int ops[1] = {pass == 0 ? R_MIN : R_MAX};
        wg_reduce(sh, red, ops);
    }
    const bool reset = red[0] > BOUND_MULT_RESET;
    for (int k = (int)threadIdx.x; k <= N; k += T) {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            if (reset) {
                c.S(S_ZLX + i, k) = c.hlx(i) ? 1.0 : 0.0;
                c.S(S_ZUX + i, k) = c.hux(i) ? 1.0 : 0.0;
            }
            c.S(S_YC + i, k) = 0.0;
        }
        if (k < N && reset)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                c.S(S_ZLU + i, k) = c.hlu(i) ? 1.0 : 0.0;
                c.S(S_ZUU + i, k) = c.huu(i) ? 1.0 : 0.0;
            }
        for (int j = 0; j < c.nbk; ++j) {
            if (reset)
#pragma unroll
                for (int e = 0; e < 8; ++e) c.B(B_ZW + e, j, k) = 1.0;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                if (reset) {
                    c.B(B_VL + r, j, k) = c.hrl(r) ? 1.0 : 0.0;
                    c.B(B_VU + r, j, k) = 1.0;
                }
                c.B(B_YD + r, j, k) = 0.0;
            }
        }
        if (k == N && c.plan())
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                if (reset) sh.vLf[i] = sh.vUf[i] = 1.0;
                sh.ydf[i] = 0.0;
            }
    }
    __syncthreads();
    if (threadIdx.x == 0) sh.R = 0;
    __syncthreads();
}

// least-squares constraint multipliers of the current NLP (IPOPT constr_mult_init_max = 1000):
// [[I, J'], [J, 0]] [d; y] = [-(grad f - z); 0] with unit slack / elastic Hessians; kept when max |y| <= 1000
__device__ __noinline__ void ls_multipliers(const Ctx& c, LShared& sh) {
    const WsView vw = ws_view(c);
    if (threadIdx.x == 0) sh.lsq = 1;
    __syncthreads();
    double red[13];
    phase_lin(c, sh, red);  // Jacobians at the iterate (y = 0: no curvature terms)
    phase_resid(c, sh, true);
    __syncthreads();
    if (newton_solve(c, sh, 0.0, 0.0, 0.0, 0) == F_OK) {
        double rec[5];
        phase_recover(c, sh, 0.0, 0.0, 0.99, 0, rec);
        if (isfinite(rec[4]) && rec[4] <= CONSTR_MULT_INIT_MAX) {
            for (int k = (int)threadIdx.x; k <= c.N; k += T) {
#pragma unroll
                for (int i = 0; i < 6; ++i) vw.S(S_YC + i, k) = vw.S(S_YCP + i, k);
                for (int j = 0; j < c.nbk; ++j)
#pragma unroll
                    for (int r = 0; r < 4; ++r) vw.B(B_YD + r, j, k) = vw.B(B_YP + r, j, k);
                if (k == c.N && c.plan())
#pragma unroll
                    for (int i = 0; i < 6; ++i) sh.ydf[i] = sh.ydpf[0][i];
            }
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) sh.lsq = 0;
    __syncthreads();
}

// IPOPT's PDPerturbationHandler, restated (oracle/c/tt_obca.c: ph_new / ph_singular / ph_inertia, which cite the
// options): delta_x (= delta_s) on the Hessian, delta_c (= delta_d) on the constraint rows, the structural degeneracy
// test of the first singular matrices (degen_iters_max 3).  Every thread carries the same (uniform) state.
struct Perturb {
    enum { UNDET = -1, NOT = 0, DEG = 1 };
    enum { T_NONE = 0, T_C0X0, T_CPX0, T_C0XP, T_CPXP };
    int hess, jac, degen, test, gdwi;
    double dx, dx_last, dc;
    __device__ void reset() {
        hess = jac = UNDET;
        degen = 0;
        test = T_NONE;
        gdwi = 0;
        dx = dx_last = dc = 0.0;
    }
    __device__ static double dcd(double mu) { return 1e-8 * pow(mu, 0.25); }
    __device__ void finalize() {
        if (test == T_C0X0) {
            if (hess == UNDET && jac == UNDET) { hess = NOT; jac = NOT; }
            else if (hess == UNDET) hess = NOT;
            else if (jac == UNDET) jac = NOT;
        } else if (test == T_CPX0) {
            if (hess == UNDET) hess = NOT;
            if (jac == UNDET && ++degen >= 3) jac = DEG;
        } else if (test == T_C0XP) {
            if (jac == UNDET) jac = NOT;
            if (hess == UNDET && ++degen >= 3) hess = DEG;
        } else if (test == T_CPXP) {
            if (++degen >= 3) { hess = DEG; jac = DEG; }
        }
    }
    // get_deltas_for_wrong_inertia: false once delta_x would exceed max_hessian_perturbation 1e20
    __device__ bool wrong_inertia_deltas() {
        if (dx == 0.0) dx = dx_last == 0.0 ? 1e-4 : fmax(1e-20, dx_last / 3.0);
        else dx *= (dx_last == 0.0 || 1e5 * dx_last < dx) ? 100.0 : 8.0;
        if (dx > 1e20) { dx_last = 0.0; return false; }
        gdwi = 1;
        return true;
    }
    __device__ bool consider_new(double mu) {  // ConsiderNewSystem
        finalize();
        if (dx > 0.0) dx_last = dx;
        test = (hess == UNDET || jac == UNDET) ? T_C0X0 : T_NONE;
        dc = jac == DEG ? dcd(mu) : 0.0;
        dx = 0.0;
        if (hess == DEG && !wrong_inertia_deltas()) return false;
        gdwi = 0;
        return true;
    }
    __device__ bool singular(double mu) {  // PerturbForSingularity
        if (hess == UNDET || jac == UNDET) {
            if (test == T_C0X0) {
                if (jac == UNDET) { dc = dcd(mu); test = T_CPX0; }
                else { if (!wrong_inertia_deltas()) return false; test = T_C0XP; }
            } else if (test == T_CPX0) {
                dc = 0.0;
                if (!wrong_inertia_deltas()) return false;
                test = T_C0XP;
            } else if (test == T_C0XP) {
                dc = dcd(mu);
                if (!wrong_inertia_deltas()) return false;
                test = T_CPXP;
            } else {
                if (!wrong_inertia_deltas()) return false;
            }
        } else if (dc > 0.0 || gdwi) {
            if (!wrong_inertia_deltas()) return false;
        } else {
            dc = dcd(mu);
        }
        return true;
    }
    __device__ bool inertia(double mu) {  // PerturbForWrongInertia
        finalize();
        if (wrong_inertia_deltas()) return true;
        if (dc != 0.0) return false;
        dc = dcd(mu);  // delta_x gave up without delta_c: again with the constraint rows regularised
        dx = 0.0;
        test = T_NONE;
        if (hess == DEG) hess = NOT;
        return wrong_inertia_deltas();
    }
};

struct IpmState {
    double mu, tau, th_max, th_min;
    int acc;
    Perturb ph;  // one handler per NLP (original / restoration), as IPOPT's restoration algorithm has its own
};

// factorisations until the inertia is right (PDFullSpaceSolver::SolveOnce); false when the perturbation gave up
__device__ __forceinline__ bool factor_loop(const Ctx& c, LShared& sh, Perturb& ph, double mu, int buf) {
#pragma unroll 1
    for (int attempt = 0; attempt < 64; ++attempt) {
        const int f = newton_solve(c, sh, mu, ph.dx, ph.dc, buf);
        if (f == F_OK) return true;
        if (!(f == F_MANY ? ph.inertia(mu) : ph.singular(mu))) return false;
    }
    return false;
}

// one step solve (factorisation current) + refinement with IPOPT's pretend-singular safeguard: a refinement that gives
// up above residual_ratio_singular 1e-5 makes the handler treat the matrix as singular once (refactorisation, solve
// again).  false when the perturbation gave up.  rec: refine()'s line-search quantities.
__device__ __forceinline__ bool pd_solve(const Ctx& c, LShared& sh, Perturb& ph, double mu, double tau, int buf,
                                         double (&rec)[5]) {
    double ratio = 0.0;
    const bool quit = refine(c, sh, mu, ph.dx, tau, buf, rec, &ratio);
    if (!quit || ratio < 1e-5) return true;
    count(sh, c.a->stamps != nullptr, OCNT_PRETEND);
    if (!ph.singular(mu)) return false;
    if (!factor_loop(c, sh, ph, mu, buf)) return false;
    refine(c, sh, mu, ph.dx, tau, buf, rec, &ratio);
    return true;
}

// ---------------- the kernel ----------------
__global__ __launch_bounds__(T) __attribute__((amdgpu_waves_per_eu(1, 1))) void obca_kernel(ObcaArgs args) {
    __shared__ Shared sh_storage;
    LShared& sh = *(LShared*)&sh_storage;
    extern __shared__ double dyn_lds[];
    __shared__ ObcaArgs args_lds;
    // an instance counts itself started first thing, so that helpers dispatched right behind the instances see the
    // whole batch started (helper_main waits briefly for that instead of leaving at the first look)
    if (threadIdx.x == 0 && args.board && blockIdx.x < (unsigned)args.B)
        __hip_atomic_fetch_add((unsigned long long*)(args.board + (size_t)args.B * kObcaBoardStride) + 2, 1ull,
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    {
        const int* src = reinterpret_cast<const int*>(&args);
        int* dst = reinterpret_cast<int*>(&args_lds);
        for (int q = threadIdx.x; q < (int)(sizeof(ObcaArgs) / sizeof(int)); q += T) dst[q] = src[q];
        __syncthreads();
    }
    LArgs& a = *(LArgs*)&args_lds;
    Ctx c;
    c.a = &a;
    c.lds = obca_lds_bytes(a.N) <= kObcaLdsMax ? dyn_lds : nullptr;
    c.slab = (__attribute__((address_space(3))) double*)dyn_lds;  // the sweeps' staging area is free then
    c.b = blockIdx.x;
    c.N = a.N;
    c.NP = a.N + 1;
    c.nbk = 2 * a.M;
    c.tid = threadIdx.x;
    c.ws = (gdouble*)(a.ws + (size_t)c.b * obca_ws_doubles(a.N, a.M));
    c.dt = a.dt;
    c.pd = (a.opts & OBCA_OPT_PD_BLOCKS) != 0;
    c.refine = (a.opts & OBCA_OPT_NO_REFINE) == 0;
    const int N = c.N, NBK = c.nbk, tid = c.tid;
    const bool plan = a.mode == OBCA_PLAN;
    c.tgt_x = plan ? a.xgoal + 6 * (size_t)c.b : a.xref + (size_t)c.b * 6 * (N + 1);
    c.tgt_u = plan ? nullptr : a.uref + (size_t)c.b * 2 * N;
    const double* xinit = a.x0 + 6 * (size_t)c.b;
    c.hx = 0;
    c.hu = 0;
#pragma unroll
    for (int i = 0; i < 6; ++i) {
        const bool l = isfinite(a.xlb[i]) && a.xlb[i] > -1e19, u = isfinite(a.xub[i]) && a.xub[i] < 1e19;
        c.hx |= (l ? 1 : 0) << i;
        c.hx |= (u ? 1 : 0) << (8 + i);
        c.xl[i] = l ? a.xlb[i] - RELAX * fmax(1.0, fabs(a.xlb[i])) : -INFINITY;
        c.xu[i] = u ? a.xub[i] + RELAX * fmax(1.0, fabs(a.xub[i])) : INFINITY;
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const bool l = isfinite(a.ulb[i]) && a.ulb[i] > -1e19, u = isfinite(a.uub[i]) && a.uub[i] < 1e19;
        c.hu |= (l ? 1 : 0) << i;
        c.hu |= (u ? 1 : 0) << (8 + i);
        c.ul[i] = l ? a.ulb[i] - RELAX * fmax(1.0, fabs(a.ulb[i])) : -INFINITY;
        c.uu[i] = u ? a.uub[i] + RELAX * fmax(1.0, fabs(a.uub[i])) : INFINITY;
    }
    c.rlo = -a.eq_tol - RELAX;
    c.rhi = a.eq_tol + RELAX;
    c.fL = -a.fin_tol - RELAX;
    c.fU = a.fin_tol + RELAX;
    // the phases read the (uniform) context from an LDS copy instead of this thread's private copy
    __shared__ Ctx cs_storage;
    if (threadIdx.x == 0) cs_storage = c;
    __syncthreads();
    const Ctx& cs = cs_storage;
    if (blockIdx.x >= (unsigned)a.B) {  // a helper workgroup (see run_pass)
        helper_main(a, cs_storage, sh);
        return;
    }
    const int st = 8 + 16 * a.M;
    const size_t nz = obca_n(N, a.M);
    const double* zg = a.zg ? a.zg + (size_t)c.b * nz : nullptr;

    const bool ston = a.stamps != nullptr;
    if (tid == 0) {
        for (int i = 0; i < kObcaPhases; ++i) sh.stamp[i] = 0;
        sh.t0 = clock64();
        sh.R = 0;
        sh.lsq = 0;
        sh.zeta = 0.0;
        sh.nfl[0] = sh.nfl[1] = 0;
        sh.hep = 0;
        sh.hfail = 0;
    }
    const unsigned long long tstart = clock64();
    // ---------------- initial point (bound push, slacks = pushed d(x0), multipliers 1 / 0) ----------------
    bool infeasible = false;
#pragma unroll
    for (int i = 0; i < 6; ++i)
        if (!isfinite(xinit[i]) || (c.hlx(i) && xinit[i] < c.xl[i]) || (c.hux(i) && xinit[i] > c.xu[i])) infeasible = true;
    __syncthreads();
    for (int k = tid; k <= N; k += T) {
        double x[6], u[2] = {0.0, 0.0};
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            if (zg) x[i] = zg[(size_t)k * st + i];
            else if (plan) { const double t = (double)k / N; x[i] = k < N ? (1 - t) * xinit[i] + t * c.tgt_x[i] : c.tgt_x[i]; }
            else x[i] = c.tgt_x[6 * k + i];
        }
        if (k < N)
#pragma unroll
            for (int i = 0; i < 2; ++i) u[i] = zg ? zg[(size_t)k * st + 6 + i] : (plan ? 0.0 : c.tgt_u[2 * k + i]);
        const int o = k < N ? 8 : 6;
        for (int j = 0; j < NBK; ++j) {
            double w[8];
            const int ob = j >> 1, bd = j & 1;
#pragma unroll
            for (int e = 0; e < 4; ++e) {
                if (zg) {
                    w[e] = zg[(size_t)k * st + o + ob * 8 + 4 * bd + e];
                    w[4 + e] = zg[(size_t)k * st + o + 8 * a.M + ob * 8 + 4 * bd + e];
                } else {
                    w[e] = 100.0;
                    w[4 + e] = 100.0 + 5.0 * e;  // kron(1_M, [100,105,110,115,...]) (trajectory_optimization.py:222)
                }
            }
            if (a.dual_init) dual_certificate(a, x, j, w);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
                c.B(B_W + e, j, k) = push_into(w[e], -RELAX, INFINITY, true, false);
                c.B(B_ZW + e, j, k) = 1.0;
            }
        }
        if (!infeasible) {
#pragma unroll
            for (int i = 0; i < 6; ++i) x[i] = push_into(x[i], c.xl[i], c.xu[i], c.hlx(i), c.hux(i));
            if (k < N)
#pragma unroll
                for (int i = 0; i < 2; ++i) u[i] = push_into(u[i], c.ul[i], c.uu[i], c.hlu(i), c.huu(i));
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            c.S(S_X + i, k) = x[i];
            c.S(S_ZLX + i, k) = c.hlx(i) ? 1.0 : 0.0;
            c.S(S_ZUX + i, k) = c.hux(i) ? 1.0 : 0.0;
            c.S(S_YC + i, k) = 0.0;
        }
        if (k < N)
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                c.S(S_U + i, k) = u[i];
                c.S(S_ZLU + i, k) = c.hlu(i) ? 1.0 : 0.0;
                c.S(S_ZUU + i, k) = c.huu(i) ? 1.0 : 0.0;
            }
        const Trig tr = stage_trig(x);
        for (int j = 0; j < NBK; ++j) {
            double w[8], d[4];
#pragma unroll
            for (int e = 0; e < 8; ++e) w[e] = c.B(B_W + e, j, k);
            blk_vals(a, x, tr, j, w, d);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                c.B(B_S + r, j, k) = push_into(d[r], c.rL(r), c.rU(r), c.hrl(r), true);
                c.B(B_VL + r, j, k) = c.hrl(r) ? 1.0 : 0.0;
                c.B(B_VU + r, j, k) = 1.0;
                c.B(B_YD + r, j, k) = 0.0;
            }
        }
        if (k == N && plan)
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                sh.sf[i] = push_into(x[i] - c.tgt_x[i], c.fL, c.fU, true, true);
                sh.vLf[i] = sh.vUf[i] = 1.0;
                sh.ydf[i] = 0.0;
            }
    }
    __syncthreads();

    int status = 2, iter = 0;
    double E0 = INFINITY;
    if (infeasible) {
        status = 3;
    } else {
        int nxb = 0, nub = 0;
#pragma unroll
        for (int i = 0; i < 6; ++i) nxb += c.hlx(i) + c.hux(i);
#pragma unroll
        for (int i = 0; i < 2; ++i) nub += c.hlu(i) + c.huu(i);
        const double n_bounds = (double)(N + 1) * nxb + (double)N * nub + (double)(N + 1) * NBK * 14 + (plan ? 12 : 0);
        const double n_rows = 6.0 * (N + 1) + 4.0 * (N + 1) * NBK + (plan ? 6 : 0);
        const bool use_resto = !(a.opts & OBCA_OPT_NO_RESTO), use_soft = !(a.opts & OBCA_OPT_NO_SOFT_RESTO);
        const bool use_lsq = !(a.opts & OBCA_OPT_NO_LSQ_MULT);
        if (use_lsq) ls_multipliers(cs, sh);
        IpmState S0, S1;
        S0.mu = 0.1; S0.tau = fmax(0.99, 1.0 - 0.1); S0.th_max = S0.th_min = 0.0; S0.acc = 0;
        S0.ph.reset();
        S1 = S0;
        int in_soft = 0, soft_cnt = 0, first_resto = 0, resto_iter0 = 0, have_acc = 0;
        double th_resto0 = 0.0;
        const double kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5, smax = 100.0;
        const double mu_min = fmin(a.tol, kComplInfTol) / (kappa_eps + 1.0);  // MonotoneMuUpdate's barrier floor
        const double g_th = 1e-5, g_ph = 1e-8, s_ph = 2.3, s_th = 1.1, delta = 1.0, eta_ph = 1e-8, g_al = 0.05;
        const double tolc = 10.0 * EPS;
        for (iter = 0;; ++iter) {
            const int R = sh.R;
            IpmState stt = R ? S1 : S0;
            bool done = false, redo = false, switched = false;
            do {
                double red[13];
                stamp(sh, ston, OPH_UPD);
                if (R) count(sh, ston, OCNT_RESTO_IT);
                phase_lin(cs, sh, red);
                stamp(sh, ston, OPH_LIN);
                double dinf = red[0], pinf = red[1], c0 = red[2];
                if (sh.hfail) { status = kStatusHandoffTimeout; done = true; break; }
                if (!isfinite(dinf) || !isfinite(pinf)) { status = 4; done = true; break; }
                const double nbd = n_bounds + (R ? 2.0 * n_rows : 0.0);
                double sd = fmax(smax, red[3] / (n_rows + nbd)) / smax, sc = fmax(smax, red[4] / nbd) / smax;
                E0 = fmax(fmax(dinf / sd, pinf), c0 / sc);
                // IPOPT's OptimalityErrorConvergenceCheck: E_0 and the UNSCALED dual infeasibility, constraint violation
                // and complementarity (pinf bounds the NLP's constraint violation from above, oracle/c/tt_obca.c)
                const bool conv = E0 <= a.tol && dinf <= kDualInfTol && pinf <= kConstrViolTol && c0 <= kComplInfTol;
                const bool accp = E0 <= a.acc_tol && dinf <= kAccDualInfTol && pinf <= kAccConstrViolTol &&
                                  c0 <= kAccComplInfTol;
                if (!R) {
                    if (conv) { status = 0; done = true; break; }
                    if (accp) {
                        phase_acc(cs, false);
                        have_acc = 1;
                        if (++stt.acc >= a.acc_iter) { status = 1; done = true; break; }
                    } else {
                        stt.acc = 0;
                    }
                    if (iter >= a.max_iter) { status = accp ? 1 : 2; done = true; break; }
                } else {
                    // restoration convergence: original infeasibility down to kappa_resto of its value at entry and
                    // the point acceptable to the augmented original filter
                    const double thO = red[9], phO = red[10] - S0.mu * red[11];
                    if (!first_resto && thO <= KAPPA_RESTO * th_resto0 && thO <= S0.th_max && !in_filter(sh, 0, thO, phO)) {
                        phase_leave_resto(cs, sh, S0.mu, S0.tau);
                        S1 = stt;
                        S0.acc = 0;
                        switched = true;
                        redo = true;
                        break;
                    }
                    first_resto = 0;
                    if (accp) ++stt.acc; else stt.acc = 0;
                    if (conv || stt.acc >= a.acc_iter) {
                        // IPOPT's RestoConvergenceCheck: the ORIGINAL problem's primal infeasibility (max norm) against
                        // resto_failure_feasibility_threshold (default 1e2 tol)
                        if (red[12] <= 1e2 * a.tol) {  // feasible but filter-unacceptable
                            phase_leave_resto(cs, sh, S0.mu, S0.tau);
                            if (tid == 0) sh.nfl[0] = 0;
                            __syncthreads();
                            S1 = stt;
                            S0.acc = 0;
                            switched = true;
                            redo = true;
                            break;
                        }
                        status = 3;  // converged to a point of local infeasibility
                        done = true;
                        break;
                    }
                    if (iter >= a.max_iter) { status = 2; done = true; break; }
                }
                // ---- barrier update (monotone, Fiacco-McCormick); the filter is reset on every change ----
                while (stt.mu > mu_min * 1.0000001) {
                    // E_mu = max(dual, primal, complementarity): when the first two already exceed kappa_eps mu the
                    // test fails whatever the complementarity is (fmax(a, b) >= a for a non-NaN a), so its pass is
                    // skipped -- the usual case away from convergence; the decision is the same as with it
                    const double e_dp = fmax(dinf / sd, pinf);
                    if (e_dp > kappa_eps * stt.mu) break;
                    const double2 cm = phase_compl(cs, sh, stt.mu);
                    stamp(sh, ston, OPH_COMPL);
                    if (!(fmax(e_dp, cm.x / sc) <= kappa_eps * stt.mu)) break;
                    stt.mu = fmax(mu_min, fmin(kappa_mu * stt.mu, pow(stt.mu, theta_mu)));
                    stt.tau = fmax(0.99, 1.0 - stt.mu);
                    __syncthreads();
                    if (tid == 0) {
                        sh.nfl[R] = 0;
                        if (R) sh.zeta = sqrt(stt.mu);
                    }
                    __syncthreads();
                    if (R) {  // the proximity weight changed: gradient and optimality error with it
                        phase_lin(cs, sh, red);
                        dinf = red[0]; pinf = red[1]; c0 = red[2];
                        sd = fmax(smax, red[3] / (n_rows + nbd)) / smax;
                        sc = fmax(smax, red[4] / nbd) / smax;
                    }
                }
                const double mu = stt.mu;
                const double th0 = red[5], phi0 = red[6] - mu * red[7];
                // the Newton right-hand side's residual rows (S_CR / B_DR / dfr) were stored by phase_lin at this
                // iterate: the same expressions as phase_resid's
                // ---- Newton step with inertia correction (IPOPT's perturbation handler) ----
                double rec[5];
                bool ok = stt.ph.consider_new(mu) && factor_loop(cs, sh, stt.ph, mu, 0);
                if (ok) {
                    if (cs.refine) {
                        ok = pd_solve(cs, sh, stt.ph, mu, stt.tau, 0, rec);
                    } else {
                        phase_recover(cs, sh, mu, stt.ph.dx, stt.tau, 0, rec);
                        stamp(sh, ston, OPH_REC);
                    }
                }
                bool go_resto = false;
                if (!ok) {
                    if (R || !use_resto) { status = 5; done = true; break; } /* Error_In_Step_Computation */
                    go_resto = true;                                         /* IPOPT's fallback: restoration */
                } else {
                    const double ap = rec[0], Dm = rec[2], rel = rec[3];
                    double az = rec[1], alpha = ap;
                    int buf = 0;
                    bool accepted = false, ftype = false;
                    if (R || !in_soft) {
                        // ---- filter line search ----
                        const bool first = (R ? iter == resto_iter0 : iter == 0) || !(stt.th_max > 0);
                        if (first) { stt.th_max = 1e4 * fmax(1.0, th0); stt.th_min = 1e-4 * fmax(1.0, th0); }
                        double amin;
                        if (Dm < 0.0) {
                            amin = fmin(g_th, g_ph * th0 / (-Dm));
                            if (th0 <= stt.th_min) amin = fmin(amin, delta * pow(th0, s_th) / pow(-Dm, s_ph));
                        } else {
                            amin = g_th;
                        }
                        amin *= g_al;
                        accepted = rel < 1e-15;
                        // backtracking trials (ls >= 1) are evaluated kTrialBatch at a time (phase_trial_multi: the
                        // loop's own alpha sequence, bitwise phase_trial's results) and consumed one by one below
                        double pre[kTrialBatch][3];
                        int npre = 0;
                        for (int ls = 0; !accepted; ++ls) {
                            double tr[3];
                            count(sh, ston, OCNT_TRIAL);
                            if (ls == 0) {
                                phase_trial(cs, sh, mu, alpha, 0, tr);
                            } else {
                                if (npre == 0) {
                                    double al[kTrialBatch], an = alpha;
#pragma unroll
                                    for (int q = 0; q < kTrialBatch; ++q) { al[q] = an; an *= 0.5; }
                                    phase_trial_multi(cs, sh, mu, al, 0, pre);
                                    npre = kTrialBatch;
                                }
                                const int q = kTrialBatch - npre--;
                                tr[0] = pre[q][0]; tr[1] = pre[q][1]; tr[2] = pre[q][2];
                            }
                            stamp(sh, ston, OPH_TRIAL);
                            const bool sw = Dm < 0.0 && alpha * pow(-Dm, s_ph) > delta * pow(th0, s_th);
                            bool okls = false;
                            if (isfinite(tr[1]) && tr[0] <= stt.th_max && !in_filter(sh, R, tr[0], tr[1])) {
                                if (th0 <= stt.th_min && sw) { ftype = true; okls = tr[1] - (phi0 + eta_ph * alpha * Dm) <= tolc * fabs(phi0); }
                                else { ftype = false; okls = tr[0] <= (1.0 - g_th) * th0 || tr[1] - (phi0 - g_ph * th0) <= tolc * fabs(phi0); }
                            }
                            if (okls) { accepted = true; break; }
                            if (ls == 0 && isfinite(tr[1]) && tr[0] >= th0) {
                                // second-order corrections into step buffer 1 (the residual rows S_CR / B_DR / dfr
                                // still hold phase_lin's values at the iterate: nothing since the linearisation
                                // writes them, and this is the iteration's only SOC sequence)
                                __syncthreads();
                                double a_soc = alpha, th_old = th0, th_t = tr[0];
                                bool soc_ok = false;
#pragma unroll 1
                                for (int p = 0; p < 4; ++p) {
                                    if (p > 0 && th_t > 0.99 * th_old) break;
                                    th_old = th_t;
                                    count(sh, ston, OCNT_SOC);
                                    phase_soc_resid(cs, sh, a_soc);
                                    __syncthreads();
                                    // the same matrix (iterate and perturbations) with the SOC right-hand side
                                    if (newton_solve(cs, sh, mu, stt.ph.dx, stt.ph.dc, 1) != F_OK) break;
                                    double rs[5];
                                    if (cs.refine) {
                                        if (!pd_solve(cs, sh, stt.ph, mu, stt.tau, 1, rs)) break;
                                    } else {
                                        phase_recover(cs, sh, mu, stt.ph.dx, stt.tau, 1, rs);
                                        stamp(sh, ston, OPH_REC);
                                    }
                                    a_soc = rs[0];
                                    double t2[3];
                                    phase_trial(cs, sh, mu, a_soc, 1, t2);
                                    stamp(sh, ston, OPH_TRIAL);
                                    th_t = t2[0];
                                    bool ok2 = false;
                                    if (isfinite(t2[1]) && t2[0] <= stt.th_max && !in_filter(sh, R, t2[0], t2[1])) {
                                        if (th0 <= stt.th_min && sw) { ftype = true; ok2 = t2[1] - (phi0 + eta_ph * alpha * Dm) <= tolc * fabs(phi0); }
                                        else { ftype = false; ok2 = t2[0] <= (1.0 - g_th) * th0 || t2[1] - (phi0 - g_ph * th0) <= tolc * fabs(phi0); }
                                    }
                                    if (ok2) { soc_ok = true; az = rs[1]; break; }
                                    if (!isfinite(t2[1])) break;
                                }
                                if (soc_ok) { accepted = true; alpha = a_soc; buf = 1; break; }
                            }
                            if (alpha * 0.5 < amin) break;
                            alpha *= 0.5;
                        }
                        __syncthreads();
                        if (accepted && !ftype && tid == 0) add_filter(sh, R, (1.0 - g_th) * th0, phi0 - g_ph * th0);
                        __syncthreads();
                    }
                    if (!accepted && !R && use_soft && (in_soft ? ++soft_cnt <= MAX_SOFT_RESTO : true)) {
                        // ---- soft restoration step: primal and dual step min(alpha_p, alpha_d), accepted when
                        // acceptable to the filter or when the primal-dual error at mu drops by 0.9999 ----
                        const double as = fmin(rec[0], rec[1]);
                        double tr[3];
                        phase_trial(cs, sh, mu, as, 0, tr);
                        const bool orig_ok = isfinite(tr[1]) && tr[0] <= stt.th_max && !in_filter(sh, 0, tr[0], tr[1]) &&
                                             (tr[0] <= (1.0 - g_th) * th0 || tr[1] - (phi0 - g_ph * th0) <= tolc * fabs(phi0));
                        bool acc_soft = orig_ok;
                        if (!orig_ok && isfinite(tr[1])) {
                            const double pd_cur = red[8] + red[5] + phase_compl(cs, sh, mu).y;
                            phase_snapshot(cs, sh, true);
                            __syncthreads();
                            phase_update(cs, sh, mu, as, as, 0);
                            __syncthreads();
                            double rt[13];
                            phase_lin(cs, sh, rt);
                            const double pd_t = rt[8] + rt[5] + phase_compl(cs, sh, mu).y;
                            const bool fin = isfinite(rt[0]) && isfinite(rt[1]);
                            phase_snapshot(cs, sh, false);
                            __syncthreads();
                            phase_lin(cs, sh, red);  // the restored iterate's linearisation (restoration needs it)
                            pinf = red[1];
                            acc_soft = fin && pd_t <= SOFT_RESTO_FACTOR * pd_cur;
                        }
                        if (acc_soft) {
                            count(sh, ston, OCNT_SOFT);
                            __syncthreads();
                            if (tid == 0) add_filter(sh, 0, (1.0 - g_th) * th0, phi0 - g_ph * th0);
                            __syncthreads();
                            in_soft = orig_ok ? 0 : 1;
                            if (orig_ok) soft_cnt = 0;
                            phase_update(cs, sh, mu, as, as, 0);
                            __syncthreads();
                            break;
                        }
                    }
                    if (!accepted) {
                        if (R && th0 <= 1e-2 * a.tol) {  // failed at an almost feasible point of the restoration
                            status = 3;                    // NLP: IPOPT's RESTORATION_FAILED (oracle: same test)
                            done = true;
                            break;
                        }
                        if (R) {  // restoration of the restoration phase: elastic pairs back to their closed form
                            phase_setpn(cs, sh, mu);
                            __syncthreads();
                            if (tid == 0) sh.nfl[1] = 0;
                            __syncthreads();
                            break;
                        }
                        if (!use_resto) {  // diagnostics only: the round-1 fallback (last trial step, filter reset)
                            __syncthreads();
                            if (tid == 0) sh.nfl[0] = 0;
                            __syncthreads();
                            phase_update(cs, sh, mu, alpha, az, buf);
                            __syncthreads();
                            break;
                        }
                        go_resto = true;
                    } else {
                        phase_update(cs, sh, mu, alpha, az, buf);
                        __syncthreads();
                        stamp(sh, ston, OPH_UPD);
                    }
                }
                if (go_resto) {
                    in_soft = 0;
                    soft_cnt = 0;
                    if (th0 <= 1e-2 * a.tol) {  // almost feasible: acceptable point or Restoration_Failed
                        if (have_acc) { phase_acc(cs, true); status = 1; } else { status = 3; }
                        done = true;
                        break;
                    }
                    __syncthreads();
                    if (tid == 0 && isfinite(phi0)) add_filter(sh, 0, (1.0 - g_th) * th0, phi0 - g_ph * th0);
                    __syncthreads();
                    if (!(stt.th_max > 0)) { stt.th_max = 1e4 * fmax(1.0, th0); stt.th_min = 1e-4 * fmax(1.0, th0); }
                    th_resto0 = th0;
                    const double muR = fmax(stt.mu, pinf);
                    phase_enter_resto(cs, sh, muR);
                    if (use_lsq) ls_multipliers(cs, sh);
                    S0 = stt;
                    S1.mu = muR; S1.tau = fmax(0.99, 1.0 - muR); S1.th_max = S1.th_min = 0.0; S1.acc = 0;
                    S1.ph.reset();
                    if (tid == 0) sh.nfl[1] = 0;
                    __syncthreads();
                    first_resto = 1;
                    resto_iter0 = iter;
                    switched = true;
                    redo = true;
                    break;
                }
            } while (0);
            if (!switched) {
                if (R) S1 = stt;
                else S0 = stt;
            }
            if (done) break;
            if (redo) --iter;
        }
    }
    // ---------------- outputs ----------------
    __syncthreads();
    for (int k = tid; k <= N; k += T) {
#pragma unroll
        for (int i = 0; i < 6; ++i) a.xout[((size_t)c.b * (N + 1) + k) * 6 + i] = c.S(S_X + i, k);
        if (k < N)
#pragma unroll
            for (int i = 0; i < 2; ++i) a.uout[((size_t)c.b * N + k) * 2 + i] = c.S(S_U + i, k);
        if (a.zout) {
            double* z = a.zout + (size_t)c.b * nz + (size_t)k * st;
#pragma unroll
            for (int i = 0; i < 6; ++i) z[i] = c.S(S_X + i, k);
            int o = 6;
            if (k < N) { z[6] = c.S(S_U, k); z[7] = c.S(S_U + 1, k); o = 8; }
            for (int j = 0; j < NBK; ++j) {
                const int ob = j >> 1, bd = j & 1;
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    z[o + ob * 8 + 4 * bd + e] = c.B(B_W + e, j, k);
                    z[o + 8 * a.M + ob * 8 + 4 * bd + e] = c.B(B_W + 4 + e, j, k);
                }
            }
        }
    }
    if (a.itout) {
        // the final primal-dual iterate, for an independent evaluation of IPOPT's optimality error at the GPU's point
        // (tests/test_gpu_obca.py; oracle/c/tt_obca.c pack_iterate has the same layout)
        double* it = a.itout + (size_t)c.b * obca_iterate_len(N, a.M);
        for (int k = tid; k <= N; k += T) {
            double* q = it + 30 * (size_t)k;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                q[i] = c.S(S_X + i, k); q[8 + i] = c.S(S_ZLX + i, k); q[14 + i] = c.S(S_ZUX + i, k);
                q[24 + i] = c.S(S_YC + i, k);
            }
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                q[6 + i] = k < N ? c.S(S_U + i, k) : 0.0;
                q[20 + i] = k < N ? c.S(S_ZLU + i, k) : 0.0;
                q[22 + i] = k < N ? c.S(S_ZUU + i, k) : 0.0;
            }
            double* bq = it + 30 * (size_t)(N + 1) + 32 * (size_t)k * NBK;
            for (int j = 0; j < NBK; ++j) {
                double* qb = bq + 32 * j;
#pragma unroll
                for (int e = 0; e < 8; ++e) { qb[e] = c.B(B_W + e, j, k); qb[8 + e] = c.B(B_ZW + e, j, k); }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    qb[16 + r] = c.B(B_S + r, j, k); qb[20 + r] = c.B(B_VL + r, j, k); qb[24 + r] = c.B(B_VU + r, j, k);
                    qb[28 + r] = c.B(B_YD + r, j, k);
                }
            }
        }
        if (tid == 0) {
            double* f = it + 30 * (size_t)(N + 1) + 32 * (size_t)(N + 1) * NBK;
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                f[i] = plan ? sh.sf[i] : 0.0; f[6 + i] = plan ? sh.vLf[i] : 0.0; f[12 + i] = plan ? sh.vUf[i] : 0.0;
                f[18 + i] = plan ? sh.ydf[i] : 0.0;
            }
        }
    }
    if (tid == 0 && a.board) {  // the helpers stop once every instance has counted itself finished
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        add_rlx(board_line(a, a.B), 1);
    }
    if (tid == 0) {
        // a hand-off timeout overrides whatever the iteration that met it concluded (its passes ran on partial chunks)
        a.status[c.b] = sh.hfail ? kStatusHandoffTimeout : status;
        if (a.iters) a.iters[c.b] = iter;
        if (a.kkt) a.kkt[c.b] = E0;
        if (ston) {
            sh.stamp[OPH_TOTAL] = clock64() - tstart;
            for (int i = 0; i < kObcaPhases; ++i) a.stamps[(size_t)c.b * kObcaPhases + i] = sh.stamp[i];
        }
    }
}

}  // namespace

hipError_t launch_obca(const ObcaArgs& a, hipStream_t stream) {
    if (a.B <= 0) return hipSuccess;
    const size_t need = obca_lds_bytes(a.N), slab = (size_t)kSlab * T * 8;
    const int bytes = (int)(need <= kObcaLdsMax ? (need > slab ? need : slab) : slab);
    // the >64 KB dynamic-LDS opt-in is a per-device function attribute: set it on every such launch
    if (bytes > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)obca_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(obca_kernel, dim3(a.B + (a.board ? a.nhelp : 0)), dim3(T), bytes, stream, a);
    return hipGetLastError();
}

}  // namespace ttmpc
