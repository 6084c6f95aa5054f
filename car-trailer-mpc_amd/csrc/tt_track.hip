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
// exact Lagrangian Hessian) and IPOPT's filter line search with one second-order correction.  The
// Newton system is never assembled: it is the KKT system of an equality-constrained LQ problem,
// solved by a stage-wise Riccati recursion on the FP64 VALU (inertia test = 2x2 Cholesky of each
// reduced input Hessian), O(N) per iteration instead of IPOPT's sparse LDL^T.
//
// Lane mapping (wave-uniform control flow everywhere):
//   * stage-parallel phases (model + Jacobian + curvature + barrier terms + residuals, step bounds,
//     merit trials, multiplier updates): lane k owns stage k (loop k += 64 for N >= 64);
//   * Riccati backward sweep and forward sweep (serial in k): entry-parallel on the VALU, lane 8i + j
//     owns entry (i, j) of the 7x7 affine-augmented blocks (see phase_riccati; the f64 MFMA was
//     measured and is not faster on this dependent chain).
//
// LDS map (doubles).  Head (fixed offsets, immediate addressing): Qw(36) Rw(4) x_init(6) lb(8)
// ub(8) pad(2) dump(32: per-lane sink for branch-free predicated stores), filter, Riccati tiles.  Stage
// k row r at sm[kHead + k*118 + r]; the even stride keeps every record 16-B aligned (see tt_kernel.hpp):
//   0-5 X | 6-7 U | 8-13 Y (eq. multipliers, IPOPT sign) | 14-21 zL | 22-29 zU | 30-37 dX,dU
//   38-43 Y+ | 44-52 dt*J (9 nnz) | 53 zero pad | 54-61 grad F (+ mu dB from ric_prep on) | 62-67 c | 68-79 K
//   80-81 k_ff | 82-102 P_k (upper) | 103 spare | 104-109 p_k | 110-117 dX,dU (soc)
// The reference window (Xref, Uref) is read from HBM (L2-resident, stage-parallel phases only).  Rows with
// a second life (their first owner is dead over that span of the iteration):
//   linearise .. Riccati   30-36 curvature W (7 nnz)          [dX is produced by the forward sweep]
//   linearise .. ric_prep  82-89 Sigma = zL/sL + zU/sU, 90-97 dB = 1/sU - 1/sL   [P_k: Riccati]
//   ric_prep .. Riccati    110-115 diag(Sigma) + diag(W), 116-117 Sigma_u      [dX_soc: SOC]
//                          38-43 b^ = -c_{k+1}                                  [Y+: step]
//   trial .. SOC forward   110-115 c(trial) / c_soc                             [dX_soc: SOC forward]
// 118 rows keep four N = 40 instances (40.8 KB each) on one CU (C3).
//
// Bound pattern: template parameter BM (bit v = finite lower bound on variable v, bit 8+v = finite
// upper bound; v = 0..5 states, 6..7 inputs) so the common patterns compile to straight-line code;
// BM < 0 = pattern read at run time.
#include <math.h>

#include <atomic>

#include "tt_kernel.hpp"
#include "tt_trig.hpp"

namespace ttmpc {
namespace {

constexpr int W = 64;
// A stage row kept in HBM (Ctx::kPG builds): raw buffer load / store through the instance's descriptor (SGPRs) with a
// 32-bit lane offset and a scalar offset -- the access form that needs no 64-bit address registers.
typedef unsigned int u32x2_t __attribute__((ext_vector_type(2)));
struct GRow {
    __amdgpu_buffer_rsrc_t rs;
    unsigned voff, soff;
    __device__ __forceinline__ operator double() const {
        return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, voff, soff, 0));
    }
    __device__ __forceinline__ const GRow& operator=(double v) const {
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2_t, v), rs, voff, soff, 0);
        return *this;
    }
};
constexpr int SR = kRowsPerStage;
constexpr int HEAD = kHead;

// head
constexpr int hQW = 0, hRW = 36, hXI = 40, hLB = 46, hUB = 54;
// dump: sink of branch-free predicated stores, one slot per lane pair (l, l+32: different LDS halves)
constexpr int hDUMP = 64, hFTH = 96, hFPH = 112;  // filter entries (theta, phi), kTrackFilter each
static_assert(hFTH + kTrackFilter == hFPH && hFPH + kTrackFilter <= 128, "filter fits the head");
static_assert(HEAD >= SR, "stage -1 of the Riccati prefetch addresses head words");
// (128..255: the P and transposed-PA tiles of the Riccati sweep, see phase_riccati)
// rows
// every multi-row block starts on an even row (the two odd-sized blocks, dt*J and P, are each followed by a single
// row: the zero pad and the spare), so with the even stride its row pairs are 16-B aligned ds_read_b128 / ds_write_b128
constexpr int rX = 0, rY = 8, rZL = 14, rZU = 22, rDX = 30, rYP = 38, rAJ = 44, PAD = 53, rGF = 54, rCC = 62, rK = 68;
constexpr int rKF = 80, rPS = 82, rPV = 104, rDXS = 110;
static_assert(rDXS + 8 == kRowsPerStage, "stage record");
static_assert(rDXS - rPS == kGlobalRows, "the HBM band of the kPG builds: P, spare, p (overlay Sigma, dB)");
// second lives (see the LDS map): curvature, Sigma, dB from the linearisation to the Riccati sweep; the
// Riccati operands diag(Sigma) + diag(W), Sigma_u and b^ = -c_{k+1} (stage k); the trial residual c
constexpr int rWC = rDX, rSG = rPS, rDB = rPS + 8, rHD = rDXS, rSGU = rDXS + 6, rBH = rYP, rCT = rDXS;
// the shifted input gradient g_u' of the Newton sweep (ric_prep .. Riccati) in the b^4, b^5 rows (see gu_shift)
constexpr int rGU = rBH + 4;

// ---- wave reductions: DPP inside each 16-lane row (xor 1, xor 2, half-mirror, mirror), then the four
// row results by v_readlane into SGPRs.  No LDS; the result is wave-uniform and bitwise identical in
// every lane (the final combine runs on uniform operands).
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
struct OpSum { __device__ double operator()(double a, double b) const { return a + b; } };
struct OpMax { __device__ double operator()(double a, double b) const { return fmax(a, b); } };
struct OpMin { __device__ double operator()(double a, double b) const { return fmin(a, b); } };
template <class Op>
__device__ __forceinline__ double wred(double v, Op op) {
    v = op(v, dppd<0xB1>(v));   // quad_perm [1,0,3,2]
    v = op(v, dppd<0x4E>(v));   // quad_perm [2,3,0,1]
    v = op(v, dppd<0x141>(v));  // row_half_mirror
    v = op(v, dppd<0x140>(v));  // row_mirror
    return op(op(readlane_d(v, 0), readlane_d(v, 16)), op(readlane_d(v, 32), readlane_d(v, 48)));
}
__device__ __forceinline__ double wsum(double v) { return wred(v, OpSum()); }
__device__ __forceinline__ double wmin(double v) { return wred(v, OpMin()); }

// Two or four reductions with one op at once.  The first log2(Q) butterfly stages (quad xor 1, xor 2)
// exchange complementary halves of the value set, so from then on each lane carries a single value: row
// rotations by 4 and 8, then the gfx950 permlane16 / permlane32 swaps across rows and wave halves finish
// every lane.  Value q is read (v_readlane, wave-uniform) from a lane that carries it.  ~40 instructions for
// four reductions instead of ~100 (and 32 fewer v_readlane).
__device__ __forceinline__ void plswap16(double v, double& a, double& b) {
    const long long w = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane16_swap((int)(w & 0xffffffffll), (int)(w & 0xffffffffll), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap((int)(w >> 32), (int)(w >> 32), false, false);
    a = __longlong_as_double(((long long)(int)hi[0] << 32) | (unsigned int)lo[0]);
    b = __longlong_as_double(((long long)(int)hi[1] << 32) | (unsigned int)lo[1]);
}
__device__ __forceinline__ void plswap32(double v, double& a, double& b) {
    const long long w = __double_as_longlong(v);
    const auto lo = __builtin_amdgcn_permlane32_swap((int)(w & 0xffffffffll), (int)(w & 0xffffffffll), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap((int)(w >> 32), (int)(w >> 32), false, false);
    a = __longlong_as_double(((long long)(int)hi[0] << 32) | (unsigned int)lo[0]);
    b = __longlong_as_double(((long long)(int)hi[1] << 32) | (unsigned int)lo[1]);
}
template <class Op>
__device__ __forceinline__ double wtail(double v, Op op) {
    v = op(v, dppd<0x124>(v));  // row_ror:4
    v = op(v, dppd<0x128>(v));  // row_ror:8
    double a, b;
    plswap16(v, a, b);          // rows (0,1), (2,3)
    v = op(a, b);
    plswap32(v, a, b);          // wave halves
    return op(a, b);
}
template <class Op>
__device__ __forceinline__ void wred2(int lane, double& a, double& b, Op op) {
    const bool o = lane & 1;
    double v = op(o ? b : a, dppd<0xB1>(o ? a : b));  // even lanes: a, odd lanes: b
    v = op(v, dppd<0x4E>(v));
    v = wtail(v, op);
    a = readlane_d(v, 0);
    b = readlane_d(v, 1);
}
template <class Op>
__device__ __forceinline__ void wred4(int lane, double& a, double& b, double& c, double& d, Op op) {
    const bool o = lane & 1, t = lane & 2;
    const double k0 = op(o ? c : a, dppd<0xB1>(o ? a : c));  // even lanes: a, c; odd lanes: b, d
    const double k1 = op(o ? d : b, dppd<0xB1>(o ? b : d));
    double v = op(t ? k1 : k0, dppd<0x4E>(t ? k0 : k1));    // lane 4m + (0, 1, 2, 3): a, c, b, d
    v = wtail(v, op);
    a = readlane_d(v, 0);
    c = readlane_d(v, 1);
    b = readlane_d(v, 2);
    d = readlane_d(v, 3);
}

// packed upper-triangle index of a symmetric 6x6
__host__ __device__ constexpr int sym_idx(int i, int j) {
    return i <= j ? i * 6 - (i * (i - 1)) / 2 + (j - i) : j * 6 - (j * (j - 1)) / 2 + (i - j);
}
// nonzeros of dt*J (rows rAJ): 0:D02 1:D05 2:D12 3:D15 4:D24 5:D25 6:D33 7:D34 8:D35  (A = I + dt*J)
__host__ __device__ constexpr int d_idx(int r, int c) {
    return (r == 0 && c == 2) ? 0 : (r == 0 && c == 5) ? 1 : (r == 1 && c == 2) ? 2 : (r == 1 && c == 5) ? 3
         : (r == 2 && c == 4) ? 4 : (r == 2 && c == 5) ? 5 : (r == 3 && c == 3) ? 6 : (r == 3 && c == 4) ? 7
         : (r == 3 && c == 5) ? 8 : -1;
}
// nonzeros of the curvature (rows rWC), symmetric: 0:(2,2) 1:(2,5) 2:(3,3) 3:(3,4) 4:(3,5) 5:(4,4) 6:(4,5)
__host__ __device__ constexpr int w_idx(int i, int j) {
    return i > j ? w_idx(j, i)
         : (i == 2 && j == 2) ? 0 : (i == 2 && j == 5) ? 1 : (i == 3 && j == 3) ? 2 : (i == 3 && j == 4) ? 3
         : (i == 3 && j == 5) ? 4 : (i == 4 && j == 4) ? 5 : (i == 4 && j == 5) ? 6 : -1;
}
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

// 1/x by v_rcp_f64 + two Newton steps (within 1 ulp of IEEE division; x finite, nonzero, normal)
__device__ __forceinline__ double frcp(double x) {
    double r = __builtin_amdgcn_rcp(x);
    double e = fma(-x, r, 1.0);
    r = fma(r, e, r);
    e = fma(-x, r, 1.0);
    return fma(r, e, r);
}

// b if p else a, for two elements of a register array: the empty asm makes both operands opaque values, so
// the compiler cannot turn the select of two array loads into one load at a lane-dependent address (which
// would send the whole array to scratch)
__device__ __forceinline__ double psel(bool p, double a, double b) {
    asm("" : "+v"(a), "+v"(b));
    return p ? b : a;
}

// sum of logs as log(prod of mantissas) + (sum of exponents) ln 2: one log per stage instead of 16
struct LogSum {
    double m = 1.0;
    int e = 0;
    __device__ __forceinline__ void add(double s) {
        int ex;
        m *= frexp(s, &ex);
        e += ex;
    }
    __device__ __forceinline__ double value() const { return log(m) + (double)e * 0.69314718055994530942; }
};

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
#define COUNT(ph) (++stamps.acc[ph])
#define SUBSTAMP(c, n) ((c).st->mark(PH_X0 + (n)))
#else
#define STAMP(ph) ((void)0)
#define COUNT(ph) ((void)0)
#define SUBSTAMP(c, n) ((void)0)
#endif

// Armijo test with IPOPT's round-off allowance (Compare_le: lhs - rhs <= 10 eps |reference|)
__device__ __forceinline__ bool armijo(double trial, double ref, double alpha, double D) {
    return trial - (ref + 1e-4 * alpha * D) <= 10.0 * 2.220446049250313e-16 * fabs(ref);
}

// IPOPT filter constants (gamma_theta, gamma_phi, s_phi, s_theta; delta = 1, eta_phi = 1e-4)
constexpr double kGTh = 1e-5, kGPh = 1e-8, kSPh = 2.3, kSTh = 1.1;

// fraction-to-boundary: largest a with s + a*d >= (1-tau) s  (divide only when the bound is active)
__device__ __forceinline__ void ftb(double s, double d, double tau, double& a) {
    if (d < 0.0 && tau * s < -a * d) a = -tau * s / d;
}

// Per-wave solver context: a handful of scalars; the data lives in LDS
template <int BM>
struct Ctx {
    double* sm;
    int N, lane;
    double dt, iL1, iL2, Mh;
    double mu, tau;
    // bit 18: the build keeps the stage rows rPS .. rDXS-1 (P, spare, p; their overlay Sigma, dB) in HBM (TrackArgs::prow)
    // and the LDS record shrinks by those kGlobalRows rows: rows from rDXS on sit kGlobalRows lower (the N = 50 build:
    // 38.8 KB per instance, four per CU instead of three).  Rows of that band are reached through g() only; r() serves
    // every other row, rl() an LDS row already mapped (lrow) -- in the other builds all three are the same LDS access.
    static constexpr bool kPG = BM >= 0 && ((BM >> 18) & 1);
    static constexpr int kSR = kPG ? SR - kGlobalRows : SR;
    __amdgpu_buffer_rsrc_t prs;  // this instance's HBM rows (kPG builds): a buffer descriptor in SGPRs
    __device__ __forceinline__ static int lrow(int row) { return kPG && row >= rDXS ? row - kGlobalRows : row; }
    __device__ __forceinline__ double& r(int row, int k) const { return sm[HEAD + k * kSR + lrow(row)]; }
    __device__ __forceinline__ double& rl(int lds_row, int k) const { return sm[HEAD + k * kSR + lds_row]; }
    __device__ __forceinline__ double& h(int i) const { return sm[i]; }
    // g: any stage k (the stage-parallel passes: k = the lane's stage); gu: a wave-uniform stage (the serial sweep's),
    // whose offset goes to the descriptor's scalar offset so no per-stage address is formed in VGPRs
    __device__ __forceinline__ decltype(auto) g(int row, int k) const {
        if constexpr (kPG) return GRow{prs, (unsigned)(k * kGlobalRows + (row - rPS)) * 8u, 0u};
        else return static_cast<double&>(sm[HEAD + k * SR + row]);
    }
    __device__ __forceinline__ decltype(auto) gu(int row, int k) const {
        if constexpr (kPG) return GRow{prs, (unsigned)(row - rPS) * 8u, (unsigned)(k * kGlobalRows) * 8u};
        else return static_cast<double&>(sm[HEAD + k * SR + row]);
    }
    // bit 16 of a specialised bound pattern: Q and R are diagonal (the reference's Q = I, R = 10 I)
    static constexpr bool kDiag = BM >= 0 && ((BM >> 16) & 1);
    // bit 17: the two-waves-per-SIMD build.  The one-wave builds issue every LDS read of a stage-parallel pass before its
    // stores (kLF, "loads first": with one wave per SIMD nothing hides a read queued behind a store); the two-wave build
    // keeps the per-variable order, whose shorter live ranges suit its 256-register budget.  Same arithmetic either way.
    static constexpr bool kLF = !(BM >= 0 && ((BM >> 17) & 1));
    __device__ __forceinline__ bool hl(int v) const {
        if constexpr (BM >= 0) return (BM >> v) & 1;
        else return sm[hLB + v] > -INFINITY;
    }
    __device__ __forceinline__ bool hu(int v) const {
        if constexpr (BM >= 0) return (BM >> (8 + v)) & 1;
        else return sm[hUB + v] < INFINITY;
    }
    __device__ __forceinline__ double lb(int v) const { return sm[hLB + v]; }
    __device__ __forceinline__ double ub(int v) const { return sm[hUB + v]; }
    // barrier gradient component: grad F + mu * (1/sU - 1/sL)
    // Lane pairs (stage-unrolled builds, N < 32, bound pattern symmetric in variable pairs (2t, 2t+1)):
    // stage k is owned by lanes 2k and 2k+1, which split its per-variable work (variables 2t + part) and its
    // six dynamics / multiplier rows (2q + part), halving the dependent chain of the stage-parallel phases.
    static constexpr bool kPairSym = BM >= 0 && (((BM ^ (BM >> 1)) & 0x5555) == 0);
    bool pair;
    __device__ __forceinline__ int k0() const { return pair ? (lane >> 1) : lane; }
    __device__ __forceinline__ int kst() const { return pair ? (W >> 1) : W; }
    __device__ __forceinline__ int part() const { return pair ? (lane & 1) : 0; }
    // barrier gradient grad F + mu dB: folded into the rGF rows by phase_ric_prep (valid from there on)
    __device__ __forceinline__ double gr(int v, int k) const { return r(rGF + v, k); }
    // the instance's reference window in HBM: Xref [N+1][6], Uref [N][2].  regref: one stage per lane
    // (stage-unrolled builds, N < 64), so lane k keeps its stage's 8 reference values in registers for the
    // whole solve (the stage-parallel phases only ever ask for k = lane); else every read goes to HBM / L2.
    const double* gxr;
    const double* gur;
    bool regref;
    double rc0, rc1, rc2, rc3, rc4, rc5, rc6, rc7;  // scalars (an array member would live in scratch)
    __device__ __forceinline__ double rcv(int i) const {
        return i == 0 ? rc0 : i == 1 ? rc1 : i == 2 ? rc2 : i == 3 ? rc3 : i == 4 ? rc4 : i == 5 ? rc5 : i == 6 ? rc6 : rc7;
    }
    __device__ __forceinline__ double xr(int i, int k) const { return regref ? rcv(i) : gxr[k * 6 + i]; }
    __device__ __forceinline__ double ur(int i, int k) const { return regref ? rcv(6 + i) : gur[k * 2 + i]; }
    // Trig cache (regref builds): the trial point's sin/cos of theta, psi, phi, kept by the lane of its stage.
    // The accepted step lands exactly on the last trial point (update computes x + alpha dz with the same
    // expression), so the next linearisation reuses them instead of three more FP64 sincos.
    mutable double ts0, tc0, ts1, tc1, ts2, tc2;
    mutable double t_alpha;
    mutable int t_dz, t_ok;
#ifdef TT_STAMPS
    struct Stamps* st;  // diagnostic build: sub-phase clocks (SUBSTAMP)
#endif
};

// sin / cos of theta, psi, phi of a stage.  Lane pairs: the two lanes evaluate theta (part 0) and phi
// (part 1) in the same instruction stream and swap the results with one DPP quad_perm [1,0,3,2], so the
// stage pays two sincos of latency instead of three; the sincos are the library's algorithm as straight-line code
// (tt_trig.hpp), so that they interleave.
template <int BM>
__device__ __forceinline__ void stage_trig(const Ctx<BM>& c, const double* x, double& sth, double& cth, double& sps,
                                           double& cps, double& sph, double& cph) {
    if (c.pair) {
        const bool p = c.part() != 0;
        double s1, c1;
        sincos2(psel(p, x[2], x[4]), s1, c1, x[3], sps, cps);
        const double os = dppd<0xB1>(s1), oc = dppd<0xB1>(c1);
        sth = p ? os : s1; cth = p ? oc : c1;
        sph = p ? s1 : os; cph = p ? c1 : oc;
    } else {
        sincos3(x[2], sth, cth, x[3], sps, cps, x[4], sph, cph);
    }
}

// ---------------- model: truck_trailer_model.py:8-24 ----------------
template <int BM>
__device__ __forceinline__ void model_f(const Ctx<BM>& c, const double* x, const double* u, double* fo) {
    double sth, cth, sps, cps, sph, cph;
    stage_trig(c, x, sth, cth, sps, cps, sph, cph);
    if (c.regref) { c.ts0 = sth; c.tc0 = cth; c.ts1 = sps; c.tc1 = cps; c.ts2 = sph; c.tc2 = cph; }
    const double t = sph * frcp(cph), v = x[5];
    fo[0] = v * cth;
    fo[1] = v * sth;
    fo[2] = v * t * c.iL1;
    fo[3] = -v * t * c.iL1 * (1.0 + c.Mh * c.iL2 * cps) - v * sps * c.iL2;
    fo[4] = u[1];
    fo[5] = u[0];
}

// f, dt*J and the curvature -dt * sum_i y_i d2f_i/dx2 in one pass (5 transcendentals)
template <int BM>
__device__ __forceinline__ void model_lin(const Ctx<BM>& c, const double* x, const double* u, const double* y,
                                          double* fo, double* aj, double* wc) {
    double sth, cth, sps, cps, sph, cph;
    if (c.t_ok) {
        sth = c.ts0; cth = c.tc0; sps = c.ts1; cps = c.tc1; sph = c.ts2; cph = c.tc2;
    } else {
        stage_trig(c, x, sth, cth, sps, cps, sph, cph);
    }
    const double v = x[5], dt = c.dt, Mh = c.Mh, iL1 = c.iL1, iL2 = c.iL2, iL1L2 = iL1 * iL2;
    const double ic = frcp(cph), t = sph * ic, c2 = ic * ic;
    const double k = 1.0 + Mh * iL2 * cps;
    fo[0] = v * cth;
    fo[1] = v * sth;
    fo[2] = v * t * iL1;
    fo[3] = -v * t * iL1 * k - v * sps * iL2;
    fo[4] = u[1];
    fo[5] = u[0];
    aj[0] = dt * (-v * sth);
    aj[1] = dt * cth;
    aj[2] = dt * (v * cth);
    aj[3] = dt * sth;
    aj[4] = dt * (v * c2 * iL1);
    aj[5] = dt * (t * iL1);
    aj[6] = dt * (v * t * Mh * sps * iL1L2 - v * cps * iL2);
    aj[7] = dt * (-v * c2 * iL1 * k);
    aj[8] = dt * (-t * iL1 * k - sps * iL2);
    const double s = -dt;
    wc[0] = s * (y[0] * (-v * cth) + y[1] * (-v * sth));
    wc[1] = s * (y[0] * (-sth) + y[1] * cth);
    wc[2] = s * (y[3] * (v * t * Mh * cps * iL1L2 + v * sps * iL2));
    wc[3] = s * (y[3] * (v * c2 * Mh * sps * iL1L2));
    wc[4] = s * (y[3] * (t * Mh * sps * iL1L2 - cps * iL2));
    wc[5] = s * (y[2] * (2.0 * v * t * c2 * iL1) + y[3] * (-2.0 * v * t * c2 * k * iL1));
    wc[6] = s * (y[2] * (c2 * iL1) + y[3] * (-c2 * k * iL1));
}

struct Lin {
    double dinf, pinf, sy, sz;   // optimality-error pieces
    double zmx, zmn;             // max / min of z*s over the bounds (-inf / +inf without bounds)
    double cost, logs, th;       // merit pieces at the current point: F, sum log s, ||c||_1
    // complementarity errors max |z s| and max |z s - mu| from the extremes of z s, exactly (rounding is
    // monotone: max_i fl(a_i - mu) = fl(max_i a_i - mu)), so a barrier update needs no pass over the stages
    __device__ __forceinline__ double c0() const { return zmx >= zmn ? fmax(fabs(zmx), fabs(zmn)) : 0.0; }
    __device__ __forceinline__ double cmu(double mu) const { return zmx >= zmn ? fmax(zmx - mu, mu - zmn) : 0.0; }
};

// ============ linearise at the current point (stage-parallel) ============
// f, dt*J, curvature, constraint residual c, grad F, Sigma, dB, and the optimality / merit pieces.
template <int BM>
__device__ __forceinline__ Lin phase_linearize(const Ctx<BM>& c) {
    const int N = c.N;
    double dinf = 0.0, pinf = 0.0, zmx = -INFINITY, zmn = INFINITY, sy = 0.0, sz = 0.0, cost = 0.0, th = 0.0,
           logs = 0.0;
    bool fin = true, bad = false;
    if constexpr (Ctx<BM>::kLF) {
    if (c.pair) {
        // lane pairs: both lanes linearise the dynamics (the curvature and dt*J feed both lanes' gradient
        // rows), each writes and accounts for its own rows (2q + part) and its own variables (2t + part)
        const int p = c.part();
        for (int k = c.k0(); k <= N; k += c.kst()) {
            const bool st = k < N;
            double x[6], u[2] = {0.0, 0.0}, yk[6], y1[6] = {0, 0, 0, 0, 0, 0}, aj[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            // Every LDS read of the stage is issued before the pass's first store: a read queued behind a store waits
            // for it, and the per-variable load -> compute -> store order made the variable loop a chain of twelve LDS
            // round trips (SUBSTAMP census, profiles/r05/track_ab/).  The arithmetic is unchanged (bitwise).
            double zl[4] = {0, 0, 0, 0}, zu[4] = {0, 0, 0, 0}, lbv[4] = {0, 0, 0, 0}, ubv[4] = {0, 0, 0, 0};
            double qw[3], xi0[3] = {0, 0, 0}, xn[3] = {0, 0, 0};
#pragma unroll
            for (int i = 0; i < 6; ++i) { x[i] = c.r(rX + i, k); yk[i] = c.r(rY + i, k); }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int vb = 2 * t, v = vb + p;
                if (vb >= 6 && k == N) break;
                if (c.hl(vb)) { zl[t] = c.r(rZL + v, k); lbv[t] = c.lb(v); }
                if (c.hu(vb)) { zu[t] = c.r(rZU + v, k); ubv[t] = c.ub(v); }
            }
#pragma unroll
            for (int t = 0; t < 3; ++t) qw[t] = c.h(hQW + (2 * t + p) * 7);
            const double rw = c.h(hRW + p * 3);
            if (k == 0)
#pragma unroll
                for (int q = 0; q < 3; ++q) xi0[q] = c.h(hXI + 2 * q + p);
            if (st) {
                u[0] = c.r(rX + 6, k);
                u[1] = c.r(rX + 7, k);
#pragma unroll
                for (int i = 0; i < 6; ++i) y1[i] = c.r(rY + i, k + 1);
#pragma unroll
                for (int q = 0; q < 3; ++q) xn[q] = c.r(rX + 2 * q + p, k + 1);
            }
#pragma unroll
            for (int q = 0; q < 3; ++q) sy += fabs(psel(p, yk[2 * q], yk[2 * q + 1]));
            double cc0[3] = {0, 0, 0}, cc1[3] = {0, 0, 0}, wc[7];
            if (k == 0) {
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const double cc = psel(p, x[2 * q], x[2 * q + 1]) - xi0[q];
                    cc0[q] = cc;
                    pinf = fmax(pinf, fabs(cc));
                    th += fabs(cc);
                }
            }
            if (st) {
                double fo[6];
                model_lin(c, x, u, y1, fo, aj, wc);
                SUBSTAMP(c, 5);
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const double cc = xn[q] - (psel(p, x[2 * q], x[2 * q + 1]) + c.dt * psel(p, fo[2 * q], fo[2 * q + 1]));
                    cc1[q] = cc;
                    pinf = fmax(pinf, fabs(cc));
                    th += fabs(cc);
                }
            }
            LogSum ls;
            double gfv[4] = {0, 0, 0, 0}, sgv[4] = {0, 0, 0, 0}, dbv[4] = {0, 0, 0, 0};
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int vb = 2 * t, v = vb + p;
                if (vb >= 6 && k == N) break;
                double gf, g, xv;
                if (vb < 6) {
                    const double dxr = psel(p, x[vb], x[vb + 1]) - c.xr(v, k);
                    gf = qw[t] * dxr;
                    cost += dxr * gf;
                    gf *= 2.0;
                    g = gf + psel(p, yk[vb], yk[vb + 1]);
                    if (k < N) g -= psel(p, y1[vb], y1[vb + 1]) + (p ? colJ(aj, vb + 1, y1, 1) : colJ(aj, vb, y1, 1));
                    xv = psel(p, x[vb], x[vb + 1]);
                } else {
                    const double du = psel(p, u[0], u[1]) - c.ur(p, k);
                    gf = rw * du;
                    cost += du * gf;
                    gf *= 2.0;
                    g = gf - c.dt * psel(p, y1[5], y1[4]);
                    xv = psel(p, u[0], u[1]);
                }
                gfv[t] = gf;
                double sg = 0.0, db = 0.0;
                if (c.hl(vb)) {
                    const double sl = xv - lbv[t], rs = frcp(sl);
                    g -= zl[t];
                    zmx = fmax(zmx, zl[t] * sl);
                    zmn = fmin(zmn, zl[t] * sl);
                    sz += zl[t];
                    sg += zl[t] * rs;
                    db -= rs;
                    if (sl <= 0.0) bad = true; else ls.add(sl);
                }
                if (c.hu(vb)) {
                    const double su = ubv[t] - xv, rs = frcp(su);
                    g += zu[t];
                    zmx = fmax(zmx, zu[t] * su);
                    zmn = fmin(zmn, zu[t] * su);
                    sz += zu[t];
                    sg += zu[t] * rs;
                    db += rs;
                    if (su <= 0.0) bad = true; else ls.add(su);
                }
                sgv[t] = sg;
                dbv[t] = db;
                if (!isfinite(g)) fin = false;
                dinf = fmax(dinf, fabs(g));
            }
            // ---- the stage's stores, after every read ----
            if (k == 0)
#pragma unroll
                for (int q = 0; q < 3; ++q) c.r(rCC + 2 * q + p, 0) = cc0[q];
            if (st) {
#pragma unroll
                for (int q = 0; q < 5; ++q) {
                    if (q == 4 && p) break;
                    c.r(rAJ + 2 * q + p, k) = psel(p, aj[2 * q], aj[2 * q + 1]);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (q == 3 && p) break;
                    c.r(rWC + 2 * q + p, k) = psel(p, wc[2 * q], wc[2 * q + 1]);
                }
#pragma unroll
                for (int q = 0; q < 3; ++q) c.r(rCC + 2 * q + p, k + 1) = cc1[q];
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int v = 2 * t + p;
                if (2 * t >= 6 && k == N) break;
                c.r(rGF + v, k) = gfv[t];
                c.g(rSG + v, k) = sgv[t];
                c.g(rDB + v, k) = dbv[t];
            }
            SUBSTAMP(c, 6);
            logs += ls.value();
        }
    } else
    for (int k = c.lane; k <= N; k += W) {
        // as in the lane-pair path: every LDS read of the stage, then the arithmetic, then the stores
        const bool st = k < N;
        double x[6], u[2] = {0.0, 0.0}, yk[6], y1[6] = {0, 0, 0, 0, 0, 0}, aj[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
        double xn[6] = {0, 0, 0, 0, 0, 0}, cc0[6] = {0, 0, 0, 0, 0, 0}, cc1[6] = {0, 0, 0, 0, 0, 0}, wc[7];
#pragma unroll
        for (int i = 0; i < 6; ++i) { x[i] = c.r(rX + i, k); yk[i] = c.r(rY + i, k); sy += fabs(yk[i]); }
        if (st) {
            u[0] = c.r(rX + 6, k);
            u[1] = c.r(rX + 7, k);
#pragma unroll
            for (int i = 0; i < 6; ++i) { y1[i] = c.r(rY + i, k + 1); xn[i] = c.r(rX + i, k + 1); }
        }
        if (k == 0) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double cc = x[i] - c.h(hXI + i);
                cc0[i] = cc;
                pinf = fmax(pinf, fabs(cc));
                th += fabs(cc);
            }
        }
        if (st) {
            double fo[6];
            model_lin(c, x, u, y1, fo, aj, wc);
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double cc = xn[i] - (x[i] + c.dt * fo[i]);
                cc1[i] = cc;
                pinf = fmax(pinf, fabs(cc));
                th += fabs(cc);
            }
        }
        // tracking cost and its gradient (no 1/2: F = dx' Qw dx + du' Rw du, grad = 2 Qw dx)
        double dxr[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) dxr[i] = x[i] - c.xr(i, k);
        double du0 = 0.0, du1 = 0.0;
        if (st) { du0 = u[0] - c.ur(0, k); du1 = u[1] - c.ur(1, k); }
        LogSum ls;
        double gfv[8] = {0, 0, 0, 0, 0, 0, 0, 0}, sgv[8] = {0, 0, 0, 0, 0, 0, 0, 0}, dbv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            if (v >= 6 && k == N) break;
            double gf;
            if (v < 6) {
                if constexpr (Ctx<BM>::kDiag) {
                    gf = c.h(hQW + v * 7) * dxr[v];
                } else {
                    gf = 0.0;
#pragma unroll
                    for (int j = 0; j < 6; ++j) gf += c.h(hQW + v * 6 + j) * dxr[j];
                }
                cost += dxr[v] * gf;
                gf *= 2.0;
            } else {
                const int rr = v - 6;
                if constexpr (Ctx<BM>::kDiag)
                    gf = c.h(hRW + rr * 3) * (rr == 0 ? du0 : du1);
                else
                    gf = c.h(hRW + rr * 2) * du0 + c.h(hRW + rr * 2 + 1) * du1;
                cost += (rr == 0 ? du0 : du1) * gf;
                gf *= 2.0;
            }
            gfv[v] = gf;
            // d/dz of the Lagrangian: grad F + y_k - A'y_{k+1} - zL + zU
            double g = gf;
            if (v < 6) {
                g += yk[v];
                if (k < N) g -= y1[v] + colJ(aj, v, y1, 1);
            } else {
                g -= c.dt * y1[v == 6 ? 5 : 4];
            }
            const double xv = v < 6 ? x[v] : u[v - 6];
            double sg = 0.0, db = 0.0;
            if (c.hl(v)) {
                const double zl = c.r(rZL + v, k), s = xv - c.lb(v), rs = frcp(s);
                g -= zl;
                zmx = fmax(zmx, zl * s);
                zmn = fmin(zmn, zl * s);
                sz += zl;
                sg += zl * rs;
                db -= rs;
                if (s <= 0.0) bad = true; else ls.add(s);
            }
            if (c.hu(v)) {
                const double zu = c.r(rZU + v, k), s = c.ub(v) - xv, rs = frcp(s);
                g += zu;
                zmx = fmax(zmx, zu * s);
                zmn = fmin(zmn, zu * s);
                sz += zu;
                sg += zu * rs;
                db += rs;
                if (s <= 0.0) bad = true; else ls.add(s);
            }
            sgv[v] = sg;
            dbv[v] = db;
            if (!isfinite(g)) fin = false;
            dinf = fmax(dinf, fabs(g));
        }
        logs += ls.value();
        // ---- the stage's stores, after every read ----
        if (k == 0)
#pragma unroll
            for (int i = 0; i < 6; ++i) c.r(rCC + i, 0) = cc0[i];
        if (st) {
#pragma unroll
            for (int i = 0; i < 9; ++i) c.r(rAJ + i, k) = aj[i];
#pragma unroll
            for (int i = 0; i < 7; ++i) c.r(rWC + i, k) = wc[i];
#pragma unroll
            for (int i = 0; i < 6; ++i) c.r(rCC + i, k + 1) = cc1[i];
        }
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            if (v >= 6 && k == N) break;
            c.r(rGF + v, k) = gfv[v];
            c.g(rSG + v, k) = sgv[v];
            c.g(rDB + v, k) = dbv[v];
        }
    }
    } else {
    // the two-wave build: the other wave on the SIMD hides the LDS round trips, and the load-first order's
    // longer live ranges cost it more than they save (C5, profiles/r05/track_ab/)
    if (c.pair) {
        // lane pairs: both lanes linearise the dynamics (the curvature and dt*J feed both lanes' gradient
        // rows), each writes and accounts for its own rows (2q + part) and its own variables (2t + part)
        const int p = c.part();
        for (int k = c.k0(); k <= N; k += c.kst()) {
            double x[6], u[2] = {0.0, 0.0}, yk[6], y1[6] = {0, 0, 0, 0, 0, 0}, aj[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
            for (int i = 0; i < 6; ++i) { x[i] = c.r(rX + i, k); yk[i] = c.r(rY + i, k); }
#pragma unroll
            for (int q = 0; q < 3; ++q) sy += fabs(psel(p, yk[2 * q], yk[2 * q + 1]));
            if (k == 0) {
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const int i = 2 * q + p;
                    const double cc = psel(p, x[2 * q], x[2 * q + 1]) - c.h(hXI + i);
                    c.r(rCC + i, 0) = cc;
                    pinf = fmax(pinf, fabs(cc));
                    th += fabs(cc);
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
                for (int q = 0; q < 5; ++q) {
                    if (q == 4 && p) break;
                    c.r(rAJ + 2 * q + p, k) = psel(p, aj[2 * q], aj[2 * q + 1]);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (q == 3 && p) break;
                    c.r(rWC + 2 * q + p, k) = psel(p, wc[2 * q], wc[2 * q + 1]);
                }
#pragma unroll
                for (int q = 0; q < 3; ++q) {
                    const int i = 2 * q + p;
                    const double cc = c.r(rX + i, k + 1) - (psel(p, x[2 * q], x[2 * q + 1]) + c.dt * psel(p, fo[2 * q], fo[2 * q + 1]));
                    c.r(rCC + i, k + 1) = cc;
                    pinf = fmax(pinf, fabs(cc));
                    th += fabs(cc);
                }
            }
            LogSum ls;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const int vb = 2 * t, v = vb + p;
                if (vb >= 6 && k == N) break;
                double gf, g, xv;
                if (vb < 6) {
                    const double dxr = psel(p, x[vb], x[vb + 1]) - c.xr(v, k);
                    gf = c.h(hQW + v * 7) * dxr;
                    cost += dxr * gf;
                    gf *= 2.0;
                    g = gf + psel(p, yk[vb], yk[vb + 1]);
                    if (k < N) g -= psel(p, y1[vb], y1[vb + 1]) + (p ? colJ(aj, vb + 1, y1, 1) : colJ(aj, vb, y1, 1));
                    xv = psel(p, x[vb], x[vb + 1]);
                } else {
                    const double du = psel(p, u[0], u[1]) - c.ur(p, k);
                    gf = c.h(hRW + p * 3) * du;
                    cost += du * gf;
                    gf *= 2.0;
                    g = gf - c.dt * psel(p, y1[5], y1[4]);
                    xv = psel(p, u[0], u[1]);
                }
                c.r(rGF + v, k) = gf;
                double sg = 0.0, db = 0.0;
                if (c.hl(vb)) {
                    const double zl = c.r(rZL + v, k), sl = xv - c.lb(v), rs = frcp(sl);
                    g -= zl;
                    zmx = fmax(zmx, zl * sl);
                    zmn = fmin(zmn, zl * sl);
                    sz += zl;
                    sg += zl * rs;
                    db -= rs;
                    if (sl <= 0.0) bad = true; else ls.add(sl);
                }
                if (c.hu(vb)) {
                    const double zu = c.r(rZU + v, k), su = c.ub(v) - xv, rs = frcp(su);
                    g += zu;
                    zmx = fmax(zmx, zu * su);
                    zmn = fmin(zmn, zu * su);
                    sz += zu;
                    sg += zu * rs;
                    db += rs;
                    if (su <= 0.0) bad = true; else ls.add(su);
                }
                c.g(rSG + v, k) = sg;
                c.g(rDB + v, k) = db;
                if (!isfinite(g)) fin = false;
                dinf = fmax(dinf, fabs(g));
            }
            logs += ls.value();
        }
    } else
    for (int k = c.lane; k <= N; k += W) {
        double x[6], u[2] = {0.0, 0.0}, yk[6], y1[6] = {0, 0, 0, 0, 0, 0}, aj[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
        for (int i = 0; i < 6; ++i) { x[i] = c.r(rX + i, k); yk[i] = c.r(rY + i, k); sy += fabs(yk[i]); }
        if (k == 0) {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                const double cc = x[i] - c.h(hXI + i);
                c.r(rCC + i, 0) = cc;
                pinf = fmax(pinf, fabs(cc));
                th += fabs(cc);
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
                th += fabs(cc);
            }
        }
        // tracking cost and its gradient (no 1/2: F = dx' Qw dx + du' Rw du, grad = 2 Qw dx)
        double dxr[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) dxr[i] = x[i] - c.xr(i, k);
        double du0 = 0.0, du1 = 0.0;
        if (k < N) { du0 = u[0] - c.ur(0, k); du1 = u[1] - c.ur(1, k); }
        LogSum ls;
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            if (v >= 6 && k == N) break;
            double gf;
            if (v < 6) {
                if constexpr (Ctx<BM>::kDiag) {
                    gf = c.h(hQW + v * 7) * dxr[v];
                } else {
                    gf = 0.0;
#pragma unroll
                    for (int j = 0; j < 6; ++j) gf += c.h(hQW + v * 6 + j) * dxr[j];
                }
                cost += dxr[v] * gf;
                gf *= 2.0;
            } else {
                const int rr = v - 6;
                if constexpr (Ctx<BM>::kDiag)
                    gf = c.h(hRW + rr * 3) * (rr == 0 ? du0 : du1);
                else
                    gf = c.h(hRW + rr * 2) * du0 + c.h(hRW + rr * 2 + 1) * du1;
                cost += (rr == 0 ? du0 : du1) * gf;
                gf *= 2.0;
            }
            c.r(rGF + v, k) = gf;
            // d/dz of the Lagrangian: grad F + y_k - A'y_{k+1} - zL + zU
            double g = gf;
            if (v < 6) {
                g += yk[v];
                if (k < N) g -= y1[v] + colJ(aj, v, y1, 1);
            } else {
                g -= c.dt * y1[v == 6 ? 5 : 4];
            }
            const double xv = v < 6 ? x[v] : u[v - 6];
            double sg = 0.0, db = 0.0;
            if (c.hl(v)) {
                const double zl = c.r(rZL + v, k), s = xv - c.lb(v), rs = frcp(s);
                g -= zl;
                zmx = fmax(zmx, zl * s);
                zmn = fmin(zmn, zl * s);
                sz += zl;
                sg += zl * rs;
                db -= rs;
                if (s <= 0.0) bad = true; else ls.add(s);
            }
            if (c.hu(v)) {
                const double zu = c.r(rZU + v, k), s = c.ub(v) - xv, rs = frcp(s);
                g += zu;
                zmx = fmax(zmx, zu * s);
                zmn = fmin(zmn, zu * s);
                sz += zu;
                sg += zu * rs;
                db += rs;
                if (s <= 0.0) bad = true; else ls.add(s);
            }
            c.g(rSG + v, k) = sg;
            c.g(rDB + v, k) = db;
            if (!isfinite(g)) fin = false;
            dinf = fmax(dinf, fabs(g));
        }
        logs += ls.value();
    }
    }
    Lin e;
    e.dinf = (fin && !bad) ? dinf : INFINITY;
    e.pinf = pinf;
    e.zmx = zmx;
    double nzmn = -zmn;
    wred4(c.lane, e.dinf, e.pinf, e.zmx, nzmn, OpMax());
    e.zmn = -nzmn;
    e.sy = sy;
    e.sz = sz;
    e.cost = cost;
    e.logs = logs;
    wred4(c.lane, e.sy, e.sz, e.cost, e.logs, OpSum());
    e.th = wsum(th);
    __syncthreads();
    return e;
}

// ============ Riccati recursion, entry-parallel on the VALU ============
// Affine augmentation x^ = [dx; 1] turns the value function, dynamics and feed-forward into 7x7
// blocks: A^ = [[A, b],[0, 1]] = I + D (b = -c_{k+1}), H^ = [[H_xx, g_x],[g_x', 0]], B^ = [B; 0]
// (B[5][0] = B[4][1] = dt), S^ = [0, g_u].  Per stage (k = N-1 .. 0):
//   PA = P^ A^ = P^ + P^ D,   F = A^' PA + H^ = PA + D' PA + H^,   G = B^' PA + S^ (rows 5, 4 of PA),
//   H_uu = 2Rw + Sig_u + dt^2 P[{5,4},{5,4}],  M = H_uu^-1 G,  P^_k = F - G' M,  K^ = -M.
// Lane 8i + j owns entry (i, j) of every 8x8 (padded) block.  The only cross-lane traffic is row i of
// P^ (read from the P tile in LDS, written by the previous stage) and column j of PA (written
// transposed into the PA tile, so both are contiguous b128 reads).  The 16x16 f64 MFMA was measured
// at ~185 cycles per srcC-chained link on gfx950 and runs no faster than the VALU for f64, so the
// whole recursion stays on the VALU with ~300 cycles of dependent latency per stage.
constexpr int hPF = 128, hPT = 192;  // P tile (i, j) and transposed PA tile (j, i), 64 doubles each, rows 4..7 XOR-swizzled

// branch-free predicated LDS store: invalid lanes write their own dump slot
template <int BM>
__device__ __forceinline__ void pstore(const Ctx<BM>& c, bool valid, int row, int k, double v) {
    c.sm[valid ? HEAD + k * Ctx<BM>::kSR + row : hDUMP + (c.lane & 31)] = v;
}
// exec-masked LDS store: with k a compile-time stage (unrolled sweeps) the address is the lane's row
// register plus an immediate offset, so the store costs no VALU address arithmetic at all
template <int BM>
__device__ __forceinline__ void mstore(const Ctx<BM>& c, bool valid, int row, int k, double v) {
    if (valid) c.sm[HEAD + k * Ctx<BM>::kSR + row] = v;
}

// The input shift of the Newton sweep (round 6).  B = dt [e5 e4]: rows 4, 5 of the dynamics (phi, v)
// are pure integrators of the inputs, so the residual's rows 4, 5 can be carried by the input instead of the affine
// column: du' = du + s with s = (b^5, b^4) / dt gives dx_{k+1} = A dx_k + B du' + (b^0..b^3, 0, 0).  Rows 4, 5 of
// dt*J are zero as well, so every entry of PA = P A^ and of F = A^' PA + H^ becomes a four-term sum (round 5: six, for
// the affine column and row).  The stage cost in du' has the linear term g_u' = g_u - H_u s, H_u = 2 Rw + Sigma_u + dw I
// (no state-input curvature: f is linear in u); P, p and K are the same, and k_ff' = k_ff + s, which the Newton forward
// sweep undoes (phase_forward: du = du' - s, with s taken from c_{k+1}).  g_u' depends on dw: ric_prep stores it for
// dw = 0 and the inertia retries rewrite it (ric_gu_shift).  A different rounding, not a different method: tolerance
// parity with the oracle (tests/test_gpu_parity.py), not bitwise identity with round 5.
template <int BM>
__device__ __forceinline__ void gu_shift(const Ctx<BM>& c, double gu0, double gu1, double su0, double su1, double cn4,
                                         double cn5, double dw, double& g0, double& g1) {
    const double idt = 1.0 / c.dt;
    const double r00 = 2.0 * c.h(hRW), r01 = 2.0 * c.h(hRW + 1), r11 = 2.0 * c.h(hRW + 3);
    const double s0 = -cn5 * idt, s1 = -cn4 * idt;  // (b^5, b^4) / dt, b^ = -c_{k+1}
    const double h00 = r00 + su0 + dw, h11 = r11 + su1 + dw;
    g0 = gu0 - fma(h00, s0, r01 * s1);
    g1 = gu1 - fma(r01, s0, h11 * s1);
}
// an inertia retry with dw > 0: g_u' for the new dw (the rows gu_shift reads are intact until the forward sweep)
template <int BM>
__device__ __forceinline__ void ric_gu_shift(const Ctx<BM>& c, double dw) {
    for (int k = c.lane; k < c.N; k += W) {
        const double gu0 = c.r(rGF + 6, k), gu1 = c.r(rGF + 7, k), su0 = c.r(rSGU, k), su1 = c.r(rSGU + 1, k);
        const double cn4 = c.r(rCC + 4, k + 1), cn5 = c.r(rCC + 5, k + 1);
        double g0, g1;
        gu_shift(c, gu0, gu1, su0, su1, cn4, cn5, dw, g0, g1);
        c.r(rGU, k) = g0;
        c.r(rGU + 1, k) = g1;
    }
    __syncthreads();
}

// stage-parallel: fold the barrier, curvature and constraint terms into the Riccati operand rows
template <int BM>
__device__ __forceinline__ void phase_ric_prep(const Ctx<BM>& c) {
    const int N = c.N;
    for (int k = c.lane; k <= N; k += W) {
        double g[8], hd[6], su0 = 0.0, su1 = 0.0;   // read every source row before the first overlay write
#pragma unroll
        for (int v = 0; v < 8; ++v) g[v] = (v >= 6 && k == N) ? 0.0 : c.r(rGF + v, k) + c.mu * c.g(rDB + v, k);
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const int wi = w_idx(i, i);
            double d = c.g(rSG + i, k);
            if (wi >= 0 && k < N) d += c.r(rWC + wi, k);
            hd[i] = d;
        }
        if (k < N) { su0 = c.g(rSG + 6, k); su1 = c.g(rSG + 7, k); }
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            if (v >= 6 && k == N) break;
            c.r(rGF + v, k) = g[v];
        }
#pragma unroll
        for (int i = 0; i < 6; ++i) c.r(rHD + i, k) = hd[i];
        c.r(rSGU, k) = su0;
        c.r(rSGU + 1, k) = su1;
        if (k < N) {
            double cn[6];
#pragma unroll
            for (int i = 0; i < 6; ++i) cn[i] = c.r(rCC + i, k + 1);
#pragma unroll
            for (int i = 0; i < 4; ++i) c.r(rBH + i, k) = -cn[i];
            double g0, g1;
            gu_shift(c, g[6], g[7], su0, su1, cn[4], cn[5], 0.0, g0, g1);
            c.r(rGU, k) = g0;
            c.r(rGU + 1, k) = g1;
        } else {  // terminal stage: no dynamics, so no curvature
#pragma unroll
            for (int i = 0; i < 7; ++i) c.r(rWC + i, k) = 0.0;
        }
    }
    __syncthreads();
}

// Per-lane slots of entry (i, j): D[m][j] (m = 0..5) for PA, D[l][i] for F, H^[i][j], store rows.
struct EpMap {
    int dj[4], di[4];
    int hs, ps;
    int gj0, gj1, gi0, gi1;  // rows of g_u at the affine column / row (j or i = 6), the zero pad elsewhere
    double q2, dg;
    // row of D[m][n], m = 0..3 (rows 4, 5 of dt*J are zero and the shifted affine column has no rows 4, 5; PAD = 0)
    __device__ __forceinline__ static int dslot(int m, int n) {
        return (m < 4 && n < 6 && d_idx(m, n) >= 0) ? rAJ + d_idx(m, n) : (m < 4 && n == 6) ? rBH + m : PAD;
    }
    __device__ __forceinline__ void init(int i, int j, const double* QW) {
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            dj[m] = dslot(m, j);
            di[m] = dslot(m, i);
        }
        const int gi = (i < 6 && j == 6) ? i : (i == 6 && j < 6) ? j : -1;
        hs = (i == j && i < 6) ? rHD + i : (i < 6 && j < 6 && w_idx(i, j) >= 0) ? rWC + w_idx(i, j)
           : gi >= 0 ? rGF + gi : PAD;
        q2 = (i < 6 && j < 6) ? 2.0 * QW[i * 6 + j] : 0.0;
        dg = (i == j && i < 6) ? 1.0 : 0.0;
        ps = (i <= j && j < 6) ? rPS + sym_idx(i, j) : (i < 6 && j == 6) ? rPV + i : -1;
        gj0 = j == 6 ? rGU : PAD;
        gj1 = j == 6 ? rGU + 1 : PAD;
        gi0 = i == 6 ? rGU : PAD;
        gi1 = i == 6 ? rGU + 1 : PAD;
    }
};

// stage operands (independent of P^_{k+1}): fetched one stage ahead so LDS latency hides
struct EpOps {
    double dj[4], di[4], h, sgu0, sgu1, gj0, gj1, gi0, gi1;
};
// in two halves: A (D[.][j], Sigma_u) is issued behind the P-row reads, B (D[.][i], H^, g_u) behind the
// PA-column reads, which spreads the LDS queue over the stage (tools/ubench_riccati.hip: -44 cycles/stage)
template <int BM>
__device__ __forceinline__ void ep_ops_a(const Ctx<BM>& c, const EpMap& m, int k, EpOps& o) {
#pragma unroll
    for (int t = 0; t < 4; ++t) o.dj[t] = c.rl(m.dj[t], k);
    o.sgu0 = c.r(rSGU, k);
    o.sgu1 = c.r(rSGU + 1, k);
}
template <int BM>
__device__ __forceinline__ void ep_ops_b(const Ctx<BM>& c, const EpMap& m, int k, double dw, EpOps& o) {
#pragma unroll
    for (int t = 0; t < 4; ++t) o.di[t] = c.rl(m.di[t], k);
    o.h = m.q2 + m.dg * dw + c.rl(m.hs, k);
    o.gj0 = c.rl(m.gj0, k);
    o.gj1 = c.rl(m.gj1, k);
    o.gi0 = c.rl(m.gi0, k);
    o.gi1 = c.rl(m.gi1, k);
}
template <int BM>
__device__ __forceinline__ EpOps ep_ops(const Ctx<BM>& c, const EpMap& m, int k, double dw) {
    EpOps o;
    ep_ops_a(c, m, k, o);
    ep_ops_b(c, m, k, dw, o);
    return o;
}

__device__ __forceinline__ double2 ld2(const double* p) { return *reinterpret_cast<const double2*>(p); }

// Backward Riccati sweep (operand rows from phase_ric_prep).  Returns false when a reduced input
// Hessian is not positive definite (the caller raises the primal regularisation dw and retries).
// NS > 0: horizon fixed at compile time, every stage unrolled (stage offsets fold into the DS immediates).
template <int BM, int NS>
__device__ __forceinline__ bool phase_riccati(const Ctx<BM>& c, double dw) {
    const int N = c.N, i = c.lane >> 3, j = c.lane & 7;
    EpMap m;
    m.init(i, j, c.sm + hQW);
    m.hs = Ctx<BM>::lrow(m.hs);  // the operand slots are LDS rows (rl); the factor slot m.ps is a logical row (g)
    const double dt = c.dt, dt2 = dt * dt;
    const double r00 = 2.0 * c.h(hRW), r01 = 2.0 * c.h(hRW + 1), r11 = 2.0 * c.h(hRW + 3);
    double* PF = c.sm + hPF;
    double* PT = c.sm + hPT;
    // Both tiles swizzle rows 4..7 by XOR 4 on the column (halves swapped): a b128 read of one chunk of every row then
    // touches 32 distinct banks (rows i and i+4 sit 64 doubles = 128 banks apart, i.e. on the same banks, unswizzled),
    // the even pairs stay aligned, and a row is still a permutation of its 8 slots (the per-lane writes stay
    // conflict-free).  Element (r, cidx) of a tile is at 8 r + (cidx ^ (r & 4)).
    const int sw_i = i & 4, sw_j = j & 4;
    const int pf_own = 8 * i + (j ^ sw_i);  // this lane's P^ entry
    // terminal P^_N = H^_N (no dynamics): padded lanes hold exact zeros
    double Pij = m.q2 + m.dg * dw + c.rl(m.hs, N);
    PF[pf_own] = Pij;
    asm volatile("" ::: "memory");
    if constexpr (Ctx<BM>::kPG) {
        if (m.ps >= 0) c.gu(m.ps, N) = Pij;
    } else {
        pstore(c, m.ps >= 0, m.ps, N, Pij);
    }
    // inertia flag accumulated without branching: a failed stage only poisons the (discarded) factors
    bool pd = true;
    // The stage's factorisation rows leave in ONE unmasked ds_write per lane (three predicated stores
    // cost ~100 cycles per stage, tools/ubench_riccati.hip): P^ entries from the lanes that own them
    // (upper triangle and the p column), K^ rows from the affine/pad rows i = 6, 7 (m0, m1 depend on j
    // only); every other lane writes into the last dX row, which the forward sweep overwrites.
    const bool own_p = m.ps >= 0;
    const bool k_row = i >= 6 && j < 7;
    const int st_row = own_p ? m.ps : k_row ? (j < 6 ? rK + 6 * (i - 6) + j : rKF + (i - 6)) : rDX + 7;
    // one stage; `o` = this stage's operands, `nx` receives stage kn's (prefetch in two halves, each issued
    // after a tile read so that waiting for the tile never waits for the prefetch)
    auto stage = [&](int k, const EpOps& o, EpOps& nx, int kn) {
        // row i of P^_{k+1} and the reduced input Hessian entries (uniform)
        const double2 r01v = ld2(PF + 8 * i + sw_i), r23v = ld2(PF + 8 * i + (2 ^ sw_i));
        const double2 p5 = ld2(PF + 40);  // P[5][4], P[5][5] (row 5: columns 4, 5 at slots 0, 1)
        const double p44 = PF[32];        // P[4][4] (row 4: column 4 at slot 0)
        __builtin_amdgcn_sched_barrier(0);
        ep_ops_a(c, m, kn, nx);  // next stage's operands, first half
        __builtin_amdgcn_sched_barrier(0);
        const double h00 = r00 + o.sgu0 + dw + dt2 * p5.y, h01 = r01 + dt2 * p5.x, h11 = r11 + o.sgu1 + dw + dt2 * p44;
        const double det = h00 * h11 - h01 * h01;
        pd = pd & (h00 > 0.0) & (h11 > 0.0) & (det > 1e-13 * h00 * h11);
        const double id = frcp(det), i00 = h11 * id, i01 = -h01 * id, i11 = h00 * id;
        // PA[i][j] = P[i][j] + sum_{m<4} P[i][m] D[m][j]
        double pa = fma(r01v.x, o.dj[0], Pij), pb = r01v.y * o.dj[1];
        pa = fma(r23v.x, o.dj[2], pa);
        pb = fma(r23v.y, o.dj[3], pb);
        const double PAij = pa + pb;
        PT[8 * j + (i ^ sw_j)] = PAij;
        asm volatile("" ::: "memory");  // the tile is read by other lanes: keep program order
        // column j of PA (rows 0..5; rows 4, 5 also give G[.][j]) and G[.][i]
        const double2 c01 = ld2(PT + 8 * j + sw_j), c23 = ld2(PT + 8 * j + (2 ^ sw_j)), c45 = ld2(PT + 8 * j + (4 ^ sw_j));
        const double2 gi = ld2(PT + 8 * i + (4 ^ sw_i));  // PA[4][i], PA[5][i]
        // next stage's operands, second half: issued behind the tile reads (LDS serves a wave in order)
        __builtin_amdgcn_sched_barrier(0);
        ep_ops_b(c, m, kn, dw, nx);
        // F[i][j] = PA[i][j] + sum_{l<4} D[l][i] PA[l][j] + H^[i][j]
        double fa = fma(o.di[0], c01.x, PAij + o.h), fb = o.di[1] * c01.y;
        fa = fma(o.di[2], c23.x, fa);
        fb = fma(o.di[3], c23.y, fb);
        const double F = fa + fb;
        // G[0][.] = dt PA[5][.] + S, G[1][.] = dt PA[4][.] + S;  M = H_uu^-1 G;  P^_k = F - G' M
        const double g0j = fma(dt, c45.y, o.gj0), g1j = fma(dt, c45.x, o.gj1);
        const double g0i = fma(dt, gi.y, o.gi0), g1i = fma(dt, gi.x, o.gi1);
        const double m0 = fma(i00, g0j, i01 * g1j), m1 = fma(i01, g0j, i11 * g1j);
        Pij = F - fma(g0i, m0, g1i * m1);
        PF[pf_own] = Pij;
        asm volatile("" ::: "memory");
        // factorisation rows for the forward sweep, the step and the SOC
        if constexpr (Ctx<BM>::kPG) {  // P^ to HBM (the kPG band), K^ rows and the dump row to LDS
            if (own_p) c.gu(m.ps, k) = Pij;
            else c.rl(st_row, k) = i == 6 ? -m0 : -m1;
        } else {
            c.r(st_row, k) = own_p ? Pij : (i == 6 ? -m0 : -m1);
        }
    };
    // two stages per trip with ping-pong operand buffers (no register copies between stages)
    EpOps oa = ep_ops(c, m, N - 1, dw), ob;
    if constexpr (NS > 0) {
#pragma unroll
        for (int k = NS - 1; k >= 1; k -= 2) {
            stage(k, oa, ob, k - 1);
            stage(k - 1, ob, oa, k >= 2 ? k - 2 : 0);
        }
        if constexpr (NS % 2 == 1) stage(0, oa, ob, 0);
    } else {
        int k = N - 1;
        for (; k >= 1; k -= 2) {
            stage(k, oa, ob, k - 1);
            stage(k - 1, ob, oa, k - 2);  // k - 2 = -1 prefetches harmless head words (HEAD >= SR)
        }
        if (k == 0) stage(0, oa, ob, 0);
    }
    __syncthreads();
    return pd;
}

// ============ forward sweep: [x^_{k+1}; du_k] = [Phi_k; K^_k] x^_k, Phi = A^ + B^ K^ ============
// Lane 8g + m owns the term Phi[row(g)][m] x^_k[m] (rows g = 0..5: dx_{k+1}; g = 6, 7: du0, du1).
// The row sums are three in-row DPP adds (quad xor 1, xor 2, half-mirror); the next stage's x^[m]
// comes from group m by one ds_bpermute.  crow: residual rows (x^_0 = [-c_0; 1]); bhrow: b^ = -c_{k+1}
// stored at stage k.
__device__ __forceinline__ double bperm_d(double v, int src_lane) {
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(b & 0xffffffffll));
    const int hi = __builtin_amdgcn_ds_bpermute(src_lane << 2, (int)(b >> 32));
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// NS > 0: the horizon is a compile-time constant and the sweep is fully unrolled, so every stage's LDS
// offsets fold into the ds_read/ds_write immediates (no per-stage address arithmetic)
template <int BM, int NS, bool BHN = false>
__device__ __forceinline__ void phase_forward(const Ctx<BM>& c, int crow, int bhrow, int orow) {
    const int N = c.N, g = c.lane >> 3, mm = c.lane & 7;
    // output row of this lane's group: 0..5 = dx_{k+1}[g], 6/7 = du0/du1 (rows 7/8 of [Phi; K^])
    const int u = (g == 5 || g == 6) ? 0 : (g == 4 || g == 7) ? 1 : -1;
    const double fone = (g < 6 && mm == g) ? 1.0 : 0.0;
    // BHN: b^_k = -c_{k+1} read straight from the residual rows of stage k+1 (row kSR + crow + g of stage k)
    // instead of a stored b^ row (the SOC sweep: c_soc lives where its own output dX_soc goes)
    // The Newton sweep (!BHN) runs in the Riccati's shifted input (gu_shift): K^'s affine column is k_ff' = k_ff + s,
    // so the state rows 4, 5 take no b^ term (dt k_ff' carries it) and du = du' - s, with -s = c_{k+1}[(5, 4)] / dt from
    // the residual rows of stage k+1.  The SOC sweep (BHN) runs on the unshifted factors of phase_soc_backward.
    const bool shf = !BHN && mm == 6;
    // the sweep's row offsets are LDS rows (rl): crow / orow mapped once, the next stage one LDS stride (kSR) ahead
    constexpr int LSR = Ctx<BM>::kSR;
    const int crl = Ctx<BM>::lrow(crow), orl = Ctx<BM>::lrow(orow);
    const int fas = (g < 6 && mm < 6 && d_idx(g, mm) >= 0) ? rAJ + d_idx(g, mm)
                  : (shf && (g == 4 || g == 5)) ? PAD
                  : (shf && g == 6) ? LSR + crl + 5 : (shf && g == 7) ? LSR + crl + 4
                  : (g < 6 && mm == 6) ? (BHN ? LSR + crl + g : bhrow + g) : PAD;
    const double fsg = (BHN && g < 6 && mm == 6) ? -1.0 : (shf && g >= 6) ? 1.0 / c.dt : 1.0;
    const int fk = (u >= 0 && mm < 6) ? rK + 6 * u + mm : (u >= 0 && mm == 6) ? rKF + u : PAD;
    const double fkc = u >= 0 ? (g < 6 ? c.dt : 1.0) : 0.0;
    // x^_0[m] = -c_0[m] (m < 6), 1 (m = 6), 0 (m = 7)
    double x = mm < 6 ? -c.rl(crl + mm, 0) : (mm == 6 ? 1.0 : 0.0);
    if (c.lane < 6) c.rl(orl + c.lane, 0) = -c.rl(crl + c.lane, 0);
    const int src = 8 * (mm < 6 ? mm : 0);  // group holding x_{k+1}[mm]
    double nph = fone + fsg * c.rl(fas, 0) + fkc * c.rl(fk, 0);
    // unrolled builds: one unmasked store per lane and stage.  Lane 8g writes its output (dx_{k+1}[g] or
    // du_k[g-6]); the other 56 lanes write a row that is dead here -- the Hessian diagonal (rHD, consumed
    // by the Riccati) in the Newton sweep, the residual c (rCC, consumed by the SOC right-hand side) in
    // the SOC sweep
    const int fst = mm == 0 ? (g < 6 ? LSR + orl + g : orl + g) : Ctx<BM>::lrow(BHN ? rCC : rHD) + (g % 6);
    auto step = [&](int k) {
        const double ph = nph;
        const int kn = k + 1 < N ? k + 1 : k;
        nph = fone + fsg * c.rl(fas, kn) + fkc * c.rl(fk, kn);
        double y = ph * x;
        y += dppd<0xB1>(y);   // quad_perm [1,0,3,2]
        y += dppd<0x4E>(y);   // quad_perm [2,3,0,1]
        y += dppd<0x141>(y);  // row_half_mirror: the 8-lane group sum, in every lane of the group
        // rows 0..5 -> dx_{k+1}; groups 6/7 -> du0/du1 at stage k
        if constexpr (NS > 0) {
            c.sm[HEAD + k * LSR + fst] = y;
        } else {
            pstore(c, mm == 0 && g < 6, orl + g, k + 1, y);
            pstore(c, mm == 0 && g >= 6, orl + g, k, y);
        }
        const double xn = bperm_d(y, src);
        x = mm < 6 ? xn : (mm == 6 ? 1.0 : 0.0);
    };
    if constexpr (NS > 0) {
#pragma unroll
        for (int k = 0; k < NS; ++k) step(k);
    } else {
        for (int k = 0; k < N; ++k) step(k);
    }
    __syncthreads();
}

// ============ SOC: backward vector pass with the stored factorisation, rhs c_soc in rCT ============
template <int BM>
__device__ __forceinline__ void phase_soc_backward(const Ctx<BM>& c, double dw) {
    if (c.lane == 0) {
        const int N = c.N;
        const double dt = c.dt, dt2 = dt * dt;
        const double r00 = 2.0 * c.h(hRW), r01 = 2.0 * c.h(hRW + 1), r11 = 2.0 * c.h(hRW + 3);
        double p[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) p[i] = c.gr(i, N);
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
                for (int l = 0; l < 6; ++l) s -= c.g(rPS + sym_idx(rr, l), k + 1) * cn[l];
                w[rr] = s;
            }
            const double h0 = c.gr(6, k) + dt * w[5], h1 = c.gr(7, k) + dt * w[4];
            // H_uu^-1 of the Riccati stage (R~ + Sigma_u + dw + dt^2 P_{k+1}[{5,4}]), recomputed
            const double h00 = r00 + c.r(rSGU, k) + dw + dt2 * c.g(rPS + sym_idx(5, 5), k + 1);
            const double h01 = r01 + dt2 * c.g(rPS + sym_idx(4, 5), k + 1);
            const double h11 = r11 + c.r(rSGU + 1, k) + dw + dt2 * c.g(rPS + sym_idx(4, 4), k + 1);
            const double id = frcp(h00 * h11 - h01 * h01), i00 = h11 * id, i01 = -h01 * id, i11 = h00 * id;
            c.r(rKF, k) = -(i00 * h0 + i01 * h1);
            c.r(rKF + 1, k) = -(i01 * h0 + i11 * h1);
#pragma unroll
            for (int rr = 0; rr < 6; ++rr) {
                p[rr] = c.gr(rr, k) + w[rr] + colJ(aj, rr, w, 1) + c.r(rK + rr, k) * h0 + c.r(rK + 6 + rr, k) * h1;
                c.g(rPV + rr, k) = p[rr];
            }
        }
    }
    __syncthreads();
}

struct StepInfo {
    double ap, az, Dg, rel;
};

// ============ new multipliers y+ = -(P dx + p), step bounds, merit slope (stage-parallel) ============
template <int BM>
__device__ __forceinline__ StepInfo phase_step(const Ctx<BM>& c, int dzr, bool primal_pieces) {
    const int N = c.N;
    double ap = 1.0, az = 1.0, Dg = 0.0, rel = 0.0;
    const int p = c.part();
    for (int k = c.k0(); k <= N; k += c.kst()) {
        // the stage's y+ stores go after every LDS read of the stage (a read queued behind a store waits for it)
        double dx[6], yp[6];
#pragma unroll
        for (int i = 0; i < 6; ++i) dx[i] = c.r(dzr + i, k);
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            if (c.pair && q >= 3) break;
            const int i = c.pair ? 2 * q + p : q;
            double s = c.g(rPV + i, k);
#pragma unroll
            for (int j = 0; j < 6; ++j) s += c.g(rPS + (c.pair ? (p ? sym_idx(2 * q + 1, j) : sym_idx(2 * q, j)) : sym_idx(q, j)), k) * dx[j];
            if constexpr (Ctx<BM>::kLF) yp[q] = -s;
            else c.r(rYP + i, k) = -s;
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            if (c.pair && t >= 4) break;
            const int vb = c.pair ? 2 * t : t, v = vb + p;
            if (vb >= 6 && k == N) break;
            const double d = c.r(dzr + v, k), xv = c.r(rX + v, k);
            Dg += c.gr(v, k) * d;
            rel = fmax(rel, fabs(d) * frcp(1.0 + fabs(xv)));  // only tested against 1e-15
            if (c.hl(vb)) {
                const double s = xv - c.lb(v), rs = frcp(s), zl = c.r(rZL + v, k);
                ftb(s, d, c.tau, ap);
                ftb(zl, (c.mu - zl * d) * rs - zl, c.tau, az);
            }
            if (c.hu(vb)) {
                const double s = c.ub(v) - xv, rs = frcp(s), zu = c.r(rZU + v, k);
                ftb(s, -d, c.tau, ap);
                ftb(zu, (c.mu + zu * d) * rs - zu, c.tau, az);
            }
        }
        if constexpr (Ctx<BM>::kLF)
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                if (c.pair && q >= 3) break;
                c.r(rYP + (c.pair ? 2 * q + p : q), k) = yp[q];
            }
    }
    StepInfo r;
    if (primal_pieces) {
        double naz = -az, nap = -ap, dum = 0.0;
        r.rel = rel;
        wred4(c.lane, naz, nap, r.rel, dum, OpMax());
        r.az = -naz;
        r.ap = -nap;
        r.Dg = wsum(Dg);
    } else {
        double naz = -az, nap = -ap;
        wred2(c.lane, naz, nap, OpMax());
        r.az = -naz;
        r.ap = -nap;
        r.Dg = r.rel = 0.0;
    }
    __syncthreads();
    return r;
}

// ============ filter trial at z + alpha*dz (rows dzr): phi_mu = F - mu*sum(log s) and theta = ||c||_1 ============
struct Trial {
    double phi, th;
};

template <int BM>
__device__ __forceinline__ Trial phase_trial(const Ctx<BM>& c, double alpha, int dzr, bool storeC) {
    const int N = c.N;
    c.t_alpha = alpha;
    c.t_dz = dzr;
    double val = 0.0, thl = 0.0;
    bool bad = false;
    const int p = c.part();
    for (int k = c.k0(); k <= N; k += c.kst()) {
        double x[6], u[2] = {0.0, 0.0};
#pragma unroll
        for (int i = 0; i < 6; ++i) x[i] = c.r(rX + i, k) + alpha * c.r(dzr + i, k);
        if (k < N) {
            u[0] = c.r(rX + 6, k) + alpha * c.r(dzr + 6, k);
            u[1] = c.r(rX + 7, k) + alpha * c.r(dzr + 7, k);
        }
        double dxr[6], cost = 0.0, th = 0.0;
#pragma unroll
        for (int i = 0; i < 6; ++i) dxr[i] = x[i] - c.xr(i, k);
        if (c.pair) {  // (pair mode implies diagonal weights) variables 2t + part of the stage
#pragma unroll
            for (int t = 0; t < 3; ++t) {
                const double e = psel(p, dxr[2 * t], dxr[2 * t + 1]);
                cost += e * (c.h(hQW + (2 * t + p) * 7) * e);
            }
        } else if constexpr (Ctx<BM>::kDiag) {
#pragma unroll
            for (int i = 0; i < 6; ++i) cost += dxr[i] * (c.h(hQW + i * 7) * dxr[i]);
        } else {
#pragma unroll
            for (int i = 0; i < 6; ++i) {
                double s = 0.0;
#pragma unroll
                for (int j = 0; j < 6; ++j) s += c.h(hQW + i * 6 + j) * dxr[j];
                cost += dxr[i] * s;
            }
        }
        if (k < N) {
            const double e0 = u[0] - c.ur(0, k), e1 = u[1] - c.ur(1, k);
            SUBSTAMP(c, 0);
            if (c.pair)
                cost += p ? e1 * (c.h(hRW + 3) * e1) : e0 * (c.h(hRW) * e0);
            else if constexpr (Ctx<BM>::kDiag)
                cost += e0 * (c.h(hRW) * e0) + e1 * (c.h(hRW + 3) * e1);
            else
                cost += e0 * (c.h(hRW) * e0 + c.h(hRW + 1) * e1) + e1 * (c.h(hRW + 2) * e0 + c.h(hRW + 3) * e1);
        }
        LogSum ls;
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            if (c.pair && t >= 4) break;
            const int vb = c.pair ? 2 * t : t, v = vb + p;
            if (vb >= 6 && k == N) break;
            const double xv = vb < 6 ? psel(p, x[vb], x[c.pair ? vb + 1 : vb]) : psel(p, u[vb - 6], u[c.pair ? vb - 5 : vb - 6]);
            if (c.hl(vb)) { const double s = xv - c.lb(v); if (s <= 0.0) bad = true; else ls.add(s); }
            if (c.hu(vb)) { const double s = c.ub(v) - xv; if (s <= 0.0) bad = true; else ls.add(s); }
        }
        const int nrow = c.pair ? 3 : 6;
        SUBSTAMP(c, 1);
        // the next stage's trial state is read before any residual store of this pass (a read queued behind a store
        // waits for it); the residual rows are stored at the end
        constexpr bool LF = Ctx<BM>::kLF;
        double xnv[6] = {0, 0, 0, 0, 0, 0}, cc0[6] = {0, 0, 0, 0, 0, 0}, cc1[6] = {0, 0, 0, 0, 0, 0};
        if (LF && k < N)
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                if (q >= nrow) break;
                const int i = c.pair ? 2 * q + p : q;
                xnv[q] = c.r(rX + i, k + 1) + alpha * c.r(dzr + i, k + 1);
            }
        if (k == 0) {
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                if (q >= nrow) break;
                const int i = c.pair ? 2 * q + p : q;
                const double cc = psel(p, x[c.pair ? 2 * q : q], x[c.pair ? 2 * q + 1 : q]) - c.h(hXI + i);
                th += fabs(cc);
                cc0[q] = cc;
                if (!LF && storeC) c.r(rCT + i, 0) = cc;
            }
        }
        if (k < N) {
            double fo[6];
            model_f(c, x, u, fo);
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                if (q >= nrow) break;
                const int i = c.pair ? 2 * q + p : q;
                const double xi = psel(p, x[c.pair ? 2 * q : q], x[c.pair ? 2 * q + 1 : q]);
                const double fi = psel(p, fo[c.pair ? 2 * q : q], fo[c.pair ? 2 * q + 1 : q]);
                const double xn = LF ? xnv[q] : c.r(rX + i, k + 1) + alpha * c.r(dzr + i, k + 1);
                const double cc = xn - (xi + c.dt * fi);
                th += fabs(cc);
                cc1[q] = cc;
                if (!LF && storeC) c.r(rCT + i, k + 1) = cc;
            }
        }
        if (LF && storeC) {
#pragma unroll
            for (int q = 0; q < 6; ++q) {
                if (q >= nrow) break;
                const int i = c.pair ? 2 * q + p : q;
                if (k == 0) c.r(rCT + i, 0) = cc0[q];
                if (k < N) c.r(rCT + i, k + 1) = cc1[q];
            }
        }
        SUBSTAMP(c, 2);
        val += cost - c.mu * ls.value();
        thl += th;
    }
    SUBSTAMP(c, 3);
    Trial t;
    t.phi = bad ? INFINITY : val;  // any lane outside the relaxed box -> +inf
    t.th = thl;
    wred2(c.lane, t.phi, t.th, OpSum());
    SUBSTAMP(c, 4);
    __syncthreads();
    return t;
}

// The switching condition alpha (-D)^s_phi > theta0^s_theta of the filter line search, and theta0^s_theta / (-D)^s_phi in
// alpha_min, need two FP64 pow calls: ~1.8 k cycles per iteration on the critical path when they were evaluated up front
// (SUBSTAMP census, profiles/r05/track_ab/).  They are now evaluated only where a decision needs them: the condition is
// first bracketed by the binary exponents of alpha, -D and theta0, and when the two sides are more than a factor 4
// apart (all of them in the normal range) the comparison of the pow values -- accurate to an ulp -- cannot come out
// otherwise; the pows are computed in the remaining cases, and for alpha_min only when the line search backtracks.
// Every decision is the one the exact pows give (the oracle evaluates them always).
struct SwitchPow {
    double mD, th0, pD = 0.0, pT = 0.0;
    bool have = false;
    __device__ __forceinline__ void pows() {
        if (!have) {
            // the empty volatile asm keeps the pows where a decision needs them: without it the compiler speculates
            // them (they are pure and loop-invariant) to the front of the line search, back on the critical path
            double a = mD, b = th0;
            asm volatile("" : "+v"(a), "+v"(b));
            pD = pow(a, kSPh);
            pT = pow(b, kSTh);
            have = true;
        }
    }
    // alpha (-D)^s_phi > theta0^s_theta, for -D > 0
    __device__ __forceinline__ bool cond(double alpha) {
        if (th0 > 0.0 && alpha > 0.0) {
            int e1, e2, e3;
            (void)frexp(mD, &e1);
            (void)frexp(th0, &e2);
            (void)frexp(alpha, &e3);
            // log2 of alpha (-D)^s_phi lies in [lo, hi), log2 of theta0^s_theta in [tlo, thi)
            const double plo = kSPh * (e1 - 1), phi = kSPh * e1, lo = (e3 - 1) + plo, hi = e3 + phi;
            const double tlo = kSTh * (e2 - 1), thi = kSTh * e2;
            const bool normal = plo > -1000.0 && phi < 1000.0 && lo > -1000.0 && hi < 1000.0 && tlo > -1000.0 &&
                                thi < 1000.0;
            if (normal && lo > thi + 2.0) return true;
            if (normal && hi < tlo - 2.0) return false;
        }
        pows();
        return alpha * pD > pT;
    }
};

// filter acceptance of a trial (theta, phi): not dominated by the filter (entries in the LDS head; lane
// f tests entry f, one ballot) and either f-type Armijo (theta0 <= theta_min and the switching
// condition) or sufficient theta / phi decrease, each compared with IPOPT's round-off allowance.
// Wave-uniform result.
template <int BM>
__device__ __forceinline__ bool filter_ok(const Ctx<BM>& c, int nf, const Trial& t, double th0, double phi0, double D,
                                          double alpha, double th_max, double th_min, SwitchPow& sp,
                                          bool& ftype) {
    if (!isfinite(t.phi) || t.th > th_max) return false;
    const int f = c.lane & (kTrackFilter - 1);
    if (__ballot(c.lane < nf && t.th >= c.sm[hFTH + f] && t.phi >= c.sm[hFPH + f]) != 0ull) return false;
    // switching condition alpha (-D)^s_phi > theta0^s_theta
    if (th0 <= th_min && D < 0.0 && sp.cond(alpha)) {
        ftype = true;
        return armijo(t.phi, phi0, alpha, D);
    }
    ftype = false;
    return t.th <= (1.0 - kGTh) * th0 || t.phi - (phi0 - kGPh * th0) <= 10.0 * 2.220446049250313e-16 * fabs(phi0);
}

// ============ accept the step (stage-parallel) ============
template <int BM>
__device__ __forceinline__ void phase_update(const Ctx<BM>& c, int dzr, double alpha, double az) {
    if constexpr (Ctx<BM>::kLF) {
    const int N = c.N, p = c.part();
    for (int k = c.k0(); k <= N; k += c.kst()) {
        // every LDS read of the stage before its stores (a read queued behind a store waits for it)
        double xnv[8], zlv[8], zuv[8], ynv[6];
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            if (c.pair && t >= 4) break;
            const int vb = c.pair ? 2 * t : t, v = vb + p;
            if (vb >= 6 && k == N) break;
            const double d = c.r(dzr + v, k), xo = c.r(rX + v, k), xn = xo + alpha * d;
            if (c.hl(vb)) {
                const double zl = c.r(rZL + v, k), rs = frcp(xo - c.lb(v));
                const double znew = zl + az * ((c.mu - zl * d) * rs - zl), rn = c.mu * frcp(xn - c.lb(v));
                zlv[t] = fmax(fmin(znew, 1e10 * rn), 1e-10 * rn);  // kappa_sigma = 1e10
            }
            if (c.hu(vb)) {
                const double zu = c.r(rZU + v, k), rs = frcp(c.ub(v) - xo);
                const double znew = zu + az * ((c.mu + zu * d) * rs - zu), rn = c.mu * frcp(c.ub(v) - xn);
                zuv[t] = fmax(fmin(znew, 1e10 * rn), 1e-10 * rn);
            }
            xnv[t] = xn;
        }
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            if (c.pair && q >= 3) break;
            const int i = c.pair ? 2 * q + p : q;
            const double y = c.r(rY + i, k);
            ynv[q] = y + alpha * (c.r(rYP + i, k) - y);
        }
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            if (c.pair && t >= 4) break;
            const int vb = c.pair ? 2 * t : t, v = vb + p;
            if (vb >= 6 && k == N) break;
            if (c.hl(vb)) c.r(rZL + v, k) = zlv[t];
            if (c.hu(vb)) c.r(rZU + v, k) = zuv[t];
            c.r(rX + v, k) = xnv[t];
        }
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            if (c.pair && q >= 3) break;
            c.r(rY + (c.pair ? 2 * q + p : q), k) = ynv[q];
        }
    }
    } else {
    const int N = c.N, p = c.part();
    for (int k = c.k0(); k <= N; k += c.kst()) {
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            if (c.pair && t >= 4) break;
            const int vb = c.pair ? 2 * t : t, v = vb + p;
            if (vb >= 6 && k == N) break;
            const double d = c.r(dzr + v, k), xo = c.r(rX + v, k), xn = xo + alpha * d;
            if (c.hl(vb)) {
                const double zl = c.r(rZL + v, k), rs = frcp(xo - c.lb(v));
                const double znew = zl + az * ((c.mu - zl * d) * rs - zl), rn = c.mu * frcp(xn - c.lb(v));
                c.r(rZL + v, k) = fmax(fmin(znew, 1e10 * rn), 1e-10 * rn);  // kappa_sigma = 1e10
            }
            if (c.hu(vb)) {
                const double zu = c.r(rZU + v, k), rs = frcp(c.ub(v) - xo);
                const double znew = zu + az * ((c.mu + zu * d) * rs - zu), rn = c.mu * frcp(c.ub(v) - xn);
                c.r(rZU + v, k) = fmax(fmin(znew, 1e10 * rn), 1e-10 * rn);
            }
            c.r(rX + v, k) = xn;
        }
#pragma unroll
        for (int q = 0; q < 6; ++q) {
            if (c.pair && q >= 3) break;
            const int i = c.pair ? 2 * q + p : q;
            c.r(rY + i, k) += alpha * (c.r(rYP + i, k) - c.r(rY + i, k));
        }
    }
    }
    __syncthreads();
}

// ============ c_soc = alpha c(z) + c(z + alpha dz), in place in rCT ============
template <int BM>
__device__ __forceinline__ void phase_soc_rhs(const Ctx<BM>& c, double alpha) {
    for (int k = c.lane; k <= c.N; k += W) {
#pragma unroll
        for (int i = 0; i < 6; ++i) {
            const double cs = alpha * c.r(rCC + i, k) + c.r(rCT + i, k);
            c.r(rCT + i, k) = cs;
        }
    }
    __syncthreads();
}

template <int BM>
__device__ __forceinline__ double phase_soc_alpha(const Ctx<BM>& c) {
    double as = 1.0;
    const int p = c.part();
    for (int k = c.k0(); k <= c.N; k += c.kst()) {
#pragma unroll
        for (int t = 0; t < 8; ++t) {
            if (c.pair && t >= 4) break;
            const int vb = c.pair ? 2 * t : t, v = vb + p;
            if (vb >= 6 && k == c.N) break;
            const double d = c.r(rDXS + v, k), xv = c.r(rX + v, k);
            if (c.hl(vb)) ftb(xv - c.lb(v), d, c.tau, as);
            if (c.hu(vb)) ftb(c.ub(v) - xv, -d, c.tau, as);
        }
    }
    return wmin(as);
}

// ---------------- load one instance into LDS (coalesced flat copies) ----------------
template <int BM>
__device__ __forceinline__ void phase_load(const Ctx<BM>& c, const TrackArgs& a, int b) {
    const int lane = c.lane, N = c.N, n = 8 * N + 6;
    if (lane < 8) {  // relaxed bounds (bound_relax_factor 1e-8), -inf/+inf = free
        const int v = lane;
        const double l = v < 6 ? a.xlb[v] : a.ulb[v - 6];
        const double u = v < 6 ? a.xub[v] : a.uub[v - 6];
        const bool hl = isfinite(l) && l > -1e19, hu = isfinite(u) && u < 1e19;
        c.h(hLB + v) = hl ? l - 1e-8 * fmax(1.0, fabs(l)) : -INFINITY;
        c.h(hUB + v) = hu ? u + 1e-8 * fmax(1.0, fabs(u)) : INFINITY;
    }
    const double* wq = a.wqwr ? a.wqwr + (size_t)b * 8 : nullptr;
    if (lane < 36) {  // Qw = diag(wq) sym(Q) diag(wq)   (mpc_control_fuzzy.py:23-24)
        const int i = lane / 6, j = lane % 6;
        const double q = 0.5 * (a.Q[i * 6 + j] + a.Q[j * 6 + i]);
        c.h(hQW + lane) = wq ? q * wq[i] * wq[j] : q;
    } else if (lane < 40) {
        const int e = lane - 36, i = e / 2, j = e % 2;
        const double r = 0.5 * (a.R[i * 2 + j] + a.R[j * 2 + i]);
        c.h(hRW + e) = wq ? r * wq[6 + i] * wq[6 + j] : r;
    } else if (lane < 46) {
        c.h(hXI + lane - 40) = a.x0[(size_t)b * 6 + (lane - 40)];
    }
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
                c.r(rX + v, k) = v < 6 ? c.gxr[k * 6 + v] : c.gur[k * 2 + v - 6];
            }
    }
    __syncthreads();
}

// Stage-unrolled builds with a specialised bound pattern and the reference-copy guess: the lane of a stage
// already holds its reference row (rc0..rc7, read at kernel entry), so the guess, the bound push, z = 1 and
// y = 0 are written straight from registers -- one global round trip before the first linearisation
// instead of two.  Same values as phase_load + phase_init (an infeasible x_init keeps the unpushed copy).
template <int BM>
__device__ __forceinline__ void phase_load_init_reg(const Ctx<BM>& c, const TrackArgs& a, int b) {
    const int lane = c.lane, N = c.N;
    if (lane < 8) {
        const int v = lane;
        const double l = v < 6 ? a.xlb[v] : a.ulb[v - 6];
        const double u = v < 6 ? a.xub[v] : a.uub[v - 6];
        const bool hl = isfinite(l) && l > -1e19, hu = isfinite(u) && u < 1e19;
        c.h(hLB + v) = hl ? l - 1e-8 * fmax(1.0, fabs(l)) : -INFINITY;
        c.h(hUB + v) = hu ? u + 1e-8 * fmax(1.0, fabs(u)) : INFINITY;
    }
    const double* wq = a.wqwr ? a.wqwr + (size_t)b * 8 : nullptr;
    if (lane < 36) {
        const int i = lane / 6, j = lane % 6;
        const double q = 0.5 * (a.Q[i * 6 + j] + a.Q[j * 6 + i]);
        c.h(hQW + lane) = wq ? q * wq[i] * wq[j] : q;
    } else if (lane < 40) {
        const int e = lane - 36, i = e / 2, j = e % 2;
        const double r = 0.5 * (a.R[i * 2 + j] + a.R[j * 2 + i]);
        c.h(hRW + e) = wq ? r * wq[6 + i] * wq[6 + j] : r;
    } else if (lane < 46) {
        c.h(hXI + lane - 40) = a.x0[(size_t)b * 6 + (lane - 40)];
    }
    // relaxed bounds (the head's values) and the infeasibility test of the kernel, evaluated per lane
    double lr[8], ur[8];
    bool infeas = false;
#pragma unroll
    for (int v = 0; v < 8; ++v) {
        const double l = v < 6 ? a.xlb[v] : a.ulb[v - 6], u = v < 6 ? a.xub[v] : a.uub[v - 6];
        lr[v] = l - 1e-8 * fmax(1.0, fabs(l));
        ur[v] = u + 1e-8 * fmax(1.0, fabs(u));
        if (v < 6) {
            const double xi = a.x0[(size_t)b * 6 + v];
            if (!isfinite(xi) || (c.hl(v) && xi < lr[v]) || (c.hu(v) && xi > ur[v])) infeas = true;
        }
    }
    const int k = c.k0(), part = c.part();
    if (k <= N) {
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            if (c.pair && (v >> 2) != part) continue;  // lane pairs: rows 0-3 on the even lane, 4-7 on the odd
            if (v >= 6 && k == N) continue;
            double z = c.rcv(v);
            if (!infeas) {
                const double l = lr[v], u = ur[v];
                if (c.hl(v) && c.hu(v)) {
                    const double pl = fmin(1e-2 * fmax(1.0, fabs(l)), 1e-2 * (u - l));
                    const double pu = fmin(1e-2 * fmax(1.0, fabs(u)), 1e-2 * (u - l));
                    z = fmin(fmax(z, l + pl), u - pu);
                } else if (c.hl(v)) {
                    z = fmax(z, l + 1e-2 * fmax(1.0, fabs(l)));
                } else if (c.hu(v)) {
                    z = fmin(z, u - 1e-2 * fmax(1.0, fabs(u)));
                }
                c.r(rZL + v, k) = c.hl(v) ? 1.0 : 0.0;
                c.r(rZU + v, k) = c.hu(v) ? 1.0 : 0.0;
            }
            c.r(rX + v, k) = z;
        }
        if (!infeas) {
            if (!c.pair || part == 0) { c.r(rY + 0, k) = 0.0; c.r(rY + 1, k) = 0.0; c.r(rY + 2, k) = 0.0; c.r(PAD, k) = 0.0; }
            if (!c.pair || part == 1) { c.r(rY + 3, k) = 0.0; c.r(rY + 4, k) = 0.0; c.r(rY + 5, k) = 0.0; }
        }
    }
    __syncthreads();
}

// bound push (IPOPT bound_push / bound_frac = 1e-2), z_L = z_U = 1, y = 0, zero pad row
template <int BM>
__device__ __forceinline__ void phase_init(const Ctx<BM>& c) {
    const int N = c.N;
    for (int k = c.lane; k <= N; k += W) {
#pragma unroll
        for (int v = 0; v < 8; ++v) {
            if (v >= 6 && k == N) break;
            double z = c.r(rX + v, k);
            const double l = c.lb(v), u = c.ub(v);
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
        c.r(PAD, k) = 0.0;
    }
    __syncthreads();
}

template <int BM, int OCC, int NS>
__global__ __launch_bounds__(W) __attribute__((amdgpu_waves_per_eu(OCC))) void track_kernel(TrackArgs a) {
    extern __shared__ __attribute__((aligned(16))) double sm[];
    // Instance b = workgroup b.  An XCD-aware map (contiguous instance ranges per XCD) was measured in round 2:
    // C2 +0.7 %, C3 -6 % (1.896 -> 2.01 ms, profiles/r02/ab_xcd.txt), so the plain map ships.
    const int b = blockIdx.x;
    const int N = NS > 0 ? NS : a.N, S = N + 1;  // NS: horizon fixed at compile time (stage offsets fold)
    Ctx<BM> c;
    c.sm = sm;
    c.N = N;
    c.lane = threadIdx.x;
    c.gxr = a.xref + (size_t)b * S * 6;
    c.gur = a.uref + (size_t)b * N * 2;
    if constexpr (Ctx<BM>::kPG)  // wave-uniform base: the descriptor lives in SGPRs; out-of-range offsets are dropped
        c.prs = __builtin_amdgcn_make_buffer_rsrc(a.prow + (size_t)b * S * kGlobalRows, (short)0,
                                                  S * kGlobalRows * (int)sizeof(double), 0x00020000);
    c.regref = NS > 0 && NS < W;
    c.pair = Ctx<BM>::kPairSym && Ctx<BM>::kDiag && NS > 0 && NS < W / 2;
    c.rc0 = c.rc1 = c.rc2 = c.rc3 = c.rc4 = c.rc5 = c.rc6 = c.rc7 = 0.0;
    c.ts0 = c.tc0 = c.ts1 = c.tc1 = c.ts2 = c.tc2 = 0.0;
    c.t_alpha = 0.0;
    c.t_dz = -1;
    c.t_ok = 0;
    if (NS > 0 && NS < W) {
        const int k = min(c.k0(), N), ku = min(k, N - 1);
        c.rc0 = c.gxr[k * 6 + 0]; c.rc1 = c.gxr[k * 6 + 1]; c.rc2 = c.gxr[k * 6 + 2];
        c.rc3 = c.gxr[k * 6 + 3]; c.rc4 = c.gxr[k * 6 + 4]; c.rc5 = c.gxr[k * 6 + 5];
        c.rc6 = c.gur[ku * 2 + 0]; c.rc7 = c.gur[ku * 2 + 1];
    }
    c.dt = a.dt;
    c.iL1 = 1.0 / a.L1;
    c.iL2 = 1.0 / a.L2;
    c.Mh = a.Mh;
    c.mu = 0.1;
    c.tau = fmax(0.99, 1.0 - c.mu);
#ifdef TT_STAMPS
    Stamps stamps;
    stamps.begin();
    c.st = &stamps;
#endif
    const bool fused = BM >= 0 && c.regref && !a.zg;
    if (fused) phase_load_init_reg(c, a, b);
    else phase_load(c, a, b);
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
        const double xi = c.h(hXI + i);
        if (!isfinite(xi) || (c.hl(i) && xi < c.lb(i)) || (c.hu(i) && xi > c.ub(i))) infeas = true;
    }
    int status = infeas ? 3 : 2, iter = 0;
    double E0 = INFINITY;
    if (!infeas) {
        if (!fused) phase_init(c);
        STAMP(PH_LOAD);
        double dw_last = 0.0, th_max = 0.0, th_min = 0.0;
        int acc_count = 0, nf = 0;
        // launch constants of the optimality-error scaling and the barrier floor: no IEEE division per iteration
        const double inv_m = 1.0 / (double)(6 * (N + 1) + nb), inv_nb = nb ? 1.0 / (double)nb : 0.0;
        // IPOPT's barrier floor (MonotoneMuUpdate::CalcNewMuAndTau): min(tol, compl_inf_tol) / (barrier_tol_factor + 1)
        const double mu_floor = fmin(a.tol, kComplInfTol) / 11.0, mu_floor_test = mu_floor * 1.0000001;
        for (iter = 0;; ++iter) {
            const Lin e = phase_linearize(c);
            STAMP(PH_LIN);
            if (!isfinite(e.dinf) || !isfinite(e.pinf)) { status = 4; break; }
            // IPOPT's s_d, s_c (s_max = 100) as reciprocals: E = max(dinf / s_d, pinf, compl / s_c)
            const double isd = 100.0 * frcp(fmax(100.0, (e.sy + e.sz) * inv_m));
            const double isc = nb ? 100.0 * frcp(fmax(100.0, e.sz * inv_nb)) : 1.0;
            const double dsc = e.dinf * isd;
            const double c0 = e.c0();
            E0 = fmax(fmax(dsc, e.pinf), c0 * isc);
            // IPOPT's OptimalityErrorConvergenceCheck: the scaled error and the UNSCALED dual infeasibility,
            // constraint violation (dynamics rows only: max |c| = pinf) and complementarity max |z s|
            const bool conv = E0 <= a.tol && e.dinf <= kDualInfTol && e.pinf <= kConstrViolTol && c0 <= kComplInfTol;
            const bool accp = E0 <= a.acc_tol && e.dinf <= kAccDualInfTol && e.pinf <= kAccConstrViolTol &&
                              c0 <= kAccComplInfTol;
            if (conv) { status = 0; break; }
            if (accp) {
                if (++acc_count >= a.acc_iter) { status = 1; break; }
            } else {
                acc_count = 0;
            }
            if (iter >= a.max_iter) { status = accp ? 1 : 2; break; }
            // barrier parameter (monotone Fiacco-McCormick)
            double cmu = e.cmu(c.mu);
            for (;;) {
                const double Emu = fmax(fmax(dsc, e.pinf), cmu * isc);
                if (!(Emu <= 10.0 * c.mu && c.mu > mu_floor_test)) break;
                c.mu = fmax(mu_floor, fmin(0.2 * c.mu, c.mu * sqrt(c.mu)));
                c.tau = fmax(0.99, 1.0 - c.mu);
                nf = 0;  // IPOPT resets the filter on every barrier update
                cmu = e.cmu(c.mu);
            }
            STAMP(PH_MU_BAR);
            // Newton step: Riccati with inertia correction
            double dw = 0.0;
            bool ok = false;
            phase_ric_prep(c);
            for (int attempt = 0; attempt < 30; ++attempt) {
                COUNT(PH_NRIC);
                if (dw > 0.0) ric_gu_shift(c, dw);
                if (phase_riccati<BM, NS>(c, dw)) { ok = true; break; }
                dw = (dw == 0.0) ? (dw_last == 0.0 ? 1e-4 : fmax(1e-20, dw_last / 3.0))
                                 : (dw_last == 0.0 ? 100.0 * dw : 8.0 * dw);
                if (dw > 1e20) break; /* IPOPT max_hessian_perturbation 1e20 */
            }
            if (!ok) { status = 5; break; } /* IPOPT Error_In_Step_Computation */
            if (dw > 0.0) dw_last = dw;
            STAMP(PH_RIC);
            phase_forward<BM, NS>(c, rCC, rBH, rDX);
            STAMP(PH_FWD);
            const StepInfo si = phase_step(c, rDX, true);
            STAMP(PH_STEP);
            // IPOPT filter line search (Waechter & Biegler 2006, IPOPT defaults) with one second-order
            // correction; theta / phi_mu of the current point come from the linearisation pass
            const double th0 = e.th, phi0 = e.cost - c.mu * e.logs, D = si.Dg;
            if (iter == 0) { th_max = 1e4 * fmax(1.0, th0); th_min = 1e-4 * fmax(1.0, th0); }
            // (-D)^s_phi and theta0^s_theta only matter when theta0 <= theta_min (switching condition, alpha_min):
            // evaluated lazily (SwitchPow)
            SwitchPow sp;
            sp.mD = -D;
            sp.th0 = th0;
            SUBSTAMP(c, 7);
            double alpha = si.ap, az = si.az;
            int accepted = si.rel < 1e-15 ? 1 : 0;
            c.t_dz = -1;  // no trial point of this iteration yet (a tiny step is taken without one)
            const bool tiny = accepted;
            bool soc = false, ftype = false;
            for (int ls = 0; !accepted; ++ls) {
                const Trial t = phase_trial(c, alpha, rDX, ls == 0);
                STAMP(PH_MERIT);
                COUNT(PH_NTRIAL);
                if (filter_ok(c, nf, t, th0, phi0, D, alpha, th_max, th_min, sp, ftype)) { accepted = 1; break; }
                if (ls == 0 && isfinite(t.phi) && t.th >= th0) {
                    phase_soc_rhs(c, alpha);
                    phase_soc_backward(c, dw);
                    phase_forward<BM, NS, true>(c, rCT, 0, rDXS);
                    const double as = phase_soc_alpha(c);
                    const Trial ts = phase_trial(c, as, rDXS, false);
                    STAMP(PH_SOC);
                    if (filter_ok(c, nf, ts, th0, phi0, D, alpha, th_max, th_min, sp, ftype)) {
                        accepted = 2;
                        soc = true;
                        alpha = as;
                        az = phase_step(c, rDXS, false).az;  // y+ and dual step bound of the corrected step
                        break;
                    }
                }
                // alpha_min (IPOPT: alpha_min_frac 0.05 of the smallest of gamma_theta, gamma_phi theta0 / (-D) and
                // delta theta0^s_theta / (-D)^s_phi), needed only now that the line search backtracks
                double amin = kGTh;
                if (D < 0.0) {
                    amin = fmin(kGTh, kGPh * th0 / (-D));
                    if (th0 <= th_min) {
                        sp.pows();
                        amin = fmin(amin, sp.pT / sp.pD);
                    }
                }
                amin *= 0.05;
                if (alpha * 0.5 < amin) break;
                alpha *= 0.5;
            }
            if (!accepted) {
                nf = 0;  // IPOPT would enter its restoration phase: take the last trial step, reset the filter
            } else if (!tiny && !ftype && nf < kTrackFilter) {
                if (c.lane == 0) {
                    c.sm[hFTH + nf] = (1.0 - kGTh) * th0;
                    c.sm[hFPH + nf] = phi0 - kGPh * th0;
                }
                ++nf;
                __syncthreads();
            }
            phase_update(c, soc ? rDXS : rDX, alpha, az);
            // the next linearisation point is the last trial point: reuse its trig (wave-uniform test)
            c.t_ok = c.regref && alpha == c.t_alpha && (soc ? rDXS : rDX) == c.t_dz;
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
            if (a.iters) a.iters[b] = iter;
            if (a.kkt) a.kkt[b] = E0;
        }
        if (a.host_done) {
            // a zero-copy host call polls status[b] in host memory instead of waiting for the stream: every other output
            // of the instance is made visible system-wide before it (vector stores, then the release)
            __syncthreads();
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        }
        if (lane == 0) a.status[b] = status;
    }
}

// bound pattern of the variables (bit v: finite lower, bit 8+v: finite upper), as the kernel sees it
int bound_mask(const TrackArgs& a) {
    int m = 0;
    for (int v = 0; v < 8; ++v) {
        const double l = v < 6 ? a.xlb[v] : a.ulb[v - 6], u = v < 6 ? a.xub[v] : a.uub[v - 6];
        if (isfinite(l) && l > -1e19) m |= 1 << v;
        if (isfinite(u) && u < 1e19) m |= 1 << (8 + v);
    }
    return m;
}

template <int BM, int OCC = 1, int NS = 0>
hipError_t launch(const TrackArgs& a, hipStream_t stream) {
    const int bytes = 8 * (Ctx<BM>::kSR * (a.N + 1) + kScratch);
    // the >64 KB opt-in is per device and cheap: set it on every launch that needs it (no process-global
    // cache that would miss a second device or race between threads)
    if (bytes > 64 * 1024) {
        hipError_t e = hipFuncSetAttribute((const void*)track_kernel<BM, OCC, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL((track_kernel<BM, OCC, NS>), dim3(a.B), dim3(W), bytes, stream, a);
    return hipGetLastError();
}

}  // namespace

// Specialised bound patterns: the reference MPC box (x, y free; theta, psi, phi, v, a, omega boxed:
// simulation.py:411-414) and the OBCA box (theta free too: trajectory_animation.py:77-80).
constexpr int kMaskMPC = 0xFCFC;
constexpr int kMaskOBCA = 0xF8F8;
constexpr int kDiagBit = 1 << 16;  // Q, R diagonal: the cost and its gradient skip the off-diagonal terms
constexpr int kOccBit = 1 << 17;   // the two-waves-per-SIMD build (Ctx::kLF)
constexpr int kPGBit = 1 << 18;    // the P / p band of the stage record in HBM (Ctx::kPG)

// Q and R diagonal after symmetrisation (the kernel's weights are 0.5 (Q + Q'), 0.5 (R + R'))
bool diagonal_weights(const TrackArgs& a) {
    for (int i = 0; i < 6; ++i)
        for (int j = i + 1; j < 6; ++j)
            if (0.5 * (a.Q[i * 6 + j] + a.Q[j * 6 + i]) != 0.0) return false;
    return 0.5 * (a.R[1] + a.R[2]) == 0.0;
}

// Above three instances per CU (768 on MI355X's 256 CUs) the LDS build of N = 50 needs a second round of instances;
// the HBM-band build fits four per CU.  Below, the LDS build is faster per instance (B = 1 host call 0.140 vs 0.161 ms).
// The two builds are bitwise one another (profiles/r06/n50_hbm_band/), so results do not depend on B.
int current_cu_count() {
    static std::atomic<int> cache[64];  // per device, 0 = not queried yet (a race only queries twice)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 256;
    if (dev < 64)
        if (const int c = cache[dev].load(std::memory_order_relaxed)) return c;
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
    if (dev < 64) cache[dev].store(cus, std::memory_order_relaxed);
    return cus;
}
bool uses_global_rows(const TrackArgs& a) {
    return bound_mask(a) == kMaskMPC && diagonal_weights(a) && a.N == 50 && a.B > 3 * current_cu_count();
}

size_t track_global_bytes(const TrackArgs& a) {
    return uses_global_rows(a) ? (size_t)a.B * (a.N + 1) * kGlobalRows * sizeof(double) : 0;
}

hipError_t launch_track(const TrackArgs& a, hipStream_t stream) {
    const int m = bound_mask(a);
    const bool d = diagonal_weights(a);
    // Two waves per SIMD only pay where LDS lets more than 4 waves share a CU (N <= 31 with the 118-double
    // stage record); at N = 40 four waves share a CU and the occupancy build's spills would be pure cost.
    const bool occ_room = 5 * lds_bytes(a.N) <= kMaxLdsBytes;
    // The BASELINE horizons (C2 N = 20, C3 N = 40) get stage-unrolled builds.  At N = 20 the large-batch
    // occupancy build is the same stage-unrolled code, so an instance's result never depends on B (or on the
    // sharded path's chunk size): only the build's register budget differs, not one operation.
    // Above B = 2048 (two rounds of one wave per SIMD) the two-waves-per-SIMD build wins: 12.6 vs 10.3 M solves/s at
    // B = 4096, 12.0 vs 9.8 at 3072, equal at 2048, 3 % slower at 1024 (profiles/r04/occ_by_batch/); round 3 switched
    // at 4096, so the 4096-instance chunks of the sharded C5 path ran one wave per SIMD.
    if (m == kMaskMPC && d && a.N == 20 && a.B > 2048) return launch<kMaskMPC | kDiagBit | kOccBit, 2, 20>(a, stream);
    if (m == kMaskMPC && d && a.N == 20) return launch<kMaskMPC | kDiagBit, 1, 20>(a, stream);
    // N = 30, the NMPC driver's horizon (simulation_nmpc.py): the same pair of stage-unrolled lane-pair builds as N = 20
    // (bitwise one another).  Against the generic builds: +30 % at B = 1024, +32 % at B = 8192, where the two-wave
    // build beats the one-wave one by 3.5 % (profiles/r06/unrolled_n30/)
    if (m == kMaskMPC && d && a.N == 30 && a.B > 2048) return launch<kMaskMPC | kDiagBit | kOccBit, 2, 30>(a, stream);
    if (m == kMaskMPC && d && a.N == 30) return launch<kMaskMPC | kDiagBit, 1, 30>(a, stream);
    // (the generic two-wave build keeps the load-first order: its one-stage-per-lane passes would otherwise contract
    // differently from the one-wave build's and results would depend on B, test_occupancy_build_boundary_n31_n32)
    if (m == kMaskMPC && d && a.B > 4096 && occ_room) return launch<kMaskMPC | kDiagBit, 2>(a, stream);
    if (m == kMaskMPC && d && a.N == 40) return launch<kMaskMPC | kDiagBit, 1, 40>(a, stream);
    // N = 50: the reference's closed-loop horizon (simulation.py), stage-unrolled like C3; large batches keep the
    // Riccati factor band in HBM so that four instances share a CU (uses_global_rows)
    if (uses_global_rows(a)) {
        if (!a.prow) return hipErrorInvalidValue;  // the caller sizes it with track_global_bytes
        return launch<kMaskMPC | kDiagBit | kPGBit, 1, 50>(a, stream);
    }
    if (m == kMaskMPC && d && a.N == 50) return launch<kMaskMPC | kDiagBit, 1, 50>(a, stream);
    if (m == kMaskMPC) return d ? launch<kMaskMPC | kDiagBit>(a, stream) : launch<kMaskMPC>(a, stream);
    if (m == kMaskOBCA) return d ? launch<kMaskOBCA | kDiagBit>(a, stream) : launch<kMaskOBCA>(a, stream);
    return launch<-1>(a, stream);
}

}  // namespace ttmpc
