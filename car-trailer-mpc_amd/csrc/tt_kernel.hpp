// Internal interface between the C-ABI layer (tt_api.hip) and the gfx950 kernels (tt_track.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace ttmpc {

// IPOPT's convergence test (OptimalityErrorConvergenceCheck, defaults): besides the scaled error E_0 <= tol, the
// unscaled dual infeasibility, constraint violation and complementarity must be below these (acceptable: the second set)
constexpr double kDualInfTol = 1.0, kConstrViolTol = 1e-4, kComplInfTol = 1e-4;
constexpr double kAccDualInfTol = 1e10, kAccConstrViolTol = 1e-2, kAccComplInfTol = 1e-2;

// Everything one launch needs; passed by value as the kernel argument (< 1 KB).
struct TrackArgs {
    int N, B, max_iter, acc_iter;
    double dt, L1, L2, Mh, tol, acc_tol;
    double Q[36], R[4];                   // row-major, symmetrised in-kernel
    double xlb[6], xub[6], ulb[2], uub[2];  // raw bounds; |b| >= 1e19 or inf = free
    const double* x0;                     // [B][6]
    const double* xref;                   // [B][N+1][6]
    const double* uref;                   // [B][N][2]
    const double* wqwr;                   // [B][8] or nullptr
    const double* zg;                     // [B][8N+6] or nullptr
    double* xout;                         // [B][N+1][6]
    double* uout;                         // [B][N][2]
    double* kkt;                          // [B] or nullptr
    int* status;                          // [B]
    int* iters;                           // [B] or nullptr
    unsigned long long* stamps;           // [B][kNumPhases] cycle sums (TT_STAMPS diagnostic build only)
    double* prow;                         // [B][N+1][kGlobalRows]: the stage rows a build keeps in HBM, or nullptr
    int host_done;                        // 1: status[b] is the instance's completion flag for a polling host (zero-copy
                                          //    host calls): written last, after a system-scope release of the rest
};

// phases timed by the TT_STAMPS diagnostic build
// PH_NRIC / PH_NTRIAL: counts (Riccati attempts, line-search trials), not cycles
// PH_X0..PH_X7: sub-phase slots for finer TT_STAMPS instrumentation inside a phase (SUBSTAMP in tt_track.hip)
enum { PH_LOAD = 0, PH_LIN, PH_MU_BAR, PH_RIC, PH_FWD, PH_STEP, PH_MERIT, PH_SOC, PH_UPDATE, PH_NRIC, PH_NTRIAL,
       PH_X0, PH_X1, PH_X2, PH_X3, PH_X4, PH_X5, PH_X6, PH_X7, PH_TOTAL, kNumPhases };

// LDS: fixed head + rows per stage (doubles); see tt_track.hip for the map.
// 116 used + 1 zero pad + 1 unused.  The even stride (= 2 mod 4, 944 B) keeps every stage record 16-B aligned and makes
// the lane-pair phases' reads conflict-free (lanes 2k, 2k+1 -> rows R, R+1 of stage k); bitwise the same as 117, C2
// -2.5 %, C3 -1.7 % (profiles/r04/stride118/).
constexpr int kRowsPerStage = 118;
constexpr int kTrackFilter = 16;  // filter line search entries (theta, phi) kept in the LDS head
constexpr int kHead = 256;  // 64 head values + 32 dump slots + 2x16 filter entries + two 8x8 Riccati tiles
constexpr int kScratch = kHead;
constexpr int kMaxLdsBytes = 160 * 1024;

inline int lds_doubles(int N) { return kRowsPerStage * (N + 1) + kScratch; }
inline int lds_bytes(int N) { return 8 * lds_doubles(N); }
inline int max_horizon() { return (kMaxLdsBytes / 8 - kScratch) / kRowsPerStage - 1; }

// The N = 50 build keeps the 28 stage rows of the Riccati factor (P, p) and of its overlay (Sigma, dB: linearise ..
// ric_prep) in HBM instead of LDS: a 38.8 KB record, four instances per CU instead of three (tt_track.hip, round 6).
constexpr int kGlobalRows = 28;
// bytes of TrackArgs::prow the launch of `a` needs (0: every stage row stays in LDS)
size_t track_global_bytes(const TrackArgs& a);

hipError_t launch_track(const TrackArgs& a, hipStream_t stream);

}  // namespace ttmpc

namespace ttmpc {

// ---------------- OBCA NLPs (tt_obca.hip) ----------------
constexpr int kObcaMaxM = 16;
constexpr int kObcaThreads = 256;  // one workgroup (4 waves) per instance
constexpr int kObcaMaxFilter = 64;
enum { OBCA_PLAN = 0, OBCA_TRACK = 1 };

// ObcaArgs::opts bits (diagnostics / A-B builds; 0 = IPOPT's algorithm): the same switches as the oracle's TTO_OPT_*
// (PD_BLOCKS: round 2's positive-definite block test instead of the exact block inertia; NO_REFINE: no iterative
// refinement)
enum { OBCA_OPT_NO_RESTO = 1, OBCA_OPT_NO_SOFT_RESTO = 2, OBCA_OPT_NO_LSQ_MULT = 4, OBCA_OPT_PD_BLOCKS = 32,
       OBCA_OPT_NO_REFINE = 64 };

struct ObcaArgs {
    int N, M, B, mode, max_iter, acc_iter, dual_init, opts;
    double dt, L1, L2, Mh, W1, W2, tol, acc_tol, dmin, eq_tol, fin_tol, tfac;
    double Q[36], R[4];
    double xlb[6], xub[6], ulb[2], uub[2];
    double obs[4 * kObcaMaxM];      // cx, cy, w, h
    const double* x0;               // [B][6]
    const double* xgoal;            // [B][6]          (plan mode)
    const double* xref;             // [B][N+1][6]     (track mode)
    const double* uref;             // [B][N][2]       (track mode)
    const double* zg;               // [B][n] reference layout, or nullptr
    double* xout;                   // [B][N+1][6]
    double* uout;                   // [B][N][2]
    double* zout;                   // [B][n] or nullptr
    int* status;                    // [B]
    int* iters;                     // [B] or nullptr
    double* kkt;                    // [B] or nullptr
    double* itout;                  // [B][obca_iterate_len] final primal-dual iterate (diagnostic export) or nullptr
    double* ws;                     // per-instance workspace, obca_ws_doubles(N, M) each
    unsigned long long* stamps;     // [B][kObcaPhases] cycle sums (diagnostics), or nullptr
    // helper workgroups (tt_obca.hip, "helper workgroups"): nhelp extra workgroups after the B instances run the block
    // passes of the instances still solving; board: (B + 1) x kObcaBoardStride words, zeroed before every launch
    unsigned long long* board;
    int nhelp;
    // hand-off diagnostics (ttx_obca_set_handoff_debug): spin limit of an instance waiting for helper chunks in
    // s_memrealtime ticks (0: kSpinTicks, 5 s), and one instance whose hand-offs never complete (-1: none), which
    // forces the TT_HANDOFF_TIMEOUT path (tests/test_gpu_obca.py)
    unsigned long long spin_ticks;
    int fail_b;
};
constexpr int kObcaBoardStride = 16;  // 128-B line per instance (+ one header line)
// claim word of an instance's board line: epoch << 40 | chunks << 20 | next chunk (20 + 20 bits: a pass of
// N = 100000 at M = 16 has 12,501 chunks, and the claim counter overshoots by at most one per claiming workgroup)
constexpr int kClaimChunkShift = 20;
constexpr unsigned long long kClaimFieldMask = (1ull << kClaimChunkShift) - 1ull;
// phase clocks, then event counters (diagnostics, tools/obca_stamps.py / obca_tail.py): factorisations (inertia
// attempts incl. the SOC and pretend-singular refactorisations), restoration-phase iterations, soft-restoration steps,
// refinement corrections, second-order corrections, pretend-singular re-solves, line-search trial points
enum { OPH_LIN = 0, OPH_COMPL, OPH_FACTOR, OPH_RIC, OPH_FWD, OPH_REC, OPH_TRIAL, OPH_UPD, OPH_RIC_SOFT, OPH_FWD_SOFT, OPH_REF_SWEEP, OPH_REF_REC,
       OPH_REF_STAGE, OPH_TOTAL,
       OCNT_FACTOR, OCNT_RESTO_IT, OCNT_SOFT, OCNT_CORR, OCNT_SOC, OCNT_PRETEND, OCNT_TRIAL, kObcaPhases };

// workspace layout (doubles): stage fields [f][k] then block fields [f][j][k], k in 0..N
constexpr int kObcaStageFields = 353;
constexpr int kObcaBlockFields = 229;
__host__ __device__ inline size_t obca_ws_doubles(int N, int M) {
    return (size_t)(kObcaStageFields + kObcaBlockFields * 2 * M) * (size_t)(N + 1);
}
__host__ __device__ inline size_t obca_n(int N, int M) { return (size_t)N * (8 + 16 * M) + 6 + 16 * M; }
// diagnostic export of the final iterate (include/ttmpc.h tt_obca_iterate_len): 30 per stage, 32 per block, 24 final rows
__host__ __device__ inline size_t obca_iterate_len(int N, int M) { return (size_t)(30 + 64 * M) * (N + 1) + 24; }

hipError_t launch_obca(const ObcaArgs& a, hipStream_t stream);

}  // namespace ttmpc
