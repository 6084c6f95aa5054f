/* CPU ORACLE for the OBCA NLPs (test infrastructure + bench cpu_baseline only; never linked into
 * the product library).
 *
 * Restates two reference NLPs that share the OBCA collision-avoidance structure:
 *   mode TTO_OBCA_PLAN  : TrajectoryOptimization (python-files/trajectory_optimization.py:9-331)
 *                         goal cost with terminal weight 100 Q (168-183), final box |x_N-g|<=1e-2
 *                         (168-174), OBCA rows (93-166), x/u/mu/lam layout (55-91).
 *   mode TTO_OBCA_TRACK : MPCTrackingControlObs (python-files/mpc_control_obs.py:8-322)
 *                         tracking cost with Q_f = Q (31-41), same OBCA rows (65-138), no final box.
 * Both on top of trajectory_planning.py:28-36 (x_0 = x_init, Euler dynamics) and
 * truck_trailer_model.py:8-72 (model, H-reps, body centres).
 *
 * Decision vector z (reference layout, trajectory_optimization.py:55-91):
 *   stage k<N : [x_k(6), u_k(2), mu_k(8M), lam_k(8M)],  stage N : [x_N(6), mu_N(8M), lam_N(8M)]
 *   n = N(8+16M) + 6 + 16M.  mu/lam slot i*8+[0:4] = truck vs obstacle i, i*8+[4:8] = trailer.
 */
#ifndef TT_OBCA_H
#define TT_OBCA_H
#ifdef __cplusplus
extern "C" {
#endif

#define TTO_MAXM 16
enum { TTO_OBCA_PLAN = 0, TTO_OBCA_TRACK = 1 };

typedef struct {
    int N, M, mode;
    double dt, L1, L2, Mh, W1, W2;  /* params dict (trajectory_animation.py:48-52) */
    double Q[36], R[4];              /* row-major, symmetrised internally */
    double xlb[6], xub[6], ulb[2], uub[2];  /* |b| >= 1e19 = free */
    double obs[4 * TTO_MAXM];        /* cx, cy, w, h per obstacle (get_obstacles.py:20-28 format) */
    double dmin;                     /* 0.2   trajectory_optimization.py:95 */
    double eq_tol;                   /* 1e-5  range of the G'mu + R'A'lam rows (136-139) */
    double fin_tol;                  /* 1e-2  final box (172-173); plan mode only */
    double tfac;                     /* 100   terminal weight factor (180); track mode uses 1 */
    double tol, acc_tol;             /* IPOPT tol / acceptable_tol (defaults 1e-8 / 1e-6) */
    int max_iter, acc_iter;          /* 5000 (trajectory_optimization.py:198) / 15 */
    int dual_init;                   /* 0: start from the guess's mu/lam (reference behaviour);
                                        1: replace them by the separating-axis certificate of each
                                        body/obstacle pair at the guess pose (see tt_obca.c) */
    int opts;                        /* TTO_OPT_* bits (diagnostics / A-B): 1, 2, 4, 32, 64 switch restated features off,
                                        8, 16, 128 switch oracle-only IPOPT features on; 0 = the kernel's algorithm */
} tto_obca_problem;

#define TTO_OPT_NO_RESTO 1       /* no restoration phase: a failed line search takes its last trial step */
#define TTO_OPT_NO_SOFT_RESTO 2  /* no soft restoration phase */
#define TTO_OPT_NO_LSQ_MULT 4    /* constraint multipliers start at 0 instead of the least-squares estimate */
/* IPOPT defaults the GPU kernel also runs (switched OFF by these bits, for A/B runs):
 *   exact block inertia: IPOPT perturbs delta_w until the whole KKT matrix has inertia (n, m, 0); per OBCA block
 *   that is In(A) + In(-T) = (8, 4, 0) (Haynsworth), tested by signed LDL' (DESIGN.md 5);
 *   iterative refinement of every step solve on the un-condensed system (min_refinement_steps 1,
 *   max_refinement_steps 10, residual_ratio_max 1e-10, residual_improvement_factor 1). */
#define TTO_OPT_PD_BLOCKS 32     /* round-2 sufficient test instead: every block's A positive definite */
#define TTO_OPT_NO_REFINE 64     /* no iterative refinement */
/* opt-in IPOPT features restated in the oracle only (A/B on the C4 census); the GPU kernel does not
 * run them, so GPU-vs-oracle parity uses opts without these bits */
#define TTO_OPT_KAPPA_D 8        /* kappa_d = 1e-5 linear damping of variables / slacks with one finite bound */
#define TTO_OPT_WATCHDOG 16      /* watchdog (trigger 10 shortened steps, 3 trial iterations) in the line search */
#define TTO_OPT_BLOCK_MW 128     /* a block with indefinite A eliminated rows-first through M_w = A + Jw' E^-1 Jw */
#define TTO_OPT_GLOBAL_INERTIA 256 /* inertia counted over the whole factorisation (blocks, Riccati G_k, soft M_k) */
#define TTO_OPT_R3_PERTURB 512   /* round 3's inertia correction (delta_x only, from 0 on every matrix; raw-residual
                                    refinement stop) instead of IPOPT's perturbation handler (delta_c, degeneracy) */

/* x_init (6); plan mode: x_goal (6); track mode: xref ((N+1)*6), uref (N*2).
 * z_guess (n) or NULL (plan: _generate_initial_trajectory_guess 209-225; track: reference copy +
 * dual pattern, mpc_control_obs.py:216-239).  z_out (n).  Returns per-instance status
 * (0 converged, 1 acceptable, 2 max_iter, 3 infeasible x_init or restoration converged to a point of local
 * infeasibility, 4 non-finite, 5 step computation failed). */
int tto_obca_solve(const tto_obca_problem* P, const double* x_init, const double* x_goal, const double* xref,
                   const double* uref, const double* z_guess, double* z_out, int* iters, double* kkt);

/* OpenMP over instances; arrays instance-major; x_goal/xref/uref/z_guess may be NULL per mode. */
int tto_obca_solve_batch(const tto_obca_problem* P, int B, const double* x_init, const double* x_goal,
                         const double* xref, const double* uref, const double* z_guess, double* z_out,
                         int* status, int* iters, double* kkt, int nthreads);

/* Same, plus the final primal-dual iterate of every instance (it_out [B][tto_obca_iterate_len], or NULL) in the layout
 * of the GPU library's diagnostic export (tt_obca_solve_batch_iterate in include/ttmpc.h). */
int tto_obca_solve_batch_it(const tto_obca_problem* P, int B, const double* x_init, const double* x_goal,
                            const double* xref, const double* uref, const double* z_guess, double* z_out,
                            int* status, int* iters, double* kkt, double* it_out, int nthreads);
long long tto_obca_iterate_len(int N, int M);
/* IPOPT's optimality error (scaled E_0; unscaled dual infeasibility, primal infeasibility, complementarity; s_d, s_c;
 * the converged / acceptable verdicts of IPOPT's convergence check) at a given primal-dual iterate -- an independent
 * evaluation of the GPU's end point.  out[8]. */
int tto_obca_eval_iterate(const tto_obca_problem* P, const double* x_init, const double* x_goal, const double* xref,
                          const double* uref, const double* it, double* out);

#ifdef __cplusplus
}
#endif
#endif
