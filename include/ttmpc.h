/* ttmpc -- MI355X-native batched truck-trailer NMPC solver, C ABI (drop-in boundary).
 *
 * The reference (Avan1ko/car-trailer-mpc) solves one NLP per controller call through CasADi:
 *     sol = self._solver(x0=vars_guess, lbx, ubx, lbg, ubg, p)          python-files/mpc_control.py:80-89
 *     self._solver.stats()['success']                                     python-files/mpc_control.py:106
 * and exposes it to its drivers as
 *     MPCTrackingControl.solve(initial_state, reference_states, reference_inputs)
 *                                                                          python-files/mpc_control.py:67-110
 *     TruckTrailerNMPC.solve(...)                                          python-files/mpc_control_nmpc.py:90-113
 *     MPCTrackingControlFuzzy.solve(...)                                   python-files/mpc_control_fuzzy.py:121-167
 * This library replaces the CasADi/IPOPT call with a batched solve of B independent instances on
 * one GPU.  The Python mirror (car-trailer-mpc_amd/ttmpc) binds it with ctypes; the binding a
 * maintainer adds to the reference is in INTEGRATION.md.
 *
 * Conventions
 *  - plain C types only; every array is C-contiguous float64, instance-major:
 *      x0    [B][nx]            initial_state                      (mpc_control.py:67)
 *      xref  [B][N+1][nx]       reference_states.T                 (p layout, mpc_control.py:45-52, 86)
 *      uref  [B][N][nu]         reference_inputs.T                 (p layout, mpc_control.py:86-87)
 *      wq_wr [B][nx+nu]         fuzzy weights w_q, w_r             (mpc_control_fuzzy.py:54-58) or NULL
 *      z_guess [B][n], n=(nx+nu)N+nx, the reference's interleaved decision vector
 *                               [x0,u0,...,x_{N-1},u_{N-1},x_N]    (trajectory_planning.py:38-58) or NULL
 *                               (NULL = reference-copy guess, mpc_control.py:58-65)
 *      x_out [B][N+1][nx], u_out [B][N][nu]  = states.T / inputs.T of _split_decision_variables
 *                                                                  (trajectory_planning.py:62-84)
 *  - nx = 6 (x, y, theta, psi, phi, v), nu = 2 (a, omega)          (truck_trailer_model.py:4-5)
 *  - bounds: +-HUGE_VAL (or |b| >= 1e19) = free (ca.inf in simulation.py:411-414)
 *  - return value: 0 ok, negative errno-style code on API errors (-EINVAL bad dims/pointers,
 *    -ENOMEM, -EIO HIP error, -ENOSYS not built); text from tt_last_error(handle).
 *  - per-instance status: TT_CONVERGED (IPOPT tol), TT_ACCEPTABLE (acceptable_tol x acc_iter),
 *    TT_MAX_ITER, TT_INFEASIBLE (x_init outside the state box -> x_0 = x_init unsatisfiable),
 *    TT_NONFINITE, TT_STEP_FAILED (inertia correction exceeded IPOPT's max_hessian_perturbation 1e20),
 *    TT_HANDOFF_TIMEOUT (OBCA only: an instance waited longer than the spin limit, 5 s, for the helper workgroups
 *    that run chunks of its block passes; a synchronisation failure of the launch, not a numerical one -- the
 *    outputs are the last iterate, possibly partial; INTEGRATION.md "Helper workgroups").
 *    CasADi's stats()['success'] == (status <= TT_ACCEPTABLE).
 *  - a handle is not thread-safe (like the reference objects, which mutate _last_solution); use
 *    one handle per host thread.  Host-pointer calls are synchronous; device-pointer calls are
 *    asynchronous on the given HIP stream.
 *  - GPU only: there is no CPU fallback; tt_create fails (-ENODEV) without a usable gfx950 device.
 */
#ifndef TTMPC_H
#define TTMPC_H

#ifdef __cplusplus
extern "C" {
#endif

enum { TT_CONVERGED = 0, TT_ACCEPTABLE = 1, TT_MAX_ITER = 2, TT_INFEASIBLE = 3, TT_NONFINITE = 4,
       TT_STEP_FAILED = 5 /* IPOPT Error_In_Step_Computation: delta_w > max_hessian_perturbation (1e20) */,
       TT_HANDOFF_TIMEOUT = 6 /* OBCA helper hand-off timed out (no IPOPT counterpart; see above) */ };

enum {
    TT_VARIANT_TRACK = 0,      /* MPCTrackingControl       mpc_control.py       (max_iter 5000, tol 1e-8)  */
    TT_VARIANT_TRACK_OBCA = 1, /* MPCTrackingControlObs    mpc_control_obs.py   (max_iter 5000, tol 1e-8)  */
    TT_VARIANT_NMPC = 2,       /* TruckTrailerNMPC         mpc_control_nmpc.py  (tol 1e-3, acc 1e-2 x5)    */
    TT_VARIANT_FUZZY = 3,      /* MPCTrackingControlFuzzy  mpc_control_fuzzy.py (tol 1e-3, per-instance w) */
    TT_VARIANT_OBCA_PLAN = 4   /* TrajectoryOptimization   trajectory_optimization.py (max_iter 5000)      */
};

typedef struct {
    int nx, nu, N, M;                 /* nx=6, nu=2, horizon N (params['horizon']), obstacles M       */
    double dt, L1, L2, Mh, W1, W2;    /* params dict keys dt, L1, L2, M, W1, W2 (simulation.py:391)  */
    int variant;                      /* TT_VARIANT_*                                                 */
    double tol, acc_tol;              /* IPOPT tol / acceptable_tol (<=0 -> variant default)          */
    int max_iter, acc_iter;           /* IPOPT max_iter / acceptable_iter (<=0 -> variant default)    */
    int warm_shift_compat;            /* reserved: warm-shift guesses are built host-side (ttmpc.nlp) */
    int dual_init;                    /* OBCA variants: 1 = start mu/lam from the separating-axis
                                         certificate of each body/obstacle pair at the guess pose,
                                         0 = from z_guess's mu/lam as the reference does            */
} tt_config;

/* Replaces the controller constructors (mpc_control.py:6-15 -> _build_solver 27-56; the CasADi
 * graph + IPOPT object).  Q: nx*nx row-major, R: nu*nu row-major (symmetrised), bounds nx / nu.
 * obstacles: M*4 (cx, cy, w, h) or NULL.  device: HIP device ordinal (>= 0). */
int tt_create(const tt_config* cfg, const double* Q, const double* R, const double* xlb, const double* xub,
              const double* ulb, const double* uub, const double* obstacles, int device, void** handle);

/* Replaces the per-call IPOPT solve + split (mpc_control.py:67-110) for B instances at once.
 * Host pointers; synchronous.  kkt_res (may be NULL): IPOPT's scaled optimality error at exit. */
int tt_solve_batch(void* handle, int B, const double* x0, const double* xref, const double* uref,
                   const double* wq_wr, const double* z_guess, double* x_out, double* u_out, int* status,
                   int* iters, double* kkt_res);

/* Same with DEVICE pointers (already resident in HBM), enqueued on `stream` (hipStream_t; NULL = the
 * default stream, as in every HIP API -- e.g. torch's default stream); asynchronous.  Used by the bench
 * and by device-resident callers. */
int tt_solve_batch_device(void* handle, int B, const double* d_x0, const double* d_xref, const double* d_uref,
                          const double* d_wq_wr, const double* d_z_guess, double* d_x_out, double* d_u_out,
                          int* d_status, int* d_iters, double* d_kkt_res, void* stream);

/* Replaces TrajectoryOptimization.plan (trajectory_optimization.py:311-331) for B scenarios of a
 * TT_VARIANT_OBCA_PLAN handle.  x0, xgoal [B][6] (ca.vertcat(initial_state, goal_state), 316-323);
 * z_guess [B][n], n = N(8+16M)+6+16M, the reference's interleaved [x_k,u_k,mu_k,lam_k] vector
 * (55-91), built host-side as _hybrid_a_star_initial_trajectory does (227-274), or NULL for
 * _generate_initial_trajectory_guess (209-225).  Host pointers; synchronous.  Like plan(), success is
 * reported (status) but never enforced (326-331). */
int tt_plan_batch(void* handle, int B, const double* x0, const double* xgoal, const double* z_guess,
                  double* x_out, double* u_out, int* status, int* iters);

/* Both OBCA variants with every output: z_out [B][n] (x, u, mu, lam; _split_decision_variables,
 * trajectory_optimization.py:277-309) and the scaled KKT error.  Plan variant: xgoal [B][6], xref/uref
 * NULL.  MPC+OBCA variant (mpc_control_obs.py:290-322): xref [B][N+1][6], uref [B][N][2], xgoal NULL;
 * z_guess NULL = _get_initial_guess (216-239).  x_out/u_out/z_out/iters/kkt may be NULL. */
int tt_obca_solve_batch(void* handle, int B, const double* x0, const double* xgoal, const double* xref,
                        const double* uref, const double* z_guess, double* x_out, double* u_out, double* z_out,
                        int* status, int* iters, double* kkt_res);
/* Same with DEVICE pointers, asynchronous on `stream` (NULL = the default stream).  The solver
 * workspace belongs to the handle (grown, never shrunk, when B exceeds its capacity): calls on one
 * handle must be serialised on ONE stream; use one handle per stream for concurrent solves. */
int tt_obca_solve_batch_device(void* handle, int B, const double* d_x0, const double* d_xgoal, const double* d_xref,
                               const double* d_uref, const double* d_z_guess, double* d_x_out, double* d_u_out,
                               double* d_z_out, int* d_status, int* d_iters, double* d_kkt_res, void* stream);
/* decision-vector length n of the OBCA variants, and device workspace bytes one instance needs */
long long tt_obca_n(int N, int M);
long long tt_obca_workspace_bytes(int N, int M);
/* Diagnostic variants of the two calls above that also export each instance's FINAL PRIMAL-DUAL ITERATE, so that
 * IPOPT's optimality error can be re-evaluated independently at the returned point (tests; the reference's IPOPT keeps
 * these multipliers internal -- CasADi returns only their lam_x / lam_g combinations).  iterate_out [B][L],
 * L = tt_obca_iterate_len(N, M) = 30(N+1) + 64M(N+1) + 24 doubles:
 *   per stage k = 0..N (30): x 6, u 2, z_L(x) 6, z_U(x) 6, z_L(u) 2, z_U(u) 2, y of the 6 dynamics rows
 *                            (u, z_L(u), z_U(u) are 0 at k = N);
 *   per OBCA block (k, j), j = 2 obstacle + body, in k-major order (32): mu|lam 8, their bound multipliers 8,
 *                            the 4 rows' slacks s, slack-bound multipliers v_L, v_U and row multipliers y_d;
 *   final-box rows (24, plan variant; zeros otherwise): slacks, v_L, v_U, y of x_N - x_goal.
 * The multipliers are IPOPT's internal ones (bound multipliers >= 0 of the relaxed bounds; rows of the slack form
 * d(x) - s = 0). */
long long tt_obca_iterate_len(int N, int M);
int tt_obca_solve_batch_iterate(void* handle, int B, const double* x0, const double* xgoal, const double* xref,
                                const double* uref, const double* z_guess, double* x_out, double* u_out, double* z_out,
                                int* status, int* iters, double* kkt_res, double* iterate_out);
int tt_obca_solve_batch_iterate_device(void* handle, int B, const double* d_x0, const double* d_xgoal,
                                       const double* d_xref, const double* d_uref, const double* d_z_guess,
                                       double* d_x_out, double* d_u_out, double* d_z_out, int* d_status, int* d_iters,
                                       double* d_kkt_res, double* d_iterate_out, void* stream);

/* ---------------------------------------------------------------------------------------------
 * Closed-loop simulation step, device pointers, asynchronous on `stream`.
 * The per-timestep glue of python-files/simulation.py:484-531 around the solve, batched over B
 * Monte-Carlo instances so that the whole loop stays in HBM:
 *   window -> [collision check] -> [warm start] -> tt_solve_batch_device -> [record] -> plant update.
 * ------------------------------------------------------------------------------------------- */
typedef struct {
    double dt, L1, L2, Mh, W1, W2;     /* params dict (simulation.py:391-397)                         */
    int enable;                        /* ENABLE_DISTURBANCES (simulation.py:21): 0 = update(q, u, p) */
    double friction_coeff;             /* DISTURBANCE_PARAMS (simulation.py:26-32)                    */
    double slippage_coeff;
    double process_noise_std;          /* std of the measurement noise the caller draws (509-513)     */
    double lateral_slip_gain;
    double slip_angle_max;
} tt_plant;

/* Reference window at step k with end padding (simulation.py:486-501) from a plan of Np inputs
 * (plan_x [P][Np+1][6], plan_u [P][Np][2]; P = 1 shared plan or B per-instance plans), and the
 * measured state x_meas = state + meas_noise (simulation.py:509-513; meas_noise NULL = exact state;
 * x_meas NULL = skip).  Outputs xref [B][N+1][6], uref [B][N][2]. */
int tt_sim_window_device(int B, int N, int k, int Np, const double* plan_x, const double* plan_u, int per_instance,
                         const double* state, const double* meas_noise, double* x_meas, double* xref, double* uref,
                         void* stream);
/* Graph-replayable closed-loop step (hipGraph capture of window -> check -> solve -> plant -> log):
 * the step index lives on the device.  tt_sim_window_indexed_device reads k = ks[*step] (the reference's
 * step sequence, precomputed host-side) and the measurement noise noise_all[*step] ([K][B][6] or NULL);
 * tt_sim_log_advance_device writes S[*step+1] = state [K+1][B][6], Ua[*step] = u_applied [K][B][2], the
 * status / iterations / collision flag [K][B] (iters, flag may be NULL), then increments *step. */
int tt_sim_window_indexed_device(int B, int N, const int* ks, const int* step, int Np, const double* plan_x,
                                 const double* plan_u, int per_instance, const double* state, const double* noise_all,
                                 double* x_meas, double* xref, double* uref, void* stream);
int tt_sim_log_advance_device(int B, int* step, const double* state, const double* u_applied, const int* status,
                              const int* iters, const int* flag, double* S, double* Ua, int* Ss, int* Si, int* Sc,
                              void* stream);
/* check_trajectory_collision (simulation.py:363-385) of K poses per instance, pose (b, j) at
 * poses + b*stride_b + j*stride_k (doubles; x, y, theta, psi first), against M axis-aligned obstacles
 * (device [M][4]: cx, cy, w, h).  flag[b] = 1 if any pose's truck or trailer touches an obstacle. */
int tt_collision_device(int B, int K, const double* poses, long long stride_b, int stride_k, const double* obstacles,
                        int M, const tt_plant* p, int* flag, void* stream);
/* update(q, u, params[, DISTURBANCE_PARAMS]) (simulation.py:167-199) in place on state [B][6] with
 * u = u[b*u_stride + 0..1] (u_out of a solve: u_stride = 2N applies inputs[:, 0]).  zero_on_fail:
 * instances with status > TT_ACCEPTABLE apply zero control (simulation_nmpc.py:204-214).
 * u_applied [B][2] (may be NULL) receives the control before friction/slippage scaling. */
int tt_plant_update_device(int B, const tt_plant* p, double* state, const double* u, long long u_stride,
                           const int* status, int zero_on_fail, double* u_applied, void* stream);
/* Closed-loop failure policy of the driver, fused with the plant update (one launch per step):
 * success (status <= TT_ACCEPTABLE): u = u[b*u_stride + 0..1], u_last = u, consecutive = 0.  Failure:
 * failures++, consecutive++, then TT_POLICY_TRACK applies u as returned (simulation.py:519-527),
 * TT_POLICY_NMPC zero control and u_last = 0, stop after 20 consecutive (simulation_nmpc.py:206-216),
 * TT_POLICY_FUZZY u_last, zero after 15 consecutive, stop after 30 (simulation_fuzzy.py:207-221).
 * Stopping (the reference's `break` before update) clears active[b]; inactive instances keep their state.
 * u_last [B][2], consecutive / failures / active [B] are device state owned by the caller (active = 1 and
 * the rest 0 at the start); u_applied [B][2] (may be NULL) receives the applied control. */
enum { TT_POLICY_TRACK = 0, TT_POLICY_NMPC = 1, TT_POLICY_FUZZY = 2 };
int tt_policy_plant_device(int B, const tt_plant* p, int policy, double* state, const double* u, long long u_stride,
                           const int* status, double* u_last, int* consecutive, int* failures, int* active,
                           double* u_applied, void* stream);
/* The NMPC and fuzzy drivers' plant (simulation_nmpc.py:94-105, simulation_fuzzy.py:94-105): the same update plus
 * the process noise inside the plant, q_ += state_noise * dt right after the Euler step (before the lateral slip);
 * those drivers solve from the exact state (no measurement noise).  state_noise [B][6] device, drawn by the caller
 * (the reference draws N(0, process_noise_std) in apply_disturbances), or NULL = none (then identical to the
 * functions above). */
int tt_plant_update_noise_device(int B, const tt_plant* p, double* state, const double* u, long long u_stride,
                                 const int* status, int zero_on_fail, const double* state_noise, double* u_applied,
                                 void* stream);
int tt_policy_plant_noise_device(int B, const tt_plant* p, int policy, double* state, const double* u,
                                 long long u_stride, const int* status, double* u_last, int* consecutive, int* failures,
                                 int* active, const double* state_noise, double* u_applied, void* stream);
/* _compute_fuzzy_weights (mpc_control_fuzzy.py:90-119) per instance from the measured state x [B][6]
 * and the window's reference xref [B][N+1][6] (speed of stage 0): wq_wr [B][8] = (q0..q5, r0, r1), the
 * per-instance weights of a TT_VARIANT_FUZZY solve. */
int tt_fuzzy_weights_device(int B, int N, const double* x, const double* xref, double* wq_wr, void* stream);
/* NMPC / fuzzy warm start (mpc_control_nmpc.py:90-100): z_guess [B][8N+6] = shift(last) where have[b],
 * else the reference-copy guess from xref / uref.  bug_compatible = the reference's last-stage slicing
 * (mpc_control_nmpc.py:83-84). */
int tt_warm_start_device(int B, int N, const double* last, const int* have, const double* xref, const double* uref,
                         int bug_compatible, double* z_guess, void* stream);
/* After a solve: last[b] = pack(x_out[b], u_out[b]) and have[b] = 1 where status <= TT_ACCEPTABLE
 * (the reference keeps _last_solution only on success, mpc_control_nmpc.py:107-111). */
int tt_record_solution_device(int B, int N, const double* x_out, const double* u_out, const int* status, double* last,
                              int* have, void* stream);
/* do_interpolation (simulation.py:201-218) of B plans: state_traj [B][Np+1][6], input_traj [B][Np][2]
 * -> [B][factor*Np+1][6], [B][factor*Np][2]; factor = floor(dt_1 / dt_2) (OBCA dt 0.1 -> MPC 0.05: 2). */
int tt_interpolate_device(int B, int Np, int factor, const double* state_traj, const double* input_traj,
                          double* state_out, double* input_out, void* stream);

/* lqr_distance (LQR_cost.py:7-41) for B instances: A, B of the forward-Euler map at (x_goal, u_goal),
 * P = DARE(A, B, Q, R) symmetrised, score[b] = (x_cur - x_goal)' P (x_cur - x_goal).  Q (6x6), R (2x2) are
 * HOST row-major arrays; x_cur, x_goal [B][6], u_goal [B][2] (may be NULL: the map is linear in u) are device
 * pointers.  P_out [B][36] and iters [B] (doublings used, -1 = not converged in 64) may be NULL. */
int tt_lqr_score_device(int B, const tt_plant* p, const double* Q, const double* R, const double* x_cur,
                        const double* x_goal, const double* u_goal, double* P_out, double* score, int* iters,
                        void* stream);

void tt_destroy(void* handle);
const char* tt_last_error(void* handle);

/* Introspection: LDS bytes one instance needs at horizon N; max horizon supported; version. */
int tt_lds_bytes(int N);
int tt_max_horizon(void);
const char* tt_version(void);

#ifdef __cplusplus
}
#endif
#endif /* TTMPC_H */
