/* CPU ORACLE (test infrastructure only; also the bench's cpu_baseline "port").
 *
 * Plain-C restatement of the reference tracking NLP (python-files/mpc_control.py:17-56 on top of
 * python-files/trajectory_planning.py:28-60, model python-files/truck_trailer_model.py:8-29) and
 * of the reference's solver *algorithm*: CasADi nlpsol('ipopt') (mpc_control.py:53), i.e. a
 * primal-dual interior-point method on the full KKT system (IPOPT + MUMPS, unvendored).  Here the
 * KKT matrix is factorised by a banded LU with partial pivoting -- deliberately NOT the Riccati
 * recursion the HIP product uses, so the two are independent implementations of the same NLP.
 *
 * Never linked into the product library (car-trailer-mpc_amd/ttmpc/libttmpc.so).
 */
#ifndef TT_ORACLE_H
#define TT_ORACLE_H
#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    int N;                 /* horizon */
    double dt, L1, L2, Mh; /* params: dt, L1, L2, M (hitch offset) */
    double Q[36];          /* 6x6 row-major state weight (Q_f = Q, mpc_control.py:22) */
    double R[4];           /* 2x2 row-major input weight */
    double xlb[6], xub[6]; /* +-HUGE_VAL = free */
    double ulb[2], uub[2];
    double tol, acc_tol;   /* IPOPT tol / acceptable_tol */
    int max_iter, acc_iter;
} tto_problem;

/* z layout = reference: [x0,u0,x1,u1,...,x_{N-1},u_{N-1},x_N]  (n = 8N+6).
 * status: 0 converged, 1 acceptable, 2 max_iter, 3 infeasible (x_init outside bounds),
 *         4 non-finite.  Returns status. */
int tto_solve(const tto_problem* P, const double* x_init, const double* xref /*(N+1)*6*/,
              const double* uref /*N*2*/, const double* wq /*6 or NULL*/, const double* wr /*2 or NULL*/,
              const double* z_guess /*n or NULL = reference copy*/, double* z_out /*n*/, int* iters,
              double* kkt /* final scaled optimality error, or NULL */);

/* OpenMP over instances (static schedule, one instance per thread at a time).
 * Arrays are instance-major; wq/wr/z_guess may be NULL.  nthreads<=0 -> OpenMP default. */
int tto_solve_batch(const tto_problem* P, int B, const double* x_init, const double* xref,
                    const double* uref, const double* wq, const double* wr, const double* z_guess,
                    double* z_out, int* status, int* iters, double* kkt, int nthreads);

#ifdef __cplusplus
}
#endif
#endif
