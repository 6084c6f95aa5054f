/* CPU ORACLE for the OBCA NLPs -- see tt_obca.h.  Test infrastructure + cpu_baseline only.
 *
 * NLP (restated; citations python-files/<file>:<line>):
 *   variables   x_k (k=0..N), u_k (k<N), mu_k, lam_k >= 0 (k=0..N)      trajectory_optimization.py:55-91
 *   dynamics    x_0 - x_init = 0, x_{k+1} - (x_k + dt f(x_k,u_k)) = 0     trajectory_planning.py:28-36
 *   OBCA rows   per stage k, obstacle i, body b in {truck, trailer}:      trajectory_optimization.py:93-166
 *     d1 = g_b'mu - (A_i p_b(x) - b_i)'lam + d_min <= 0
 *     d2,d3 = G_b'mu + R_b(x)' A_i' lam in [-1e-5, 1e-5]
 *     d4 = ||A_i' lam||_2 - 1 <= 0
 *     with A_i = [I;-I], b_i = [w/2,h/2,w/2,h/2] + A_i c_i (32-53), G_b = [I;-I], g_b = [L/2,W/2,L/2,W/2]
 *     and p_b / R_b the body centre / rotation of truck_trailer_model.py:31-72.
 *   plan  : J = sum_{k<N} u'Ru + (x-g)'Q(x-g) + (x_N-g)'(100Q)(x_N-g), |x_N - g| <= 1e-2  (168-183)
 *   track : J = sum_{k<N} (u-ur)'R(u-ur) + (x-xr)'Q(x-xr) + (x_N-xr_N)'Q(x_N-xr_N)   mpc_control_obs.py:31-41
 *
 * Algorithm: the reference calls IPOPT with its defaults (trajectory_optimization.py:195-205,
 * mpc_control_obs.py:203-211); this file restates that algorithm:
 *   * primal-dual barrier method in slack form (d(x) - s = 0, d_L <= s <= d_U, multipliers y_d and
 *     slack-bound multipliers v_L, v_U): tol 1e-8, acceptable 1e-6 x 15, monotone mu from 0.1,
 *     bound_relax_factor 1e-8 on variable AND constraint bounds, bound_push/frac 1e-2, kappa_sigma 1e10;
 *   * initial constraint multipliers by least squares (constr_mult_init_max 1000: discarded if larger);
 *   * inertia correction with IPOPT's delta_w schedule (1e-4 / x100 / x8 / /3, cap 1e20) and iterative
 *     refinement of every step (PDFullSpaceSolver: min 1, max 10 steps, residual ratio 1e-10);
 *   * filter line search (Waechter & Biegler 2006) with up to four second-order corrections;
 *   * the soft restoration phase (soft_resto_pderror_reduction_factor 0.9999, max_soft_resto_iters 10);
 *   * the feasibility restoration phase MinC_1Nrm: the restoration NLP
 *         min rho sum(p + n) + zeta/2 ||D_R (xbar - xbar_R)||^2   s.t.  r(xbar, s) - p + n = 0,  p, n >= 0
 *     over every constraint row r (dynamics, OBCA rows, final box) with rho 1000, zeta = sqrt(mu_R),
 *     D_R = diag(min(1, 1/|xbar_R|)), mu_R = max(mu, ||r||_inf), p/n started at the closed-form barrier
 *     minimiser; solved by the same barrier / filter machinery; left when the original infeasibility is
 *     reduced to 0.9 of its value at entry and the point is acceptable to the (augmented) original
 *     filter; bound multipliers then updated with the whole restoration change as one Newton step
 *     (reset to 1 above 1000), constraint multipliers reset to 0 (constr_mult_reset_threshold 0).
 *     A failed step computation activates the restoration phase (IPOPT's fallback mechanism); a failed
 *     restoration line search resets p/n to the closed form (IPOPT's restoration of the restoration).
 *
 * Newton system (new-multiplier form, D = Sigma_s + delta_w):
 *   (W + Sigma_x + dw) dx + J_c' y_c+ + J_d' y_d+ = -grad phi_x
 *   D ds - y_d+ = -grad phi_s,  J_c dx - E_c y_c+ = -r_c,  J_d dx - ds - E_p y_d+ = -(d - s)
 * (E = 0 outside the restoration phase; inside it the eliminated p/n give E = 1/D_p + 1/D_n per row.)
 * Slacks and y_d are eliminated; every OBCA block (8 duals mu/lam, 4 rows) couples only to
 * (X, Y, theta, psi) of its stage: its dual Hessian A = W_ww + Sigma_w + dw and T = E + Jw A^-1 Jw' are factored
 * by signed LDL' and the block is Schur-eliminated into the 6x6 stage Hessian; the remaining stage-wise LQ
 * problem is solved by a Riccati recursion (soft dynamics rows inside the restoration phase:
 * P~ = P - P S M^-1 S P, M = I + S P S, S = E_c^1/2).  Inertia test (IPOPT's (n, m, 0) of the whole KKT matrix,
 * restated by blocks): every block In(A) + In(-T) = (8, 4, 0), every M and every Riccati input block R~ + B'P~B
 * positive definite.  Every step solve is followed by IPOPT's iterative refinement on the un-condensed system.
 * IPOPT's gradient-based NLP scaling is not applied: it is the identity at the bench workloads' starting
 * points (all gradients < 100; DESIGN.md §1, tests/test_obca_oracle.py).
 */
#include "tt_obca.h"

#include <float.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NX 6
#define NU 2
#define NW 8
#define NR 4
#define RELAX 1e-8
#define TTO_MAXF 64
#define RHO 1000.0              /* resto_penalty_parameter */
#define KAPPA_RESTO 0.9         /* required_infeasibility_reduction */
#define BOUND_MULT_RESET 1000.0 /* bound_mult_reset_threshold */
#define CONSTR_MULT_INIT_MAX 1000.0
#define SOFT_RESTO_FACTOR 0.9999
#define WD_TRIGGER 10            /* watchdog_shortened_iter_trigger */
#define WD_TRIAL_MAX 3           /* watchdog_trial_iter_max */
#define KAPPA_D 1e-5            /* kappa_d: linear damping of variables with one finite bound */
#define MAX_SOFT_RESTO 10
/* IPOPT's OptimalityErrorConvergenceCheck defaults (dual_inf_tol, constr_viol_tol, compl_inf_tol and the acceptable
 * ones) and MonotoneMuUpdate's barrier floor min(tol, compl_inf_tol) / (barrier_tol_factor + 1) */
#define DUAL_INF_TOL 1.0
#define CONSTR_VIOL_TOL 1e-4
#define COMPL_INF_TOL 1e-4
#define ACC_DUAL_INF_TOL 1e10
#define ACC_CONSTR_VIOL_TOL 1e-2
#define ACC_COMPL_INF_TOL 1e-2
#define BARRIER_TOL_FACTOR 10.0

static int isfree(double b) { return !isfinite(b) || fabs(b) >= 1e19; }

typedef struct {
    double th[TTO_MAXF], ph[TTO_MAXF];
    int n;
} filter_t;

enum { M_ORIG = 0, M_RESTO = 1 };

/* IPOPT's PDPerturbationHandler state (see ph_new below): degeneracy flags, test status, current / last deltas */
typedef struct {
    int hess, jac, degen, test, gdwi;
    double dx_curr, dx_last, dc_curr, dc_last;
} perturb_t;
static void ph_reset(perturb_t* H);

typedef struct {
    const tto_obca_problem* P;
    int N, M, nbk, nb, n, mode;
    int R;          /* M_ORIG / M_RESTO: which NLP the Newton machinery assembles */
    double kd;      /* kappa_d (0 when switched off) */
    int lsq;        /* least-squares multiplier system: unit Hessian, gradients grad f - z */
    double Qc[36], Rc[4];
    double xl[6], xu[6], ul[2], uu[2];
    char hxl[6], hxu[6], hul[2], huu[2];
    double rL[4], rU[4];
    char hrL[4], hrU[4];
    double fL, fU;
    const double *xinit, *xgoal, *xref, *uref;
    /* iterate */
    double *x, *u, *w, *s, *zLx, *zUx, *zLu, *zUu, *zw, *vL, *vU, *yc, *yd;
    double sf[6], vLf[6], vUf[6], ydf[6];
    /* linearisation */
    double *A, *c, *d, *gx, *gu, *gw, *Wd, *Jx, *Jw, *Hxx, *Hxw, *Hww;
    double df[6];
    double *rc0, *rd0; /* residual rows at the iterate: c - (p - n), d - s - (p - n) */
    double rf0[6];
    /* factorisation */
    double *Dd, *Ed, *L, *V, *Qt, *Rt, *Pm, *G, *H, *K;
    double* Sg;     /* signs of the block LDL' pivots: 8 of A, 4 of T per block (all +1 unless indefinite) */
    double* alt;    /* 1: the block was eliminated rows-first through M_w = A + Jw' E^-1 Jw (TTO_OPT_BLOCK_MW) */
    double Dsf[6], Dfe[6];
    double *Sd, *Mch, *Ptl, *ptl; /* soft dynamics rows (restoration) */
    double *Gsg, *Msg; /* signs of the LDL' pivots of every G_k (2) and M_k (6) (all +1 unless indefinite) */
    int negx;      /* global inertia test: negative pivots beyond IPOPT's (n, m, 0) count, summed over the factorisation */
    /* rhs + step */
    double *qt, *rt, *vv, *rd, *pv, *kf, *Yb, *LT, *Gm, *tv, *rct;
    double rf[6];
    double *dx, *du, *dw, *ds, *ycp, *ydp, *dzLx, *dzUx, *dzLu, *dzUu, *dzw, *dvL, *dvU;
    double dsf[6], ydpf[6], dvLf[6], dvUf[6];
    /* trial + soc */
    double *xt, *ut, *wt, *st, *ct, *dtr, *cr, *dr;
    double sft[6], dft[6];
    /* restoration phase: one elastic pair (p, n) per constraint row.  Row index: dynamics 6k+i,
     * OBCA rows nrc + 4 bi + r, final rows nrc + nrd + i. */
    int nrc, nrd, nrow;
    double rho, zeta;
    double *xR, *uR, *wR, *sR, sfR[6];
    double *dRx, *dRu, *dRw;
    double *pr, *nr, *zp, *zn, *dpr, *dnr, *dzp, *dzn, *prt, *nrt, *Dpr, *Dnr, *gpn;
    /* original multipliers saved at entry into the restoration phase */
    double *szLx, *szUx, *szLu, *szUu, *szw, *svL, *svU, svLf[6], svUf[6];
    /* last acceptable iterate (IPOPT's stored acceptable point) */
    double *xacc, *uacc, *wacc;
    int have_acc;
    /* soft restoration / SOC save area; watchdog save area (iterate + search direction) */
    double* sv;
    double* wdv;
    /* iterative refinement (IPOPT PDFullSpaceSolver): while ov != NULL the stationarity constants of the
     * condensed solve come from these arrays (x u w s sf p n) instead of the barrier gradients */
    double *ov, *ovx, *ovu, *ovw, *ovs, *ovsf, *ovp, *ovn;
    double *rsx, *rsu, *rsw, *rss, *rssf, *rsp, *rsn, *rrc, *rrd, *rrf; /* residuals of the un-condensed rows */
    double *sol;    /* refinement save area of the solution */
    double dw_cur, dc_cur; /* the perturbations (delta_x = delta_s, delta_c = delta_d) of the current factorisation */
    int soft;              /* soft dynamics rows: restoration phase (E = 1/D_p + 1/D_n) and/or delta_c > 0 (E += delta_c) */
    double* csh;           /* the solve's row constants shifted by delta_c y (new-multiplier form of IPOPT's -delta_c dy) */
    int dbg;        /* diagnostics, read once per solve: 1 TTO_DEBUG, 2 TTO_DEBUG2, 4 TTO_CHECK */
    double* cc;     /* refinement row-residual constants */
    double* mem;
} ws_t;

/* ------------------------------------------------------------------ model (truck_trailer_model.py:8-24) */
static void fdyn(const tto_obca_problem* P, const double* x, const double* u, double* fo) {
    const double th = x[2], psi = x[3], phi = x[4], v = x[5], t = tan(phi);
    fo[0] = v * cos(th);
    fo[1] = v * sin(th);
    fo[2] = v * t / P->L1;
    fo[3] = -v * t / P->L1 * (1.0 + P->Mh / P->L2 * cos(psi)) - v * sin(psi) / P->L2;
    fo[4] = u[1];
    fo[5] = u[0];
}

static void jac_A(const tto_obca_problem* P, const double* x, double* A) {
    const double th = x[2], psi = x[3], phi = x[4], v = x[5];
    const double L1 = P->L1, L2 = P->L2, M = P->Mh, dt = P->dt;
    const double t = tan(phi), cphi = cos(phi), c2 = 1.0 / (cphi * cphi), k = 1.0 + M / L2 * cos(psi);
    memset(A, 0, 36 * sizeof(double));
    for (int i = 0; i < 6; ++i) A[i * 6 + i] = 1.0;
    A[0 * 6 + 2] += dt * (-v * sin(th));
    A[0 * 6 + 5] += dt * cos(th);
    A[1 * 6 + 2] += dt * (v * cos(th));
    A[1 * 6 + 5] += dt * sin(th);
    A[2 * 6 + 4] += dt * (v * c2 / L1);
    A[2 * 6 + 5] += dt * (t / L1);
    A[3 * 6 + 3] += dt * (v * t * M * sin(psi) / (L1 * L2) - v * cos(psi) / L2);
    A[3 * 6 + 4] += dt * (-v * c2 / L1 * k);
    A[3 * 6 + 5] += dt * (-t / L1 * k - sin(psi) / L2);
}

/* H += s * sum_i y_i d2 f_i / dx2 */
static void hess_dyn(const tto_obca_problem* P, const double* x, const double* y, double s, double* H) {
    const double th = x[2], psi = x[3], phi = x[4], v = x[5];
    const double L1 = P->L1, L2 = P->L2, M = P->Mh;
    const double sn = sin(th), cs = cos(th), t = tan(phi), cphi = cos(phi), c2 = 1.0 / (cphi * cphi);
    const double sp = sin(psi), cp = cos(psi), k = 1.0 + M / L2 * cp;
    const double h22 = y[0] * (-v * cs) + y[1] * (-v * sn);
    const double h25 = y[0] * (-sn) + y[1] * cs;
    const double h44 = y[2] * (2 * v * t * c2 / L1) + y[3] * (-2 * v * t * c2 * k / L1);
    const double h45 = y[2] * (c2 / L1) + y[3] * (-c2 * k / L1);
    const double h33 = y[3] * (v * t * M * cp / (L1 * L2) + v * sp / L2);
    const double h34 = y[3] * (v * c2 * M * sp / (L1 * L2));
    const double h35 = y[3] * (t * M * sp / (L1 * L2) - cp / L2);
    H[2 * 6 + 2] += s * h22;
    H[2 * 6 + 5] += s * h25; H[5 * 6 + 2] += s * h25;
    H[4 * 6 + 4] += s * h44;
    H[4 * 6 + 5] += s * h45; H[5 * 6 + 4] += s * h45;
    H[3 * 6 + 3] += s * h33;
    H[3 * 6 + 4] += s * h34; H[4 * 6 + 3] += s * h34;
    H[3 * 6 + 5] += s * h35; H[5 * 6 + 3] += s * h35;
}

/* ------------------------------------------------------------------ OBCA block (trajectory_optimization.py:93-166)
 * block j of a stage: obstacle o = j/2, body b = j%2 (0 truck, 1 trailer).  Local duals
 * wv = (mu_0..3, lam_0..3) = z[mu slot o*8+4b+0..3], z[lam slot o*8+4b+0..3].
 * Jx columns: (X, Y, theta, psi).  Hessians are y-weighted (y = the block's 4 row multipliers). */
typedef struct {
    double p[2], dpt[2], dpp[2], ppt[2], ptp[2], ppp[2], ca, sa, angp, hl, hw;
} geom_t;

static void body_geom(const tto_obca_problem* P, const double* xk, int b, geom_t* g) {
    const double X = xk[0], Y = xk[1], th = xk[2], ps = xk[3];
    const double ct = cos(th), st = sin(th);
    if (b == 0) { /* truck centre = rear axle + L1/2 (cos th, sin th)   truck_trailer_model.py:58-61 */
        const double h1 = 0.5 * P->L1;
        g->ca = ct; g->sa = st; g->angp = 0.0; g->hl = 0.5 * P->L1; g->hw = 0.5 * P->W1;
        g->p[0] = X + h1 * ct; g->p[1] = Y + h1 * st;
        g->dpt[0] = -h1 * st; g->dpt[1] = h1 * ct;
        g->dpp[0] = 0.0; g->dpp[1] = 0.0;
        g->ppt[0] = -h1 * ct; g->ppt[1] = -h1 * st;
        g->ptp[0] = g->ptp[1] = g->ppp[0] = g->ppp[1] = 0.0;
    } else {      /* trailer centre = hitch - L2/2 (cos(th+psi), sin(th+psi)), hitch = rear - M (cos, sin)  63-72 */
        const double h2 = 0.5 * P->L2, M = P->Mh, ca = cos(th + ps), sa = sin(th + ps);
        g->ca = ca; g->sa = sa; g->angp = 1.0; g->hl = 0.5 * P->L2; g->hw = 0.5 * P->W2;
        g->p[0] = X - M * ct - h2 * ca; g->p[1] = Y - M * st - h2 * sa;
        g->dpt[0] = M * st + h2 * sa; g->dpt[1] = -M * ct - h2 * ca;
        g->dpp[0] = h2 * sa; g->dpp[1] = -h2 * ca;
        g->ppt[0] = M * ct + h2 * ca; g->ppt[1] = M * st + h2 * sa;
        g->ptp[0] = h2 * ca; g->ptp[1] = h2 * sa;
        g->ppp[0] = h2 * ca; g->ppp[1] = h2 * sa;
    }
}

static void blk_vals(const tto_obca_problem* P, const double* xk, int j, const double* wv, double* dv) {
    geom_t g;
    body_geom(P, xk, j & 1, &g);
    const double* ob = P->obs + 4 * (j >> 1);
    const double cx = ob[0], cy = ob[1], hwo = 0.5 * ob[2], hho = 0.5 * ob[3];
    const double* m = wv;
    const double* l = wv + 4;
    const double a = l[0] - l[2], c = l[1] - l[3];
    dv[0] = g.hl * (m[0] + m[2]) + g.hw * (m[1] + m[3]) -
            ((g.p[0] - cx - hwo) * l[0] + (g.p[1] - cy - hho) * l[1] + (-g.p[0] + cx - hwo) * l[2] +
             (-g.p[1] + cy - hho) * l[3]) + P->dmin;
    dv[1] = (m[0] - m[2]) + g.ca * a + g.sa * c;
    dv[2] = (m[1] - m[3]) - g.sa * a + g.ca * c;
    dv[3] = sqrt(a * a + c * c) - 1.0;
}

static void blk_lin(const tto_obca_problem* P, const double* xk, int j, const double* wv, const double* y, double* dv,
                    double* Jx, double* Jw, double* Hxx, double* Hxw, double* Hww) {
    geom_t g;
    body_geom(P, xk, j & 1, &g);
    const double* ob = P->obs + 4 * (j >> 1);
    const double cx = ob[0], cy = ob[1], hwo = 0.5 * ob[2], hho = 0.5 * ob[3];
    const double* m = wv;
    const double* l = wv + 4;
    const double a = l[0] - l[2], c = l[1] - l[3];
    double nr = sqrt(a * a + c * c);
    const double ex = g.p[0] - cx, ey = g.p[1] - cy;
    dv[0] = g.hl * (m[0] + m[2]) + g.hw * (m[1] + m[3]) -
            ((ex - hwo) * l[0] + (ey - hho) * l[1] + (-ex - hwo) * l[2] + (-ey - hho) * l[3]) + P->dmin;
    dv[1] = (m[0] - m[2]) + g.ca * a + g.sa * c;
    dv[2] = (m[1] - m[3]) - g.sa * a + g.ca * c;
    dv[3] = nr - 1.0;
    if (nr < 1e-12) nr = 1e-12;
    const double e2 = -g.sa * a + g.ca * c, e3 = -g.ca * a - g.sa * c;
    memset(Jx, 0, 16 * sizeof(double));
    memset(Jw, 0, 32 * sizeof(double));
    Jx[0] = -a; Jx[1] = -c;
    Jx[2] = -(a * g.dpt[0] + c * g.dpt[1]);
    Jx[3] = -(a * g.dpp[0] + c * g.dpp[1]);
    Jx[4 + 2] = e2; Jx[4 + 3] = e2 * g.angp;
    Jx[8 + 2] = e3; Jx[8 + 3] = e3 * g.angp;
    /* row 1 */
    Jw[0] = g.hl; Jw[1] = g.hw; Jw[2] = g.hl; Jw[3] = g.hw;
    Jw[4] = -(ex - hwo); Jw[5] = -(ey - hho); Jw[6] = ex + hwo; Jw[7] = ey + hho;
    /* row 2 */
    Jw[8 + 0] = 1.0; Jw[8 + 2] = -1.0;
    Jw[8 + 4] = g.ca; Jw[8 + 5] = g.sa; Jw[8 + 6] = -g.ca; Jw[8 + 7] = -g.sa;
    /* row 3 */
    Jw[16 + 1] = 1.0; Jw[16 + 3] = -1.0;
    Jw[16 + 4] = -g.sa; Jw[16 + 5] = g.ca; Jw[16 + 6] = g.sa; Jw[16 + 7] = -g.ca;
    /* row 4 */
    Jw[24 + 4] = a / nr; Jw[24 + 5] = c / nr; Jw[24 + 6] = -a / nr; Jw[24 + 7] = -c / nr;
    if (!y) return;
    const double y1 = y[0], y2 = y[1], y3 = y[2], y4 = y[3];
    /* x-x (only theta/psi) */
    memset(Hxx, 0, 16 * sizeof(double));
    const double rot = y2 * (-g.ca * a - g.sa * c) + y3 * (g.sa * a - g.ca * c);
    Hxx[2 * 4 + 2] = -y1 * (a * g.ppt[0] + c * g.ppt[1]) + rot;
    Hxx[2 * 4 + 3] = -y1 * (a * g.ptp[0] + c * g.ptp[1]) + rot * g.angp;
    Hxx[3 * 4 + 2] = Hxx[2 * 4 + 3];
    Hxx[3 * 4 + 3] = -y1 * (a * g.ppp[0] + c * g.ppp[1]) + rot * g.angp;
    /* x-w (only lam columns 4..7) */
    memset(Hxw, 0, 32 * sizeof(double));
    Hxw[0 * 8 + 4] = -y1; Hxw[0 * 8 + 6] = y1;
    Hxw[1 * 8 + 5] = -y1; Hxw[1 * 8 + 7] = y1;
    const double r0 = -y2 * g.sa - y3 * g.ca, r1 = y2 * g.ca - y3 * g.sa; /* d(y2 e2 + y3 e3)/d(a,c) */
    Hxw[2 * 8 + 4] = -y1 * g.dpt[0] + r0; Hxw[2 * 8 + 5] = -y1 * g.dpt[1] + r1;
    Hxw[2 * 8 + 6] = y1 * g.dpt[0] - r0;  Hxw[2 * 8 + 7] = y1 * g.dpt[1] - r1;
    Hxw[3 * 8 + 4] = -y1 * g.dpp[0] + g.angp * r0; Hxw[3 * 8 + 5] = -y1 * g.dpp[1] + g.angp * r1;
    Hxw[3 * 8 + 6] = y1 * g.dpp[0] - g.angp * r0;  Hxw[3 * 8 + 7] = y1 * g.dpp[1] - g.angp * r1;
    /* lam-lam: y4 T' H4 T, H4 = (1/n^3)[[c^2,-ac],[-ac,a^2]], T = [[1,0,-1,0],[0,1,0,-1]] */
    const double n3 = nr * nr * nr, haa = y4 * c * c / n3, hac = -y4 * a * c / n3, hcc = y4 * a * a / n3;
    const double T[2][4] = {{1, 0, -1, 0}, {0, 1, 0, -1}};
    for (int i = 0; i < 4; ++i)
        for (int k = 0; k < 4; ++k)
            Hww[i * 4 + k] = T[0][i] * (haa * T[0][k] + hac * T[1][k]) + T[1][i] * (hac * T[0][k] + hcc * T[1][k]);
}

/* ------------------------------------------------------------------ workspace */
static int ws_init(ws_t* W, const tto_obca_problem* P) {
    memset(W, 0, sizeof(*W));
    W->P = P;
    W->N = P->N; W->M = P->M; W->mode = P->mode;
    W->nbk = 2 * P->M;
    W->nb = (P->N + 1) * W->nbk;
    W->n = P->N * (8 + 16 * P->M) + 6 + 16 * P->M;
    W->nrc = 6 * (P->N + 1);
    W->nrd = 4 * W->nb;
    W->nrow = W->nrc + W->nrd + (P->mode == TTO_OBCA_PLAN ? 6 : 0);
    const size_t N1 = (size_t)P->N + 1, N = (size_t)P->N, nb = (size_t)W->nb, nr = (size_t)W->nrow;
    const size_t nsv = N1 * 6 * 4 + N * 2 * 3 + nb * 8 * 2 + nb * 4 * 4 + 2 * nr + 64; /* soft-resto snapshot */
    size_t tot = 0;
    double** slots[256];
    size_t cnts[256];
    int ns = 0;
#define TAKE(ptr, cnt) (slots[ns] = &(ptr), cnts[ns] = (cnt), tot += (cnt), ++ns)
    TAKE(W->x, N1 * 6); TAKE(W->u, N * 2); TAKE(W->w, nb * 8); TAKE(W->s, nb * 4);
    TAKE(W->zLx, N1 * 6); TAKE(W->zUx, N1 * 6); TAKE(W->zLu, N * 2); TAKE(W->zUu, N * 2); TAKE(W->zw, nb * 8);
    TAKE(W->vL, nb * 4); TAKE(W->vU, nb * 4);
    TAKE(W->yc, N1 * 6); TAKE(W->yd, nb * 4);
    TAKE(W->A, N * 36); TAKE(W->c, N1 * 6); TAKE(W->d, nb * 4); TAKE(W->gx, N1 * 6); TAKE(W->gu, N * 2);
    TAKE(W->gw, nb * 8); TAKE(W->Wd, N * 36);
    TAKE(W->Jx, nb * 16); TAKE(W->Jw, nb * 32); TAKE(W->Hxx, nb * 16); TAKE(W->Hxw, nb * 32); TAKE(W->Hww, nb * 16);
    TAKE(W->rc0, N1 * 6); TAKE(W->rd0, nb * 4);
    TAKE(W->Dd, nb * 4); TAKE(W->Ed, nb * 4); TAKE(W->Sg, nb * 12); TAKE(W->alt, nb); TAKE(W->L, nb * 64); TAKE(W->V, nb * 32); TAKE(W->Qt, N1 * 36);
    TAKE(W->Rt, N * 4);
    TAKE(W->Pm, N1 * 36); TAKE(W->G, N * 4); TAKE(W->H, N * 12); TAKE(W->K, N * 12);
    TAKE(W->Sd, N1 * 6); TAKE(W->Mch, N1 * 36); TAKE(W->Ptl, N1 * 36); TAKE(W->ptl, N1 * 6);
    TAKE(W->Gsg, N * 2); TAKE(W->Msg, N1 * 6);
    TAKE(W->qt, N1 * 6); TAKE(W->rt, N * 2); TAKE(W->vv, nb * 8); TAKE(W->rd, nb * 4); TAKE(W->pv, N1 * 6);
    TAKE(W->kf, N * 2); TAKE(W->rct, N1 * 6);
    TAKE(W->dx, N1 * 6); TAKE(W->du, N * 2); TAKE(W->dw, nb * 8); TAKE(W->ds, nb * 4); TAKE(W->ycp, N1 * 6);
    TAKE(W->ydp, nb * 4);
    TAKE(W->dzLx, N1 * 6); TAKE(W->dzUx, N1 * 6); TAKE(W->dzLu, N * 2); TAKE(W->dzUu, N * 2); TAKE(W->dzw, nb * 8);
    TAKE(W->dvL, nb * 4); TAKE(W->dvU, nb * 4);
    TAKE(W->xt, N1 * 6); TAKE(W->ut, N * 2); TAKE(W->wt, nb * 8); TAKE(W->st, nb * 4); TAKE(W->ct, N1 * 6);
    TAKE(W->dtr, nb * 4);
    TAKE(W->cr, N1 * 6); TAKE(W->dr, nb * 4);
    TAKE(W->Yb, nb * 32); TAKE(W->LT, nb * 16); TAKE(W->Gm, nb * 16); TAKE(W->tv, nb * 4);
    TAKE(W->xR, N1 * 6); TAKE(W->uR, N * 2); TAKE(W->wR, nb * 8); TAKE(W->sR, nb * 4);
    TAKE(W->dRx, N1 * 6); TAKE(W->dRu, N * 2); TAKE(W->dRw, nb * 8);
    TAKE(W->pr, nr); TAKE(W->nr, nr); TAKE(W->zp, nr); TAKE(W->zn, nr); TAKE(W->dpr, nr); TAKE(W->dnr, nr);
    TAKE(W->dzp, nr); TAKE(W->dzn, nr); TAKE(W->prt, nr); TAKE(W->nrt, nr); TAKE(W->Dpr, nr); TAKE(W->Dnr, nr);
    TAKE(W->gpn, nr);
    TAKE(W->szLx, N1 * 6); TAKE(W->szUx, N1 * 6); TAKE(W->szLu, N * 2); TAKE(W->szUu, N * 2); TAKE(W->szw, nb * 8);
    TAKE(W->svL, nb * 4); TAKE(W->svU, nb * 4);
    TAKE(W->xacc, N1 * 6); TAKE(W->uacc, N * 2); TAKE(W->wacc, nb * 8);
    TAKE(W->sv, 4 * (N1 * 6 + N * 2 + nb * 8 + nb * 4) + 2 * nr + nsv);
    TAKE(W->wdv, 2 * (N1 * 6 * 4 + N * 2 * 3 + nb * 8 * 2 + nb * 4 * 4 + 4 * nr + 24) + 64);
    TAKE(W->ovx, N1 * 6); TAKE(W->ovu, N * 2); TAKE(W->ovw, nb * 8); TAKE(W->ovs, nb * 4); TAKE(W->ovsf, 6);
    TAKE(W->ovp, nr); TAKE(W->ovn, nr);
    TAKE(W->rsx, N1 * 6); TAKE(W->rsu, N * 2); TAKE(W->rsw, nb * 8); TAKE(W->rss, nb * 4); TAKE(W->rssf, 6);
    TAKE(W->rsp, nr); TAKE(W->rsn, nr); TAKE(W->rrc, N1 * 6); TAKE(W->rrd, nb * 4); TAKE(W->rrf, 6);
    TAKE(W->sol, N1 * 12 + N * 2 + nb * 16 + 12 + 2 * nr);
    TAKE(W->cc, N1 * 6 + nb * 4 + 6);
    TAKE(W->csh, N1 * 6 + nb * 4 + 6);
#undef TAKE
    W->mem = (double*)calloc(tot, sizeof(double));
    if (!W->mem) return -1;
    double* q = W->mem;
    for (int i = 0; i < ns; ++i) { *slots[i] = q; q += cnts[i]; }
    return 0;
}

/* ------------------------------------------------------------------ NLP functions */
static double cost_eval(const ws_t* W, const double* x, const double* u) {
    const tto_obca_problem* P = W->P;
    double F = 0.0;
    for (int k = 0; k <= W->N; ++k) {
        const double* tgt = W->mode == TTO_OBCA_PLAN ? W->xgoal : W->xref + 6 * k;
        const double sc = (k == W->N && W->mode == TTO_OBCA_PLAN) ? P->tfac : 1.0;
        double e[6];
        for (int i = 0; i < 6; ++i) e[i] = x[6 * k + i] - tgt[i];
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) F += sc * e[i] * W->Qc[i * 6 + j] * e[j];
        if (k < W->N) {
            double r[2];
            for (int i = 0; i < 2; ++i) r[i] = u[2 * k + i] - (W->mode == TTO_OBCA_TRACK ? W->uref[2 * k + i] : 0.0);
            for (int i = 0; i < 2; ++i)
                for (int j = 0; j < 2; ++j) F += r[i] * W->Rc[i * 2 + j] * r[j];
        }
    }
    return F;
}

/* restoration objective rho sum(p + n) + zeta/2 ||D_R (xbar - xbar_R)||^2 */
static double resto_obj(const ws_t* W, const double* x, const double* u, const double* w, const double* p,
                        const double* n) {
    double F = 0.0, Q = 0.0;
    for (int i = 0; i < W->nrow; ++i) F += p[i] + n[i];
    for (int i = 0; i < 6 * (W->N + 1); ++i) { const double e = x[i] - W->xR[i]; Q += W->dRx[i] * e * e; }
    for (int i = 0; i < 2 * W->N; ++i) { const double e = u[i] - W->uR[i]; Q += W->dRu[i] * e * e; }
    for (int i = 0; i < 8 * W->nb; ++i) { const double e = w[i] - W->wR[i]; Q += W->dRw[i] * e * e; }
    return W->rho * F + 0.5 * W->zeta * Q;
}

static void obj_grad(ws_t* W) {
    const tto_obca_problem* P = W->P;
    if (W->R == M_RESTO) {
        for (int i = 0; i < 6 * (W->N + 1); ++i) W->gx[i] = W->zeta * W->dRx[i] * (W->x[i] - W->xR[i]);
        for (int i = 0; i < 2 * W->N; ++i) W->gu[i] = W->zeta * W->dRu[i] * (W->u[i] - W->uR[i]);
        for (int i = 0; i < 8 * W->nb; ++i) W->gw[i] = W->zeta * W->dRw[i] * (W->w[i] - W->wR[i]);
        return;
    }
    memset(W->gw, 0, 8 * (size_t)W->nb * sizeof(double));
    for (int k = 0; k <= W->N; ++k) {
        const double* tgt = W->mode == TTO_OBCA_PLAN ? W->xgoal : W->xref + 6 * k;
        const double sc = (k == W->N && W->mode == TTO_OBCA_PLAN) ? P->tfac : 1.0;
        for (int i = 0; i < 6; ++i) {
            double g = 0.0;
            for (int j = 0; j < 6; ++j) g += W->Qc[i * 6 + j] * (W->x[6 * k + j] - tgt[j]);
            W->gx[6 * k + i] = 2.0 * sc * g;
        }
        if (k < W->N)
            for (int i = 0; i < 2; ++i) {
                double g = 0.0;
                for (int j = 0; j < 2; ++j)
                    g += W->Rc[i * 2 + j] * (W->u[2 * k + j] - (W->mode == TTO_OBCA_TRACK ? W->uref[2 * k + j] : 0.0));
                W->gu[2 * k + i] = 2.0 * g;
            }
    }
}

static void dyn_cons(const ws_t* W, const double* x, const double* u, double* c) {
    for (int i = 0; i < 6; ++i) c[i] = x[i] - W->xinit[i];
    for (int k = 0; k < W->N; ++k) {
        double fo[6];
        fdyn(W->P, x + 6 * k, u + 2 * k, fo);
        for (int i = 0; i < 6; ++i) c[6 * (k + 1) + i] = x[6 * (k + 1) + i] - (x[6 * k + i] + W->P->dt * fo[i]);
    }
}

static void obca_cons(const ws_t* W, const double* x, const double* w, double* d, double* df) {
    for (int k = 0; k <= W->N; ++k)
        for (int j = 0; j < W->nbk; ++j) {
            const int bi = k * W->nbk + j;
            blk_vals(W->P, x + 6 * k, j, w + 8 * bi, d + 4 * bi);
        }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) df[i] = x[6 * W->N + i] - W->xgoal[i];
}

/* residual rows r - (p - n) from raw values c, d, df and slacks s, sf (p, n NULL: original residuals) */
static void residuals(const ws_t* W, const double* c, const double* d, const double* s, const double* df,
                      const double* sf, const double* p, const double* n, double* rc, double* rd, double* rf) {
    for (int i = 0; i < W->nrc; ++i) rc[i] = c[i] - (p ? p[i] - n[i] : 0.0);
    for (int i = 0; i < W->nrd; ++i) rd[i] = d[i] - s[i] - (p ? p[W->nrc + i] - n[W->nrc + i] : 0.0);
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            const int ro = W->nrc + W->nrd + i;
            rf[i] = df[i] - sf[i] - (p ? p[ro] - n[ro] : 0.0);
        }
}

static double infeas1(const ws_t* W, const double* rc, const double* rd, const double* rf) {
    double t = 0.0;
    for (int i = 0; i < W->nrc; ++i) t += fabs(rc[i]);
    for (int i = 0; i < W->nrd; ++i) t += fabs(rd[i]);
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) t += fabs(rf[i]);
    return t;
}

/* barrier value over every bounded component (p, n: the restoration's elastic variables, or NULL);
 * returns 0 and sets *bad if any slack is <= 0 */
static double barrier(const ws_t* W, const double* x, const double* u, const double* w, const double* s,
                      const double* sf, const double* p, const double* n, double mu, int* bad) {
    double b = 0.0;
    *bad = 0;
    const double kdm = W->kd * mu;
#define BL(val, lo) do { double t_ = (val) - (lo); if (!(t_ > 0)) { *bad = 1; return 0; } b -= mu * log(t_); } while (0)
#define BU(val, hi) do { double t_ = (hi) - (val); if (!(t_ > 0)) { *bad = 1; return 0; } b -= mu * log(t_); } while (0)
#define DL(val, lo) (b += kdm * ((val) - (lo)))
#define DU(val, hi) (b += kdm * ((hi) - (val)))
    for (int k = 0; k <= W->N; ++k) {
        for (int i = 0; i < 6; ++i) {
            if (W->hxl[i]) BL(x[6 * k + i], W->xl[i]);
            if (W->hxu[i]) BU(x[6 * k + i], W->xu[i]);
            if (W->hxl[i] && !W->hxu[i]) DL(x[6 * k + i], W->xl[i]);
            if (W->hxu[i] && !W->hxl[i]) DU(x[6 * k + i], W->xu[i]);
        }
        if (k < W->N)
            for (int i = 0; i < 2; ++i) {
                if (W->hul[i]) BL(u[2 * k + i], W->ul[i]);
                if (W->huu[i]) BU(u[2 * k + i], W->uu[i]);
                if (W->hul[i] && !W->huu[i]) DL(u[2 * k + i], W->ul[i]);
                if (W->huu[i] && !W->hul[i]) DU(u[2 * k + i], W->uu[i]);
            }
    }
    for (int bi = 0; bi < W->nb; ++bi) {
        for (int e = 0; e < 8; ++e) { BL(w[8 * bi + e], -RELAX); DL(w[8 * bi + e], -RELAX); }
        for (int r = 0; r < 4; ++r) {
            if (W->hrL[r]) BL(s[4 * bi + r], W->rL[r]);
            if (W->hrU[r]) BU(s[4 * bi + r], W->rU[r]);
            if (W->hrL[r] && !W->hrU[r]) DL(s[4 * bi + r], W->rL[r]);
            if (W->hrU[r] && !W->hrL[r]) DU(s[4 * bi + r], W->rU[r]);
        }
    }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) { BL(sf[i], W->fL); BU(sf[i], W->fU); }
    if (p)
        for (int i = 0; i < W->nrow; ++i) { BL(p[i], 0.0); BL(n[i], 0.0); DL(p[i], 0.0); DL(n[i], 0.0); }
#undef BL
#undef BU
#undef DL
#undef DU
    return b;
}

/* ------------------------------------------------------------------ small dense helpers */
/* in-place lower Cholesky, row-major n x n; 0 ok, F_MANY on a negative pivot (one negative eigenvalue too many),
 * F_ZERO on a numerically zero pivot (|s| <= 1e-14 |a_jj|: the matrix is singular to round-off) */
enum { F_OK = 0, F_MANY = 1, F_ZERO = 2, F_FEW = 3 };
static int pivot_fail(double s, double ajj) { return s < -1e-14 * fabs(ajj) ? F_MANY : F_ZERO; }
static int chol(double* a, int n) {
    for (int j = 0; j < n; ++j) {
        double s = a[j * n + j];
        for (int k = 0; k < j; ++k) s -= a[j * n + k] * a[j * n + k];
        if (!(s >= DBL_MIN)) return pivot_fail(s, a[j * n + j]); /* a subnormal pivot counts as zero */
        const double r = sqrt(s);
        a[j * n + j] = r;
        for (int i = j + 1; i < n; ++i) {
            double t = a[i * n + j];
            for (int k = 0; k < j; ++k) t -= a[i * n + k] * a[j * n + k];
            a[i * n + j] = t / r;
        }
    }
    return 0;
}
/* signed Cholesky A = L S L' (S = diag(+-1), L_jj = sqrt|d_j|), no pivoting; identical to chol() on a
 * positive definite matrix (IPOPT's inertia test needs the signs, not definiteness).  Returns the number of negative pivots, -1 on a (numerically) zero pivot. */
/* TTO_CENSUS diagnostic counters (per solve): factorisations, block inertia failures by kind, zero pivots,
 * refinements that stop above IPOPT's residual_ratio_singular 1e-5 */
static _Thread_local long g_cen[10]; /* [8] refinement corrections, [9] refined step solves */
static int schol(double* a, int n, double* S) {
    int neg = 0;
    for (int j = 0; j < n; ++j) {
        const double ajj = a[j * n + j];
        double s = ajj;
        for (int k = 0; k < j; ++k) s -= a[j * n + k] * a[j * n + k] * S[k];
        /* a positive pivot is taken as chol() takes it (a subnormal one counts as zero, as there); a negative one only
         * when it is not numerically zero */
        if (!(s >= DBL_MIN) && !(s < -1e-14 * fabs(ajj))) return -1;
        S[j] = s > 0.0 ? 1.0 : -1.0;
        neg += s < 0.0;
        const double r = sqrt(fabs(s));
        a[j * n + j] = r;
        for (int i = j + 1; i < n; ++i) {
            double t = a[i * n + j];
            for (int k = 0; k < j; ++k) t -= a[i * n + k] * S[k] * a[j * n + k];
            a[i * n + j] = t / (S[j] * r);
        }
    }
    return neg;
}
static void fsub(const double* L, int n, double* b) { /* b <- L^-1 b */
    for (int i = 0; i < n; ++i) {
        double t = b[i];
        for (int k = 0; k < i; ++k) t -= L[i * n + k] * b[k];
        b[i] = t / L[i * n + i];
    }
}
static void bsub(const double* L, int n, double* b) { /* b <- L^-T b */
    for (int i = n - 1; i >= 0; --i) {
        double t = b[i];
        for (int k = i + 1; k < n; ++k) t -= L[k * n + i] * b[k];
        b[i] = t / L[i * n + i];
    }
}

/* b <- (L S L')^-1 b */
static void ssolve(const double* L, const double* S, int n, double* b) {
    fsub(L, n, b);
    for (int i = 0; i < n; ++i) b[i] *= S[i];
    bsub(L, n, b);
}

/* ------------------------------------------------------------------ Newton system */
static double sig_x(const ws_t* W, int k, int i) {
    const double v = W->x[6 * k + i];
    double s = 0.0;
    if (W->hxl[i]) s += W->zLx[6 * k + i] / (v - W->xl[i]);
    if (W->hxu[i]) s += W->zUx[6 * k + i] / (W->xu[i] - v);
    return s;
}
static double sig_u(const ws_t* W, int k, int i) {
    const double v = W->u[2 * k + i];
    double s = 0.0;
    if (W->hul[i]) s += W->zLu[2 * k + i] / (v - W->ul[i]);
    if (W->huu[i]) s += W->zUu[2 * k + i] / (W->uu[i] - v);
    return s;
}
/* gradient of the barrier objective; in the least-squares multiplier mode: grad f - z_L + z_U */
static double bgrad_x(const ws_t* W, int k, int i, double mu) {
    const double v = W->x[6 * k + i];
    double g = W->gx[6 * k + i];
    if (W->lsq) return g - (W->hxl[i] ? W->zLx[6 * k + i] : 0.0) + (W->hxu[i] ? W->zUx[6 * k + i] : 0.0);
    if (W->hxl[i]) g -= mu / (v - W->xl[i]);
    if (W->hxu[i]) g += mu / (W->xu[i] - v);
    if (W->hxl[i] != W->hxu[i]) g += W->hxl[i] ? W->kd * mu : -W->kd * mu;
    return g;
}
static double bgrad_u(const ws_t* W, int k, int i, double mu) {
    const double v = W->u[2 * k + i];
    double g = W->gu[2 * k + i];
    if (W->lsq) return g - (W->hul[i] ? W->zLu[2 * k + i] : 0.0) + (W->huu[i] ? W->zUu[2 * k + i] : 0.0);
    if (W->hul[i]) g -= mu / (v - W->ul[i]);
    if (W->huu[i]) g += mu / (W->uu[i] - v);
    if (W->hul[i] != W->huu[i]) g += W->hul[i] ? W->kd * mu : -W->kd * mu;
    return g;
}
static double bgrad_w(const ws_t* W, int v, double mu) {
    if (W->lsq) return W->gw[v] - W->zw[v];
    return W->gw[v] - mu / (W->w[v] + RELAX) + W->kd * mu;
}
static double bgrad_s(const ws_t* W, int bi, int r, double mu) {
    const int v = 4 * bi + r;
    if (W->lsq) return (W->hrL[r] ? -W->vL[v] : 0.0) + (W->hrU[r] ? W->vU[v] : 0.0);
    const double sv = W->s[v];
    double g = 0.0;
    if (W->hrL[r]) g -= mu / (sv - W->rL[r]);
    if (W->hrU[r]) g += mu / (W->rU[r] - sv);
    if (W->hrL[r] != W->hrU[r]) g += W->hrL[r] ? W->kd * mu : -W->kd * mu;
    return g;
}
static double bgrad_sf(const ws_t* W, int i, double mu) {
    if (W->lsq) return -W->vLf[i] + W->vUf[i];
    return -mu / (W->sf[i] - W->fL) + mu / (W->fU - W->sf[i]);
}
static double sig_s(const ws_t* W, int bi, int r) {
    const double sv = W->s[4 * bi + r];
    double s = 0.0;
    if (W->hrL[r]) s += W->vL[4 * bi + r] / (sv - W->rL[r]);
    if (W->hrU[r]) s += W->vU[4 * bi + r] / (W->rU[r] - sv);
    return s;
}

/* linearise at the current iterate (values, Jacobians, y-weighted Hessians) + residual rows */
static void linearise(ws_t* W) {
    const tto_obca_problem* P = W->P;
    obj_grad(W);
    dyn_cons(W, W->x, W->u, W->c);
    for (int k = 0; k < W->N; ++k) {
        jac_A(P, W->x + 6 * k, W->A + 36 * k);
        memset(W->Wd + 36 * k, 0, 36 * sizeof(double));
        hess_dyn(P, W->x + 6 * k, W->yc + 6 * (k + 1), -P->dt, W->Wd + 36 * k);
    }
    for (int k = 0; k <= W->N; ++k)
        for (int j = 0; j < W->nbk; ++j) {
            const int bi = k * W->nbk + j;
            blk_lin(P, W->x + 6 * k, j, W->w + 8 * bi, W->yd + 4 * bi, W->d + 4 * bi, W->Jx + 16 * bi,
                    W->Jw + 32 * bi, W->Hxx + 16 * bi, W->Hxw + 32 * bi, W->Hww + 16 * bi);
        }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) W->df[i] = W->x[6 * W->N + i] - W->xgoal[i];
    const int rs = W->R == M_RESTO;
    residuals(W, W->c, W->d, W->s, W->df, W->sf, rs ? W->pr : NULL, rs ? W->nr : NULL, W->rc0, W->rd0, W->rf0);
}

/* One OBCA block's elimination into its stage Hessian Q (6x6, rows/cols X,Y,theta,psi touched).
 * Local system in (dw, y+):  M = [[A, C'], [C, -E]],  A = W_ww + Sigma_w + dw (8x8), C = Jw (4x8),
 * E = D^-1 (D = Sigma_s + dw; plus 1/D_p + 1/D_n in the restoration phase), coupled to dx^ by
 * b1 = W_wx (8x4) and b2 = Jx (4x4).  With A = L L', Y = L^-1 C', Z = L^-1 b1, T = E + Y'Y = L_T L_T',
 * G = Y'Z - b2, the Schur complement onto dx^ is
 *     W_xx - Z'Z + G' T^-1 G
 * which never forms C' D C: with D ~ 1e10 on the near-equality range rows that product cancels
 * catastrophically, while T stays well conditioned.  Inertia (IPOPT tests the whole KKT matrix): by
 * Haynsworth In(M) = In(A) + In(-T), so the block has the correct inertia (8, 4, 0) iff T has exactly as many
 * negative pivots as A; both are factored by the signed Cholesky A = L S_A L', T = L_T S_T L_T', and every
 * A^-1 / T^-1 carries its sign vector.  That exact test is the default (the GPU kernel runs it too); TTO_OPT_PD_BLOCKS
 * switches back to round 2's sufficient condition A positive definite (S = I), which raises delta_w where IPOPT
 * would not. */
static int block_factor(ws_t* W, int bi, double dw, double dc, double* Q) {
    const double *Jx = W->Jx + 16 * bi, *Jw = W->Jw + 32 * bi;
    double* D = W->Dd + 4 * bi;
    double* E = W->Ed + 4 * bi;
    for (int r = 0; r < 4; ++r) {
        D[r] = W->lsq ? 1.0 : sig_s(W, bi, r) + dw;
        E[r] = 1.0 / D[r] + dc;
        if (W->R == M_RESTO) {
            const int ro = W->nrc + 4 * bi + r;
            E[r] += 1.0 / W->Dpr[ro] + 1.0 / W->Dnr[ro];
        }
    }
    double* Lb = W->L + 64 * bi;
    memset(Lb, 0, 64 * sizeof(double));
    if (!W->lsq)
        for (int a = 0; a < 4; ++a)
            for (int b = 0; b < 4; ++b) Lb[(4 + a) * 8 + 4 + b] = W->Hww[16 * bi + a * 4 + b];
    for (int e = 0; e < 8; ++e) {
        if (W->lsq) { Lb[e * 8 + e] = 1.0; continue; }
        Lb[e * 8 + e] += W->zw[8 * bi + e] / (W->w[8 * bi + e] + RELAX) + dw;
        if (W->R == M_RESTO) Lb[e * 8 + e] += W->zeta * W->dRw[8 * bi + e];
    }
    double* SA = W->Sg + 12 * bi;
    double* ST = SA + 8;
    const int inert = !(W->P->opts & TTO_OPT_PD_BLOCKS);
    int negA = 0;
    W->alt[bi] = 0.0;
    if ((W->P->opts & TTO_OPT_BLOCK_MW) && !W->lsq) {
        for (int e = 0; e < 8; ++e) SA[e] = 1.0;
        for (int r = 0; r < 4; ++r) ST[r] = 1.0;
        double Ab[64];
        memcpy(Ab, Lb, sizeof(Ab));
        if (chol(Lb, 8) != 0) {
            /* A indefinite: the block still has IPOPT's inertia (8, 4, 0) iff M_w = A + Jw' E^-1 Jw > 0;
             * eliminate the rows first (stable Cholesky of M_w; E^-1 moderate where this happens) */
            for (int a = 0; a < 8; ++a)
                for (int b = 0; b < 8; ++b) {
                    double t = Ab[a * 8 + b];
                    for (int r = 0; r < 4; ++r) t += Jw[r * 8 + a] * Jw[r * 8 + b] / E[r];
                    Lb[a * 8 + b] = t;
                }
            if (chol(Lb, 8) != 0) return F_MANY;
            W->alt[bi] = 1.0;
            double* Zb = W->V + 32 * bi;
            for (int q = 0; q < 4; ++q) {
                double col[8];
                for (int a = 0; a < 8; ++a) {
                    double t = W->Hxw[32 * bi + q * 8 + a];
                    for (int r = 0; r < 4; ++r) t += Jw[r * 8 + a] / E[r] * Jx[r * 4 + q];
                    col[a] = t;
                }
                fsub(Lb, 8, col);
                for (int a = 0; a < 8; ++a) Zb[a * 4 + q] = col[a];
            }
            for (int p = 0; p < 4; ++p)
                for (int q = 0; q < 4; ++q) {
                    double t = W->Hxx[16 * bi + p * 4 + q];
                    for (int r = 0; r < 4; ++r) t += Jx[r * 4 + p] / E[r] * Jx[r * 4 + q];
                    for (int a = 0; a < 8; ++a) t -= Zb[a * 4 + p] * Zb[a * 4 + q];
                    Q[p * 6 + q] += t;
                }
            return 0;
        }
    } else if (inert) {
        negA = schol(Lb, 8, SA);
        if (negA < 0) { ++g_cen[3]; return F_ZERO; }
    } else {
        const int f = chol(Lb, 8);
        if (f != 0) return f;
        for (int e = 0; e < 8; ++e) SA[e] = 1.0;
    }
    double *Yb = W->Yb + 32 * bi, *Zb = W->V + 32 * bi, *LT = W->LT + 16 * bi, *Gm = W->Gm + 16 * bi;
    for (int r = 0; r < 4; ++r) {
        double col[8];
        for (int a = 0; a < 8; ++a) col[a] = Jw[r * 8 + a];
        fsub(Lb, 8, col);
        for (int a = 0; a < 8; ++a) Yb[a * 4 + r] = col[a];
    }
    for (int q = 0; q < 4; ++q) {
        double col[8];
        for (int a = 0; a < 8; ++a) col[a] = W->lsq ? 0.0 : W->Hxw[32 * bi + q * 8 + a];
        fsub(Lb, 8, col);
        for (int a = 0; a < 8; ++a) Zb[a * 4 + q] = col[a];
    }
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) {
            double t = (r == c) ? E[r] : 0.0, g = -Jx[r * 4 + c];
            for (int a = 0; a < 8; ++a) { t += Yb[a * 4 + r] * SA[a] * Yb[a * 4 + c]; g += Yb[a * 4 + r] * SA[a] * Zb[a * 4 + c]; }
            LT[r * 4 + c] = t;
            Gm[r * 4 + c] = g;
        }
    if (inert) {
        /* inertia of the block [[A, C'], [C, -E]] = In(A) + In(-T): (8, 4, 0) iff T has as many negative
         * pivots as A (Haynsworth); the stage Riccati then tests the Schur complement onto dx^.  Global test
         * (IPOPT counts the negative eigenvalues of the whole KKT matrix): the block's surplus of negative
         * pivots negA - negT is summed with the Riccati's and must vanish overall */
        const int negT = schol(LT, 4, ST);
        if (negT < 0) { ++g_cen[3]; return F_ZERO; }
        if (W->P->opts & TTO_OPT_GLOBAL_INERTIA) W->negx += negA - negT;
        /* negT > negA: the block has fewer negative eigenvalues than its 4 rows need (IPOPT's "too few negative
         * eigenvalues", which it treats as a singular matrix); negT < negA: too many (negative curvature) */
        else if (negT != negA) { ++g_cen[negT > negA ? 1 : 2]; return negT > negA ? F_FEW : F_MANY; }
    } else {
        /* pd mode: A is positive definite here (negA = 0), so a negative pivot of T leaves the block with too FEW
         * negative eigenvalues by Haynsworth (IPOPT: singular -> delta_c), not too many */
        const int f = chol(LT, 4);
        if (f != 0) return f == F_MANY ? F_FEW : f;
        for (int r = 0; r < 4; ++r) ST[r] = 1.0;
    }
    /* Q += W_xx - Z'Z + G' T^-1 G   (T^-1 G via two triangular solves per column) */
    double TG[16];
    for (int c = 0; c < 4; ++c) {
        double col[4] = {Gm[0 * 4 + c], Gm[1 * 4 + c], Gm[2 * 4 + c], Gm[3 * 4 + c]};
        fsub(LT, 4, col);
        for (int r = 0; r < 4; ++r) col[r] *= ST[r];
        bsub(LT, 4, col);
        for (int r = 0; r < 4; ++r) TG[r * 4 + c] = col[r];
    }
    for (int p = 0; p < 4; ++p)
        for (int q = 0; q < 4; ++q) {
            double t = W->lsq ? 0.0 : W->Hxx[16 * bi + p * 4 + q];
            for (int a = 0; a < 8; ++a) t -= Zb[a * 4 + p] * SA[a] * Zb[a * 4 + q];
            for (int r = 0; r < 4; ++r) t += Gm[r * 4 + p] * TG[r * 4 + q];
            Q[p * 6 + q] += t;
        }
    return 0;
}

/* soft dynamics rows (restoration): M_k = I + S P_k S (Cholesky into Mch), P~_k = P_k - P S M^-1 S P */
static int soften(ws_t* W, int k) {
    const double* Pk = W->Pm + 36 * k;
    double* Pt = W->Ptl + 36 * k;
    if (!W->soft) { memcpy(Pt, Pk, 36 * sizeof(double)); return 0; }
    const double* S = W->Sd + 6 * k;
    double* Mk = W->Mch + 36 * k;
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) Mk[i * 6 + j] = (i == j ? 1.0 : 0.0) + S[i] * Pk[i * 6 + j] * S[j];
    double* Ms = W->Msg + 6 * k;
    if (W->P->opts & TTO_OPT_GLOBAL_INERTIA) {
        /* the soft row pair [[P, -I], [-I, -E]] has inertia (6, 6) iff M > 0; each negative pivot of M is one
         * surplus negative eigenvalue of the KKT matrix */
        const int negM = schol(Mk, 6, Ms);
        if (negM < 0) return F_ZERO;
        W->negx += negM;
    } else {
        const int f = chol(Mk, 6);
        if (f != 0) return f;
        for (int i = 0; i < 6; ++i) Ms[i] = 1.0;
    }
    /* X = M^-1 S P (column by column), P~ = P - (P S) X */
    double X[36];
    for (int j = 0; j < 6; ++j) {
        double col[6];
        for (int i = 0; i < 6; ++i) col[i] = S[i] * Pk[i * 6 + j];
        ssolve(Mk, Ms, 6, col);
        for (int i = 0; i < 6; ++i) X[i * 6 + j] = col[i];
    }
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double t = Pk[i * 6 + j];
            for (int l = 0; l < 6; ++l) t -= Pk[i * 6 + l] * S[l] * X[l * 6 + j];
            Pt[i * 6 + j] = t;
        }
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < i; ++j) Pt[i * 6 + j] = Pt[j * 6 + i] = 0.5 * (Pt[i * 6 + j] + Pt[j * 6 + i]);
    return 0;
}
/* v <- v - S M^-1 S b   (the soft-row correction applied to a vector) */
static void soft_apply(const ws_t* W, int k, const double* b, double* v) {
    const double* S = W->Sd + 6 * k;
    double t[6];
    for (int i = 0; i < 6; ++i) t[i] = S[i] * b[i];
    ssolve(W->Mch + 36 * k, W->Msg + 6 * k, 6, t);
    for (int i = 0; i < 6; ++i) v[i] -= S[i] * t[i];
}

/* matrices: block eliminations, stage Hessians, Riccati factorisation with the perturbations dw (delta_x = delta_s)
 * and dc (delta_c = delta_d: -dc on the diagonal of every constraint row).  F_OK = inertia ok; F_MANY a negative
 * pivot where IPOPT's (n, m, 0) wants a positive one (PerturbForWrongInertia); F_ZERO a numerically zero pivot or
 * F_FEW too few negative eigenvalues (both PerturbForSingularity in IPOPT's PDFullSpaceSolver::SolveOnce, the second
 * after IncreaseQuality fails -- there is no pivot tolerance to raise in this elimination) */
static int factor(ws_t* W, double dw, double dc) {
    const tto_obca_problem* P = W->P;
    const int N = W->N;
    const double dt = P->dt;
    int fz = 0, fm = 0, ff = 0;
    W->negx = 0;
    W->dw_cur = dw;
    W->dc_cur = dc;
    W->soft = W->R == M_RESTO || dc > 0.0;
    ++g_cen[0];
    if (W->R == M_RESTO)
        for (int i = 0; i < W->nrow; ++i) {
            W->Dpr[i] = W->lsq ? 1.0 : W->zp[i] / W->pr[i] + dw;
            W->Dnr[i] = W->lsq ? 1.0 : W->zn[i] / W->nr[i] + dw;
        }
    for (int k = 0; k <= N; ++k) {
        double* Q = W->Qt + 36 * k;
        const double sc = (k == N && W->mode == TTO_OBCA_PLAN) ? P->tfac : 1.0;
        if (W->lsq) {
            for (int i = 0; i < 36; ++i) Q[i] = (i % 7 == 0) ? 1.0 : 0.0;
        } else if (W->R == M_ORIG) {
            for (int i = 0; i < 36; ++i) Q[i] = 2.0 * sc * W->Qc[i] + (k < N ? W->Wd[36 * k + i] : 0.0);
            for (int i = 0; i < 6; ++i) Q[i * 6 + i] += sig_x(W, k, i) + dw;
        } else {
            for (int i = 0; i < 36; ++i) Q[i] = k < N ? W->Wd[36 * k + i] : 0.0;
            for (int i = 0; i < 6; ++i) Q[i * 6 + i] += W->zeta * W->dRx[6 * k + i] + sig_x(W, k, i) + dw;
        }
        for (int j = 0; j < W->nbk; ++j) {
            const int bi = k * W->nbk + j;
            const int f = block_factor(W, bi, dw, dc, Q);
            fm |= f == F_MANY; fz |= f == F_ZERO; ff |= f == F_FEW;
        }
        if (k == N && W->mode == TTO_OBCA_PLAN)
            for (int i = 0; i < 6; ++i) {
                double s = W->lsq ? 1.0 : dw + W->vLf[i] / (W->sf[i] - W->fL) + W->vUf[i] / (W->fU - W->sf[i]);
                W->Dsf[i] = s;
                double E = 1.0 / s + dc;
                if (W->R == M_RESTO) {
                    const int ro = W->nrc + W->nrd + i;
                    E += 1.0 / W->Dpr[ro] + 1.0 / W->Dnr[ro];
                }
                W->Dfe[i] = 1.0 / E;
                Q[i * 6 + i] += W->Dfe[i];
            }
        if (k < N) {
            double* R = W->Rt + 4 * k;
            if (W->lsq) { R[0] = R[3] = 1.0; R[1] = R[2] = 0.0; continue; }
            for (int i = 0; i < 4; ++i) R[i] = W->R == M_ORIG ? 2.0 * W->Rc[i] : 0.0;
            for (int i = 0; i < 2; ++i)
                R[i * 2 + i] += sig_u(W, k, i) + dw + (W->R == M_RESTO ? W->zeta * W->dRu[2 * k + i] : 0.0);
        }
    }
    if (fz | fm | ff) return fz ? F_ZERO : fm ? F_MANY : F_FEW;
    ++g_cen[4]; /* blocks passed: the stage Riccati decides */
    if (W->soft)
        for (int i = 0; i < W->nrc; ++i)
            W->Sd[i] = sqrt((W->R == M_RESTO ? 1.0 / W->Dpr[i] + 1.0 / W->Dnr[i] : 0.0) + dc);
    /* Riccati: P_N = Q~_N; G = R~ + B'P~B, H = B'P~A, K = -G^-1 H, P = Q~ + A'P~A + H'K  (P~ = P unless the
     * dynamics rows are soft) */
    memcpy(W->Pm + 36 * N, W->Qt + 36 * N, 36 * sizeof(double));
    for (int k = N; k >= 1; --k) {
        const int fs = soften(W, k);
        if (fs != 0) return fs;
        const double* Pn = W->Ptl + 36 * k;
        const double* A = W->A + 36 * (k - 1);
        const int kk = k - 1;
        /* B = dt [e5 e4]: rows of B'X = dt * (X row 5, X row 4) */
        double* G = W->G + 4 * kk;
        G[0] = W->Rt[4 * kk + 0] + dt * dt * Pn[5 * 6 + 5];
        G[1] = W->Rt[4 * kk + 1] + dt * dt * Pn[5 * 6 + 4];
        G[2] = W->Rt[4 * kk + 2] + dt * dt * Pn[4 * 6 + 5];
        G[3] = W->Rt[4 * kk + 3] + dt * dt * Pn[4 * 6 + 4];
        double* H = W->H + 12 * kk;
        for (int j = 0; j < 6; ++j) {
            double h0 = 0.0, h1 = 0.0;
            for (int i = 0; i < 6; ++i) { h0 += Pn[5 * 6 + i] * A[i * 6 + j]; h1 += Pn[4 * 6 + i] * A[i * 6 + j]; }
            H[j] = dt * h0;
            H[6 + j] = dt * h1;
        }
        G[1] = G[2] = 0.5 * (G[1] + G[2]);
        double* Gs = W->Gsg + 2 * kk;
        if (P->opts & TTO_OPT_GLOBAL_INERTIA) {
            /* each negative pivot of the reduced input Hessian is one surplus negative eigenvalue */
            const int negG = schol(G, 2, Gs);
            if (negG < 0) return F_ZERO;
            W->negx += negG;
        } else {
            const int f = chol(G, 2);
            if (f != 0) return f;
            Gs[0] = Gs[1] = 1.0;
        }
        double* Kk = W->K + 12 * kk;
        for (int j = 0; j < 6; ++j) {
            double col[2] = {H[j], H[6 + j]};
            ssolve(G, Gs, 2, col);
            Kk[j] = -col[0];
            Kk[6 + j] = -col[1];
        }
        double* Pk = W->Pm + 36 * kk;
        double PA[36];
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                double t = 0.0;
                for (int l = 0; l < 6; ++l) t += Pn[i * 6 + l] * A[l * 6 + j];
                PA[i * 6 + j] = t;
            }
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                double t = W->Qt[36 * kk + i * 6 + j];
                for (int l = 0; l < 6; ++l) t += A[l * 6 + i] * PA[l * 6 + j];
                t += H[i] * Kk[j] + H[6 + i] * Kk[6 + j];
                Pk[i * 6 + j] = t;
            }
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < i; ++j) Pk[i * 6 + j] = Pk[j * 6 + i] = 0.5 * (Pk[i * 6 + j] + Pk[j * 6 + i]);
    }
    const int fs = soften(W, 0);
    if (fs != 0) return fs;
    return W->negx != 0 ? F_MANY : F_OK; /* global inertia test: IPOPT's (n, m, 0) (W->negx stays 0 in the other modes) */
}

/* right-hand side + back-substitution.  cres: dynamics residual rows ((N+1)*6), dres: OBCA residual rows
 * (nb*4), fres: final residual rows (6) -- all in the form r - (p - n) of the current system.
 * Fills dx du dw ds ycp ydp dsf ydpf (and dp dn in the restoration phase). */
static void solve_rhs(ws_t* W, double mu, const double* cres, const double* dres, const double* fres) {
    const tto_obca_problem* P = W->P;
    const int N = W->N;
    const double dt = P->dt;
    const int rs = W->R == M_RESTO;
    if (rs)
        for (int i = 0; i < W->nrow; ++i) {
            const double gp = W->ov ? W->ovp[i] : W->rho - (W->lsq ? W->zp[i] : mu / W->pr[i] - W->kd * mu);
            const double gn = W->ov ? W->ovn[i] : W->rho - (W->lsq ? W->zn[i] : mu / W->nr[i] - W->kd * mu);
            W->gpn[i] = gp / W->Dpr[i] - gn / W->Dnr[i];
        }
    for (int i = 0; i < W->nrc; ++i) W->rct[i] = cres[i] + (rs ? W->gpn[i] : 0.0);
    for (int k = 0; k <= N; ++k) {
        double* q = W->qt + 6 * k;
        for (int i = 0; i < 6; ++i) q[i] = W->ov ? W->ovx[6 * k + i] : bgrad_x(W, k, i, mu);
        for (int j = 0; j < W->nbk; ++j) {
            const int bi = k * W->nbk + j;
            const double *D = W->Dd + 4 * bi, *Yb = W->Yb + 32 * bi, *Zb = W->V + 32 * bi, *Gm = W->Gm + 16 * bi;
            double* rd = W->rd + 4 * bi;
            for (int r = 0; r < 4; ++r)
                rd[r] = dres[4 * bi + r] + (W->ov ? W->ovs[4 * bi + r] : bgrad_s(W, bi, r, mu)) / D[r] +
                        (rs ? W->gpn[W->nrc + 4 * bi + r] : 0.0);
            double* zf = W->vv + 8 * bi;
            for (int a = 0; a < 8; ++a) zf[a] = W->ov ? W->ovw[8 * bi + a] : bgrad_w(W, 8 * bi + a, mu);
            const double *SA = W->Sg + 12 * bi, *ST = SA + 8;
            if (W->alt[bi] != 0.0) {
                const double *Jx = W->Jx + 16 * bi, *Jw = W->Jw + 32 * bi, *E = W->Ed + 4 * bi;
                for (int a = 0; a < 8; ++a)
                    for (int r = 0; r < 4; ++r) zf[a] += Jw[r * 8 + a] / E[r] * rd[r];
                fsub(W->L + 64 * bi, 8, zf);
                for (int p = 0; p < 4; ++p) {
                    double g = 0.0;
                    for (int r = 0; r < 4; ++r) g += Jx[r * 4 + p] / E[r] * rd[r];
                    for (int a = 0; a < 8; ++a) g -= Zb[a * 4 + p] * zf[a];
                    q[p] += g;
                }
                continue;
            }
            fsub(W->L + 64 * bi, 8, zf);
            double* t = W->tv + 4 * bi;
            for (int r = 0; r < 4; ++r) {
                double h = rd[r];
                for (int a = 0; a < 8; ++a) h -= Yb[a * 4 + r] * SA[a] * zf[a];
                t[r] = h;
            }
            fsub(W->LT + 16 * bi, 4, t);
            for (int r = 0; r < 4; ++r) t[r] *= ST[r];
            bsub(W->LT + 16 * bi, 4, t);
            for (int p = 0; p < 4; ++p) {
                double g = 0.0;
                for (int a = 0; a < 8; ++a) g -= Zb[a * 4 + p] * SA[a] * zf[a];
                for (int r = 0; r < 4; ++r) g -= Gm[r * 4 + p] * t[r];
                q[p] += g;
            }
        }
        if (k == N && W->mode == TTO_OBCA_PLAN)
            for (int i = 0; i < 6; ++i) {
                W->rf[i] = fres[i] + (W->ov ? W->ovsf[i] : bgrad_sf(W, i, mu)) / W->Dsf[i] +
                           (rs ? W->gpn[W->nrc + W->nrd + i] : 0.0);
                q[i] += W->Dfe[i] * W->rf[i];
            }
        if (k < N)
            for (int i = 0; i < 2; ++i) W->rt[2 * k + i] = W->ov ? W->ovu[2 * k + i] : bgrad_u(W, k, i, mu);
    }
    /* Riccati vector pass (p~ = p - P S M^-1 S p for soft rows) */
    memcpy(W->pv + 6 * N, W->qt + 6 * N, 6 * sizeof(double));
    for (int k = N;; --k) {
        double* pt = W->ptl + 6 * k;
        memcpy(pt, W->pv + 6 * k, 6 * sizeof(double));
        if (W->soft) {
            double Pp[6];
            for (int i = 0; i < 6; ++i) Pp[i] = W->pv[6 * k + i];
            /* pt -= P S M^-1 S p  */
            const double* S = W->Sd + 6 * k;
            double t[6];
            for (int i = 0; i < 6; ++i) t[i] = S[i] * Pp[i];
            ssolve(W->Mch + 36 * k, W->Msg + 6 * k, 6, t);
            for (int i = 0; i < 6; ++i) {
                double a = 0.0;
                for (int l = 0; l < 6; ++l) a += W->Pm[36 * k + i * 6 + l] * S[l] * t[l];
                pt[i] -= a;
            }
        }
        if (k == 0) break;
        const int kk = k - 1;
        const double* Pn = W->Ptl + 36 * k;
        const double* A = W->A + 36 * kk;
        const double* e = W->rct + 6 * k;
        double pp[6];
        for (int i = 0; i < 6; ++i) {
            double t = pt[i];
            for (int j = 0; j < 6; ++j) t -= Pn[i * 6 + j] * e[j];
            pp[i] = t;
        }
        double g[2] = {W->rt[2 * kk] + dt * pp[5], W->rt[2 * kk + 1] + dt * pp[4]};
        ssolve(W->G + 4 * kk, W->Gsg + 2 * kk, 2, g);
        W->kf[2 * kk] = -g[0];
        W->kf[2 * kk + 1] = -g[1];
        const double* H = W->H + 12 * kk;
        for (int i = 0; i < 6; ++i) {
            double t = W->qt[6 * kk + i];
            for (int l = 0; l < 6; ++l) t += A[l * 6 + i] * pp[l];
            t += H[i] * W->kf[2 * kk] + H[6 + i] * W->kf[2 * kk + 1];
            W->pv[6 * kk + i] = t;
        }
    }
    /* forward sweep: yhat = A dx + B du - r~;  dx = yhat (hard rows) or yhat - S M^-1 S (P yhat + p) */
    for (int i = 0; i < 6; ++i) W->dx[i] = -W->rct[i];
    for (int k = 0; k <= N; ++k) {
        double* dxk = W->dx + 6 * k;
        if (W->soft) {
            double b[6];
            for (int i = 0; i < 6; ++i) {
                double t = W->pv[6 * k + i];
                for (int j = 0; j < 6; ++j) t += W->Pm[36 * k + i * 6 + j] * dxk[j];
                b[i] = t;
            }
            soft_apply(W, k, b, dxk);
        }
        for (int i = 0; i < 6; ++i) {
            double t = W->pv[6 * k + i];
            for (int j = 0; j < 6; ++j) t += W->Pm[36 * k + i * 6 + j] * dxk[j];
            W->ycp[6 * k + i] = -t;
        }
        if (k == N) break;
        const double* Kk = W->K + 12 * k;
        double du0 = W->kf[2 * k], du1 = W->kf[2 * k + 1];
        for (int j = 0; j < 6; ++j) { du0 += Kk[j] * dxk[j]; du1 += Kk[6 + j] * dxk[j]; }
        W->du[2 * k] = du0;
        W->du[2 * k + 1] = du1;
        const double* A = W->A + 36 * k;
        double* dxn = W->dx + 6 * (k + 1);
        for (int i = 0; i < 6; ++i) {
            double t = -W->rct[6 * (k + 1) + i];
            for (int j = 0; j < 6; ++j) t += A[i * 6 + j] * dxk[j];
            dxn[i] = t;
        }
        dxn[5] += dt * du0;
        dxn[4] += dt * du1;
    }
    /* block recovery: y+ = t - T^-1 G dx^,  dw = -L^-T (zf + Z dx^ + Y y+),  ds = D^-1 (y+ - grad phi_s) */
    for (int k = 0; k <= N; ++k)
        for (int j = 0; j < W->nbk; ++j) {
            const int bi = k * W->nbk + j;
            const double *Yb = W->Yb + 32 * bi, *Zb = W->V + 32 * bi, *Gm = W->Gm + 16 * bi, *dxk = W->dx + 6 * k;
            const double* D = W->Dd + 4 * bi;
            const double *SA = W->Sg + 12 * bi, *ST = SA + 8;
            if (W->alt[bi] != 0.0) {
                const double *Jx = W->Jx + 16 * bi, *Jw = W->Jw + 32 * bi, *E = W->Ed + 4 * bi;
                double t8[8];
                for (int a = 0; a < 8; ++a) {
                    double t = W->vv[8 * bi + a];
                    for (int q = 0; q < 4; ++q) t += Zb[a * 4 + q] * dxk[q];
                    t8[a] = t;
                }
                bsub(W->L + 64 * bi, 8, t8);
                for (int a = 0; a < 8; ++a) W->dw[8 * bi + a] = -t8[a];
                double* yp = W->ydp + 4 * bi;
                for (int r = 0; r < 4; ++r) {
                    double t = W->rd[4 * bi + r];
                    for (int a = 0; a < 8; ++a) t += Jw[r * 8 + a] * W->dw[8 * bi + a];
                    for (int q = 0; q < 4; ++q) t += Jx[r * 4 + q] * dxk[q];
                    yp[r] = t / E[r];
                }
                for (int r = 0; r < 4; ++r) W->ds[4 * bi + r] = (yp[r] - (W->ov ? W->ovs[4 * bi + r] : bgrad_s(W, bi, r, mu))) / D[r];
                continue;
            }
            double g4[4];
            for (int r = 0; r < 4; ++r) {
                double t = 0.0;
                for (int q = 0; q < 4; ++q) t += Gm[r * 4 + q] * dxk[q];
                g4[r] = t;
            }
            fsub(W->LT + 16 * bi, 4, g4);
            for (int r = 0; r < 4; ++r) g4[r] *= ST[r];
            bsub(W->LT + 16 * bi, 4, g4);
            double* yp = W->ydp + 4 * bi;
            for (int r = 0; r < 4; ++r) yp[r] = W->tv[4 * bi + r] - g4[r];
            double t8[8];
            for (int a = 0; a < 8; ++a) {
                double t = W->vv[8 * bi + a];
                for (int q = 0; q < 4; ++q) t += Zb[a * 4 + q] * dxk[q];
                for (int r = 0; r < 4; ++r) t += Yb[a * 4 + r] * yp[r];
                t8[a] = SA[a] * t;
            }
            bsub(W->L + 64 * bi, 8, t8);
            for (int a = 0; a < 8; ++a) W->dw[8 * bi + a] = -t8[a];
            for (int r = 0; r < 4; ++r)
                W->ds[4 * bi + r] = (yp[r] - (W->ov ? W->ovs[4 * bi + r] : bgrad_s(W, bi, r, mu))) / D[r];
        }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            W->ydpf[i] = W->Dfe[i] * (W->dx[6 * N + i] + W->rf[i]);
            W->dsf[i] = (W->ydpf[i] - (W->ov ? W->ovsf[i] : bgrad_sf(W, i, mu))) / W->Dsf[i];
        }
    if (rs) /* elastic variables: D_p dp - y+ = -(rho - mu/p),  D_n dn + y+ = -(rho - mu/n) */
        for (int i = 0; i < W->nrow; ++i) {
            const double yp = i < W->nrc ? W->ycp[i] : i < W->nrc + W->nrd ? W->ydp[i - W->nrc] : W->ydpf[i - W->nrc - W->nrd];
            const double gp = W->ov ? W->ovp[i] : W->rho - mu / W->pr[i] + W->kd * mu;
            const double gn = W->ov ? W->ovn[i] : W->rho - mu / W->nr[i] + W->kd * mu;
            W->dpr[i] = (yp - gp) / W->Dpr[i];
            W->dnr[i] = (-yp - gn) / W->Dnr[i];
        }
}

/* ------------------------------------------------------------------ solver */
static void push_into(double* v, double lo, double hi, int hl, int hu) {
    const double k1 = 1e-2, k2 = 1e-2;
    if (hl && hu) {
        const double pl = fmin(k1 * fmax(1.0, fabs(lo)), k2 * (hi - lo));
        const double pu = fmin(k1 * fmax(1.0, fabs(hi)), k2 * (hi - lo));
        *v = fmin(fmax(*v, lo + pl), hi - pu);
    } else if (hl) {
        *v = fmax(*v, lo + k1 * fmax(1.0, fabs(lo)));
    } else if (hu) {
        *v = fmin(*v, hi - k1 * fmax(1.0, fabs(hi)));
    }
}

static void default_guess(const ws_t* W, double* z) {
    /* plan : _generate_initial_trajectory_guess (trajectory_optimization.py:209-225)
     * track: _get_initial_guess (mpc_control_obs.py:216-239) */
    const int N = W->N, M = W->M, st = 8 + 16 * M;
    static const double lam_pat[8] = {100, 105, 110, 115, 100, 105, 110, 115};
    for (int k = 0; k <= N; ++k) {
        double* zk = z + (size_t)k * st;
        for (int i = 0; i < 6; ++i) {
            if (W->mode == TTO_OBCA_PLAN) {
                const double t = (double)k / N;
                zk[i] = k < N ? (1 - t) * W->xinit[i] + t * W->xgoal[i] : W->xgoal[i];
            } else {
                zk[i] = W->xref[6 * k + i];
            }
        }
        int o = 6;
        if (k < N) {
            for (int i = 0; i < 2; ++i) zk[6 + i] = W->mode == TTO_OBCA_TRACK ? W->uref[2 * k + i] : 0.0;
            o = 8;
        }
        for (int e = 0; e < 8 * M; ++e) zk[o + e] = 100.0;
        for (int e = 0; e < 8 * M; ++e) zk[o + 8 * M + e] = lam_pat[e % 8];
    }
}

/* Dual warm start (opt-in, dual_init = 1): for body/obstacle pair j at pose x_k, pick the unit direction
 * n among the 8 face normals (obstacle +-e_x, +-e_y; body +-R e_x, +-R e_y) maximising the separation
 * gap(n) = n'p - h_B(-R'n) - h_O(n), and set lam = 0.99 (n+_x, n+_y, n-_x, n-_y) (so A'lam = 0.99 n),
 * mu = 0.99 (m+_x, m+_y, m-_x, m-_y) with m = -R'n (so G'mu + R'A'lam = 0).  Then d2 = d3 = 0,
 * d4 = -0.01 and d1 = d_min - 0.99 gap(n). */
static void dual_certificate(const tto_obca_problem* P, const double* xk, int j, double* wv) {
    geom_t g;
    body_geom(P, xk, j & 1, &g);
    const double* ob = P->obs + 4 * (j >> 1);
    double best = -INFINITY, bn[2] = {1.0, 0.0};
    for (int c = 0; c < 8; ++c) {
        double n[2];
        const double s = (c & 1) ? -1.0 : 1.0;
        if (c < 4) { n[0] = (c < 2) ? s : 0.0; n[1] = (c < 2) ? 0.0 : s; }
        else if (c < 6) { n[0] = s * g.ca; n[1] = s * g.sa; }      /* R e_x */
        else { n[0] = -s * g.sa; n[1] = s * g.ca; }                 /* R e_y */
        const double mx = -(g.ca * n[0] + g.sa * n[1]), my = -(-g.sa * n[0] + g.ca * n[1]); /* -R'n */
        const double hB = g.hl * fabs(mx) + g.hw * fabs(my);
        const double hO = n[0] * ob[0] + n[1] * ob[1] + 0.5 * ob[2] * fabs(n[0]) + 0.5 * ob[3] * fabs(n[1]);
        const double gap = n[0] * g.p[0] + n[1] * g.p[1] - hB - hO;
        if (gap > best) { best = gap; bn[0] = n[0]; bn[1] = n[1]; }
    }
    const double sc = 0.99;
    const double mx = -(g.ca * bn[0] + g.sa * bn[1]), my = -(-g.sa * bn[0] + g.ca * bn[1]);
    wv[0] = sc * fmax(mx, 0.0); wv[1] = sc * fmax(my, 0.0); wv[2] = sc * fmax(-mx, 0.0); wv[3] = sc * fmax(-my, 0.0);
    wv[4] = sc * fmax(bn[0], 0.0); wv[5] = sc * fmax(bn[1], 0.0); wv[6] = sc * fmax(-bn[0], 0.0); wv[7] = sc * fmax(-bn[1], 0.0);
}

static void unpack(ws_t* W, const double* z) {
    const int N = W->N, M = W->M, st = 8 + 16 * M;
    for (int k = 0; k <= N; ++k) {
        const double* zk = z + (size_t)k * st;
        for (int i = 0; i < 6; ++i) W->x[6 * k + i] = zk[i];
        int o = 6;
        if (k < N) { W->u[2 * k] = zk[6]; W->u[2 * k + 1] = zk[7]; o = 8; }
        for (int j = 0; j < W->nbk; ++j) {
            const int bi = k * W->nbk + j, ob = j >> 1, b = j & 1;
            for (int e = 0; e < 4; ++e) {
                W->w[8 * bi + e] = zk[o + ob * 8 + 4 * b + e];
                W->w[8 * bi + 4 + e] = zk[o + 8 * M + ob * 8 + 4 * b + e];
            }
        }
    }
}

static void pack(const ws_t* W, double* z) {
    const int N = W->N, M = W->M, st = 8 + 16 * M;
    for (int k = 0; k <= N; ++k) {
        double* zk = z + (size_t)k * st;
        for (int i = 0; i < 6; ++i) zk[i] = W->x[6 * k + i];
        int o = 6;
        if (k < N) { zk[6] = W->u[2 * k]; zk[7] = W->u[2 * k + 1]; o = 8; }
        for (int j = 0; j < W->nbk; ++j) {
            const int bi = k * W->nbk + j, ob = j >> 1, b = j & 1;
            for (int e = 0; e < 4; ++e) {
                zk[o + ob * 8 + 4 * b + e] = W->w[8 * bi + e];
                zk[o + 8 * M + ob * 8 + 4 * b + e] = W->w[8 * bi + 4 + e];
            }
        }
    }
}

static void mult_steps(ws_t* W, double mu) {
    const int N = W->N;
    for (int k = 0; k <= N; ++k) {
        for (int i = 0; i < 6; ++i) {
            const int v = 6 * k + i;
            W->dzLx[v] = W->hxl[i] ? mu / (W->x[v] - W->xl[i]) - W->zLx[v] - W->zLx[v] / (W->x[v] - W->xl[i]) * W->dx[v] : 0.0;
            W->dzUx[v] = W->hxu[i] ? mu / (W->xu[i] - W->x[v]) - W->zUx[v] + W->zUx[v] / (W->xu[i] - W->x[v]) * W->dx[v] : 0.0;
        }
        if (k < N)
            for (int i = 0; i < 2; ++i) {
                const int v = 2 * k + i;
                W->dzLu[v] = W->hul[i] ? mu / (W->u[v] - W->ul[i]) - W->zLu[v] - W->zLu[v] / (W->u[v] - W->ul[i]) * W->du[v] : 0.0;
                W->dzUu[v] = W->huu[i] ? mu / (W->uu[i] - W->u[v]) - W->zUu[v] + W->zUu[v] / (W->uu[i] - W->u[v]) * W->du[v] : 0.0;
            }
    }
    for (int bi = 0; bi < W->nb; ++bi) {
        for (int e = 0; e < 8; ++e) {
            const int v = 8 * bi + e;
            const double sl = W->w[v] + RELAX;
            W->dzw[v] = mu / sl - W->zw[v] - W->zw[v] / sl * W->dw[v];
        }
        for (int r = 0; r < 4; ++r) {
            const int v = 4 * bi + r;
            W->dvL[v] = W->hrL[r] ? mu / (W->s[v] - W->rL[r]) - W->vL[v] - W->vL[v] / (W->s[v] - W->rL[r]) * W->ds[v] : 0.0;
            W->dvU[v] = W->hrU[r] ? mu / (W->rU[r] - W->s[v]) - W->vU[v] + W->vU[v] / (W->rU[r] - W->s[v]) * W->ds[v] : 0.0;
        }
    }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            W->dvLf[i] = mu / (W->sf[i] - W->fL) - W->vLf[i] - W->vLf[i] / (W->sf[i] - W->fL) * W->dsf[i];
            W->dvUf[i] = mu / (W->fU - W->sf[i]) - W->vUf[i] + W->vUf[i] / (W->fU - W->sf[i]) * W->dsf[i];
        }
    if (W->R == M_RESTO)
        for (int i = 0; i < W->nrow; ++i) {
            W->dzp[i] = mu / W->pr[i] - W->zp[i] - W->zp[i] / W->pr[i] * W->dpr[i];
            W->dzn[i] = mu / W->nr[i] - W->zn[i] - W->zn[i] / W->nr[i] * W->dnr[i];
        }
}

#define FTB_P(val, lo, step, tau, a) do { if ((step) < 0) a = fmin(a, -(tau) * ((val) - (lo)) / (step)); } while (0)
#define FTB_PU(val, hi, step, tau, a) do { if ((step) > 0) a = fmin(a, (tau) * ((hi) - (val)) / (step)); } while (0)
#define FTB_D(zv, step, tau, a) do { if ((step) < 0) a = fmin(a, -(tau) * (zv) / (step)); } while (0)

static double ftb_primal(const ws_t* W, double tau) {
    double a = 1.0;
    for (int k = 0; k <= W->N; ++k) {
        for (int i = 0; i < 6; ++i) {
            const int v = 6 * k + i;
            if (W->hxl[i]) FTB_P(W->x[v], W->xl[i], W->dx[v], tau, a);
            if (W->hxu[i]) FTB_PU(W->x[v], W->xu[i], W->dx[v], tau, a);
        }
        if (k < W->N)
            for (int i = 0; i < 2; ++i) {
                const int v = 2 * k + i;
                if (W->hul[i]) FTB_P(W->u[v], W->ul[i], W->du[v], tau, a);
                if (W->huu[i]) FTB_PU(W->u[v], W->uu[i], W->du[v], tau, a);
            }
    }
    for (int bi = 0; bi < W->nb; ++bi) {
        for (int e = 0; e < 8; ++e) FTB_P(W->w[8 * bi + e], -RELAX, W->dw[8 * bi + e], tau, a);
        for (int r = 0; r < 4; ++r) {
            const int v = 4 * bi + r;
            if (W->hrL[r]) FTB_P(W->s[v], W->rL[r], W->ds[v], tau, a);
            if (W->hrU[r]) FTB_PU(W->s[v], W->rU[r], W->ds[v], tau, a);
        }
    }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            FTB_P(W->sf[i], W->fL, W->dsf[i], tau, a);
            FTB_PU(W->sf[i], W->fU, W->dsf[i], tau, a);
        }
    if (W->R == M_RESTO)
        for (int i = 0; i < W->nrow; ++i) {
            FTB_P(W->pr[i], 0.0, W->dpr[i], tau, a);
            FTB_P(W->nr[i], 0.0, W->dnr[i], tau, a);
        }
    return a;
}

/* TTO_DEBUG: the primal fraction to the boundary per variable class (x u w s sf p n) */
static void ftb_classes(const ws_t* W, double tau, double* c) {
    for (int q = 0; q < 7; ++q) c[q] = 1.0;
    for (int k = 0; k <= W->N; ++k) {
        for (int i = 0; i < 6; ++i) {
            const int v = 6 * k + i;
            if (W->hxl[i]) FTB_P(W->x[v], W->xl[i], W->dx[v], tau, c[0]);
            if (W->hxu[i]) FTB_PU(W->x[v], W->xu[i], W->dx[v], tau, c[0]);
        }
        if (k < W->N)
            for (int i = 0; i < 2; ++i) {
                const int v = 2 * k + i;
                if (W->hul[i]) FTB_P(W->u[v], W->ul[i], W->du[v], tau, c[1]);
                if (W->huu[i]) FTB_PU(W->u[v], W->uu[i], W->du[v], tau, c[1]);
            }
    }
    for (int bi = 0; bi < W->nb; ++bi) {
        for (int e = 0; e < 8; ++e) FTB_P(W->w[8 * bi + e], -RELAX, W->dw[8 * bi + e], tau, c[2]);
        for (int r = 0; r < 4; ++r) {
            const int v = 4 * bi + r;
            if (W->hrL[r]) FTB_P(W->s[v], W->rL[r], W->ds[v], tau, c[3]);
            if (W->hrU[r]) FTB_PU(W->s[v], W->rU[r], W->ds[v], tau, c[3]);
        }
    }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            FTB_P(W->sf[i], W->fL, W->dsf[i], tau, c[4]);
            FTB_PU(W->sf[i], W->fU, W->dsf[i], tau, c[4]);
        }
    if (W->R == M_RESTO)
        for (int i = 0; i < W->nrow; ++i) {
            FTB_P(W->pr[i], 0.0, W->dpr[i], tau, c[5]);
            FTB_P(W->nr[i], 0.0, W->dnr[i], tau, c[6]);
        }
}

static double ftb_dual(const ws_t* W, double tau) {
    double a = 1.0;
    for (int k = 0; k <= W->N; ++k) {
        for (int i = 0; i < 6; ++i) {
            const int v = 6 * k + i;
            if (W->hxl[i]) FTB_D(W->zLx[v], W->dzLx[v], tau, a);
            if (W->hxu[i]) FTB_D(W->zUx[v], W->dzUx[v], tau, a);
        }
        if (k < W->N)
            for (int i = 0; i < 2; ++i) {
                const int v = 2 * k + i;
                if (W->hul[i]) FTB_D(W->zLu[v], W->dzLu[v], tau, a);
                if (W->huu[i]) FTB_D(W->zUu[v], W->dzUu[v], tau, a);
            }
    }
    for (int bi = 0; bi < W->nb; ++bi) {
        for (int e = 0; e < 8; ++e) FTB_D(W->zw[8 * bi + e], W->dzw[8 * bi + e], tau, a);
        for (int r = 0; r < 4; ++r) {
            const int v = 4 * bi + r;
            if (W->hrL[r]) FTB_D(W->vL[v], W->dvL[v], tau, a);
            if (W->hrU[r]) FTB_D(W->vU[v], W->dvU[v], tau, a);
        }
    }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            FTB_D(W->vLf[i], W->dvLf[i], tau, a);
            FTB_D(W->vUf[i], W->dvUf[i], tau, a);
        }
    if (W->R == M_RESTO)
        for (int i = 0; i < W->nrow; ++i) {
            FTB_D(W->zp[i], W->dzp[i], tau, a);
            FTB_D(W->zn[i], W->dzn[i], tau, a);
        }
    return a;
}

/* scaled optimality error at the current iterate (IPOPT eq. (5)) of the current system (original or
 * restoration NLP); also the 1-norm primal-dual system error at mu (soft restoration test) */
typedef struct { double E0, Emu, dinf, pinf, c0, sd, sc, pderr; int finite; } opterr_t;

/* IPOPT's convergence tests on an evaluated error (OptimalityErrorConvergenceCheck::CheckConvergence and
 * CurrentIsAcceptable): the scaled error E_0 and the UNSCALED dual infeasibility, constraint violation and
 * complementarity max |z s|.  The constraint violation of the NLP (max |c| and the violation of d(x) against its
 * bounds) is at most pinf = max(|c|, |d(x) - s|) because every slack s lies inside the (relaxed) bounds, and pinf
 * <= E_0, so with tol <= constr_viol_tol that test can only pass where the E_0 test does; pinf stands in for it. */
static int converged(const opterr_t* o, double tol) {
    return o->E0 <= tol && o->dinf <= DUAL_INF_TOL && o->pinf <= CONSTR_VIOL_TOL && o->c0 <= COMPL_INF_TOL;
}
static int acceptable_pt(const opterr_t* o, double acc_tol) {
    return o->E0 <= acc_tol && o->dinf <= ACC_DUAL_INF_TOL && o->pinf <= ACC_CONSTR_VIOL_TOL && o->c0 <= ACC_COMPL_INF_TOL;
}

static opterr_t opt_error(ws_t* W, double mu) {
    const tto_obca_problem* P = W->P;
    const int N = W->N;
    const int rs = W->R == M_RESTO;
    double dinf = 0.0, pinf = 0.0, c0 = 0.0, cmu = 0.0, sy = 0.0, sz = 0.0, d1 = 0.0, p1 = 0.0, cm1 = 0.0;
    long nb_ = 0, my = 0;
    opterr_t o;
    double dcl[8] = {0};
    o.finite = 1;
#define DINF(t, c_) do { const double t_ = (t); dinf = fmax(dinf, fabs(t_)); dcl[c_] = fmax(dcl[c_], fabs(t_)); d1 += fabs(t_); if (!isfinite(t_)) o.finite = 0; } while (0)
#define CMPL(z, sl) do { const double z_ = (z), s_ = (sl); c0 = fmax(c0, fabs(z_ * s_)); cmu = fmax(cmu, fabs(z_ * s_ - mu)); cm1 += fabs(z_ * s_ - mu); sz += z_; ++nb_; } while (0)
    for (int k = 0; k <= N; ++k) {
        double gl[6];
        for (int i = 0; i < 6; ++i) {
            gl[i] = W->gx[6 * k + i] + W->yc[6 * k + i];
            if (k < N)
                for (int r = 0; r < 6; ++r) gl[i] -= W->A[36 * k + r * 6 + i] * W->yc[6 * (k + 1) + r];
            if (k == N && W->mode == TTO_OBCA_PLAN) gl[i] += W->ydf[i];
        }
        for (int j = 0; j < W->nbk; ++j) {
            const int bi = k * W->nbk + j;
            for (int q = 0; q < 4; ++q)
                for (int r = 0; r < 4; ++r) gl[q] += W->Jx[16 * bi + r * 4 + q] * W->yd[4 * bi + r];
            for (int a = 0; a < 8; ++a) {
                double t = W->gw[8 * bi + a] - W->zw[8 * bi + a];
                for (int r = 0; r < 4; ++r) t += W->Jw[32 * bi + r * 8 + a] * W->yd[4 * bi + r];
                DINF(t, 2);
                CMPL(W->zw[8 * bi + a], W->w[8 * bi + a] + RELAX);
            }
            for (int r = 0; r < 4; ++r) {
                const int v = 4 * bi + r;
                DINF(-W->yd[v] - W->vL[v] + W->vU[v], 3);
                pinf = fmax(pinf, fabs(W->rd0[v]));
                p1 += fabs(W->rd0[v]);
                sy += fabs(W->yd[v]); ++my;
                if (W->hrL[r]) CMPL(W->vL[v], W->s[v] - W->rL[r]);
                if (W->hrU[r]) CMPL(W->vU[v], W->rU[r] - W->s[v]);
            }
        }
        for (int i = 0; i < 6; ++i) {
            const int v = 6 * k + i;
            gl[i] += -W->zLx[v] + W->zUx[v];
            DINF(gl[i], 0);
            if (W->hxl[i]) CMPL(W->zLx[v], W->x[v] - W->xl[i]);
            if (W->hxu[i]) CMPL(W->zUx[v], W->xu[i] - W->x[v]);
            pinf = fmax(pinf, fabs(W->rc0[v]));
            p1 += fabs(W->rc0[v]);
            sy += fabs(W->yc[v]); ++my;
        }
        if (k < N)
            for (int i = 0; i < 2; ++i) {
                const int v = 2 * k + i;
                DINF(W->gu[v] - P->dt * W->yc[6 * (k + 1) + (i == 0 ? 5 : 4)] - W->zLu[v] + W->zUu[v], 1);
                if (W->hul[i]) CMPL(W->zLu[v], W->u[v] - W->ul[i]);
                if (W->huu[i]) CMPL(W->zUu[v], W->uu[i] - W->u[v]);
            }
    }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            DINF(-W->ydf[i] - W->vLf[i] + W->vUf[i], 4);
            pinf = fmax(pinf, fabs(W->rf0[i]));
            p1 += fabs(W->rf0[i]);
            sy += fabs(W->ydf[i]); ++my;
            CMPL(W->vLf[i], W->sf[i] - W->fL);
            CMPL(W->vUf[i], W->fU - W->sf[i]);
        }
    if (rs) /* elastic variables: rho - y - z_p = 0, rho + y - z_n = 0 */
        for (int i = 0; i < W->nrow; ++i) {
            const double y = i < W->nrc ? W->yc[i] : i < W->nrc + W->nrd ? W->yd[i - W->nrc] : W->ydf[i - W->nrc - W->nrd];
            DINF(W->rho - y - W->zp[i], 5);
            DINF(W->rho + y - W->zn[i], 6);
            CMPL(W->zp[i], W->pr[i]);
            CMPL(W->zn[i], W->nr[i]);
        }
#undef DINF
#undef CMPL
    if (!isfinite(pinf)) o.finite = 0;
    const double smax = 100.0;
    const double sd = fmax(smax, (sy + sz) / (double)(my + nb_)) / smax;
    const double sc = nb_ ? fmax(smax, sz / (double)nb_) / smax : 1.0;
    o.E0 = fmax(fmax(dinf / sd, pinf), c0 / sc);
    o.Emu = fmax(fmax(dinf / sd, pinf), cmu / sc);
    o.dinf = dinf;
    o.pinf = pinf;
    o.c0 = c0;
    o.sd = sd;
    o.sc = sc;
    o.pderr = d1 + p1 + cm1;
    if (W->dbg & 2) {
        double my_ = 0, mz = 0, mzw = 0, mv = 0;
        for (int i = 0; i < W->nrc; ++i) my_ = fmax(my_, fabs(W->yc[i]));
        double myd = 0; for (int i = 0; i < W->nrd; ++i) myd = fmax(myd, fabs(W->yd[i]));
        for (int i = 0; i < 6 * (N + 1); ++i) mz = fmax(mz, fmax(W->zLx[i], W->zUx[i]));
        for (int i = 0; i < 8 * W->nb; ++i) mzw = fmax(mzw, W->zw[i]);
        for (int i = 0; i < 4 * W->nb; ++i) mv = fmax(mv, fmax(W->vL[i], W->vU[i]));
        fprintf(stderr, "   dinf by class: w %.1e s %.1e x %.1e u %.1e sf %.1e p %.1e n %.1e | |yc| %.1e |yd| %.1e zx %.1e zw %.1e v %.1e sd %.1e\n",
                dcl[2], dcl[3], dcl[0], dcl[1], dcl[4], dcl[5], dcl[6], my_, myd, mz, mzw, mv, sd);
    }
    return o;
}

/* trial point (xt, ut, wt, st, sft, prt, nrt) of the current system: theta (l1 norm of the residual rows,
 * stored into ct / dtr / dft for second-order corrections) and the barrier objective phi */
static void trial_eval(ws_t* W, double mu, double* th, double* ph) {
    int bad = 0;
    const int rs = W->R == M_RESTO;
    const double b = barrier(W, W->xt, W->ut, W->wt, W->st, W->sft, rs ? W->prt : NULL, rs ? W->nrt : NULL, mu, &bad);
    if (bad) { *th = INFINITY; *ph = INFINITY; return; }
    /* raw values into the residual buffers, then subtract slacks / elastic variables in place */
    dyn_cons(W, W->xt, W->ut, W->ct);
    double dfr[6] = {0};
    obca_cons(W, W->xt, W->wt, W->dtr, dfr);
    residuals(W, W->ct, W->dtr, W->st, dfr, W->sft, rs ? W->prt : NULL, rs ? W->nrt : NULL, W->ct, W->dtr, W->dft);
    *th = infeas1(W, W->ct, W->dtr, W->dft);
    *ph = (rs ? resto_obj(W, W->xt, W->ut, W->wt, W->prt, W->nrt) : cost_eval(W, W->xt, W->ut)) + b;
}

static int in_filter(const filter_t* F, double th, double ph) {
    for (int i = 0; i < F->n; ++i)
        if (th >= F->th[i] && ph >= F->ph[i]) return 1;
    return 0;
}

/* add a filter entry; entries it dominates are dropped; when full the oldest is evicted */
static void add_filter(filter_t* F, double th, double ph) {
    int j = 0;
    for (int i = 0; i < F->n; ++i)
        if (!(F->th[i] >= th && F->ph[i] >= ph)) { F->th[j] = F->th[i]; F->ph[j] = F->ph[i]; ++j; }
    F->n = j;
    if (F->n == TTO_MAXF) {
        memmove(F->th, F->th + 1, (TTO_MAXF - 1) * sizeof(double));
        memmove(F->ph, F->ph + 1, (TTO_MAXF - 1) * sizeof(double));
        --F->n;
    }
    F->th[F->n] = th;
    F->ph[F->n] = ph;
    ++F->n;
}

static void clamp_mult(double* z, double sl, double mu) {
    const double ks = 1e10;
    *z = fmax(fmin(*z, ks * mu / sl), mu / (ks * sl));
}

/* ------------------------------------------------------------------ iterate moves */
static void set_trial(ws_t* W, double a) {
    const size_t nx_ = 6 * (size_t)(W->N + 1), nu_ = 2 * (size_t)W->N, nw_ = 8 * (size_t)W->nb, ns_ = 4 * (size_t)W->nb;
    for (size_t i = 0; i < nx_; ++i) W->xt[i] = W->x[i] + a * W->dx[i];
    for (size_t i = 0; i < nu_; ++i) W->ut[i] = W->u[i] + a * W->du[i];
    for (size_t i = 0; i < nw_; ++i) W->wt[i] = W->w[i] + a * W->dw[i];
    for (size_t i = 0; i < ns_; ++i) W->st[i] = W->s[i] + a * W->ds[i];
    for (int i = 0; i < 6; ++i) W->sft[i] = W->sf[i] + a * W->dsf[i];
    if (W->R == M_RESTO)
        for (int i = 0; i < W->nrow; ++i) { W->prt[i] = W->pr[i] + a * W->dpr[i]; W->nrt[i] = W->nr[i] + a * W->dnr[i]; }
}

/* accept the step: primal alpha, constraint multipliers alpha (new-multiplier form), bound multipliers az
 * followed by the kappa_sigma safeguard */
static void take_step(ws_t* W, double mu, double alpha, double az) {
    const int N = W->N;
    const size_t nx_ = 6 * (size_t)(N + 1), nu_ = 2 * (size_t)N, nw_ = 8 * (size_t)W->nb, ns_ = 4 * (size_t)W->nb;
    for (size_t i = 0; i < nx_; ++i) W->x[i] += alpha * W->dx[i];
    for (size_t i = 0; i < nu_; ++i) W->u[i] += alpha * W->du[i];
    for (size_t i = 0; i < nw_; ++i) W->w[i] += alpha * W->dw[i];
    for (size_t i = 0; i < ns_; ++i) W->s[i] += alpha * W->ds[i];
    for (size_t i = 0; i < nx_; ++i) W->yc[i] += alpha * (W->ycp[i] - W->yc[i]);
    for (size_t i = 0; i < ns_; ++i) W->yd[i] += alpha * (W->ydp[i] - W->yd[i]);
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            W->sf[i] += alpha * W->dsf[i];
            W->ydf[i] += alpha * (W->ydpf[i] - W->ydf[i]);
            W->vLf[i] += az * W->dvLf[i];
            W->vUf[i] += az * W->dvUf[i];
            clamp_mult(&W->vLf[i], W->sf[i] - W->fL, mu);
            clamp_mult(&W->vUf[i], W->fU - W->sf[i], mu);
        }
    for (int k = 0; k <= N; ++k) {
        for (int i = 0; i < 6; ++i) {
            const int v = 6 * k + i;
            if (W->hxl[i]) { W->zLx[v] += az * W->dzLx[v]; clamp_mult(&W->zLx[v], W->x[v] - W->xl[i], mu); }
            if (W->hxu[i]) { W->zUx[v] += az * W->dzUx[v]; clamp_mult(&W->zUx[v], W->xu[i] - W->x[v], mu); }
        }
        if (k < N)
            for (int i = 0; i < 2; ++i) {
                const int v = 2 * k + i;
                if (W->hul[i]) { W->zLu[v] += az * W->dzLu[v]; clamp_mult(&W->zLu[v], W->u[v] - W->ul[i], mu); }
                if (W->huu[i]) { W->zUu[v] += az * W->dzUu[v]; clamp_mult(&W->zUu[v], W->uu[i] - W->u[v], mu); }
            }
    }
    for (int bi = 0; bi < W->nb; ++bi) {
        for (int e = 0; e < 8; ++e) {
            const int v = 8 * bi + e;
            W->zw[v] += az * W->dzw[v];
            clamp_mult(&W->zw[v], W->w[v] + RELAX, mu);
        }
        for (int r = 0; r < 4; ++r) {
            const int v = 4 * bi + r;
            if (W->hrL[r]) { W->vL[v] += az * W->dvL[v]; clamp_mult(&W->vL[v], W->s[v] - W->rL[r], mu); }
            if (W->hrU[r]) { W->vU[v] += az * W->dvU[v]; clamp_mult(&W->vU[v], W->rU[r] - W->s[v], mu); }
        }
    }
    if (W->R == M_RESTO)
        for (int i = 0; i < W->nrow; ++i) {
            W->pr[i] += alpha * W->dpr[i];
            W->nr[i] += alpha * W->dnr[i];
            W->zp[i] += az * W->dzp[i];
            W->zn[i] += az * W->dzn[i];
            clamp_mult(&W->zp[i], W->pr[i], mu);
            clamp_mult(&W->zn[i], W->nr[i], mu);
        }
}

/* full iterate snapshot (soft restoration trial), behind the second-order-correction save area */
static void snapshot(ws_t* W, int restore) {
    double* o = W->sv + 4 * (6 * ((size_t)W->N + 1) + 2 * (size_t)W->N + 8 * (size_t)W->nb + 4 * (size_t)W->nb) +
                2 * (size_t)W->nrow;
    const size_t N1 = (size_t)W->N + 1, N = (size_t)W->N, nb = (size_t)W->nb;
#define SV(ptr, cnt) do { if (restore) memcpy(ptr, o, (cnt) * 8); else memcpy(o, ptr, (cnt) * 8); o += (cnt); } while (0)
    SV(W->x, N1 * 6); SV(W->u, N * 2); SV(W->w, nb * 8); SV(W->s, nb * 4);
    SV(W->zLx, N1 * 6); SV(W->zUx, N1 * 6); SV(W->zLu, N * 2); SV(W->zUu, N * 2); SV(W->zw, nb * 8);
    SV(W->vL, nb * 4); SV(W->vU, nb * 4); SV(W->yc, N1 * 6); SV(W->yd, nb * 4);
    SV(W->sf, 6); SV(W->vLf, 6); SV(W->vUf, 6); SV(W->ydf, 6);
#undef SV
}

/* watchdog save area: the iterate and the search direction of the iteration the watchdog started at */
static void wd_save(ws_t* W, int restore) {
    double* o = W->wdv;
    const size_t N1 = (size_t)W->N + 1, N = (size_t)W->N, nb = (size_t)W->nb, nr = (size_t)W->nrow;
    const int rs = W->R == M_RESTO;
#define SV(ptr, cnt) do { if (restore) memcpy(ptr, o, (cnt) * 8); else memcpy(o, ptr, (cnt) * 8); o += (cnt); } while (0)
    SV(W->x, N1 * 6); SV(W->u, N * 2); SV(W->w, nb * 8); SV(W->s, nb * 4);
    SV(W->zLx, N1 * 6); SV(W->zUx, N1 * 6); SV(W->zLu, N * 2); SV(W->zUu, N * 2); SV(W->zw, nb * 8);
    SV(W->vL, nb * 4); SV(W->vU, nb * 4); SV(W->yc, N1 * 6); SV(W->yd, nb * 4);
    SV(W->sf, 6); SV(W->vLf, 6); SV(W->vUf, 6); SV(W->ydf, 6);
    SV(W->dx, N1 * 6); SV(W->du, N * 2); SV(W->dw, nb * 8); SV(W->ds, nb * 4); SV(W->ycp, N1 * 6); SV(W->ydp, nb * 4);
    SV(W->dzLx, N1 * 6); SV(W->dzUx, N1 * 6); SV(W->dzLu, N * 2); SV(W->dzUu, N * 2); SV(W->dzw, nb * 8);
    SV(W->dvL, nb * 4); SV(W->dvU, nb * 4);
    SV(W->dsf, 6); SV(W->ydpf, 6); SV(W->dvLf, 6); SV(W->dvUf, 6);
    if (rs) {
        SV(W->pr, nr); SV(W->nr, nr); SV(W->zp, nr); SV(W->zn, nr);
        SV(W->dpr, nr); SV(W->dnr, nr); SV(W->dzp, nr); SV(W->dzn, nr);
    }
#undef SV
}

/* ------------------------------------------------------------------ restoration phase */
/* closed-form minimiser of rho (p + n) - mu (ln p + ln n) subject to p - n = r  (IPOPT's p/n start) */
static void pn_closed_form(double r, double mu, double rho, double* p, double* n) {
    const double S = sqrt(mu * mu + rho * rho * r * r);
    const double a = mu - rho * r, b = mu + rho * r;
    *n = a >= 0.0 ? (a + S) / (2.0 * rho) : mu * r / (S - a);
    *p = b >= 0.0 ? (b + S) / (2.0 * rho) : -mu * r / (S - b);
}

static double row_resid_max(const ws_t* W) {
    double m = 0.0;
    for (int i = 0; i < W->nrc; ++i) m = fmax(m, fabs(W->rc0[i]));
    for (int i = 0; i < W->nrd; ++i) m = fmax(m, fabs(W->rd0[i]));
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) m = fmax(m, fabs(W->rf0[i]));
    return m;
}

static void set_pn(ws_t* W, double muR) {
    for (int i = 0; i < W->nrow; ++i) {
        const double r = i < W->nrc ? W->c[i] : i < W->nrc + W->nrd ? W->d[i - W->nrc] - W->s[i - W->nrc]
                                                                    : W->df[i - W->nrc - W->nrd] - W->sf[i - W->nrc - W->nrd];
        pn_closed_form(r, muR, W->rho, &W->pr[i], &W->nr[i]);
        W->zp[i] = muR / W->pr[i];
        W->zn[i] = muR / W->nr[i];
    }
}

/* enter the restoration phase at the current (linearised, original) iterate; returns mu_R */
static double enter_resto(ws_t* W, double mu) {
    const size_t N1 = (size_t)W->N + 1, N = (size_t)W->N, nb = (size_t)W->nb;
    memcpy(W->xR, W->x, N1 * 6 * 8); memcpy(W->uR, W->u, N * 2 * 8); memcpy(W->wR, W->w, nb * 8 * 8);
    memcpy(W->sR, W->s, nb * 4 * 8); memcpy(W->sfR, W->sf, 48);
    memcpy(W->szLx, W->zLx, N1 * 6 * 8); memcpy(W->szUx, W->zUx, N1 * 6 * 8); memcpy(W->szLu, W->zLu, N * 2 * 8);
    memcpy(W->szUu, W->zUu, N * 2 * 8); memcpy(W->szw, W->zw, nb * 8 * 8); memcpy(W->svL, W->vL, nb * 4 * 8);
    memcpy(W->svU, W->vU, nb * 4 * 8); memcpy(W->svLf, W->vLf, 48); memcpy(W->svUf, W->vUf, 48);
    for (size_t i = 0; i < N1 * 6; ++i) W->dRx[i] = fmin(1.0, 1.0 / fabs(W->x[i]));
    for (size_t i = 0; i < N * 2; ++i) W->dRu[i] = fmin(1.0, 1.0 / fabs(W->u[i]));
    for (size_t i = 0; i < nb * 8; ++i) W->dRw[i] = fmin(1.0, 1.0 / fabs(W->w[i]));
    for (size_t i = 0; i < N1 * 6; ++i) W->dRx[i] *= W->dRx[i];
    for (size_t i = 0; i < N * 2; ++i) W->dRu[i] *= W->dRu[i];
    for (size_t i = 0; i < nb * 8; ++i) W->dRw[i] *= W->dRw[i];
    const double muR = fmax(mu, row_resid_max(W));
    W->rho = RHO;
    W->zeta = sqrt(muR);
    set_pn(W, muR);
    /* bound multipliers of the shared variables: min(rho, z); constraint multipliers 0 */
    for (size_t i = 0; i < N1 * 6; ++i) { W->zLx[i] = fmin(W->zLx[i], W->rho); W->zUx[i] = fmin(W->zUx[i], W->rho); }
    for (size_t i = 0; i < N * 2; ++i) { W->zLu[i] = fmin(W->zLu[i], W->rho); W->zUu[i] = fmin(W->zUu[i], W->rho); }
    for (size_t i = 0; i < nb * 8; ++i) W->zw[i] = fmin(W->zw[i], W->rho);
    for (size_t i = 0; i < nb * 4; ++i) { W->vL[i] = fmin(W->vL[i], W->rho); W->vU[i] = fmin(W->vU[i], W->rho); }
    for (int i = 0; i < 6; ++i) { W->vLf[i] = fmin(W->vLf[i], W->rho); W->vUf[i] = fmin(W->vUf[i], W->rho); }
    memset(W->yc, 0, N1 * 6 * 8);
    memset(W->yd, 0, nb * 4 * 8);
    memset(W->ydf, 0, 48);
    W->R = M_RESTO;
    return muR;
}

/* leave the restoration phase: original bound multipliers updated by the complementarity Newton step of
 * the whole restoration change (fraction to the boundary tau), reset to 1 when above 1000; constraint
 * multipliers 0 */
static void leave_resto(ws_t* W, double mu, double tau) {
    const int N = W->N;
    double a = 1.0, zmax = 0.0;
#define DZL(z, sl0, d) (mu / (sl0) - (z) - (z) / (sl0) * (d))
    /* pass 1: fraction to the boundary; pass 2: apply */
    for (int pass = 0; pass < 2; ++pass) {
        for (int k = 0; k <= N; ++k) {
            for (int i = 0; i < 6; ++i) {
                const int v = 6 * k + i;
                const double d = W->x[v] - W->xR[v];
                if (W->hxl[i]) { const double dz = DZL(W->szLx[v], W->xR[v] - W->xl[i], d); if (!pass) FTB_D(W->szLx[v], dz, tau, a); else W->zLx[v] = W->szLx[v] + a * dz; }
                if (W->hxu[i]) { const double dz = DZL(W->szUx[v], W->xu[i] - W->xR[v], -d); if (!pass) FTB_D(W->szUx[v], dz, tau, a); else W->zUx[v] = W->szUx[v] + a * dz; }
            }
            if (k < N)
                for (int i = 0; i < 2; ++i) {
                    const int v = 2 * k + i;
                    const double d = W->u[v] - W->uR[v];
                    if (W->hul[i]) { const double dz = DZL(W->szLu[v], W->uR[v] - W->ul[i], d); if (!pass) FTB_D(W->szLu[v], dz, tau, a); else W->zLu[v] = W->szLu[v] + a * dz; }
                    if (W->huu[i]) { const double dz = DZL(W->szUu[v], W->uu[i] - W->uR[v], -d); if (!pass) FTB_D(W->szUu[v], dz, tau, a); else W->zUu[v] = W->szUu[v] + a * dz; }
                }
        }
        for (int bi = 0; bi < W->nb; ++bi) {
            for (int e = 0; e < 8; ++e) {
                const int v = 8 * bi + e;
                const double dz = DZL(W->szw[v], W->wR[v] + RELAX, W->w[v] - W->wR[v]);
                if (!pass) FTB_D(W->szw[v], dz, tau, a); else W->zw[v] = W->szw[v] + a * dz;
            }
            for (int r = 0; r < 4; ++r) {
                const int v = 4 * bi + r;
                const double d = W->s[v] - W->sR[v];
                if (W->hrL[r]) { const double dz = DZL(W->svL[v], W->sR[v] - W->rL[r], d); if (!pass) FTB_D(W->svL[v], dz, tau, a); else W->vL[v] = W->svL[v] + a * dz; }
                if (W->hrU[r]) { const double dz = DZL(W->svU[v], W->rU[r] - W->sR[v], -d); if (!pass) FTB_D(W->svU[v], dz, tau, a); else W->vU[v] = W->svU[v] + a * dz; }
            }
        }
        if (W->mode == TTO_OBCA_PLAN)
            for (int i = 0; i < 6; ++i) {
                const double d = W->sf[i] - W->sfR[i];
                const double dl = DZL(W->svLf[i], W->sfR[i] - W->fL, d), du = DZL(W->svUf[i], W->fU - W->sfR[i], -d);
                if (!pass) { FTB_D(W->svLf[i], dl, tau, a); FTB_D(W->svUf[i], du, tau, a); }
                else { W->vLf[i] = W->svLf[i] + a * dl; W->vUf[i] = W->svUf[i] + a * du; }
            }
    }
#undef DZL
    /* kappa_sigma safeguard, then the reset test */
    for (int k = 0; k <= N; ++k) {
        for (int i = 0; i < 6; ++i) {
            const int v = 6 * k + i;
            if (W->hxl[i]) { clamp_mult(&W->zLx[v], W->x[v] - W->xl[i], mu); zmax = fmax(zmax, W->zLx[v]); }
            if (W->hxu[i]) { clamp_mult(&W->zUx[v], W->xu[i] - W->x[v], mu); zmax = fmax(zmax, W->zUx[v]); }
        }
        if (k < N)
            for (int i = 0; i < 2; ++i) {
                const int v = 2 * k + i;
                if (W->hul[i]) { clamp_mult(&W->zLu[v], W->u[v] - W->ul[i], mu); zmax = fmax(zmax, W->zLu[v]); }
                if (W->huu[i]) { clamp_mult(&W->zUu[v], W->uu[i] - W->u[v], mu); zmax = fmax(zmax, W->zUu[v]); }
            }
    }
    for (int bi = 0; bi < W->nb; ++bi) {
        for (int e = 0; e < 8; ++e) { clamp_mult(&W->zw[8 * bi + e], W->w[8 * bi + e] + RELAX, mu); zmax = fmax(zmax, W->zw[8 * bi + e]); }
        for (int r = 0; r < 4; ++r) {
            const int v = 4 * bi + r;
            if (W->hrL[r]) { clamp_mult(&W->vL[v], W->s[v] - W->rL[r], mu); zmax = fmax(zmax, W->vL[v]); }
            if (W->hrU[r]) { clamp_mult(&W->vU[v], W->rU[r] - W->s[v], mu); zmax = fmax(zmax, W->vU[v]); }
        }
    }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            clamp_mult(&W->vLf[i], W->sf[i] - W->fL, mu);
            clamp_mult(&W->vUf[i], W->fU - W->sf[i], mu);
            zmax = fmax(zmax, fmax(W->vLf[i], W->vUf[i]));
        }
    if (zmax > BOUND_MULT_RESET) {
        for (int k = 0; k <= N; ++k) {
            for (int i = 0; i < 6; ++i) { W->zLx[6 * k + i] = W->hxl[i] ? 1.0 : 0.0; W->zUx[6 * k + i] = W->hxu[i] ? 1.0 : 0.0; }
            if (k < N)
                for (int i = 0; i < 2; ++i) { W->zLu[2 * k + i] = W->hul[i] ? 1.0 : 0.0; W->zUu[2 * k + i] = W->huu[i] ? 1.0 : 0.0; }
        }
        for (int bi = 0; bi < W->nb; ++bi) {
            for (int e = 0; e < 8; ++e) W->zw[8 * bi + e] = 1.0;
            for (int r = 0; r < 4; ++r) { W->vL[4 * bi + r] = W->hrL[r] ? 1.0 : 0.0; W->vU[4 * bi + r] = W->hrU[r] ? 1.0 : 0.0; }
        }
        for (int i = 0; i < 6; ++i) W->vLf[i] = W->vUf[i] = 1.0;
    }
    memset(W->yc, 0, 6 * ((size_t)N + 1) * 8);
    memset(W->yd, 0, 4 * (size_t)W->nb * 8);
    memset(W->ydf, 0, 48);
    W->R = M_ORIG;
}

/* least-squares constraint multipliers at the starting point (IPOPT constr_mult_init_max):
 * [[I, J'], [J, 0]] [d; y] = [-(grad f - z_L + z_U); 0], slack rows with unit Hessian */
static void ls_multipliers(ws_t* W) {
    const size_t N1 = (size_t)W->N + 1, nb = (size_t)W->nb;
    W->lsq = 1;
    linearise(W); /* y = 0: no curvature terms */
    double zero6[6] = {0};
    for (size_t i = 0; i < N1 * 6; ++i) W->cr[i] = 0.0;
    for (size_t i = 0; i < nb * 4; ++i) W->dr[i] = 0.0;
    int ok = factor(W, 0.0, 0.0) == F_OK;
    if (ok) {
        solve_rhs(W, 0.0, W->cr, W->dr, zero6);
        double m = 0.0;
        for (size_t i = 0; i < N1 * 6; ++i) m = fmax(m, fabs(W->ycp[i]));
        for (size_t i = 0; i < nb * 4; ++i) m = fmax(m, fabs(W->ydp[i]));
        if (W->mode == TTO_OBCA_PLAN)
            for (int i = 0; i < 6; ++i) m = fmax(m, fabs(W->ydpf[i]));
        ok = isfinite(m) && m <= CONSTR_MULT_INIT_MAX;
    }
    if (ok) {
        memcpy(W->yc, W->ycp, N1 * 6 * 8);
        memcpy(W->yd, W->ydp, nb * 4 * 8);
        memcpy(W->ydf, W->ydpf, 48);
    }
    W->lsq = 0;
}

/* ------------------------------------------------------------------ one barrier solve (original or restoration) */
typedef struct {
    double mu, tau, th_max, th_min;
    perturb_t ph;   /* one handler per NLP (original / restoration), as IPOPT's restoration algorithm has its own */
    int acc_count;
    filter_t F;
    /* watchdog (IPOPT BacktrackingLineSearch): shortened-step count, active flag, trials, reference point */
    int wd_short, wd_on, wd_trial;
    double wd_th, wd_ph, wd_Dm, wd_alpha;
} ipm_state_t;

static void ipm_reset(ipm_state_t* S, double mu) {
    S->mu = mu;
    S->tau = fmax(0.99, 1.0 - mu);
    S->th_max = S->th_min = 0.0;
    ph_reset(&S->ph);
    S->acc_count = 0;
    S->F.n = 0;
    S->wd_short = S->wd_on = S->wd_trial = 0;
}

static double dir_deriv(ws_t* W, double mu, double* rel_out) {
    const int N = W->N;
    double Dm = 0.0, rel = 0.0;
    for (int k = 0; k <= N; ++k) {
        for (int i = 0; i < 6; ++i) {
            Dm += bgrad_x(W, k, i, mu) * W->dx[6 * k + i];
            rel = fmax(rel, fabs(W->dx[6 * k + i]) / (1.0 + fabs(W->x[6 * k + i])));
        }
        if (k < N)
            for (int i = 0; i < 2; ++i) {
                Dm += bgrad_u(W, k, i, mu) * W->du[2 * k + i];
                rel = fmax(rel, fabs(W->du[2 * k + i]) / (1.0 + fabs(W->u[2 * k + i])));
            }
    }
    for (int bi = 0; bi < W->nb; ++bi) {
        for (int e = 0; e < 8; ++e) {
            Dm += bgrad_w(W, 8 * bi + e, mu) * W->dw[8 * bi + e];
            rel = fmax(rel, fabs(W->dw[8 * bi + e]) / (1.0 + fabs(W->w[8 * bi + e])));
        }
        for (int r = 0; r < 4; ++r) {
            Dm += bgrad_s(W, bi, r, mu) * W->ds[4 * bi + r];
            rel = fmax(rel, fabs(W->ds[4 * bi + r]) / (1.0 + fabs(W->s[4 * bi + r])));
        }
    }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            Dm += bgrad_sf(W, i, mu) * W->dsf[i];
            rel = fmax(rel, fabs(W->dsf[i]) / (1.0 + fabs(W->sf[i])));
        }
    if (W->R == M_RESTO)
        for (int i = 0; i < W->nrow; ++i) {
            Dm += (W->rho - mu / W->pr[i] + W->kd * mu) * W->dpr[i] + (W->rho - mu / W->nr[i] + W->kd * mu) * W->dnr[i];
            rel = fmax(rel, fmax(fabs(W->dpr[i]) / (1.0 + fabs(W->pr[i])), fabs(W->dnr[i]) / (1.0 + fabs(W->nr[i]))));
        }
    *rel_out = rel;
    return Dm;
}


/* TTO_CHECK diagnostic: relative residuals of the un-condensed primal-dual Newton rows (x, u, w, s, p/n
 * stationarity and the linearised constraint rows) for the step in dx du dw ds (dp dn) ycp ydp ydpf dsf */
static void check_newton(ws_t* W, double mu, double dw) {
    const tto_obca_problem* P = W->P;
    const int N = W->N, rs = W->R == M_RESTO;
    double wx = 0, wu = 0, ww = 0, wsl = 0, wpn = 0, wrow = 0;
#define ACC(t_, sc_) do { t += (t_); sc += fabs(t_); } while (0)
    for (int k = 0; k <= N; ++k) {
        const double tf = (k == N && W->mode == TTO_OBCA_PLAN) ? P->tfac : 1.0;
        for (int i = 0; i < 6; ++i) {
            double t = 0, sc = 0;
            ACC(bgrad_x(W, k, i, mu), 0);
            for (int j = 0; j < 6; ++j) {
                double h = (k < N ? W->Wd[36 * k + i * 6 + j] : 0.0);
                if (!rs) h += 2.0 * tf * W->Qc[i * 6 + j];
                ACC(h * W->dx[6 * k + j], 0);
            }
            ACC((sig_x(W, k, i) + dw + (rs ? W->zeta * W->dRx[6 * k + i] : 0.0)) * W->dx[6 * k + i], 0);
            ACC(W->ycp[6 * k + i], 0);
            if (k < N) for (int l = 0; l < 6; ++l) ACC(-W->A[36 * k + l * 6 + i] * W->ycp[6 * (k + 1) + l], 0);
            if (k == N && W->mode == TTO_OBCA_PLAN) ACC(W->ydpf[i], 0);
            if (i < 4)
                for (int j = 0; j < W->nbk; ++j) {
                    const int bi = k * W->nbk + j;
                    for (int q = 0; q < 4; ++q) ACC(W->Hxx[16 * bi + i * 4 + q] * W->dx[6 * k + q], 0);
                    for (int a = 0; a < 8; ++a) ACC(W->Hxw[32 * bi + i * 8 + a] * W->dw[8 * bi + a], 0);
                    for (int r = 0; r < 4; ++r) ACC(W->Jx[16 * bi + r * 4 + i] * W->ydp[4 * bi + r], 0);
                }
            wx = fmax(wx, fabs(t) / (sc + 1e-300));
        }
        if (k < N)
            for (int i = 0; i < 2; ++i) {
                double t = 0, sc = 0;
                ACC(bgrad_u(W, k, i, mu), 0);
                if (!rs) for (int j = 0; j < 2; ++j) ACC(2.0 * W->Rc[i * 2 + j] * W->du[2 * k + j], 0);
                ACC((sig_u(W, k, i) + dw + (rs ? W->zeta * W->dRu[2 * k + i] : 0.0)) * W->du[2 * k + i], 0);
                ACC(-P->dt * W->ycp[6 * (k + 1) + (i == 0 ? 5 : 4)], 0);
                wu = fmax(wu, fabs(t) / (sc + 1e-300));
            }
        for (int j = 0; j < W->nbk; ++j) {
            const int bi = k * W->nbk + j;
            for (int a = 0; a < 8; ++a) {
                double t = 0, sc = 0;
                ACC(bgrad_w(W, 8 * bi + a, mu), 0);
                ACC((W->zw[8 * bi + a] / (W->w[8 * bi + a] + RELAX) + dw + (rs ? W->zeta * W->dRw[8 * bi + a] : 0.0)) * W->dw[8 * bi + a], 0);
                for (int q = 0; q < 4; ++q) ACC(W->Hxw[32 * bi + q * 8 + a] * W->dx[6 * k + q], 0);
                if (a >= 4) for (int b = 0; b < 4; ++b) ACC(W->Hww[16 * bi + (a - 4) * 4 + b] * W->dw[8 * bi + 4 + b], 0);
                for (int r = 0; r < 4; ++r) ACC(W->Jw[32 * bi + r * 8 + a] * W->ydp[4 * bi + r], 0);
                ww = fmax(ww, fabs(t) / (sc + 1e-300));
            }
            for (int r = 0; r < 4; ++r) {
                const int v = 4 * bi + r, ro = W->nrc + v;
                double t = 0, sc = 0;
                ACC((sig_s(W, bi, r) + dw) * W->ds[v], 0);
                ACC(-W->ydp[v], 0);
                ACC(bgrad_s(W, bi, r, mu), 0);
                wsl = fmax(wsl, fabs(t) / (sc + 1e-300));
                t = 0; sc = 0;
                ACC(W->rd0[v], 0);
                for (int q = 0; q < 4; ++q) ACC(W->Jx[16 * bi + r * 4 + q] * W->dx[6 * k + q], 0);
                for (int a = 0; a < 8; ++a) ACC(W->Jw[32 * bi + r * 8 + a] * W->dw[8 * bi + a], 0);
                ACC(-W->ds[v], 0);
                if (rs) { ACC(-W->dpr[ro], 0); ACC(W->dnr[ro], 0); }
                wrow = fmax(wrow, fabs(t) / (sc + 1e-300));
            }
        }
        for (int i = 0; i < 6; ++i) { /* dynamics rows */
            double t = 0, sc = 0;
            const int v = 6 * k + i;
            ACC(W->rc0[v], 0);
            ACC(W->dx[v], 0);
            if (k > 0) {
                for (int j = 0; j < 6; ++j) ACC(-W->A[36 * (k - 1) + i * 6 + j] * W->dx[6 * (k - 1) + j], 0);
                if (i == 5) ACC(-P->dt * W->du[2 * (k - 1)], 0);
                if (i == 4) ACC(-P->dt * W->du[2 * (k - 1) + 1], 0);
            }
            if (rs) { ACC(-W->dpr[v], 0); ACC(W->dnr[v], 0); }
            wrow = fmax(wrow, fabs(t) / (sc + 1e-300));
        }
    }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            const int ro = W->nrc + W->nrd + i;
            double t = 0, sc = 0;
            ACC(W->rf0[i], 0); ACC(W->dx[6 * N + i], 0); ACC(-W->dsf[i], 0);
            if (rs) { ACC(-W->dpr[ro], 0); ACC(W->dnr[ro], 0); }
            wrow = fmax(wrow, fabs(t) / (sc + 1e-300));
            t = 0; sc = 0;
            ACC((W->vLf[i] / (W->sf[i] - W->fL) + W->vUf[i] / (W->fU - W->sf[i]) + dw) * W->dsf[i], 0);
            ACC(-W->ydpf[i], 0); ACC(bgrad_sf(W, i, mu), 0);
            wsl = fmax(wsl, fabs(t) / (sc + 1e-300));
        }
    if (rs)
        for (int i = 0; i < W->nrow; ++i) {
            const double yp = i < W->nrc ? W->ycp[i] : i < W->nrc + W->nrd ? W->ydp[i - W->nrc] : W->ydpf[i - W->nrc - W->nrd];
            double t = 0, sc = 0;
            ACC((W->zp[i] / W->pr[i] + dw) * W->dpr[i], 0); ACC(-yp, 0); ACC(W->rho - mu / W->pr[i] + W->kd * mu, 0);
            wpn = fmax(wpn, fabs(t) / (sc + 1e-300));
            t = 0; sc = 0;
            ACC((W->zn[i] / W->nr[i] + dw) * W->dnr[i], 0); ACC(yp, 0); ACC(W->rho - mu / W->nr[i] + W->kd * mu, 0);
            wpn = fmax(wpn, fabs(t) / (sc + 1e-300));
        }
#undef ACC
    fprintf(stderr, "   check(R=%d): x %.1e u %.1e w %.1e s %.1e pn %.1e rows %.1e\n", W->R, wx, wu, ww, wsl, wpn, wrow);
}

/* residuals of the un-condensed primal-dual Newton rows at the solution in dx.. ycp ydp dsf ydpf (dp dn), with
 * the constants of the solve (barrier gradients or the override, and cres / dres / fres); returns the max
 * norm of all of them and of the constants in *rhs_inf */
static double newton_resid(ws_t* W, double mu, const double* cres, const double* dres, const double* fres,
                           double* rhs_inf) {
    const tto_obca_problem* P = W->P;
    const int N = W->N, rs = W->R == M_RESTO;
    const double dw = W->dw_cur;
    double rmax = 0.0, bmax = 0.0;
#define CST(v) (bmax = fmax(bmax, fabs(v)), (v))
    for (int k = 0; k <= N; ++k) {
        const double tf = (k == N && W->mode == TTO_OBCA_PLAN) ? P->tfac : 1.0;
        for (int i = 0; i < 6; ++i) {
            double t = CST(W->ov ? W->ovx[6 * k + i] : bgrad_x(W, k, i, mu));
            for (int j = 0; j < 6; ++j) {
                double h = (k < N ? W->Wd[36 * k + i * 6 + j] : 0.0);
                if (!rs) h += 2.0 * tf * W->Qc[i * 6 + j];
                t += h * W->dx[6 * k + j];
            }
            t += (sig_x(W, k, i) + dw + (rs ? W->zeta * W->dRx[6 * k + i] : 0.0)) * W->dx[6 * k + i];
            t += W->ycp[6 * k + i];
            if (k < N) for (int l = 0; l < 6; ++l) t -= W->A[36 * k + l * 6 + i] * W->ycp[6 * (k + 1) + l];
            if (k == N && W->mode == TTO_OBCA_PLAN) t += W->ydpf[i];
            if (i < 4)
                for (int j = 0; j < W->nbk; ++j) {
                    const int bi = k * W->nbk + j;
                    for (int q = 0; q < 4; ++q) t += W->Hxx[16 * bi + i * 4 + q] * W->dx[6 * k + q];
                    for (int a = 0; a < 8; ++a) t += W->Hxw[32 * bi + i * 8 + a] * W->dw[8 * bi + a];
                    for (int r = 0; r < 4; ++r) t += W->Jx[16 * bi + r * 4 + i] * W->ydp[4 * bi + r];
                }
            W->rsx[6 * k + i] = t;
            rmax = fmax(rmax, fabs(t));
        }
        if (k < N)
            for (int i = 0; i < 2; ++i) {
                double t = CST(W->ov ? W->ovu[2 * k + i] : bgrad_u(W, k, i, mu));
                if (!rs) for (int j = 0; j < 2; ++j) t += 2.0 * W->Rc[i * 2 + j] * W->du[2 * k + j];
                t += (sig_u(W, k, i) + dw + (rs ? W->zeta * W->dRu[2 * k + i] : 0.0)) * W->du[2 * k + i];
                t -= P->dt * W->ycp[6 * (k + 1) + (i == 0 ? 5 : 4)];
                W->rsu[2 * k + i] = t;
                rmax = fmax(rmax, fabs(t));
            }
        for (int j = 0; j < W->nbk; ++j) {
            const int bi = k * W->nbk + j;
            for (int a = 0; a < 8; ++a) {
                double t = CST(W->ov ? W->ovw[8 * bi + a] : bgrad_w(W, 8 * bi + a, mu));
                t += (W->zw[8 * bi + a] / (W->w[8 * bi + a] + RELAX) + dw + (rs ? W->zeta * W->dRw[8 * bi + a] : 0.0)) * W->dw[8 * bi + a];
                for (int q = 0; q < 4; ++q) t += W->Hxw[32 * bi + q * 8 + a] * W->dx[6 * k + q];
                if (a >= 4) for (int b = 0; b < 4; ++b) t += W->Hww[16 * bi + (a - 4) * 4 + b] * W->dw[8 * bi + 4 + b];
                for (int r = 0; r < 4; ++r) t += W->Jw[32 * bi + r * 8 + a] * W->ydp[4 * bi + r];
                W->rsw[8 * bi + a] = t;
                rmax = fmax(rmax, fabs(t));
            }
            for (int r = 0; r < 4; ++r) {
                const int v = 4 * bi + r, ro = W->nrc + v;
                double t = CST(W->ov ? W->ovs[v] : bgrad_s(W, bi, r, mu));
                t += (sig_s(W, bi, r) + dw) * W->ds[v] - W->ydp[v];
                W->rss[v] = t;
                rmax = fmax(rmax, fabs(t));
                t = CST(dres[v]);
                for (int q = 0; q < 4; ++q) t += W->Jx[16 * bi + r * 4 + q] * W->dx[6 * k + q];
                for (int a = 0; a < 8; ++a) t += W->Jw[32 * bi + r * 8 + a] * W->dw[8 * bi + a];
                t -= W->ds[v];
                if (rs) t += -W->dpr[ro] + W->dnr[ro];
                t -= W->dc_cur * W->ydp[v];
                W->rrd[v] = t;
                rmax = fmax(rmax, fabs(t));
            }
        }
        for (int i = 0; i < 6; ++i) {
            const int v = 6 * k + i;
            double t = CST(cres[v]) + W->dx[v];
            if (k > 0) {
                for (int j = 0; j < 6; ++j) t -= W->A[36 * (k - 1) + i * 6 + j] * W->dx[6 * (k - 1) + j];
                if (i == 5) t -= P->dt * W->du[2 * (k - 1)];
                if (i == 4) t -= P->dt * W->du[2 * (k - 1) + 1];
            }
            if (rs) t += -W->dpr[v] + W->dnr[v];
            t -= W->dc_cur * W->ycp[v];
            W->rrc[v] = t;
            rmax = fmax(rmax, fabs(t));
        }
    }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            const int ro = W->nrc + W->nrd + i;
            double t = CST(fres[i]) + W->dx[6 * N + i] - W->dsf[i];
            if (rs) t += -W->dpr[ro] + W->dnr[ro];
            t -= W->dc_cur * W->ydpf[i];
            W->rrf[i] = t;
            rmax = fmax(rmax, fabs(t));
            t = CST(W->ov ? W->ovsf[i] : bgrad_sf(W, i, mu));
            t += (W->vLf[i] / (W->sf[i] - W->fL) + W->vUf[i] / (W->fU - W->sf[i]) + dw) * W->dsf[i] - W->ydpf[i];
            W->rssf[i] = t;
            rmax = fmax(rmax, fabs(t));
        }
    if (rs)
        for (int i = 0; i < W->nrow; ++i) {
            const double yp = i < W->nrc ? W->ycp[i] : i < W->nrc + W->nrd ? W->ydp[i - W->nrc] : W->ydpf[i - W->nrc - W->nrd];
            double t = CST(W->ov ? W->ovp[i] : W->rho - mu / W->pr[i] + W->kd * mu);
            t += (W->zp[i] / W->pr[i] + dw) * W->dpr[i] - yp;
            W->rsp[i] = t;
            rmax = fmax(rmax, fabs(t));
            t = CST(W->ov ? W->ovn[i] : W->rho - mu / W->nr[i] + W->kd * mu);
            t += (W->zn[i] / W->nr[i] + dw) * W->dnr[i] + yp;
            W->rsn[i] = t;
            rmax = fmax(rmax, fabs(t));
        }
#undef CST
    if (rhs_inf) *rhs_inf = bmax;
    return rmax;
}

/* the solution norm and the residual ratio of IPOPT's PDFullSpaceSolver::ComputeResidualRatio:
 * max|resid| / (min(max|sol|, 1e6) + max|rhs|) */
static double resid_ratio(const ws_t* W, double res, double bnorm) {
    const size_t N1 = (size_t)W->N + 1, nb = (size_t)W->nb;
    double snorm = 0.0;
    for (size_t i = 0; i < N1 * 6; ++i) snorm = fmax(snorm, fmax(fabs(W->dx[i]), fabs(W->ycp[i])));
    for (size_t i = 0; i < nb * 8; ++i) snorm = fmax(snorm, fabs(W->dw[i]));
    return res / (fmin(snorm, 1e6) + bnorm);
}

/* the step solve with IPOPT's iterative refinement on the un-condensed system (PDFullSpaceSolver::Solve:
 * min_refinement_steps 1, max_refinement_steps 10, residual_ratio_max 1e-10, residual_improvement_factor 1):
 * correction solves reuse the factorisation with the residuals as constants (TTO_OPT_NO_REFINE switches it off).
 * With delta_c > 0 the row constants are shifted by delta_c y (IPOPT perturbs dy; the unknowns here are y+ = y + dy).
 * Returns 1 when the refinement quit (IPOPT's "iterative refinement failed"), with the final residual ratio. */
static int refined_solve(ws_t* W, double mu, double* cres, double* dres, double* fres, double* ratio_out) {
    const int N = W->N, rs = W->R == M_RESTO;
    const size_t N1 = (size_t)N + 1, nb = (size_t)W->nb, nr = (size_t)W->nrow;
    *ratio_out = 0.0;
    if (W->dc_cur > 0.0 && !W->lsq) {
        double* c = W->csh;
        for (size_t i = 0; i < N1 * 6; ++i) c[i] = cres[i] + W->dc_cur * W->yc[i];
        for (size_t i = 0; i < nb * 4; ++i) c[N1 * 6 + i] = dres[i] + W->dc_cur * W->yd[i];
        for (int i = 0; i < 6; ++i) c[N1 * 6 + nb * 4 + i] = fres[i] + (W->mode == TTO_OBCA_PLAN ? W->dc_cur * W->ydf[i] : 0.0);
        cres = c; dres = c + N1 * 6; fres = c + N1 * 6 + nb * 4;
    }
    solve_rhs(W, mu, cres, dres, fres);
    if ((W->P->opts & TTO_OPT_NO_REFINE) || W->lsq) return 0;
    ++g_cen[9];
    const int r3 = (W->P->opts & TTO_OPT_R3_PERTURB) != 0;
    double bnorm = 0.0;
    double res = newton_resid(W, mu, cres, dres, fres, &bnorm);
    double ratio = resid_ratio(W, res, bnorm);
    double* cc = W->cc;
    int quit = 0;
    for (int it = 0; !quit && (it < 1 || ratio > 1e-10); ++it) {
        if (r3 && it >= 10) break;
        ++g_cen[8];
        /* save the solution, solve for the correction with the residuals as constants, add */
        double* o = W->sol;
        memcpy(o, W->dx, N1 * 48); o += N1 * 6; memcpy(o, W->ycp, N1 * 48); o += N1 * 6;
        memcpy(o, W->du, (size_t)N * 16); o += N * 2; memcpy(o, W->dw, nb * 64); o += nb * 8;
        memcpy(o, W->ds, nb * 32); o += nb * 4; memcpy(o, W->ydp, nb * 32); o += nb * 4;
        memcpy(o, W->dsf, 48); o += 6; memcpy(o, W->ydpf, 48); o += 6;
        if (rs) { memcpy(o, W->dpr, nr * 8); o += nr; memcpy(o, W->dnr, nr * 8); o += nr; }
        memcpy(W->ovx, W->rsx, N1 * 48); memcpy(W->ovu, W->rsu, (size_t)N * 16); memcpy(W->ovw, W->rsw, nb * 64);
        memcpy(W->ovs, W->rss, nb * 32); memcpy(W->ovsf, W->rssf, 48);
        if (rs) { memcpy(W->ovp, W->rsp, nr * 8); memcpy(W->ovn, W->rsn, nr * 8); }
        memcpy(cc, W->rrc, N1 * 48); memcpy(cc + N1 * 6, W->rrd, nb * 32); memcpy(cc + N1 * 6 + nb * 4, W->rrf, 48);
        W->ov = W->ovx;
        solve_rhs(W, mu, cc, cc + N1 * 6, cc + N1 * 6 + nb * 4);
        W->ov = NULL;
        o = W->sol;
#define ADD(ptr, cnt) do { for (size_t q_ = 0; q_ < (cnt); ++q_) (ptr)[q_] += o[q_]; o += (cnt); } while (0)
        ADD(W->dx, N1 * 6); ADD(W->ycp, N1 * 6); ADD(W->du, (size_t)N * 2); ADD(W->dw, nb * 8); ADD(W->ds, nb * 4);
        ADD(W->ydp, nb * 4); ADD(W->dsf, 6); ADD(W->ydpf, 6);
        if (rs) { ADD(W->dpr, nr); ADD(W->dnr, nr); }
#undef ADD
        const double res2 = newton_resid(W, mu, cres, dres, fres, NULL);
        const double ratio2 = resid_ratio(W, res2, bnorm);
        if (r3) {
            /* round 3: raw residuals, stop on the first non-improvement or when the ratio test passes */
            const int stop = !(res2 < res);
            res = res2;
            ratio = ratio2;
            if (stop) break;
            if (ratio <= 1e-10) break;
            continue;
        }
        /* IPOPT gives up when the ratio is still above residual_ratio_max after more than min_refinement_steps
         * corrections and either max_refinement_steps is exceeded or the ratio did not improve */
        if (ratio2 > 1e-10 && it + 1 > 1 && (it + 1 > 10 || ratio2 > ratio)) quit = 1;
        res = res2;
        ratio = ratio2;
    }
    if (ratio > 1e-10) ++g_cen[5];
    if (ratio > 1e-5) ++g_cen[6];
    *ratio_out = ratio;
    return quit;
}

/* ---------------- IPOPT's PDPerturbationHandler (restated) ----------------
 * delta_x (= delta_s) regularises the Hessian, delta_c (= delta_d) the constraint rows.  Each new matrix starts from
 * ConsiderNewSystem; a singular factorisation (or too few negative eigenvalues, IncreaseQuality being unavailable)
 * goes to PerturbForSingularity, a wrong inertia to PerturbForWrongInertia.  The Hessian / Jacobian structural
 * degeneracy flags are determined in the first iterations whose unperturbed matrix is singular (degen_iters_max 3);
 * a structurally degenerate Jacobian gets delta_c = 1e-8 mu^0.25 on every matrix, a degenerate Hessian starts from the
 * decreased last delta_x instead of 0.  Options are IPOPT's defaults: first_hessian_perturbation 1e-4,
 * perturb_inc_fact_first 100, perturb_inc_fact 8, perturb_dec_fact 1/3, min/max_hessian_perturbation 1e-20 / 1e20,
 * jacobian_regularization_value 1e-8, jacobian_regularization_exponent 0.25, perturb_always_cd no. */
enum { PH_UNDET = -1, PH_NOT = 0, PH_DEG = 1 };
enum { PT_NONE = 0, PT_C0X0, PT_CPX0, PT_C0XP, PT_CPXP };
static void ph_reset(perturb_t* H) {
    H->hess = H->jac = PH_UNDET;
    H->degen = 0;
    H->test = PT_NONE;
    H->gdwi = 0;
    H->dx_curr = H->dx_last = H->dc_curr = H->dc_last = 0.0;
}
static double ph_dcd(double mu) { return 1e-8 * pow(mu, 0.25); }
static void ph_finalize(perturb_t* H) {
    switch (H->test) {
    case PT_C0X0:
        if (H->hess == PH_UNDET && H->jac == PH_UNDET) { H->hess = PH_NOT; H->jac = PH_NOT; }
        else if (H->hess == PH_UNDET) H->hess = PH_NOT;
        else if (H->jac == PH_UNDET) H->jac = PH_NOT;
        break;
    case PT_CPX0:
        if (H->hess == PH_UNDET) H->hess = PH_NOT;
        if (H->jac == PH_UNDET && ++H->degen >= 3) H->jac = PH_DEG;
        break;
    case PT_C0XP:
        if (H->jac == PH_UNDET) H->jac = PH_NOT;
        if (H->hess == PH_UNDET && ++H->degen >= 3) H->hess = PH_DEG;
        break;
    case PT_CPXP:
        if (++H->degen >= 3) { H->hess = PH_DEG; H->jac = PH_DEG; }
        break;
    default:
        break;
    }
}
/* get_deltas_for_wrong_inertia: 0 when delta_x would exceed max_hessian_perturbation */
static int ph_gdwi(perturb_t* H) {
    if (H->dx_curr == 0.0) H->dx_curr = H->dx_last == 0.0 ? 1e-4 : fmax(1e-20, H->dx_last / 3.0);
    else H->dx_curr *= (H->dx_last == 0.0 || 1e5 * H->dx_last < H->dx_curr) ? 100.0 : 8.0;
    if (H->dx_curr > 1e20) { H->dx_last = 0.0; return 0; }
    H->gdwi = 1;
    return 1;
}
static int ph_new(perturb_t* H, double mu) {
    ph_finalize(H);
    if (H->dx_curr > 0.0) H->dx_last = H->dx_curr;
    if (H->dc_curr > 0.0) H->dc_last = H->dc_curr;
    H->test = (H->hess == PH_UNDET || H->jac == PH_UNDET) ? PT_C0X0 : PT_NONE;
    H->dc_curr = H->jac == PH_DEG ? ph_dcd(mu) : 0.0;
    H->dx_curr = 0.0;
    if (H->hess == PH_DEG && !ph_gdwi(H)) return 0;
    H->gdwi = 0;
    return 1;
}
static int ph_singular(perturb_t* H, double mu) {
    if (H->hess == PH_UNDET || H->jac == PH_UNDET) {
        switch (H->test) {
        case PT_C0X0:
            if (H->jac == PH_UNDET) { H->dc_curr = ph_dcd(mu); H->test = PT_CPX0; }
            else { if (!ph_gdwi(H)) return 0; H->test = PT_C0XP; }
            break;
        case PT_CPX0:
            H->dc_curr = 0.0;
            if (!ph_gdwi(H)) return 0;
            H->test = PT_C0XP;
            break;
        case PT_C0XP:
            H->dc_curr = ph_dcd(mu);
            if (!ph_gdwi(H)) return 0;
            H->test = PT_CPXP;
            break;
        default:
            if (!ph_gdwi(H)) return 0;
            break;
        }
    } else if (H->dc_curr > 0.0 || H->gdwi) {
        if (!ph_gdwi(H)) return 0;
    } else {
        H->dc_curr = ph_dcd(mu);
    }
    return 1;
}
static int ph_inertia(perturb_t* H, double mu) {
    ph_finalize(H);
    if (ph_gdwi(H)) return 1;
    if (H->dc_curr != 0.0) return 0;
    /* delta_x gave up without delta_c: try again with the constraint rows regularised */
    H->dc_curr = ph_dcd(mu);
    H->dx_curr = 0.0;
    H->test = PT_NONE;
    if (H->hess == PH_DEG) H->hess = PH_NOT;
    return ph_gdwi(H);
}
/* round 3's schedule (TTO_OPT_R3_PERTURB, A/B only): delta_x from 0 on every matrix, no delta_c */
static int ph_r3(perturb_t* H) {
    const double dw = H->dx_curr;
    H->dx_curr = dw == 0.0 ? (H->dx_last == 0.0 ? 1e-4 : fmax(1e-20, H->dx_last / 3.0))
                           : (H->dx_last == 0.0 ? 100.0 * dw : 8.0 * dw);
    return H->dx_curr <= 1e20;
}

/* factorisations until the inertia is right (PDFullSpaceSolver::SolveOnce); 0 when the perturbation gave up */
static int factor_loop(ws_t* W, ipm_state_t* S) {
    perturb_t* H = &S->ph;
    const int r3 = (W->P->opts & TTO_OPT_R3_PERTURB) != 0;
    for (int attempt = 0; attempt < 64; ++attempt) {
        const int f = factor(W, H->dx_curr, H->dc_curr);
        if (f == F_OK) return 1;
        const int ok = r3 ? ph_r3(H) : (f == F_MANY ? ph_inertia(H, S->mu) : ph_singular(H, S->mu));
        if (!ok) return 0;
    }
    return 0;
}

/* one linear solve of the current matrix with IPOPT's safeguards (PDFullSpaceSolver::Solve): refinement, and when it
 * fails with a residual ratio above residual_ratio_singular 1e-5 the matrix is treated as singular once
 * (pretend_singular: PerturbForSingularity, refactorisation, solve again).  0 when the perturbation gave up. */
static int pd_solve(ws_t* W, ipm_state_t* S, double* cres, double* dres, double* fres) {
    double ratio = 0.0;
    const int quit = refined_solve(W, S->mu, cres, dres, fres, &ratio);
    if (!quit || (W->P->opts & TTO_OPT_R3_PERTURB) || ratio < 1e-5) return 1;
    ++g_cen[7];
    if (!ph_singular(&S->ph, S->mu)) return 0;
    if (!factor_loop(W, S)) return 0;
    refined_solve(W, S->mu, cres, dres, fres, &ratio);
    return 1;
}

/* Newton step with inertia correction into dx..; 0 on success */
static int newton(ws_t* W, ipm_state_t* S, double* dw_out) {
    perturb_t* H = &S->ph;
    if (W->P->opts & TTO_OPT_R3_PERTURB) {
        if (H->dx_curr > 0.0) H->dx_last = H->dx_curr;
        H->dx_curr = H->dc_curr = 0.0;
    } else if (!ph_new(H, S->mu)) {
        return 1;
    }
    if (!factor_loop(W, S)) return 1;
    memcpy(W->cr, W->rc0, (size_t)W->nrc * 8);
    memcpy(W->dr, W->rd0, (size_t)W->nrd * 8);
    if (!pd_solve(W, S, W->cr, W->dr, W->rf0)) return 1;
    *dw_out = W->dw_cur;
    if (W->dbg & 4) check_newton(W, S->mu, W->dw_cur);
    mult_steps(W, S->mu);
    return 0;
}

/* filter line search with second-order corrections on the current system.  Returns 1 (accepted, h-type
 * adds a filter entry), 0 (line search failed); *alpha_out / *az_out the step sizes. */
static _Thread_local double g_dbg_ap, g_dbg_sw; /* TTO_DEBUG trace of the last line search */
static _Thread_local int g_dbg_acc;

/* filter acceptability of a trial (th, ph) against the reference (th0, phi0, Dm) at the step alpha
 * (FilterLSAcceptor::CheckAcceptabilityOfTrialPoint); *ftype: the switching condition held (f-type) */
static int acceptable(const ipm_state_t* S, double th, double ph, double th0, double phi0, double Dm, double alpha,
                      int* ftype) {
    const double g_th = 1e-5, g_ph = 1e-8, s_ph = 2.3, s_th = 1.1, delta = 1.0, eta_ph = 1e-8;
    const double tolc = 10.0 * DBL_EPSILON;
    const int sw = Dm < 0.0 && alpha * pow(-Dm, s_ph) > delta * pow(th0, s_th);
    *ftype = 0;
    if (!(isfinite(ph) && th <= S->th_max && !in_filter(&S->F, th, ph))) return 0;
    if (th0 <= S->th_min && sw) { *ftype = 1; return ph - (phi0 + eta_ph * alpha * Dm) <= tolc * fabs(phi0); }
    return th <= (1.0 - g_th) * th0 || ph - (phi0 - g_ph * th0) <= tolc * fabs(phi0);
}

/* filter line search with second-order corrections and IPOPT's watchdog on the current system.  Returns 1
 * (accepted; h-type steps add a filter entry), 0 (line search failed); *alpha_out / *az_out the step sizes.
 * *th0 / *phi0 are the reference values; they change when a failed watchdog restores its stored iterate
 * (the iterate is then re-linearised, so a caller that falls back to restoration sees the restored point). */
static int line_search(ws_t* W, ipm_state_t* S, int iter0, double* th0p, double* phi0p, double* alpha_out,
                       double* az_out) {
    const double mu = S->mu, tau = S->tau;
    double th0 = *th0p, phi0 = *phi0p;
    double ap = ftb_primal(W, tau), az = ftb_dual(W, tau), rel = 0.0;
    double Dm = dir_deriv(W, mu, &rel);
    if (iter0 || !(S->th_max > 0)) { S->th_max = 1e4 * fmax(1.0, th0); S->th_min = 1e-4 * fmax(1.0, th0); }
    const double g_th = 1e-5, g_ph = 1e-8, s_ph = 2.3, s_th = 1.1, delta = 1.0, g_al = 0.05;
    const int rs = W->R == M_RESTO;
    const size_t nx_ = 6 * (size_t)(W->N + 1), nu_ = 2 * (size_t)W->N, nw_ = 8 * (size_t)W->nb, ns_ = 4 * (size_t)W->nb;
    const size_t nr_ = (size_t)W->nrow;
    double tht = 0.0, pht = 0.0;
    int accepted = 0, ftype = 0, skip_first = 0, nsteps = 0;
    const int use_wd = (W->P->opts & TTO_OPT_WATCHDOG) && rel >= 1e-15;
    /* watchdog: after WD_TRIGGER consecutive shortened steps, store the iterate and direction and take full
     * steps, each tested against the stored point, for at most WD_TRIAL_MAX iterations */
    if (use_wd && !S->wd_on && S->wd_short >= WD_TRIGGER) {
        wd_save(W, 0);
        S->wd_on = 1;
        S->wd_trial = 0;
        S->wd_th = th0; S->wd_ph = phi0; S->wd_Dm = Dm; S->wd_alpha = ap;
    }
    if (S->wd_on) {
        set_trial(W, ap);
        trial_eval(W, mu, &tht, &pht);
        if (acceptable(S, tht, pht, S->wd_th, S->wd_ph, S->wd_Dm, S->wd_alpha, &ftype)) {
            S->wd_on = 0; /* watchdog successful */
            S->wd_short = 0;
            if (!ftype) add_filter(&S->F, (1.0 - g_th) * S->wd_th, S->wd_ph - g_ph * S->wd_th);
            g_dbg_ap = ap; g_dbg_acc = 3; g_dbg_sw = Dm;
            *alpha_out = ap; *az_out = az;
            return 1;
        }
        if (isfinite(pht) && ++S->wd_trial <= WD_TRIAL_MAX) {
            /* watchdog step: the full step is taken anyway; the filter gets the stored reference */
            add_filter(&S->F, (1.0 - g_th) * S->wd_th, S->wd_ph - g_ph * S->wd_th);
            g_dbg_ap = ap; g_dbg_acc = 4; g_dbg_sw = Dm;
            *alpha_out = ap; *az_out = az;
            return 1;
        }
        /* StopWatchDog: back to the stored iterate and direction; backtrack from there without the full step */
        wd_save(W, 1);
        S->wd_on = 0;
        S->wd_short = 0;
        th0 = S->wd_th; phi0 = S->wd_ph; Dm = S->wd_Dm; ap = S->wd_alpha;
        az = ftb_dual(W, tau);
        skip_first = 1;
    }
    double amin;
    if (Dm < 0.0) {
        amin = fmin(g_th, g_ph * th0 / (-Dm));
        if (th0 <= S->th_min) amin = fmin(amin, delta * pow(th0, s_th) / pow(-Dm, s_ph));
    } else {
        amin = g_th;
    }
    amin *= g_al;
    double alpha = ap;
    accepted = rel < 1e-15;
    for (int ls = 0; !accepted; ++ls) {
        if (!(ls == 0 && skip_first)) {
            set_trial(W, alpha);
            trial_eval(W, mu, &tht, &pht);
            if (acceptable(S, tht, pht, th0, phi0, Dm, alpha, &ftype)) { accepted = 1; break; }
        }
        if (ls == 0 && !skip_first && isfinite(pht) && tht >= th0) {
            /* second-order corrections (IPOPT max_soc 4, kappa_soc 0.99) */
            double* o = W->sv;
            memcpy(o, W->dx, nx_ * 8); o += nx_; memcpy(o, W->du, nu_ * 8); o += nu_;
            memcpy(o, W->dw, nw_ * 8); o += nw_; memcpy(o, W->ds, ns_ * 8); o += ns_;
            memcpy(o, W->ycp, nx_ * 8); o += nx_; memcpy(o, W->ydp, ns_ * 8); o += ns_;
            memcpy(o, W->dsf, 48); o += 6; memcpy(o, W->ydpf, 48); o += 6;
            if (rs) { memcpy(o, W->dpr, nr_ * 8); o += nr_; memcpy(o, W->dnr, nr_ * 8); o += nr_; }
            /* c_soc(0) = alpha r(x) + r(x + alpha d), c_soc(p+1) = a_soc(p) c_soc(p) + r(x + a_soc(p) d_soc(p)) */
            double frs[6], a_soc = alpha, th_old = th0;
            memcpy(W->cr, W->rc0, nx_ * 8);
            memcpy(W->dr, W->rd0, ns_ * 8);
            memcpy(frs, W->rf0, 48);
            int soc_ok = 0;
            for (int p = 0; p < 4; ++p) {
                if (p > 0 && tht > 0.99 * th_old) break;
                th_old = tht;
                for (size_t i = 0; i < nx_; ++i) W->cr[i] = a_soc * W->cr[i] + W->ct[i];
                for (size_t i = 0; i < ns_; ++i) W->dr[i] = a_soc * W->dr[i] + W->dtr[i];
                if (W->mode == TTO_OBCA_PLAN) for (int i = 0; i < 6; ++i) frs[i] = a_soc * frs[i] + W->dft[i];
                if (!pd_solve(W, S, W->cr, W->dr, frs)) break;
                a_soc = ftb_primal(W, tau);
                set_trial(W, a_soc);
                trial_eval(W, mu, &tht, &pht);
                /* the acceptance test of a corrected step uses the uncorrected alpha in the Armijo term */
                int ft2 = 0;
                if (acceptable(S, tht, pht, th0, phi0, Dm, alpha, &ft2)) { soc_ok = 1; ftype = ft2; break; }
                if (!isfinite(pht)) break;
            }
            if (soc_ok) {
                accepted = 2;
                alpha = a_soc;
                mult_steps(W, mu);
                az = ftb_dual(W, tau);
                break;
            }
            o = W->sv;
            memcpy(W->dx, o, nx_ * 8); o += nx_; memcpy(W->du, o, nu_ * 8); o += nu_;
            memcpy(W->dw, o, nw_ * 8); o += nw_; memcpy(W->ds, o, ns_ * 8); o += ns_;
            memcpy(W->ycp, o, nx_ * 8); o += nx_; memcpy(W->ydp, o, ns_ * 8); o += ns_;
            memcpy(W->dsf, o, 48); o += 6; memcpy(W->ydpf, o, 48); o += 6;
            if (rs) { memcpy(W->dpr, o, nr_ * 8); o += nr_; memcpy(W->dnr, o, nr_ * 8); o += nr_; }
        }
        if (alpha * 0.5 < amin) break;
        alpha *= 0.5;
        ++nsteps;
    }
    if (accepted && !ftype) add_filter(&S->F, (1.0 - g_th) * th0, phi0 - g_ph * th0);
    if (accepted) S->wd_short = nsteps > 0 ? S->wd_short + 1 : 0;
    g_dbg_ap = ap; g_dbg_acc = accepted; g_dbg_sw = Dm;
    if (W->dbg & 1) {
        double c[7];
        ftb_classes(W, tau, c);
        fprintf(stderr, "     ftb x %.1e u %.1e w %.1e s %.1e sf %.1e p %.1e n %.1e\n", c[0], c[1], c[2], c[3], c[4], c[5], c[6]);
    }
    if (skip_first) {
        /* the iterate is the watchdog's stored one: re-linearise it for the caller */
        linearise(W);
        *th0p = th0;
        *phi0p = phi0;
    }
    *alpha_out = alpha;
    *az_out = az;
    return accepted != 0;
}

/* original-problem theta / phi at the current iterate (also valid at a restoration iterate: the shared
 * variables x, u, w, s, sf); *pmax: the original problem's primal infeasibility (max norm) */
static void orig_th_phi(ws_t* W, double mu, double* th, double* ph, double* pmax) {
    double rfo[6] = {0};
    residuals(W, W->c, W->d, W->s, W->df, W->sf, NULL, NULL, W->cr, W->dr, rfo);
    *th = infeas1(W, W->cr, W->dr, rfo);
    double m = 0.0;
    for (int i = 0; i < W->nrc; ++i) m = fmax(m, fabs(W->cr[i]));
    for (int i = 0; i < W->nrd; ++i) m = fmax(m, fabs(W->dr[i]));
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) m = fmax(m, fabs(rfo[i]));
    *pmax = m;
    int bad = 0;
    const double b = barrier(W, W->x, W->u, W->w, W->s, W->sf, NULL, NULL, mu, &bad);
    *ph = bad ? INFINITY : cost_eval(W, W->x, W->u) + b;
}

/* The primal-dual iterate in the layout of the kernel's diagnostic export (include/ttmpc.h tt_obca_iterate_len):
 * per stage k (30): x 6, u 2, zLx 6, zUx 6, zLu 2, zUu 2, yc 6 (u, zLu, zUu zero at k = N); per block bi = k nbk + j
 * (32): w 8, zw 8, s 4, vL 4, vU 4, yd 4; then the final-box rows (24): sf 6, vLf 6, vUf 6, ydf 6 (zero in track mode). */
static void pack_iterate(const ws_t* W, double* it) {
    const int N = W->N;
    for (int k = 0; k <= N; ++k) {
        double* q = it + 30 * (size_t)k;
        for (int i = 0; i < 6; ++i) {
            q[i] = W->x[6 * k + i]; q[8 + i] = W->zLx[6 * k + i]; q[14 + i] = W->zUx[6 * k + i]; q[24 + i] = W->yc[6 * k + i];
        }
        for (int i = 0; i < 2; ++i) {
            q[6 + i] = k < N ? W->u[2 * k + i] : 0.0;
            q[20 + i] = k < N ? W->zLu[2 * k + i] : 0.0;
            q[22 + i] = k < N ? W->zUu[2 * k + i] : 0.0;
        }
    }
    double* bq = it + 30 * ((size_t)N + 1);
    for (int bi = 0; bi < W->nb; ++bi) {
        double* q = bq + 32 * (size_t)bi;
        for (int e = 0; e < 8; ++e) { q[e] = W->w[8 * bi + e]; q[8 + e] = W->zw[8 * bi + e]; }
        for (int r = 0; r < 4; ++r) {
            q[16 + r] = W->s[4 * bi + r]; q[20 + r] = W->vL[4 * bi + r]; q[24 + r] = W->vU[4 * bi + r];
            q[28 + r] = W->yd[4 * bi + r];
        }
    }
    double* f = bq + 32 * (size_t)W->nb;
    for (int i = 0; i < 6; ++i) {
        const int pl = W->mode == TTO_OBCA_PLAN;
        f[i] = pl ? W->sf[i] : 0.0; f[6 + i] = pl ? W->vLf[i] : 0.0; f[12 + i] = pl ? W->vUf[i] : 0.0;
        f[18 + i] = pl ? W->ydf[i] : 0.0;
    }
}

static void unpack_iterate(ws_t* W, const double* it) {
    const int N = W->N;
    for (int k = 0; k <= N; ++k) {
        const double* q = it + 30 * (size_t)k;
        for (int i = 0; i < 6; ++i) {
            W->x[6 * k + i] = q[i]; W->zLx[6 * k + i] = q[8 + i]; W->zUx[6 * k + i] = q[14 + i]; W->yc[6 * k + i] = q[24 + i];
        }
        if (k < N)
            for (int i = 0; i < 2; ++i) { W->u[2 * k + i] = q[6 + i]; W->zLu[2 * k + i] = q[20 + i]; W->zUu[2 * k + i] = q[22 + i]; }
    }
    const double* bq = it + 30 * ((size_t)N + 1);
    for (int bi = 0; bi < W->nb; ++bi) {
        const double* q = bq + 32 * (size_t)bi;
        for (int e = 0; e < 8; ++e) { W->w[8 * bi + e] = q[e]; W->zw[8 * bi + e] = q[8 + e]; }
        for (int r = 0; r < 4; ++r) {
            W->s[4 * bi + r] = q[16 + r]; W->vL[4 * bi + r] = q[20 + r]; W->vU[4 * bi + r] = q[24 + r];
            W->yd[4 * bi + r] = q[28 + r];
        }
    }
    const double* f = bq + 32 * (size_t)W->nb;
    for (int i = 0; i < 6; ++i) { W->sf[i] = f[i]; W->vLf[i] = f[6 + i]; W->vUf[i] = f[12 + i]; W->ydf[i] = f[18 + i]; }
}

/* weights, bounds (bound_relax_factor 1e-8 on every finite bound), row bounds */
static void setup_bounds(ws_t* W) {
    const tto_obca_problem* P = W->P;
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) W->Qc[i * 6 + j] = 0.5 * (P->Q[i * 6 + j] + P->Q[j * 6 + i]);
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) W->Rc[i * 2 + j] = 0.5 * (P->R[i * 2 + j] + P->R[j * 2 + i]);
    for (int i = 0; i < 6; ++i) {
        W->hxl[i] = !isfree(P->xlb[i]); W->hxu[i] = !isfree(P->xub[i]);
        W->xl[i] = W->hxl[i] ? P->xlb[i] - RELAX * fmax(1.0, fabs(P->xlb[i])) : -INFINITY;
        W->xu[i] = W->hxu[i] ? P->xub[i] + RELAX * fmax(1.0, fabs(P->xub[i])) : INFINITY;
    }
    for (int i = 0; i < 2; ++i) {
        W->hul[i] = !isfree(P->ulb[i]); W->huu[i] = !isfree(P->uub[i]);
        W->ul[i] = W->hul[i] ? P->ulb[i] - RELAX * fmax(1.0, fabs(P->ulb[i])) : -INFINITY;
        W->uu[i] = W->huu[i] ? P->uub[i] + RELAX * fmax(1.0, fabs(P->uub[i])) : INFINITY;
    }
    /* row bounds: d1 <= 0, d2/d3 in [-eq_tol, eq_tol], d4 <= 0; final |.| <= fin_tol */
    W->hrL[0] = 0; W->hrU[0] = 1; W->rU[0] = RELAX;
    for (int r = 1; r < 3; ++r) {
        W->hrL[r] = 1; W->hrU[r] = 1;
        W->rL[r] = -P->eq_tol - RELAX; W->rU[r] = P->eq_tol + RELAX;
    }
    W->hrL[3] = 0; W->hrU[3] = 1; W->rU[3] = RELAX;
    W->rL[0] = W->rL[3] = -INFINITY;
    W->fL = -P->fin_tol - RELAX; W->fU = P->fin_tol + RELAX;
}

static int solve_one(ws_t* W, const double* xinit, const double* xgoal, const double* xref, const double* uref,
                     const double* zg, double* zout, int* iters_out, double* kkt_out, double* it_out) {
    const tto_obca_problem* P = W->P;
    const int N = W->N;
    W->xinit = xinit; W->xgoal = xgoal; W->xref = xref; W->uref = uref;
    memset(g_cen, 0, sizeof(g_cen));
    W->R = M_ORIG;
    W->lsq = 0;
    W->have_acc = 0;
    W->kd = (P->opts & TTO_OPT_KAPPA_D) ? KAPPA_D : 0.0;
    W->dbg = (getenv("TTO_DEBUG") ? 1 : 0) | (getenv("TTO_DEBUG2") ? 2 : 0) | (getenv("TTO_CHECK") ? 4 : 0);
    const int dbg = W->dbg & 1;
    const int use_resto = !(P->opts & TTO_OPT_NO_RESTO), use_soft = !(P->opts & TTO_OPT_NO_SOFT_RESTO);
    setup_bounds(W);

    if (zg) unpack(W, zg); else { default_guess(W, zout); unpack(W, zout); }
    if (P->dual_init)
        for (int k = 0; k <= N; ++k)
            for (int j = 0; j < W->nbk; ++j) dual_certificate(P, W->x + 6 * k, j, W->w + 8 * (k * W->nbk + j));
    int status = 2, iter = 0;
    double E0 = INFINITY;
    for (int i = 0; i < 6; ++i)
        if (!isfinite(xinit[i]) || (W->hxl[i] && xinit[i] < W->xl[i]) || (W->hxu[i] && xinit[i] > W->xu[i])) status = 3;
    if (status == 3) {
        pack(W, zout);
        if (it_out) memset(it_out, 0, tto_obca_iterate_len(N, P->M) * sizeof(double));
        if (iters_out) *iters_out = 0;
        if (kkt_out) *kkt_out = INFINITY;
        return 3;
    }
    /* bound push of the primal guess, slacks = d(x0) pushed, bound multipliers 1, constraint multipliers by
     * least squares */
    for (int k = 0; k <= N; ++k) {
        for (int i = 0; i < 6; ++i) push_into(&W->x[6 * k + i], W->xl[i], W->xu[i], W->hxl[i], W->hxu[i]);
        if (k < N)
            for (int i = 0; i < 2; ++i) push_into(&W->u[2 * k + i], W->ul[i], W->uu[i], W->hul[i], W->huu[i]);
    }
    for (int v = 0; v < 8 * W->nb; ++v) push_into(&W->w[v], -RELAX, INFINITY, 1, 0);
    obca_cons(W, W->x, W->w, W->d, W->df);
    for (int bi = 0; bi < W->nb; ++bi)
        for (int r = 0; r < 4; ++r) {
            W->s[4 * bi + r] = W->d[4 * bi + r];
            push_into(&W->s[4 * bi + r], W->rL[r], W->rU[r], W->hrL[r], W->hrU[r]);
            W->vL[4 * bi + r] = W->hrL[r] ? 1.0 : 0.0;
            W->vU[4 * bi + r] = W->hrU[r] ? 1.0 : 0.0;
            W->yd[4 * bi + r] = 0.0;
        }
    for (int v = 0; v < 8 * W->nb; ++v) W->zw[v] = 1.0;
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            W->sf[i] = W->df[i];
            push_into(&W->sf[i], W->fL, W->fU, 1, 1);
            W->vLf[i] = W->vUf[i] = 1.0;
            W->ydf[i] = 0.0;
        }
    for (int k = 0; k <= N; ++k) {
        for (int i = 0; i < 6; ++i) {
            W->zLx[6 * k + i] = W->hxl[i] ? 1.0 : 0.0;
            W->zUx[6 * k + i] = W->hxu[i] ? 1.0 : 0.0;
            W->yc[6 * k + i] = 0.0;
        }
        if (k < N)
            for (int i = 0; i < 2; ++i) {
                W->zLu[2 * k + i] = W->hul[i] ? 1.0 : 0.0;
                W->zUu[2 * k + i] = W->huu[i] ? 1.0 : 0.0;
            }
    }
    if (!(P->opts & TTO_OPT_NO_LSQ_MULT)) ls_multipliers(W);

    ipm_state_t SO, SR;
    ipm_reset(&SO, 0.1);
    ipm_reset(&SR, 0.1);
    const double kappa_eps = BARRIER_TOL_FACTOR, kappa_mu = 0.2, theta_mu = 1.5;
    const double mu_min = fmin(P->tol, COMPL_INF_TOL) / (BARRIER_TOL_FACTOR + 1.0);
    int in_soft = 0, soft_cnt = 0, first_resto = 0, n_resto = 0, n_soft = 0, fallback = 0, resto_iter0 = 0;
    double th_resto0 = 0.0;
    for (iter = 0;; ++iter) {
        ipm_state_t* S = W->R == M_RESTO ? &SR : &SO;
        linearise(W);
        opterr_t oe = opt_error(W, S->mu);
        E0 = oe.E0;
        if (!oe.finite) { status = 4; break; }
        if (W->R == M_ORIG) {
            if (dbg) fprintf(stderr, "it %4d E0 %.3e dinf %.3e pinf %.3e mu %.2e f %.6e\n", iter, E0, oe.dinf, oe.pinf,
                             S->mu, cost_eval(W, W->x, W->u));
            const int accp = acceptable_pt(&oe, P->acc_tol);
            if (converged(&oe, P->tol)) { status = 0; break; }
            if (accp) {
                memcpy(W->xacc, W->x, 6 * ((size_t)N + 1) * 8);
                memcpy(W->uacc, W->u, 2 * (size_t)N * 8);
                memcpy(W->wacc, W->w, 8 * (size_t)W->nb * 8);
                W->have_acc = 1;
                if (++S->acc_count >= P->acc_iter) { status = 1; break; }
            } else {
                S->acc_count = 0;
            }
            if (iter >= P->max_iter) { status = accp ? 1 : 2; break; }
        } else {
            /* restoration convergence (RestoConvergenceCheck): original infeasibility reduced to kappa_resto of
             * its value at entry and the point acceptable to the augmented original filter */
            double thO, phO, pinfO;
            orig_th_phi(W, SO.mu, &thO, &phO, &pinfO);
            if (dbg) fprintf(stderr, "rit %3d E0 %.3e dinf %.3e pinf %.3e muR %.2e thO %.3e (%.3e)\n", iter, E0, oe.dinf,
                             oe.pinf, S->mu, thO, th_resto0);
            if (!first_resto && thO <= KAPPA_RESTO * th_resto0 && thO <= SO.th_max && !in_filter(&SO.F, thO, phO)) {
                leave_resto(W, SO.mu, SO.tau);
                SO.acc_count = 0;
                --iter; /* the return itself is not an iteration */
                continue;
            }
            first_resto = 0;
            if (acceptable_pt(&oe, P->acc_tol)) ++S->acc_count; else S->acc_count = 0;
            if (converged(&oe, P->tol) || S->acc_count >= P->acc_iter) {
                /* the restoration NLP converged (or converged to an acceptable point) without reaching a point
                 * acceptable to the original problem: IPOPT (RestoConvergenceCheck) compares the ORIGINAL problem's
                 * primal infeasibility (max norm) with resto_failure_feasibility_threshold (default 1e2 tol) */
                if (pinfO <= 1e2 * P->tol) {
                    leave_resto(W, SO.mu, SO.tau); /* feasible but filter-unacceptable: continue with a fresh filter */
                    SO.F.n = 0;
                    --iter;
                    continue;
                }
                status = 3; /* IPOPT: converged to a point of local infeasibility */
                break;
            }
            if (iter >= P->max_iter) { status = 2; break; }
        }
        /* barrier update (monotone, Fiacco-McCormick); the filter is reset on every change */
        while (oe.Emu <= kappa_eps * S->mu && S->mu > mu_min * 1.0000001) {
            S->mu = fmax(mu_min, fmin(kappa_mu * S->mu, pow(S->mu, theta_mu)));
            S->tau = fmax(0.99, 1.0 - S->mu);
            S->F.n = 0;
            if (W->R == M_RESTO) { W->zeta = sqrt(S->mu); obj_grad(W); }
            oe = opt_error(W, S->mu);
        }
        const double mu = S->mu;
        int bad = 0;
        double th0 = infeas1(W, W->rc0, W->rd0, W->rf0);
        double phi0 = (W->R == M_RESTO ? resto_obj(W, W->x, W->u, W->w, W->pr, W->nr) : cost_eval(W, W->x, W->u)) +
                            barrier(W, W->x, W->u, W->w, W->s, W->sf, W->R == M_RESTO ? W->pr : NULL,
                                    W->R == M_RESTO ? W->nr : NULL, mu, &bad);
        double dw = 0.0, alpha = 0.0, az = 0.0;
        int accepted = 0;
        if (fallback || newton(W, S, &dw) != 0) {
            fallback = 0;
            if (W->R == M_RESTO || !use_resto) { status = 5; break; } /* IPOPT Error_In_Step_Computation */
            goto restoration;                                         /* IPOPT's fallback: restoration phase */
        }
        if (W->R == M_ORIG && in_soft) {
            accepted = 0; /* handled below as a soft restoration step */
        } else {
            accepted = line_search(W, S, (W->R == M_RESTO ? iter == resto_iter0 : iter == 0), &th0, &phi0, &alpha, &az);
            if (!accepted) oe = opt_error(W, mu); /* a stopped watchdog may have restored its stored iterate */
        }
        if (!accepted && W->R == M_ORIG && use_soft && (in_soft ? ++soft_cnt <= MAX_SOFT_RESTO : 1)) {
            /* soft restoration step (BacktrackingLineSearch::TrySoftRestoStep): primal and dual step
             * min(alpha_p, alpha_d); accepted when acceptable to the filter or when the primal-dual error
             * at mu drops by 0.9999 */
            const double ap = ftb_primal(W, S->tau), azd = ftb_dual(W, S->tau), as = fmin(ap, azd);
            set_trial(W, as);
            double tht, pht;
            trial_eval(W, mu, &tht, &pht);
            const double g_th = 1e-5, g_ph = 1e-8, tolc = 10.0 * DBL_EPSILON;
            const int orig_ok = isfinite(pht) && tht <= S->th_max && !in_filter(&S->F, tht, pht) &&
                                (tht <= (1.0 - g_th) * th0 || pht - (phi0 - g_ph * th0) <= tolc * fabs(phi0));
            int acc_soft = orig_ok;
            if (!orig_ok && isfinite(pht)) {
                snapshot(W, 0);
                take_step(W, mu, as, as);
                linearise(W);
                const opterr_t ot = opt_error(W, mu);
                snapshot(W, 1);
                linearise(W);
                acc_soft = ot.finite && ot.pderr <= SOFT_RESTO_FACTOR * oe.pderr;
            }
            if (acc_soft) {
                ++n_soft;
                add_filter(&S->F, (1.0 - g_th) * th0, phi0 - g_ph * th0);
                in_soft = !orig_ok;
                if (orig_ok) soft_cnt = 0;
                if (dbg) fprintf(stderr, "     soft-resto step a %.3e (orig %d)\n", as, orig_ok);
                take_step(W, mu, as, as);
                continue;
            }
        }
        if (!accepted) {
            if (W->R == M_RESTO) {
                if (th0 <= 1e-2 * P->tol) {
                    /* the restoration NLP's own line search failed at one of its almost feasible points: IPOPT
                     * (BacktrackingLineSearch, inside the restoration algorithm) tries to restore an acceptable
                     * point of that NLP and otherwise throws RESTORATION_FAILED, which ends the solve
                     * (Restoration_Failed; status 3 here) instead of resetting p/n forever */
                    status = 3;
                    break;
                }
                /* restoration of the restoration phase: elastic variables back to their closed form */
                set_pn(W, mu);
                S->F.n = 0;
                if (dbg) fprintf(stderr, "     resto line search failed: p/n reset\n");
                continue;
            }
            if (!use_resto) { S->F.n = 0; take_step(W, mu, alpha, az); continue; } /* round-1 fallback (opt-out) */
        restoration:
            in_soft = 0;
            soft_cnt = 0;
            if (th0 <= 1e-2 * P->tol) {
                /* restoration called at an almost feasible point: IPOPT restores the last acceptable iterate
                 * (Solved_To_Acceptable_Level) or stops with Restoration_Failed */
                if (W->have_acc) {
                    memcpy(W->x, W->xacc, 6 * ((size_t)N + 1) * 8);
                    memcpy(W->u, W->uacc, 2 * (size_t)N * 8);
                    memcpy(W->w, W->wacc, 8 * (size_t)W->nb * 8);
                    status = 1;
                } else {
                    status = 3;
                }
                break;
            }
            {
                /* PrepareRestoPhaseStart: the current iterate enters the original filter */
                const double g_th = 1e-5, g_ph = 1e-8;
                if (isfinite(phi0)) add_filter(&SO.F, (1.0 - g_th) * th0, phi0 - g_ph * th0);
                if (!(SO.th_max > 0)) { SO.th_max = 1e4 * fmax(1.0, th0); SO.th_min = 1e-4 * fmax(1.0, th0); }
                th_resto0 = th0;
                const double muR = enter_resto(W, SO.mu);
                if (!(P->opts & TTO_OPT_NO_LSQ_MULT)) ls_multipliers(W);
                ipm_reset(&SR, muR);
                first_resto = 1;
                resto_iter0 = iter;
                ++n_resto;
                if (dbg) fprintf(stderr, "     -> restoration #%d (theta %.3e, muR %.3e)\n", n_resto, th0, muR);
            }
            --iter; /* entering is not an iteration */
            continue;
        }
        if (dbg) fprintf(stderr, "     alpha %.3e (ap %.3e acc %d Dm %.2e) az %.3e dw %.2e th %.3e nf %d\n", alpha, g_dbg_ap, g_dbg_acc, g_dbg_sw, az, dw, th0, S->F.n);
        take_step(W, mu, alpha, az);
    }
    if (W->R == M_RESTO) W->R = M_ORIG;
    if (dbg) fprintf(stderr, "status %d iters %d resto %d soft %d\n", status, iter, n_resto, n_soft);
    if (getenv("TTO_CENSUS"))
        fprintf(stderr, "CENSUS status %d iters %d fact %ld blocks_ok %ld few %ld many %ld zero %ld ref>1e-10 %ld ref>1e-5 %ld pretend %ld corr %ld solves %ld\n",
                status, iter, g_cen[0], g_cen[4], g_cen[1], g_cen[2], g_cen[3], g_cen[5], g_cen[6], g_cen[7], g_cen[8], g_cen[9]);
    pack(W, zout);
    if (it_out) pack_iterate(W, it_out);
    if (iters_out) *iters_out = iter;
    if (kkt_out) *kkt_out = E0;
    return status;
}

int tto_obca_solve(const tto_obca_problem* P, const double* x_init, const double* x_goal, const double* xref,
                   const double* uref, const double* z_guess, double* z_out, int* iters, double* kkt) {
    if (P->N < 1 || P->M < 1 || P->M > TTO_MAXM) return -1;
    if (P->mode == TTO_OBCA_PLAN && !x_goal) return -1;
    if (P->mode == TTO_OBCA_TRACK && (!xref || !uref)) return -1;
    ws_t W;
    if (ws_init(&W, P) != 0) return -1;
    const int st = solve_one(&W, x_init, x_goal, xref, uref, z_guess, z_out, iters, kkt, NULL);
    free(W.mem);
    return st;
}

int tto_obca_solve_batch(const tto_obca_problem* P, int B, const double* x_init, const double* x_goal,
                         const double* xref, const double* uref, const double* z_guess, double* z_out,
                         int* status, int* iters, double* kkt, int nthreads) {
    return tto_obca_solve_batch_it(P, B, x_init, x_goal, xref, uref, z_guess, z_out, status, iters, kkt, NULL, nthreads);
}

int tto_obca_solve_batch_it(const tto_obca_problem* P, int B, const double* x_init, const double* x_goal,
                            const double* xref, const double* uref, const double* z_guess, double* z_out,
                            int* status, int* iters, double* kkt, double* it_out, int nthreads) {
    if (P->N < 1 || P->M < 1 || P->M > TTO_MAXM || B < 0) return -1;
    const int N = P->N;
    const size_t n = (size_t)N * (8 + 16 * P->M) + 6 + 16 * P->M;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    int err = 0;
#pragma omp parallel
    {
        ws_t W;
        const int bad = ws_init(&W, P);
#pragma omp for schedule(dynamic, 1)
        for (int b = 0; b < B; ++b) {
            if (bad) { status[b] = -1; continue; }
            int it = 0;
            double e = 0.0;
            status[b] = solve_one(&W, x_init + 6 * (size_t)b, x_goal ? x_goal + 6 * (size_t)b : NULL,
                                  xref ? xref + (size_t)b * 6 * (N + 1) : NULL, uref ? uref + (size_t)b * 2 * N : NULL,
                                  z_guess ? z_guess + (size_t)b * n : NULL, z_out + (size_t)b * n, &it, &e,
                                  it_out ? it_out + (size_t)b * tto_obca_iterate_len(N, P->M) : NULL);
            if (iters) iters[b] = it;
            if (kkt) kkt[b] = e;
        }
        if (bad) err = -1;
        free(W.mem);
    }
    return err;
}

/* test hook: one OBCA block's linearisation (values, Jacobians, y-weighted Hessians) for finite-difference
 * checks in tests/test_obca_oracle.py */
void tto_obca_block_lin(const tto_obca_problem* P, const double* xk, int j, const double* wv, const double* y,
                        double* d, double* Jx, double* Jw, double* Hxx, double* Hxw, double* Hww) {
    blk_lin(P, xk, j, wv, y, d, Jx, Jw, Hxx, Hxw, Hww);
}

long long tto_obca_iterate_len(int N, int M) { return 30LL * (N + 1) + 64LL * M * (N + 1) + 24; }

/* IPOPT's optimality error at a GIVEN primal-dual point (the GPU's returned iterate, or the oracle's own), in the
 * original problem: out = {E_0 (scaled, IPOPT eq. (5)), unscaled dual infeasibility, primal infeasibility (max norm of
 * the dynamics / slack / final rows), complementarity max |z s|, s_d, s_c, converged (IPOPT's test at P->tol),
 * acceptable}.  The point must be strictly interior (the slacks inside their relaxed bounds); returns -1 if not. */
int tto_obca_eval_iterate(const tto_obca_problem* P, const double* x_init, const double* x_goal, const double* xref,
                          const double* uref, const double* it, double* out) {
    if (P->N < 1 || P->M < 1 || P->M > TTO_MAXM) return -1;
    ws_t W;
    if (ws_init(&W, P) != 0) return -1;
    W.xinit = x_init; W.xgoal = x_goal; W.xref = xref; W.uref = uref;
    W.R = M_ORIG;
    setup_bounds(&W);
    unpack_iterate(&W, it);
    int bad = 0;
    (void)barrier(&W, W.x, W.u, W.w, W.s, W.sf, NULL, NULL, 1.0, &bad);
    linearise(&W);
    const opterr_t o = opt_error(&W, 0.0);
    out[0] = o.E0; out[1] = o.dinf; out[2] = o.pinf; out[3] = o.c0; out[4] = o.sd; out[5] = o.sc;
    out[6] = converged(&o, P->tol); out[7] = acceptable_pt(&o, P->acc_tol);
    free(W.mem);
    return bad ? -1 : 0;
}
