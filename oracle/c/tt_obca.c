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
 * Algorithm: the same restatement of IPOPT's primal-dual barrier method as tt_oracle.c (IPOPT defaults
 * of trajectory_optimization.py:196-199: tol 1e-8, acceptable 1e-6 x 15, monotone mu from 0.1,
 * bound_relax_factor 1e-8 on variable AND constraint bounds, bound_push/frac 1e-2, kappa_sigma 1e10),
 * extended by IPOPT's slack formulation of inequality rows: d(x) - s = 0, d_L <= s <= d_U, with
 * multipliers y_d and slack-bound multipliers v_L, v_U.
 *
 * Newton system (new-multiplier form, D = Sigma_s + delta_w):
 *   (W + Sigma_x + dw) dx + J_c' y_c+ + J_d' y_d+ = -grad phi_x
 *   D ds - y_d+ = -grad phi_s,  J_c dx = -c,  J_d dx - ds = -(d - s)
 * Slacks and y_d are eliminated (y_d+ = D (J_d dx + r_d), r_d = d - s + D^-1 grad phi_s); every OBCA block
 * (8 duals mu/lam, 4 rows) couples only to (X, Y, theta, psi) of its stage, so its 8x8 block
 * K = W_ww + Sigma_w + dw + Jw' D Jw is Cholesky-factorised and Schur-eliminated into the 6x6 stage
 * Hessian; the remaining stage-wise LQ problem is solved by a Riccati recursion.  Inertia test: every
 * K and every Riccati input block R~ + B'PB must be positive definite (otherwise dw is raised with
 * IPOPT's 1e-4 / x100 / x8 / /3 schedule).  Globalisation: IPOPT's filter line search with up to
 * four second-order corrections; where IPOPT would enter its restoration phase we take the
 * smallest tried step and reset the filter (only the iterate path can differ, not the KKT point).
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

static int isfree(double b) { return !isfinite(b) || fabs(b) >= 1e19; }

typedef struct {
    const tto_obca_problem* P;
    int N, M, nbk, nb, n, mode;
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
    double *A, *c, *d, *gx, *gu, *Wd, *Jx, *Jw, *Hxx, *Hxw, *Hww;
    double df[6];
    /* factorisation */
    double *Dd, *L, *V, *Qt, *Rt, *Pm, *G, *H, *K;
    double Df[6];
    /* rhs + step */
    double *qt, *rt, *vv, *rd, *pv, *kf, *Yb, *LT, *Gm, *tv;
    double rf[6];
    double *dx, *du, *dw, *ds, *ycp, *ydp, *dzLx, *dzUx, *dzLu, *dzUu, *dzw, *dvL, *dvU;
    double dsf[6], ydpf[6], dvLf[6], dvUf[6];
    /* trial + soc */
    double *xt, *ut, *wt, *st, *ct, *dtr, *cr, *dr;
    double sft[6], dft[6], dfr[6];
    double fth[TTO_MAXF], fph[TTO_MAXF];
    int nf;
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
    const size_t N1 = (size_t)P->N + 1, N = (size_t)P->N, nb = (size_t)W->nb;
    size_t tot = 0;
#define NEED(cnt) tot += (cnt)
    /* count */
    NEED(N1 * 6); NEED(N * 2); NEED(nb * 8); NEED(nb * 4);              /* x u w s */
    NEED(N1 * 6 * 2); NEED(N * 2 * 2); NEED(nb * 8); NEED(nb * 4 * 2);  /* zLx zUx zLu zUu zw vL vU */
    NEED(N1 * 6); NEED(nb * 4);                                          /* yc yd */
    NEED(N * 36); NEED(N1 * 6); NEED(nb * 4); NEED(N1 * 6); NEED(N * 2); NEED(N * 36);  /* A c d gx gu Wd */
    NEED(nb * 16); NEED(nb * 32); NEED(nb * 16); NEED(nb * 32); NEED(nb * 16);          /* Jx Jw Hxx Hxw Hww */
    NEED(nb * 4); NEED(nb * 64); NEED(nb * 32); NEED(N1 * 36); NEED(N * 4);              /* Dd L V Qt Rt */
    NEED(N1 * 36); NEED(N * 4); NEED(N * 12); NEED(N * 12);                              /* Pm G H K */
    NEED(N1 * 6); NEED(N * 2); NEED(nb * 8); NEED(nb * 4); NEED(N1 * 6); NEED(N * 2);    /* qt rt vv rd pv kf */
    NEED(N1 * 6); NEED(N * 2); NEED(nb * 8); NEED(nb * 4); NEED(N1 * 6); NEED(nb * 4);   /* dx du dw ds ycp ydp */
    NEED(N1 * 6 * 2); NEED(N * 2 * 2); NEED(nb * 8); NEED(nb * 4 * 2);                   /* dz* dzw dvL dvU */
    NEED(N1 * 6); NEED(N * 2); NEED(nb * 8); NEED(nb * 4); NEED(N1 * 6); NEED(nb * 4);   /* xt ut wt st ct dtr */
    NEED(N1 * 6); NEED(nb * 4);                                                           /* cr dr */
    NEED(nb * 32); NEED(nb * 16); NEED(nb * 16); NEED(nb * 4);                           /* Yb LT Gm tv */
#undef NEED
    W->mem = (double*)calloc(tot, sizeof(double));
    if (!W->mem) return -1;
    double* q = W->mem;
#define TAKE(ptr, cnt) (ptr = q, q += (cnt))
    TAKE(W->x, N1 * 6); TAKE(W->u, N * 2); TAKE(W->w, nb * 8); TAKE(W->s, nb * 4);
    TAKE(W->zLx, N1 * 6); TAKE(W->zUx, N1 * 6); TAKE(W->zLu, N * 2); TAKE(W->zUu, N * 2); TAKE(W->zw, nb * 8);
    TAKE(W->vL, nb * 4); TAKE(W->vU, nb * 4);
    TAKE(W->yc, N1 * 6); TAKE(W->yd, nb * 4);
    TAKE(W->A, N * 36); TAKE(W->c, N1 * 6); TAKE(W->d, nb * 4); TAKE(W->gx, N1 * 6); TAKE(W->gu, N * 2);
    TAKE(W->Wd, N * 36);
    TAKE(W->Jx, nb * 16); TAKE(W->Jw, nb * 32); TAKE(W->Hxx, nb * 16); TAKE(W->Hxw, nb * 32); TAKE(W->Hww, nb * 16);
    TAKE(W->Dd, nb * 4); TAKE(W->L, nb * 64); TAKE(W->V, nb * 32); TAKE(W->Qt, N1 * 36); TAKE(W->Rt, N * 4);
    TAKE(W->Pm, N1 * 36); TAKE(W->G, N * 4); TAKE(W->H, N * 12); TAKE(W->K, N * 12);
    TAKE(W->qt, N1 * 6); TAKE(W->rt, N * 2); TAKE(W->vv, nb * 8); TAKE(W->rd, nb * 4); TAKE(W->pv, N1 * 6);
    TAKE(W->kf, N * 2);
    TAKE(W->dx, N1 * 6); TAKE(W->du, N * 2); TAKE(W->dw, nb * 8); TAKE(W->ds, nb * 4); TAKE(W->ycp, N1 * 6);
    TAKE(W->ydp, nb * 4);
    TAKE(W->dzLx, N1 * 6); TAKE(W->dzUx, N1 * 6); TAKE(W->dzLu, N * 2); TAKE(W->dzUu, N * 2); TAKE(W->dzw, nb * 8);
    TAKE(W->dvL, nb * 4); TAKE(W->dvU, nb * 4);
    TAKE(W->xt, N1 * 6); TAKE(W->ut, N * 2); TAKE(W->wt, nb * 8); TAKE(W->st, nb * 4); TAKE(W->ct, N1 * 6);
    TAKE(W->dtr, nb * 4);
    TAKE(W->cr, N1 * 6); TAKE(W->dr, nb * 4);
    TAKE(W->Yb, nb * 32); TAKE(W->LT, nb * 16); TAKE(W->Gm, nb * 16); TAKE(W->tv, nb * 4);
#undef TAKE
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

static void cost_grad(ws_t* W) {
    const tto_obca_problem* P = W->P;
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

/* barrier value over every bounded component; returns 0 and sets *bad if any slack is <= 0 */
static double barrier(const ws_t* W, const double* x, const double* u, const double* w, const double* s,
                      const double* sf, double mu, int* bad) {
    double b = 0.0;
    *bad = 0;
#define BL(val, lo) do { double t_ = (val) - (lo); if (!(t_ > 0)) { *bad = 1; return 0; } b -= mu * log(t_); } while (0)
#define BU(val, hi) do { double t_ = (hi) - (val); if (!(t_ > 0)) { *bad = 1; return 0; } b -= mu * log(t_); } while (0)
    for (int k = 0; k <= W->N; ++k) {
        for (int i = 0; i < 6; ++i) {
            if (W->hxl[i]) BL(x[6 * k + i], W->xl[i]);
            if (W->hxu[i]) BU(x[6 * k + i], W->xu[i]);
        }
        if (k < W->N)
            for (int i = 0; i < 2; ++i) {
                if (W->hul[i]) BL(u[2 * k + i], W->ul[i]);
                if (W->huu[i]) BU(u[2 * k + i], W->uu[i]);
            }
    }
    for (int bi = 0; bi < W->nb; ++bi) {
        for (int e = 0; e < 8; ++e) BL(w[8 * bi + e], -RELAX);
        for (int r = 0; r < 4; ++r) {
            if (W->hrL[r]) BL(s[4 * bi + r], W->rL[r]);
            if (W->hrU[r]) BU(s[4 * bi + r], W->rU[r]);
        }
    }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) { BL(sf[i], W->fL); BU(sf[i], W->fU); }
#undef BL
#undef BU
    return b;
}

static double infeas1(const ws_t* W, const double* c, const double* d, const double* s, const double* df,
                      const double* sf) {
    double t = 0.0;
    for (int i = 0; i < 6 * (W->N + 1); ++i) t += fabs(c[i]);
    for (int i = 0; i < 4 * W->nb; ++i) t += fabs(d[i] - s[i]);
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) t += fabs(df[i] - sf[i]);
    return t;
}

/* ------------------------------------------------------------------ small dense helpers */
static int chol(double* a, int n) { /* in-place lower Cholesky, row-major n x n; 0 ok */
    for (int j = 0; j < n; ++j) {
        double s = a[j * n + j];
        for (int k = 0; k < j; ++k) s -= a[j * n + k] * a[j * n + k];
        if (!(s > 0.0)) return -1;
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
static double bgrad_x(const ws_t* W, int k, int i, double mu) {
    const double v = W->x[6 * k + i];
    double g = W->gx[6 * k + i];
    if (W->hxl[i]) g -= mu / (v - W->xl[i]);
    if (W->hxu[i]) g += mu / (W->xu[i] - v);
    return g;
}
static double bgrad_u(const ws_t* W, int k, int i, double mu) {
    const double v = W->u[2 * k + i];
    double g = W->gu[2 * k + i];
    if (W->hul[i]) g -= mu / (v - W->ul[i]);
    if (W->huu[i]) g += mu / (W->uu[i] - v);
    return g;
}
static double bgrad_s(const ws_t* W, int r, double sv, double mu) {
    double g = 0.0;
    if (W->hrL[r]) g -= mu / (sv - W->rL[r]);
    if (W->hrU[r]) g += mu / (W->rU[r] - sv);
    return g;
}
static double sig_s(const ws_t* W, int bi, int r) {
    const double sv = W->s[4 * bi + r];
    double s = 0.0;
    if (W->hrL[r]) s += W->vL[4 * bi + r] / (sv - W->rL[r]);
    if (W->hrU[r]) s += W->vU[4 * bi + r] / (W->rU[r] - sv);
    return s;
}

/* linearise at the current iterate (values, Jacobians, y-weighted Hessians) */
static void linearise(ws_t* W) {
    const tto_obca_problem* P = W->P;
    cost_grad(W);
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
}

/* One OBCA block's elimination into its stage Hessian Q (6x6, rows/cols X,Y,theta,psi touched).
 * Local system in (dw, y+):  M = [[A, C'], [C, -E]],  A = W_ww + Sigma_w + dw (8x8), C = Jw (4x8),
 * E = D^-1 (D = Sigma_s + dw), coupled to dx^ by b1 = W_wx (8x4) and b2 = Jx (4x4).  With A = L L',
 * Y = L^-1 C', Z = L^-1 b1, T = E + Y'Y = L_T L_T', G = Y'Z - b2, the Schur complement onto dx^ is
 *     W_xx - Z'Z + G' T^-1 G
 * which never forms C' D C: with D ~ 1e10 on the near-equality range rows that product cancels
 * catastrophically, while T stays well conditioned.  Inertia: A must be positive definite. */
static int block_factor(ws_t* W, int bi, double dw, double* Q) {
    const double *Jx = W->Jx + 16 * bi, *Jw = W->Jw + 32 * bi;
    double* D = W->Dd + 4 * bi;
    for (int r = 0; r < 4; ++r) D[r] = sig_s(W, bi, r) + dw;
    double* Lb = W->L + 64 * bi;
    memset(Lb, 0, 64 * sizeof(double));
    for (int a = 0; a < 4; ++a)
        for (int b = 0; b < 4; ++b) Lb[(4 + a) * 8 + 4 + b] = W->Hww[16 * bi + a * 4 + b];
    for (int e = 0; e < 8; ++e) Lb[e * 8 + e] += W->zw[8 * bi + e] / (W->w[8 * bi + e] + RELAX) + dw;
    if (chol(Lb, 8) != 0) return 1;
    double *Yb = W->Yb + 32 * bi, *Zb = W->V + 32 * bi, *LT = W->LT + 16 * bi, *Gm = W->Gm + 16 * bi;
    for (int r = 0; r < 4; ++r) {
        double col[8];
        for (int a = 0; a < 8; ++a) col[a] = Jw[r * 8 + a];
        fsub(Lb, 8, col);
        for (int a = 0; a < 8; ++a) Yb[a * 4 + r] = col[a];
    }
    for (int q = 0; q < 4; ++q) {
        double col[8];
        for (int a = 0; a < 8; ++a) col[a] = W->Hxw[32 * bi + q * 8 + a];
        fsub(Lb, 8, col);
        for (int a = 0; a < 8; ++a) Zb[a * 4 + q] = col[a];
    }
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) {
            double t = (r == c) ? 1.0 / D[r] : 0.0, g = -Jx[r * 4 + c];
            for (int a = 0; a < 8; ++a) { t += Yb[a * 4 + r] * Yb[a * 4 + c]; g += Yb[a * 4 + r] * Zb[a * 4 + c]; }
            LT[r * 4 + c] = t;
            Gm[r * 4 + c] = g;
        }
    if (chol(LT, 4) != 0) return 1;
    /* Q += W_xx - Z'Z + G' T^-1 G   (T^-1 G via two triangular solves per column) */
    double TG[16];
    for (int c = 0; c < 4; ++c) {
        double col[4] = {Gm[0 * 4 + c], Gm[1 * 4 + c], Gm[2 * 4 + c], Gm[3 * 4 + c]};
        fsub(LT, 4, col);
        bsub(LT, 4, col);
        for (int r = 0; r < 4; ++r) TG[r * 4 + c] = col[r];
    }
    for (int p = 0; p < 4; ++p)
        for (int q = 0; q < 4; ++q) {
            double t = W->Hxx[16 * bi + p * 4 + q];
            for (int a = 0; a < 8; ++a) t -= Zb[a * 4 + p] * Zb[a * 4 + q];
            for (int r = 0; r < 4; ++r) t += Gm[r * 4 + p] * TG[r * 4 + q];
            Q[p * 6 + q] += t;
        }
    return 0;
}

/* matrices: block eliminations, stage Hessians, Riccati factorisation.  0 = inertia ok */
static int factor(ws_t* W, double dw) {
    const tto_obca_problem* P = W->P;
    const int N = W->N;
    const double dt = P->dt;
    int fail = 0;
    for (int k = 0; k <= N; ++k) {
        double* Q = W->Qt + 36 * k;
        const double sc = (k == N && W->mode == TTO_OBCA_PLAN) ? P->tfac : 1.0;
        for (int i = 0; i < 36; ++i) Q[i] = 2.0 * sc * W->Qc[i] + (k < N ? W->Wd[36 * k + i] : 0.0);
        for (int i = 0; i < 6; ++i) Q[i * 6 + i] += sig_x(W, k, i) + dw;
        for (int j = 0; j < W->nbk; ++j) {
            const int bi = k * W->nbk + j;
            if (block_factor(W, bi, dw, Q) != 0) fail = 1;
        }
        if (k == N && W->mode == TTO_OBCA_PLAN)
            for (int i = 0; i < 6; ++i) {
                double s = dw;
                s += W->vLf[i] / (W->sf[i] - W->fL) + W->vUf[i] / (W->fU - W->sf[i]);
                W->Df[i] = s;
                Q[i * 6 + i] += s;
            }
        if (k < N) {
            double* R = W->Rt + 4 * k;
            for (int i = 0; i < 4; ++i) R[i] = 2.0 * W->Rc[i];
            for (int i = 0; i < 2; ++i) R[i * 2 + i] += sig_u(W, k, i) + dw;
        }
    }
    if (fail) return 1;
    /* Riccati: P_N = Q~_N; G = R~ + B'PB, H = B'PA, K = -G^-1 H, P = Q~ + A'PA + H'K */
    memcpy(W->Pm + 36 * N, W->Qt + 36 * N, 36 * sizeof(double));
    for (int k = N - 1; k >= 0; --k) {
        const double* Pn = W->Pm + 36 * (k + 1);
        const double* A = W->A + 36 * k;
        /* B = dt [e5 e4]: rows of B'X = dt * (X row 5, X row 4) */
        double* G = W->G + 4 * k;
        G[0] = W->Rt[4 * k + 0] + dt * dt * Pn[5 * 6 + 5];
        G[1] = W->Rt[4 * k + 1] + dt * dt * Pn[5 * 6 + 4];
        G[2] = W->Rt[4 * k + 2] + dt * dt * Pn[4 * 6 + 5];
        G[3] = W->Rt[4 * k + 3] + dt * dt * Pn[4 * 6 + 4];
        double* H = W->H + 12 * k;
        for (int j = 0; j < 6; ++j) {
            double h0 = 0.0, h1 = 0.0;
            for (int i = 0; i < 6; ++i) { h0 += Pn[5 * 6 + i] * A[i * 6 + j]; h1 += Pn[4 * 6 + i] * A[i * 6 + j]; }
            H[j] = dt * h0;
            H[6 + j] = dt * h1;
        }
        G[1] = G[2] = 0.5 * (G[1] + G[2]);
        if (chol(G, 2) != 0) return 1;
        double* Kk = W->K + 12 * k;
        for (int j = 0; j < 6; ++j) {
            double col[2] = {H[j], H[6 + j]};
            fsub(G, 2, col);
            bsub(G, 2, col);
            Kk[j] = -col[0];
            Kk[6 + j] = -col[1];
        }
        double* Pk = W->Pm + 36 * k;
        double PA[36];
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                double t = 0.0;
                for (int l = 0; l < 6; ++l) t += Pn[i * 6 + l] * A[l * 6 + j];
                PA[i * 6 + j] = t;
            }
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                double t = W->Qt[36 * k + i * 6 + j];
                for (int l = 0; l < 6; ++l) t += A[l * 6 + i] * PA[l * 6 + j];
                t += H[i] * Kk[j] + H[6 + i] * Kk[6 + j];
                Pk[i * 6 + j] = t;
            }
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < i; ++j) Pk[i * 6 + j] = Pk[j * 6 + i] = 0.5 * (Pk[i * 6 + j] + Pk[j * 6 + i]);
    }
    return 0;
}

/* right-hand side + back-substitution.  cres: dynamics residual ((N+1)*6), dres: OBCA row residual d - s
 * (nb*4), fres: final row residual d_f - s_f (6).  Fills dx du dw ds ycp ydp dsf ydpf. */
static void solve_rhs(ws_t* W, double mu, const double* cres, const double* dres, const double* fres) {
    const tto_obca_problem* P = W->P;
    const int N = W->N;
    const double dt = P->dt;
    for (int k = 0; k <= N; ++k) {
        double* q = W->qt + 6 * k;
        for (int i = 0; i < 6; ++i) q[i] = bgrad_x(W, k, i, mu);
        for (int j = 0; j < W->nbk; ++j) {
            const int bi = k * W->nbk + j;
            const double *D = W->Dd + 4 * bi, *Yb = W->Yb + 32 * bi, *Zb = W->V + 32 * bi, *Gm = W->Gm + 16 * bi;
            double* rd = W->rd + 4 * bi;
            for (int r = 0; r < 4; ++r) rd[r] = dres[4 * bi + r] + bgrad_s(W, r, W->s[4 * bi + r], mu) / D[r];
            double* zf = W->vv + 8 * bi;
            for (int a = 0; a < 8; ++a) zf[a] = -mu / (W->w[8 * bi + a] + RELAX);
            fsub(W->L + 64 * bi, 8, zf);
            double* t = W->tv + 4 * bi;
            for (int r = 0; r < 4; ++r) {
                double h = rd[r];
                for (int a = 0; a < 8; ++a) h -= Yb[a * 4 + r] * zf[a];
                t[r] = h;
            }
            fsub(W->LT + 16 * bi, 4, t);
            bsub(W->LT + 16 * bi, 4, t);
            for (int p = 0; p < 4; ++p) {
                double g = 0.0;
                for (int a = 0; a < 8; ++a) g -= Zb[a * 4 + p] * zf[a];
                for (int r = 0; r < 4; ++r) g -= Gm[r * 4 + p] * t[r];
                q[p] += g;
            }
        }
        if (k == N && W->mode == TTO_OBCA_PLAN)
            for (int i = 0; i < 6; ++i) {
                const double gs = -mu / (W->sf[i] - W->fL) + mu / (W->fU - W->sf[i]);
                W->rf[i] = fres[i] + gs / W->Df[i];
                q[i] += W->Df[i] * W->rf[i];
            }
        if (k < N)
            for (int i = 0; i < 2; ++i) W->rt[2 * k + i] = bgrad_u(W, k, i, mu);
    }
    /* Riccati vector pass */
    memcpy(W->pv + 6 * N, W->qt + 6 * N, 6 * sizeof(double));
    for (int k = N - 1; k >= 0; --k) {
        const double* Pn = W->Pm + 36 * (k + 1);
        const double* pn = W->pv + 6 * (k + 1);
        const double* A = W->A + 36 * k;
        const double* e = cres + 6 * (k + 1);
        double pp[6];
        for (int i = 0; i < 6; ++i) {
            double t = pn[i];
            for (int j = 0; j < 6; ++j) t -= Pn[i * 6 + j] * e[j];
            pp[i] = t;
        }
        double g[2] = {W->rt[2 * k] + dt * pp[5], W->rt[2 * k + 1] + dt * pp[4]};
        fsub(W->G + 4 * k, 2, g);
        bsub(W->G + 4 * k, 2, g);
        W->kf[2 * k] = -g[0];
        W->kf[2 * k + 1] = -g[1];
        const double* H = W->H + 12 * k;
        for (int i = 0; i < 6; ++i) {
            double t = W->qt[6 * k + i];
            for (int l = 0; l < 6; ++l) t += A[l * 6 + i] * pp[l];
            t += H[i] * W->kf[2 * k] + H[6 + i] * W->kf[2 * k + 1];
            W->pv[6 * k + i] = t;
        }
    }
    /* forward sweep */
    for (int i = 0; i < 6; ++i) W->dx[i] = -cres[i];
    for (int k = 0; k <= N; ++k) {
        const double* dxk = W->dx + 6 * k;
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
            double t = -cres[6 * (k + 1) + i];
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
            double g4[4];
            for (int r = 0; r < 4; ++r) {
                double t = 0.0;
                for (int q = 0; q < 4; ++q) t += Gm[r * 4 + q] * dxk[q];
                g4[r] = t;
            }
            fsub(W->LT + 16 * bi, 4, g4);
            bsub(W->LT + 16 * bi, 4, g4);
            double* yp = W->ydp + 4 * bi;
            for (int r = 0; r < 4; ++r) yp[r] = W->tv[4 * bi + r] - g4[r];
            double t8[8];
            for (int a = 0; a < 8; ++a) {
                double t = W->vv[8 * bi + a];
                for (int q = 0; q < 4; ++q) t += Zb[a * 4 + q] * dxk[q];
                for (int r = 0; r < 4; ++r) t += Yb[a * 4 + r] * yp[r];
                t8[a] = t;
            }
            bsub(W->L + 64 * bi, 8, t8);
            for (int a = 0; a < 8; ++a) W->dw[8 * bi + a] = -t8[a];
            for (int r = 0; r < 4; ++r) W->ds[4 * bi + r] = (yp[r] - bgrad_s(W, r, W->s[4 * bi + r], mu)) / D[r];
        }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            const double gs = -mu / (W->sf[i] - W->fL) + mu / (W->fU - W->sf[i]);
            W->ydpf[i] = W->Df[i] * (W->dx[6 * N + i] + W->rf[i]);
            W->dsf[i] = (W->ydpf[i] - gs) / W->Df[i];
        }
}

/* TTO_CHECK diagnostic: residual of the un-condensed first Newton row block (primal stationarity) */
static double check_newton(ws_t* W, double mu, double dwreg) {
    const tto_obca_problem* P = W->P;
    const int N = W->N;
    double worst = 0.0, wx = 0.0, ww = 0.0, wr = 0.0, wu = 0.0;
    for (int k = 0; k <= N; ++k) {
        double r[6], rs[6];
        for (int i = 0; i < 6; ++i) {
            double t = bgrad_x(W, k, i, mu) + W->ycp[6 * k + i];
            double sc = fabs(bgrad_x(W, k, i, mu)) + fabs(W->ycp[6 * k + i]);
            const double tf = (k == N && W->mode == TTO_OBCA_PLAN) ? P->tfac : 1.0;
            for (int j = 0; j < 6; ++j) {
                const double e = (2.0 * tf * W->Qc[i * 6 + j] + (k < N ? W->Wd[36 * k + i * 6 + j] : 0.0)) * W->dx[6 * k + j];
                t += e; sc += fabs(e);
            }
            t += (sig_x(W, k, i) + dwreg) * W->dx[6 * k + i];
            sc += fabs((sig_x(W, k, i) + dwreg) * W->dx[6 * k + i]);
            if (k < N)
                for (int l = 0; l < 6; ++l) { t -= W->A[36 * k + l * 6 + i] * W->ycp[6 * (k + 1) + l]; sc += fabs(W->A[36 * k + l * 6 + i] * W->ycp[6 * (k + 1) + l]); }
            if (k == N && W->mode == TTO_OBCA_PLAN) { t += W->ydpf[i]; sc += fabs(W->ydpf[i]); }
            r[i] = t; rs[i] = sc;
        }
        for (int j = 0; j < W->nbk; ++j) {
            const int bi = k * W->nbk + j;
            for (int q = 0; q < 4; ++q) {
                double t = 0.0;
                double sc = 0.0;
                for (int p = 0; p < 4; ++p) { double e = W->Hxx[16 * bi + q * 4 + p] * W->dx[6 * k + p]; t += e; sc += fabs(e); }
                for (int a = 0; a < 8; ++a) { double e = W->Hxw[32 * bi + q * 8 + a] * W->dw[8 * bi + a]; t += e; sc += fabs(e); }
                for (int rr = 0; rr < 4; ++rr) { double e = W->Jx[16 * bi + rr * 4 + q] * W->ydp[4 * bi + rr]; t += e; sc += fabs(e); }
                r[q] += t; rs[q] += sc;
            }
            /* w rows */
            for (int a = 0; a < 8; ++a) {
                double t1 = -mu / (W->w[8 * bi + a] + RELAX), t2 = (W->zw[8 * bi + a] / (W->w[8 * bi + a] + RELAX) + dwreg) * W->dw[8 * bi + a];
                double t = t1 + t2, sc = fabs(t1) + fabs(t2);
                for (int q = 0; q < 4; ++q) { double e = W->Hxw[32 * bi + q * 8 + a] * W->dx[6 * k + q]; t += e; sc += fabs(e); }
                if (a >= 4)
                    for (int b = 0; b < 4; ++b) { double e = W->Hww[16 * bi + (a - 4) * 4 + b] * W->dw[8 * bi + 4 + b]; t += e; sc += fabs(e); }
                for (int rr = 0; rr < 4; ++rr) { double e = W->Jw[32 * bi + rr * 8 + a] * W->ydp[4 * bi + rr]; t += e; sc += fabs(e); }
                ww = fmax(ww, fabs(t) / (sc + 1e-300));
            }
            /* linearised OBCA rows: J dx - ds + (d - s) */
            for (int rr = 0; rr < 4; ++rr) {
                double t = W->d[4 * bi + rr] - W->s[4 * bi + rr] - W->ds[4 * bi + rr];
                double sc = fabs(W->d[4 * bi + rr]) + fabs(W->s[4 * bi + rr]) + fabs(W->ds[4 * bi + rr]);
                for (int q = 0; q < 4; ++q) { double e = W->Jx[16 * bi + rr * 4 + q] * W->dx[6 * k + q]; t += e; sc += fabs(e); }
                for (int a = 0; a < 8; ++a) { double e = W->Jw[32 * bi + rr * 8 + a] * W->dw[8 * bi + a]; t += e; sc += fabs(e); }
                wr = fmax(wr, fabs(t) / (sc + 1e-300));
            }
        }
        for (int i = 0; i < 6; ++i) wx = fmax(wx, fabs(r[i]) / (rs[i] + 1e-300));
        if (k < N)
            for (int i = 0; i < 2; ++i) {
                double t = bgrad_u(W, k, i, mu) + (sig_u(W, k, i) + dwreg) * W->du[2 * k + i];
                double sc = fabs(bgrad_u(W, k, i, mu)) + fabs((sig_u(W, k, i) + dwreg) * W->du[2 * k + i]);
                for (int j = 0; j < 2; ++j) { t += 2.0 * W->Rc[i * 2 + j] * W->du[2 * k + j]; sc += fabs(2.0 * W->Rc[i * 2 + j] * W->du[2 * k + j]); }
                t -= P->dt * W->ycp[6 * (k + 1) + (i == 0 ? 5 : 4)];
                sc += fabs(P->dt * W->ycp[6 * (k + 1) + (i == 0 ? 5 : 4)]);
                wu = fmax(wu, fabs(t) / (sc + 1e-300));
            }
    }
    fprintf(stderr, "   check: x %.2e w %.2e rows %.2e u %.2e\n", wx, ww, wr, wu);
    worst = fmax(fmax(wx, ww), fmax(wr, wu));
    return worst;
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

/* Dual warm start: for body/obstacle pair j at pose x_k, pick the unit direction n among the 8 face
 * normals (obstacle +-e_x, +-e_y; body +-R e_x, +-R e_y) maximising the separation
 * gap(n) = n'p - h_B(-R'n) - h_O(n), and set lam = 0.99 (n+_x, n+_y, n-_x, n-_y) (so A'lam = 0.99 n),
 * mu = 0.99 (m+_x, m+_y, m-_x, m-_y) with m = -R'n (so G'mu + R'A'lam = 0).  Then d2 = d3 = 0,
 * d4 = -0.01 and d1 = d_min - 0.99 gap(n): the OBCA rows are satisfied wherever the guess pose is
 * separated by more than d_min (the dual certificate of the reference's own constraint rows). */
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
}

#define FTB_P(val, lo, step, tau, a) do { if ((step) < 0) a = fmin(a, -(tau) * ((val) - (lo)) / (step)); } while (0)
#define FTB_PU(val, hi, step, tau, a) do { if ((step) > 0) a = fmin(a, (tau) * ((hi) - (val)) / (step)); } while (0)
#define FTB_D(zv, step, tau, a) do { if ((step) < 0) a = fmin(a, -(tau) * (zv) / (step)); } while (0)

static double ftb_primal(const ws_t* W, const double* dx, const double* du, const double* dw, const double* ds,
                         const double* dsf, double tau) {
    double a = 1.0;
    for (int k = 0; k <= W->N; ++k) {
        for (int i = 0; i < 6; ++i) {
            const int v = 6 * k + i;
            if (W->hxl[i]) FTB_P(W->x[v], W->xl[i], dx[v], tau, a);
            if (W->hxu[i]) FTB_PU(W->x[v], W->xu[i], dx[v], tau, a);
        }
        if (k < W->N)
            for (int i = 0; i < 2; ++i) {
                const int v = 2 * k + i;
                if (W->hul[i]) FTB_P(W->u[v], W->ul[i], du[v], tau, a);
                if (W->huu[i]) FTB_PU(W->u[v], W->uu[i], du[v], tau, a);
            }
    }
    for (int bi = 0; bi < W->nb; ++bi) {
        for (int e = 0; e < 8; ++e) FTB_P(W->w[8 * bi + e], -RELAX, dw[8 * bi + e], tau, a);
        for (int r = 0; r < 4; ++r) {
            const int v = 4 * bi + r;
            if (W->hrL[r]) FTB_P(W->s[v], W->rL[r], ds[v], tau, a);
            if (W->hrU[r]) FTB_PU(W->s[v], W->rU[r], ds[v], tau, a);
        }
    }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            FTB_P(W->sf[i], W->fL, dsf[i], tau, a);
            FTB_PU(W->sf[i], W->fU, dsf[i], tau, a);
        }
    return a;
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
    return a;
}

/* scaled optimality error at the current iterate (IPOPT eq. (5)); cmu = complementarity vs mu */
static void opt_error(ws_t* W, double mu, double* E0, double* Emu, double* dinf_o, double* pinf_o, int* finite) {
    const tto_obca_problem* P = W->P;
    const int N = W->N;
    double dinf = 0.0, pinf = 0.0, c0 = 0.0, cmu = 0.0, sy = 0.0, sz = 0.0;
    long nb_ = 0, my = 0;
    *finite = 1;
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
                double t = -W->zw[8 * bi + a];
                for (int r = 0; r < 4; ++r) t += W->Jw[32 * bi + r * 8 + a] * W->yd[4 * bi + r];
                dinf = fmax(dinf, fabs(t));
                if (!isfinite(t)) *finite = 0;
                const double sl = W->w[8 * bi + a] + RELAX, zz = W->zw[8 * bi + a];
                c0 = fmax(c0, fabs(zz * sl)); cmu = fmax(cmu, fabs(zz * sl - mu)); sz += zz; ++nb_;
            }
            for (int r = 0; r < 4; ++r) {
                const int v = 4 * bi + r;
                const double t = -W->yd[v] - W->vL[v] + W->vU[v];
                dinf = fmax(dinf, fabs(t));
                pinf = fmax(pinf, fabs(W->d[v] - W->s[v]));
                sy += fabs(W->yd[v]); ++my;
                if (W->hrL[r]) { const double sl = W->s[v] - W->rL[r]; c0 = fmax(c0, fabs(W->vL[v] * sl)); cmu = fmax(cmu, fabs(W->vL[v] * sl - mu)); sz += W->vL[v]; ++nb_; }
                if (W->hrU[r]) { const double sl = W->rU[r] - W->s[v]; c0 = fmax(c0, fabs(W->vU[v] * sl)); cmu = fmax(cmu, fabs(W->vU[v] * sl - mu)); sz += W->vU[v]; ++nb_; }
            }
        }
        for (int i = 0; i < 6; ++i) {
            const int v = 6 * k + i;
            gl[i] += -W->zLx[v] + W->zUx[v];
            dinf = fmax(dinf, fabs(gl[i]));
            if (!isfinite(gl[i])) *finite = 0;
            if (W->hxl[i]) { const double sl = W->x[v] - W->xl[i]; c0 = fmax(c0, fabs(W->zLx[v] * sl)); cmu = fmax(cmu, fabs(W->zLx[v] * sl - mu)); sz += W->zLx[v]; ++nb_; }
            if (W->hxu[i]) { const double sl = W->xu[i] - W->x[v]; c0 = fmax(c0, fabs(W->zUx[v] * sl)); cmu = fmax(cmu, fabs(W->zUx[v] * sl - mu)); sz += W->zUx[v]; ++nb_; }
            pinf = fmax(pinf, fabs(W->c[v]));
            sy += fabs(W->yc[v]); ++my;
        }
        if (k < N)
            for (int i = 0; i < 2; ++i) {
                const int v = 2 * k + i;
                double t = W->gu[v] - P->dt * W->yc[6 * (k + 1) + (i == 0 ? 5 : 4)] - W->zLu[v] + W->zUu[v];
                dinf = fmax(dinf, fabs(t));
                if (!isfinite(t)) *finite = 0;
                if (W->hul[i]) { const double sl = W->u[v] - W->ul[i]; c0 = fmax(c0, fabs(W->zLu[v] * sl)); cmu = fmax(cmu, fabs(W->zLu[v] * sl - mu)); sz += W->zLu[v]; ++nb_; }
                if (W->huu[i]) { const double sl = W->uu[i] - W->u[v]; c0 = fmax(c0, fabs(W->zUu[v] * sl)); cmu = fmax(cmu, fabs(W->zUu[v] * sl - mu)); sz += W->zUu[v]; ++nb_; }
            }
    }
    if (W->mode == TTO_OBCA_PLAN)
        for (int i = 0; i < 6; ++i) {
            const double t = -W->ydf[i] - W->vLf[i] + W->vUf[i];
            dinf = fmax(dinf, fabs(t));
            pinf = fmax(pinf, fabs(W->df[i] - W->sf[i]));
            sy += fabs(W->ydf[i]); ++my;
            const double sl = W->sf[i] - W->fL, su = W->fU - W->sf[i];
            c0 = fmax(c0, fmax(fabs(W->vLf[i] * sl), fabs(W->vUf[i] * su)));
            cmu = fmax(cmu, fmax(fabs(W->vLf[i] * sl - mu), fabs(W->vUf[i] * su - mu)));
            sz += W->vLf[i] + W->vUf[i];
            nb_ += 2;
        }
    if (!isfinite(pinf)) *finite = 0;
    const double smax = 100.0;
    const double sd = fmax(smax, (sy + sz) / (double)(my + nb_)) / smax;
    const double sc = nb_ ? fmax(smax, sz / (double)nb_) / smax : 1.0;
    *E0 = fmax(fmax(dinf / sd, pinf), c0 / sc);
    *Emu = fmax(fmax(dinf / sd, pinf), cmu / sc);
    if (dinf_o) *dinf_o = dinf;
    if (pinf_o) *pinf_o = pinf;
}

/* theta (l1 infeasibility) and barrier objective phi at the trial point (xt, ut, wt, st, sft) */
static void trial_eval(ws_t* W, double mu, double* th, double* ph) {
    int bad = 0;
    const double b = barrier(W, W->xt, W->ut, W->wt, W->st, W->sft, mu, &bad);
    if (bad) { *th = INFINITY; *ph = INFINITY; return; }
    dyn_cons(W, W->xt, W->ut, W->ct);
    obca_cons(W, W->xt, W->wt, W->dtr, W->dft);
    *th = infeas1(W, W->ct, W->dtr, W->st, W->dft, W->sft);
    *ph = cost_eval(W, W->xt, W->ut) + b;
}

static int in_filter(const ws_t* W, double th, double ph) {
    for (int i = 0; i < W->nf; ++i)
        if (th >= W->fth[i] && ph >= W->fph[i]) return 1;
    return 0;
}

/* add a filter entry; entries it dominates are dropped; when full the oldest is evicted */
static void add_filter(ws_t* W, double th, double ph) {
    int j = 0;
    for (int i = 0; i < W->nf; ++i)
        if (!(W->fth[i] >= th && W->fph[i] >= ph)) { W->fth[j] = W->fth[i]; W->fph[j] = W->fph[i]; ++j; }
    W->nf = j;
    if (W->nf == TTO_MAXF) {
        memmove(W->fth, W->fth + 1, (TTO_MAXF - 1) * sizeof(double));
        memmove(W->fph, W->fph + 1, (TTO_MAXF - 1) * sizeof(double));
        --W->nf;
    }
    W->fth[W->nf] = th;
    W->fph[W->nf] = ph;
    ++W->nf;
}

static void clamp_mult(double* z, double sl, double mu) {
    const double ks = 1e10;
    *z = fmax(fmin(*z, ks * mu / sl), mu / (ks * sl));
}

static int solve_one(ws_t* W, const double* xinit, const double* xgoal, const double* xref, const double* uref,
                     const double* zg, double* zout, int* iters_out, double* kkt_out) {
    const tto_obca_problem* P = W->P;
    const int N = W->N;
    W->xinit = xinit; W->xgoal = xgoal; W->xref = xref; W->uref = uref;
    const int dbg = getenv("TTO_DEBUG") != NULL, chk = getenv("TTO_CHECK") != NULL;
    /* weights, bounds (bound_relax_factor 1e-8 on every finite bound) */
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
        if (iters_out) *iters_out = 0;
        if (kkt_out) *kkt_out = INFINITY;
        return 3;
    }
    /* bound push of the primal guess, slacks = d(x0) pushed, multipliers 1 / 0 */
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
    double mu = 0.1, tau = fmax(0.99, 1.0 - mu), dw_last = 0.0, th_max = 0.0, th_min = 0.0;
    int acc_count = 0, n_fallback = 0;
    W->nf = 0;
    const double kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5;

    for (iter = 0;; ++iter) {
        linearise(W);
        double Emu, dinf, pinf;
        int finite;
        opt_error(W, mu, &E0, &Emu, &dinf, &pinf, &finite);
        if (!finite) { status = 4; break; }
        if (dbg) fprintf(stderr, "it %4d E0 %.3e dinf %.3e pinf %.3e mu %.2e f %.6e\n", iter, E0, dinf, pinf, mu,
                         cost_eval(W, W->x, W->u));
        if (E0 <= P->tol) { status = 0; break; }
        if (E0 <= P->acc_tol) {
            if (++acc_count >= P->acc_iter) { status = 1; break; }
        } else {
            acc_count = 0;
        }
        if (iter >= P->max_iter) { status = E0 <= P->acc_tol ? 1 : 2; break; }
        while (Emu <= kappa_eps * mu && mu > P->tol / 10.0 * 1.0000001) {
            mu = fmax(P->tol / 10.0, fmin(kappa_mu * mu, pow(mu, theta_mu)));
            tau = fmax(0.99, 1.0 - mu);
            W->nf = 0; /* IPOPT resets the filter on every barrier update */
            opt_error(W, mu, &E0, &Emu, &dinf, &pinf, &finite);
        }
        /* Newton step with inertia correction */
        double dw = 0.0;
        int ok = 0;
        for (int attempt = 0; attempt < 40; ++attempt) {
            if (factor(W, dw) == 0) { ok = 1; break; }
            dw = (dw == 0.0) ? (dw_last == 0.0 ? 1e-4 : fmax(1e-20, dw_last / 3.0)) : (dw_last == 0.0 ? 100.0 * dw : 8.0 * dw);
            if (dw > 1e20) break; /* IPOPT max_hessian_perturbation 1e20 */
        }
        if (!ok) { status = 5; break; } /* IPOPT Error_In_Step_Computation */
        if (dw > 0) dw_last = dw;
        for (int i = 0; i < 4 * W->nb; ++i) W->dr[i] = W->d[i] - W->s[i];
        double fr[6] = {0};
        if (W->mode == TTO_OBCA_PLAN)
            for (int i = 0; i < 6; ++i) fr[i] = W->df[i] - W->sf[i];
        solve_rhs(W, mu, W->c, W->dr, fr);
        if (chk) fprintf(stderr, "   newton residual %.3e (dw %.2e)\n", check_newton(W, mu, dw), dw);
        mult_steps(W, mu);
        double ap = ftb_primal(W, W->dx, W->du, W->dw, W->ds, W->dsf, tau);
        if (getenv("TTO_FTBDBG")) {
            double aw = 1, as_[4] = {1, 1, 1, 1}, ax = 1, au = 1, af = 1; int kw = -1, kx = -1, ix = -1;
            for (int bi = 0; bi < W->nb; ++bi) {
                for (int e = 0; e < 8; ++e) { double t = aw; FTB_P(W->w[8 * bi + e], -RELAX, W->dw[8 * bi + e], tau, aw); if (aw < t) kw = bi / W->nbk; }
                for (int r = 0; r < 4; ++r) { const int v = 4 * bi + r; if (W->hrL[r]) FTB_P(W->s[v], W->rL[r], W->ds[v], tau, as_[r]); if (W->hrU[r]) FTB_PU(W->s[v], W->rU[r], W->ds[v], tau, as_[r]); }
            }
            for (int k = 0; k <= N; ++k) for (int i = 0; i < 6; ++i) { double t = ax; if (W->hxl[i]) FTB_P(W->x[6 * k + i], W->xl[i], W->dx[6 * k + i], tau, ax); if (W->hxu[i]) FTB_PU(W->x[6 * k + i], W->xu[i], W->dx[6 * k + i], tau, ax); if (ax < t) { kx = k; ix = i; } }
            for (int k = 0; k < N; ++k) for (int i = 0; i < 2; ++i) { if (W->hul[i]) FTB_P(W->u[2 * k + i], W->ul[i], W->du[2 * k + i], tau, au); if (W->huu[i]) FTB_PU(W->u[2 * k + i], W->uu[i], W->du[2 * k + i], tau, au); }
            if (W->mode == TTO_OBCA_PLAN) for (int i = 0; i < 6; ++i) { FTB_P(W->sf[i], W->fL, W->dsf[i], tau, af); FTB_PU(W->sf[i], W->fU, W->dsf[i], tau, af); }
            fprintf(stderr, "     ftb w %.1e(k%d) s %.1e %.1e %.1e %.1e x %.1e(k%d,i%d) u %.1e f %.1e\n", aw, kw, as_[0], as_[1], as_[2], as_[3], ax, kx, ix, au, af);
        }
        double az = ftb_dual(W, tau);
        /* filter line search (Waechter & Biegler 2006, IPOPT defaults) */
        double ymax = 0.0;
        for (int i = 0; i < 6 * (N + 1); ++i) ymax = fmax(ymax, fabs(W->ycp[i]));
        for (int i = 0; i < 4 * W->nb; ++i) ymax = fmax(ymax, fabs(W->ydp[i]));
        if (W->mode == TTO_OBCA_PLAN)
            for (int i = 0; i < 6; ++i) ymax = fmax(ymax, fabs(W->ydpf[i]));
        int bad = 0;
        const double th0 = infeas1(W, W->c, W->d, W->s, W->df, W->sf);
        const double phi0 = cost_eval(W, W->x, W->u) + barrier(W, W->x, W->u, W->w, W->s, W->sf, mu, &bad);
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
                Dm += -mu / (W->w[8 * bi + e] + RELAX) * W->dw[8 * bi + e];
                rel = fmax(rel, fabs(W->dw[8 * bi + e]) / (1.0 + fabs(W->w[8 * bi + e])));
            }
            for (int r = 0; r < 4; ++r) {
                Dm += bgrad_s(W, r, W->s[4 * bi + r], mu) * W->ds[4 * bi + r];
                rel = fmax(rel, fabs(W->ds[4 * bi + r]) / (1.0 + fabs(W->s[4 * bi + r])));
            }
        }
        if (W->mode == TTO_OBCA_PLAN)
            for (int i = 0; i < 6; ++i) {
                Dm += (-mu / (W->sf[i] - W->fL) + mu / (W->fU - W->sf[i])) * W->dsf[i];
                rel = fmax(rel, fabs(W->dsf[i]) / (1.0 + fabs(W->sf[i])));
            }
        if (iter == 0 || !(th_max > 0)) { th_max = 1e4 * fmax(1.0, th0); th_min = 1e-4 * fmax(1.0, th0); }
        const double g_th = 1e-5, g_ph = 1e-8, s_ph = 2.3, s_th = 1.1, delta = 1.0, eta_ph = 1e-8, g_al = 0.05;
        double amin;
        if (Dm < 0.0) {
            amin = fmin(g_th, g_ph * th0 / (-Dm));
            if (th0 <= th_min) amin = fmin(amin, delta * pow(th0, s_th) / pow(-Dm, s_ph));
        } else {
            amin = g_th;
        }
        amin *= g_al;
        const double tolc = 10.0 * DBL_EPSILON;
        double alpha = ap;
        int accepted = rel < 1e-15, ftype = 0;
        const size_t nx_ = 6 * (size_t)(N + 1), nu_ = 2 * (size_t)N, nw_ = 8 * (size_t)W->nb, ns_ = 4 * (size_t)W->nb;
#define TRIAL(a_) do { \
            for (size_t i = 0; i < nx_; ++i) W->xt[i] = W->x[i] + (a_) * W->dx[i]; \
            for (size_t i = 0; i < nu_; ++i) W->ut[i] = W->u[i] + (a_) * W->du[i]; \
            for (size_t i = 0; i < nw_; ++i) W->wt[i] = W->w[i] + (a_) * W->dw[i]; \
            for (size_t i = 0; i < ns_; ++i) W->st[i] = W->s[i] + (a_) * W->ds[i]; \
            for (int i = 0; i < 6; ++i) W->sft[i] = W->sf[i] + (a_) * W->dsf[i]; \
            trial_eval(W, mu, &tht, &pht); } while (0)
        double tht = 0.0, pht = 0.0;
        for (int ls = 0; !accepted; ++ls) {
            TRIAL(alpha);
            const int sw = Dm < 0.0 && alpha * pow(-Dm, s_ph) > delta * pow(th0, s_th);
            int ok = 0;
            if (isfinite(pht) && tht <= th_max && !in_filter(W, tht, pht)) {
                if (th0 <= th_min && sw) { ftype = 1; ok = pht - (phi0 + eta_ph * alpha * Dm) <= tolc * fabs(phi0); }
                else { ftype = 0; ok = tht <= (1.0 - g_th) * th0 || pht - (phi0 - g_ph * th0) <= tolc * fabs(phi0); }
            }
            if (ok) { accepted = 1; break; }
            if (ls == 0 && isfinite(pht) && tht >= th0) {
                /* second-order corrections (IPOPT max_soc 4, kappa_soc 0.99) */
                double* sv = (double*)malloc((nx_ + nu_ + nw_ + ns_ + nx_ + ns_ + 12) * sizeof(double));
                if (!sv) break;
                double* o = sv;
                memcpy(o, W->dx, nx_ * 8); o += nx_; memcpy(o, W->du, nu_ * 8); o += nu_;
                memcpy(o, W->dw, nw_ * 8); o += nw_; memcpy(o, W->ds, ns_ * 8); o += ns_;
                memcpy(o, W->ycp, nx_ * 8); o += nx_; memcpy(o, W->ydp, ns_ * 8); o += ns_;
                memcpy(o, W->dsf, 48); o += 6; memcpy(o, W->ydpf, 48);
                /* c_soc(0) = alpha r(x) + r(x + alpha d), c_soc(p+1) = a_soc(p) c_soc(p) + r(x + a_soc(p) d_soc(p)) */
                double frs[6] = {0}, a_soc = alpha, th_old = th0;
                for (size_t i = 0; i < nx_; ++i) W->cr[i] = W->c[i];
                for (size_t i = 0; i < ns_; ++i) W->dr[i] = W->d[i] - W->s[i];
                if (W->mode == TTO_OBCA_PLAN) for (int i = 0; i < 6; ++i) frs[i] = W->df[i] - W->sf[i];
                int soc_ok = 0;
                for (int p = 0; p < 4; ++p) {
                    if (p > 0 && tht > 0.99 * th_old) break;
                    th_old = tht;
                    for (size_t i = 0; i < nx_; ++i) W->cr[i] = a_soc * W->cr[i] + W->ct[i];
                    for (size_t i = 0; i < ns_; ++i) W->dr[i] = a_soc * W->dr[i] + (W->dtr[i] - W->st[i]);
                    if (W->mode == TTO_OBCA_PLAN) for (int i = 0; i < 6; ++i) frs[i] = a_soc * frs[i] + (W->dft[i] - W->sft[i]);
                    solve_rhs(W, mu, W->cr, W->dr, frs);
                    a_soc = ftb_primal(W, W->dx, W->du, W->dw, W->ds, W->dsf, tau);
                    TRIAL(a_soc);
                    int ok2 = 0;
                    if (isfinite(pht) && tht <= th_max && !in_filter(W, tht, pht)) {
                        if (th0 <= th_min && sw) { ftype = 1; ok2 = pht - (phi0 + eta_ph * alpha * Dm) <= tolc * fabs(phi0); }
                        else { ftype = 0; ok2 = tht <= (1.0 - g_th) * th0 || pht - (phi0 - g_ph * th0) <= tolc * fabs(phi0); }
                    }
                    if (ok2) { soc_ok = 1; break; }
                    if (!isfinite(pht)) break;
                }
                if (soc_ok) {
                    accepted = 2;
                    alpha = a_soc;
                    mult_steps(W, mu);
                    az = ftb_dual(W, tau);
                    free(sv);
                    break;
                }
                o = sv;
                memcpy(W->dx, o, nx_ * 8); o += nx_; memcpy(W->du, o, nu_ * 8); o += nu_;
                memcpy(W->dw, o, nw_ * 8); o += nw_; memcpy(W->ds, o, ns_ * 8); o += ns_;
                memcpy(W->ycp, o, nx_ * 8); o += nx_; memcpy(W->ydp, o, ns_ * 8); o += ns_;
                memcpy(W->dsf, o, 48); o += 6; memcpy(W->ydpf, o, 48);
                free(sv);
            }
            if (alpha * 0.5 < amin) break;
            alpha *= 0.5;
        }
        if (!accepted) { /* IPOPT would enter restoration here; we take a fallback step and reset the filter */
            W->nf = 0;
            ++n_fallback;
        } else if (!ftype) {
            add_filter(W, (1.0 - g_th) * th0, phi0 - g_ph * th0);
        }
#undef TRIAL
        if (dbg) fprintf(stderr, "     ap %.3e az %.3e alpha %.3e acc %d f %d dw %.2e D %.3e th %.3e nf %d fb %d\n", ap, az, alpha, accepted, ftype, dw, Dm, th0, W->nf, n_fallback);
        /* update */
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
    }
    pack(W, zout);
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
    const int st = solve_one(&W, x_init, x_goal, xref, uref, z_guess, z_out, iters, kkt);
    free(W.mem);
    return st;
}

int tto_obca_solve_batch(const tto_obca_problem* P, int B, const double* x_init, const double* x_goal,
                         const double* xref, const double* uref, const double* z_guess, double* z_out,
                         int* status, int* iters, double* kkt, int nthreads) {
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
                                  z_guess ? z_guess + (size_t)b * n : NULL, z_out + (size_t)b * n, &it, &e);
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
