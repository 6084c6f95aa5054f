/* CPU ORACLE -- see tt_oracle.h.  Test infrastructure + cpu_baseline only.
 *
 * NLP (restated from the reference, citations python-files/<file>:<line>):
 *   min  sum_{k<N} (x_k-xr_k)' Qw (x_k-xr_k) + (u_k-ur_k)' Rw (u_k-ur_k) + (x_N-xr_N)' Qw (x_N-xr_N)
 *                                                  mpc_control.py:17-25 (fuzzy Qw = DQD: 23-24)
 *   s.t. x_0 - x_init = 0,  x_{k+1} - (x_k + dt f(x_k,u_k)) = 0     trajectory_planning.py:28-36
 *        lbx <= z <= ubx on every x_k (k=0..N) and u_k              trajectory_planning.py:38-60
 *   f: truck_trailer_model.py:8-24, Euler: truck_trailer_model.py:26-29.
 *
 * Algorithm (restatement of IPOPT's primal-dual barrier method as configured by
 * mpc_control.py:35-39 -- tol 1e-8, acceptable 1e-6 x15, monotone mu, tau = max(.99, 1-mu),
 * bound_relax_factor 1e-8, bound_push/frac 1e-2, kappa_eps 10, kappa_mu .2, theta_mu 1.5,
 * kappa_sigma 1e10, exact Lagrangian Hessian).  Globalisation: IPOPT's filter line search with one
 * second-order correction.  Termination: IPOPT's OptimalityErrorConvergenceCheck -- the scaled error E_0 <= tol
 * AND the unscaled dual infeasibility <= dual_inf_tol (1), constraint violation <= constr_viol_tol (1e-4) and
 * complementarity <= compl_inf_tol (1e-4); "acceptable" with acceptable_tol and 1e10 / 1e-2 / 1e-2.  Barrier floor
 * of MonotoneMuUpdate::CalcNewMuAndTau: min(tol, compl_inf_tol) / (barrier_tol_factor + 1).
 * Linear algebra: full (n+m) KKT in banded storage (half-bandwidth 13 for the stage-interleaved
 * ordering [y_k, x_k, u_k]), LU with partial pivoting (LAPACK dgbtf2/dgbtrs restated), inertia-free
 * curvature test for the Hessian regularisation.
 */
#include "tt_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#define TTO_MAX_FILTER 16 /* = kTrackFilter of the GPU kernel */
/* IPOPT defaults of the convergence check (OptimalityErrorConvergenceCheck) and of the barrier floor */
#define DUAL_INF_TOL 1.0
#define CONSTR_VIOL_TOL 1e-4
#define COMPL_INF_TOL 1e-4
#define ACC_DUAL_INF_TOL 1e10
#define ACC_CONSTR_VIOL_TOL 1e-2
#define ACC_COMPL_INF_TOL 1e-2
#define BARRIER_TOL_FACTOR 10.0
#ifdef _OPENMP
#include <omp.h>
#endif

#define NX 6
#define NU 2
#define NS 8
#define KL 13
#define KU 13
#define KV (KL + KU)
#define LDAB (2 * KL + KU + 1)

typedef struct {
    int N, n, m, nk;
    double *z, *zL, *zU, *y, *lb, *ub;
    char *hasL, *hasU;
    double *gF, *c, *A, *Wc;
    double *ab, *rhs, *rhs2;
    int* ipiv;
    double *dz, *yp, *dzL, *dzU, *zt, *ct, *dzs;
    double Qw[36], Rw[4];
} ws_t;

/* ---------------- model: truck_trailer_model.py:8-24 ---------------- */
static void fdyn(const tto_problem* P, const double* x, const double* u, double* fo) {
    const double th = x[2], psi = x[3], phi = x[4], v = x[5];
    const double t = tan(phi);
    fo[0] = v * cos(th);
    fo[1] = v * sin(th);
    fo[2] = v * t / P->L1;
    fo[3] = -v * t / P->L1 * (1.0 + P->Mh / P->L2 * cos(psi)) - v * sin(psi) / P->L2;
    fo[4] = u[1];
    fo[5] = u[0];
}

/* A = I + dt * df/dx (row-major 6x6) */
static void jac_A(const tto_problem* P, const double* x, double* A) {
    const double th = x[2], psi = x[3], phi = x[4], v = x[5];
    const double L1 = P->L1, L2 = P->L2, M = P->Mh, dt = P->dt;
    const double t = tan(phi), cphi = cos(phi), c2 = 1.0 / (cphi * cphi);
    const double k = 1.0 + M / L2 * cos(psi);
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

/* H += s * sum_i w_i d2 f_i / dx2 */
static void hess_acc(const tto_problem* P, const double* x, const double* w, double s, double* H) {
    const double th = x[2], psi = x[3], phi = x[4], v = x[5];
    const double L1 = P->L1, L2 = P->L2, M = P->Mh;
    const double sn = sin(th), cs = cos(th), t = tan(phi), cphi = cos(phi), c2 = 1.0 / (cphi * cphi);
    const double sp = sin(psi), cp = cos(psi), k = 1.0 + M / L2 * cp;
    double h22 = w[0] * (-v * cs) + w[1] * (-v * sn);
    double h25 = w[0] * (-sn) + w[1] * cs;
    double h44 = w[2] * (2 * v * t * c2 / L1) + w[3] * (-2 * v * t * c2 * k / L1);
    double h45 = w[2] * (c2 / L1) + w[3] * (-c2 * k / L1);
    double h33 = w[3] * (v * t * M * cp / (L1 * L2) + v * sp / L2);
    double h34 = w[3] * (v * c2 * M * sp / (L1 * L2));
    double h35 = w[3] * (t * M * sp / (L1 * L2) - cp / L2);
    H[2 * 6 + 2] += s * h22;
    H[2 * 6 + 5] += s * h25; H[5 * 6 + 2] += s * h25;
    H[4 * 6 + 4] += s * h44;
    H[4 * 6 + 5] += s * h45; H[5 * 6 + 4] += s * h45;
    H[3 * 6 + 3] += s * h33;
    H[3 * 6 + 4] += s * h34; H[4 * 6 + 3] += s * h34;
    H[3 * 6 + 5] += s * h35; H[5 * 6 + 3] += s * h35;
}

/* ---------------- banded LU (LAPACK dgbtf2 / dgbtrs restated) ---------------- */
#define ABI(i, j) ((size_t)(j) * LDAB + (KV + (i) - (j)))

static int gbtf2(int n, double* ab, int* ipiv) {
    int ju = 0, info = 0;
    for (int j = 0; j < n; ++j) {
        int km = KL < n - 1 - j ? KL : n - 1 - j;
        int jp = 0;
        double amax = fabs(ab[ABI(j, j)]);
        for (int i = 1; i <= km; ++i) {
            double a = fabs(ab[ABI(j + i, j)]);
            if (a > amax) { amax = a; jp = i; }
        }
        ipiv[j] = j + jp;
        if (ab[ABI(j + jp, j)] != 0.0) {
            int lim = j + KU + jp;
            if (lim > n - 1) lim = n - 1;
            if (lim > ju) ju = lim;
            if (jp != 0)
                for (int c = j; c <= ju; ++c) {
                    double t = ab[ABI(j + jp, c)];
                    ab[ABI(j + jp, c)] = ab[ABI(j, c)];
                    ab[ABI(j, c)] = t;
                }
            if (km > 0) {
                double r = 1.0 / ab[ABI(j, j)];
                for (int i = 1; i <= km; ++i) ab[ABI(j + i, j)] *= r;
                for (int c = j + 1; c <= ju; ++c) {
                    double ujc = ab[ABI(j, c)];
                    if (ujc != 0.0)
                        for (int i = 1; i <= km; ++i) ab[ABI(j + i, c)] -= ab[ABI(j + i, j)] * ujc;
                }
            }
        } else if (info == 0) {
            info = j + 1;
        }
    }
    return info;
}

static void gbtrs(int n, const double* ab, const int* ipiv, double* b) {
    for (int j = 0; j < n - 1; ++j) {
        int lm = KL < n - 1 - j ? KL : n - 1 - j;
        int l = ipiv[j];
        if (l != j) { double t = b[l]; b[l] = b[j]; b[j] = t; }
        for (int i = 1; i <= lm; ++i) b[j + i] -= ab[ABI(j + i, j)] * b[j];
    }
    for (int j = n - 1; j >= 0; --j) {
        b[j] /= ab[ABI(j, j)];
        int i0 = j - KV < 0 ? 0 : j - KV;
        for (int i = i0; i < j; ++i) b[i] -= ab[ABI(i, j)] * b[j];
    }
}

/* ---------------- NLP pieces ---------------- */
static inline int kx(int k) { return 14 * k + 6; }  /* kkt index of x_k[0] */
static inline int ku_(int k) { return 14 * k + 12; } /* kkt index of u_k[0] */
static inline int ky(int k) { return 14 * k; }      /* kkt index of y_k[0] (row block of c_k) */

static double eval_cost(const ws_t* w, const double* z, const double* xref, const double* uref) {
    double F = 0.0;
    for (int k = 0; k <= w->N; ++k) {
        double d[6];
        for (int i = 0; i < 6; ++i) d[i] = z[NS * k + i] - xref[6 * k + i];
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) F += d[i] * w->Qw[i * 6 + j] * d[j];
        if (k < w->N) {
            double e[2];
            for (int i = 0; i < 2; ++i) e[i] = z[NS * k + 6 + i] - uref[2 * k + i];
            for (int i = 0; i < 2; ++i)
                for (int j = 0; j < 2; ++j) F += e[i] * w->Rw[i * 2 + j] * e[j];
        }
    }
    return F;
}

static void eval_grad(const ws_t* w, const double* z, const double* xref, const double* uref, double* g) {
    for (int k = 0; k <= w->N; ++k) {
        double d[6];
        for (int i = 0; i < 6; ++i) d[i] = z[NS * k + i] - xref[6 * k + i];
        for (int i = 0; i < 6; ++i) {
            double s = 0.0;
            for (int j = 0; j < 6; ++j) s += w->Qw[i * 6 + j] * d[j];
            g[NS * k + i] = 2.0 * s;
        }
        if (k < w->N) {
            double e[2];
            for (int i = 0; i < 2; ++i) e[i] = z[NS * k + 6 + i] - uref[2 * k + i];
            for (int i = 0; i < 2; ++i) g[NS * k + 6 + i] = 2.0 * (w->Rw[i * 2] * e[0] + w->Rw[i * 2 + 1] * e[1]);
        }
    }
}

static void eval_cons(const tto_problem* P, const ws_t* w, const double* z, const double* xinit, double* c) {
    for (int i = 0; i < 6; ++i) c[i] = z[i] - xinit[i];
    for (int k = 0; k < w->N; ++k) {
        double fo[6];
        fdyn(P, z + NS * k, z + NS * k + 6, fo);
        for (int i = 0; i < 6; ++i) c[6 * (k + 1) + i] = z[NS * (k + 1) + i] - (z[NS * k + i] + P->dt * fo[i]);
    }
}

static double barrier(const ws_t* w, const double* z, double mu, int* bad) {
    double s = 0.0;
    *bad = 0;
    for (int i = 0; i < w->n; ++i) {
        if (w->hasL[i]) { double d = z[i] - w->lb[i]; if (d <= 0) { *bad = 1; return 0; } s -= mu * log(d); }
        if (w->hasU[i]) { double d = w->ub[i] - z[i]; if (d <= 0) { *bad = 1; return 0; } s -= mu * log(d); }
    }
    return s;
}

static double norm1(const double* v, int n) { double s = 0; for (int i = 0; i < n; ++i) s += fabs(v[i]); return s; }

static void assemble(const tto_problem* P, ws_t* w, double mu, double dw, double dc) {
    const int N = w->N;
    memset(w->ab, 0, (size_t)LDAB * w->nk * sizeof(double));
#define SET(i, j, v) (w->ab[ABI((i), (j))] += (v))
    (void)mu;
    for (int k = 0; k <= N; ++k) {
        /* y_k rows */
        for (int i = 0; i < 6; ++i) { SET(ky(k) + i, ky(k) + i, -dc); SET(ky(k) + i, kx(k) + i, 1.0); SET(kx(k) + i, ky(k) + i, 1.0); }
        /* x_k Hessian block */
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j) {
                double h = 2.0 * w->Qw[i * 6 + j] + (k < N ? w->Wc[36 * k + i * 6 + j] : 0.0);
                SET(kx(k) + i, kx(k) + j, h);
            }
        for (int i = 0; i < 6; ++i) {
            int v = NS * k + i;
            double sig = dw;
            if (w->hasL[v]) sig += w->zL[v] / (w->z[v] - w->lb[v]);
            if (w->hasU[v]) sig += w->zU[v] / (w->ub[v] - w->z[v]);
            SET(kx(k) + i, kx(k) + i, sig);
        }
        if (k < N) {
            for (int i = 0; i < 2; ++i) {
                for (int j = 0; j < 2; ++j) SET(ku_(k) + i, ku_(k) + j, 2.0 * w->Rw[i * 2 + j]);
                int v = NS * k + 6 + i;
                double sig = dw;
                if (w->hasL[v]) sig += w->zL[v] / (w->z[v] - w->lb[v]);
                if (w->hasU[v]) sig += w->zU[v] / (w->ub[v] - w->z[v]);
                SET(ku_(k) + i, ku_(k) + i, sig);
            }
            /* c_{k+1} = x_{k+1} - A x_k - dt B u_k  (rows y_{k+1}) */
            const double* A = w->A + 36 * k;
            for (int i = 0; i < 6; ++i)
                for (int j = 0; j < 6; ++j)
                    if (A[i * 6 + j] != 0.0) { SET(ky(k + 1) + i, kx(k) + j, -A[i * 6 + j]); SET(kx(k) + j, ky(k + 1) + i, -A[i * 6 + j]); }
            /* B: v_dot <- a (row 5, u0), phi_dot <- omega (row 4, u1) */
            SET(ky(k + 1) + 5, ku_(k) + 0, -P->dt); SET(ku_(k) + 0, ky(k + 1) + 5, -P->dt);
            SET(ky(k + 1) + 4, ku_(k) + 1, -P->dt); SET(ku_(k) + 1, ky(k + 1) + 4, -P->dt);
        }
    }
#undef SET
}

/* d' (W + Sigma + dw) d over the primal block */
static double curvature(const ws_t* w, const double* d, double dw) {
    double s = 0.0;
    for (int k = 0; k <= w->N; ++k) {
        const double* x = d + NS * k;
        for (int i = 0; i < 6; ++i)
            for (int j = 0; j < 6; ++j)
                s += x[i] * (2.0 * w->Qw[i * 6 + j] + (k < w->N ? w->Wc[36 * k + i * 6 + j] : 0.0)) * x[j];
        int nv = k < w->N ? 8 : 6;
        if (k < w->N)
            for (int i = 0; i < 2; ++i)
                for (int j = 0; j < 2; ++j) s += x[6 + i] * 2.0 * w->Rw[i * 2 + j] * x[6 + j];
        for (int i = 0; i < nv; ++i) {
            int v = NS * k + i;
            double sig = dw;
            if (w->hasL[v]) sig += w->zL[v] / (w->z[v] - w->lb[v]);
            if (w->hasU[v]) sig += w->zU[v] / (w->ub[v] - w->z[v]);
            s += sig * x[i] * x[i];
        }
    }
    return s;
}

static void* xalloc(size_t n) { void* p = calloc(1, n); return p; }

static int ws_init(ws_t* w, int N) {
    w->N = N;
    w->n = NS * N + 6;
    w->m = 6 * (N + 1);
    w->nk = w->n + w->m;
    size_t n = (size_t)w->n, m = (size_t)w->m, nk = (size_t)w->nk;
    w->z = xalloc(n * 8); w->zL = xalloc(n * 8); w->zU = xalloc(n * 8); w->y = xalloc(m * 8);
    w->lb = xalloc(n * 8); w->ub = xalloc(n * 8); w->hasL = xalloc(n); w->hasU = xalloc(n);
    w->gF = xalloc(n * 8); w->c = xalloc(m * 8); w->A = xalloc((size_t)N * 36 * 8); w->Wc = xalloc((size_t)N * 36 * 8);
    w->ab = xalloc((size_t)LDAB * nk * 8); w->rhs = xalloc(nk * 8); w->rhs2 = xalloc(nk * 8); w->ipiv = xalloc(nk * sizeof(int));
    w->dz = xalloc(n * 8); w->yp = xalloc(m * 8); w->dzL = xalloc(n * 8); w->dzU = xalloc(n * 8);
    w->zt = xalloc(n * 8); w->ct = xalloc(m * 8); w->dzs = xalloc(n * 8);
    return w->dzs ? 0 : -1;
}

static void ws_free(ws_t* w) {
    free(w->z); free(w->zL); free(w->zU); free(w->y); free(w->lb); free(w->ub); free(w->hasL); free(w->hasU);
    free(w->gF); free(w->c); free(w->A); free(w->Wc); free(w->ab); free(w->rhs); free(w->rhs2); free(w->ipiv);
    free(w->dz); free(w->yp); free(w->dzL); free(w->dzU); free(w->zt); free(w->ct); free(w->dzs);
}

/* merit = F - mu*sum(log s) + nu*||c||_1 ; returns +inf if outside the bounds */
/* filter trial point: returns the barrier objective phi_mu(z) (+inf outside the relaxed box) and
 * theta(z) = ||c(z)||_1 in *th_out; c(z) is left in w->ct for the second-order correction */
static double trial_at(const tto_problem* P, ws_t* w, const double* z, const double* xinit, const double* xref,
                       const double* uref, double mu, double* th_out) {
    int bad = 0;
    double b = barrier(w, z, mu, &bad);
    eval_cons(P, w, z, xinit, w->ct);
    *th_out = norm1(w->ct, w->m);
    if (bad) return INFINITY;
    return eval_cost(w, z, xref, uref) + b;
}

static int solve_one(const tto_problem* P, ws_t* w, const double* xinit, const double* xref, const double* uref,
                     const double* wq, const double* wr, const double* zg, double* zout, int* iters_out,
                     double* kkt_out) {
    const int N = w->N, n = w->n, m = w->m, nk = w->nk;
    const double kappa1 = 1e-2, kappa2 = 1e-2, smax = 100.0, kappa_eps = 10.0, kappa_mu = 0.2, theta_mu = 1.5;
    const double kappa_sigma = 1e10, eta = 1e-4;
    const double tol = P->tol, acc_tol = P->acc_tol;
    const double mu_min = fmin(tol, COMPL_INF_TOL) / (BARRIER_TOL_FACTOR + 1.0); /* MonotoneMuUpdate floor */
    /* weights: Qw = diag(wq) Qs diag(wq) (mpc_control_fuzzy.py:23-24); Qs = sym(Q) */
    for (int i = 0; i < 6; ++i)
        for (int j = 0; j < 6; ++j) {
            double q = 0.5 * (P->Q[i * 6 + j] + P->Q[j * 6 + i]);
            w->Qw[i * 6 + j] = q * (wq ? wq[i] * wq[j] : 1.0);
        }
    for (int i = 0; i < 2; ++i)
        for (int j = 0; j < 2; ++j) {
            double r = 0.5 * (P->R[i * 2 + j] + P->R[j * 2 + i]);
            w->Rw[i * 2 + j] = r * (wr ? wr[i] * wr[j] : 1.0);
        }
    /* relaxed bounds (bound_relax_factor 1e-8) */
    for (int k = 0; k <= N; ++k)
        for (int i = 0; i < (k < N ? 8 : 6); ++i) {
            int v = NS * k + i;
            double l = i < 6 ? P->xlb[i] : P->ulb[i - 6], u = i < 6 ? P->xub[i] : P->uub[i - 6];
            w->hasL[v] = l > -1e19 && isfinite(l);
            w->hasU[v] = u < 1e19 && isfinite(u);
            w->lb[v] = w->hasL[v] ? l - 1e-8 * fmax(1.0, fabs(l)) : -INFINITY;
            w->ub[v] = w->hasU[v] ? u + 1e-8 * fmax(1.0, fabs(u)) : INFINITY;
        }
    /* initial guess: reference copy (mpc_control.py:58-65) */
    for (int k = 0; k <= N; ++k) {
        for (int i = 0; i < 6; ++i) w->z[NS * k + i] = zg ? zg[NS * k + i] : xref[6 * k + i];
        if (k < N)
            for (int i = 0; i < 2; ++i) w->z[NS * k + 6 + i] = zg ? zg[NS * k + 6 + i] : uref[2 * k + i];
    }
    int status = 2, iter = 0;
    double E0 = INFINITY;
    /* infeasible: x_0 = x_init must lie in the (relaxed) bounds of x_0 */
    for (int i = 0; i < 6; ++i) {
        if (!isfinite(xinit[i]) || (w->hasL[i] && xinit[i] < w->lb[i]) || (w->hasU[i] && xinit[i] > w->ub[i])) {
            status = 3;
        }
    }
    if (status == 3) {
        memcpy(zout, w->z, (size_t)n * 8);
        if (iters_out) *iters_out = 0;
        if (kkt_out) *kkt_out = INFINITY;
        return 3;
    }
    /* bound push (IPOPT bound_push / bound_frac) */
    for (int v = 0; v < n; ++v) {
        double l = w->lb[v], u = w->ub[v], z = w->z[v];
        if (w->hasL[v] && w->hasU[v]) {
            double pl = fmin(kappa1 * fmax(1.0, fabs(l)), kappa2 * (u - l));
            double pu = fmin(kappa1 * fmax(1.0, fabs(u)), kappa2 * (u - l));
            z = fmin(fmax(z, l + pl), u - pu);
        } else if (w->hasL[v]) {
            z = fmax(z, l + kappa1 * fmax(1.0, fabs(l)));
        } else if (w->hasU[v]) {
            z = fmin(z, u - kappa1 * fmax(1.0, fabs(u)));
        }
        w->z[v] = z;
        w->zL[v] = w->hasL[v] ? 1.0 : 0.0;
        w->zU[v] = w->hasU[v] ? 1.0 : 0.0;
    }
    memset(w->y, 0, (size_t)m * 8);
    double mu = 0.1, tau = fmax(0.99, 1.0 - mu), nu = 1.0, dw_last = 0.0, th_max = 0.0, th_min = 0.0;
    double fth[TTO_MAX_FILTER], fph[TTO_MAX_FILTER];
    int nf = 0;
    int acc_count = 0, nb = 0;
    for (int v = 0; v < n; ++v) nb += w->hasL[v] + w->hasU[v];

    for (iter = 0;; ++iter) {
        /* ---- evaluate ---- */
        eval_grad(w, w->z, xref, uref, w->gF);
        eval_cons(P, w, w->z, xinit, w->c);
        for (int k = 0; k < N; ++k) {
            jac_A(P, w->z + NS * k, w->A + 36 * k);
            memset(w->Wc + 36 * k, 0, 36 * 8);
            hess_acc(P, w->z + NS * k, w->y + 6 * (k + 1), -P->dt, w->Wc + 36 * k);
        }
        /* ---- optimality error ---- */
        double dinf = 0.0, pinf = 0.0, c0 = 0.0, cmu = 0.0, sy = norm1(w->y, m), sz = 0.0;
        int finite = 1;
        for (int k = 0; k <= N; ++k)
            for (int i = 0; i < (k < N ? 8 : 6); ++i) {
                int v = NS * k + i;
                double gl = w->gF[v] - w->zL[v] + w->zU[v];
                if (i < 6) {
                    gl += w->y[6 * k + i];
                    if (k < N)
                        for (int r = 0; r < 6; ++r) gl -= w->A[36 * k + r * 6 + i] * w->y[6 * (k + 1) + r];
                } else {
                    gl -= P->dt * w->y[6 * (k + 1) + (i == 6 ? 5 : 4)];
                }
                if (!isfinite(gl)) finite = 0;
                dinf = fmax(dinf, fabs(gl));
                if (w->hasL[v]) { double s = w->z[v] - w->lb[v]; c0 = fmax(c0, fabs(w->zL[v] * s)); cmu = fmax(cmu, fabs(w->zL[v] * s - mu)); sz += w->zL[v]; }
                if (w->hasU[v]) { double s = w->ub[v] - w->z[v]; c0 = fmax(c0, fabs(w->zU[v] * s)); cmu = fmax(cmu, fabs(w->zU[v] * s - mu)); sz += w->zU[v]; }
            }
        for (int j = 0; j < m; ++j) pinf = fmax(pinf, fabs(w->c[j]));
        if (!finite || !isfinite(pinf)) { status = 4; break; }
        double sd = fmax(smax, (sy + sz) / (double)(m + nb)) / smax;
        double sc = nb ? fmax(smax, sz / (double)nb) / smax : 1.0;
        E0 = fmax(fmax(dinf / sd, pinf), c0 / sc);
        if (getenv("TTO_DEBUG"))
            fprintf(stderr, "it %3d E0 %.3e dinf %.3e pinf %.3e c0 %.3e mu %.2e sd %.2e nu %.2e\n", iter, E0, dinf, pinf, c0,
                    mu, sd, nu);
        /* IPOPT's convergence test: the scaled error and the unscaled dual infeasibility, constraint violation
         * (the dynamics rows: max |c| = pinf) and complementarity max |z s| = c0 */
        const int conv = E0 <= tol && dinf <= DUAL_INF_TOL && pinf <= CONSTR_VIOL_TOL && c0 <= COMPL_INF_TOL;
        const int accp = E0 <= acc_tol && dinf <= ACC_DUAL_INF_TOL && pinf <= ACC_CONSTR_VIOL_TOL && c0 <= ACC_COMPL_INF_TOL;
        if (conv) { status = 0; break; }
        if (accp) {
            if (++acc_count >= P->acc_iter) { status = 1; break; }
        } else {
            acc_count = 0;
        }
        if (iter >= P->max_iter) { status = accp ? 1 : 2; break; }
        /* ---- barrier parameter update (monotone, Fiacco-McCormick) ---- */
        for (;;) {
            double Emu = fmax(fmax(dinf / sd, pinf), cmu / sc);
            if (Emu <= kappa_eps * mu && mu > mu_min * 1.0000001) {
                mu = fmax(mu_min, fmin(kappa_mu * mu, pow(mu, theta_mu)));
                tau = fmax(0.99, 1.0 - mu);
                nf = 0; /* IPOPT resets the filter on every barrier update */
                cmu = 0.0;
                for (int v = 0; v < n; ++v) {
                    if (w->hasL[v]) cmu = fmax(cmu, fabs(w->zL[v] * (w->z[v] - w->lb[v]) - mu));
                    if (w->hasU[v]) cmu = fmax(cmu, fabs(w->zU[v] * (w->ub[v] - w->z[v]) - mu));
                }
            } else {
                break;
            }
        }
        /* ---- Newton step with inertia-free regularisation ---- */
        double dw = 0.0, dc = 0.0;
        int ok = 0;
        for (int attempt = 0; attempt < 30; ++attempt) {
            assemble(P, w, mu, dw, dc);
            int info = gbtf2(nk, w->ab, w->ipiv);
            if (info == 0) {
                for (int k = 0; k <= N; ++k) {
                    for (int i = 0; i < (k < N ? 8 : 6); ++i) {
                        int v = NS * k + i;
                        double g = w->gF[v];
                        if (w->hasL[v]) g -= mu / (w->z[v] - w->lb[v]);
                        if (w->hasU[v]) g += mu / (w->ub[v] - w->z[v]);
                        w->rhs[(i < 6 ? kx(k) + i : ku_(k) + i - 6)] = -g;
                    }
                    for (int i = 0; i < 6; ++i) w->rhs[ky(k) + i] = -w->c[6 * k + i];
                }
                gbtrs(nk, w->ab, w->ipiv, w->rhs);
                for (int k = 0; k <= N; ++k) {
                    for (int i = 0; i < (k < N ? 8 : 6); ++i) w->dz[NS * k + i] = w->rhs[i < 6 ? kx(k) + i : ku_(k) + i - 6];
                    for (int i = 0; i < 6; ++i) w->yp[6 * k + i] = w->rhs[ky(k) + i];
                }
                double dd = 0.0;
                for (int v = 0; v < n; ++v) dd += w->dz[v] * w->dz[v];
                if (curvature(w, w->dz, dw) >= 1e-11 * dd) { ok = 1; break; }
            } else {
                dc = 1e-8 * pow(mu, 0.25);
            }
            dw = (dw == 0.0) ? (dw_last == 0.0 ? 1e-4 : fmax(1e-20, dw_last / 3.0)) : (dw_last == 0.0 ? 100.0 * dw : 8.0 * dw);
            if (dw > 1e20) break; /* IPOPT max_hessian_perturbation 1e20 */
        }
        if (!ok) { status = 5; break; } /* IPOPT Error_In_Step_Computation */
        if (dw > 0) dw_last = dw;
        /* ---- bound-multiplier steps ---- */
        for (int v = 0; v < n; ++v) {
            w->dzL[v] = w->hasL[v] ? mu / (w->z[v] - w->lb[v]) - w->zL[v] - w->zL[v] / (w->z[v] - w->lb[v]) * w->dz[v] : 0.0;
            w->dzU[v] = w->hasU[v] ? mu / (w->ub[v] - w->z[v]) - w->zU[v] + w->zU[v] / (w->ub[v] - w->z[v]) * w->dz[v] : 0.0;
        }
        /* ---- fraction to the boundary ---- */
        double ap = 1.0, az = 1.0;
        for (int v = 0; v < n; ++v) {
            if (w->hasL[v]) {
                double s = w->z[v] - w->lb[v];
                if (w->dz[v] < 0) ap = fmin(ap, -tau * s / w->dz[v]);
                if (w->dzL[v] < 0) az = fmin(az, -tau * w->zL[v] / w->dzL[v]);
            }
            if (w->hasU[v]) {
                double s = w->ub[v] - w->z[v];
                if (w->dz[v] > 0) ap = fmin(ap, tau * s / w->dz[v]);
                if (w->dzU[v] < 0) az = fmin(az, -tau * w->zU[v] / w->dzU[v]);
            }
        }
        /* ---- filter line search (Waechter & Biegler 2006; IPOPT defaults) + one second-order correction ---- */
        double ymax = 0.0;
        for (int j = 0; j < m; ++j) ymax = fmax(ymax, fabs(w->yp[j]));
        if (nu < ymax + 1.0) nu = fmax(1.1 * ymax + 1.0, nu); /* diagnostics only (printed) */
        int bad = 0;
        const double th0 = norm1(w->c, m);
        const double phi0 = eval_cost(w, w->z, xref, uref) + barrier(w, w->z, mu, &bad);
        double D = 0.0;
        for (int v = 0; v < n; ++v) {
            double g = w->gF[v];
            if (w->hasL[v]) g -= mu / (w->z[v] - w->lb[v]);
            if (w->hasU[v]) g += mu / (w->ub[v] - w->z[v]);
            D += g * w->dz[v];
        }
        if (iter == 0) { th_max = 1e4 * fmax(1.0, th0); th_min = 1e-4 * fmax(1.0, th0); }
        const double g_th = 1e-5, g_ph = 1e-8, s_ph = 2.3, s_th = 1.1, delta = 1.0, g_al = 0.05;
        double amin = g_th;
        if (D < 0.0) {
            amin = fmin(g_th, g_ph * th0 / (-D));
            if (th0 <= th_min) amin = fmin(amin, delta * pow(th0, s_th) / pow(-D, s_ph));
        }
        amin *= g_al;
        const double tolc = 10.0 * DBL_EPSILON;
        double alpha = ap;
        int accepted = 0, ftype = 0;
        /* tiny step -> accept */
        double rel = 0.0;
        for (int v = 0; v < n; ++v) rel = fmax(rel, fabs(w->dz[v]) / (1.0 + fabs(w->z[v])));
        if (rel < 1e-15) accepted = 1;
#define FILTER_OK(tht_, pht_, a_, ok_) do { \
            ok_ = 0; \
            if (isfinite(pht_) && (tht_) <= th_max) { \
                int blocked = 0; \
                for (int f_ = 0; f_ < nf; ++f_) if ((tht_) >= fth[f_] && (pht_) >= fph[f_]) { blocked = 1; break; } \
                if (!blocked) { \
                    const int sw_ = D < 0.0 && (a_) * pow(-D, s_ph) > delta * pow(th0, s_th); \
                    if (th0 <= th_min && sw_) { ftype = 1; ok_ = (pht_) - (phi0 + eta * (a_) * D) <= tolc * fabs(phi0); } \
                    else { ftype = 0; ok_ = (tht_) <= (1.0 - g_th) * th0 || (pht_) - (phi0 - g_ph * th0) <= tolc * fabs(phi0); } \
                } \
            } } while (0)
        for (int ls = 0; !accepted; ++ls) {
            for (int v = 0; v < n; ++v) w->zt[v] = w->z[v] + alpha * w->dz[v];
            double tht = 0.0;
            const double pht = trial_at(P, w, w->zt, xinit, xref, uref, mu, &tht);
            int ok;
            FILTER_OK(tht, pht, alpha, ok);
            if (ok) { accepted = 1; break; }
            if (ls == 0 && isfinite(pht) && tht >= th0) {
                /* second-order correction: c_soc = alpha c(z) + c(z + alpha dz) */
                for (int k = 0; k <= N; ++k) {
                    for (int i = 0; i < (k < N ? 8 : 6); ++i) {
                        int v = NS * k + i;
                        double g = w->gF[v];
                        if (w->hasL[v]) g -= mu / (w->z[v] - w->lb[v]);
                        if (w->hasU[v]) g += mu / (w->ub[v] - w->z[v]);
                        w->rhs2[(i < 6 ? kx(k) + i : ku_(k) + i - 6)] = -g;
                    }
                    for (int i = 0; i < 6; ++i) w->rhs2[ky(k) + i] = -(alpha * w->c[6 * k + i] + w->ct[6 * k + i]);
                }
                gbtrs(nk, w->ab, w->ipiv, w->rhs2);
                double as = 1.0;
                for (int k = 0; k <= N; ++k)
                    for (int i = 0; i < (k < N ? 8 : 6); ++i) w->dzs[NS * k + i] = w->rhs2[i < 6 ? kx(k) + i : ku_(k) + i - 6];
                for (int v = 0; v < n; ++v) {
                    if (w->hasL[v] && w->dzs[v] < 0) as = fmin(as, -tau * (w->z[v] - w->lb[v]) / w->dzs[v]);
                    if (w->hasU[v] && w->dzs[v] > 0) as = fmin(as, tau * (w->ub[v] - w->z[v]) / w->dzs[v]);
                }
                for (int v = 0; v < n; ++v) w->zt[v] = w->z[v] + as * w->dzs[v];
                double ths = 0.0;
                const double phs = trial_at(P, w, w->zt, xinit, xref, uref, mu, &ths);
                int ok2;
                FILTER_OK(ths, phs, alpha, ok2);
                if (ok2) {
                    accepted = 2;
                    alpha = as;
                    for (int j = 0; j < m; ++j) w->yp[j] = w->rhs2[ky(j / 6) + j % 6];
                    memcpy(w->dz, w->dzs, (size_t)n * 8);
                    for (int v = 0; v < n; ++v) {
                        w->dzL[v] = w->hasL[v] ? mu / (w->z[v] - w->lb[v]) - w->zL[v] - w->zL[v] / (w->z[v] - w->lb[v]) * w->dz[v] : 0.0;
                        w->dzU[v] = w->hasU[v] ? mu / (w->ub[v] - w->z[v]) - w->zU[v] + w->zU[v] / (w->ub[v] - w->z[v]) * w->dz[v] : 0.0;
                    }
                    az = 1.0;
                    for (int v = 0; v < n; ++v) {
                        if (w->hasL[v] && w->dzL[v] < 0) az = fmin(az, -tau * w->zL[v] / w->dzL[v]);
                        if (w->hasU[v] && w->dzU[v] < 0) az = fmin(az, -tau * w->zU[v] / w->dzU[v]);
                    }
                    break;
                }
            }
            if (alpha * 0.5 < amin) break;
            alpha *= 0.5;
        }
#undef FILTER_OK
        if (!accepted) {
            nf = 0; /* IPOPT would enter its restoration phase; take the last trial step and reset the filter */
        } else if (accepted == 1 && rel < 1e-15) {
            /* negligible step: nothing to add */
        } else if (!ftype && nf < TTO_MAX_FILTER) {
            fth[nf] = (1.0 - g_th) * th0;
            fph[nf] = phi0 - g_ph * th0;
            ++nf;
        }
        if (getenv("TTO_DEBUG")) fprintf(stderr, "   ap %.3e az %.3e alpha %.3e acc %d D %.3e\n", ap, az, alpha, accepted, D);
        /* ---- update ---- */
        for (int v = 0; v < n; ++v) w->z[v] += alpha * w->dz[v];
        for (int j = 0; j < m; ++j) w->y[j] += alpha * (w->yp[j] - w->y[j]);
        for (int v = 0; v < n; ++v) {
            if (w->hasL[v]) {
                double s = w->z[v] - w->lb[v], zl = w->zL[v] + az * w->dzL[v];
                w->zL[v] = fmax(fmin(zl, kappa_sigma * mu / s), mu / (kappa_sigma * s));
            }
            if (w->hasU[v]) {
                double s = w->ub[v] - w->z[v], zu = w->zU[v] + az * w->dzU[v];
                w->zU[v] = fmax(fmin(zu, kappa_sigma * mu / s), mu / (kappa_sigma * s));
            }
        }
    }
    memcpy(zout, w->z, (size_t)n * 8);
    if (iters_out) *iters_out = iter;
    if (kkt_out) *kkt_out = E0;
    return status;
}

int tto_solve(const tto_problem* P, const double* x_init, const double* xref, const double* uref,
              const double* wq, const double* wr, const double* z_guess, double* z_out, int* iters, double* kkt) {
    ws_t w;
    if (P->N < 1 || ws_init(&w, P->N) != 0) return -1;
    int st = solve_one(P, &w, x_init, xref, uref, wq, wr, z_guess, z_out, iters, kkt);
    ws_free(&w);
    return st;
}

int tto_solve_batch(const tto_problem* P, int B, const double* x_init, const double* xref, const double* uref,
                    const double* wq, const double* wr, const double* z_guess, double* z_out, int* status,
                    int* iters, double* kkt, int nthreads) {
    if (P->N < 1 || B < 0) return -1;
    const int N = P->N, n = NS * N + 6;
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    int err = 0;
#pragma omp parallel
    {
        ws_t w;
        int bad = ws_init(&w, N);
#pragma omp for schedule(static)
        for (int b = 0; b < B; ++b) {
            if (bad) { status[b] = -1; continue; }
            int it = 0;
            double e = 0.0;
            status[b] = solve_one(P, &w, x_init + 6 * (size_t)b, xref + (size_t)b * 6 * (N + 1), uref + (size_t)b * 2 * N,
                                  wq ? wq + 6 * (size_t)b : NULL, wr ? wr + 2 * (size_t)b : NULL,
                                  z_guess ? z_guess + (size_t)b * n : NULL, z_out + (size_t)b * n, &it, &e);
            if (iters) iters[b] = it;
            if (kkt) kkt[b] = e;
        }
        if (bad) err = -1;
        ws_free(&w);
    }
    return err;
}
