/* Structured interior-point solver for the SQP-RTI feedback-phase QP -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of what acados' SQP_RTI hands to HPIPM (sdf_nmpc/ocp.py:110-120: NONLINEAR_LS +
 * GAUSS_NEWTON cost with levenberg_marquardt, input boxes, soft h rows with L1/L2 slack penalties
 * ocp.py:80-92, x_0 fixed) on the stage structure: a Mehrotra predictor-corrector whose Newton systems
 * are LQRs solved by a backward Riccati recursion -- HPIPM's OCP-QP IPM family (HPIPM itself is an
 * absent third-party dependency).  It is
 *   - a second, independent checker of csrc/rti_qp.hip (same QP as oracle/qp_oracle.py's dense KKT
 *     solver, different linear algebra), and
 *   - the QP half of bench.py's cpu_baseline for the full-RTI metric (one C solve per instance, as
 *     the reference runs one acados solver per process).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg call it.
 *
 * QP of one instance (w_k = [dx_k; du_k]; s_k = dt_k for k < N with cost scaling, else 1; s_N = 1):
 *   min  sum_{k<N} s_k 1/2 |J_y,k w_k + r_k|^2_{W_k} + lm_k/2 |w_k|^2 + s_N 1/2 |J_yN dx_N + r_N|^2_{W_N}
 *        + lm/2 |dx_N|^2 + sum_{k<=N} s_k (zl.sl_k + Zl/2 sl_k^2 + zl.su_k + Zl/2 su_k^2)
 *   lm_k = lm dt_k with lm_scaling (acados adds Ts[k] * levenberg_marquardt for k < N), else lm
 *   s.t. dx_0 = x0 - xbar_0,  dx_{k+1} = A_k dx_k + B_k du_k + (xn_k - xbar_{k+1})
 *        u_k + du_k in [lbu, ubu];  lh - sl_k <= h_k + C_k dx_k <= uh + su_k;  sl, su >= 0
 * Inputs use the sdfnmpc_linearize layouts (include/sdfnmpc.h): AB [N][14][10] with AB[j][i] =
 * d xn_i / d (x,u)_j, Jy [N][14][11] (Jy[j][a] = d y_a / d w_j), JyN [10][4], Jh [N+1][10][3].
 */
#include <math.h>
#include <stdlib.h>
#include <string.h>

enum { NX = 10, NU = 4, NS = 3, NW = 14, NR = 8 /* rows per node at most (terminal: SDFNMPC_NHN_MAX) */ };

typedef struct {
    double lbu[4], ubu[4], lh[3], uh[3], zl[3], Zl[3], lm, tol;
    int max_iter, cost_scaling, lm_scaling, nseg;
    double t0, l0, lc, tau_lo, tau_hi;  /* starting point / step fraction (rti_qp.hip's QP_T0 ... QP_TAU_HI) */
    /* Gondzio centrality correctors (off at gk = 0): up to gk extra solves on the factorisation of the
     * iteration when the Mehrotra step is below ga; trial step min(1, alpha + gd), products projected
     * onto [gbmin, gbmax] sigma mu; a corrector is kept when it lengthens the step by >= 0.1 gd */
    int gk;
    double ga, gd, gbmin, gbmax;
    /* primal warm start (HPIPM's qp_solver_warm_start = 1, ocp.py:116): the start point takes du from the
     * du buffer on entry (the previous QP's solution) instead of 0; dx is the dynamics rollout from x0 under
     * that du, t / lambda follow the cold start's rule on the rows there */
    int ws;
    /* the constraint set (include/sdfnmpc.h sdfnmpc_qp_opts): stage rows j < nh = column h_col[j] of h / J_h
     * (bounds lh .. Zl above), the last nhs of them hard (slack weight None, base_model.py:142-155); terminal
     * rows j < nhN (the first nsN soft) = h[N][hN_col[j]] + hE[hE_col[j]] */
    int nh, h_col[3], nhN, nsN, hN_col[NR], hE_col[NR], nyN, nhs;
    double lhN[NR], uhN[NR], zlN[3], ZlN[3];
} qp_opts_c;

typedef struct {                  /* stage k < N, or the terminal node k = N (x part only) */
    double A[NX][NX], Bm[NX][NU], c[NX];
    double H[NW][NW], g[NW];
    /* constraint rows j < nrow, the first nsoft soft: C dx + sl + hl >= 0, -C dx + su + hu >= 0 (slacks with
     * L1 / L2 weights zl / Zl); the rest hard: C dx + hl >= 0, -C dx + hu >= 0 */
    double C[NR][NX], hl[NR], hu[NR], zl[NR], Zl[NR];
    int nsoft, nrow;
    double dlo[NU], dup[NU];            /* box rows: du + dlo >= 0, -du + dup >= 0 */
    double s;                           /* cost scaling s_k */
} stage_t;

/* in-place lower Cholesky of an n x n SPD matrix; 0 on success */
static int chol(int n, double* a) {
    for (int j = 0; j < n; ++j) {
        double d = a[j * n + j];
        for (int k = 0; k < j; ++k) d -= a[j * n + k] * a[j * n + k];
        if (!(d > 0.0)) return 1;
        d = sqrt(d);
        a[j * n + j] = d;
        for (int i = j + 1; i < n; ++i) {
            double v = a[i * n + j];
            for (int k = 0; k < j; ++k) v -= a[i * n + k] * a[j * n + k];
            a[i * n + j] = v / d;
        }
    }
    return 0;
}
/* x <- (L L^T)^-1 x */
static void chol_solve(int n, const double* L, double* x) {
    for (int i = 0; i < n; ++i) {
        double v = x[i];
        for (int k = 0; k < i; ++k) v -= L[i * n + k] * x[k];
        x[i] = v / L[i * n + i];
    }
    for (int i = n - 1; i >= 0; --i) {
        double v = x[i];
        for (int k = i + 1; k < n; ++k) v -= L[k * n + i] * x[k];
        x[i] = v / L[i * n + i];
    }
}

/* Rows, the order of rti_qp.hip: box rows 8 k + 4 up + i; soft group e (stage groups k ns + j, then the
 * terminal's soft rows) at 8 N + 4 e + q with q = 0 (h lower), 1 (h upper), 2 (sl >= 0), 3 (su >= 0); hard
 * row i (stage rows (k - 1) nhs + j - ns of 0 < k < N, then the terminal's hard rows) at RH0 + 2 i (lower), + 1 (upper),
 * RH0 = 8 N + 4 (N ns + nsN). */
typedef struct {
    int N, m, ns, nhs, rh0;       /* ns / nhs: soft / hard rows of a stage k < N */
    const qp_opts_c* o;
    stage_t* st;
    double x0[NX];                /* dx_0 */
    double *P, *p, *K, *kf;       /* Riccati workspace: (N+1) x NX x NX, (N+1) x NX, N x NU x NX, N x NU */
    double* G;                    /* N x NU x NX: terminal-multiplier gains of the segmented solve */
    int nseg;                     /* segments of the partitioned Riccati (1: the serial recursion) */
    double seg_dev;               /* max relative gap between a segment's own x_b and the coupled one */
    int gcount;                   /* Gondzio correctors kept (diagnostic) */
} ipm_t;

static int grp(const ipm_t* Q, int k, int j) { return (k < Q->N ? k * Q->ns : Q->N * Q->ns) + j; }
/* hard row j (>= the node's soft rows) of node 0 < k <= N: its index among the hard rows (node 0 has none:
 * acados 0.3.1 takes initial-node nonlinear rows only from con_h_expr_0, which ocp.py does not set) */
static int hgrp(const ipm_t* Q, int k, int j) { return (k - 1) * Q->nhs + j - Q->st[k].nsoft; }

static void rows_at(const ipm_t* Q, const double* dx, const double* du, const double* sl, const double* su, double* v) {
    const int N = Q->N;
    for (int k = 0; k < N; ++k)
        for (int i = 0; i < NU; ++i) {
            v[8 * k + i] = du[k * NU + i] + Q->st[k].dlo[i];
            v[8 * k + 4 + i] = -du[k * NU + i] + Q->st[k].dup[i];
        }
    for (int k = 0; k <= N; ++k)
        for (int j = 0; j < Q->st[k].nrow; ++j) {
            double cx = 0.0;
            for (int l = 0; l < NX; ++l) cx += Q->st[k].C[j][l] * dx[k * NX + l];
            if (j < Q->st[k].nsoft) {
                const int e = grp(Q, k, j), r = 8 * N + 4 * e;
                v[r] = cx + Q->st[k].hl[j] + sl[e];
                v[r + 1] = -cx + Q->st[k].hu[j] + su[e];
                v[r + 2] = sl[e];
                v[r + 3] = su[e];
            } else {
                const int r = Q->rh0 + 2 * hgrp(Q, k, j);
                v[r] = cx + Q->st[k].hl[j];
                v[r + 1] = -cx + Q->st[k].hu[j];
            }
        }
}

/* Stage data of the Newton system at node k: the state block with the eliminated slack pairs folded
 * in (Qx, qx), and the input block with the box terms (R0, ru). */
static void stage_terms(const ipm_t* Q, int k, const double* sig, const double* v, double* Qx, double* qx, double* R0,
                        double* S0, double* ru, double* bd) {
    const int N = Q->N;
    const qp_opts_c* o = Q->o;
    const stage_t* S = &Q->st[k];
    for (int a = 0; a < NX; ++a) {
        for (int b = 0; b < NX; ++b) Qx[a * NX + b] = S->H[a][b];
        qx[a] = S->g[a];
    }
    (void)o;
    for (int j = 0; j < S->nrow; ++j) {
        double fw, fg;
        if (j < S->nsoft) {  /* eliminated slack pair */
            const int r0 = 8 * N + 4 * grp(Q, k, j);
            const double Zs = S->s * S->Zl[j], zs = S->s * S->zl[j];
            const double Hl = Zs + sig[r0] + sig[r0 + 2], Hu = Zs + sig[r0 + 1] + sig[r0 + 3];
            /* written without the cancellation of Hl - sig (sig -> inf on an active row); equal to
             * sig (Hl - sig) / Hl and -(v + sig gl / Hl) + ... */
            fw = sig[r0] * (Zs + sig[r0 + 2]) / Hl + sig[r0 + 1] * (Zs + sig[r0 + 3]) / Hu;
            fg = -(v[r0] * (Zs + sig[r0 + 2]) + sig[r0] * (zs - v[r0 + 2])) / Hl +
                 (v[r0 + 1] * (Zs + sig[r0 + 3]) + sig[r0 + 1] * (zs - v[r0 + 3])) / Hu;
        } else {  /* hard row: the two sides fold like box rows */
            const int r = Q->rh0 + 2 * hgrp(Q, k, j);
            fw = sig[r] + sig[r + 1];
            fg = -v[r] + v[r + 1];
        }
        for (int a = 0; a < NX; ++a) {
            for (int b = 0; b < NX; ++b) Qx[a * NX + b] += fw * S->C[j][a] * S->C[j][b];
            qx[a] += fg * S->C[j][a];
        }
    }
    if (k == N) return;
    for (int i = 0; i < NU; ++i) {
        for (int j = 0; j < NU; ++j) R0[i * NU + j] = S->H[NX + i][NX + j];
        bd[i] = sig[8 * k + i] + sig[8 * k + 4 + i];
        R0[i * NU + i] += bd[i];
        for (int b = 0; b < NX; ++b) S0[i * NX + b] = S->H[NX + i][b];
        ru[i] = S->g[NX + i] - v[8 * k + i] + v[8 * k + 4 + i];
    }
}

/* One backward Riccati stage k < N from the cost-to-go [P1 | p1] of node k + 1:
 * R^ = R0 + B^T P1 B (Cholesky factor into Rc), [K | kf] = -R^-1 ([S0 | ru] + B^T [P1 A | P1 c + p1]),
 * Ab = A + B K, and [Pk | pk] in the Joseph form [I;K]^T Hh [I;K] + Ab^T P1 Ab (a sum of PSD terms). */
static int ric_stage(const ipm_t* Q, int k, const double* Qx, const double* qx, const double* R0, const double* S0,
                     const double* ru, const double* bd, const double* P1, const double* p1, double* Pk, double* pk, double* Kk,
                     double* kf, double* Ab, double* Rc) {
    const stage_t* S = &Q->st[k];
    /* PA = P A, PB = P B, Pc = P c + p */
    double PA[NX * NX], PB[NX * NU], Pc[NX];
    for (int a = 0; a < NX; ++a) {
        for (int b = 0; b < NX; ++b) {
            double s = 0.0;
            for (int l = 0; l < NX; ++l) s += P1[a * NX + l] * S->A[l][b];
            PA[a * NX + b] = s;
        }
        for (int b = 0; b < NU; ++b) {
            double s = 0.0;
            for (int l = 0; l < NX; ++l) s += P1[a * NX + l] * S->Bm[l][b];
            PB[a * NU + b] = s;
        }
        double s = p1[a];
        for (int l = 0; l < NX; ++l) s += P1[a * NX + l] * S->c[l];
        Pc[a] = s;
    }
    double* Rm = Rc;
    double Sm[NU * NX], r[NU];
    for (int i = 0; i < NU; ++i) {
        for (int j = 0; j < NU; ++j) {
            double s = S->H[NX + i][NX + j];
            for (int l = 0; l < NX; ++l) s += S->Bm[l][i] * PB[l * NU + j];
            Rm[i * NU + j] = s;
        }
        Rm[i * NU + i] += bd[i];
        for (int b = 0; b < NX; ++b) {
            double s = S0[i * NX + b];
            for (int l = 0; l < NX; ++l) s += S->Bm[l][i] * PA[l * NX + b];
            Sm[i * NX + b] = s;
        }
        double s = ru[i];
        for (int l = 0; l < NX; ++l) s += S->Bm[l][i] * Pc[l];
        r[i] = s;
    }
    if (chol(NU, Rm)) return 1;
    for (int b = 0; b < NX; ++b) {  /* K = -R^-1 S, column by column */
        double col[NU];
        for (int i = 0; i < NU; ++i) col[i] = Sm[i * NX + b];
        chol_solve(NU, Rm, col);
        for (int i = 0; i < NU; ++i) Kk[i * NX + b] = -col[i];
    }
    for (int i = 0; i < NU; ++i) kf[i] = r[i];
    chol_solve(NU, Rm, kf);
    for (int i = 0; i < NU; ++i) kf[i] = -kf[i];
    {   /* P = [I;K]^T Hh [I;K] + Ab^T P1 Ab (sum of PSD terms), Ab = A + B K */
        double PB1[NX];
        for (int a = 0; a < NX; ++a)
            for (int b = 0; b < NX; ++b) {
                double s = S->A[a][b];
                for (int i = 0; i < NU; ++i) s += S->Bm[a][i] * Kk[i * NX + b];
                Ab[a * NX + b] = s;
            }
        double xb[NX];  /* B kf + c */
        for (int a = 0; a < NX; ++a) {
            double s = S->c[a];
            for (int i = 0; i < NU; ++i) s += S->Bm[a][i] * kf[i];
            xb[a] = s;
        }
        for (int a = 0; a < NX; ++a) {
            double s = p1[a];
            for (int l = 0; l < NX; ++l) s += P1[a * NX + l] * xb[l];
            PB1[a] = s;
        }
        double PAb[NX * NX];
        for (int a = 0; a < NX; ++a)
            for (int b = 0; b < NX; ++b) {
                double s = 0.0;
                for (int l = 0; l < NX; ++l) s += P1[a * NX + l] * Ab[l * NX + b];
                PAb[a * NX + b] = s;
            }
        double KR[NX * NU];  /* S0^T + K^T R0 : [NX][NU] */
        for (int a = 0; a < NX; ++a)
            for (int j = 0; j < NU; ++j) {
                double s = S0[j * NX + a];
                for (int i = 0; i < NU; ++i) s += Kk[i * NX + a] * R0[i * NU + j];
                KR[a * NU + j] = s;
            }
        for (int a = 0; a < NX; ++a) {
            for (int b = 0; b < NX; ++b) {
                double s = Qx[a * NX + b];
                for (int l = 0; l < NX; ++l) s += Ab[l * NX + a] * PAb[l * NX + b];
                for (int j = 0; j < NU; ++j) s += KR[a * NU + j] * Kk[j * NX + b] + Kk[j * NX + a] * S0[j * NX + b];
                Pk[a * NX + b] = s;
            }
            double s = qx[a];
            for (int i = 0; i < NU; ++i) s += Kk[i * NX + a] * ru[i] + KR[a * NU + i] * kf[i];
            for (int l = 0; l < NX; ++l) s += Ab[l * NX + a] * PB1[l];
            pk[a] = s;
        }
    }
    return 0;
}

/* slacks of node k from the eliminated rows at the state xk */
static void node_slacks(const ipm_t* Q, int k, const double* sig, const double* v, const double* xk, double* sl,
                        double* su) {
    const int N = Q->N;
    const qp_opts_c* o = Q->o;
    const stage_t* S = &Q->st[k];
    (void)o;
    for (int j = 0; j < S->nsoft; ++j) {
        const int e = grp(Q, k, j), r0 = 8 * N + 4 * e;
        const double Zs = S->s * S->Zl[j], zs = S->s * S->zl[j];
        const double Hl = Zs + sig[r0] + sig[r0 + 2], Hu = Zs + sig[r0 + 1] + sig[r0 + 3];
        const double gl = zs - v[r0] - v[r0 + 2], gu = zs - v[r0 + 1] - v[r0 + 3];
        double cx = 0.0;
        for (int l = 0; l < NX; ++l) cx += S->C[j][l] * xk[l];
        sl[e] = -(gl + sig[r0] * cx) / Hl;
        su[e] = -(gu - sig[r0 + 1] * cx) / Hu;
    }
}

/* u_k = K x_k + kf - G lam,  x_{k+1} = A x_k + B u_k + c  (G = NULL: no terminal multiplier) */
static void fwd_stage(const ipm_t* Q, int k, const double* Kk, const double* kf, const double* G, const double* lam,
                      const double* xk, double* uk, double* xn) {
    const stage_t* S = &Q->st[k];
    for (int i = 0; i < NU; ++i) {
        double s = kf[i];
        for (int l = 0; l < NX; ++l) s += Kk[i * NX + l] * xk[l];
        if (G)
            for (int l = 0; l < NX; ++l) s -= G[i * NX + l] * lam[l];
        uk[i] = s;
    }
    for (int a = 0; a < NX; ++a) {
        double s = S->c[a];
        for (int l = 0; l < NX; ++l) s += S->A[a][l] * xk[l];
        for (int i = 0; i < NU; ++i) s += S->Bm[a][i] * uk[i];
        xn[a] = s;
    }
}

/* The Newton system as an LQR in the new iterate: Hessian H + D^T diag(sig) D, gradient g - D^T v.
 * Soft slacks are eliminated per row pair (a rank-3 fold on the node's state block), box terms land
 * on the input block.  Writes the solution (dx, du, sl, su); returns nonzero on a failed factorisation. */
static int lqr(ipm_t* Q, const double* sig, const double* v, double* dx, double* du, double* sl, double* su) {
    const int N = Q->N;
    for (int k = N; k >= 0; --k) {
        double Qx[NX * NX], qx[NX], R0[NU * NU], S0[NU * NX], ru[NU], bd[NU], Rc[NU * NU], Ab[NX * NX];
        stage_terms(Q, k, sig, v, Qx, qx, R0, S0, ru, bd);
        double* Pk = Q->P + (size_t)k * NX * NX;
        double* pk = Q->p + (size_t)k * NX;
        if (k == N) {
            memcpy(Pk, Qx, sizeof Qx);
            memcpy(pk, qx, sizeof qx);
            continue;
        }
        if (ric_stage(Q, k, Qx, qx, R0, S0, ru, bd, Pk + NX * NX, pk + NX, Pk, pk, Q->K + (size_t)k * NU * NX,
                      Q->kf + (size_t)k * NU, Ab, Rc))
            return 1;
    }
    /* forward: dx_0 fixed, du = K dx + k_ff, dx+ = A dx + B du + c; slacks from the eliminated rows */
    memcpy(dx, Q->x0, sizeof(double) * NX);
    for (int k = 0; k <= N; ++k) {
        node_slacks(Q, k, sig, v, dx + (size_t)k * NX, sl, su);
        if (k == N) break;
        fwd_stage(Q, k, Q->K + (size_t)k * NU * NX, Q->kf + (size_t)k * NU, NULL, NULL, dx + (size_t)k * NX,
                  du + (size_t)k * NU, dx + (size_t)(k + 1) * NX);
    }
    return 0;
}

/* ---- partitioned (parallel-in-time) Riccati: the scheme of csrc/rti_qp_seg.hip, in its order of
 * operations.  The nodes split into P segments [a_i, a_{i+1}) (a_i = i (N+1) / P; the last one holds the
 * terminal node).  Every segment i < P-1 runs the backward recursion with a zero cost-to-go at its end
 * b = a_{i+1} and carries, besides its factors, the element (J, eta, Phi, beta, C) of its conditional value
 * function (the Riccati form of the parallel LQ element of Sarkka & Garcia-Fernandez):
 *     x_b = Phi x_a + beta - C lam_b,    lam_a = J x_a + eta + Phi^T lam_b,
 * Phi the product of the closed-loop matrices A~, beta the closed-loop offsets, C the sum of
 * Z_k R^_k^-1 Z_k^T over Z_k = Phi_{k+1->b} B_k, and lam_b = P_b x_b + p_b the costate at b.  With the true
 * cost-to-go, the input of node k is u_k = K_k x_k + kf_k - G_k lam_b, G_k = R^_k^-1 Z_k^T.
 * Coupling, serial over the segments: P_b = L L^T, S = I + L^T C L = U U^T, V = L U^-T (so Y = V V^T =
 * (I + P_b C)^-1 P_b), X = V^T Phi,  z = V^T beta + U^-1 L^-1 p_b,
 *     P_a = J + X^T X,   p_a = eta + X^T z              (sums of PSD terms)
 *     lam_b = Lam x_a + lam0,  Lam = V X, lam0 = V z    (the costate offset by triangular solves)
 *     x_b   = M x_a + m,       M = Phi - C Lam, m = beta - C lam0
 * Measured on the C3 bench problem (tools/ipm_sweep.py, 4 seeds x 3 RTI steps x 256 instances):
 * identical iteration counts to the serial recursion at P = 4 and 8.  Forming lam0 as Y (beta - C p_b)
 * + p_b instead (cancellation of p_b against Y C p_b when C P_b is large) took the worst case from 13 to
 * 34 (P = 4) / 100 iterations (P = 8); an explicit W = V U^-1 L^-1 for the p_b term to 15 / 24. */
static int seg_a(int N, int P, int i) { return i * (N + 1) / P; }

static void lsolve(const double* L, double* x) {  /* x <- L^-1 x (L lower) */
    for (int i = 0; i < NX; ++i) {
        double v = x[i];
        for (int k = 0; k < i; ++k) v -= L[i * NX + k] * x[k];
        x[i] = v / L[i * NX + i];
    }
}

typedef struct {  /* a segment's element and coupling matrices */
    double Phi[NX * NX], C[NX * NX], beta[NX], L[NX * NX], U[NX * NX], V[NX * NX], X[NX * NX];
    double Lam[NX * NX], M[NX * NX];
} seg_t;

/* the vector part of a coupling: z = V^T beta + U^-1 L^-1 p_b (into z), lam0 = V z, m = beta - C lam0 */
static void seg_vec(const seg_t* e, const double* pb, double* z, double* lam0, double* m) {
    double q[NX];
    memcpy(q, pb, sizeof q);
    lsolve(e->L, q);
    lsolve(e->U, q);
    for (int r = 0; r < NX; ++r) {
        double s = 0.0;
        for (int k = 0; k < NX; ++k) s += e->V[k * NX + r] * e->beta[k];
        z[r] = s + q[r];
    }
    for (int r = 0; r < NX; ++r) {
        double s = 0.0;
        for (int k = 0; k < NX; ++k) s += e->V[r * NX + k] * z[k];
        lam0[r] = s;
    }
    for (int r = 0; r < NX; ++r) {
        double s = 0.0;
        for (int k = 0; k < NX; ++k) s += e->C[r * NX + k] * lam0[k];
        m[r] = e->beta[r] - s;
    }
}

static void matmul(const double* A, int ta, const double* B, double* D) {  /* D = op(A) B, op = A^T if ta */
    for (int r = 0; r < NX; ++r)
        for (int c = 0; c < NX; ++c) {
            double s = 0.0;
            for (int k = 0; k < NX; ++k) s += (ta ? A[k * NX + r] : A[r * NX + k]) * B[k * NX + c];
            D[r * NX + c] = s;
        }
}

static int lqr_seg(ipm_t* Q, int P, const double* sig, const double* v, double* dx, double* du, double* sl, double* su) {
    const int N = Q->N;
    seg_t sg[16];
    if (P > 16) P = 16;
    if (P > N) P = N > 0 ? N : 1;
    static const double zP[NX * NX], zp[NX];
    for (int i = P - 1; i >= 0; --i) {  /* pass 1, every segment on its own */
        const int a = seg_a(N, P, i), b = seg_a(N, P, i + 1);
        seg_t* e = &sg[i];
        memset(e, 0, sizeof *e);
        for (int l = 0; l < NX; ++l) e->Phi[l * NX + l] = 1.0;
        for (int k = (i == P - 1 ? N : b - 1); k >= a; --k) {
            double Qx[NX * NX], qx[NX], R0[NU * NU], S0[NU * NX], ru[NU], bd[NU], Rc[NU * NU], Ab[NX * NX];
            stage_terms(Q, k, sig, v, Qx, qx, R0, S0, ru, bd);
            double* Pk = Q->P + (size_t)k * NX * NX;
            double* pk = Q->p + (size_t)k * NX;
            if (k == N) {
                memcpy(Pk, Qx, sizeof Qx);
                memcpy(pk, qx, sizeof qx);
                continue;
            }
            const int end = (i < P - 1 && k == b - 1);
            double* Kk = Q->K + (size_t)k * NU * NX;
            double* kf = Q->kf + (size_t)k * NU;
            if (ric_stage(Q, k, Qx, qx, R0, S0, ru, bd, end ? zP : Pk + NX * NX, end ? zp : pk + NX, Pk, pk, Kk, kf, Ab, Rc))
                return 1;
            if (i == P - 1) continue;
            const stage_t* S = &Q->st[k];
            double Z[NX * NU], *G = Q->G + (size_t)k * NU * NX, t[NX], Pn[NX * NX];
            for (int l = 0; l < NX; ++l) {  /* Z = Phi B, G = R^-1 Z^T, C += Z G */
                for (int j = 0; j < NU; ++j) {
                    double s = 0.0;
                    for (int q = 0; q < NX; ++q) s += e->Phi[l * NX + q] * S->Bm[q][j];
                    Z[l * NU + j] = s;
                }
                double col[NU];
                for (int j = 0; j < NU; ++j) col[j] = Z[l * NU + j];
                chol_solve(NU, Rc, col);
                for (int j = 0; j < NU; ++j) G[j * NX + l] = col[j];
            }
            for (int l = 0; l < NX; ++l)
                for (int q = 0; q < NX; ++q) {
                    double s = 0.0;
                    for (int j = 0; j < NU; ++j) s += Z[l * NU + j] * G[j * NX + q];
                    e->C[l * NX + q] += s;
                }
            for (int l = 0; l < NX; ++l) {  /* closed-loop offset c + B kf */
                double s = S->c[l];
                for (int j = 0; j < NU; ++j) s += S->Bm[l][j] * kf[j];
                t[l] = s;
            }
            for (int l = 0; l < NX; ++l) {  /* [Phi | beta] <- [Phi A~ | Phi b~ + beta] */
                double s = 0.0;
                for (int q = 0; q < NX; ++q) s += e->Phi[l * NX + q] * t[q];
                e->beta[l] += s;
                for (int q = 0; q < NX; ++q) {
                    double s2 = 0.0;
                    for (int r = 0; r < NX; ++r) s2 += e->Phi[l * NX + r] * Ab[r * NX + q];
                    Pn[l * NX + q] = s2;
                }
            }
            memcpy(e->Phi, Pn, sizeof Pn);
        }
    }
    double lam0[16][NX], mv[16][NX];
    for (int i = P - 2; i >= 0; --i) {  /* coupling, backward: the true cost-to-go at every a_i */
        const int a = seg_a(N, P, i), b = seg_a(N, P, i + 1);
        seg_t* e = &sg[i];
        const double* Pb = Q->P + (size_t)b * NX * NX;
        const double* pb = Q->p + (size_t)b * NX;
        memcpy(e->L, Pb, sizeof e->L);
        if (chol(NX, e->L)) return 1;
        for (int r = 0; r < NX; ++r)
            for (int c = r + 1; c < NX; ++c) e->L[r * NX + c] = 0.0;
        double T[NX * NX];
        matmul(e->C, 0, e->L, T);       /* T = C L */
        matmul(e->L, 1, T, e->U);       /* S = I + L^T T */
        for (int r = 0; r < NX; ++r) e->U[r * NX + r] += 1.0;
        if (chol(NX, e->U)) return 1;
        for (int r = 0; r < NX; ++r)
            for (int c = r + 1; c < NX; ++c) e->U[r * NX + c] = 0.0;
        for (int r = 0; r < NX; ++r) {  /* row r of V = L U^-T: (U^-1 (row r of L)^T)^T */
            double row[NX];
            for (int c = 0; c < NX; ++c) row[c] = e->L[r * NX + c];
            lsolve(e->U, row);
            for (int c = 0; c < NX; ++c) e->V[r * NX + c] = row[c];
        }
        matmul(e->V, 1, e->Phi, e->X);  /* X = V^T Phi */
        double z[NX];
        seg_vec(e, pb, z, lam0[i], mv[i]);
        matmul(e->V, 0, e->X, e->Lam);  /* Lam = V X */
        matmul(e->C, 0, e->Lam, T);     /* M = Phi - C Lam */
        for (int r = 0; r < NX * NX; ++r) e->M[r] = e->Phi[r] - T[r];
        if (i == 0) continue;  /* x_0 is fixed: the cost-to-go at node 0 is never used */
        double* Pa = Q->P + (size_t)a * NX * NX;
        double* pa = Q->p + (size_t)a * NX;
        for (int r = 0; r < NX; ++r) {
            for (int c = 0; c < NX; ++c) {
                double s = 0.0;
                for (int q = 0; q < NX; ++q) s += e->X[q * NX + r] * e->X[q * NX + c];
                Pa[r * NX + c] += s;
            }
            double s = 0.0;
            for (int q = 0; q < NX; ++q) s += e->X[q * NX + r] * z[q];
            pa[r] += s;
        }
    }
    /* forward: boundary states by the coupling, then every segment on its own */
    memcpy(dx, Q->x0, sizeof(double) * NX);
    for (int i = 0; i < P; ++i) {
        const int a = seg_a(N, P, i), b = seg_a(N, P, i + 1);
        const seg_t* e = &sg[i];
        double lam[NX], xb[NX];
        const double* xa = dx + (size_t)a * NX;
        if (i < P - 1)
            for (int r = 0; r < NX; ++r) {
                double sx = mv[i][r], sl2 = lam0[i][r];
                for (int c = 0; c < NX; ++c) {
                    sx += e->M[r * NX + c] * xa[c];
                    sl2 += e->Lam[r * NX + c] * xa[c];
                }
                xb[r] = sx;
                lam[r] = sl2;
            }
        for (int k = a; k < b; ++k) {
            node_slacks(Q, k, sig, v, dx + (size_t)k * NX, sl, su);
            if (k == N) break;
            double xn[NX];
            fwd_stage(Q, k, Q->K + (size_t)k * NU * NX, Q->kf + (size_t)k * NU, i < P - 1 ? Q->G + (size_t)k * NU * NX : NULL,
                      lam, dx + (size_t)k * NX, du + (size_t)k * NU, k + 1 == b ? xn : dx + (size_t)(k + 1) * NX);
            if (k + 1 == b) {
                double d = 0.0;
                for (int r = 0; r < NX; ++r) d = fmax(d, fabs(xn[r] - xb[r]) / (1.0 + fabs(xb[r])));
                if (d > Q->seg_dev) Q->seg_dev = d;
                memcpy(dx + (size_t)b * NX, xb, sizeof xb);
            }
        }
    }
    return 0;
}

static double step_max(int m, const double* t, const double* l, const double* dt, const double* dl) {
    double a = 1.0;
    for (int r = 0; r < m; ++r) {
        if (dt[r] < 0.0 && -t[r] / dt[r] < a) a = -t[r] / dt[r];
        if (dl[r] < 0.0 && -l[r] / dl[r] < a) a = -l[r] / dl[r];
    }
    return a;
}

/* diagnostic trace (tools/ipm_trace.py; single instance, one thread): per iteration
 * [alpha_aff, alpha, mu, max t*lambda, rp, sigma*mu, the row of the max product, its t, its lambda] */
#define TRACE_W 9
static double* g_trace = NULL;
static int g_trace_max = 0;
void orc_qp_trace(double* buf, int max_rows) { g_trace = buf; g_trace_max = buf ? max_rows : 0; }

/* One instance.  Returns IPM iterations (status via *conv: 1 converged). */
static int solve_one(int N, const double* xn, const double* AB, const double* y, const double* Jy, const double* yN,
                     const double* JyN, const double* h, const double* Jh, const double* hE, const double* JhE,
                     const double* x, const double* u,
                     const double* x0, const double* yref, const double* W, const double* yNref, const double* WN,
                     const double* dtv, const qp_opts_c* o, int ny, double* dx, double* du, double* slack, int* conv,
                     double* res) {
    const int N1 = N + 1, nsl = N * (o->nh - o->nhs) + o->nsN;
    const int m = 8 * N + 4 * nsl + 2 * ((N - 1) * o->nhs + o->nhN - o->nsN);
    ipm_t Q;
    Q.N = N; Q.m = m; Q.o = o; Q.ns = o->nh - o->nhs; Q.nhs = o->nhs; Q.rh0 = 8 * N + 4 * nsl;
    Q.st = (stage_t*)calloc((size_t)N1, sizeof(stage_t));
    Q.P = (double*)malloc(sizeof(double) * (size_t)N1 * NX * NX);
    Q.p = (double*)malloc(sizeof(double) * (size_t)N1 * NX);
    Q.K = (double*)malloc(sizeof(double) * (size_t)N * NU * NX);
    Q.kf = (double*)malloc(sizeof(double) * (size_t)N * NU);
    Q.G = (double*)calloc((size_t)N * NU * NX, sizeof(double));
    Q.nseg = o->nseg;
    Q.seg_dev = 0.0;
    Q.gcount = 0;
    double* buf = (double*)calloc((size_t)(16 * m + 5 * (N1 * NX + N * NU + 2 * N1 * NS)), sizeof(double));
    double *t = buf, *lam = t + m, *sig = lam + m, *v = sig + m, *rv = v + m, *dta = rv + m, *dla = dta + m;
    double *dtc = dla + m, *dlc = dtc + m, *rw = dlc + m;  /* rw: spare */
    (void)rw;
    double* zs = buf + 12 * m;  /* 5 z-vectors, then dtg, dlg, gcum (3 m) */
    const int nz = N1 * NX + N * NU + 2 * N1 * NS;
    double *zdx = zs, *zdu = zdx + N1 * NX, *zsl = zdu + N * NU, *zsu = zsl + N1 * NS;          /* iterate */
    double *adx = zs + nz, *adu = adx + N1 * NX, *asl = adu + N * NU, *asu = asl + N1 * NS;     /* affine */
    double *cdx = zs + 2 * nz, *cdu = cdx + N1 * NX, *csl = cdu + N * NU, *csu = csl + N1 * NS; /* corrector */
    double* gz = zs + 4 * nz;                                                                   /* Gondzio */
    double *gdx = gz, *gdu = gdx + N1 * NX, *gsl = gdu + N * NU, *gsu = gsl + N1 * NS;
    double *dtg = zs + 5 * nz, *dlg = dtg + m, *gcum = dlg + m;

    /* ---- stage data (the pack step of rti_qp.hip) */
    for (int k = 0; k <= N; ++k) {
        stage_t* S = &Q.st[k];
        S->s = (o->cost_scaling && k < N) ? dtv[k] : 1.0;
        if (k < N) {  /* stage rows: columns h_col of h / J_h */
            S->nsoft = o->nh - o->nhs;
            S->nrow = k > 0 ? o->nh : S->nsoft;  /* node 0: no hard row (hgrp) */
            for (int j = 0; j < o->nh; ++j) {
                const int c = o->h_col[j];
                for (int l = 0; l < NX; ++l) S->C[j][l] = Jh[((size_t)k * NX + l) * NS + c];
                S->hl[j] = h[(size_t)k * NS + c] - o->lh[j];
                S->hu[j] = o->uh[j] - h[(size_t)k * NS + c];
                S->zl[j] = o->zl[j];
                S->Zl[j] = o->Zl[j];
            }
        } else {  /* terminal rows: sums of an h[N] column and an hE column */
            S->nsoft = o->nsN;
            S->nrow = o->nhN;
            for (int j = 0; j < o->nhN; ++j) {
                const int c1 = o->hN_col[j], c2 = o->hE_col[j];
                double hv = 0.0;
                for (int l = 0; l < NX; ++l) S->C[j][l] = 0.0;
                if (c1 >= 0) {
                    hv += h[(size_t)k * NS + c1];
                    for (int l = 0; l < NX; ++l) S->C[j][l] += Jh[((size_t)k * NX + l) * NS + c1];
                }
                if (c2 >= 0) {
                    hv += hE[c2];
                    for (int l = 0; l < NX; ++l) S->C[j][l] += JhE[l * 6 + c2];
                }
                S->hl[j] = hv - o->lhN[j];
                S->hu[j] = o->uhN[j] - hv;
                S->zl[j] = j < o->nsN ? o->zlN[j] : 0.0;
                S->Zl[j] = j < o->nsN ? o->ZlN[j] : 0.0;
            }
        }
        if (k < N) {
            const double* ab = AB + (size_t)k * NW * NX;
            for (int i = 0; i < NX; ++i) {
                for (int j = 0; j < NX; ++j) S->A[i][j] = ab[j * NX + i];
                for (int j = 0; j < NU; ++j) S->Bm[i][j] = ab[(NX + j) * NX + i];
                S->c[i] = xn[(size_t)k * NX + i] - x[(size_t)(k + 1) * NX + i];
            }
            double J[NW][12], Ws[12], r[12];  /* J_y as [w][residual]; with ny = 12 the sdf cost row */
            for (int i = 0; i < NW; ++i)
                for (int a = 0; a < 11; ++a) J[i][a] = Jy[((size_t)k * NW + i) * 11 + a];
            for (int a = 0; a < ny; ++a) {
                Ws[a] = S->s * W[(size_t)k * ny + a];
                r[a] = (a < 11 ? y[(size_t)k * 11 + a] : 0.0) - yref[(size_t)k * ny + a];
            }
            if (ny == 12) {  /* flags.sdf_cost (gen_model.py:65-66): (1 - s/2)^4 of s = h[2] */
                const double tq = 1.0 - 0.5 * h[(size_t)k * NS + 2];
                r[11] += tq * tq * tq * tq;
                for (int i = 0; i < NW; ++i) J[i][11] = i < NX ? -2.0 * tq * tq * tq * Jh[((size_t)k * NX + i) * NS + 2] : 0.0;
            }
            for (int i = 0; i < NW; ++i) {
                double gs = 0.0;
                for (int a = 0; a < ny; ++a) gs += J[i][a] * Ws[a] * r[a];
                S->g[i] = gs;
                for (int j = 0; j < NW; ++j) {
                    double hs = 0.0;
                    for (int a = 0; a < ny; ++a) hs += J[i][a] * Ws[a] * J[j][a];
                    S->H[i][j] = hs + (i == j ? (o->lm_scaling ? o->lm * dtv[k] : o->lm) : 0.0);
                }
            }
            for (int i = 0; i < NU; ++i) {
                S->dlo[i] = u[(size_t)k * NU + i] - o->lbu[i];
                S->dup[i] = o->ubu[i] - u[(size_t)k * NU + i];
            }
        } else {
            for (int i = 0; i < NX; ++i) {
                double gs = 0.0;
                for (int a = 0; a < o->nyN; ++a) gs += JyN[i * o->nyN + a] * WN[a] * (yN[a] - yNref[a]);
                S->g[i] = gs;
                for (int j = 0; j < NX; ++j) {
                    double hs = 0.0;
                    for (int a = 0; a < o->nyN; ++a) hs += JyN[i * o->nyN + a] * WN[a] * JyN[j * o->nyN + a];
                    S->H[i][j] = hs + (i == j ? o->lm : 0.0);
                }
            }
        }
    }
    for (int i = 0; i < NX; ++i) Q.x0[i] = x0[i] - x[i];

    /* ---- starting point (rti_qp.hip's): dynamics-feasible with du = sl = su = 0 (o->ws: du = the du
     * buffer's entry values, if all finite); t = max(row, t0); lambda = l0 on box rows, max(l0, lc s_k zl_j) on the rows
     * of soft group (k, j) */
    memcpy(zdx, Q.x0, sizeof(double) * NX);
    if (o->ws) {
        /* a du with a non-finite entry (the output of a failed QP) gives a cold start: a failure must not
         * stick to the instance through the warm start */
        int fin = 1;
        for (int e = 0; e < N * NU; ++e) fin &= isfinite(du[e]) != 0;
        if (fin) memcpy(zdu, du, sizeof(double) * N * NU);
    }
    for (int k = 0; k < N; ++k)
        for (int a = 0; a < NX; ++a) {
            double s = Q.st[k].c[a];
            for (int l = 0; l < NX; ++l) s += Q.st[k].A[a][l] * zdx[k * NX + l];
            for (int j = 0; j < NU; ++j) s += Q.st[k].Bm[a][j] * zdu[k * NU + j];
            zdx[(k + 1) * NX + a] = s;
        }
    rows_at(&Q, zdx, zdu, zsl, zsu, rv);
    double rp = 0.0, mu = 0.0, cm = 0.0;  /* mean / max complementarity; stop on max (HPIPM's res_m) */
    for (int r = 0; r < m; ++r) {
        t[r] = rv[r] > o->t0 ? rv[r] : o->t0;
        lam[r] = o->l0;
        if (r >= 8 * N && r < Q.rh0) {  /* soft group e's rows (hard rows start at l0) */
            const int e = (r - 8 * N) >> 2, k = (Q.ns > 0 && e < N * Q.ns) ? e / Q.ns : N, j = e - grp(&Q, k, 0);
            const double lj = o->lc * Q.st[k].s * Q.st[k].zl[j];
            if (lj > lam[r]) lam[r] = lj;
        }
        if (fabs(rv[r] - t[r]) > rp) rp = fabs(rv[r] - t[r]);
        mu += t[r] * lam[r];
        if (t[r] * lam[r] > cm) cm = t[r] * lam[r];
    }
    mu /= m;
    /* row constants d (rows at z = 0) for v = sig (t - d) */
    double* d0 = (double*)calloc((size_t)m, sizeof(double));
    {
        double* zero = (double*)calloc((size_t)nz, sizeof(double));
        rows_at(&Q, zero, zero + N1 * NX, zero + N1 * NX + N * NU, zero + N1 * NX + N * NU + N1 * NS, d0);  /* sl, su: nsl <= N1 NS */
        free(zero);
    }
    int it = 0, fail = 0;
    double gap = 1.0;  /* prod (1 - alpha): the decay of the stationarity residual of the start point */
    while (!(cm < o->tol && rp < o->tol && gap < o->tol) && it < o->max_iter && isfinite(mu + rp)) {
        /* predictor */
        for (int r = 0; r < m; ++r) {
            sig[r] = lam[r] / t[r];
            v[r] = sig[r] * (t[r] - d0[r]);
        }
        if (Q.nseg > 1 ? lqr_seg(&Q, Q.nseg, sig, v, adx, adu, asl, asu) : lqr(&Q, sig, v, adx, adu, asl, asu)) { fail = 1; break; }
        rows_at(&Q, adx, adu, asl, asu, rv);
        for (int r = 0; r < m; ++r) {
            dta[r] = rv[r] - t[r];
            dla[r] = -sig[r] * dta[r] - lam[r];
        }
        const double aa = step_max(m, t, lam, dta, dla);
        double mua = 0.0;
        for (int r = 0; r < m; ++r) mua += (t[r] + aa * dta[r]) * (lam[r] + aa * dla[r]);
        mua /= m;
        /* Mehrotra's centring target, floored at 1e-2 tol (HPIPM's tau_min): rows are never pushed below
         * the complementarity the stop test needs, which keeps lambda / t -- and the Riccati data -- bounded */
        double sigmu = (mua / mu) * (mua / mu) * (mua / mu) * mu;
        if (sigmu < 1e-2 * o->tol) sigmu = 1e-2 * o->tol;
        /* corrector */
        for (int r = 0; r < m; ++r) v[r] = sig[r] * (t[r] - d0[r]) - (dta[r] * dla[r] - sigmu) / t[r];
        if (Q.nseg > 1 ? lqr_seg(&Q, Q.nseg, sig, v, cdx, cdu, csl, csu) : lqr(&Q, sig, v, cdx, cdu, csl, csu)) { fail = 1; break; }
        rows_at(&Q, cdx, cdu, csl, csu, rv);
        for (int r = 0; r < m; ++r) {
            dtc[r] = rv[r] - t[r];
            dlc[r] = -sig[r] * dtc[r] - lam[r] - (dta[r] * dla[r] - sigmu) / t[r];
        }
        double tau = 1.0 - mu;  /* step fraction min(tau_hi, max(tau_lo, 1 - mu)) */
        if (tau < o->tau_lo) tau = o->tau_lo;
        if (tau > o->tau_hi) tau = o->tau_hi;
        double amax = step_max(m, t, lam, dtc, dlc);
        for (int gi = 0; gi < o->gk && amax < o->ga; ++gi) {  /* Gondzio correctors */
            double at = amax + o->gd;
            if (at > 1.0) at = 1.0;
            const double lo = o->gbmin * sigmu, hi = o->gbmax * sigmu;
            for (int r = 0; r < m; ++r) {
                const double pv = (t[r] + at * dtc[r]) * (lam[r] + at * dlc[r]);
                double c = 0.0;
                if (pv < lo) c = lo - pv;
                else if (pv > hi) c = (hi - pv) > -hi ? hi - pv : -hi;
                rw[r] = c;  /* extra complementarity right-hand side */
                v[r] = sig[r] * (t[r] - d0[r]) - (dta[r] * dla[r] - sigmu - rw[r] - gcum[r]) / t[r];
            }
            if (Q.nseg > 1 ? lqr_seg(&Q, Q.nseg, sig, v, gdx, gdu, gsl, gsu) : lqr(&Q, sig, v, gdx, gdu, gsl, gsu)) { fail = 1; break; }
            rows_at(&Q, gdx, gdu, gsl, gsu, rv);
            for (int r = 0; r < m; ++r) {
                dtg[r] = rv[r] - t[r];
                dlg[r] = -sig[r] * dtg[r] - lam[r] - (dta[r] * dla[r] - sigmu - rw[r] - gcum[r]) / t[r];
            }
            const double an = step_max(m, t, lam, dtg, dlg);
            if (an < amax + 0.1 * o->gd) break;
            amax = an;
            for (int r = 0; r < m; ++r) { dtc[r] = dtg[r]; dlc[r] = dlg[r]; gcum[r] += rw[r]; }
            memcpy(zs + 2 * nz, gz, sizeof(double) * nz);
            Q.gcount++;
        }
        if (fail) break;
        for (int r = 0; r < m; ++r) gcum[r] = 0.0;
        double al = tau * amax;
        if (al > 1.0) al = 1.0;
        mu = 0.0;
        cm = 0.0;
        for (int r = 0; r < m; ++r) {
            t[r] += al * dtc[r];
            lam[r] += al * dlc[r];
            mu += t[r] * lam[r];
            if (t[r] * lam[r] > cm) cm = t[r] * lam[r];
        }
        mu /= m;
        for (int e = 0; e < nz; ++e) zs[e] += al * (zs[2 * nz + e] - zs[e]);
        rp *= (1.0 - al);
        gap *= (1.0 - al);
        if (g_trace && it < g_trace_max) {
            double* tr = g_trace + (size_t)it * TRACE_W;
            int rm = 0;
            for (int r = 1; r < m; ++r)
                if (t[r] * lam[r] > t[rm] * lam[rm]) rm = r;
            tr[0] = aa + 10.0 * Q.gcount; tr[1] = al; tr[2] = mu; tr[3] = cm; tr[4] = rp; tr[5] = sigmu; tr[6] = rm; tr[7] = t[rm]; tr[8] = lam[rm];
        }
        ++it;

    }
    memcpy(dx, zdx, sizeof(double) * N1 * NX);
    memcpy(du, zdu, sizeof(double) * N * NU);
    if (slack)  /* [N+1][3][2] by (node, row) */
        for (int k = 0; k <= N; ++k)
            for (int j = 0; j < NS; ++j) {
                const int live = j < Q.st[k].nsoft, e = live ? grp(&Q, k, j) : 0;
                slack[(k * NS + j) * 2] = live ? zsl[e] : 0.0;
                slack[(k * NS + j) * 2 + 1] = live ? zsu[e] : 0.0;
            }
    if (!isfinite(mu + rp)) fail = 1;
    *conv = fail ? -1 : (cm < o->tol && rp < o->tol && gap < o->tol);
    if (res) { res[0] = cm; res[1] = rp; res[2] = Q.seg_dev; res[3] = Q.gcount; }
    free(d0); free(buf); free(Q.st); free(Q.P); free(Q.p); free(Q.K); free(Q.kf); free(Q.G);
    return it;
}

/* Batched entry point (OpenMP over instances).  opts: lbu 4, ubu 4, lh 3, uh 3, zl 3, Zl 3, lm, tol,
 * lm_scaling, then the IPM start / step parameters t0, l0, lc, tau_lo, tau_hi, nseg, the Gondzio options,
 * ws, and from opts[35] the constraint set (see the body).  status (rti_qp.hip's convention): 0 converged, 1 max_iter, 2 numerical failure. */
void orc_qp_ipm_batch(int B, int N, const double* xn, const double* AB, const double* y, const double* Jy,
                      const double* yN, const double* JyN, const double* h, const double* Jh, const double* hE,
                      const double* JhE, const double* x,
                      const double* u, const double* x0, const double* yref, const double* W, const double* yNref,
                      const double* WN, const double* dt, const double* opts, int max_iter, int cost_scaling, int ny,
                      double* dx, double* du, double* slack, int* iters, int* status, double* res, int nthreads) {
    qp_opts_c o;
    memcpy(o.lbu, opts, 4 * sizeof(double));
    memcpy(o.ubu, opts + 4, 4 * sizeof(double));
    memcpy(o.lh, opts + 8, 3 * sizeof(double));
    memcpy(o.uh, opts + 11, 3 * sizeof(double));
    memcpy(o.zl, opts + 14, 3 * sizeof(double));
    memcpy(o.Zl, opts + 17, 3 * sizeof(double));
    o.lm = opts[20];
    o.tol = opts[21];
    o.lm_scaling = opts[22] != 0.0;
    o.t0 = opts[23]; o.l0 = opts[24]; o.lc = opts[25]; o.tau_lo = opts[26]; o.tau_hi = opts[27];
    o.nseg = (int)opts[28];
    o.gk = (int)opts[29]; o.ga = opts[30]; o.gd = opts[31]; o.gbmin = opts[32]; o.gbmax = opts[33];
    o.ws = opts[34] != 0.0;
    /* the constraint set: opts[35 ..] = nh, h_col 3, nhN, nsN, hN_col 8, hE_col 8, lhN 8, uhN 8, zlN 3, ZlN 3, nyN,
     * nhs */
    const double* cs = opts + 35;
    o.nh = (int)cs[0];
    for (int j = 0; j < 3; ++j) o.h_col[j] = (int)cs[1 + j];
    o.nhN = (int)cs[4];
    o.nsN = (int)cs[5];
    for (int j = 0; j < NR; ++j) {
        o.hN_col[j] = (int)cs[6 + j];
        o.hE_col[j] = (int)cs[14 + j];
        o.lhN[j] = cs[22 + j];
        o.uhN[j] = cs[30 + j];
    }
    for (int j = 0; j < 3; ++j) { o.zlN[j] = cs[38 + j]; o.ZlN[j] = cs[41 + j]; }
    o.nyN = (int)cs[44];
    o.nhs = (int)cs[45];
    o.max_iter = max_iter;
    o.cost_scaling = cost_scaling;
    const int N1 = N + 1;
#pragma omp parallel for schedule(dynamic) num_threads(nthreads > 0 ? nthreads : 1)
    for (int b = 0; b < B; ++b) {
        int conv = 0;
        const int nyN = o.nyN;
        iters[b] = solve_one(N, xn + (size_t)b * N * NX, AB + (size_t)b * N * NW * NX, y + (size_t)b * N * 11,
                             Jy + (size_t)b * N * NW * 11, yN + (size_t)b * nyN, JyN + (size_t)b * 10 * nyN,
                             h + (size_t)b * N1 * NS, Jh + (size_t)b * N1 * NX * NS, hE ? hE + (size_t)b * 6 : NULL,
                             JhE ? JhE + (size_t)b * 60 : NULL, x + (size_t)b * N1 * NX,
                             u + (size_t)b * N * NU, x0 + (size_t)b * NX, yref + (size_t)b * N * ny,
                             W + (size_t)b * N * ny, yNref + (size_t)b * nyN, WN + (size_t)b * nyN, dt, &o, ny,
                             dx + (size_t)b * N1 * NX, du + (size_t)b * N * NU,
                             slack ? slack + (size_t)b * N1 * NS * 2 : NULL, &conv, res ? res + 4 * b : NULL);
        status[b] = conv < 0 ? 2 : conv ? 0 : 1;
    }
}
