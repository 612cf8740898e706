/* CPU restatement of the sdf-nmpc hot path -- TEST INFRASTRUCTURE ONLY.
 *
 * This library is the parity checker for the HIP product path and the "port" CPU baseline timed by
 * bench.py.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it; the
 * product (sdf-nmpc_amd/, libsdfnmpc.so, libsdf_l4c.so) never links or calls it.
 *
 * Pinning: the network against tests/golden/sdf_golden.npz (made by the reference's own NeuralDF),
 * the dynamics/cost/constraints against tests/golden/lin_golden.npz (reference numpy helpers +
 * finite differences), the grid against tests/golden/grid_golden.npz (ocp.py:21-27).
 *
 * Reference lines followed (paths relative to /root/reference):
 *   network ............ see sdf_net.inc
 *   dynamics ........... sdf_nmpc/model/quad_rollpitchyawrate.py:19-42, utils/math.py:7-54,177-192
 *   ERK4 + sensitivities acados ERK (ocp.py:106: integrator 'ERK', defaults RK4 / 1 step /
 *                        forward sensitivities) == exact derivative of the RK4 map
 *   NLS residual ....... quad_rollpitchyawrate.py:48-55, utils/math.py:169-174
 *   constraints h ...... cost_const_helpers.py:48-75 (add_fov_const_trigo) + gen_model.py:46-70
 *   terminal extras .... gen_model.py:72-149 (rec_feas braking row, fov at Co_p_E, stability), utils/math.py:294-321
 *   shooting grid ...... ocp.py:18-27 (numpy linspace / hstack / diff semantics)
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef struct {
    int L, n1, n2, n3, n4, nf, nd;
    float w0, max_df;
} orc_spec;

/* ------------------------------------------------------------------ PRNG (weights.py mirror) */
static uint64_t mix64(uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

void orc_prng_uniform(uint64_t seed, uint64_t stream, int64_t n, double* out) {
    uint64_t key = mix64(seed * 0x9E3779B97F4A7C15ULL + stream * 0xD1B54A32D192ED03ULL + 1ULL);
    for (int64_t i = 0; i < n; ++i) {
        uint64_t x = mix64(key + (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ULL);
        out[i] = (double)(x >> 40) * (1.0 / 16777216.0);
    }
}

/* ------------------------------------------------------------------ network, fp32 and fp64 */
#define REAL float
#define SUFFIX _f32
#define SIN sinf
#define COS cosf
#include "sdf_net.inc"
#undef REAL
#undef SUFFIX
#undef SIN
#undef COS
#define REAL double
#define SUFFIX _f64
#define SIN sin
#define COS cos
#include "sdf_net.inc"
#undef REAL
#undef SUFFIX
#undef SIN
#undef COS

static size_t orc_param_counts(const orc_spec* s, size_t cnt[10]) {
    int E = 3 + 2 * s->nd * s->nf, L = s->L;
    cnt[0] = (size_t)s->n1 * (E + L); cnt[1] = s->n1;
    cnt[2] = (size_t)s->n2 * s->n1;   cnt[3] = s->n2;
    cnt[4] = (size_t)s->n3 * (s->n2 + E + L); cnt[5] = s->n3;
    cnt[6] = (size_t)s->n4 * s->n3;   cnt[7] = s->n4;
    cnt[8] = s->n4;                   cnt[9] = 1;
    size_t t = 0;
    for (int i = 0; i < 10; ++i) t += cnt[i];
    return t;
}

static size_t orc_work_len(const orc_spec* s) {
    int E = 3 + 2 * s->nd * s->nf;
    return 4 * (size_t)(E + s->L + s->n1 + s->n2 + s->n3 + s->n4) + 2 * (size_t)s->nd * s->nf;
}

/* n rows of in[n][3+L] -> df[n], grad[n][3+L] (optional), gpos[n][3] (optional).  fp32 math. */
int orc_sdf_f32(const orc_spec* s, const float* dirs, const float* freqs, const float* params,
                int64_t n, const float* in, float* df, float* grad, float* gpos, int nthreads) {
    size_t cnt[10];
    orc_param_counts(s, cnt);
    const float* P[10];
    const float* q = params;
    for (int i = 0; i < 10; ++i) { P[i] = q; q += cnt[i]; }
    const int D = 3 + s->L;
    const size_t wl = orc_work_len(s);
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
#endif
    {
        float* work = (float*)malloc(wl * sizeof(float));
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t r = 0; r < n; ++r)
            sdf_row_f32(s, dirs, freqs, P, in + r * D, df + r, grad ? grad + r * D : NULL,
                        gpos ? gpos + r * 3 : NULL, work);
        free(work);
    }
    return 0;
}

/* same network evaluated in fp64 (weights/inputs widened from fp32) */
int orc_sdf_f64(const orc_spec* s, const float* dirs, const float* freqs, const float* params,
                int64_t n, const double* in, double* df, double* grad, double* gpos) {
    size_t cnt[10];
    size_t tot = orc_param_counts(s, cnt);
    double* pd = (double*)malloc(tot * sizeof(double));
    for (size_t i = 0; i < tot; ++i) pd[i] = params[i];
    const double* P[10];
    const double* q = pd;
    for (int i = 0; i < 10; ++i) { P[i] = q; q += cnt[i]; }
    double dd[64], fd[32];
    for (int i = 0; i < 3 * s->nd; ++i) dd[i] = dirs[i];
    for (int i = 0; i < s->nf; ++i) fd[i] = freqs[i];
    const int D = 3 + s->L;
    double* work = (double*)malloc(orc_work_len(s) * sizeof(double));
    for (int64_t r = 0; r < n; ++r)
        sdf_row_f64(s, dd, fd, P, in + r * D, df + r, grad ? grad + r * D : NULL, gpos ? gpos + r * 3 : NULL,
                    work);
    free(work);
    free(pd);
    return 0;
}

/* ------------------------------------------------------------------ forward-mode duals (14 dirs) */
#define ND 14
typedef struct { double v, d[ND]; } dn;

static inline dn dc(double c) { dn r; r.v = c; memset(r.d, 0, sizeof r.d); return r; }
static inline dn dadd(dn a, dn b) { dn r; r.v = a.v + b.v; for (int i = 0; i < ND; ++i) r.d[i] = a.d[i] + b.d[i]; return r; }
static inline dn dsub(dn a, dn b) { dn r; r.v = a.v - b.v; for (int i = 0; i < ND; ++i) r.d[i] = a.d[i] - b.d[i]; return r; }
static inline dn dmul(dn a, dn b) { dn r; r.v = a.v * b.v; for (int i = 0; i < ND; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i]; return r; }
static inline dn dscl(dn a, double c) { dn r; r.v = a.v * c; for (int i = 0; i < ND; ++i) r.d[i] = a.d[i] * c; return r; }
static inline dn ddiv(dn a, dn b) {
    dn r; r.v = a.v / b.v;
    for (int i = 0; i < ND; ++i) r.d[i] = (a.d[i] - r.v * b.d[i]) / b.v;
    return r;
}
static inline dn dsqrt(dn a) { dn r; r.v = sqrt(a.v); for (int i = 0; i < ND; ++i) r.d[i] = a.d[i] / (2 * r.v); return r; }
static inline dn dsin(dn a) { dn r; r.v = sin(a.v); double c = cos(a.v); for (int i = 0; i < ND; ++i) r.d[i] = c * a.d[i]; return r; }
static inline dn dcos(dn a) { dn r; r.v = cos(a.v); double s = -sin(a.v); for (int i = 0; i < ND; ++i) r.d[i] = s * a.d[i]; return r; }
static inline dn datan2(dn y, dn x) {
    dn r; r.v = atan2(y.v, x.v);
    double den = x.v * x.v + y.v * y.v;
    for (int i = 0; i < ND; ++i) r.d[i] = (x.v * y.d[i] - y.v * x.d[i]) / den;
    return r;
}

typedef struct {
    double gamma, roll, pitch, wz;  /* robot.limits (default.yaml:97-110) */
    double g;                       /* base_model.py:10 */
    double B_p_C[3];                /* sensor extrinsics position (default.yaml:88-89) */
    double B_R_C[9];                /* euler2rot(orientation), row-major (config.py:43-44) */
    double fov_offset;              /* mpc.fov_const_offset (default.yaml:60) */
    double max_df;                  /* NeuralDF.max_df (neural_df.py:33) */
} orc_quad;

/* quad_rollpitchyawrate.py:19-42 ; W_a also returned (used by y) */
static void quad_f(const orc_quad* m, const dn* x, const dn* u, dn* f, dn* W_a_out) {
    dn nq = dsqrt(dadd(dadd(dmul(x[3], x[3]), dmul(x[4], x[4])), dadd(dmul(x[5], x[5]), dmul(x[6], x[6]))));
    dn q[4] = {ddiv(x[3], nq), ddiv(x[4], nq), ddiv(x[5], nq), ddiv(x[6], nq)};
    dn th = datan2(q[3], q[0]);
    dn c = dcos(th), s = dsin(th);
    dn gamma = dscl(u[0], m->gamma), roll = dscl(u[1], m->roll), pitch = dscl(u[2], m->pitch),
       wz = dscl(u[3], m->wz);
    /* V_R_B = euler2rot([roll, pitch, 0]) third column (math.py:34-42 with yaw = 0) */
    dn sr = dsin(roll), cr = dcos(roll), sp = dsin(pitch), cp = dcos(pitch);
    dn b0 = dmul(dmul(cr, sp), gamma), b1 = dmul(dscl(sr, -1.0), gamma), b2 = dmul(dmul(cr, cp), gamma);
    /* W_R_V = quat2rot([c,0,0,s]) (math.py:11-19) */
    dn r11 = dsub(dmul(c, c), dmul(s, s)), r21 = dscl(dmul(c, s), 2.0), r33 = dadd(dmul(c, c), dmul(s, s));
    dn W_a[3];
    W_a[0] = dsub(dmul(r11, b0), dmul(r21, b1));
    W_a[1] = dadd(dmul(r21, b0), dmul(r11, b1));
    W_a[2] = dsub(dmul(r33, b2), dc(m->g));
    /* dq = hamilton_prod(q, [0,0,0,wz]) / 2 (math.py:177-192) */
    f[0] = x[7]; f[1] = x[8]; f[2] = x[9];
    f[3] = dscl(dmul(dscl(q[3], -1.0), wz), 0.5);
    f[4] = dscl(dmul(q[2], wz), 0.5);
    f[5] = dscl(dmul(dscl(q[1], -1.0), wz), 0.5);
    f[6] = dscl(dmul(q[0], wz), 0.5);
    f[7] = W_a[0]; f[8] = W_a[1]; f[9] = W_a[2];
    if (W_a_out) { W_a_out[0] = W_a[0]; W_a_out[1] = W_a[1]; W_a_out[2] = W_a[2]; }
}

static void seed_xu(const double* x, const double* u, dn* X, dn* U) {
    for (int i = 0; i < 10; ++i) { X[i] = dc(x[i]); X[i].d[i] = 1.0; }
    if (U) for (int i = 0; i < 4; ++i) { U[i] = dc(u[i]); U[i].d[10 + i] = 1.0; }
}

/* ERK4 step and its exact Jacobian.  xn[10]; AB col-major [14][10] (column j = d xn / d (x,u)_j) */
void orc_quad_rk4(const orc_quad* m, const double* x, const double* u, double dt, double* xn, double* AB) {
    /* acados ERK accumulation: x_out = x + sum_s (h b_s) k_s, stage input x + (h a_s) k_{s-1} */
    const double hb[4] = {dt / 6, dt / 3, dt / 3, dt / 6}, ha[4] = {0.0, dt / 2, dt / 2, dt};
    dn X[10], U[4], k[10], t[10], xo[10];
    seed_xu(x, u, X, U);
    quad_f(m, X, U, k, NULL);
    for (int i = 0; i < 10; ++i) xo[i] = dadd(X[i], dscl(k[i], hb[0]));
    for (int s = 1; s < 4; ++s) {
        for (int i = 0; i < 10; ++i) t[i] = dadd(X[i], dscl(k[i], ha[s]));
        quad_f(m, t, U, k, NULL);
        for (int i = 0; i < 10; ++i) xo[i] = dadd(xo[i], dscl(k[i], hb[s]));
    }
    for (int i = 0; i < 10; ++i) {
        xn[i] = xo[i].v;
        if (AB) for (int j = 0; j < ND; ++j) AB[j * 10 + i] = xo[i].d[j];
    }
}

static void quat_inv_prod(const dn* qd_c, const dn* q, dn* qe) {
    /* q_e = hamilton_prod(q_d, invert(q)), invert = conj / |q| (math.py:169-174) */
    dn nq = dsqrt(dadd(dadd(dmul(q[0], q[0]), dmul(q[1], q[1])), dadd(dmul(q[2], q[2]), dmul(q[3], q[3]))));
    dn qi[4] = {ddiv(q[0], nq), ddiv(dscl(q[1], -1.0), nq), ddiv(dscl(q[2], -1.0), nq), ddiv(dscl(q[3], -1.0), nq)};
    const dn* a = qd_c;
    qe[0] = dsub(dsub(dmul(a[0], qi[0]), dmul(a[1], qi[1])), dadd(dmul(a[2], qi[2]), dmul(a[3], qi[3])));
    qe[1] = dadd(dadd(dmul(a[0], qi[1]), dmul(a[1], qi[0])), dsub(dmul(a[2], qi[3]), dmul(a[3], qi[2])));
    qe[2] = dadd(dsub(dmul(a[0], qi[2]), dmul(a[1], qi[3])), dadd(dmul(a[2], qi[0]), dmul(a[3], qi[1])));
    qe[3] = dadd(dsub(dadd(dmul(a[0], qi[3]), dmul(a[1], qi[2])), dmul(a[2], qi[1])), dmul(a[3], qi[0]));
}

/* stage residual y (11) and J_y col-major [14][11]; terminal yN (4), J_yN [10][4] */
void orc_quad_cost(const orc_quad* m, const double* x, const double* u, const double* p, double* y, double* Jy,
                   double* yN, double* JyN) {
    dn X[10], U[4], f[10], W_a[3], qd[4], qe[4], Y[11];
    seed_xu(x, u, X, U);
    for (int i = 0; i < 4; ++i) qd[i] = dc(p[13 + i]);  /* p_idx.q_d (default.yaml:67) */
    dn nq = dsqrt(dadd(dadd(dmul(X[3], X[3]), dmul(X[4], X[4])), dadd(dmul(X[5], X[5]), dmul(X[6], X[6]))));
    dn q[4] = {ddiv(X[3], nq), ddiv(X[4], nq), ddiv(X[5], nq), ddiv(X[6], nq)};
    quat_inv_prod(qd, q, qe);
    quad_f(m, X, U, f, W_a);
    Y[0] = X[0]; Y[1] = X[1]; Y[2] = X[2]; Y[3] = qe[3];
    Y[4] = X[7]; Y[5] = X[8]; Y[6] = X[9];
    Y[7] = dscl(U[1], m->roll); Y[8] = dscl(U[2], m->pitch); Y[9] = dscl(U[3], m->wz); Y[10] = W_a[2];
    for (int i = 0; i < 11; ++i) {
        if (y) y[i] = Y[i].v;
        if (Jy) for (int j = 0; j < ND; ++j) Jy[j * 11 + i] = Y[i].d[j];
    }
    for (int i = 0; i < 4; ++i) {
        if (yN) yN[i] = Y[i].v;
        if (JyN) for (int j = 0; j < 10; ++j) JyN[j * 4 + i] = Y[i].d[j];
    }
}

/* h = [hfov, vfov, sdf] (3) and J_h col-major [10][3]; df/gdf = fp32 network output at Co_p_B */
void orc_quad_constr(const orc_quad* m, const double* x, const double* p, double df, const double* gdf,
                     double* h, double* Jh, double* Co_p_B_out) {
    dn X[10];
    seed_xu(x, NULL, X, NULL);
    const double flag = p[0];
    const double* W_p_Co = p + 1;
    const double* R = p + 4;  /* W_R_Co row-major == casadi reshape((3,3)).T (gen_model.py:47) */
    dn d[3] = {dsub(X[0], dc(W_p_Co[0])), dsub(X[1], dc(W_p_Co[1])), dsub(X[2], dc(W_p_Co[2]))};
    dn C[3];
    double off[3];
    for (int i = 0; i < 3; ++i)  /* B_R_C^T B_p_C */
        off[i] = m->B_R_C[0 * 3 + i] * m->B_p_C[0] + m->B_R_C[1 * 3 + i] * m->B_p_C[1] + m->B_R_C[2 * 3 + i] * m->B_p_C[2];
    for (int i = 0; i < 3; ++i) {  /* Co_p_B = W_R_Co^T (W_p_B - W_p_Co) */
        C[i] = dadd(dadd(dscl(d[0], R[0 * 3 + i]), dscl(d[1], R[1 * 3 + i])), dscl(d[2], R[2 * 3 + i]));
        if (Co_p_B_out) Co_p_B_out[i] = C[i].v;
    }
    dn Cf[3] = {dadd(C[0], dc(off[0] + m->fov_offset)), dadd(C[1], dc(off[1])), dadd(C[2], dc(off[2]))};
    dn hf = dscl(datan2(Cf[1], Cf[0]), flag);
    dn vf = dscl(datan2(Cf[2], dsqrt(dadd(dmul(Cf[0], Cf[0]), dmul(Cf[1], Cf[1])))), flag);
    if (h) { h[0] = hf.v; h[1] = vf.v; h[2] = flag * df + (1.0 - flag) * m->max_df; }
    if (Jh) {
        for (int j = 0; j < 10; ++j) { Jh[j * 3 + 0] = hf.d[j]; Jh[j * 3 + 1] = vf.d[j]; Jh[j * 3 + 2] = 0.0; }
        for (int j = 0; j < 3; ++j)  /* d s / d W_p_B = flag * gdf * W_R_Co^T */
            Jh[j * 3 + 2] = flag * (gdf[0] * R[j * 3 + 0] + gdf[1] * R[j * 3 + 1] + gdf[2] * R[j * 3 + 2]);
    }
}

/* Terminal extras of flags.recursive_feasibility / stability at node N (gen_model.py:72-149,
 * quad_rollpitchyawrate.py:52-55, utils/math.py:294-321):
 *   hE = [-flag poly(v), flag atan2(E_y, E_x), flag atan2(E_z, |E_xy|), v_x, v_y, v_z] with
 *   E = Co_p_E = W_R_Co^T (p + poly(v) v / sqrt(|v|^2 + 1e-4) - W_p_Co) + B_R_C^T B_p_C + [fov_offset, 0, 0]
 *   (braking_dist_flag with the flag forced to 1 inside Co_p_E, gen_model.py:86-87,110-112);
 *   poly in polynomial_3variate's term order (total degree d, then x exponent a, then y exponent b).
 * hE [6], JhE col-major [10][6].  With stability, yN5 = flag [p, q_e[3], |v|^2] and JyN5 [10][5]. */
void orc_quad_term(const orc_quad* m, const double* x, const double* p, int deg, const double* poly, int rec_feas,
                   int stability, double* hE, double* JhE, double* yN5, double* JyN5) {
    dn X[10];
    seed_xu(x, NULL, X, NULL);
    const double flag = p[0];
    dn H[6] = {dc(0.0), dc(0.0), dc(0.0), X[7], X[8], X[9]};
    dn vv = dadd(dadd(dmul(X[7], X[7]), dmul(X[8], X[8])), dmul(X[9], X[9]));
    if (rec_feas) {
        dn pw[3][16];
        for (int i = 0; i < 3; ++i) {
            pw[i][0] = dc(1.0);
            for (int a = 1; a <= deg; ++a) pw[i][a] = dmul(pw[i][a - 1], X[7 + i]);
        }
        dn pv = dc(0.0);
        int q = 0;
        for (int d = 0; d <= deg; ++d)
            for (int a = 0; a <= d; ++a)
                for (int b = 0; b <= d - a; ++b, ++q)
                    pv = dadd(pv, dscl(dmul(dmul(pw[0][a], pw[1][b]), pw[2][d - a - b]), poly[q]));
        H[0] = dscl(pv, -flag);
        dn sc = ddiv(pv, dsqrt(dadd(vv, dc(1e-4))));
        const double* R = p + 4;
        dn e[3];
        for (int i = 0; i < 3; ++i) e[i] = dsub(dadd(X[i], dmul(X[7 + i], sc)), dc(p[1 + i]));
        double off[3];
        for (int i = 0; i < 3; ++i)
            off[i] = m->B_R_C[0 * 3 + i] * m->B_p_C[0] + m->B_R_C[1 * 3 + i] * m->B_p_C[1] + m->B_R_C[2 * 3 + i] * m->B_p_C[2];
        dn E[3];
        for (int i = 0; i < 3; ++i)
            E[i] = dadd(dadd(dadd(dscl(e[0], R[0 * 3 + i]), dscl(e[1], R[1 * 3 + i])), dscl(e[2], R[2 * 3 + i])),
                        dc(off[i] + (i == 0 ? m->fov_offset : 0.0)));
        H[1] = dscl(datan2(E[1], E[0]), flag);
        H[2] = dscl(datan2(E[2], dsqrt(dadd(dmul(E[0], E[0]), dmul(E[1], E[1])))), flag);
    }
    for (int i = 0; i < 6; ++i) {
        if (hE) hE[i] = H[i].v;
        if (JhE) for (int j = 0; j < 10; ++j) JhE[j * 6 + i] = H[i].d[j];
    }
    if (stability && (yN5 || JyN5)) {
        double u0[4] = {0, 0, 0, 0}, yN[4], JyN[40];
        orc_quad_cost(m, x, u0, p, NULL, NULL, yN, JyN);
        for (int i = 0; i < 4; ++i) {
            if (yN5) yN5[i] = flag * yN[i];
            if (JyN5) for (int j = 0; j < 10; ++j) JyN5[j * 5 + i] = flag * JyN[j * 4 + i];
        }
        if (yN5) yN5[4] = flag * vv.v;
        if (JyN5) for (int j = 0; j < 10; ++j) JyN5[j * 5 + 4] = flag * vv.d[j];
    }
}

/* ------------------------------------------------------------------ shooting grid (ocp.py:18-27) */
static void np_linspace(double start, double stop, int num, double* y) {
    /* numpy.linspace(endpoint=True): y_i = i*step + start, y[-1] = stop (numpy/_core/function_base.py) */
    if (num == 1) { y[0] = start; return; }  /* numpy: div = 0 -> [start] */
    int div = num - 1;
    double delta = stop - start;
    double step = delta / div;
    for (int i = 0; i < num; ++i) {
        volatile double t = (double)i * step;  /* keep two roundings, no FMA contraction */
        y[i] = t + start;
    }
    if (num > 1) y[num - 1] = stop;
}

int orc_shooting_grid(int N, double T, int uniform, int n_short, double dt_short, double* nodes, double* dt) {
    if (N < 1) return -1;
    if (uniform) {
        np_linspace(0.0, T, N + 1, nodes);
    } else {
        if (n_short < 1 || n_short > N) return -1;
        np_linspace(0.0, dt_short * (n_short - 1), n_short, nodes);
        np_linspace(dt_short * n_short, T, N - n_short + 1, nodes + n_short);
    }
    for (int k = 0; k < N; ++k) dt[k] = nodes[k + 1] - nodes[k];
    return 0;
}

/* ------------------------------------------------------------------ full preparation phase (CPU baseline)
 * Per instance b and node k: Co_p_B, fp32 SDF fwd+grad, ERK4+sensitivities (k<N), NLS (k<N / N),
 * h and J_h (all k).  Output layouts are those of sdfnmpc_linearize (include/sdfnmpc.h). */
int orc_linearize_batch(const orc_quad* m, const orc_spec* s, const float* dirs, const float* freqs,
                        const float* params, int B, int N, int np_, const double* x, const double* u,
                        const double* p, const double* dt, double* xn, double* AB, double* y, double* Jy,
                        double* yN, double* JyN, double* h, double* Jh, float* sdf_out, int nthreads) {
    size_t cnt[10];
    orc_param_counts(s, cnt);
    const float* P[10];
    const float* q = params;
    for (int i = 0; i < 10; ++i) { P[i] = q; q += cnt[i]; }
    const int D = 3 + s->L;
    const size_t wl = orc_work_len(s);
    const int64_t rows = (int64_t)B * (N + 1);
#ifdef _OPENMP
    if (nthreads < 1) nthreads = 1;
#pragma omp parallel num_threads(nthreads)
#endif
    {
        float* work = (float*)malloc(wl * sizeof(float));
        float* in = (float*)malloc(D * sizeof(float));
#ifdef _OPENMP
#pragma omp for schedule(static)
#endif
        for (int64_t r = 0; r < rows; ++r) {
            int b = (int)(r / (N + 1)), k = (int)(r % (N + 1));
            const double* xk = x + r * 10;
            const double* pk = p + r * np_;
            double Cpb[3], df, g[3];
            orc_quad_constr(m, xk, pk, 0.0, (double[3]){0, 0, 0}, NULL, NULL, Cpb);
            for (int i = 0; i < 3; ++i) in[i] = (float)Cpb[i];
            for (int i = 0; i < s->L; ++i) in[3 + i] = (float)pk[17 + i];
            float dff, gf[3];
            sdf_row_f32(s, dirs, freqs, P, in, &dff, NULL, gf, work);
            df = dff; g[0] = gf[0]; g[1] = gf[1]; g[2] = gf[2];
            if (sdf_out) { sdf_out[r * 4] = dff; sdf_out[r * 4 + 1] = gf[0]; sdf_out[r * 4 + 2] = gf[1]; sdf_out[r * 4 + 3] = gf[2]; }
            orc_quad_constr(m, xk, pk, df, g, h + r * 3, Jh + r * 30, NULL);
            if (k < N) {
                int64_t s_ = (int64_t)b * N + k;
                const double* uk = u + s_ * 4;
                orc_quad_rk4(m, xk, uk, dt[k], xn + s_ * 10, AB + s_ * 140);
                orc_quad_cost(m, xk, uk, pk, y + s_ * 11, Jy + s_ * 154, NULL, NULL);
            } else {
                double u0[4] = {0, 0, 0, 0};
                orc_quad_cost(m, xk, u0, pk, NULL, NULL, yN + (int64_t)b * 4, JyN + (int64_t)b * 40);
            }
        }
        free(in);
        free(work);
    }
    return 0;
}

int orc_max_threads(void) {
#ifdef _OPENMP
    return omp_get_max_threads();
#else
    return 1;
#endif
}
