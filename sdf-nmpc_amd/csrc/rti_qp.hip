// SQP-RTI feedback phase: the OCP QP of every instance solved by a batched interior-point method.
//
// The QP is what acados builds from the preparation phase and hands to HPIPM (sdf_nmpc/ocp.py:54-120:
// NONLINEAR_LS + GAUSS_NEWTON, levenberg_marquardt, soft h constraints with L1/L2 slack penalties,
// input boxes, x_0 fixed), stated in oracle/qp_oracle.py.  The reference condenses it
// (FULL_CONDENSING_HPIPM) and runs a dense IPM; the solution is unique (lm > 0), so this build keeps
// the stage structure instead -- a Riccati recursion per Newton step -- which is O(N (nx+nu)^3) and
// maps one instance to one wavefront:
//   * Mehrotra predictor-corrector on t = D z + d >= 0, lambda >= 0 (20 rows per stage, 12 at N)
//   * each Newton system is an LQR in the new iterate z+ with Hessian H + D^T Sigma D and gradient
//     g - D^T v (v folds the residuals), so dynamics hold exactly and no costate is carried
//   * the soft-constraint slacks have diagonal Hessians and are eliminated row by row, leaving a
//     rank-3 update of each node's state block
//   * one factorisation per iteration serves the predictor and the corrector solve
// 64 lanes cooperate on the 10x14 stage products; iterates, slacks and duals live in LDS, the
// factors (P, K, S, chol R) in a global workspace re-read by the corrector sweep.
#include <hip/hip_runtime.h>

#include "qp_kernels.h"

namespace sdfn {

namespace {

constexpr int NX = 10, NU = 4, NS = 3, NW = 14;
constexpr int FSTRIDE = QP_FSTRIDE;

struct Lds {  // carve of the dynamic LDS block, sizes depend on N
    double *dx, *du, *sl, *su;      // current iterate z
    double *px, *pu, *psl, *psu;    // LQR solution z+
    double *t, *lam, *dta, *dla;    // inequality slacks / duals / affine deltas
    double *P, *p, *W, *M, *m, *Pb, *AB, *K, *S, *L, *kff, *c;  // stage scratch
    double* red;                    // reduction scratch [64]
};

__device__ __forceinline__ int n_ineq(int N) { return 8 * N + 12 * (N + 1); }

__device__ Lds carve(double* base, int N) {
    Lds s;
    double* q = base;
    auto take = [&](int n) { double* r = q; q += n; return r; };
    s.dx = take((N + 1) * NX); s.du = take(N * NU); s.sl = take((N + 1) * NS); s.su = take((N + 1) * NS);
    s.px = take((N + 1) * NX); s.pu = take(N * NU); s.psl = take((N + 1) * NS); s.psu = take((N + 1) * NS);
    const int m = n_ineq(N);
    s.t = take(m); s.lam = take(m); s.dta = take(m); s.dla = take(m);
    s.P = take(100); s.p = take(10); s.W = take(140); s.M = take(196); s.m = take(14); s.Pb = take(10);
    s.AB = take(140); s.K = take(40); s.S = take(40); s.L = take(16); s.kff = take(4); s.c = take(10);
    s.red = take(64);
    return s;
}

__device__ __forceinline__ double wave_max(double v, double* red, int lane) {
    red[lane] = v;
    __syncthreads();
    for (int o = 32; o > 0; o >>= 1) {
        if (lane < o) red[lane] = fmax(red[lane], red[lane + o]);
        __syncthreads();
    }
    const double r = red[0];
    __syncthreads();
    return r;
}
__device__ __forceinline__ double wave_min(double v, double* red, int lane) { return -wave_max(-v, red, lane); }
__device__ __forceinline__ double wave_sum(double v, double* red, int lane) {
    red[lane] = v;
    __syncthreads();
    for (int o = 32; o > 0; o >>= 1) {
        if (lane < o) red[lane] += red[lane + o];
        __syncthreads();
    }
    const double r = red[0];
    __syncthreads();
    return r;
}

// row r of the inequality system t = D z + d: its value at (dx, du, sl, su)
struct Row {
    int kind;  // 0 u-lower, 1 u-upper, 2 h-lower, 3 h-upper, 4 sl >= 0, 5 su >= 0
    int k, i;  // node, component
};
__device__ __forceinline__ Row row_of(int r, int N) {
    Row o;
    if (r < 8 * N) {
        o.k = r >> 3;
        const int q = r & 7;
        o.kind = q >> 2;
        o.i = q & 3;
    } else {
        const int q = r - 8 * N;
        o.k = q / 12;
        const int w = q - 12 * o.k;
        o.i = w >> 2;
        o.kind = 2 + (w & 3);
    }
    return o;
}

}  // namespace

__global__ __launch_bounds__(64) void rti_qp_kernel(QpArgs A) {
    extern __shared__ __align__(16) double lds_q[];
    const int b = blockIdx.x;
    const int lane = threadIdx.x;
    const int N = A.N, N1 = A.N + 1;
    const int m = n_ineq(N);
    Lds s = carve(lds_q, N);
    double* ws = A.work + (size_t)b * qp_work_doubles(N);
    double* Hs = ws;                        // [N][196] stage Hessians, then [100] terminal
    double* gs = Hs + (size_t)N * 196 + 100;  // [N][14], then [10]
    double* F = gs + (size_t)N * 14 + 10;   // [N+1][FSTRIDE] factors
    const double* AB = A.AB + (size_t)b * N * 140;
    const double* xn = A.xn + (size_t)b * N * 10;
    const double* Jh = A.Jh + (size_t)b * N1 * 30;
    const double* hh = A.h + (size_t)b * N1 * 3;
    const double* xb = A.x + (size_t)b * N1 * 10;
    const double* ub = A.u + (size_t)b * N * 4;

    // ---------------------------------------------------------------- setup: GN Hessians / gradients
    // H_k = s_k J^T W J + lm I, g_k = s_k J^T W (y - yref)  (J = J_y column-major [14][11])
    for (int k = 0; k < N; ++k) {
        const double sk = A.cost_scaling ? A.dt[k] : 1.0;
        const double* J = A.Jy + ((size_t)b * N + k) * 154;
        const double* Wk = A.W + ((size_t)b * N + k) * 11;
        const double* yk = A.y + ((size_t)b * N + k) * 11;
        const double* rk = A.yref + ((size_t)b * N + k) * 11;
        for (int e = lane; e < 196 + 14; e += 64) {
            double acc = 0.0;
            if (e < 196) {
                const int a = e / 14, c = e % 14;
                for (int i = 0; i < 11; ++i) acc += J[a * 11 + i] * Wk[i] * J[c * 11 + i];
                Hs[(size_t)k * 196 + e] = sk * acc + (a == c ? A.lm : 0.0);
            } else {
                const int a = e - 196;
                for (int i = 0; i < 11; ++i) acc += J[a * 11 + i] * Wk[i] * (yk[i] - rk[i]);
                gs[(size_t)k * 14 + a] = sk * acc;
            }
        }
    }
    {
        const double sN = 1.0;
        const double* J = A.JyN + (size_t)b * 40;  // [10][4]
        const double* Wn = A.WN + (size_t)b * 4;
        const double* yn = A.yN + (size_t)b * 4;
        const double* rn = A.yNref + (size_t)b * 4;
        for (int e = lane; e < 110; e += 64) {
            double acc = 0.0;
            if (e < 100) {
                const int a = e / 10, c = e % 10;
                for (int i = 0; i < 4; ++i) acc += J[a * 4 + i] * Wn[i] * J[c * 4 + i];
                Hs[(size_t)N * 196 + e] = sN * acc + (a == c ? A.lm : 0.0);
            } else {
                const int a = e - 100;
                for (int i = 0; i < 4; ++i) acc += J[a * 4 + i] * Wn[i] * (yn[i] - rn[i]);
                gs[(size_t)N * 14 + a] = sN * acc;
            }
        }
    }
    // ---------------------------------------------------------------- initial iterate (dynamics-feasible)
    for (int e = lane; e < N * NU; e += 64) s.du[e] = 0.0;
    for (int e = lane; e < N1 * NS; e += 64) { s.sl[e] = 0.0; s.su[e] = 0.0; }
    if (lane < NX) s.dx[lane] = A.x0[(size_t)b * 10 + lane] - xb[lane];
    __syncthreads();
    for (int k = 0; k < N; ++k) {  // dx_{k+1} = A dx_k + c_k
        if (lane < NX) {
            double acc = xn[k * 10 + lane] - xb[(k + 1) * 10 + lane];
            for (int j = 0; j < NX; ++j) acc += AB[k * 140 + j * 10 + lane] * s.dx[k * NX + j];
            s.dx[(k + 1) * NX + lane] = acc;
        }
        __syncthreads();
    }

    // value a.z + d of inequality row r at iterate (dx, du, sl, su)
    auto row_val = [&](int r, const double* dx, const double* du, const double* sl, const double* su) -> double {
        const Row o = row_of(r, N);
        const double* Ck = Jh + (size_t)o.k * 30;  // col-major [10][3]: Ck[j*3 + i] = d h_i / d x_j
        switch (o.kind) {
            case 0: return du[o.k * NU + o.i] - (A.lbu[o.i] - ub[o.k * 4 + o.i]);
            case 1: return (A.ubu[o.i] - ub[o.k * 4 + o.i]) - du[o.k * NU + o.i];
            case 2: case 3: {
                double cx = 0.0;
                for (int j = 0; j < NX; ++j) cx += Ck[j * 3 + o.i] * dx[o.k * NX + j];
                const double hv = hh[o.k * 3 + o.i];
                return o.kind == 2 ? cx + (hv - A.lh[o.i]) + sl[o.k * NS + o.i]
                                   : -cx + (A.uh[o.i] - hv) + su[o.k * NS + o.i];
            }
            case 4: return sl[o.k * NS + o.i];
            default: return su[o.k * NS + o.i];
        }
    };
    auto row_d = [&](int r) -> double {  // constant term d of row r
        const Row o = row_of(r, N);
        switch (o.kind) {
            case 0: return ub[o.k * 4 + o.i] - A.lbu[o.i];
            case 1: return A.ubu[o.i] - ub[o.k * 4 + o.i];
            case 2: return hh[o.k * 3 + o.i] - A.lh[o.i];
            case 3: return A.uh[o.i] - hh[o.k * 3 + o.i];
            default: return 0.0;
        }
    };

    for (int r = lane; r < m; r += 64) {
        s.t[r] = fmax(row_val(r, s.dx, s.du, s.sl, s.su), 1.0);
        s.lam[r] = 1.0;
    }
    __syncthreads();

    // v of row r for the current right-hand side (phase 0: predictor, 1: corrector)
    auto row_v = [&](int r, int phase, double sigmu) -> double {
        const double t = s.t[r], l = s.lam[r];
        double v = (l / t) * (t - row_d(r));
        if (phase) v -= (s.dta[r] * s.dla[r] - sigmu) / t;
        return v;
    };

    // Node-k soft rows folded into the state block: weight w_j (C_j^T C_j) and gradient gamma_j C_j^T.
    // Lane j < 3 computes (w_j, gamma_j); result in out[0..2] = w, out[3..5] = gamma.
    auto soft_fold = [&](int k, int phase, double sigmu, double* out) {
        if (lane < NS) {
            const int j = lane;
            const double sk = (A.cost_scaling && k < N) ? A.dt[k] : 1.0;
            const int r0 = 8 * N + 12 * k + 4 * j;
            const double s1 = s.lam[r0] / s.t[r0], s2 = s.lam[r0 + 2] / s.t[r0 + 2];
            const double s3 = s.lam[r0 + 1] / s.t[r0 + 1], s4 = s.lam[r0 + 3] / s.t[r0 + 3];
            const double v1 = row_v(r0, phase, sigmu), v2 = row_v(r0 + 2, phase, sigmu);
            const double v3 = row_v(r0 + 1, phase, sigmu), v4 = row_v(r0 + 3, phase, sigmu);
            const double Zs = sk * A.Zl[j], zs = sk * A.zl[j];
            const double Hl = Zs + s1 + s2, Hu = Zs + s3 + s4;
            const double gl = zs - v1 - v2, gu = zs - v3 - v4;
            out[j] = s1 * (Zs + s2) / Hl + s3 * (Zs + s4) / Hu;
            out[3 + j] = -(v1 + s1 * gl / Hl) + (v3 + s3 * gu / Hu);
        }
    };

    // ---------------------------------------------------------------- Riccati sweeps
    // factor == true : build and store the factorisation (and solve for the predictor gradient)
    // factor == false: reuse the stored factors with the corrector gradient
    auto backward = [&](bool factor, int phase, double sigmu) {
        double* sf = s.red;  // soft fold scratch [6] (red is free during sweeps)
        // terminal node
        soft_fold(N, phase, sigmu, sf);
        __syncthreads();
        const double* CN = Jh + (size_t)N * 30;
        for (int e = lane; e < 110; e += 64) {
            if (e < 100) {
                const int a = e / 10, c = e % 10;
                double v = Hs[(size_t)N * 196 + e];
                for (int j = 0; j < NS; ++j) v += sf[j] * CN[a * 3 + j] * CN[c * 3 + j];
                if (factor) { s.P[e] = v; F[(size_t)N * FSTRIDE + e] = v; }
            } else {
                const int a = e - 100;
                double v = gs[(size_t)N * 14 + a];
                for (int j = 0; j < NS; ++j) v += sf[3 + j] * CN[a * 3 + j];
                s.p[a] = v;
            }
        }
        __syncthreads();
        for (int k = N - 1; k >= 0; --k) {
            double* Fk = F + (size_t)k * FSTRIDE;
            const double* Fk1 = F + (size_t)(k + 1) * FSTRIDE;
            soft_fold(k, phase, sigmu, sf);
            for (int e = lane; e < 150; e += 64) {
                if (e < 140) s.AB[e] = AB[(size_t)k * 140 + e];
                else s.c[e - 140] = xn[k * 10 + e - 140] - xb[(k + 1) * 10 + e - 140];
            }
            if (!factor)
                for (int e = lane; e < 100; e += 64) s.P[e] = Fk1[e];
            __syncthreads();
            // W = P [A B] (10 x 14, row-major W[i*14+j]); Pb = P c + p
            for (int e = lane; e < 150; e += 64) {
                if (e < 140) {
                    if (!factor) continue;
                    const int i = e / 14, j = e % 14;
                    double acc = 0.0;
                    for (int l = 0; l < NX; ++l) acc += s.P[i * 10 + l] * s.AB[j * 10 + l];
                    s.W[e] = acc;
                } else {
                    const int i = e - 140;
                    double acc = s.p[i];
                    for (int l = 0; l < NX; ++l) acc += s.P[i * 10 + l] * s.c[l];
                    s.Pb[i] = acc;
                }
            }
            __syncthreads();
            // M = H~ + [A B]^T W (14 x 14); m = g~ + [A B]^T Pb
            const double* Ck = Jh + (size_t)k * 30;
            for (int e = lane; e < 210; e += 64) {
                if (e < 196) {
                    if (!factor) continue;
                    const int a = e / 14, c = e % 14;
                    double v = Hs[(size_t)k * 196 + e];
                    for (int l = 0; l < NX; ++l) v += s.AB[a * 10 + l] * s.W[l * 14 + c];
                    if (a < NX && c < NX) {
                        for (int j = 0; j < NS; ++j) v += sf[j] * Ck[a * 3 + j] * Ck[c * 3 + j];
                    } else if (a == c) {  // input box rows (u lower, u upper)
                        const int i = a - NX, r0 = 8 * k + i;
                        v += s.lam[r0] / s.t[r0] + s.lam[r0 + 4] / s.t[r0 + 4];
                    }
                    s.M[e] = v;
                } else {
                    const int a = e - 196;
                    double v = gs[(size_t)k * 14 + a];
                    for (int l = 0; l < NX; ++l) v += s.AB[a * 10 + l] * s.Pb[l];
                    if (a < NX) {
                        for (int j = 0; j < NS; ++j) v += sf[3 + j] * Ck[a * 3 + j];
                    } else {
                        const int i = a - NX, r0 = 8 * k + i;
                        v += -row_v(r0, phase, sigmu) + row_v(r0 + 4, phase, sigmu);
                    }
                    s.m[a] = v;
                }
            }
            __syncthreads();
            // Cholesky of R^ = M_uu (every active lane, in registers); K = -R^-1 S, k_ff = -R^-1 m_u
            // (corrector: only k_ff, with the stored factor)
            if (factor ? lane <= NX : lane == NX) {
                double L[4][4];
                if (factor) {
                    for (int i = 0; i < 4; ++i)
                        for (int j = 0; j <= i; ++j) {
                            double v = s.M[(NX + i) * 14 + NX + j];
                            for (int q = 0; q < j; ++q) v -= L[i][q] * L[j][q];
                            L[i][j] = (i == j) ? sqrt(v) : v / L[j][j];
                        }
                    if (lane == 0)
                        for (int i = 0; i < 16; ++i) Fk[180 + i] = (i / 4 >= i % 4) ? L[i / 4][i % 4] : 0.0;
                } else {
                    for (int i = 0; i < 4; ++i)
                        for (int j = 0; j < 4; ++j) L[i][j] = Fk[180 + i * 4 + j];
                }
                double rhs[4];
                for (int i = 0; i < 4; ++i) rhs[i] = (lane < NX) ? s.M[(NX + i) * 14 + lane] : s.m[NX + i];
                double yv[4];
                for (int i = 0; i < 4; ++i) {
                    double v = rhs[i];
                    for (int q = 0; q < i; ++q) v -= L[i][q] * yv[q];
                    yv[i] = v / L[i][i];
                }
                double xv[4];
                for (int i = 3; i >= 0; --i) {
                    double v = yv[i];
                    for (int q = i + 1; q < 4; ++q) v -= L[q][i] * xv[q];
                    xv[i] = v / L[i][i];
                }
                if (lane < NX) {
                    if (factor)
                        for (int i = 0; i < 4; ++i) {
                            s.K[i * 10 + lane] = -xv[i];
                            s.S[i * 10 + lane] = rhs[i];
                        }
                } else {
                    for (int i = 0; i < 4; ++i) s.kff[i] = -xv[i];
                }
            }
            if (!factor)
                for (int e = lane; e < 80; e += 64) (e < 40 ? s.K[e] : s.S[e - 40]) = Fk[100 + e];
            __syncthreads();
            // P <- Q^ + S^T K ; p <- m_x + S^T k_ff ; store factors
            for (int e = lane; e < 110; e += 64) {
                if (e < 100) {
                    if (!factor) continue;
                    const int a = e / 10, c = e % 10;
                    double v = 0.5 * (s.M[a * 14 + c] + s.M[c * 14 + a]);
                    for (int i = 0; i < 4; ++i) v += 0.5 * (s.S[i * 10 + a] * s.K[i * 10 + c] + s.S[i * 10 + c] * s.K[i * 10 + a]);
                    s.W[e] = v;  // W is free now: new P
                } else {
                    const int a = e - 100;
                    double v = s.m[a];
                    for (int i = 0; i < 4; ++i) v += s.S[i * 10 + a] * s.kff[i];
                    s.Pb[a] = v;  // new p
                }
            }
            __syncthreads();
            for (int e = lane; e < 110; e += 64) {
                if (e < 100) {
                    if (factor) {
                        s.P[e] = s.W[e];
                        Fk[e] = s.W[e];
                    }
                } else {
                    s.p[e - 100] = s.Pb[e - 100];
                }
            }
            if (factor)
                for (int e = lane; e < 80; e += 64) Fk[100 + e] = e < 40 ? s.K[e] : s.S[e - 40];
            if (lane < 4) Fk[196 + lane] = s.kff[lane];
            __syncthreads();
        }
    };

    // forward sweep: z+ from the stored K_k, k_ff_k; then the slacks of the soft rows
    auto forward = [&](int phase, double sigmu) {
        if (lane < NX) s.px[lane] = s.dx[lane];  // x_0 is fixed (the iterate already satisfies it)
        __syncthreads();
        for (int k = 0; k < N; ++k) {
            const double* Fk = F + (size_t)k * FSTRIDE;
            if (lane < NU) {
                double v = Fk[196 + lane];
                for (int j = 0; j < NX; ++j) v += Fk[100 + lane * 10 + j] * s.px[k * NX + j];
                s.pu[k * NU + lane] = v;
            }
            __syncthreads();
            if (lane < NX) {
                double v = xn[k * 10 + lane] - xb[(k + 1) * 10 + lane];
                for (int j = 0; j < NX; ++j) v += AB[(size_t)k * 140 + j * 10 + lane] * s.px[k * NX + j];
                for (int i = 0; i < NU; ++i) v += AB[(size_t)k * 140 + (NX + i) * 10 + lane] * s.pu[k * NU + i];
                s.px[(k + 1) * NX + lane] = v;
            }
            __syncthreads();
        }
        // slacks: sl = -(g_s + sigma_1 C x)/H_s,  su = -(g_s' - sigma_3 C x)/H_s'
        for (int e = lane; e < N1 * NS; e += 64) {
            const int k = e / NS, j = e % NS;
            const double sk = (A.cost_scaling && k < N) ? A.dt[k] : 1.0;
            const int r0 = 8 * N + 12 * k + 4 * j;
            const double* Ck = Jh + (size_t)k * 30;
            double cx = 0.0;
            for (int l = 0; l < NX; ++l) cx += Ck[l * 3 + j] * s.px[k * NX + l];
            const double s1 = s.lam[r0] / s.t[r0], s2 = s.lam[r0 + 2] / s.t[r0 + 2];
            const double s3 = s.lam[r0 + 1] / s.t[r0 + 1], s4 = s.lam[r0 + 3] / s.t[r0 + 3];
            const double Zs = sk * A.Zl[j], zs = sk * A.zl[j];
            const double gl = zs - row_v(r0, phase, sigmu) - row_v(r0 + 2, phase, sigmu);
            const double gu = zs - row_v(r0 + 1, phase, sigmu) - row_v(r0 + 3, phase, sigmu);
            s.psl[e] = -(gl + s1 * cx) / (Zs + s1 + s2);
            s.psu[e] = -(gu - s3 * cx) / (Zs + s3 + s4);
        }
        __syncthreads();
    };

    // ---------------------------------------------------------------- IPM iterations
    int it = 0;
    double mu = 0.0, rp = 0.0;
    for (it = 0; it < A.max_iter; ++it) {
        double lmu = 0.0, lrp = 0.0;
        for (int r = lane; r < m; r += 64) {
            lmu += s.t[r] * s.lam[r];
            lrp = fmax(lrp, fabs(row_val(r, s.dx, s.du, s.sl, s.su) - s.t[r]));
        }
        mu = wave_sum(lmu, s.red, lane) / m;
        rp = wave_max(lrp, s.red, lane);
        if (mu < A.tol && rp < A.tol) break;
        // predictor
        backward(true, 0, 0.0);
        forward(0, 0.0);
        double amax = 1.0;
        for (int r = lane; r < m; r += 64) {
            const double t = s.t[r], l = s.lam[r];
            const double dt = row_val(r, s.px, s.pu, s.psl, s.psu) - t;
            const double dl = -(l / t) * dt - l;
            s.dta[r] = dt;
            s.dla[r] = dl;
            if (dt < 0.0) amax = fmin(amax, -t / dt);
            if (dl < 0.0) amax = fmin(amax, -l / dl);
        }
        const double aa = wave_min(amax, s.red, lane);
        double lmua = 0.0;
        for (int r = lane; r < m; r += 64) lmua += (s.t[r] + aa * s.dta[r]) * (s.lam[r] + aa * s.dla[r]);
        const double mua = wave_sum(lmua, s.red, lane) / m;
        const double sig = (mua / mu) * (mua / mu) * (mua / mu);
        const double sigmu = sig * mu;
        // corrector (same factorisation, new gradient)
        backward(false, 1, sigmu);
        forward(1, sigmu);
        amax = 1.0;
        for (int r = lane; r < m; r += 64) {
            const double t = s.t[r], l = s.lam[r];
            const double dt = row_val(r, s.px, s.pu, s.psl, s.psu) - t;
            const double dl = -(l / t) * dt - l - (s.dta[r] * s.dla[r] - sigmu) / t;
            s.dta[r] = dt;  // reuse as the final direction
            s.dla[r] = dl;
            if (dt < 0.0) amax = fmin(amax, -t / dt);
            if (dl < 0.0) amax = fmin(amax, -l / dl);
        }
        const double al = fmin(1.0, 0.995 * wave_min(amax, s.red, lane));
        for (int r = lane; r < m; r += 64) {
            s.t[r] += al * s.dta[r];
            s.lam[r] += al * s.dla[r];
        }
        for (int e = lane; e < N1 * NX; e += 64) s.dx[e] += al * (s.px[e] - s.dx[e]);
        for (int e = lane; e < N * NU; e += 64) s.du[e] += al * (s.pu[e] - s.du[e]);
        for (int e = lane; e < N1 * NS; e += 64) {
            s.sl[e] += al * (s.psl[e] - s.sl[e]);
            s.su[e] += al * (s.psu[e] - s.su[e]);
        }
        __syncthreads();
    }
    // ---------------------------------------------------------------- outputs
    for (int e = lane; e < N1 * NX; e += 64) A.dx[(size_t)b * N1 * NX + e] = s.dx[e];
    for (int e = lane; e < N * NU; e += 64) A.du[(size_t)b * N * NU + e] = s.du[e];
    if (A.slack)
        for (int e = lane; e < N1 * NS; e += 64) {
            A.slack[((size_t)b * N1 * NS + e) * 2] = s.sl[e];
            A.slack[((size_t)b * N1 * NS + e) * 2 + 1] = s.su[e];
        }
    if (lane == 0) {
        A.iters[b] = it;
        A.status[b] = (mu < A.tol && rp < A.tol) ? 0 : 1;  // 1: max_iter reached (acados status 2)
        A.res[b * 2] = mu;
        A.res[b * 2 + 1] = rp;
    }
}

__global__ __launch_bounds__(256) void rti_apply_kernel(int B, int N, double* x, double* u, const double* dx,
                                                       const double* du, double* u0) {
    const long long nx = (long long)B * (N + 1) * 10, nu = (long long)B * N * 4;
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nx) x[i] += dx[i];
    if (i < nu) {
        const double v = u[i] + du[i];
        u[i] = v;
        const long long bb = i / ((long long)N * 4), r = i - bb * N * 4;
        if (u0 && r < 4) u0[bb * 4 + r] = v;
    }
}

hipError_t launch_rti_apply(int B, int N, double* x, double* u, const double* dx, const double* du, double* u0,
                            hipStream_t s) {
    const long long n = (long long)B * (N + 1) * 10;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(rti_apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, B, N, x, u, dx, du, u0);
    return hipGetLastError();
}

hipError_t launch_rti_qp(const QpArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    const size_t lds = qp_lds_bytes(a.N);
    hipError_t e = hipFuncSetAttribute((const void*)rti_qp_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(rti_qp_kernel, dim3(a.B), dim3(64), lds, s, a);
    return hipGetLastError();
}

}  // namespace sdfn
