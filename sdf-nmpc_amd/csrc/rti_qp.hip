// SQP-RTI feedback phase: the OCP QP of every instance solved by a batched interior-point method.
//
// The QP is what acados builds from the preparation phase and hands to HPIPM (sdf_nmpc/ocp.py:54-120:
// NONLINEAR_LS + GAUSS_NEWTON, levenberg_marquardt, soft h constraints with L1/L2 slack penalties,
// input boxes, x_0 fixed), stated in oracle/qp_oracle.py.  The reference condenses it
// (FULL_CONDENSING_HPIPM) and runs a dense IPM; the solution is unique (lm > 0), so this build keeps
// the stage structure -- a Riccati recursion per Newton step, O(N (nx+nu)^3) -- and maps one
// instance to one wavefront:
//   * Mehrotra predictor-corrector on t = D z + d >= 0, lambda >= 0 (8 box rows per stage,
//     4 rows (h-lower, h-upper, sl >= 0, su >= 0) per soft constraint and node)
//   * each Newton system is an LQR in the new iterate z+ with Hessian H + D^T Sigma D and gradient
//     g - D^T v (v folds the residuals), so dynamics hold exactly and no costate is carried
//   * soft-constraint slacks (diagonal Hessian) are eliminated per row: a rank-3 update of the
//     node's state block; recovered in closed form after each sweep
//   * one factorisation per iteration serves predictor and corrector:
//       Y = L^-1 S, P <- Q^ - Y^T Y, p <- m_x - Y^T (L^-1 m_u), K = -L^-T Y, k = -L^-T L^-1 m_u
//     with L = chol(R^); the corrector and forward sweeps reuse (Y, L) and P_{k+1}
// Memory: per-stage records [A B | c | g | C | H] are packed once per solve into a global workspace
// and streamed through registers one stage ahead of the sweep (statically indexed: a runtime-indexed
// ring would live in scratch); iterate, slacks and
// duals live in LDS (< 40 KB: 4 instances per CU, one round for B = 1024).  Residuals are tracked
// incrementally (r_p <- (1 - alpha) r_p) and the affine deltas are recomputed, not stored.
#include <hip/hip_runtime.h>

#include "qp_kernels.h"

namespace sdfn {

namespace {

// LDS pointers must keep address space 3: a generic pointer compiles to flat_load/store, whose waits
// (vmcnt(0) AND lgkmcnt(0)) drain every global prefetch in flight at each LDS access.
typedef __attribute__((address_space(3))) double ldsd;

constexpr int NX = 10, NU = 4, NS = 3;
// stage record (doubles): [AB 140 | c 10 | g 14 | C 30 | H 105 (upper triangle, row-major)] -> 300
constexpr int R_AB = 0, R_C = 140, R_G = 150, R_CH = 164, R_H = 194, REC = QP_REC;
constexpr int PF_REC = (REC + 63) / 64;  // prefetch registers per lane per record
// factor record: [Y 40 (4x10 row-major) | L 10 (lower packed) | kff 4 | P_{k+1} 55 (upper)] -> 110
constexpr int F_Y = 0, F_L = 40, F_K = 50, F_P = 54, FREC = QP_FREC;
constexpr int PF_F = (FREC + 63) / 64;

__device__ __forceinline__ int tri10(int a, int c) { return a * 10 - a * (a - 1) / 2 + (c - a); }  // a <= c
__device__ __forceinline__ int ltri4(int i, int j) { return i * (i + 1) / 2 + j; }                  // j <= i

__device__ __forceinline__ double wsum(double v) {
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}
__device__ __forceinline__ double wmax(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
    return v;
}
__device__ __forceinline__ double wmin(double v) {
    for (int o = 32; o > 0; o >>= 1) v = fmin(v, __shfl_xor(v, o));
    return v;
}

struct Smem {
    ldsd *t, *lam;                  // [m] inequality slacks / duals
    ldsd *dx, *du, *sl, *su, *cx;   // iterate z and cx[k][j] = C_j dx_k
    ldsd *dua, *cxa;                // affine (predictor) solution: du, C dx
    ldsd *dxc, *duc, *cxc;          // corrector solution (dxc is also the predictor sweep buffer)
    ldsd *rec0, *rec1;              // stage record double buffer
    ldsd *frc0, *frc1;              // factor record double buffer (corrector / forward sweeps)
    ldsd *P0, *P1, *p0, *p1;        // Riccati P (full 10x10) / p ping-pong
    ldsd *W, *M, *m, *Pb, *fold;    // stage scratch; fold: node's soft rows [w_j, gamma_j]
};

__device__ __forceinline__ Smem carve(ldsd* q, int N) {
    Smem s;
    auto take = [&](int n) { ldsd* r = q; q += n; return r; };
    const int m = 8 * N + 12 * (N + 1), N1 = N + 1;
    s.t = take(m); s.lam = take(m);
    s.dx = take(N1 * NX); s.du = take(N * NU); s.sl = take(N1 * NS); s.su = take(N1 * NS); s.cx = take(N1 * NS);
    s.dua = take(N * NU); s.cxa = take(N1 * NS);
    s.dxc = take(N1 * NX); s.duc = take(N * NU); s.cxc = take(N1 * NS);
    s.rec0 = take(REC); s.rec1 = take(REC);
    s.frc0 = take(FREC); s.frc1 = take(FREC);
    s.P0 = take(100); s.P1 = take(100); s.p0 = take(10); s.p1 = take(10);
    s.W = take(140); s.M = take(196); s.m = take(14); s.Pb = take(10); s.fold = take(6);
    return s;
}

}  // namespace

#ifdef QP_STAMPS  // diagnostic build only: per-phase cycle accounting (never in the product build)
#define STAMP_DECL long long st_t0 = clock64(), st_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define STAMP(i) do { const long long t1_ = clock64(); st_acc[i] += t1_ - st_t0; st_t0 = t1_; } while (0)
#define STAMP_OUT if (lane == 0 && A.stamps) for (int i_ = 0; i_ < 8; ++i_) A.stamps[(size_t)b * 8 + i_] = (double)st_acc[i_];
#else
#define STAMP_DECL
#define STAMP(i)
#define STAMP_OUT
#endif

__global__ __launch_bounds__(64) void rti_qp_kernel(QpArgs A) {
    extern __shared__ __align__(16) double lds_q[];
    STAMP_DECL
    const int b = blockIdx.x, lane = threadIdx.x;
    const int N = A.N, N1 = N + 1, m = 8 * N + 12 * N1;
    Smem s = carve((ldsd*)lds_q, N);
    double* R = A.work + (size_t)b * qp_work_doubles(N);  // [N+1][REC] stage records
    double* F = R + (size_t)N1 * REC;                     // [N+1][FREC] factor records
    const double* ub = A.u + (size_t)b * N * 4;
    const double* hh = A.h + (size_t)b * N1 * 3;

    // ------------------------------------------------------------ setup: pack the stage records
    // (AB, c = xn_k - xbar_{k+1}, g, C = J_h, H = s_k J^T W J + lm I upper triangle); terminal:
    // H_N = J_N^T W_N J_N + lm I (10x10 upper in the H field), g_N (first 10 of g), C_N.
    for (int k = 0; k < N1; ++k) {
        double* Rk = R + (size_t)k * REC;
        const double sk = (A.cost_scaling && k < N) ? A.dt[k] : 1.0;
        const double* Jh = A.Jh + ((size_t)b * N1 + k) * 30;
        if (k < N) {
            const double* AB = A.AB + ((size_t)b * N + k) * 140;
            const double* J = A.Jy + ((size_t)b * N + k) * 154;
            const double* Wk = A.W + ((size_t)b * N + k) * 11;
            const double* yk = A.y + ((size_t)b * N + k) * 11;
            const double* rk = A.yref + ((size_t)b * N + k) * 11;
            const double* xn = A.xn + ((size_t)b * N + k) * 10;
            const double* xb1 = A.x + ((size_t)b * N1 + k + 1) * 10;
            for (int e = lane; e < REC; e += 64) {
                double v = 0.0;
                if (e < R_C) {
                    v = AB[e];
                } else if (e < R_G) {
                    v = xn[e - R_C] - xb1[e - R_C];
                } else if (e < R_CH) {
                    const int a = e - R_G;
                    for (int i = 0; i < 11; ++i) v += J[a * 11 + i] * Wk[i] * (yk[i] - rk[i]);
                    v *= sk;
                } else if (e < R_H) {
                    v = Jh[e - R_CH];
                } else if (e < R_H + 105) {
                    int q = e - R_H, a = 0;
                    while (q >= 14 - a) { q -= 14 - a; ++a; }
                    const int c = a + q;
                    for (int i = 0; i < 11; ++i) v += J[a * 11 + i] * Wk[i] * J[c * 11 + i];
                    v = sk * v + (a == c ? A.lm : 0.0);
                }
                Rk[e] = v;
            }
        } else {
            const double* J = A.JyN + (size_t)b * 40;  // [10][4]
            const double* Wn = A.WN + (size_t)b * 4;
            const double* yn = A.yN + (size_t)b * 4;
            const double* rn = A.yNref + (size_t)b * 4;
            for (int e = lane; e < REC; e += 64) {
                double v = 0.0;
                if (e >= R_G && e < R_G + 10) {
                    const int a = e - R_G;
                    for (int i = 0; i < 4; ++i) v += J[a * 4 + i] * Wn[i] * (yn[i] - rn[i]);
                } else if (e >= R_CH && e < R_H) {
                    v = Jh[e - R_CH];
                } else if (e >= R_H && e < R_H + 55) {
                    int q = e - R_H, a = 0;
                    while (q >= 10 - a) { q -= 10 - a; ++a; }
                    const int c = a + q;
                    for (int i = 0; i < 4; ++i) v += J[a * 4 + i] * Wn[i] * J[c * 4 + i];
                    v += (a == c ? A.lm : 0.0);
                }
                Rk[e] = v;
            }
        }
    }
    __syncthreads();  // records are re-read below by other lanes of this wave (same CU: L1/L2 coherent)
    STAMP(0);

    // ------------------------------------------------------------ record streaming (register ring)
    double nxt[PF_REC];  // record in flight (filled one stage ahead; static indexing keeps it in VGPRs)
    auto fetch = [&](double* dst, int k, int n) {
        const double* src = R + (size_t)k * REC;
#pragma unroll
        for (int i = 0; i < PF_REC; ++i) {
            const int e = lane + 64 * i;
            dst[i] = (e < n) ? src[e] : 0.0;
        }
    };
    auto commit = [&](ldsd* lds, const double* reg, int n) {
#pragma unroll
        for (int i = 0; i < PF_REC; ++i) {
            const int e = lane + 64 * i;
            if (e < n) lds[e] = reg[i];
        }
    };
    double fnxt[PF_F];
    auto ffetch = [&](double* dst, int k, int n) {
        const double* src = F + (size_t)k * FREC;
#pragma unroll
        for (int i = 0; i < PF_F; ++i) {
            const int e = lane + 64 * i;
            dst[i] = (e < n) ? src[e] : 0.0;
        }
    };
    auto fcommit = [&](ldsd* lds, const double* reg, int n) {
#pragma unroll
        for (int i = 0; i < PF_F; ++i) {
            const int e = lane + 64 * i;
            if (e < n) lds[e] = reg[i];
        }
    };

    // ------------------------------------------------------------ initial iterate (dynamics-feasible):
    // du = sl = su = 0, dx_0 = x0 - xbar_0, dx_{k+1} = A dx_k + c_k, cx = C dx
    for (int e = lane; e < N * NU; e += 64) s.du[e] = 0.0;
    for (int e = lane; e < N1 * NS; e += 64) { s.sl[e] = 0.0; s.su[e] = 0.0; }
    if (lane < NX) s.dx[lane] = A.x0[(size_t)b * 10 + lane] - A.x[(size_t)b * N1 * 10 + lane];
    fetch(nxt, 0, R_H);
    __syncthreads();
    for (int k = 0; k < N1; ++k) {
        ldsd* rk = (k & 1) ? s.rec1 : s.rec0;
        commit(rk, nxt, R_H);
        if (k + 1 < N1) fetch(nxt, k + 1, R_H);
        __syncthreads();
        if (lane < NX && k < N) {
            double v = rk[R_C + lane];
            for (int j = 0; j < NX; ++j) v += rk[R_AB + j * 10 + lane] * s.dx[k * NX + j];
            s.dx[(k + 1) * NX + lane] = v;
        }
        if (lane >= 16 && lane < 16 + NS) {
            const int j = lane - 16;
            double v = 0.0;
            for (int l = 0; l < NX; ++l) v += rk[R_CH + l * 3 + j] * s.dx[k * NX + l];
            s.cx[k * NS + j] = v;
        }
        __syncthreads();
    }

    // box rows (k, i, up): t = +-du + d, d = (u - lbu) | (ubu - u)
    auto box_d = [&](int k, int i, int up) -> double {
        const double u = ub[k * 4 + i];
        return up ? A.ubu[i] - u : u - A.lbu[i];
    };
    double rp = 0.0;
    for (int r = lane; r < m; r += 64) {
        double v;
        if (r < 8 * N) {
            const int k = r >> 3, q = r & 7, i = q & 3, up = q >> 2;
            v = (up ? -s.du[k * NU + i] : s.du[k * NU + i]) + box_d(k, i, up);
        } else {
            const int q = r - 8 * N, k = q / 12, w = q - 12 * k, j = w >> 2, kind = w & 3;
            const double h = hh[k * 3 + j];
            v = kind == 0 ? s.cx[k * NS + j] + (h - A.lh[j]) + s.sl[k * NS + j]
              : kind == 1 ? -s.cx[k * NS + j] + (A.uh[j] - h) + s.su[k * NS + j]
              : kind == 2 ? s.sl[k * NS + j] : s.su[k * NS + j];
        }
        const double t = fmax(v, 1.0);
        s.t[r] = t;
        s.lam[r] = 1.0;
        rp = fmax(rp, fabs(v - t));
    }
    rp = wmax(rp);
    __syncthreads();
    STAMP(1);

    // soft group (k, j) = rows (hl, hu, sl, su): barrier weights, v's, eliminated slack block
    struct Grp {
        double s1, s2, s3, s4, v1, v2, v3, v4, Hl, Hu, gl, gu;
    };
    auto group = [&](int k, int j, int phase, double sigmu) -> Grp {
        Grp g;
        const int r0 = 8 * N + 12 * k + 4 * j;
        const double sk = (A.cost_scaling && k < N) ? A.dt[k] : 1.0;
        const double t1 = s.t[r0], t2 = s.t[r0 + 1], t3 = s.t[r0 + 2], t4 = s.t[r0 + 3];
        const double l1 = s.lam[r0], l2 = s.lam[r0 + 1], l3 = s.lam[r0 + 2], l4 = s.lam[r0 + 3];
        g.s1 = l1 / t1; g.s3 = l2 / t2; g.s2 = l3 / t3; g.s4 = l4 / t4;
        const double h = hh[k * 3 + j];
        g.v1 = g.s1 * (t1 - (h - A.lh[j]));
        g.v3 = g.s3 * (t2 - (A.uh[j] - h));
        g.v2 = g.s2 * t3;
        g.v4 = g.s4 * t4;
        const double Zs = sk * A.Zl[j], zs = sk * A.zl[j];
        g.Hl = Zs + g.s1 + g.s2;
        g.Hu = Zs + g.s3 + g.s4;
        if (phase) {  // corrector: affine deltas of the four rows, recomputed from the affine solution
            const double cxa = s.cxa[k * NS + j];
            const double sla = -((zs - g.v1 - g.v2) + g.s1 * cxa) / g.Hl;
            const double sua = -((zs - g.v3 - g.v4) - g.s3 * cxa) / g.Hu;
            const double d1 = cxa + (h - A.lh[j]) + sla - t1;
            const double d2 = -cxa + (A.uh[j] - h) + sua - t2;
            const double d3 = sla - t3, d4 = sua - t4;
            g.v1 -= (d1 * (-g.s1 * d1 - l1) - sigmu) / t1;
            g.v3 -= (d2 * (-g.s3 * d2 - l2) - sigmu) / t2;
            g.v2 -= (d3 * (-g.s2 * d3 - l3) - sigmu) / t3;
            g.v4 -= (d4 * (-g.s4 * d4 - l4) - sigmu) / t4;
        }
        g.gl = zs - g.v1 - g.v2;
        g.gu = zs - g.v3 - g.v4;
        return g;
    };
    auto box_v = [&](int k, int i, int up, int phase, double sigmu) -> double {
        const int r = 8 * k + 4 * up + i;
        const double t = s.t[r], l = s.lam[r], sg = l / t;
        double v = sg * (t - box_d(k, i, up));
        if (phase) {
            const double da = (up ? -s.dua[k * NU + i] : s.dua[k * NU + i]) + box_d(k, i, up) - t;
            v -= (da * (-sg * da - l) - sigmu) / t;
        }
        return v;
    };
    auto fold_node = [&](int k, int phase, double sigmu) {  // lanes 0..2: soft rows of node k
        if (lane < NS) {
            const Grp g = group(k, lane, phase, sigmu);
            s.fold[lane] = g.s1 * (g.Hl - g.s1) / g.Hl + g.s3 * (g.Hu - g.s3) / g.Hu;
            s.fold[3 + lane] = -(g.v1 + g.s1 * g.gl / g.Hl) + (g.v3 + g.s3 * g.gu / g.Hu);
        }
    };

    // ------------------------------------------------------------ backward sweep
    // factor: factorisation + predictor gradient (3 barriers per stage);
    // corrector: stored factors + corrector gradient (1 barrier per stage)
    auto backward = [&](bool factor, int phase, double sigmu) {
        const int nrec = factor ? REC : R_H;
        int cur = 0;
        fetch(nxt, N, REC);
        fold_node(N, phase, sigmu);
        commit(s.rec0, nxt, REC);
        fetch(nxt, N - 1, nrec);
        if (!factor) ffetch(fnxt, N - 1, FREC);
        __syncthreads();
        {  // terminal node: P_N = H_N + sum_j w_j C_j^T C_j, p_N = g_N + sum_j gamma_j C_j^T
            const ldsd* rN = s.rec0;
            for (int e = lane; e < 110; e += 64) {
                if (e < 100) {
                    if (!factor) continue;
                    const int a = e / 10, c = e % 10;
                    double v = rN[R_H + tri10(a < c ? a : c, a < c ? c : a)];
                    for (int j = 0; j < NS; ++j) v += s.fold[j] * rN[R_CH + a * 3 + j] * rN[R_CH + c * 3 + j];
                    s.P0[e] = v;
                } else {
                    const int a = e - 100;
                    double v = rN[R_G + a];
                    for (int j = 0; j < NS; ++j) v += s.fold[3 + j] * rN[R_CH + a * 3 + j];
                    s.p0[a] = v;
                }
            }
        }
        __syncthreads();
        for (int k = N - 1; k >= 0; --k) {
            const int slot = (N - k) & 1;
            ldsd* rk = slot ? s.rec1 : s.rec0;
            ldsd* fk = slot ? s.frc1 : s.frc0;
            commit(rk, nxt, nrec);
            if (!factor) fcommit(fk, fnxt, FREC);
            if (k >= 1) {
                fetch(nxt, k - 1, nrec);
                if (!factor) ffetch(fnxt, k - 1, FREC);
            }
            fold_node(k, phase, sigmu);
            __syncthreads();
            const ldsd* Pk1 = cur ? s.P1 : s.P0;
            const ldsd* pk1 = cur ? s.p1 : s.p0;
            ldsd* pn = cur ? s.p0 : s.p1;
            if (factor) {
                // ---- step 1: W = P [A B] (10 x 14), Pb = P c + p
                for (int e = lane; e < 150; e += 64) {
                    if (e < 140) {
                        const int i = e / 14, j = e % 14;
                        double acc = 0.0;
#pragma unroll
                        for (int l = 0; l < NX; ++l) acc += Pk1[i * 10 + l] * rk[R_AB + j * 10 + l];
                        s.W[e] = acc;
                    } else {
                        const int i = e - 140;
                        double acc = pk1[i];
#pragma unroll
                        for (int l = 0; l < NX; ++l) acc += Pk1[i * 10 + l] * rk[R_C + l];
                        s.Pb[i] = acc;
                    }
                }
                __syncthreads();
                // ---- step 2: M = H~ + [A B]^T W (from the upper triangle), m = g~ + [A B]^T Pb
                for (int e = lane; e < 119; e += 64) {
                    if (e < 105) {
                        int q = e, a = 0;
                        while (q >= 14 - a) { q -= 14 - a; ++a; }
                        const int c = a + q;
                        double v = rk[R_H + e];
#pragma unroll
                        for (int l = 0; l < NX; ++l) v += rk[R_AB + a * 10 + l] * s.W[l * 14 + c];
                        if (c < NX) {
                            for (int j = 0; j < NS; ++j) v += s.fold[j] * rk[R_CH + a * 3 + j] * rk[R_CH + c * 3 + j];
                        } else if (a == c) {
                            const int r0 = 8 * k + (a - NX);
                            v += s.lam[r0] / s.t[r0] + s.lam[r0 + 4] / s.t[r0 + 4];
                        }
                        s.M[a * 14 + c] = v;
                        s.M[c * 14 + a] = v;
                    } else {
                        const int a = e - 105;
                        double v = rk[R_G + a];
#pragma unroll
                        for (int l = 0; l < NX; ++l) v += rk[R_AB + a * 10 + l] * s.Pb[l];
                        if (a < NX) {
                            for (int j = 0; j < NS; ++j) v += s.fold[3 + j] * rk[R_CH + a * 3 + j];
                        } else {
                            const int i = a - NX;
                            v += -box_v(k, i, 0, phase, sigmu) + box_v(k, i, 1, phase, sigmu);
                        }
                        s.m[a] = v;
                    }
                }
                __syncthreads();
                // ---- step 3: L = chol(R^) (every lane, registers), y_a = L^-1 S[:, a], w = L^-1 m_u;
                //      P_k = Q^ - Y^T Y, p_k = m_x - Y^T w; factor record (Y, L, k_ff, P_{k+1})
                double L[4][4];
#pragma unroll
                for (int i = 0; i < 4; ++i)
#pragma unroll
                    for (int j = 0; j <= i; ++j) {
                        double v = s.M[(NX + i) * 14 + NX + j];
#pragma unroll
                        for (int q = 0; q < j; ++q) v -= L[i][q] * L[j][q];
                        L[i][j] = (i == j) ? sqrt(v) : v / L[j][j];
                    }
                // y = L^-1 col (forward substitution with the reciprocal diagonal)
                const double id0 = 1.0 / L[0][0], id1 = 1.0 / L[1][1], id2 = 1.0 / L[2][2], id3 = 1.0 / L[3][3];
#define FSUB(col, stride, y)                                                                  \
    do {                                                                                      \
        y[0] = (col)[0] * id0;                                                                \
        y[1] = ((col)[(stride)] - L[1][0] * y[0]) * id1;                                      \
        y[2] = ((col)[2 * (stride)] - L[2][0] * y[0] - L[2][1] * y[1]) * id2;                 \
        y[3] = ((col)[3 * (stride)] - L[3][0] * y[0] - L[3][1] * y[1] - L[3][2] * y[2]) * id3; \
    } while (0)
                double w[4];
                FSUB(s.m + NX, 1, w);
                ldsd* Pn = cur ? s.P0 : s.P1;
                double* Fk = F + (size_t)k * FREC;
                for (int e = lane; e < 110; e += 64) {
                    if (e < 100) {
                        const int a = e / 10, c = e % 10;
                        double ya[4], yc[4];
                        FSUB(s.M + NX * 14 + a, 14, ya);
                        FSUB(s.M + NX * 14 + c, 14, yc);
                        double v = s.M[a * 14 + c];
#pragma unroll
                        for (int i = 0; i < 4; ++i) v -= ya[i] * yc[i];
                        Pn[e] = v;
                        if (a <= c) Fk[F_P + tri10(a, c)] = Pk1[e];
                        if (a == 0) {
#pragma unroll
                            for (int i = 0; i < 4; ++i) Fk[F_Y + i * 10 + c] = yc[i];
                        }
                    } else {
                        const int a = e - 100;
                        double ya[4];
                        FSUB(s.M + NX * 14 + a, 14, ya);
                        double v = s.m[a];
#pragma unroll
                        for (int i = 0; i < 4; ++i) v -= ya[i] * w[i];
                        pn[a] = v;
                    }
                }
                if (lane == 0) {
#pragma unroll
                    for (int i = 0; i < 4; ++i)
#pragma unroll
                        for (int j = 0; j <= i; ++j) Fk[F_L + ltri4(i, j)] = L[i][j];
                }
                if (lane >= 48 && lane < 52) {  // k_ff = -L^-T w
                    double kf[4];
#pragma unroll
                    for (int i = 3; i >= 0; --i) {
                        double v = w[i];
#pragma unroll
                        for (int q = i + 1; q < 4; ++q) v -= L[q][i] * kf[q];
                        kf[i] = v / L[i][i];
                    }
                    Fk[F_K + lane - 48] = -kf[lane - 48];
                }
#undef FSUB
            } else {
                // ---- corrector: every lane forms Pb = P_{k+1} c + p and m_u, w = L^-1 m_u;
                //      lane a < 10: p_k[a] = m_x[a] - Y[:, a]^T w; lanes 16..19: k_ff = -L^-T w
                const ldsd* Pf = fk + F_P;
                double Pb[NX];
#pragma unroll
                for (int i = 0; i < NX; ++i) {
                    double acc = pk1[i];
#pragma unroll
                    for (int l = 0; l < NX; ++l) acc += Pf[tri10(i < l ? i : l, i < l ? l : i)] * rk[R_C + l];
                    Pb[i] = acc;
                }
                double w[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    double v = rk[R_G + NX + i];
#pragma unroll
                    for (int l = 0; l < NX; ++l) v += rk[R_AB + (NX + i) * 10 + l] * Pb[l];
                    v += -box_v(k, i, 0, phase, sigmu) + box_v(k, i, 1, phase, sigmu);
#pragma unroll
                    for (int q = 0; q < i; ++q) v -= fk[F_L + ltri4(i, q)] * w[q];
                    w[i] = v / fk[F_L + ltri4(i, i)];
                }
                if (lane < NX) {
                    const int a = lane;
                    double v = rk[R_G + a];
#pragma unroll
                    for (int l = 0; l < NX; ++l) v += rk[R_AB + a * 10 + l] * Pb[l];
                    for (int j = 0; j < NS; ++j) v += s.fold[3 + j] * rk[R_CH + a * 3 + j];
#pragma unroll
                    for (int i = 0; i < 4; ++i) v -= fk[F_Y + i * 10 + a] * w[i];
                    pn[a] = v;
                }
                if (lane >= 16 && lane < 20) {
                    double kf[4];
#pragma unroll
                    for (int i = 3; i >= 0; --i) {
                        double v = w[i];
#pragma unroll
                        for (int q = i + 1; q < 4; ++q) v -= fk[F_L + ltri4(q, i)] * kf[q];
                        kf[i] = v / fk[F_L + ltri4(i, i)];
                    }
                    F[(size_t)k * FREC + F_K + lane - 16] = -kf[lane - 16];
                }
            }
            cur ^= 1;
            __syncthreads();
        }
    };

    // ------------------------------------------------------------ forward sweep (1 barrier per stage)
    // u_k = k_ff - L^-T (Y x_k), x_{k+1} = A x_k + B u_k + c_k; cx = C x
    auto forward = [&](ldsd* dxo, ldsd* duo, ldsd* cxo) {
        if (lane < NX) dxo[lane] = s.dx[lane];
        fetch(nxt, 0, R_H);
        ffetch(fnxt, 0, F_P);
        for (int k = 0; k < N1; ++k) {
            ldsd* rk = (k & 1) ? s.rec1 : s.rec0;
            ldsd* fk = (k & 1) ? s.frc1 : s.frc0;
            commit(rk, nxt, R_H);
            fcommit(fk, fnxt, F_P);
            if (k + 1 < N1) {
                fetch(nxt, k + 1, R_H);
                ffetch(fnxt, k + 1, F_P);
            }
            __syncthreads();
            const ldsd* x = dxo + k * NX;
            if (lane >= 16 && lane < 16 + NS) {
                const int j = lane - 16;
                double v = 0.0;
#pragma unroll
                for (int l = 0; l < NX; ++l) v += rk[R_CH + l * 3 + j] * x[l];
                cxo[k * NS + j] = v;
            }
            if (k < N && lane < NX) {
                double yx[4], u[4];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    double v = 0.0;
#pragma unroll
                    for (int l = 0; l < NX; ++l) v += fk[F_Y + i * 10 + l] * x[l];
                    yx[i] = v;
                }
#pragma unroll
                for (int i = 3; i >= 0; --i) {
                    double v = yx[i];
#pragma unroll
                    for (int q = i + 1; q < 4; ++q) v -= fk[F_L + ltri4(q, i)] * u[q];
                    u[i] = v / fk[F_L + ltri4(i, i)];
                }
#pragma unroll
                for (int i = 0; i < 4; ++i) u[i] = fk[F_K + i] - u[i];
                double v = rk[R_C + lane];
#pragma unroll
                for (int j = 0; j < NX; ++j) v += rk[R_AB + j * 10 + lane] * x[j];
#pragma unroll
                for (int i = 0; i < 4; ++i) v += rk[R_AB + (NX + i) * 10 + lane] * u[i];
                dxo[(k + 1) * NX + lane] = v;
                if (lane < 4) duo[k * NU + lane] = u[lane];
            }
            __syncthreads();
        }
    };

    // row values of a soft group (k, j) at an LQR solution with C dx = cxs, and its slacks
    auto soft_vals = [&](const Grp& g, int k, int j, double cxs, double* v, double* slo, double* suo) {
        const double h = hh[k * 3 + j];
        const double sl = -(g.gl + g.s1 * cxs) / g.Hl, su = -(g.gu - g.s3 * cxs) / g.Hu;
        v[0] = cxs + (h - A.lh[j]) + sl;
        v[1] = -cxs + (A.uh[j] - h) + su;
        v[2] = sl;
        v[3] = su;
        if (slo) *slo = sl;
        if (suo) *suo = su;
    };

    // ------------------------------------------------------------ IPM iterations
    int it = 0;
    double mu;
    {
        double lmu = 0.0;
        for (int r = lane; r < m; r += 64) lmu += s.t[r] * s.lam[r];
        mu = wsum(lmu) / m;
    }
    for (it = 0; it < A.max_iter; ++it) {
        if (mu < A.tol && rp < A.tol) break;
        // -------- predictor: factorise, solve, affine step length and mu_aff
        STAMP(7);
        backward(true, 0, 0.0);
        STAMP(2);
        forward(s.dxc, s.dua, s.cxa);
        STAMP(3);
        double amax = 1.0;
        auto bound = [&](double t, double l, double dt, double dl) {
            if (dt < 0.0) amax = fmin(amax, -t / dt);
            if (dl < 0.0) amax = fmin(amax, -l / dl);
        };
        for (int r = lane; r < 8 * N; r += 64) {
            const int k = r >> 3, q = r & 7, i = q & 3, up = q >> 2;
            const double t = s.t[r], l = s.lam[r];
            const double dt = (up ? -s.dua[k * NU + i] : s.dua[k * NU + i]) + box_d(k, i, up) - t;
            bound(t, l, dt, -(l / t) * dt - l);
        }
        for (int e = lane; e < N1 * NS; e += 64) {
            const int k = e / NS, j = e % NS, r0 = 8 * N + 12 * k + 4 * j;
            const Grp g = group(k, j, 0, 0.0);
            double v[4];
            soft_vals(g, k, j, s.cxa[e], v, nullptr, nullptr);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double t = s.t[r0 + q], l = s.lam[r0 + q], dt = v[q] - t;
                bound(t, l, dt, -(l / t) * dt - l);
            }
        }
        const double aa = wmin(amax);
        double lmua = 0.0;
        for (int r = lane; r < 8 * N; r += 64) {
            const int k = r >> 3, q = r & 7, i = q & 3, up = q >> 2;
            const double t = s.t[r], l = s.lam[r];
            const double dt = (up ? -s.dua[k * NU + i] : s.dua[k * NU + i]) + box_d(k, i, up) - t;
            lmua += (t + aa * dt) * (l + aa * (-(l / t) * dt - l));
        }
        for (int e = lane; e < N1 * NS; e += 64) {
            const int k = e / NS, j = e % NS, r0 = 8 * N + 12 * k + 4 * j;
            const Grp g = group(k, j, 0, 0.0);
            double v[4];
            soft_vals(g, k, j, s.cxa[e], v, nullptr, nullptr);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double t = s.t[r0 + q], l = s.lam[r0 + q], dt = v[q] - t;
                lmua += (t + aa * dt) * (l + aa * (-(l / t) * dt - l));
            }
        }
        const double mua = wsum(lmua) / m;
        const double sig = (mua / mu) * (mua / mu) * (mua / mu);
        const double sigmu = sig * mu;
        // -------- corrector: same factorisation, new gradient
        STAMP(4);
        backward(false, 1, sigmu);
        STAMP(5);
        forward(s.dxc, s.duc, s.cxc);
        STAMP(3);
        // direction of row r: dt = val(z_c) - t, dl = -sigma dt - l - (dt_a dl_a - sigma mu) / t
        amax = 1.0;
        for (int r = lane; r < 8 * N; r += 64) {
            const int k = r >> 3, q = r & 7, i = q & 3, up = q >> 2;
            const double t = s.t[r], l = s.lam[r];
            const double dt = (up ? -s.duc[k * NU + i] : s.duc[k * NU + i]) + box_d(k, i, up) - t;
            const double dta = (up ? -s.dua[k * NU + i] : s.dua[k * NU + i]) + box_d(k, i, up) - t;
            bound(t, l, dt, -(l / t) * dt - l - (dta * (-(l / t) * dta - l) - sigmu) / t);
        }
        for (int e = lane; e < N1 * NS; e += 64) {
            const int k = e / NS, j = e % NS, r0 = 8 * N + 12 * k + 4 * j;
            const Grp ga = group(k, j, 0, 0.0), gc = group(k, j, 1, sigmu);
            double va[4], vc[4];
            soft_vals(ga, k, j, s.cxa[e], va, nullptr, nullptr);
            soft_vals(gc, k, j, s.cxc[e], vc, nullptr, nullptr);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double t = s.t[r0 + q], l = s.lam[r0 + q];
                const double dta = va[q] - t, dt = vc[q] - t;
                bound(t, l, dt, -(l / t) * dt - l - (dta * (-(l / t) * dta - l) - sigmu) / t);
            }
        }
        const double al = fmin(1.0, 0.995 * wmin(amax));
        // -------- update (rows read everything they need before writing their own entries)
        double lmu = 0.0;
        for (int r = lane; r < 8 * N; r += 64) {
            const int k = r >> 3, q = r & 7, i = q & 3, up = q >> 2;
            const double t = s.t[r], l = s.lam[r];
            const double dt = (up ? -s.duc[k * NU + i] : s.duc[k * NU + i]) + box_d(k, i, up) - t;
            const double dta = (up ? -s.dua[k * NU + i] : s.dua[k * NU + i]) + box_d(k, i, up) - t;
            const double dl = -(l / t) * dt - l - (dta * (-(l / t) * dta - l) - sigmu) / t;
            const double tn = t + al * dt, ln = l + al * dl;
            lmu += tn * ln;
            s.t[r] = tn;
            s.lam[r] = ln;
        }
        for (int e = lane; e < N1 * NS; e += 64) {
            const int k = e / NS, j = e % NS, r0 = 8 * N + 12 * k + 4 * j;
            const Grp ga = group(k, j, 0, 0.0), gc = group(k, j, 1, sigmu);
            double va[4], vc[4], slc, suc;
            soft_vals(ga, k, j, s.cxa[e], va, nullptr, nullptr);
            soft_vals(gc, k, j, s.cxc[e], vc, &slc, &suc);
            double tn[4], ln[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double t = s.t[r0 + q], l = s.lam[r0 + q];
                const double dta = va[q] - t, dt = vc[q] - t;
                const double dl = -(l / t) * dt - l - (dta * (-(l / t) * dta - l) - sigmu) / t;
                tn[q] = t + al * dt;
                ln[q] = l + al * dl;
                lmu += tn[q] * ln[q];
            }
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                s.t[r0 + q] = tn[q];
                s.lam[r0 + q] = ln[q];
            }
            s.sl[e] += al * (slc - s.sl[e]);
            s.su[e] += al * (suc - s.su[e]);
            s.cx[e] += al * (s.cxc[e] - s.cx[e]);
        }
        for (int e = lane; e < N1 * NX; e += 64) s.dx[e] += al * (s.dxc[e] - s.dx[e]);
        for (int e = lane; e < N * NU; e += 64) s.du[e] += al * (s.duc[e] - s.du[e]);
        mu = wsum(lmu) / m;
        rp *= (1.0 - al);
        __syncthreads();
        STAMP(6);
    }
    STAMP_OUT
    // ------------------------------------------------------------ outputs
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
