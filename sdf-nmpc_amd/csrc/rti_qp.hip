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
//     node's state block; these folds and the box terms are formed for all nodes in one parallel
//     pass before each sweep, so the serial sweeps hold no division
//   * one factorisation per iteration serves predictor and corrector:
//       Y = L^-1 S, P <- Q^ - Y^T Y, p <- m_x - Y^T (L^-1 m_u), K = -L^-T Y, k = -L^-T L^-1 m_u
//     with L = chol(R^) (rsq + Newton; the reciprocal diagonal is what is stored)
// Memory: rti_qp_pack_kernel packs per-stage records [A B | c | g | C | H] into a global workspace
// (a wide launch, one block per stage).  Each IPM iteration then walks the records in a fixed order
// -- backward (factor), forward, backward (corrector), forward -- so they form one stream that is
// prefetched QP_RING records ahead through registers, across sweep boundaries.  Iterate, duals and
// stage scratch live in LDS (< 40 KB at N = 40: 4 instances per CU, one round for B = 1024).
#include <hip/hip_runtime.h>

#include "qp_kernels.h"

namespace sdfn {

namespace {

// LDS pointers must keep address space 3: a generic pointer compiles to flat_load/store, whose waits
// (vmcnt(0) AND lgkmcnt(0)) drain every global prefetch in flight at each LDS access.
typedef __attribute__((address_space(3))) double ldsd;

constexpr int NX = 10, NU = 4, NS = 3;
// stage record (doubles): [AB 140 (column j = d xn / d (x,u)_j) | c 10 | g 14 | C 30 | H 105 upper]
constexpr int R_AB = 0, R_C = 140, R_G = 150, R_CH = 164, R_H = 194, REC = QP_REC;
constexpr int RR = (REC + 63) / 64;  // prefetch registers per lane per record
// factor record: [Y 40 (4x10 row-major) | L 10 (lower packed, diagonal holds 1/L_ii) | kff 4 | P c 10]
constexpr int F_Y = 0, F_L = 40, F_K = 50, F_PC = 54, FREC = QP_FREC;
constexpr int PD = QP_RING;
static_assert(FREC <= 64 && PD == 3, "ring layout");

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
// 1/sqrt(v), v > 0: hardware estimate + two Newton steps (full double precision)
__device__ __forceinline__ double rsqrt_nr(double v) {
    double y = __builtin_amdgcn_rsq(v);
    const double h = 0.5 * v;
    y = y * fma(-h * y, y, 1.5);
    y = y * fma(-h * y, y, 1.5);
    return y;
}

struct Smem {
    ldsd *t, *lam;                 // [m] inequality slacks / duals
    ldsd *dx, *dxc;                // iterate dx; sweep solution (x of predictor, then corrector)
    ldsd *du, *dua, *duc;          // iterate du; affine / corrector du
    ldsd *cxa, *cxc;               // C dx of the affine / corrector solution
    ldsd *rec, *frc, *fsave;       // committed stage record, factor record; F records of nodes < PD
    ldsd *P, *p;                   // Riccati P (full 10x10), p (updated in place, one wavefront)
    ldsd *W, *M, *m;               // W = P [A B c] (10 x 15), M (14 x 14), m (14)
    ldsd *uu, *hv, *skv;           // u (box constants), h, cost scaling per node
    ldsd *fw, *fg, *bd, *bv;       // soft folds [N+1][3] (w, gamma), box terms [N][4] (diag, v)
    ldsd* cst;                     // lbu 4 | ubu 4 | lh 3 | uh 3 | zl 3 | Zl 3 (lane-indexed kernel arguments
                                   // would be vector loads that wait behind the record stream)
};

__device__ __forceinline__ Smem carve(ldsd* q, int N) {  // mirrors qp_lds_doubles()
    Smem s;
    auto take = [&](int n) { ldsd* r = q; q += n; return r; };
    const int m = 8 * N + 12 * (N + 1), N1 = N + 1;
    s.t = take(m); s.lam = take(m);
    s.dx = take(N1 * NX); s.dxc = take(N1 * NX);
    s.du = take(N * NU); s.dua = take(N * NU); s.duc = take(N * NU);
    s.cxa = take(N1 * NS); s.cxc = take(N1 * NS);
    s.rec = take(REC); s.frc = take(FREC); s.fsave = take(PD * FREC);
    s.P = take(100); s.p = take(10);
    s.W = take(150); s.M = take(196); s.m = take(14);
    s.uu = take(N * NU); s.hv = take(N1 * NS); s.skv = take(N1);
    s.fw = take(N1 * NS); s.fg = take(N1 * NS); s.bd = take(N * NU); s.bv = take(N * NU);
    s.cst = take(20);
    return s;
}

}  // namespace

// ---------------------------------------------------------------------------------------------------
// Stage records, one block per (instance, node): AB, c = xn_k - xbar_{k+1}, g = s_k J^T W r,
// C = J_h, H = s_k J^T W J + lm I (upper); terminal: H_N = J_N^T W_N J_N + lm I (10x10 upper in the
// H field), g_N (first 10 of g), C_N.
__global__ __launch_bounds__(256) void rti_qp_pack_kernel(QpArgs A) {
    const int N = A.N, N1 = N + 1;
    const int b = blockIdx.x / N1, k = blockIdx.x - b * N1;
    double* Rk = A.work + (size_t)b * qp_work_doubles(N) + (size_t)k * REC;
    const double* Jh = A.Jh + ((size_t)b * N1 + k) * 30;
    __shared__ double Js[154], Ws[11], rs[11];
    if (k < N) {
        const size_t bk = (size_t)b * N + k;
        const double sk = A.cost_scaling ? A.dt[k] : 1.0;
        for (int e = threadIdx.x; e < 154; e += 256) Js[e] = A.Jy[bk * 154 + e];
        if (threadIdx.x < 11) {
            Ws[threadIdx.x] = sk * A.W[bk * 11 + threadIdx.x];
            rs[threadIdx.x] = A.y[bk * 11 + threadIdx.x] - A.yref[bk * 11 + threadIdx.x];
        }
        __syncthreads();
        const double* AB = A.AB + bk * 140;
        const double* xn = A.xn + bk * 10;
        const double* xb1 = A.x + ((size_t)b * N1 + k + 1) * 10;
        for (int e = threadIdx.x; e < REC; e += 256) {
            double v = 0.0;
            if (e < R_C) {
                v = AB[e];
            } else if (e < R_G) {
                v = xn[e - R_C] - xb1[e - R_C];
            } else if (e < R_CH) {
                const int a = e - R_G;
                for (int i = 0; i < 11; ++i) v += Js[a * 11 + i] * Ws[i] * rs[i];
            } else if (e < R_H) {
                v = Jh[e - R_CH];
            } else if (e < R_H + 105) {
                int q = e - R_H, a = 0;
                while (q >= 14 - a) { q -= 14 - a; ++a; }
                const int c = a + q;
                for (int i = 0; i < 11; ++i) v += Js[a * 11 + i] * Ws[i] * Js[c * 11 + i];
                v += (a == c ? A.lm : 0.0);
            }
            Rk[e] = v;
        }
    } else {
        const double* J = A.JyN + (size_t)b * 40;  // [10][4]
        const double* Wn = A.WN + (size_t)b * 4;
        const double* yn = A.yN + (size_t)b * 4;
        const double* rn = A.yNref + (size_t)b * 4;
        for (int e = threadIdx.x; e < REC; e += 256) {
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
    const double* R = A.work + (size_t)b * qp_work_doubles(N);  // [N+1][REC] stage records
    double* F = A.work + (size_t)b * qp_work_doubles(N) + (size_t)N1 * REC;  // [N+1][FREC]

    // ------------------------------------------------------------ record stream
    // stream index j: [0, N1) initial forward (k = j); then per IPM iteration 4 sweeps of N1 records:
    // backward-factor (full record), forward (record + Y, L, kff), backward-corrector (record + F),
    // forward.  Slot j % PD of the register ring holds record j; consuming j issues j + PD.
    double rr[PD][RR], fr[PD];
    auto decode = [&](int j, int& k, int& n, int& nf) {
        if (j < N1) { k = j; n = R_H; nf = 0; return; }
        const int jj = j - N1, q = jj % N1, t = (jj / N1) & 3;
        k = (t & 1) ? q : N - q;
        n = t == 0 ? REC : R_H;
        nf = t == 0 ? 0 : (t == 2 ? FREC : F_PC);
    };
    // every issue is the same RR + 1 unpredicated loads (clamped addresses): a data-dependent load
    // count would make the compiler's wait counters conservative (vmcnt(0) at every commit)
    auto issue_to = [&](double* rd, double& fd, int j) {
        int k, n, nf;
        decode(j, k, n, nf);
        const double* src = R + (size_t)k * REC;
#pragma unroll
        for (int i = 0; i < RR; ++i) {
            const int e = lane + 64 * i;
            rd[i] = src[e < REC ? e : REC - 1];
        }
        fd = F[(size_t)k * FREC + lane];
    };
    auto commit_from = [&](const double* rd, double fd) {
#pragma unroll
        for (int i = 0; i < RR; ++i) {
            const int e = lane + 64 * i;
            if (e < REC) s.rec[e] = rd[i];
        }
        s.frc[lane] = fd;
    };
    int pos = 0;
    auto advance = [&]() {  // commit record `pos` to LDS, refill its slot with record pos + PD
        const int sl = pos % PD;
        if (sl == 0) { commit_from(rr[0], fr[0]); issue_to(rr[0], fr[0], pos + PD); }
        else if (sl == 1) { commit_from(rr[1], fr[1]); issue_to(rr[1], fr[1], pos + PD); }
        else { commit_from(rr[2], fr[2]); issue_to(rr[2], fr[2], pos + PD); }
        ++pos;
    };
    issue_to(rr[0], fr[0], 0);
    issue_to(rr[1], fr[1], 1);
    issue_to(rr[2], fr[2], 2);

    // ------------------------------------------------------------ per-node constants into LDS
    for (int e = lane; e < N * NU; e += 64) {
        s.uu[e] = A.u[(size_t)b * N * NU + e];
        s.du[e] = 0.0;
    }
    for (int e = lane; e < N1 * NS; e += 64) s.hv[e] = A.h[(size_t)b * N1 * NS + e];
    {
        double v = 0.0;  // constant indices: scalar loads of the kernel arguments
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (lane == i) v = A.lbu[i];
            if (lane == 4 + i) v = A.ubu[i];
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            if (lane == 8 + j) v = A.lh[j];
            if (lane == 11 + j) v = A.uh[j];
            if (lane == 14 + j) v = A.zl[j];
            if (lane == 17 + j) v = A.Zl[j];
        }
        if (lane < 20) s.cst[lane] = v;
    }
    for (int e = lane; e < N1; e += 64) s.skv[e] = (A.cost_scaling && e < N) ? A.dt[e] : 1.0;
    if (lane < NX) s.dx[lane] = A.x0[(size_t)b * 10 + lane] - A.x[(size_t)b * N1 * 10 + lane];
    __syncthreads();
    STAMP(0);

    // per-lane output maps of the three factor steps (fixed for the whole solve)
    // step 1: W[i][j] = P[i,:] . [A B c][:, j], e = i * 15 + j < 150
    const int e1b = lane + 64, e1c = (lane + 128 < 150) ? lane + 128 : 149;
    const int w_i0 = lane / 15, w_j0 = lane % 15, w_i1 = e1b / 15, w_j1 = e1b % 15, w_i2 = e1c / 15, w_j2 = e1c % 15;
    // step 2: (a, c), a <= c < 14 (M upper, row-major) then (a, 14) = m
    auto m_map = [](int e, int& a, int& c) {
        if (e >= 105) { a = e - 105; c = 14; return; }
        int q = e;
        a = 0;
        while (q >= 14 - a) { q -= 14 - a; ++a; }
        c = a + q;
    };
    int m_a0, m_c0, m_a1, m_c1;
    m_map(lane, m_a0, m_c0);
    m_map(lane + 64 < 119 ? lane + 64 : 118, m_a1, m_c1);
    const bool m_has1 = lane + 64 < 119;
    // step 3: e < 100: P[a][c]; e >= 100: p[e - 100]
    const int p_a0 = lane / 10, p_c0 = lane % 10;
    const int p_e1 = (lane + 64 < 110) ? lane + 64 : 109;
    const int p_a1 = p_e1 < 100 ? p_e1 / 10 : p_e1 - 100, p_c1 = p_e1 < 100 ? p_e1 % 10 : -1;
    const bool p_has1 = lane + 64 < 110;

    // box rows (k, i, up): t = +-du + d, d = (u - lbu) | (ubu - u)
    auto box_d = [&](int k, int i, int up) -> double {
        const double u = s.uu[k * 4 + i];
        return up ? s.cst[4 + i] - u : u - s.cst[0 + i];
    };

    // ------------------------------------------------------------ forward sweep (1 barrier per stage)
    // mode 0: initial iterate (u = 0); mode 1: u_k = k_ff - L^-T (Y x_k).  x_{k+1} = A x_k + B u_k + c_k,
    // cx = C x.  Factor data of nodes < PD comes from fsave (written late in the backward sweep).
    auto forward = [&](int mode, ldsd* dxo, ldsd* duo, ldsd* cxo) {
        if (lane < NX) dxo[lane] = s.dx[lane];
        for (int k = 0; k < N1; ++k) {
            advance();
            __syncthreads();
            const ldsd* rk = s.rec;
            const ldsd* fk = (k < PD) ? s.fsave + k * FREC : s.frc;
            const ldsd* x = dxo + k * NX;
            if (lane >= 16 && lane < 16 + NS) {
                const int j = lane - 16;
                double v = 0.0;
#pragma unroll
                for (int l = 0; l < NX; ++l) v += rk[R_CH + l * 3 + j] * x[l];
                cxo[k * NS + j] = v;
            }
            if (k < N && lane < NX) {
                double xv[NX];
#pragma unroll
                for (int l = 0; l < NX; ++l) xv[l] = x[l];
                double u[4] = {0.0, 0.0, 0.0, 0.0};
                if (mode) {
                    double yx[4];
#pragma unroll
                    for (int i = 0; i < 4; ++i) {
                        double v = 0.0;
#pragma unroll
                        for (int l = 0; l < NX; ++l) v += fk[F_Y + i * 10 + l] * xv[l];
                        yx[i] = v;
                    }
#pragma unroll
                    for (int i = 3; i >= 0; --i) {
                        double v = yx[i];
#pragma unroll
                        for (int q = i + 1; q < 4; ++q) v -= fk[F_L + ltri4(q, i)] * u[q];
                        u[i] = v * fk[F_L + ltri4(i, i)];
                    }
#pragma unroll
                    for (int i = 0; i < 4; ++i) u[i] = fk[F_K + i] - u[i];
                }
                double v = rk[R_C + lane];
#pragma unroll
                for (int j = 0; j < NX; ++j) v += rk[R_AB + j * 10 + lane] * xv[j];
#pragma unroll
                for (int i = 0; i < 4; ++i) v += rk[R_AB + (NX + i) * 10 + lane] * u[i];
                dxo[(k + 1) * NX + lane] = v;
                if (mode && lane < 4) duo[k * NU + lane] = u[lane];
            }
            __syncthreads();
        }
    };

    // ------------------------------------------------------------ initial iterate (dynamics-feasible):
    // du = sl = su = 0, dx_0 = x0 - xbar_0, dx_{k+1} = A dx_k + c_k
    forward(0, s.dx, nullptr, s.cxa);
    double rp = 0.0;
    for (int r = lane; r < m; r += 64) {
        double v;
        if (r < 8 * N) {
            const int k = r >> 3, q = r & 7, i = q & 3, up = q >> 2;
            v = box_d(k, i, up);
        } else {
            const int q = r - 8 * N, k = q / 12, w = q - 12 * k, j = w >> 2, kind = w & 3;
            const double h = s.hv[k * 3 + j];
            v = kind == 0 ? s.cxa[k * NS + j] + (h - s.cst[8 + j]) : kind == 1 ? -s.cxa[k * NS + j] + (s.cst[11 + j] - h) : 0.0;
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
        const double sk = s.skv[k];
        const double t1 = s.t[r0], t2 = s.t[r0 + 1], t3 = s.t[r0 + 2], t4 = s.t[r0 + 3];
        const double l1 = s.lam[r0], l2 = s.lam[r0 + 1], l3 = s.lam[r0 + 2], l4 = s.lam[r0 + 3];
        g.s1 = l1 / t1; g.s3 = l2 / t2; g.s2 = l3 / t3; g.s4 = l4 / t4;
        const double h = s.hv[k * 3 + j];
        g.v1 = g.s1 * (t1 - (h - s.cst[8 + j]));
        g.v3 = g.s3 * (t2 - (s.cst[11 + j] - h));
        g.v2 = g.s2 * t3;
        g.v4 = g.s4 * t4;
        const double Zs = sk * s.cst[17 + j], zs = sk * s.cst[14 + j];
        g.Hl = Zs + g.s1 + g.s2;
        g.Hu = Zs + g.s3 + g.s4;
        if (phase) {  // corrector: affine deltas of the four rows, recomputed from the affine solution
            const double cxa = s.cxa[k * NS + j];
            const double sla = -((zs - g.v1 - g.v2) + g.s1 * cxa) / g.Hl;
            const double sua = -((zs - g.v3 - g.v4) - g.s3 * cxa) / g.Hu;
            const double d1 = cxa + (h - s.cst[8 + j]) + sla - t1;
            const double d2 = -cxa + (s.cst[11 + j] - h) + sua - t2;
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
    // all nodes at once, before a backward sweep: fw = w_j (factor only), fg = gamma_j, box diag / v
    auto terms = [&](int phase, double sigmu) {
        for (int e = lane; e < N1 * NS; e += 64) {
            const int k = e / NS, j = e - NS * k;
            const Grp g = group(k, j, phase, sigmu);
            const double iHl = 1.0 / g.Hl, iHu = 1.0 / g.Hu;
            if (!phase) s.fw[e] = g.s1 * (g.Hl - g.s1) * iHl + g.s3 * (g.Hu - g.s3) * iHu;
            s.fg[e] = -(g.v1 + g.s1 * g.gl * iHl) + (g.v3 + g.s3 * g.gu * iHu);
        }
        for (int e = lane; e < N * NU; e += 64) {
            const int k = e >> 2, i = e & 3;
            if (!phase) s.bd[e] = s.lam[8 * k + i] / s.t[8 * k + i] + s.lam[8 * k + 4 + i] / s.t[8 * k + 4 + i];
            s.bv[e] = -box_v(k, i, 0, phase, sigmu) + box_v(k, i, 1, phase, sigmu);
        }
        __syncthreads();
    };

    // ------------------------------------------------------------ backward sweep, factor (3 barriers / stage)
    auto backward_factor = [&]() {
        for (int q = 0; q < N1; ++q) {
            const int k = N - q;
            advance();
            __syncthreads();
            const ldsd* rk = s.rec;
            if (q == 0) {  // P_N = H_N + sum_j w_j C_j^T C_j, p_N = g_N + sum_j gamma_j C_j^T
                for (int e = lane; e < 110; e += 64) {
                    if (e < 100) {
                        const int a = e / 10, c = e % 10;
                        double v = rk[R_H + tri10(a < c ? a : c, a < c ? c : a)];
                        for (int j = 0; j < NS; ++j) v += s.fw[N * NS + j] * rk[R_CH + a * 3 + j] * rk[R_CH + c * 3 + j];
                        s.P[e] = v;
                    } else {
                        const int a = e - 100;
                        double v = rk[R_G + a];
                        for (int j = 0; j < NS; ++j) v += s.fg[N * NS + j] * rk[R_CH + a * 3 + j];
                        s.p[a] = v;
                    }
                }
                __syncthreads();
                continue;
            }
            double* Fk = F + (size_t)k * FREC;
            ldsd* Fs = s.fsave + k * FREC;  // meaningful for k < PD only
            // ---- step 1: W = P [A B c] (10 x 15); column 14 -> P c (factor record) and P c + p
            {
                double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll
                for (int l = 0; l < NX; ++l) {
                    a0 += s.P[w_i0 * 10 + l] * rk[w_j0 * 10 + l];
                    a1 += s.P[w_i1 * 10 + l] * rk[w_j1 * 10 + l];
                    a2 += s.P[w_i2 * 10 + l] * rk[w_j2 * 10 + l];
                }
                if (w_j0 == 14) { Fk[F_PC + w_i0] = a0; if (k < PD) Fs[F_PC + w_i0] = a0; a0 += s.p[w_i0]; }
                if (w_j1 == 14) { Fk[F_PC + w_i1] = a1; if (k < PD) Fs[F_PC + w_i1] = a1; a1 += s.p[w_i1]; }
                if (w_j2 == 14) { Fk[F_PC + w_i2] = a2; if (k < PD) Fs[F_PC + w_i2] = a2; a2 += s.p[w_i2]; }
                s.W[lane] = a0;
                s.W[e1b] = a1;
                if (lane + 128 < 150) s.W[lane + 128] = a2;
            }
            __syncthreads();
            // ---- step 2: M = H~ + [A B]^T W (upper), m = g~ + [A B]^T (P c + p), plus soft folds / box terms
            {
                const int fk3 = k * NS, bk4 = k * 4;
                auto mval = [&](int a, int c, double acc) -> double {
                    double v = acc;
                    if (c < 14) {
                        v += rk[R_H + a * 14 - a * (a - 1) / 2 + (c - a)];
                        if (c < NX) {
#pragma unroll
                            for (int j = 0; j < NS; ++j) v += s.fw[fk3 + j] * rk[R_CH + a * 3 + j] * rk[R_CH + c * 3 + j];
                        } else if (a == c) {
                            v += s.bd[bk4 + a - NX];
                        }
                    } else {
                        v += rk[R_G + a];
                        if (a < NX) {
#pragma unroll
                            for (int j = 0; j < NS; ++j) v += s.fg[fk3 + j] * rk[R_CH + a * 3 + j];
                        } else {
                            v += s.bv[bk4 + a - NX];
                        }
                    }
                    return v;
                };
                double a0 = 0.0, a1 = 0.0;
#pragma unroll
                for (int l = 0; l < NX; ++l) {
                    a0 += rk[m_a0 * 10 + l] * s.W[l * 15 + m_c0];
                    a1 += rk[m_a1 * 10 + l] * s.W[l * 15 + m_c1];
                }
                const double v0 = mval(m_a0, m_c0, a0), v1 = mval(m_a1, m_c1, a1);
                if (m_c0 < 14) { s.M[m_a0 * 14 + m_c0] = v0; s.M[m_c0 * 14 + m_a0] = v0; } else { s.m[m_a0] = v0; }
                if (m_has1) {
                    if (m_c1 < 14) { s.M[m_a1 * 14 + m_c1] = v1; s.M[m_c1 * 14 + m_a1] = v1; } else { s.m[m_a1] = v1; }
                }
            }
            __syncthreads();
            // ---- step 3: L = chol(R^) (every lane, registers), y_a = L^-1 S[:, a], w = L^-1 m_u;
            //      P_k = Q^ - Y^T Y, p_k = m_x - Y^T w (in place); factor record (Y, L, k_ff)
            double L[4][4], id[4];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int j = 0; j <= i; ++j) {
                    double v = s.M[(NX + i) * 14 + NX + j];
#pragma unroll
                    for (int q2 = 0; q2 < j; ++q2) v -= L[i][q2] * L[j][q2];
                    if (i == j) {
                        id[i] = rsqrt_nr(v);
                        L[i][i] = v * id[i];
                    } else {
                        L[i][j] = v * id[j];
                    }
                }
            auto fsub = [&](const ldsd* col, int stride, double* y) {
                y[0] = col[0] * id[0];
                y[1] = (col[stride] - L[1][0] * y[0]) * id[1];
                y[2] = (col[2 * stride] - L[2][0] * y[0] - L[2][1] * y[1]) * id[2];
                y[3] = (col[3 * stride] - L[3][0] * y[0] - L[3][1] * y[1] - L[3][2] * y[2]) * id[3];
            };
            double w[4], ya0[4], yc0[4], ya1[4], yc1[4];
            fsub(s.m + NX, 1, w);
            fsub(s.M + NX * 14 + p_a0, 14, ya0);
            fsub(s.M + NX * 14 + p_c0, 14, yc0);
            fsub(s.M + NX * 14 + p_a1, 14, ya1);
            if (p_c1 >= 0) {
                fsub(s.M + NX * 14 + p_c1, 14, yc1);
            } else {
#pragma unroll
                for (int i = 0; i < 4; ++i) yc1[i] = w[i];
            }
            double v0 = s.M[p_a0 * 14 + p_c0];
            double v1 = p_c1 >= 0 ? s.M[p_a1 * 14 + p_c1] : s.m[p_a1];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                v0 -= ya0[i] * yc0[i];
                v1 -= ya1[i] * yc1[i];
            }
            s.P[lane] = v0;
            if (p_has1) {
                if (p_c1 >= 0) s.P[p_e1] = v1; else s.p[p_a1] = v1;
            }
            if (lane < NX) {  // Y[:, c] with c = lane (a = 0)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    Fk[F_Y + i * 10 + lane] = yc0[i];
                    if (k < PD) Fs[F_Y + i * 10 + lane] = yc0[i];
                }
            }
            if (lane >= 16 && lane < 26) {  // L, diagonal stored as 1/L_ii
                const int e = lane - 16;
                const int i = e >= 6 ? 3 : e >= 3 ? 2 : e >= 1 ? 1 : 0, j = e - i * (i + 1) / 2;
                double v = 0.0;
#pragma unroll
                for (int ii = 0; ii < 4; ++ii)
#pragma unroll
                    for (int jj = 0; jj <= ii; ++jj)
                        if (ii == i && jj == j) v = (ii == jj) ? id[ii] : L[ii][jj];
                Fk[F_L + e] = v;
                if (k < PD) Fs[F_L + e] = v;
            }
            if (lane >= 48 && lane < 52) {  // k_ff = -L^-T w
                double kf[4];
#pragma unroll
                for (int i = 3; i >= 0; --i) {
                    double v = w[i];
#pragma unroll
                    for (int q2 = i + 1; q2 < 4; ++q2) v -= L[q2][i] * kf[q2];
                    kf[i] = v * id[i];
                }
                double v = 0.0;
#pragma unroll
                for (int i = 0; i < 4; ++i) if (lane - 48 == i) v = -kf[i];
                Fk[F_K + lane - 48] = v;
                if (k < PD) Fs[F_K + lane - 48] = v;
            }
            __syncthreads();
        }
    };

    // ------------------------------------------------------------ backward sweep, corrector (1 barrier / stage)
    // stored factors + corrector gradient: Pb = P c + p, w = L^-1 m_u, p_k = m_x - Y^T w, k_ff = -L^-T w
    auto backward_corrector = [&]() {
        for (int q = 0; q < N1; ++q) {
            const int k = N - q;
            advance();
            __syncthreads();
            const ldsd* rk = s.rec;
            if (q == 0) {
                if (lane < NX) {
                    double v = rk[R_G + lane];
                    for (int j = 0; j < NS; ++j) v += s.fg[N * NS + j] * rk[R_CH + lane * 3 + j];
                    s.p[lane] = v;
                }
                __syncthreads();
                continue;
            }
            const ldsd* fk = s.frc;
            double Pb[NX];
#pragma unroll
            for (int l = 0; l < NX; ++l) Pb[l] = fk[F_PC + l] + s.p[l];
            double mu[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                double v = rk[R_G + NX + i] + s.bv[k * 4 + i];
#pragma unroll
                for (int l = 0; l < NX; ++l) v += rk[R_AB + (NX + i) * 10 + l] * Pb[l];
                mu[i] = v;
            }
            double w[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                double v = mu[i];
#pragma unroll
                for (int q2 = 0; q2 < i; ++q2) v -= fk[F_L + ltri4(i, q2)] * w[q2];
                w[i] = v * fk[F_L + ltri4(i, i)];
            }
            if (lane < NX) {
                const int a = lane;
                double v = rk[R_G + a];
#pragma unroll
                for (int l = 0; l < NX; ++l) v += rk[R_AB + a * 10 + l] * Pb[l];
#pragma unroll
                for (int j = 0; j < NS; ++j) v += s.fg[k * NS + j] * rk[R_CH + a * 3 + j];
#pragma unroll
                for (int i = 0; i < 4; ++i) v -= fk[F_Y + i * 10 + a] * w[i];
                s.p[a] = v;
            }
            if (lane >= 16 && lane < 20) {
                double kf[4];
#pragma unroll
                for (int i = 3; i >= 0; --i) {
                    double v = w[i];
#pragma unroll
                    for (int q2 = i + 1; q2 < 4; ++q2) v -= fk[F_L + ltri4(q2, i)] * kf[q2];
                    kf[i] = v * fk[F_L + ltri4(i, i)];
                }
                double v = 0.0;
#pragma unroll
                for (int i = 0; i < 4; ++i) if (lane - 16 == i) v = -kf[i];
                F[(size_t)k * FREC + F_K + lane - 16] = v;
                if (k < PD) s.fsave[k * FREC + F_K + lane - 16] = v;
            }
            __syncthreads();
        }
    };

    // row values of a soft group (k, j) at an LQR solution with C dx = cxs, and its slacks
    auto soft_vals = [&](const Grp& g, int k, int j, double cxs, double* v) {
        const double h = s.hv[k * 3 + j];
        const double sl = -(g.gl + g.s1 * cxs) / g.Hl, su = -(g.gu - g.s3 * cxs) / g.Hu;
        v[0] = cxs + (h - s.cst[8 + j]) + sl;
        v[1] = -cxs + (s.cst[11 + j] - h) + su;
        v[2] = sl;
        v[3] = su;
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
        terms(0, 0.0);
        backward_factor();
        STAMP(2);
        forward(1, s.dxc, s.dua, s.cxa);
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
            soft_vals(g, k, j, s.cxa[e], v);
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
            soft_vals(g, k, j, s.cxa[e], v);
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
        terms(1, sigmu);
        backward_corrector();
        STAMP(5);
        forward(1, s.dxc, s.duc, s.cxc);
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
            soft_vals(ga, k, j, s.cxa[e], va);
            soft_vals(gc, k, j, s.cxc[e], vc);
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
            double va[4], vc[4];
            soft_vals(ga, k, j, s.cxa[e], va);
            soft_vals(gc, k, j, s.cxc[e], vc);
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
    if (A.slack)  // slacks = the t of rows sl >= 0, su >= 0 (equal to the iterate's sl, su up to r_p)
        for (int e = lane; e < N1 * NS; e += 64) {
            const int k = e / NS, j = e % NS, r0 = 8 * N + 12 * k + 4 * j;
            A.slack[((size_t)b * N1 * NS + e) * 2] = s.t[r0 + 2];
            A.slack[((size_t)b * N1 * NS + e) * 2 + 1] = s.t[r0 + 3];
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
    hipLaunchKernelGGL(rti_qp_pack_kernel, dim3((unsigned)(a.B * (a.N + 1))), dim3(256), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    const size_t lds = qp_lds_bytes(a.N);
    e = hipFuncSetAttribute((const void*)rti_qp_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(rti_qp_kernel, dim3(a.B), dim3(64), lds, s, a);
    return hipGetLastError();
}

}  // namespace sdfn
