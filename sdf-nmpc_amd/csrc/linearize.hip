// Per-node linearisation of the SQP-RTI preparation phase (fp64) -- the HBM-bound half of the path.
//
// For every (instance b, shooting node k) this computes what acados evaluates per node
// (SURVEY.md §3.2 step 4):
//   k < N : x_{k+1} = RK4(x_k, u_k, dt_k) and [A_k | B_k] = d x_{k+1} / d (x_k, u_k)
//           (acados ERK, ocp.py:106: RK4, 1 step, forward sensitivities == exact derivative of the
//           RK4 map); NONLINEAR_LS residual y_k (11) and J_y (11 x 14)
//   k = N : terminal residual y_N (4) and J_yN (4 x 10)
//   all k : h_k = [hfov, vfov, sdf] and J_h = d h / d x (3 x 10; d h / d u == 0)
// Model: quad_rollpitchyawrate.py:19-55 ('att'), utils/math.py:7-54,169-192; constraints
// cost_const_helpers.py:48-75 (add_fov_const_trigo) and gen_model.py:46-70 (sdf with flag).
//
// Derivatives are forward-mode dual numbers with ONE tangent per lane: a node is served by 8 lanes,
// each carrying one of the eight directions whose Jacobian columns are not constants of the model
// (linearize_kernel), so every lane writes one or two Jacobian columns (column-major blocks, 80-112
// contiguous bytes per column).  The sdf row of h / J_h is written by sdf_mlp_kernel's
// epilogue, so this kernel is independent of the network and runs concurrently with it.
#include <hip/hip_runtime.h>

#include "lin_kernels.h"

namespace sdfn {

struct dd {
    double v, t;
};
__device__ __forceinline__ dd C(double c) { return {c, 0.0}; }
__device__ __forceinline__ dd operator+(dd a, dd b) { return {a.v + b.v, a.t + b.t}; }
__device__ __forceinline__ dd operator-(dd a, dd b) { return {a.v - b.v, a.t - b.t}; }
__device__ __forceinline__ dd operator-(dd a) { return {-a.v, -a.t}; }
__device__ __forceinline__ dd operator*(dd a, dd b) { return {a.v * b.v, a.t * b.v + a.v * b.t}; }
__device__ __forceinline__ dd operator*(dd a, double c) { return {a.v * c, a.t * c}; }
__device__ __forceinline__ dd operator/(dd a, dd b) {
    const double q = a.v / b.v;
    return {q, (a.t - q * b.t) / b.v};
}
__device__ __forceinline__ dd dsqrt(dd a) {
    const double s = sqrt(a.v);
    return {s, a.t / (2.0 * s)};
}
__device__ __forceinline__ dd datan2(dd y, dd x) {
    const double den = x.v * x.v + y.v * y.v;
    return {atan2(y.v, x.v), (x.v * y.t - y.v * x.t) / den};
}

// the value of the partner lane of a pair (lanes 2i, 2i + 1: DPP quad_perm [1, 0, 3, 2])
__device__ __forceinline__ double pair_swap(double x) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(x);
    const unsigned lo = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)u, 0xB1, 0xF, 0xF, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_mov_dpp((int)(unsigned)(u >> 32), 0xB1, 0xF, 0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// atan2 as a dual number from its value (computed elsewhere)
__device__ __forceinline__ dd datan2_v(dd y, dd x, double v) {
    const double den = x.v * x.v + y.v * y.v;
    return {v, (x.v * y.t - y.v * x.t) / den};
}

// 1 / sqrt(a) as a dual number (a > 0): the hardware estimate and two Newton steps y += y (1 - a y^2) / 2
// (each squares the relative error: within an ulp or two of the rounded 1 / sqrt(a), 8 instructions in
// place of a correctly rounded sqrt and division)
__device__ __forceinline__ dd drsqrt(dd a) {
    double r = __builtin_amdgcn_rsq(a.v);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const double e = __builtin_fma(-(a.v * r), r, 1.0);
        r = __builtin_fma(0.5 * r, e, r);
    }
    return {r, -0.5 * a.t * r * r * r};
}

// f_expl of the 'att' model; sr/cr/sp/cp = sin/cos of roll, pitch (constant over RK4 stages).
// q = x[3:7] / |x[3:7]|; theta_z = atan2(q3, q0) is scale-invariant, so
// (cos, sin)(theta_z) = (x3, x6) / |(x3, x6)| without forming q first.
__device__ __forceinline__ void quad_f(const QuadModel& m, const dd* x, dd gamma, dd sr, dd cr, dd sp, dd cp, dd wz,
                                       dd* f) {
    const dd inv = drsqrt(x[3] * x[3] + x[4] * x[4] + (x[5] * x[5] + x[6] * x[6]));
    const dd s03 = x[3] * x[3] + x[6] * x[6];
    dd c, s;
    if (s03.v > 0.0) {
        const dd r = drsqrt(s03);
        c = x[3] * r;
        s = x[6] * r;
    } else {  // atan2(0, 0) = 0
        c = C(1.0);
        s = C(0.0);
    }
    // V_R_B e_z gamma = [cr sp, -sr, cr cp] gamma (euler2rot with yaw = 0, math.py:34-42)
    const dd b0 = cr * sp * gamma, b1 = -sr * gamma, b2 = cr * cp * gamma;
    // W_R_V = quat2rot([c,0,0,s]) (math.py:11-19)
    const dd r11 = c * c - s * s, r21 = (c * s) * 2.0, r33 = c * c + s * s;
    const dd hw = (wz * inv) * 0.5;  // hamilton_prod(q, [0,0,0,wz]) / 2 with q = x * inv
    f[0] = x[7];
    f[1] = x[8];
    f[2] = x[9];
    f[3] = -(x[6] * hw);
    f[4] = x[5] * hw;
    f[5] = -(x[4] * hw);
    f[6] = x[3] * hw;
    f[7] = r11 * b0 - r21 * b1;
    f[8] = r21 * b0 + r11 * b1;
    f[9] = r33 * b2 - C(m.g);
}

// (q_d (x) invert(q))[3] with q = x[3:7]/|x[3:7]| (|q| = 1 up to rounding): quad_rollpitchyawrate.py:48-51
__device__ __forceinline__ dd qerr3(const dd* x, const double* qd) {
    const dd inv = drsqrt(x[3] * x[3] + x[4] * x[4] + (x[5] * x[5] + x[6] * x[6]));
    return (((x[3] * qd[3] + x[4] * qd[2]) - x[5] * qd[1]) - x[6] * qd[0]) * inv;
}

#ifndef LIN_WAVES
#define LIN_WAVES 1
#endif
// Eight lanes per node.  f_expl does not depend on the position and only f[0:3] = v depends on the
// velocity, so the columns of [A|B], J_y for d/dp and d/dv are constants (the dual evaluation would give
// exactly these: d x+/dp_j = e_j; d x+/dv_j = ((h b1 + h b2) + h b3) + h b4 e_j + e_{7+j}, summed in the
// RK4 accumulation's order; J_y: unit columns) and the lanes carry the eight others: slot s -> direction
// q_{s} (s < 4) or u_{s-4}.  The fov rows of J_h depend on the position only: slots 0..2 seed p_s there.
// The terminal node (all ten directions of x) takes two passes.
__global__ __launch_bounds__(256, LIN_WAVES) void linearize_kernel(LinArgs A) {
    const int tid = threadIdx.x;
    const int sl = tid & 7;                           // lane slot within the node
    const long long r = (long long)blockIdx.x * 32 + (tid >> 3);  // node row = b * (N+1) + k
    const int N = A.N, N1 = A.N + 1;
    if (r >= (long long)A.B * N1) return;
    const long long b = r / N1;
    const int k = (int)(r - b * N1);
    const QuadModel& m = A.m;
    const double* xr = A.x + r * 10;
    double xv[10];
#pragma unroll
    for (int i = 0; i < 10; ++i) xv[i] = xr[i];

    if (k < N) {
        const int t = sl < 4 ? 3 + sl : 6 + sl;  // the tangent direction of this lane: q0..q3, u0..u3
        dd X[10];
#pragma unroll
        for (int i = 0; i < 10; ++i) X[i] = {xv[i], (i >= 3 && i < 7 && i == t) ? 1.0 : 0.0};  // t: q0..q3 or u
        const long long s = b * N + k;
        const double* ur = A.u + s * 4;
        dd U[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) U[i] = {ur[i], (10 + i == t) ? 1.0 : 0.0};
        const dd gamma = U[0] * m.gamma, roll = U[1] * m.roll, pitch = U[2] * m.pitch, wz = U[3] * m.wz;
        double s_r, c_r, s_p, c_p;
        {  // the node's lanes share roll and pitch: a lane pair splits the two sincos and swaps results
            const bool odd = sl & 1;
            double sa, ca;
            sincos(odd ? pitch.v : roll.v, &sa, &ca);
            const double sb = pair_swap(sa), cb = pair_swap(ca);
            s_r = odd ? sb : sa;
            c_r = odd ? cb : ca;
            s_p = odd ? sa : sb;
            c_p = odd ? ca : cb;
        }
        const dd sr = {s_r, c_r * roll.t}, cr = {c_r, -s_r * roll.t};
        const dd sp = {s_p, c_p * pitch.t}, cp = {c_p, -s_p * pitch.t};
        // ---- ERK4 (Butcher c = [0, 1/2, 1/2, 1], b = [1/6, 1/3, 1/3, 1/6]); acados-style
        //      accumulation x_out = x + (h b_1) k_1 + ... + (h b_4) k_4, stage input x + (h a_s) k_{s-1}
        const double dt = A.dt[k];
        const double hb[4] = {dt / 6, dt / 3, dt / 3, dt / 6}, ha[4] = {0.0, dt / 2, dt / 2, dt};
        dd xo[10], kk[10], tmp[10];
        quad_f(m, X, gamma, sr, cr, sp, cp, wz, kk);
        const dd W_a2 = kk[9];
#pragma unroll
        for (int i = 0; i < 10; ++i) xo[i] = X[i] + kk[i] * hb[0];
#pragma unroll
        for (int st = 1; st < 4; ++st) {
#pragma unroll
            for (int i = 0; i < 10; ++i) tmp[i] = X[i] + kk[i] * ha[st];
            quad_f(m, tmp, gamma, sr, cr, sp, cp, wz, kk);
#pragma unroll
            for (int i = 0; i < 10; ++i) xo[i] = xo[i] + kk[i] * hb[st];
        }
        double* AB = A.AB + s * 140;
#pragma unroll
        for (int i = 0; i < 10; ++i) AB[t * 10 + i] = xo[i].t;
        if (sl < 6) {  // the constant columns p_j (sl = j) and v_j (sl = 3 + j)
            const int j = sl < 3 ? sl : sl - 3, col = sl < 3 ? j : 7 + j;
            const double hs = ((hb[0] + hb[1]) + hb[2]) + hb[3];
#pragma unroll
            for (int i = 0; i < 10; ++i) AB[col * 10 + i] = (i == col) ? 1.0 : (sl >= 3 && i == j) ? hs : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 10; ++i)
            if (i == sl || i == sl + 8) A.xn[s * 10 + i] = xo[i].v;
        // ---- NONLINEAR_LS residual (quad_rollpitchyawrate.py:48-55)
        const double* pr = A.p + r * A.np;
        const dd qe3 = qerr3(X, pr + 13);  // p_idx.q_d
        dd Y[11] = {X[0], X[1], X[2], qe3, X[7], X[8], X[9], roll, pitch, wz, W_a2};
        double* Jy = A.Jy + s * 154;
#pragma unroll
        for (int i = 0; i < 11; ++i) Jy[t * 11 + i] = Y[i].t;
        if (sl < 6) {  // y = [p, qe3, v, ...]: unit columns for p_j -> row j, v_j -> row 4 + j
            const int col = sl < 3 ? sl : 4 + sl, row = sl < 3 ? sl : 1 + sl;
#pragma unroll
            for (int i = 0; i < 11; ++i) Jy[col * 11 + i] = (i == row) ? 1.0 : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 11; ++i)
            if (i == sl || i == sl + 8) A.y[s * 11 + i] = Y[i].v;
    } else {
        // ---- terminal residual y_N = [p, q_e[3]]; with flags.stability scaled by the flag, plus the
        //      stability cost row flag |v|^2 (quad_rollpitchyawrate.py:52-55, gen_model.py:142-149);
        //      directions sl and sl + 8
        const double* pr = A.p + r * A.np;
        const int nyN = A.nyN;
        const double fl = m.stability ? pr[0] : 1.0;
        for (int t = sl; t < 10; t += 8) {
            dd X[10];
#pragma unroll
            for (int i = 0; i < 10; ++i) X[i] = {xv[i], (i == t) ? 1.0 : 0.0};
            const dd qe3 = qerr3(X, pr + 13);
            const dd Y[5] = {X[0] * fl, X[1] * fl, X[2] * fl, qe3 * fl, ((X[7] * X[7] + X[8] * X[8]) + X[9] * X[9]) * pr[0]};
            double* J = A.JyN + (b * 10 + t) * nyN;
#pragma unroll
            for (int i = 0; i < 5; ++i)
                if (i < nyN) J[i] = Y[i].t;
#pragma unroll
            for (int i = 0; i < 5; ++i)
                if (t == i && i < nyN) A.yN[b * nyN + i] = Y[i].v;
            if (m.rec_feas | m.stability) {
                // ---- terminal extras (gen_model.py:81-121): -flag poly(v), the fov functions at
                //      Co_p_E = W_R_Co^T (p + poly(v) v / sqrt(|v|^2 + 1e-4) - W_p_Co) + B_R_C^T B_p_C + [off, 0, 0]
                //      (braking_dist_flag with the flag forced to 1, gen_model.py:86-87,110), and v
                dd H[6] = {C(0.0), C(0.0), C(0.0), X[7], X[8], X[9]};
                if (m.rec_feas) {
                    const int deg = m.poly_deg;
                    dd pw[3][7];  // v_i^a, a <= 6
#pragma unroll
                    for (int i = 0; i < 3; ++i) {
                        pw[i][0] = C(1.0);
#pragma unroll
                        for (int a = 1; a < 7; ++a) pw[i][a] = pw[i][a - 1] * X[7 + i];
                    }
                    dd poly = C(0.0);
                    int q = 0;  // polynomial_3variate's order (utils/math.py:307-314)
                    for (int d = 0; d <= deg; ++d)
                        for (int a = 0; a <= d; ++a)
                            for (int bb = 0; bb <= d - a; ++bb, ++q) {
                                dd pa = C(1.0), pb = C(1.0), pc = C(1.0);
#pragma unroll
                                for (int e = 0; e < 7; ++e) {
                                    if (e == a) pa = pw[0][e];
                                    if (e == bb) pb = pw[1][e];
                                    if (e == d - a - bb) pc = pw[2][e];
                                }
                                poly = poly + ((pa * pb) * pc) * m.poly[q];
                            }
                    H[0] = -(poly * pr[0]);
                    const dd nrm = dsqrt(((X[7] * X[7] + X[8] * X[8]) + X[9] * X[9]) + C(1e-4));
                    const dd sc = poly / nrm;
                    const double* R = pr + 4;
                    const dd e0 = (X[0] + X[7] * sc) - C(pr[1]), e1 = (X[1] + X[8] * sc) - C(pr[2]),
                             e2 = (X[2] + X[9] * sc) - C(pr[3]);
                    const dd cx = (e0 * R[0] + e1 * R[3]) + e2 * R[6] + C(m.fov_off[0]);
                    const dd cy = (e0 * R[1] + e1 * R[4]) + e2 * R[7] + C(m.fov_off[1]);
                    const dd cz = (e0 * R[2] + e1 * R[5]) + e2 * R[8] + C(m.fov_off[2]);
                    H[1] = datan2(cy, cx) * pr[0];
                    H[2] = datan2(cz, dsqrt(cx * cx + cy * cy)) * pr[0];
                }
                double* JE = A.JhE + (b * 10 + t) * 6;
#pragma unroll
                for (int i = 0; i < 6; ++i) JE[i] = H[i].t;
#pragma unroll
                for (int i = 0; i < 6; ++i)
                    if (t == i) A.hE[b * 6 + i] = H[i].v;
            }
        }
    }

    // ---- constraints h = [hfov, vfov, sdf] (cost_const_helpers.py:48-75, gen_model.py:46-61): functions
    //      of the position only; slot sl < 3 carries d/dp_sl
    const double* pr = A.p + r * A.np;
    const double flag = pr[0];
    const double Wp0 = pr[1], Wp1 = pr[2], Wp2 = pr[3];
    const double* R = pr + 4;  // W_R_Co row-major (== casadi reshape((3,3)).T)
    const dd e0 = {xv[0] - Wp0, sl == 0 ? 1.0 : 0.0}, e1 = {xv[1] - Wp1, sl == 1 ? 1.0 : 0.0},
             e2 = {xv[2] - Wp2, sl == 2 ? 1.0 : 0.0};
    const dd cx = (e0 * R[0] + e1 * R[3]) + e2 * R[6] + C(m.fov_off[0]);
    const dd cy = (e0 * R[1] + e1 * R[4]) + e2 * R[7] + C(m.fov_off[1]);
    const dd cz = (e0 * R[2] + e1 * R[5]) + e2 * R[8] + C(m.fov_off[2]);
    const dd rho = dsqrt(cx * cx + cy * cy);
    // a lane pair splits the two atan2 values (the node's lanes share them) and swaps results
    const bool odd = sl & 1;
    const double at = atan2(odd ? cz.v : cy.v, odd ? rho.v : cx.v), atp = pair_swap(at);
    const dd hf = datan2_v(cy, cx, odd ? atp : at) * flag;
    const dd vf = datan2_v(cz, rho, odd ? at : atp) * flag;
    // rows 0, 1 of columns sl (< 3: d/dp_sl) and 3 + sl (zero); row 2 (sdf) is the SDF kernel's epilogue
    double* J = A.Jh + r * 30;
    if (sl < 3) {
        J[sl * 3 + 0] = hf.t;
        J[sl * 3 + 1] = vf.t;
    }
    if (sl < 7) {
        J[(3 + sl) * 3 + 0] = 0.0;
        J[(3 + sl) * 3 + 1] = 0.0;
    }
    if (sl == 0) A.h[r * 3 + 0] = hf.v;
    if (sl == 1) A.h[r * 3 + 1] = vf.v;
}

hipError_t launch_linearize(const LinArgs& a, hipStream_t s) {
    const long long rows = (long long)a.B * (a.N + 1);
    if (rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(linearize_kernel, dim3((unsigned)((rows + 31) / 32)), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace sdfn
