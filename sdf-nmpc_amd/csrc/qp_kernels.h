// Batched RTI QP (rti_qp.hip): argument block shared with the engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace sdfn {

struct QpArgs {
    int B, N;
    // preparation-phase outputs (sdfnmpc_lin_args layouts)
    const double *xn, *AB, *y, *Jy, *yN, *JyN, *h, *Jh;
    // current iterate, initial state, references (W, WN: diagonals of the weight matrices)
    const double *x, *u, *x0, *yref, *W, *yNref, *WN, *dt;
    // outputs
    double *dx, *du;  // [B][N+1][10], [B][N][4]
    double* slack;    // [B][N+1][3][2] (sl, su) or NULL
    int *status, *iters;
    double* res;      // [B][2] (mu, max primal residual)
    double* work;     // [B][qp_work_doubles(N)]
    // model / options
    double lbu[4], ubu[4], lh[3], uh[3], zl[3], Zl[3];
    double lm, tol;
    int max_iter, cost_scaling;
};

constexpr int QP_FSTRIDE = 100 + 40 + 40 + 16 + 4;  // per-stage factors: P, K, S, chol(R), k_ff

// global workspace per instance: GN Hessians / gradients per stage, then the Riccati factors
__host__ __device__ inline size_t qp_work_doubles(int N) {
    return (size_t)N * 196 + 100 + (size_t)N * 14 + 10 + (size_t)(N + 1) * QP_FSTRIDE;
}
__host__ __device__ inline size_t qp_lds_bytes(int N) {
    const size_t m = 8 * (size_t)N + 12 * (size_t)(N + 1);
    const size_t n = 2 * ((size_t)(N + 1) * 10 + (size_t)N * 4 + 2 * (size_t)(N + 1) * 3) + 4 * m +
                     100 + 10 + 140 + 196 + 14 + 10 + 140 + 40 + 40 + 16 + 4 + 10 + 64;
    return n * sizeof(double);
}
hipError_t launch_rti_qp(const QpArgs& a, hipStream_t s);
hipError_t launch_rti_apply(int B, int N, double* x, double* u, const double* dx, const double* du, double* u0,
                            hipStream_t s);

}  // namespace sdfn
