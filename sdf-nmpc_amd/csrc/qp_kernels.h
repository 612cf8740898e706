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
    double* stamps;   // [B][8] cycle counters of the QP_STAMPS diagnostic build (NULL otherwise)
    // model / options
    double lbu[4], ubu[4], lh[3], uh[3], zl[3], Zl[3];
    double lm, tol;
    int max_iter, cost_scaling;
};

constexpr int QP_REC = 300;   // stage record: [A B | c | g | C | H upper]          (rti_qp.hip)
constexpr int QP_FREC = 216;  // factor record: [A~|b~ | K|k_ff | Y | chol(R^) (1/diag) | P_{k+1} c_k | 2 spare]
constexpr int QP_RING = 3;    // records in flight per wavefront

// global workspace per instance: stage records and factor records for nodes 0..N
__host__ __device__ inline size_t qp_work_doubles(int N) { return (size_t)(N + 1) * (QP_REC + QP_FREC); }
// LDS per instance (one wavefront); the order and sizes mirror carve() in rti_qp.hip
__host__ __device__ inline size_t qp_lds_doubles(int N) {
    const size_t N1 = N + 1, m = 8 * (size_t)N + 12 * N1;
    return 2 * m                    // t, lambda
           + 2 * N1 * 10            // dx, dxc
           + 3 * (size_t)N * 4      // du, dua, duc
           + 2 * N1 * 3             // cxa, cxc
           + 320 + 192              // committed stage-record / factor-record windows
           + QP_RING * 154          // [A~|b~ K|k_ff] of nodes 0..RING-1 (written late in a backward sweep)
           + 16                     // corrector p
           + 4 * (size_t)N + 4 * N1 // u, (h, s_k)
           + 6 * N1 + 8 * (size_t)N // soft-row folds (w, gamma), box terms (diag, v)
           + 20;                    // box / soft-row constants
}
__host__ __device__ inline size_t qp_lds_bytes(int N) { return qp_lds_doubles(N) * sizeof(double); }

hipError_t launch_rti_qp(const QpArgs& a, hipStream_t s);
hipError_t launch_rti_apply(int B, int N, double* x, double* u, const double* dx, const double* du, double* u0,
                            hipStream_t s);

}  // namespace sdfn
