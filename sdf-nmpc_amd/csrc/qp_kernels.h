// Batched RTI QP (rti_qp.hip): argument block shared with the engine.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>

namespace sdfn {

constexpr int QP_NHN = 8;  // terminal rows at most (SDFNMPC_NHN_MAX)

struct QpArgs {
    int B, N;
    // preparation-phase outputs (sdfnmpc_lin_args layouts)
    const double *xn, *AB, *y, *Jy, *yN, *JyN, *h, *Jh;
    const double *hE, *JhE;  // terminal extras [B][6], [B][10][6] (NULL unless a terminal row reads them)
    // current iterate, initial state, references (W, WN: diagonals of the weight matrices)
    const double *x, *u, *x0, *yref, *W, *yNref, *WN, *dt;
    // outputs
    double *dx, *du;  // [B][N+1][10], [B][N][4]
    double* slack;    // [B][N+1][3][2] (sl, su) or NULL
    int *status, *iters;
    double* res;      // [B][2] (mu, max primal residual)
    double* work;     // [B][qp_work_doubles(N)]
    double* stamps;   // cycle counters of the stamps diagnostic builds, serial [B][16] / segmented [B][4][24] of the QP_STAMPS diagnostic build (NULL otherwise)
    // model / options
    double lbu[4], ubu[4], lh[3], uh[3], zl[3], Zl[3];  // lh .. Zl: stage row j < nh
    // constraint set (include/sdfnmpc.h sdfnmpc_qp_opts): stage rows j < nh read column h_col[j] of h / J_h;
    // terminal rows j < nhN (the first nsN soft) read h[N][hN_col[j]] + hE[hE_col[j]] (a column < 0: none)
    int nh, h_col[3], nhN, nsN, hN_col[QP_NHN], hE_col[QP_NHN];
    double lhN[QP_NHN], uhN[QP_NHN], zlN[3], ZlN[3];
    int nyN;      // terminal residual rows (yN / JyN / yNref / WN width): 4 or 5
    int sdf_row;  // stage row fed by the sdf column (h_col[j] == 2), -1: none
    double lm, tol;
    int max_iter, cost_scaling;
    int lm_scaling;  // 1: lm dt_k at stages k < N, lm at N (acados' Ts-scaled Levenberg-Marquardt term)
    int ny;  // 11, or 12 with the sdf cost residual (formed in the pack kernel from h[2], J_h[2])
    int pack_part;  // 0: whole stage records; 1: all but the sdf row of C^T (row sdf_row; needs ny == 11), which
                    // rti_qp_kernel then copies from J_h itself (sdf_row_patch)
    int sdf_row_patch;  // rti_qp_kernel: copy J_h[.][2] into the records' C^T row 2 before the sweeps
    int warm_start;     // 1: the IPM starts from the du found in du on entry (qp_solver_warm_start, ocp.py:116)
    int nhs;            // hard stage rows: the last nhs of the nh (slack weight None, base_model.py:142-155)
    int seg_rows;       // 1: a row set the segmented kernel serves (engine.cpp qp_is_seg_set)
};

// the default constraint set (h = [hfov, vfov, sdf] at every node, soft) from lh .. Zl (diagnostic drivers)
inline void qp_default_rows(QpArgs& q) {
    q.nh = 3; q.nhN = 3; q.nsN = 3; q.nyN = 4; q.sdf_row = 2; q.nhs = 0; q.seg_rows = 1;
    for (int j = 0; j < 3; ++j) {
        q.h_col[j] = j; q.zlN[j] = q.zl[j]; q.ZlN[j] = q.Zl[j];
    }
    for (int j = 0; j < QP_NHN; ++j) {
        q.hN_col[j] = j < 3 ? j : -1; q.hE_col[j] = -1;
        q.lhN[j] = j < 3 ? q.lh[j] : 0.0; q.uhN[j] = j < 3 ? q.uh[j] : 0.0;
    }
}

constexpr int QP_REC = 304;   // stage record: [A B | c | g | C^T | H upper | 0 ..] (128-B rows) (rti_qp.hip)
constexpr int QP_FREC = 192;  // factor record: [A~|b~ | K|k_ff (rows of 12) | chol(R^) (1/diag) | P_{k+1} c_k | 4 junk]
#ifndef QP_RING_DEPTH
#define QP_RING_DEPTH 3
#endif
constexpr int QP_RING = QP_RING_DEPTH;  // stream positions in flight per wavefront
constexpr int QP_SLOT = 5;    // 64-double loads per stream position (committed LDS window = 320 doubles)
// segmented kernel (rti_qp_seg.hip): four wavefronts per instance, each a segment of the horizon
constexpr int QP_NSEG = 4;  // at most
constexpr int QP_FRECS = 368;  // its factor record: rows (+ chol(R^), kf_pred) | J c | Z | c, g, B, C^T copies | G | junk
constexpr int QP_CPL = 640;    // coupling block per segment 0..2 (packed L, U, C; V, X, M, Lam; beta)
constexpr int QP_PARK = 12 * 64;  // parked row state per wave

// global workspace per instance: stage records of nodes 0..N, then factor records (each kernel lays its own
// out from offset (N + 1) QP_REC; QP_FRECS >= QP_FREC), then the segmented kernel's coupling blocks
__host__ __device__ inline size_t qp_work_doubles(int N) {
    return (size_t)(N + 1) * (QP_REC + QP_FRECS) + 3 * (size_t)QP_CPL + QP_NSEG * (size_t)QP_PARK;
}
// The row set of one instance: 8 box rows per stage k < N; 4 rows (h lower, h upper, sl >= 0, su >= 0) per
// soft group -- ns - nhs per stage, nsN at the terminal node; 2 rows (lower, upper) per hard row -- nhs per
// stage 0 < k < N, nhN - nsN at the terminal node.  Node 0 has no hard row: acados (0.3.1, the reference's,
// README.md:50) imposes nonlinear rows at the initial node only through con_h_expr_0, which ocp.py never
// sets, and with x_0 fixed a violated one would make the QP infeasible; its soft rows, kept, only add a
// slack term decoupled from (dx, du).  Row order: boxes, soft groups (stage, then terminal), hard rows
// (stage, then terminal).  Groups (one fold / C dx / h entry each): the N ns stage groups (k ns + j; a
// stage's soft rows first), then the nhN terminal rows (soft first).
struct QpRows {
    int ns, nhN, nsN;  // stage rows; terminal rows, soft among them
    int nhs = 0;       // hard stage rows (the last nhs of the ns)
    __host__ __device__ int groups(int N) const { return N * ns + nhN; }
    __host__ __device__ int soft(int N) const { return N * (ns - nhs) + nsN; }
    __host__ __device__ int hard(int N) const { return (N - 1) * nhs + nhN - nsN; }
    __host__ __device__ int rows(int N) const { return 8 * N + 4 * soft(N) + 2 * hard(N); }
};
__host__ __device__ inline QpRows qp_rows_default() { return QpRows{3, 3, 3}; }  // h = [hfov, vfov, sdf] everywhere
// LDS per instance (one wavefront); the order and sizes mirror carve() in rti_qp.hip (every block
// rounded up to an even number of doubles so that 16-byte vector reads stay aligned)
__host__ __device__ inline size_t qp_even(size_t n) { return (n + 1) & ~(size_t)1; }
__host__ __device__ inline size_t qp_lds_doubles(int N, QpRows q) {
    const size_t N1 = N + 1, m = q.rows(N), G = q.groups(N);
    return 2 * qp_even(m)                   // t, lambda
           + 2 * qp_even(N1 * 10)           // dx, dxc
           + 3 * qp_even((size_t)N * 4)     // du, dua, duc
           + 2 * qp_even(G)                 // cxa, cxc
           + QP_SLOT * 64                   // committed stream window
           + QP_RING * 168                  // [A~|b~ K|k_ff] of nodes 0..RING-1 (written late in a backward sweep)
           + 48 + 2                         // zero rows; junk
           + qp_even((size_t)N * 4) + qp_even(G) + qp_even(N1)  // u, h per group, s_k
           + 2 * qp_even(G)                 // folds (w, gamma) per group
           + 2 * qp_even((size_t)N * 4)     // box terms (diag, v)
           + 8 + 4 * (3 + QP_NHN)           // box constants; (lh, uh, zl, Zl) of the stage / terminal rows
           + qp_even((size_t)q.nhN * 10);   // terminal C rows
}
__host__ __device__ inline size_t qp_lds_bytes(int N, QpRows q) { return qp_lds_doubles(N, q) * sizeof(double); }
__host__ __device__ inline size_t qp_lds_bytes(int N) { return qp_lds_bytes(N, qp_rows_default()); }
size_t qp_seg_lds_bytes(int N);  // LDS per instance of the segmented kernel chosen for N (static; 0: unsupported)

int rti_qp_blocks_per_cu(int N, QpRows q);  // instances per CU the serial IPM runs at once (0: does not fit)
int rti_qp_seg_blocks_per_cu(int N);  // the same for the segmented IPM
hipError_t launch_rti_qp_pack(const QpArgs& a, hipStream_t s);  // stage records into the workspace
hipError_t launch_rti_qp(const QpArgs& a, hipStream_t s);       // the IPM (after launch_rti_qp_pack)
bool rti_qp_seg_supported(int N);                               // the segmented IPM handles this horizon
int rti_qp_seg_count(int N);                                    // its segments (wavefronts) per instance
hipError_t launch_rti_qp_seg(const QpArgs& a, hipStream_t s);   // the IPM, four wavefronts per instance
hipError_t launch_rti_apply(int B, int N, double* x, double* u, const double* dx, const double* du, double* u0,
                            const int* status, hipStream_t s);

}  // namespace sdfn
