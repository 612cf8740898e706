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
//   * one factorisation per iteration serves predictor and corrector.  With G = [A B c] (10 x 15),
//     the factor stage's critical chain runs on f64 MFMA 16x16x4 tiles held in registers:
//         W  = P G                      (P c -> factor record; p added to column 14)
//         M' = G_ab^T W + [H | g] + C^T diag(w) [C | gamma] + box terms       ([R^ S; S^T Q^ | m])
//         L  = chol(R^), Y = L^-1 S,  [P | p] <- M' - Y^T [Y | w]
//     P is symmetric, so the accumulator of one stage is the A operand of the next with no lane
//     movement (C/D lane (g, c) holds rows g + 4r of column c; A/B lane (g, c) holds k = 4s + g).
//     Off that chain, on the VALU: the fold and box terms, [K | k_ff] = -L^-T [Y | w] and the closed
//     loop [A~ | b~] = [A | c] + B [K | k_ff].
//   * forward sweep: one 17-row matvec per stage, [A~; K; C^T] x + [b~; k_ff; 0].
//   * corrector backward sweep: the closed-loop recursion p_k = A~^T (P c + p_{k+1}) + g_x + K^T g_u
//     (g with the corrector's fold / box terms); k_ff = -R^-1 (g_u + B^T (P c + p_{k+1})) and b~ hang
//     off it.
// Memory: rti_qp_pack_kernel packs per-stage records [A B | c | g | C^T | H | 0] into a global
// workspace (a wide launch, one block per stage).  Each IPM iteration walks the records in a fixed
// order -- backward (factor), forward, backward (corrector), forward -- so they form one stream
// prefetched QP_RING positions ahead through registers, across sweep boundaries.  Every sweep kind has
// its own loop, its own window of the stage / factor records and straight-line stages whose lane
// selections are precomputed LDS addresses (zero / junk slots for inactive lanes): no divergent branch
// and no per-stage address arithmetic beyond a node offset.  Iterate, duals and stage scratch live in
// LDS (< 40 KB at N = 40: 4 instances per CU, one round for B = 1024).
#include <hip/hip_runtime.h>

#include <type_traits>
#include <utility>

#include "qp_kernels.h"
#include "qp_dev.h"

namespace sdfn {

namespace {

using namespace qpd;

// factor record: [A~|b~ 10 x 12 | K|k_ff 4 x 12 | L 10 (lower packed, diagonal 1/L_ii) | P c 10 | junk 2]; rows are
// 12 doubles (11 used) so that a forward stage reads its row with five 16-byte LDS reads
constexpr int F_AB = 0, F_K = 10 * FR, F_L = 14 * FR, F_PC = F_L + 10, F_J = F_PC + 10, FREC = QP_FREC;
constexpr int F_FW = 14 * FR;  // forward sweeps read [0, F_FW)
constexpr int SLOT = QP_SLOT, PD = QP_RING;
// Window of one stream position per sweep kind: n_loads(K) loads of 64 consecutive doubles (lanes
// clamped to the record), load j landing at window offset 64 j:
//   0 initial forward     R[0, 256)                    AB, c, C^T in place
//   1 backward factor     R[0, 320)                    the stage record in place; [R_Z, 320) reads 0
//   2, 4 forward          F[0, 192) | R[164, 228)      factor rows at 0, C^T at WF_CT
//   3 backward corrector  F[0, 192) | R[96, 224)       factor record at 0, R[i] at WB_R + i (i >= 96; loads
//                                                      start on a 128-byte line)
constexpr int WF_CT = 192, WB_R = 192 - 96;
static_assert((WB_R + R_G + NX) % 2 == 0, "g~_u block of the corrector window is 16-byte aligned");
__host__ __device__ constexpr int n_loads(int K) { return (K == 1 || K == 3) ? 5 : 4; }
__host__ __device__ constexpr bool load_f(int K, int j) { return (K == 2 || K == 3 || K == 4) ? j < 3 : false; }
__host__ __device__ constexpr int load_at(int K, int j) {
    return (K == 0 || K == 1) ? 64 * j : (K == 2 || K == 4) ? (j < 3 ? 64 * j : R_CT) : (j < 3 ? 64 * j : 96 + 64 * (j - 3));
}
// extent of each record a sweep kind reads (lanes past it load the last needed element again, so a
// 64-lane load touches only the cache lines the stage uses)
__host__ __device__ constexpr int f_end(int K) { return (K == 2 || K == 4) ? F_FW : F_J; }
__host__ __device__ constexpr int r_end(int K) { return K == 1 ? REC : R_CT + 30; }
static_assert(FREC == F_J + 4 && (REC * 8) % 128 == 0 && (FREC * 8) % 128 == 0 && F_FW <= WF_CT && FREC <= 192 && PD >= 2 && SLOT == 5, "record layout");
static_assert(WB_R + R_G + 14 <= 64 * SLOT && WF_CT + 30 <= 64 * SLOT && WB_R + 96 + 128 <= 64 * SLOT && (96 * 8) % 128 == 0 && R_Z < 64 * SLOT,
              "window layout");

template <typename Fn, int... S>
__device__ __forceinline__ void for_each_ic(Fn& fn, std::integer_sequence<int, S...>) {
    (fn(IC<S>{}), ...);
}

struct Smem {
    ldsd *t, *lam;                 // [m] inequality slacks / duals
    ldsd *dx, *dxc;                // iterate dx; sweep solution (x of predictor, then corrector)
    ldsd *du, *dua, *duc;          // iterate du; affine / corrector du
    ldsd *cxa, *cxc;               // C dx of the affine / corrector solution, per group
    ldsd* win;                     // committed stream window
    ldsd* fsave;                   // [A~|b~ K|k_ff] of nodes < PD
    ldsd *zero, *junk;             // 48 doubles that stay 0 (zero rows for strided reads); a store sink
    ldsd *uu, *hv, *skv;           // u (box constants), h per group, cost scaling per node
    ldsd *fw, *fg, *bd, *bv;       // folds per group (w, gamma), box terms [N][4] (diag, v)
    ldsd* cst;                     // lbu 4 | ubu 4 | (lh, uh, zl, Zl) of stage rows 0..2 | of terminal rows 0..7
                                   // (lane-indexed kernel arguments would be vector loads that wait behind the
                                   // record stream)
    ldsd* ctN;                     // terminal C rows [nhN][10]
};
constexpr int CST_ROW = 8, CST_TERM = 8 + 4 * 3;  // group constants: stage row j at CST_ROW + 4 j, terminal CST_TERM + 4 j

// groups: e < N NSS are stage groups (node e / NSS, row e % NSS); then the nhN terminal rows (soft first)
template <int NSS>
__device__ __forceinline__ Smem carve(ldsd* q, int N, QpRows rw) {  // mirrors qp_lds_doubles()
    Smem s;
    auto take = [&](int n) { ldsd* r = q; q += (n + 1) & ~1; return r; };
    const int m = rw.rows(N), N1 = N + 1, G = rw.groups(N);
    s.t = take(m); s.lam = take(m);
    s.dx = take(N1 * NX); s.dxc = take(N1 * NX);
    s.du = take(N * NU); s.dua = take(N * NU); s.duc = take(N * NU);
    s.cxa = take(G); s.cxc = take(G);
    s.win = take(SLOT * 64); s.fsave = take(PD * F_FW);
    s.zero = take(48); s.junk = take(2);
    s.uu = take(N * NU); s.hv = take(G); s.skv = take(N1);
    s.fw = take(G); s.fg = take(G); s.bd = take(N * NU); s.bv = take(N * NU);
    s.cst = take(8 + 4 * (3 + QP_NHN));
    s.ctN = take(rw.nhN * 10);
    return s;
}

// Lane constants of the backward factor stage: window indices (R_Z: a zero slot) and record-store byte
// offsets (F_J: a junk slot).  Built once per factor sweep; every field goes through opaque(), so the
// compiler keeps them in registers instead of rematerialising the index arithmetic (with its
// divergent branches) at every stage.
constexpr int FJB = 8 * F_J;
struct FConst {
    int g, c, og01, og2, cgi, gj, ab01, ab2, bmi, hxu_i, huu_i, v0_i;
    int h_i[4], bq[3];
    unsigned spc[3], sab[3], sk_;
};

template <int NSS>
__device__ __forceinline__ FConst fconst(int lane) {
    FConst f;
    const int g = lane >> 4, c = lane & 15;
    f.g = g;
    f.c = c;
    // G = [A B c] (column 14 is c at R_C + k): G[4 st + g][c] at og01 + 4 st (st = 0, 1), og2
    f.og01 = opaque(c < 15 ? c * 10 + g : R_Z);
    f.og2 = opaque((c < 15 && g < 2) ? c * 10 + g + 8 : R_Z);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int a = g + 4 * r, lo = a < c ? a : c, hi = a < c ? c : a;
        f.h_i[r] = opaque((a < 14 && c < 14) ? R_H + tri14(lo, hi) : (a < 14 && c == 14) ? R_G + a : R_Z);
    }
    // fold operands: A = C[c][g] (g < 3), B = w_g C[c][g] (c < 10) | gamma_g (c = 14)
    f.cgi = opaque((c < NX && g < NSS) ? R_CT + g * 10 + c : R_Z);
    f.gj = g < NSS ? g : 0;
    // closed loop: [A | c][a][c] at ab01 + 4 r (r = 0, 1), ab2; A operand B[a = c][g] at bmi
    const bool xcol = c < NX || c == 14;  // columns of [P | p], [A | c], [K | k_ff]
    const int xo = c < NX ? c : 10;       // their column in the 11-wide factor-record rows
    f.ab01 = opaque(xcol ? (c < NX ? c : 14) * 10 + g : R_Z);
    f.ab2 = opaque((xcol && g < 2) ? (c < NX ? c : 14) * 10 + g + 8 : R_Z);
    f.bmi = opaque(c < NX ? (NX + g) * 10 + c : R_Z);
    // factor-record store offsets in bytes (F_J: junk)
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const int a = g + 4 * r;
        f.spc[r] = (unsigned)opaque((c == 14 && a < NX) ? 8 * (F_PC + a) : FJB);
        f.sab[r] = (unsigned)opaque((xcol && a < NX) ? 8 * (F_AB + a * FR + xo) : FJB);
    }
    f.sk_ = (unsigned)opaque(xcol ? 8 * (F_K + g * FR + xo) : FJB);
    // Joseph form operands (window indices; R_Z reads 0):  A operand H^_xu[c][g] (c < 10);
    // A operand R^0[c][g] = H_uu[c][g] (+ box diagonal, c < 4); C init H^[10 + g][c] of V's row g
    f.hxu_i = opaque(c < NX ? R_H + tri14(c, NX + g) : R_Z);
    // 4x4x4 A operands (one 4 x 4 block, replicated over the instruction's four column blocks: lane
    // (g, c) holds A[c & 3][g]):  R^0[i][g] = H_uu[i][g];  B^T of k-step st: B[4 st + g][i] = G[4 st + g][10 + i]
    const int c3 = c & 3;
    f.huu_i = opaque(R_H + tri14(NX + (c3 < g ? c3 : g), NX + (c3 < g ? g : c3)));
#pragma unroll
    for (int st = 0; st < 3; ++st) f.bq[st] = opaque(4 * st + g < NX ? (NX + c3) * 10 + 4 * st + g : R_Z);
    f.v0_i = opaque(c < 14 ? R_H + tri14(c < NX + g ? c : NX + g, c < NX + g ? NX + g : c) : c == 14 ? R_G + NX + g : R_Z);
    return f;
}

}  // namespace

// ---------------------------------------------------------------------------------------------------
// Stage records, one wavefront per (instance, node), four nodes per workgroup: AB, c = xn_k - xbar_{k+1},
// g = s_k J^T W r, C^T = J_h^T, H = s_k J^T W J + lm I (upper); terminal: H_N = J_N^T W_N J_N + lm I
// (10x10 upper in the H field), g_N (first 10 of g), C_N.  Lane e writes record entries e, e + 64, ...
// (coalesced); the upper-triangle positions come from a constant table instead of a search.
struct PackTri {
    unsigned char a14[105], c14[105], a10[55], c10[55];
};
constexpr PackTri make_tri() {
    PackTri t{};
    int q = 0;
    for (int a = 0; a < 14; ++a)
        for (int c = a; c < 14; ++c, ++q) t.a14[q] = (unsigned char)a, t.c14[q] = (unsigned char)c;
    q = 0;
    for (int a = 0; a < 10; ++a)
        for (int c = a; c < 10; ++c, ++q) t.a10[q] = (unsigned char)a, t.c10[q] = (unsigned char)c;
    return t;
}
__constant__ PackTri c_tri = make_tri();

constexpr int PACK_NODES = 4;  // wavefronts (nodes) per workgroup

__global__ __launch_bounds__(64 * PACK_NODES) void rti_qp_pack_kernel(QpArgs A) {
    const int N = A.N, N1 = N + 1;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int node = blockIdx.x * PACK_NODES + wv;
    if (node >= A.B * N1) return;  // whole wavefronts only: no workgroup barrier below
    const int b = node / N1, k = node - b * N1;
    double* Rk = A.work + (size_t)b * qp_work_doubles(N) + (size_t)k * REC;
    const double* Jh = A.Jh + ((size_t)b * N1 + k) * 30;
    const int ny = A.ny;
    if (k < N) {
        // H = s_k J^T W J + lm_k I and g = s_k J^T W r in one f64 MFMA chain over the residuals (K = ny <= 12):
        // A lane (g, c) = J(c, k) s_k W_k, B lane (g, c) = J(c, k) for c < 14 and r_k for c = 14, k = 4 st + g;
        // D lane (g, c), register q: [H | g][g + 4 q][c]
        const size_t bk = (size_t)b * N + k;
        const double sk = A.cost_scaling ? A.dt[k] : 1.0;
        const double lmk = A.lm_scaling ? A.lm * A.dt[k] : A.lm;  // acados: Ts_k lm for k < N, lm at N
        const int g = lane >> 4, c = lane & 15;
        // sdf cost (gen_model.py:65-66); h[2] is read only then (pack_part 1 runs beside the SDF kernel)
        const double ts = ny > 11 ? 1.0 - 0.5 * A.h[((size_t)b * N1 + k) * 3 + 2] : 0.0;
        // C^T row j = J_h column h_col[j] (j < nh; zero rows past it); with pack_part 1 the sdf row is left to
        // rti_qp_kernel (sdf_row_patch)
        const int skip_row = A.pack_part == 1 ? A.sdf_row : -1;
        auto ct_val = [&](int q) -> double {  // C^T entry q = 10 j + l
            const int j = q / 10;
            return j < A.nh ? Jh[(q - 10 * j) * 3 + A.h_col[j < 3 ? j : 0]] : 0.0;
        };
        d4 D = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int st = 0; st < 3; ++st) {
            const int kk = 4 * st + g;
            double jv = 0.0, wk = 0.0, rv = 0.0;
            if (kk < ny) {
                wk = sk * A.W[bk * ny + kk];
                const double y = kk < 11 ? A.y[bk * 11 + kk] : ts * ts * ts * ts;
                rv = y - A.yref[bk * ny + kk];
                if (c < 14)  // d y_kk / d (x, u)_c; the sdf cost row: -2 (1 - s/2)^3 J_h[2] on the state part
                    jv = kk < 11 ? A.Jy[bk * 154 + c * 11 + kk] : (c < NX ? -2.0 * ts * ts * ts * Jh[c * 3 + 2] : 0.0);
            }
            D = mfma(jv * wk, c == 14 ? rv : jv, D);
        }
        const double* AB = A.AB + bk * 140;
        const double* xn = A.xn + bk * 10;
        const double* xb1 = A.x + ((size_t)b * N1 + k + 1) * 10;
        // e = lane, lane + 64: [A B]; lane + 128: AB tail | c | (g below) | C^T; lane + 192, + 256: C^T tail | 0
        Rk[lane] = AB[lane];
        Rk[64 + lane] = AB[64 + lane];
        {
            const int e = 128 + lane;
            if (e < R_C) Rk[e] = AB[e];
            else if (e < R_G) Rk[e] = xn[e - R_C] - xb1[e - R_C];
            else if (e >= R_CT && (e - R_CT) / 10 != skip_row) {
                Rk[e] = ct_val(e - R_CT);
            }
        }
        for (int e = 192 + lane; e < REC; e += 64) {
            if (e < R_H) {
                if ((e - R_CT) / 10 != skip_row) Rk[e] = ct_val(e - R_CT);
            } else if (e >= R_H + 105) {
                Rk[e] = 0.0;
            }
        }
        // H (upper, + lm_k on the diagonal) and g from the accumulator lanes
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            const int a = g + 4 * q;
            if (a < 14 && c < 14 && a <= c) Rk[R_H + tri14(a, c)] = D[q] + (a == c ? lmk : 0.0);
            else if (a < 14 && c == 14) Rk[R_G + a] = D[q];
        }
    } else {
        // terminal record: H_N = J_N^T W_N J_N + lm I, g_N, and C^T of terminal rows 0..2 (rti_qp_seg.hip reads
        // them; rti_qp_kernel assembles every terminal row from J_h / J_hE itself); with pack_part 1 a row that
        // reads the sdf column is left to the QP kernel's sdf_row_patch
        const int nyN = A.nyN;
        auto ctN_val = [&](int q, bool& skip) -> double {
            const int j = q / 10, l = q - 10 * j;
            int c1 = -1, c2 = -1;
#pragma unroll
            for (int i = 0; i < 3; ++i)
                if (i == j && i < A.nhN) { c1 = A.hN_col[i]; c2 = A.hE_col[i]; }
            double v = 0.0;
            if (c1 >= 0) v += Jh[l * 3 + c1];
            if (c2 >= 0) v += A.JhE[((size_t)b * 10 + l) * 6 + c2];
            skip = A.pack_part == 1 && c1 == 2;
            return v;
        };
        const double* J = A.JyN + (size_t)b * 10 * nyN;  // [10][nyN]
        const double* Wn = A.WN + (size_t)b * nyN;
        const double* yn = A.yN + (size_t)b * nyN;
        const double* rn = A.yNref + (size_t)b * nyN;
        for (int e = lane; e < REC; e += 64) {
            double v = 0.0;
            if (e >= R_G && e < R_G + 10) {
                const int a = e - R_G;
                for (int i = 0; i < nyN; ++i) v += J[a * nyN + i] * Wn[i] * (yn[i] - rn[i]);
            } else if (e >= R_H && e < R_H + 55) {
                const int a = c_tri.a10[e - R_H], c = c_tri.c10[e - R_H];
                for (int i = 0; i < nyN; ++i) v += J[a * nyN + i] * Wn[i] * J[c * nyN + i];
                v += (a == c ? A.lm : 0.0);
            } else if (e >= R_CT && e < R_H) {
                bool skip = false;
                v = ctN_val(e - R_CT, skip);
                if (skip) continue;
            }
            Rk[e] = v;
        }
    }
}

#ifdef QP_STAMPS  // diagnostic build only: per-phase cycle accounting (never in the product build)
#define STAMP_DECL long long st_t0 = clock64(), st_acc[16] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#define STAMP(i) do { const long long t1_ = clock64(); st_acc[i] += t1_ - st_t0; st_t0 = t1_; } while (0)
#define STAMP_OUT if (lane == 0 && A.stamps) for (int i_ = 0; i_ < 16; ++i_) A.stamps[(size_t)b * 16 + i_] = (double)st_acc[i_];
#ifdef QP_FSTAMPS  // finer: slices of the backward factor stage, each ending when value v is available
#define FSTAMP(i, v) do { long long t1_; asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t1_) : "v"(v)); st_acc[i] += t1_ - st_t0; st_t0 = t1_; } while (0)
#endif
#else
#define STAMP_DECL
#define STAMP(i)
#define STAMP_OUT
#endif
#ifndef FSTAMP
#define FSTAMP(i, v)
#endif
#ifdef QP_RSTAMPS  // row phases split: rows_pred | terms(1), rows_update | terms(0)
#define RSTAMP(i) STAMP(i)
#else
#define RSTAMP(i)
#endif

#ifndef QP_LB_WAVES  // diagnostic: minimum waves per SIMD the register allocation must allow
#define QP_LB_WAVES 1
#endif
// small unsigned division x / d for d in 1..3 (x < 2^17): the row phases' group maps of a HARD kernel
__device__ __forceinline__ int div123(int x, int d) {
    return d == 1 ? x : d == 2 ? x >> 1 : (int)(((unsigned)x * 0xAAABu) >> 17);
}
template <int NSS, bool HARD>  // stage rows (0..3); hard rows present (stage rows with slack None, rec_feas, stability)
__global__ __launch_bounds__(64, QP_LB_WAVES) void rti_qp_kernel(QpArgs A) {
    extern __shared__ __align__(16) double lds_q[];
    STAMP_DECL
    constexpr int NS = NSS;  // this kernel's stage rows (shadows qpd::NS, the width of the h / J_h arrays)
    const int b = blockIdx.x, lane = threadIdx.x;
    const int N = A.N, N1 = N + 1;
    const int nhs = HARD ? A.nhs : 0;  // hard stage rows: the last nhs of a stage's NSS
    const int nss = NSS - nhs;         // soft stage rows
    const QpRows rw{NSS, A.nhN, A.nsN, nhs};
    const int m = rw.rows(N);
    const int NGS = N * NSS;          // stage groups (group e = k NSS + j; soft rows j < nss first)
    const int NSG = N * nss;          // soft stage groups
    const int NG1 = rw.soft(N);       // soft groups: soft index si = stage (k nss + j), then terminal (NSG + j)
    const int NHG = (N - 1) * nhs;    // hard stage rows (nodes 0 < k < N: qp_kernels.h QpRows)
    const int NHT = HARD ? rw.hard(N) : 0;  // hard rows: hard index i = stage ((k - 1) nhs + j - nss), then terminal
    const int RH0 = 8 * N + 4 * NG1;  // hard row i: rows RH0 + 2 i (lower), + 1 (upper)
    const int nhN = A.nhN;
    // group of soft index si / of hard index i
    auto soft_e = [&](int si) -> int {
        if constexpr (!HARD) return si;
        else {
            if (si >= NSG) return NGS + si - NSG;
            const int k = div123(si, nss);
            return k * NSS + si - k * nss;
        }
    };
    auto hard_e = [&](int i) -> int {
        if (i >= NHG) return NGS + A.nsN + i - NHG;
        const int k = div123(i, nhs);
        return (k + 1) * NSS + nss + i - k * nhs;
    };
    const Smem s = carve<NSS>((ldsd*)lds_q, N, rw);
    // node and row of soft group e (stage groups first, then the terminal's)
    auto gnode = [&](int e) -> int {
        if constexpr (NSS == 0) return N;
        else return e < NGS ? e / NSS : N;
    };
    auto gcst = [&](int e) -> const ldsd* {  // (lh, uh, zl, Zl) of group e
        return e < NGS ? s.cst + CST_ROW + 4 * (e - gnode(e) * NSS) : s.cst + CST_TERM + 4 * (e - NGS);
    };
    ldsd* const win = s.win;
    const double* R = A.work + (size_t)b * qp_work_doubles(N);  // [N+1][REC] stage records
    double* F = A.work + (size_t)b * qp_work_doubles(N) + (size_t)N1 * REC;  // [N+1][FREC]
    const __amdgpu_buffer_rsrc_t rsF = __builtin_amdgcn_make_buffer_rsrc(F, (short)0, N1 * FREC * 8, 0x00020000);

    // ------------------------------------------------------------ per-node constants into LDS
    {
        // primal warm start: the previous QP's du -- unless it holds a non-finite entry (a failed QP's
        // output), which gives a cold start, so a failure does not stick to the instance
        bool fin = true;
        for (int e = lane; e < N * NU; e += 64) {
            s.uu[e] = A.u[(size_t)b * N * NU + e];
            const double v = A.warm_start ? A.du[(size_t)b * N * NU + e] : 0.0;
            fin = fin && __builtin_isfinite(v);
            s.du[e] = v;
        }
        if (__builtin_amdgcn_ballot_w64(!fin) != 0)
            for (int e = lane; e < N * NU; e += 64) s.du[e] = 0.0;
    }
    // h per group: stage group (k, j) = h[k][h_col[j]]; terminal row j = h[N][hN_col[j]] + hE[hE_col[j]]
    {
        int hc[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) hc[j] = A.h_col[j];
        for (int e = lane; e < NGS; e += 64) {
            const int k = gnode(e), j = e - k * NSS;
            s.hv[e] = A.h[((size_t)b * N1 + k) * 3 + (j == 0 ? hc[0] : j == 1 ? hc[1] : hc[2])];
        }
    }
    {
        // terminal rows: values and C rows (lane 10 j + l: row j, entry l), sums of an h[N] and an hE column
        const double* hN = A.h + ((size_t)b * N1 + N) * 3;
        const double* JhN = A.Jh + ((size_t)b * N1 + N) * 30;
        for (int e = lane; e < nhN * 10; e += 64) {
            const int j = e / 10, l = e - 10 * j;
            int c1 = -1, c2 = -1;
#pragma unroll
            for (int q = 0; q < QP_NHN; ++q)
                if (q == j) { c1 = A.hN_col[q]; c2 = A.hE_col[q]; }
            double v = 0.0, cv = 0.0;
            if (c1 >= 0) { v += hN[c1]; cv += JhN[l * 3 + c1]; }
            if (c2 >= 0) { v += A.hE[(size_t)b * 6 + c2]; cv += A.JhE[((size_t)b * 10 + l) * 6 + c2]; }
            s.ctN[e] = cv;
            if (l == 0) s.hv[NGS + j] = v;
        }
    }
    {
        double v = 0.0;  // constant indices: scalar loads of the kernel arguments
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (lane == i) v = A.lbu[i];
            if (lane == 4 + i) v = A.ubu[i];
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            if (lane == CST_ROW + 4 * j) v = A.lh[j];
            if (lane == CST_ROW + 4 * j + 1) v = A.uh[j];
            if (lane == CST_ROW + 4 * j + 2) v = A.zl[j];
            if (lane == CST_ROW + 4 * j + 3) v = A.Zl[j];
        }
#pragma unroll
        for (int j = 0; j < QP_NHN; ++j) {
            if (lane == CST_TERM + 4 * j) v = A.lhN[j];
            if (lane == CST_TERM + 4 * j + 1) v = A.uhN[j];
            if (lane == CST_TERM + 4 * j + 2) v = j < 3 ? A.zlN[j < 3 ? j : 0] : 0.0;
            if (lane == CST_TERM + 4 * j + 3) v = j < 3 ? A.ZlN[j < 3 ? j : 0] : 0.0;
        }
        if (lane < CST_TERM + 4 * QP_NHN) s.cst[lane] = v;
    }
    for (int e = lane; e < N1; e += 64) s.skv[e] = (A.cost_scaling && e < N) ? A.dt[e] : 1.0;
    if (A.sdf_row_patch && A.sdf_row >= 0) {  // records packed beside the SDF kernel (pack_part 1): their sdf row of C^T
        double* Rw = A.work + (size_t)b * qp_work_doubles(N);
        const int ro = R_CT + 10 * A.sdf_row;
        for (int e = lane; e < N * NX; e += 64) {
            const int k = e / NX, l = e - k * NX;
            Rw[(size_t)k * REC + ro + l] = A.Jh[((size_t)b * N1 + k) * 30 + l * 3 + 2];
        }
        __threadfence_block();  // stored before any lane of the wave streams the records
    }
    if (lane < NX) s.dx[lane] = A.x0[(size_t)b * 10 + lane] - A.x[(size_t)b * N1 * 10 + lane];
    if (lane < 48) s.zero[lane] = 0.0;
    if (HARD && lane >= nss && lane < NSS) {  // node 0's hard groups: no row, a zero fold (QpRows)
        s.fw[lane] = 0.0;
        s.fg[lane] = 0.0;
    }
    __syncthreads();
    STAMP(0);

    // ------------------------------------------------------------ record stream
    // Stream positions: sweep 0 (initial forward), then per IPM iteration sweeps 1 (backward factor),
    // 2 (forward), 3 (backward corrector), 4 (forward); each sweep has NP = N+1 rounded up to a
    // multiple of PD positions (tail positions load a clamped record and compute nothing).  The ring
    // slot of a position is static (loops unrolled by PD), so the compiler waits only for the slot it
    // commits; the window loads of every kind are unpredicated (clamped addresses).
    const int NP = (N1 + PD - 1) / PD * PD;
    double ring[PD][SLOT];
    // fn(IC<S>) for the ring slots S = 0 .. PD - 1 in order (static slots: the loops are unrolled by PD)
    auto each_slot = [](auto&& fn) { for_each_ic(fn, std::make_integer_sequence<int, PD>{}); };
    auto issue = [&](auto KIc, double* rs, int q) {
        constexpr int KI = decltype(KIc)::value;
        const int qq = q < N ? q : N;
        const int k = (KI == 1 || KI == 3) ? N - qq : qq;
        const double* rb = R + (size_t)k * REC;
        const double* fb = F + (size_t)k * FREC;
#pragma unroll
        for (int j = 0; j < n_loads(KI); ++j) {
            const int e = load_at(KI, j) + lane;
            if (load_f(KI, j)) rs[j] = fb[e < f_end(KI) ? e : f_end(KI) - 1];
            else rs[j] = rb[e < r_end(KI) ? e : r_end(KI) - 1];
        }
    };
    auto commit = [&](auto Kc, const double* rs) {
        constexpr int K = decltype(Kc)::value;
#pragma unroll
        for (int j = 0; j < n_loads(K); ++j) win[lane + 64 * j] = rs[j];
    };

    // box rows (k, i, up): t = +-du + d, d = (u - lbu) | (ubu - u)
    auto box_d = [&](int k, int i, int up) -> double {
        const double u = s.uu[k * 4 + i];
        return up ? s.cst[4 + i] - u : u - s.cst[0 + i];
    };

    // ------------------------------------------------------------ forward stage
    // lane r < 10: row r of A~ x + b~ (x_{k+1}); r = 10..13: row of K x + k_ff (u_k); r = 14..16:
    // (C x)_{r-14}; kind 0 (initial iterate, u = 0): rows r < 10 of A x + c from the stage record.
    // Factor rows of nodes < PD come from fsave (written late in the backward sweeps).
    double chain = 0.0;  // p_{k+1} of the corrector sweep in lanes 0..9
    auto fw_stage = [&](auto Kc, int k, const int lane, auto&& hook) {
        const bool fx = lane < NX, fu = lane >= NX && lane < 14, fc = lane >= 14 && lane < 14 + NS;
        const int fcj = fc ? lane - 14 : 0;
        constexpr int K = decltype(Kc)::value;
        ldsd* const dxo = K == 0 ? s.dx : s.dxc;
        ldsd* const duo = K == 4 ? s.duc : s.dua;
        ldsd* const cxo = K == 4 ? s.cxc : s.cxa;
        double row[NX], off;
        if constexpr (K == 0) {
            const ldsd* rp = fx ? win + R_AB + lane : fc ? win + R_CT + fcj * 10 : win;
            const int str = fx ? 10 : 1;
#pragma unroll
            for (int l = 0; l < NX; ++l) row[l] = rp[l * str];
            off = *(fx ? win + R_C + lane : s.zero);
            // + B du_k of the start iterate (0 on a cold start): B[r][j] at R_AB + 10 (NX + j) + r
            const int bx = fx ? lane : 0, ku = k < N ? k : N - 1;
            const double bdu = win[R_AB + 100 + bx] * s.du[ku * NU] + win[R_AB + 110 + bx] * s.du[ku * NU + 1] +
                               win[R_AB + 120 + bx] * s.du[ku * NU + 2] + win[R_AB + 130 + bx] * s.du[ku * NU + 3];
            off += (fx ? 1.0 : 0.0) * bdu;
        } else {
            const ldsd* fk = k < PD ? s.fsave + k * F_FW : win;
            // 16-byte aligned rows: [A~ | b~] / [K | k_ff] row `lane`, C^T row lane - 14, zeros
            const ldsd2* rp = (const ldsd2*)(lane < 14 ? fk + lane * FR : fc ? win + WF_CT + fcj * 10 : s.zero);
#pragma unroll
            for (int l = 0; l < NX / 2; ++l) {
                const d2 v = rp[l];
                row[2 * l] = v.x;
                row[2 * l + 1] = v.y;
            }
            off = *(lane < 14 ? fk + lane * FR + 10 : s.zero);
        }
        const ldsd2* xp = (const ldsd2*)(dxo + k * NX);
        d2 xv[NX / 2];  // the chain input x_k, read after everything else
#pragma unroll
        for (int l = 0; l < NX / 2; ++l) xv[l] = xp[l];
        hook();  // every window read of the stage is issued: the next position's window may be committed
        __builtin_amdgcn_sched_barrier(0);
        double a0 = off, a1 = 0.0;
#pragma unroll
        for (int l = 0; l < NX / 2; ++l) {
            a0 = fma(row[2 * l], xv[l].x, a0);
            a1 = fma(row[2 * l + 1], xv[l].y, a1);
        }
        const double z = a0 + a1;
        // the terminal node's rows are formed after the sweep (term_cx): any row set, C rows from LDS
        ldsd* dst = (fc && k < N) ? cxo + k * NS + fcj
                  : (k < N && fx) ? dxo + (k + 1) * NX + lane
                  : (K != 0 && k < N && fu) ? duo + k * NU + lane - NX : s.junk;
        *dst = z;
    };

    // C dx_N of the terminal rows into cxo[NGS + j] (after a forward sweep): lane j < nhN, the fw_stage's
    // two-chain order (even / odd entries)
    auto term_cx = [&](ldsd* cxo, const ldsd* dxv) {
        if (lane < nhN) {
            const ldsd* cr = s.ctN + 10 * lane;
            const ldsd* xr = dxv + N * NX;
            double a0 = 0.0, a1 = 0.0;
#pragma unroll
            for (int l = 0; l < NX / 2; ++l) {
                a0 = fma(cr[2 * l], xr[2 * l], a0);
                a1 = fma(cr[2 * l + 1], xr[2 * l + 1], a1);
            }
            cxo[NGS + lane] = a0 + a1;
        }
        wave_sync();
    };

    // ------------------------------------------------------------ backward stage, factor
    // Lane maps (fixed for the solve): accumulator rows a_r = g + 4 r of column c; operand k-step st
    // covers k = 4 st + g.  Every lane-dependent read is a precomputed window index (R_Z: a zero) and
    // every store of an inactive lane goes to a junk slot.
    auto fs_at = [&](int k, int e) -> ldsd* { return e < F_FW ? s.fsave + k * F_FW + e : s.junk; };

#define FBST(v, off) bst(v, rsF, off, sko)
    d4 Pa = {0.0, 0.0, 0.0, 0.0};  // [P | p] of the node ahead, accumulator layout
    auto bf_stage = [&](auto Fc, int q, const FConst& f, auto&& hook) {
        constexpr bool FIRST = decltype(Fc)::value;  // q == 0: the terminal node
        const int g = f.g, c = f.c;
        const int og01 = f.og01, og2 = f.og2, cgi = f.cgi, gj = f.gj, gj4 = f.g, ab01 = f.ab01, ab2 = f.ab2;
        const int bmi = f.bmi, hxu_i = f.hxu_i, huu_i = f.huu_i, v0_i = f.v0_i;
        int h_i[4], bi[2];
        unsigned spc[3], sab[3];
#pragma unroll
        for (int r = 0; r < 4; ++r) h_i[r] = f.h_i[r];
#pragma unroll
        for (int r = 0; r < 3; ++r) {
            spc[r] = f.spc[r];
            sab[r] = f.sab[r];
        }
        const unsigned sk_ = f.sk_;
        const double m14 = c == 14 ? 1.0 : 0.0, mg3 = g < NS ? 1.0 : 0.0;  // fold lanes: stage rows g < NS
        double bxm[2], bvm[2], mg[4];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int a = g + 4 * (2 + h);
            const bool in = a >= NX && a < 14;
            bi[h] = in ? a - NX : 0;
            bxm[h] = (in && c == a) ? 1.0 : 0.0;
            bvm[h] = (in && c == 14) ? 1.0 : 0.0;
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) mg[i] = g == i ? 1.0 : 0.0;
        const double huu_b = (c & 3) == g ? 1.0 : 0.0;  // box diagonal of R^0 (replicated 4x4x4 A block)
        const double v0_bd = c == NX + g ? 1.0 : 0.0, v0_bv = c == 14 ? 1.0 : 0.0;

        const int k = N - q;
        if constexpr (FIRST) {  // [P_N | p_N] = [H_N | g_N] + fold of the terminal rows (C from LDS, K = 4 per MFMA)
            d4 T;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int a = g + 4 * r, lo = a < c ? a : c, hi = a < c ? c : a;
                T[r] = win[(a < NX && c < NX) ? R_H + tri10(lo, hi) : (a < NX && c == 14) ? R_G + a : R_Z];
            }
            Pa = T;
            hook();
            for (int t0 = 0; t0 < nhN; t0 += 4) {
                const int jr = t0 + g;
                const bool live = jr < nhN;
                const double cg = (live && c < NX) ? s.ctN[10 * (live ? jr : 0) + (c < NX ? c : 0)] : 0.0;
                const double fb = live ? fma(s.fw[NGS + jr], cg, m14 * s.fg[NGS + jr]) : 0.0;
                Pa = mfma(cg, fb, Pa);
            }
            return;
        }
        const double cg = win[cgi];
        const double fb = mg3 * fma(s.fw[k * NS + gj], cg, m14 * s.fg[k * NS + gj]);
        const unsigned sko = (unsigned)k * (FREC * 8u);
        FSTAMP(8, Pa[0]);
        // ---- W = P G (K = 10: k-steps 0..2); column 14 -> P c, then + p
        const double og0 = win[og01], og1 = win[og01 + 4], og2v = win[og2];
        const double bq0 = win[f.bq[0]], bq1 = win[f.bq[1]], bq2 = win[f.bq[2]];
        const double hv0 = win[v0_i] + v0_bd * s.bd[k * NU + gj4] + v0_bv * s.bv[k * NU + gj4];
        FSTAMP(8, og0 + og1 + og2v);
        d4 W = {0.0, 0.0, 0.0, 0.0};
        W = mfma(Pa[0], og0, W);
        W = mfma(Pa[1], og1, W);
        W = mfma(Pa[2], og2v, W);
        __builtin_amdgcn_sched_barrier(0);  // the W chain goes first; the rest fills its latency
        FSTAMP(8, W[3]);
#pragma unroll
        for (int r = 0; r < 3; ++r) FBST(W[r], spc[r]);
#pragma unroll
        for (int r = 0; r < 3; ++r) W[r] = fma(m14, Pa[r], W[r]);
        // ---- rows 10..13 of M' ([S | R^ | m_u] = [H_u | g_u] + box terms + B^T W), lane (i, c): M'[10 + i][c]
        double Mu = mfma4(bq0, W[0], hv0);
        Mu = mfma4(bq1, W[1], Mu);
        Mu = mfma4(bq2, W[2], Mu);
        __builtin_amdgcn_sched_barrier(0);  // M_u ahead of everything else on the matrix pipe
        // B^T P (lane (g, c): (P B)[c][g], the A operand of P B [K | k_ff] below)
        double Ub = mfma4(bq0, Pa[0], 0.0);
        Ub = mfma4(bq1, Pa[1], Ub);
        Ub = mfma4(bq2, Pa[2], Ub);
        // H^ = [H | g] + C^T diag(w) [C | gamma] + box terms (the Joseph form's stage term)
        d4 Hh;
#pragma unroll
        for (int r = 0; r < 4; ++r) Hh[r] = win[h_i[r]];
#pragma unroll
        for (int h = 0; h < 2; ++h)
            Hh[2 + h] += bxm[h] * s.bd[k * NU + bi[h]] + bvm[h] * s.bv[k * NU + bi[h]];
        d4 Ab;  // closed-loop init [A | c] (rows 12..15: don't care)
        Ab[0] = win[ab01];
        Ab[1] = win[ab01 + 4];
        Ab[2] = win[ab2];
        Ab[3] = 0.0;
        const double bm = win[bmi];
        const double hxa = win[hxu_i];
        const double hua = win[huu_i] + huu_b * s.bd[k * NU + gj4];
        hook();  // the last window read of the stage: the next position's window may be committed
        Hh = mfma(cg, fb, Hh);
        FSTAMP(9, Mu);
        // ---- L = chol(R^): R^[i][j] = M'[10+i][10+j] at lane 16 i + 10 + j
        const double r00 = rdlane(Mu, 10), r10 = rdlane(Mu, 26), r20 = rdlane(Mu, 42), r30 = rdlane(Mu, 58);
        const double r11 = rdlane(Mu, 27), r21 = rdlane(Mu, 43), r31 = rdlane(Mu, 59);
        const double r22 = rdlane(Mu, 44), r32 = rdlane(Mu, 60), r33 = rdlane(Mu, 61);
        // rows 10..13 of M' of column c into every lane of that column
        const double s0 = __shfl(Mu, c), s1 = __shfl(Mu, 16 + c), s2 = __shfl(Mu, 32 + c), s3 = __shfl(Mu, 48 + c);
        const double i0 = rsqrt_nr(r00);
        const double l10 = r10 * i0, l20 = r20 * i0, l30 = r30 * i0;
        const double i1 = rsqrt_nr(r11 - l10 * l10);
        const double l21 = (r21 - l20 * l10) * i1, l31 = (r31 - l30 * l10) * i1;
        const double i2 = rsqrt_nr(r22 - l20 * l20 - l21 * l21);
        const double l32 = (r32 - l30 * l20 - l31 * l21) * i2;
        const double i3 = rsqrt_nr(r33 - l30 * l30 - l31 * l31 - l32 * l32);
        // column c of [Y | w] = L^-1 [S | m_u],  [K | k_ff] = -L^-T [Y | w]
        const double y0 = s0 * i0;
        const double y1 = (s1 - l10 * y0) * i1;
        const double y2 = (s2 - l20 * y0 - l21 * y1) * i2;
        const double y3 = (s3 - l30 * y0 - l31 * y1 - l32 * y2) * i3;
        const double k3 = -y3 * i3;
        const double k2 = (-y2 - l32 * k3) * i2;
        const double k1 = (-y1 - l21 * k2 - l31 * k3) * i1;
        const double k0 = (-y0 - l10 * k1 - l20 * k2 - l30 * k3) * i0;
        const double kg = mg[0] * k0 + mg[1] * k1 + mg[2] * k2 + mg[3] * k3;
        FSTAMP(10, kg);
        // ---- Joseph form: [P | p] <- T^T H^ T + A~^T [P A~ | P b~ + p],  T = [I 0; K k_ff; 0 1]
        // (a sum of PSD terms: no cancellation of M'_xx - Y^T Y when a hard state row puts a huge fold
        // into P; that cancellation costs ~1e-6 absolute accuracy and the IPM its worst-case iterations)
        // with [P A~ | P b~ + p] = [P A | P c + p] + (P B) [K | k_ff]: one product after K, from W
        const double V = mfma4(hua, kg, hv0);                       // rows 10..13 of H^ T
        Ab = mfma(bm, kg, Ab);                                      // [A~ | b~] = [A | c] + B [K | k_ff]
        const d4 W2 = mfma(Ub, kg, W);                              // [P A~ | P b~ + p]
        Hh = mfma(hxa, kg, Hh);                                     // H^_x T
        Hh = mfma(kg, V, Hh);                                       // + K^T (H^_u T)
        Pa = mfma(Ab[0], W2[0], Hh);
        Pa = mfma(Ab[1], W2[1], Pa);
        Pa = mfma(Ab[2], W2[2], Pa);
        FSTAMP(11, Pa[2]);
        __builtin_amdgcn_sched_barrier(0);  // hand P to the next stage before the record stores
        // ---- factor record (and its LDS copy for the first forward stages)
        FBST(kg, sk_);
        {  // the (uniform) Cholesky factor: every lane stores the same 16 bytes, no lane selection
            d2* Lp = (d2*)(F + (size_t)k * FREC + F_L);
            Lp[0] = d2{i0, l10}; Lp[1] = d2{i1, l20}; Lp[2] = d2{l21, i2}; Lp[3] = d2{l30, l31}; Lp[4] = d2{l32, i3};
        }
#pragma unroll
        for (int r = 0; r < 3; ++r) FBST(Ab[r], sab[r]);
        if (k < PD) {
#pragma unroll
            for (int r = 0; r < 3; ++r) *fs_at(k, sab[r] / 8) = Ab[r];
            *fs_at(k, sk_ / 8) = kg;
        }
        FSTAMP(12, kg);
    };

    // ------------------------------------------------------------ backward stage, corrector
    // v = P c + p_{k+1};  lane r < 10: p_k[r] = g~_x[r] + (K^T g~_u)[r] + (A~^T v)[r]   (the chain)
    //                     lane 10 + i: z_u[i] = g~_u[i] + (B^T v)[i]
    // then w = L^-1 z_u, k_ff = -L^-T w, b~ = c + B k_ff (off the chain).  g~ = g + fold | box.
    auto bc_stage = [&](auto Fc, int q, const int lane, auto&& hook) {
        constexpr bool FIRST = decltype(Fc)::value;
        const bool fx = lane < NX, fu = lane >= NX && lane < 14;
        const ldsd* bc_row = fx ? win + F_AB + lane : fu ? win + WB_R + lane * 10 : win;
        const int bc_str = fx ? FR : 1;
        const ldsd* bc_ct = fx ? win + WB_R + R_CT + lane : s.zero;  // C^T[j][r] at + 10 j
        const ldsd* bc_k = fx ? win + F_K + lane : s.zero;           // K[i][r] at + FR i
        const ldsd* bc_g = lane < 14 ? win + WB_R + R_G + lane : s.zero;
        const double mfx = fx ? 1.0 : 0.0;
        double mu_[NU];
    #pragma unroll
        for (int i = 0; i < NU; ++i) mu_[i] = lane == NX + i ? 1.0 : 0.0;
        const int bx = fx ? lane : 0;
        const unsigned bc_st = lane < 14 ? lane * FR + 10 : F_J;  // b~ rows (lanes < 10), k_ff rows (lanes 10..13)
        const int k = N - q;
        FSTAMP(7, mfx);
        double off = *bc_g;
        if constexpr (FIRST) {  // p_N = g_N + sum_j gamma_j C_j^T over the terminal rows (C from LDS)
            hook();
            const ldsd* ct = fx ? s.ctN + lane : s.zero;
            for (int j = 0; j < nhN; ++j) off += s.fg[NGS + j] * ct[fx ? 10 * j : 0];
            chain = off;
            return;
        }
#pragma unroll
        for (int j = 0; j < NS; ++j) off += s.fg[k * NS + j] * bc_ct[10 * j];
        // ---- every LDS read of the stage first (one round trip), the chain input p_{k+1} last
        double bvv[NU], guw[NU], kk[NU], row[NX];
        {  // the uniform box and g~_u terms as 16-byte reads (both blocks are 16-byte aligned)
            const ldsd2* bq = (const ldsd2*)(s.bv + k * NU);
            const ldsd2* gq = (const ldsd2*)(win + WB_R + R_G + NX);
            const d2 b0 = bq[0], b1 = bq[1], g0 = gq[0], g1 = gq[1];
            bvv[0] = b0.x; bvv[1] = b0.y; bvv[2] = b1.x; bvv[3] = b1.y;
            guw[0] = g0.x; guw[1] = g0.y; guw[2] = g1.x; guw[3] = g1.y;
        }
#pragma unroll
        for (int i = 0; i < NU; ++i) kk[i] = bc_k[FR * i];
#pragma unroll
        for (int l = 0; l < NX; ++l) row[l] = bc_row[l * bc_str];
        const ldsd2* pc = (const ldsd2*)(win + F_PC);
        const ldsd2* Lq = (const ldsd2*)(win + F_L);
        d2 pcv[NX / 2], Lv[5];
#pragma unroll
        for (int l = 0; l < NX / 2; ++l) {
            pcv[l] = pc[l];
            Lv[l] = Lq[l];
        }
        const double cb = win[WB_R + R_C + bx], B0 = win[WB_R + 100 + bx], B1 = win[WB_R + 110 + bx];
        const double B2 = win[WB_R + 120 + bx], B3 = win[WB_R + 130 + bx];
        hook();  // the last window read of the stage: the next position's window may be committed
        // the chain input p_{k+1}: lanes 0..9 of the register chain, broadcast through scalar registers
        double pv[NX];
#pragma unroll
        for (int l = 0; l < NX; ++l) pv[l] = rdlane(chain, l);
        FSTAMP(13, pv[9] + B3 + row[9] + Lv[4].y + pcv[4].y + kk[3]);
        // g~_u (uniform) and the per-lane offset of the chain
#pragma unroll
        for (int i = 0; i < NU; ++i) off += kk[i] * (guw[i] + bvv[i]) + mu_[i] * bvv[i];
        double a0 = off, a1 = 0.0;
#pragma unroll
        for (int l = 0; l < NX / 2; ++l) {
            a0 = fma(row[2 * l], pcv[l].x + pv[2 * l], a0);
            a1 = fma(row[2 * l + 1], pcv[l].y + pv[2 * l + 1], a1);
        }
        const double z = a0 + a1;
        chain = z;
        FSTAMP(14, z);
        // off the chain: k_ff, b~
        const double z0 = rdlane(z, 10), z1 = rdlane(z, 11), z2 = rdlane(z, 12), z3 = rdlane(z, 13);
        const double i0 = Lv[0].x, l10 = Lv[0].y, i1 = Lv[1].x, l20 = Lv[1].y, l21 = Lv[2].x;
        const double i2 = Lv[2].y, l30 = Lv[3].x, l31 = Lv[3].y, l32 = Lv[4].x, i3 = Lv[4].y;
        const double w0 = z0 * i0;
        const double w1 = (z1 - l10 * w0) * i1;
        const double w2 = (z2 - l20 * w0 - l21 * w1) * i2;
        const double w3 = (z3 - l30 * w0 - l31 * w1 - l32 * w2) * i3;
        const double k3 = -w3 * i3;
        const double k2 = (-w2 - l32 * k3) * i2;
        const double k1 = (-w1 - l21 * k2 - l31 * k3) * i1;
        const double k0 = (-w0 - l10 * k1 - l20 * k2 - l30 * k3) * i0;
        const double bb = cb + B0 * k0 + B1 * k1 + B2 * k2 + B3 * k3;
        const double fv = mfx * bb + mu_[0] * k0 + mu_[1] * k1 + mu_[2] * k2 + mu_[3] * k3;
        bst(fv, rsF, 8u * bc_st, (unsigned)k * (FREC * 8u));
        if (k < PD) *fs_at(k, bc_st) = fv;
        FSTAMP(15, fv);
    };

    // ------------------------------------------------------------ initial iterate (dynamics-feasible):
    // du = sl = su = 0 (warm start: du = the previous QP's), dx_0 = x0 - xbar_0, dx_{k+1} = A dx_k + B du_k + c_k
    // (sweep 0), then the rows
    auto rows_init = [&]() -> double {
    double rp = 0.0;
    for (int r = lane; r < RH0; r += 64) {
        double v, l0 = L0;
        if (r < 8 * N) {
            const int k = r >> 3, q = r & 7, i = q & 3, up = q >> 2;
            v = box_d(k, i, up) + (up ? -s.du[k * NU + i] : s.du[k * NU + i]);
        } else {
            const int e = soft_e((r - 8 * N) >> 2), kind = (r - 8 * N) & 3, k = gnode(e);
            const ldsd* gc = gcst(e);
            const double h = s.hv[e];
            v = kind == 0 ? s.cxa[e] + (h - gc[0]) : kind == 1 ? -s.cxa[e] + (gc[1] - h) : 0.0;
            l0 = fmax(L0, LC * s.skv[k] * gc[2]);
        }
        const double t = fmax(v, T0);
        s.t[r] = t;
        s.lam[r] = l0;
        rp = fmax(rp, fabs(v - t));
    }
    if constexpr (HARD) for (int r = RH0 + lane; r < m; r += 64) {  // hard rows: lower, upper
        const int i = (r - RH0) >> 1, up = (r - RH0) & 1, e = hard_e(i);
        const ldsd* gc = gcst(e);
        const double v = up ? -s.cxa[e] + (gc[1] - s.hv[e]) : s.cxa[e] + (s.hv[e] - gc[0]);
        const double t = fmax(v, T0);
        s.t[r] = t;
        s.lam[r] = L0;
        rp = fmax(rp, fabs(v - t));
    }
    return wmax(rp);
    };

    // soft group e = rows (hl, hu, sl, su): barrier weights, v's, eliminated slack block.
    // Divisions are reciprocal multiplications (rcp_nr: v_rcp_f64 + two Newton steps), one per
    // denominator.
    struct Grp {
        double s1, s2, s3, s4, v1, v2, v3, v4, Hl, Hu, iHl, iHu, gl, gu;
    };
    auto group = [&](int e, int r0, int phase, double sigmu) -> Grp {  // group e, rows r0 .. r0 + 3
        Grp g;
        const double sk = s.skv[gnode(e)];
        const ldsd* gc = gcst(e);
        const double t1 = s.t[r0], t2 = s.t[r0 + 1], t3 = s.t[r0 + 2], t4 = s.t[r0 + 3];
        const double l1 = s.lam[r0], l2 = s.lam[r0 + 1], l3 = s.lam[r0 + 2], l4 = s.lam[r0 + 3];
        const double it1 = rcp_nr(t1), it2 = rcp_nr(t2), it3 = rcp_nr(t3), it4 = rcp_nr(t4);
        g.s1 = l1 * it1; g.s3 = l2 * it2; g.s2 = l3 * it3; g.s4 = l4 * it4;
        const double h = s.hv[e];
        g.v1 = g.s1 * (t1 - (h - gc[0]));
        g.v3 = g.s3 * (t2 - (gc[1] - h));
        g.v2 = g.s2 * t3;
        g.v4 = g.s4 * t4;
        const double Zs = sk * gc[3], zs = sk * gc[2];
        g.Hl = Zs + g.s1 + g.s2;
        g.Hu = Zs + g.s3 + g.s4;
        g.iHl = rcp_nr(g.Hl);
        g.iHu = rcp_nr(g.Hu);
        if (phase) {  // corrector: affine deltas of the four rows, recomputed from the affine solution
            const double cxa = s.cxa[e];
            const double sla = -((zs - g.v1 - g.v2) + g.s1 * cxa) * g.iHl;
            const double sua = -((zs - g.v3 - g.v4) - g.s3 * cxa) * g.iHu;
            const double d1 = cxa + (h - gc[0]) + sla - t1;
            const double d2 = -cxa + (gc[1] - h) + sua - t2;
            const double d3 = sla - t3, d4 = sua - t4;
            g.v1 -= (d1 * (-g.s1 * d1 - l1) - sigmu) * it1;
            g.v3 -= (d2 * (-g.s3 * d2 - l2) - sigmu) * it2;
            g.v2 -= (d3 * (-g.s2 * d3 - l3) - sigmu) * it3;
            g.v4 -= (d4 * (-g.s4 * d4 - l4) - sigmu) * it4;
        }
        g.gl = zs - g.v1 - g.v2;
        g.gu = zs - g.v3 - g.v4;
        return g;
    };
    auto box_v = [&](int k, int i, int up, int phase, double sigmu) -> double {
        const int r = 8 * k + 4 * up + i;
        const double t = s.t[r], l = s.lam[r], it = rcp_nr(t), sg = l * it;
        double v = sg * (t - box_d(k, i, up));
        if (phase) {
            const double da = (up ? -s.dua[k * NU + i] : s.dua[k * NU + i]) + box_d(k, i, up) - t;
            v -= (da * (-sg * da - l) - sigmu) * it;
        }
        return v;
    };
    // hard row i, side up: the constant d of t = +-C dx + d, and the value at C dx = cxs
    auto hard_d = [&](int i, int up) -> double {
        const int e = hard_e(i);
        const ldsd* gc = gcst(e);
        return up ? gc[1] - s.hv[e] : s.hv[e] - gc[0];
    };
    auto hard_v = [&](int i, int up, int phase, double sigmu) -> double {  // box_v of a hard row
        const int r = RH0 + 2 * i + up;
        const double t = s.t[r], l = s.lam[r], it = rcp_nr(t), sg = l * it, d = hard_d(i, up);
        double v = sg * (t - d);
        if (phase) {
            const double cxa = s.cxa[hard_e(i)];
            const double da = (up ? -cxa : cxa) + d - t;
            v -= (da * (-sg * da - l) - sigmu) * it;
        }
        return v;
    };
    // all groups at once, before a backward sweep: fw = w (factor only), fg = gamma, box diag / v
    auto terms = [&](int phase, double sigmu) {
        for (int si = lane; si < NG1; si += 64) {
            const int e = soft_e(si);
            const Grp g = group(e, 8 * N + 4 * si, phase, sigmu);
            // fold of the eliminated slack pair, written without the cancellation of H - s1 (H = Zs + s1 + s2
            // with s1 -> inf on an active row):  w = s1 (Zs + s2) / Hl + ...,  gamma = -(v1 + s1 gl / Hl) + ...
            const ldsd* gc = gcst(e);
            const double sk = s.skv[gnode(e)];
            const double Zs = sk * gc[3], zs = sk * gc[2];
            if (!phase) s.fw[e] = g.s1 * (Zs + g.s2) * g.iHl + g.s3 * (Zs + g.s4) * g.iHu;
            s.fg[e] = -(g.v1 * (Zs + g.s2) + g.s1 * (zs - g.v2)) * g.iHl + (g.v3 * (Zs + g.s4) + g.s3 * (zs - g.v4)) * g.iHu;
        }
        if constexpr (HARD)  // hard rows fold like box rows: w = sigma_l + sigma_u, gamma = -v_l + v_u
            for (int i = lane; i < NHT; i += 64) {
                const int r = RH0 + 2 * i, e = hard_e(i);
                if (!phase) s.fw[e] = s.lam[r] * rcp_nr(s.t[r]) + s.lam[r + 1] * rcp_nr(s.t[r + 1]);
                s.fg[e] = -hard_v(i, 0, phase, sigmu) + hard_v(i, 1, phase, sigmu);
            }
        for (int e = lane; e < N * NU; e += 64) {
            const int k = e >> 2, i = e & 3;
            if (!phase) s.bd[e] = s.lam[8 * k + i] * rcp_nr(s.t[8 * k + i]) + s.lam[8 * k + 4 + i] * rcp_nr(s.t[8 * k + 4 + i]);
            s.bv[e] = -box_v(k, i, 0, phase, sigmu) + box_v(k, i, 1, phase, sigmu);
        }
        wave_sync();
    };


    // row values of soft group e at an LQR solution with C dx = cxs, and its slacks
    auto soft_vals = [&](const Grp& g, int e, double cxs, double* v) {
        const double h = s.hv[e];
        const ldsd* gc = gcst(e);
        const double sl = -(g.gl + g.s1 * cxs) * g.iHl, su = -(g.gu - g.s3 * cxs) * g.iHu;
        v[0] = cxs + (h - gc[0]) + sl;
        v[1] = -cxs + (gc[1] - h) + su;
        v[2] = sl;
        v[3] = su;
    };

    // ------------------------------------------------------------ IPM: sweep driver
    // predictor rows: affine step length, mu_aff -> sigma mu (Mehrotra)
    // mu: mean complementarity (Mehrotra's centring); cm: max complementarity -- the stop test is
    // HPIPM's, max_i t_i lambda_i <= tol and max primal residual <= tol
    // gap = prod (1 - alpha): the stationarity residual of the starting point decays by exactly this
    // factor (every Newton system is solved for the new iterate), the stand-in for HPIPM's res_g test
    double mu = 0.0, cm = 0.0, rp = 0.0, gap = 1.0;
    // (GPL > 0: the soft rows' affine directions are computed once and kept in registers for both passes)
    auto rows_pred_t = [&](auto GPLc) -> double {
        constexpr int GPL = decltype(GPLc)::value;
        constexpr int GA = GPL > 0 ? GPL : 1;
        double amax = 1.0;
        auto bound = [&](double t, double l, double dt, double dl) {
            if (dt < 0.0) amax = fmin(amax, -t * rcp_nr(dt));
            if (dl < 0.0) amax = fmin(amax, -l * rcp_nr(dl));
        };
        for (int r = lane; r < 8 * N; r += 64) {
            const int k = r >> 3, q = r & 7, i = q & 3, up = q >> 2;
            const double t = s.t[r], l = s.lam[r];
            const double dt = (up ? -s.dua[k * NU + i] : s.dua[k * NU + i]) + box_d(k, i, up) - t;
            bound(t, l, dt, -(l * rcp_nr(t)) * dt - l);
        }
        // hard rows (lane 2 i + up)
        auto hard_dir = [&](int r, double& dt, double& dl) {
            const int i = (r - RH0) >> 1, up = (r - RH0) & 1;
            const double t = s.t[r], l = s.lam[r], cxa = s.cxa[hard_e(i)];
            dt = (up ? -cxa : cxa) + hard_d(i, up) - t;
            dl = -(l * rcp_nr(t)) * dt - l;
        };
        if constexpr (HARD)
            for (int r = RH0 + lane; r < m; r += 64) {
                double dt, dl;
                hard_dir(r, dt, dl);
                bound(s.t[r], s.lam[r], dt, dl);
            }
        // affine direction of the four rows of soft group si: dt = val(z_a) - t, dl = -(lambda / t) dt - lambda
        auto soft_dir = [&](int si, double* dt, double* dl) {
            const int r0 = 8 * N + 4 * si, e = soft_e(si);
            const Grp g = group(e, r0, 0, 0.0);
            double v[4];
            soft_vals(g, e, s.cxa[e], v);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double t = s.t[r0 + q], l = s.lam[r0 + q];
                dt[q] = v[q] - t;
                dl[q] = -(l * rcp_nr(t)) * dt[q] - l;
            }
        };
        double sdt[GA][4], sdl[GA][4];
        if constexpr (GPL > 0) {
#pragma unroll
            for (int gi = 0; gi < GPL; ++gi) {
                const int e = lane + 64 * gi;
                if (e < NG1) {
                    soft_dir(e, sdt[gi], sdl[gi]);
#pragma unroll
                    for (int q = 0; q < 4; ++q) bound(s.t[8 * N + 4 * e + q], s.lam[8 * N + 4 * e + q], sdt[gi][q], sdl[gi][q]);
                }
            }
        } else {
            for (int e = lane; e < NG1; e += 64) {
                soft_dir(e, sdt[0], sdl[0]);
#pragma unroll
                for (int q = 0; q < 4; ++q) bound(s.t[8 * N + 4 * e + q], s.lam[8 * N + 4 * e + q], sdt[0][q], sdl[0][q]);
            }
        }
        const double aa = wmin(amax);
        double lmua = 0.0;
        for (int r = lane; r < 8 * N; r += 64) {
            const int k = r >> 3, q = r & 7, i = q & 3, up = q >> 2;
            const double t = s.t[r], l = s.lam[r];
            const double dt = (up ? -s.dua[k * NU + i] : s.dua[k * NU + i]) + box_d(k, i, up) - t;
            lmua += (t + aa * dt) * (l + aa * (-(l * rcp_nr(t)) * dt - l));
        }
        if constexpr (HARD)
            for (int r = RH0 + lane; r < m; r += 64) {
                double dt, dl;
                hard_dir(r, dt, dl);
                lmua += (s.t[r] + aa * dt) * (s.lam[r] + aa * dl);
            }
        auto soft_mu = [&](int si, const double* dt, const double* dl) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double t = s.t[8 * N + 4 * si + q], l = s.lam[8 * N + 4 * si + q];
                lmua += (t + aa * dt[q]) * (l + aa * dl[q]);
            }
        };
        if constexpr (GPL > 0) {
#pragma unroll
            for (int gi = 0; gi < GPL; ++gi) {
                const int e = lane + 64 * gi;
                if (e < NG1) soft_mu(e, sdt[gi], sdl[gi]);
            }
        } else {
            for (int e = lane; e < NG1; e += 64) {
                double dt[4], dl[4];
                soft_dir(e, dt, dl);
                soft_mu(e, dt, dl);
            }
        }
        const double mua = wsum(lmua) / m;
        const double sig = (mua / mu) * (mua / mu) * (mua / mu);
        // centring target floored at 1e-2 tol (HPIPM's tau_min): no row is pushed below the complementarity
        // the stop test needs, which keeps lambda / t -- and the Riccati data -- bounded
        return fmax(sig * mu, 1e-2 * A.tol);
    };
    const int gpl = (NG1 + 63) / 64;
    auto rows_pred = [&]() -> double {
        if (gpl == 1) return rows_pred_t(IC<1>{});
        if (gpl == 2) return rows_pred_t(IC<2>{});
        if (gpl == 3) return rows_pred_t(IC<3>{});
        return rows_pred_t(IC<0>{});
    };
    // corrector rows: step length, update of (t, lambda, du, dx), mu and the primal residual.
    // GPL > 0: every lane owns at most GPL soft groups (NG1 <= 64 GPL); their directions (dt, dl) --
    // the expensive part, two group evaluations with six reciprocals each -- are computed once, kept in
    // registers between the step-length pass and the update pass.  GPL == 0: the generic loops recompute.
    auto rows_update_t = [&](auto GPLc, double sigmu) {
        constexpr int GPL = decltype(GPLc)::value;
        constexpr int GA = GPL > 0 ? GPL : 1;
        double amax = 1.0;
        auto bound = [&](double t, double l, double dt, double dl) {
            if (dt < 0.0) amax = fmin(amax, -t * rcp_nr(dt));
            if (dl < 0.0) amax = fmin(amax, -l * rcp_nr(dl));
        };
        // direction of row r: dt = val(z_c) - t, dl = -sigma dt - l - (dt_a dl_a - sigma mu) / t
        for (int r = lane; r < 8 * N; r += 64) {
            const int k = r >> 3, q = r & 7, i = q & 3, up = q >> 2;
            const double t = s.t[r], l = s.lam[r];
            const double dt = (up ? -s.duc[k * NU + i] : s.duc[k * NU + i]) + box_d(k, i, up) - t;
            const double dta = (up ? -s.dua[k * NU + i] : s.dua[k * NU + i]) + box_d(k, i, up) - t;
            const double it = rcp_nr(t), sg = l * it;
            bound(t, l, dt, -sg * dt - l - (dta * (-sg * dta - l) - sigmu) * it);
        }
        auto hard_dir = [&](int r, double& dt, double& dl) {
            const int i = (r - RH0) >> 1, up = (r - RH0) & 1;
            const double t = s.t[r], l = s.lam[r], d = hard_d(i, up);
            const int e = hard_e(i);
            const double cc = s.cxc[e], ca = s.cxa[e];
            dt = (up ? -cc : cc) + d - t;
            const double dta = (up ? -ca : ca) + d - t;
            const double it = rcp_nr(t), sg = l * it;
            dl = -sg * dt - l - (dta * (-sg * dta - l) - sigmu) * it;
        };
        if constexpr (HARD)
            for (int r = RH0 + lane; r < m; r += 64) {
                double dt, dl;
                hard_dir(r, dt, dl);
                bound(s.t[r], s.lam[r], dt, dl);
            }
        auto soft_dir = [&](int si, double* dt, double* dl) {
            const int r0 = 8 * N + 4 * si, e = soft_e(si);
            const Grp ga = group(e, r0, 0, 0.0), gc = group(e, r0, 1, sigmu);
            double va[4], vc[4];
            soft_vals(ga, e, s.cxa[e], va);
            soft_vals(gc, e, s.cxc[e], vc);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double t = s.t[r0 + q], l = s.lam[r0 + q];
                const double dta = va[q] - t;
                dt[q] = vc[q] - t;
                const double it = rcp_nr(t), sg = l * it;
                dl[q] = -sg * dt[q] - l - (dta * (-sg * dta - l) - sigmu) * it;
            }
        };
        double sdt[GA][4], sdl[GA][4];
        if constexpr (GPL > 0) {
#pragma unroll
            for (int gi = 0; gi < GPL; ++gi) {
                const int e = lane + 64 * gi;
                if (e < NG1) {
                    soft_dir(e, sdt[gi], sdl[gi]);
                    const int r0 = 8 * N + 4 * e;
#pragma unroll
                    for (int q = 0; q < 4; ++q) bound(s.t[r0 + q], s.lam[r0 + q], sdt[gi][q], sdl[gi][q]);
                }
            }
        } else {
            for (int e = lane; e < NG1; e += 64) {
                soft_dir(e, sdt[0], sdl[0]);
                const int r0 = 8 * N + 4 * e;
#pragma unroll
                for (int q = 0; q < 4; ++q) bound(s.t[r0 + q], s.lam[r0 + q], sdt[0][q], sdl[0][q]);
            }
        }
        const double tau = fmin(TAU_HI, fmax(TAU_LO, 1.0 - mu));
        const double al = fmin(1.0, tau * wmin(amax));
        // -------- update (rows read everything they need before writing their own entries)
        double lmu = 0.0, lcm = 0.0;
        for (int r = lane; r < 8 * N; r += 64) {
            const int k = r >> 3, q = r & 7, i = q & 3, up = q >> 2;
            const double t = s.t[r], l = s.lam[r];
            const double dt = (up ? -s.duc[k * NU + i] : s.duc[k * NU + i]) + box_d(k, i, up) - t;
            const double dta = (up ? -s.dua[k * NU + i] : s.dua[k * NU + i]) + box_d(k, i, up) - t;
            const double it = rcp_nr(t), sg = l * it;
            const double dl = -sg * dt - l - (dta * (-sg * dta - l) - sigmu) * it;
            const double tn = t + al * dt, ln = l + al * dl;
            lmu += tn * ln;
            lcm = fmax(lcm, tn * ln);
            s.t[r] = tn;
            s.lam[r] = ln;
        }
        {
            auto soft_upd = [&](int e, const double* dt, const double* dl) {
                const int r0 = 8 * N + 4 * e;
                double tn[4], ln[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    tn[q] = s.t[r0 + q] + al * dt[q];
                    ln[q] = s.lam[r0 + q] + al * dl[q];
                    lmu += tn[q] * ln[q];
                    lcm = fmax(lcm, tn[q] * ln[q]);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    s.t[r0 + q] = tn[q];
                    s.lam[r0 + q] = ln[q];
                }
            };
            if constexpr (GPL > 0) {
#pragma unroll
                for (int gi = 0; gi < GPL; ++gi) {
                    const int e = lane + 64 * gi;
                    if (e < NG1) soft_upd(e, sdt[gi], sdl[gi]);
                }
            } else {
                for (int e = lane; e < NG1; e += 64) {
                    double dt[4], dl[4];
                    soft_dir(e, dt, dl);
                    soft_upd(e, dt, dl);
                }
            }
            if constexpr (HARD)
                for (int r = RH0 + lane; r < m; r += 64) {
                    double hdt, hdl;
                    hard_dir(r, hdt, hdl);
                    const double tn = s.t[r] + al * hdt, ln = s.lam[r] + al * hdl;
                    lmu += tn * ln;
                    lcm = fmax(lcm, tn * ln);
                    s.t[r] = tn;
                    s.lam[r] = ln;
                }
        }
        for (int e = lane; e < N1 * NX; e += 64) s.dx[e] += al * (s.dxc[e] - s.dx[e]);
        for (int e = lane; e < N * NU; e += 64) s.du[e] += al * (s.duc[e] - s.du[e]);
        mu = wsum(lmu) / m;
        cm = wmax(lcm);
        rp *= (1.0 - al);
        gap *= (1.0 - al);
    };
    auto rows_update = [&](double sigmu) {
        if (gpl == 1) rows_update_t(IC<1>{}, sigmu);
        else if (gpl == 2) rows_update_t(IC<2>{}, sigmu);
        else if (gpl == 3) rows_update_t(IC<3>{}, sigmu);
        else rows_update_t(IC<0>{}, sigmu);
    };

    // ------------------------------------------------------------ IPM: sweeps over the record stream
    auto stage = [&](auto Kc, auto Fc, int q, const auto& ln, auto&& hook) {
        constexpr int K = decltype(Kc)::value;
        if constexpr (K == 1) bf_stage(Fc, q, ln, hook);
        else if constexpr (K == 3) bc_stage(Fc, q, ln, hook);
        else fw_stage(Kc, q, ln, hook);
    };
#ifndef QP_LATE_COMMIT
    // one stream position: its window was committed by the previous position's hook; refill its ring slot S
    // with position qi of a sweep of kind KI, run the stage, whose hook -- after the stage's last window read
    // -- commits the next position (ring slot S + 1, kind KN) into the window: the commit's wait for the
    // record loads and its LDS writes run under the stage's arithmetic instead of heading the next stage
    auto position = [&](auto Kc, auto KIc, auto KNc, auto Sc, auto Fc, int q, int qi, bool live, const auto& ln) {
        constexpr int S = decltype(Sc)::value, S1 = (S + 1) % PD;
        issue(KIc, ring[S], qi);
        wave_sync();
        auto hook = [&]() { commit(KNc, ring[S1]); };
        if (live) stage(Kc, Fc, q, ln, hook);
        else hook();
        wave_sync();
    };
#else  // diagnostic: the round-5 schedule (commit at the head of each position)
    auto position = [&](auto Kc, auto KIc, auto KNc, auto Sc, auto Fc, int q, int qi, bool live, const auto& ln) {
        constexpr int S = decltype(Sc)::value;
        commit(Kc, ring[S]);
        issue(KIc, ring[S], qi);
        wave_sync();
        if (live) stage(Kc, Fc, q, ln, [] {});
        wave_sync();
    };
#endif
    auto sweep = [&](auto Kc) {
        constexpr int K = decltype(Kc)::value, KN = K == 4 ? 1 : K + 1;
        // the stages' lane constants derive from an opaque copy of the lane id, so they are hoisted
        // to this sweep's preheader and live only during the sweep (not across the whole solve); the
        // factor sweep's are built up front (fconst) and pinned in registers
        const auto ln = [&] {
            if constexpr (K == 1) return fconst<NSS>(opaque(lane));
            else return opaque(lane);
        }();
        using T_ = IC<1>;
        using F_ = IC<0>;
        // slot S of a trip: position q0 + S (the first position of the sweep is its first node: the
        // terminal node of a backward sweep)
        // KN of a position: the kind of the position after it (the next sweep's first one after the last slot
        // of the last trip)
        using KNL = IC<KN>;
        if (NP > PD) {
            // first trip
            each_slot([&](auto Sc) {
                constexpr int S = decltype(Sc)::value;
                position(Kc, Kc, Kc, Sc, std::conditional_t<S == 0, T_, F_>{}, S, S + PD, true, ln);
            });
            int q0 = PD;
            for (; q0 < NP - PD; q0 += PD)  // every position of these trips is a node
                each_slot([&](auto Sc) {
                    constexpr int S = decltype(Sc)::value;
                    position(Kc, Kc, Kc, Sc, F_{}, q0 + S, q0 + S + PD, true, ln);
                });
            // last trip: refill with the next sweep's first positions; tail positions compute nothing
            each_slot([&](auto Sc) {
                constexpr int S = decltype(Sc)::value;
                position(Kc, IC<KN>{}, std::conditional_t<S == PD - 1, KNL, decltype(Kc)>{}, Sc, F_{}, q0 + S, S,
                         q0 + S < N1, ln);
            });
        } else {  // N + 1 <= PD: a single trip
            each_slot([&](auto Sc) {
                constexpr int S = decltype(Sc)::value;
                position(Kc, IC<KN>{}, std::conditional_t<S == PD - 1, KNL, decltype(Kc)>{}, Sc,
                         std::conditional_t<S == 0, T_, F_>{}, S, S, S == 0 || S < N1, ln);
            });
        }
    };

    each_slot([&](auto Sc) { issue(IC<0>{}, ring[decltype(Sc)::value], decltype(Sc)::value); });
#ifndef QP_LATE_COMMIT
    commit(IC<0>{}, ring[0]);  // the stream's first position (later ones: the previous stage's hook)
    wave_sync();
#endif
    sweep(IC<0>{});
    term_cx(s.cxa, s.dx);
    STAMP(1);
    rp = rows_init();
    {
        double lmu = 0.0, lcm = 0.0;
        for (int r = lane; r < m; r += 64) {
            lmu += s.t[r] * s.lam[r];
            lcm = fmax(lcm, s.t[r] * s.lam[r]);
        }
        mu = wsum(lmu) / m;
        cm = wmax(lcm);
    }
    wave_sync();
    int it = 0;
    // a non-finite iterate (NaN / Inf in the linearisation) stops the instance at once: status 2
    while (!(cm < A.tol && rp < A.tol && gap < A.tol) && it < A.max_iter && __builtin_isfinite(mu + rp)) {
        terms(0, 0.0);
        STAMP(6);
        sweep(IC<1>{});
        STAMP(2);
        if (lane < NX) s.dxc[lane] = s.dx[lane];
        wave_sync();
        sweep(IC<2>{});
        term_cx(s.cxa, s.dxc);
        STAMP(3);
        const double sigmu = rows_pred();
        RSTAMP(8);
        terms(1, sigmu);
        STAMP(4);
        sweep(IC<3>{});
        STAMP(5);
        if (lane < NX) s.dxc[lane] = s.dx[lane];
        wave_sync();
        sweep(IC<4>{});
        term_cx(s.cxc, s.dxc);
        STAMP(3);
        rows_update(sigmu);
        RSTAMP(9);
        wave_sync();
        STAMP(6);
        ++it;
    }
    STAMP_OUT
    // ------------------------------------------------------------ outputs
    for (int e = lane; e < N1 * NX; e += 64) A.dx[(size_t)b * N1 * NX + e] = s.dx[e];
    for (int e = lane; e < N * NU; e += 64) A.du[(size_t)b * N * NU + e] = s.du[e];
    if (A.slack)  // slacks = the t of rows sl >= 0, su >= 0 (equal to the iterate's sl, su up to r_p); [N+1][3][2]
        for (int e = lane; e < N1 * 3; e += 64) {
            const int k = e / 3, j = e - 3 * k;
            const int g = k < N ? (j < nss ? k * nss + j : -1) : (j < A.nsN ? NSG + j : -1);  // soft index
            A.slack[((size_t)b * N1 * 3 + e) * 2] = g >= 0 ? s.t[8 * N + 4 * g + 2] : 0.0;
            A.slack[((size_t)b * N1 * 3 + e) * 2 + 1] = g >= 0 ? s.t[8 * N + 4 * g + 3] : 0.0;
        }
    if (lane == 0) {
        A.iters[b] = it;
        // 0 converged; 1 max_iter reached (acados status 2, the step is kept); 2 numerical failure (acados
        // QP failure, status 4: rti_apply keeps this instance's iterate)
        A.status[b] = !__builtin_isfinite(mu + rp) ? 2 : (cm < A.tol && rp < A.tol && gap < A.tol) ? 0 : 1;
        A.res[b * 2] = cm;
        A.res[b * 2 + 1] = rp;
    }
}

__global__ __launch_bounds__(256) void rti_apply_kernel(int B, int N, double* x, double* u, const double* dx,
                                                       const double* du, double* u0, const int* status) {
    const long long nx = (long long)B * (N + 1) * 10, nu = (long long)B * N * 4;
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < nx) {
        const bool keep = status && status[i / ((long long)(N + 1) * 10)] >= 2;
        if (!keep) x[i] += dx[i];
    }
    if (i < nu) {
        const long long bb = i / ((long long)N * 4), r = i - bb * N * 4;
        const bool keep = status && status[bb] >= 2;
        const double v = keep ? u[i] : u[i] + du[i];
        u[i] = v;
        if (u0 && r < 4) u0[bb * 4 + r] = v;
    }
}

hipError_t launch_rti_apply(int B, int N, double* x, double* u, const double* dx, const double* du, double* u0,
                            const int* status, hipStream_t s) {
    const long long n = (long long)B * (N + 1) * 10;
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(rti_apply_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, B, N, x, u, dx, du, u0,
                       status);
    return hipGetLastError();
}

hipError_t launch_rti_qp_pack(const QpArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    hipLaunchKernelGGL(rti_qp_pack_kernel, dim3((unsigned)((a.B * (a.N + 1) + PACK_NODES - 1) / PACK_NODES)),
                       dim3(64 * PACK_NODES), 0, s, a);
    return hipGetLastError();
}

// the kernel instantiation of a stage row count
template <bool HARD>
static const void* rti_qp_fn_h(int nh) {
    switch (nh) {
        case 0: return (const void*)rti_qp_kernel<0, HARD>;
        case 1: return (const void*)rti_qp_kernel<1, HARD>;
        case 2: return (const void*)rti_qp_kernel<2, HARD>;
        default: return (const void*)rti_qp_kernel<3, HARD>;
    }
}
// the kernel instantiation of a row set
static const void* rti_qp_fn(QpRows q) {
    return (q.nhN > q.nsN || q.nhs > 0) ? rti_qp_fn_h<true>(q.ns) : rti_qp_fn_h<false>(q.ns);
}

int rti_qp_blocks_per_cu(int N, QpRows q) {
    // every limit at once (LDS per instance, the register allocation: one wave per SIMD, waves per CU), as the
    // runtime applies them
    const size_t lds = qp_lds_bytes(N, q);
    const void* fn = rti_qp_fn(q);
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess) return 0;
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, fn, 64, lds) != hipSuccess) return 0;
    return n;
}

hipError_t launch_rti_qp(const QpArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    if (a.nh < 0 || a.nh > 3 || a.nhN < 0 || a.nhN > QP_NHN || a.nsN < 0 || a.nsN > 3 || a.nsN > a.nhN ||
        a.nhN - a.nsN > 6 || a.nhs < 0 || a.nhs > a.nh)
        return hipErrorInvalidValue;
    const QpRows q{a.nh, a.nhN, a.nsN, a.nhs};
    const size_t lds = qp_lds_bytes(a.N, q);
    const void* fn = rti_qp_fn(q);
    hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    void* args[] = {(void*)&a};
    e = hipLaunchKernel(fn, dim3(a.B), dim3(64), args, lds, s);
    if (e != hipSuccess) return e;
    return hipGetLastError();
}

}  // namespace sdfn
