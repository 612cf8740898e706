// SQP-RTI feedback phase, partitioned in time: the OCP QP of every instance on one workgroup of four
// wavefronts (the same QP and IPM semantics as rti_qp.hip; oracle/qp_ipm.c lqr_seg states the scheme).
//
// rti_qp.hip walks all N + 1 nodes of an instance with one wavefront: every Newton system is a chain
// of 4 (N + 1) dependent stage steps, and at B = 1024 one wave per SIMD has nothing to hide them
// behind.  Here wavefront w owns the nodes [a_w, a_{w+1}), a_w = w (N + 1) / 4, and each Newton system
// is
//   1. backward, all four segments at once: segment 3 runs the Riccati recursion from the terminal
//      node; segments 0..2 run it from a zero cost-to-go at their end b and carry the element of their
//      conditional value function (J, eta = the recursion's own [P | p]; [Phi | beta] = the closed-loop
//      transition from a to b and its offset; C = sum_k Z_k R^_k^-1 Z_k^T, Z_k = Phi_{k+1->b} B_k) plus
//      per node G_k = R^_k^-1 Z_k^T, the gain of the costate lam_b = P_b x_b + p_b at b;
//   2. a serial coupling over the three boundaries (P_b = L L^T, S = I + L^T C L = U U^T, V = L U^-T,
//      X = V^T Phi): P_a = J + X^T X; z = V^T beta + U^-1 L^-1 p_b, p_a = eta + X^T z; and for the
//      forward pass lam_b = Lam x_a + lam0, x_b = M x_a + m with Lam = V X, lam0 = V z, M = Phi - C Lam,
//      m = beta - C lam0;
//   3. the boundary states x_a by three 10 x 10 matvecs, then every segment's forward pass at once with
//      u_k = K_k x_k + kf_k - G_k lam_b.
// One factorisation serves predictor and corrector (the corrector repeats the vector parts: backward
// with the stored factors, the p coupling, the x chain, forward).  The dependent depth of a Newton
// system drops from 4 (N + 1) stages to about 4 (N + 1) / 4 plus the couplings, and B = 1024 fills
// every SIMD with four waves.
//
// Layout: stage records (rti_qp_pack_kernel) as in rti_qp.hip; the factor record of a node holds
// [A~|b~ ; K|kf] rows of 12, chol(R^) (1/diagonal), J_{k+1} c_k, a copy of the predictor kf, Z_k (10 x 4)
// and G_k (4 x 10).  The coupling matrices of each segment (packed L, U, C; V, X, M, Lam) go to a small
// per-instance block of the workspace.  Iterate rows (t, lambda) live in registers of the lane that
// owns them (a box pair or a soft group of the wave's own nodes); node vectors in LDS.
// Cross-wave traffic is LDS only (the hand-off slots), behind raw s_barrier (no vmcnt drain: global
// memory stays wave-private).
#include <hip/hip_runtime.h>

#include "qp_dev.h"
#include "qp_kernels.h"

#include <cstdlib>

namespace sdfn {

namespace {

using namespace qpd;

constexpr int NSEG_MAX = QP_NSEG;
// factor record of the segmented kernel.  Rows of FR doubles: r < 10 [A~ row r | b~_r | Lp_r], r = 10..13
// [K row | kf | kf of the predictor]; Lp = chol(R^) packed (i0 l10 i1 l20 l21 i2 l30 l31 l32 i3, i = 1/L_ii).
// Then J_{k+1} c_k, Z (row r: Z[r][0..3]), and copies of the stage record's c, g, B (B[r][i] at +10 i + r)
// and C^T (C^T[j][r] at +10 j + r) written once per QP, so that every sweep's operands are two ranges of
// one record; then G (row i: G[i][0..9]) and junk.
constexpr int S_AB = 0, S_K = 10 * FR, S_PC = 14 * FR, S_Z = S_PC + 10, S_C = S_Z + 40, S_GV = S_C + 10, S_B = S_GV + 14,
              S_CT = S_B + 40, S_G = S_CT + 30, S_J = S_G + 40, FRECS = QP_FRECS;
static_assert(S_PC == 168 && S_B == 242 && S_G == 312 && S_J + 4 <= FRECS && (FRECS * 8) % 128 == 0 && (S_GV + NX) % 2 == 0,
              "segmented factor record");
// stream: per position WIN doubles land in one of two LDS windows of the wave by three 16-byte LDS-DMA
// wave-instructions; each lane's source granule is a per-sweep lane constant:
//   0 initial forward   R[0, 194) in place
//   1 backward factor   R[0, 320) in place (granules past the record repeat its last zero granule)
//   2, 4 forward        F[0, 168) | F[S_B, S_J) at WF_B: B at WF_B, C^T at WF_CT, G at WF_G
//   3 corrector         F[0, S_G) in place
constexpr int WIN = 384, WF_B = 168, WF_CT = WF_B + (S_CT - S_B), WF_G = WF_B + (S_G - S_B);
static_assert(WF_G + 40 <= WIN && S_G <= WIN && REC / 2 <= WIN / 2, "windows");
__device__ __forceinline__ int src_granule(int K, int wg) {  // source granule (2 doubles) of window granule wg
    if (K == 0) return wg < (R_CT + 30) / 2 ? wg : (R_CT + 30) / 2 - 1;
    if (K == 1) return wg < REC / 2 ? wg : REC / 2 - 1;
    if (K == 3) return wg < S_G / 2 ? wg : S_G / 2 - 1;
    return wg < S_PC / 2 ? wg : wg < S_PC / 2 + (S_J - S_B) / 2 ? wg - S_PC / 2 + S_B / 2 : S_J / 2 - 1;
}
// coupling block per segment w < 3 (doubles, in the workspace after the records): packed lower L, U, C
// (true diagonals), V and X (row-major 10 x 10) -- the first CP_SC doubles also live in the wave's two
// windows during a coupling -- then M and Lam (row-major), beta of the predictor; then the row state
// of the wave's lanes parked during the factor sweep
constexpr int CP_L = 0, CP_U = 56, CP_V = 112, CP_X = 212, CP_C = 312, CP_SC = 368, CP_M = 368, CP_LM = 468, CP_B = 568,
              CPL = QP_CPL;
constexpr int CP_PHI = WIN;  // [Phi | beta] tile (16 x 16) from mchain to moff, in the second window
static_assert(CP_B + 10 <= CPL && CP_SC <= WIN && CP_PHI + 256 <= 2 * WIN, "coupling block");

__device__ __forceinline__ int trl(int i, int j) { return i * (i + 1) / 2 + j; }  // packed lower, j <= i
// v[i] in the lanes with i == idx, as a chain of v_cndmask (a nested ?: of computed values compiles to a
// divergent branch tree: exec save / restore per level)
// an LDS read the source performs only where `ok` (0 elsewhere), as an unconditional read of a clamped
// index: a conditional read compiles to a divergent branch around it
__device__ __forceinline__ double ldsel(const sdfn::qpd::ldsd* base, int idx, bool ok) {
    const double v = base[ok ? idx : 0];
    return ok ? v : 0.0;
}
__device__ __forceinline__ double sel4(int i, double v0, double v1, double v2, double v3) {
    double r = v3;
    r = i == 2 ? v2 : r;
    r = i == 1 ? v1 : r;
    return i == 0 ? v0 : r;
}

// raw workgroup barrier: LDS operations drained, nothing else (global memory is wave-private here)
__device__ __forceinline__ void wg_sync() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// 1/sqrt(v), v > 0: hardware estimate + two Newton steps (the coupling's Cholesky factors)
__device__ __forceinline__ double rsqrt2(double v) {
    double y = __builtin_amdgcn_rsq(v);
    const double h = 0.5 * v;
    y = y * fma(-h * y, y, 1.5);
    return y * fma(-h * y, y, 1.5);
}

// In-register Cholesky, one column per lane: lane c < 10 holds column c of an SPD 10 x 10 matrix in
// col[0..9]; on return column c of L (col[i] = L[i][c], 0 above the diagonal) and inv[j] = 1 / L[j][j]
// (uniform).  Lanes >= 10 compute garbage that is never read.
// The elimination runs on the unscaled columns (the Schur complements A'); lane c scales its column by
// 1 / L[c][c] once at the end, and the rank-1 update is masked through its multiplier (0 in lanes <= j:
// fma(-a, 0, x) = x exactly), so a pivot costs its broadcasts, its 1/sqrt and one fma per row instead of
// a branch, ten multiplies and two selects per row -- the same operations on the same values as the
// column-at-a-time form, so the same bits.
__device__ __forceinline__ void chol_cols(double (&col)[NX], double (&inv)[NX], int lane) {
    double myinv = 0.0;
#pragma unroll
    for (int j = 0; j < NX; ++j) {
        const double d = rdlane(col[j], j);
        const double iv = rsqrt_nr(d);
        inv[j] = iv;
        myinv = lane == j ? iv : myinv;
        // A'[i][c] -= A'[i][j] A'[c][j] / d for c > j, i > j  (A' symmetric: A'[c][j] = col[j] in lane c)
        const double tcj = lane > j ? col[j] * (iv * iv) : 0.0;
#pragma unroll
        for (int i = j + 1; i < NX; ++i) col[i] = fma(-rdlane(col[i], j), tcj, col[i]);
    }
    // L[i][c] = A'[i][c] / L[c][c] for i >= c
#pragma unroll
    for (int i = 0; i < NX; ++i) col[i] = i < lane ? 0.0 : col[i] * myinv;
}

// constant table (s.cst): box bounds, then per row kind ci (0..2 stage rows j, 3 + j terminal rows j) its
// lower / upper bound and L1 / L2 slack weights
constexpr int C_LO = 8, C_HI = C_LO + 3 + QP_NHN, C_ZL = C_HI + 3 + QP_NHN, C_ZU = C_ZL + 3 + QP_NHN, C_N = C_ZU + 3 + QP_NHN;
struct SegSmem {
    ldsd *dxc, *dua, *duc, *cxa, *cxc, *fw, *fg, *bd, *bv, *skv, *cst, *ctn, *zero;
    ldsd *win, *junk, *xlam, *vec;  // this wave's
    ldsd *slot, *red;               // hand-off slots [3][112], reduction partials
};

// LDS layout for horizons N <= NMAX, at compile-time offsets (every LDS address an immediate: no base
// registers); per-node arrays sized for NMAX
template <int NSEG, int NMAX>
struct SegLds {
    static constexpr int ev(int n) { return (n + 1) & ~1; }
    static constexpr int N1 = NMAX + 1;
    static constexpr int NG = NMAX * NS + QP_NHN;  // groups: k NS + j at stages k < N, N NS + j the terminal rows
    static constexpr int DXC = 0, DUA = DXC + ev(N1 * NX), DUC = DUA + ev(NMAX * NU), CXA = DUC + ev(NMAX * NU),
                         CXC = CXA + ev(NG), FW = CXC + ev(NG), FG = FW + ev(NG), BD = FG + ev(NG),
                         BV = BD + ev(NMAX * NU), SKV = BV + ev(NMAX * NU), CST = SKV + ev(N1), CTN = CST + ev(C_N),
                         ZERO = CTN + 10 * QP_NHN, WINS = ZERO + 48,
                         JUNK = WINS + NSEG * 2 * WIN, XLAM = JUNK + NSEG * 2, VEC = XLAM + NSEG * 16, SLOT = VEC + NSEG * 64,
                         RED = SLOT + (NSEG_MAX - 1) * 112, TOTAL = RED + 64;
};

template <int NSEG, int NMAX>
__device__ __forceinline__ SegSmem seg_carve(ldsd* q, int w) {
    using L = SegLds<NSEG, NMAX>;
    SegSmem s;
    s.dxc = q + L::DXC; s.dua = q + L::DUA; s.duc = q + L::DUC; s.cxa = q + L::CXA; s.cxc = q + L::CXC;
    s.fw = q + L::FW; s.fg = q + L::FG; s.bd = q + L::BD; s.bv = q + L::BV; s.skv = q + L::SKV;
    s.cst = q + L::CST; s.ctn = q + L::CTN; s.zero = q + L::ZERO; s.slot = q + L::SLOT; s.red = q + L::RED;
    s.win = q + L::WINS + w * 2 * WIN;
    s.junk = q + L::JUNK + 2 * w;
    s.xlam = q + L::XLAM + 16 * w;
    s.vec = q + L::VEC + 64 * w;
    return s;
}
// vec area of a wave: invL 0, invU 10, beta 20, z 30, lam0 40, m 50
constexpr int V_IL = 0, V_IU = 10, V_B = 20, V_Z = 30, V_L0 = 40, V_M = 50;

// Lane constants of the factor stage: window indices (R_Z: a zero slot) and record-store byte offsets
// (S_J: junk), two 16-bit fields per register, built once per factor sweep behind opaque() so they stay
// packed in 13 registers instead of being rematerialised at every stage.
constexpr int SJB = 8 * S_J;
struct FConst {
    unsigned p[13];
};
__device__ __forceinline__ int lo16(unsigned v) { return (int)(v & 0xffffu); }
__device__ __forceinline__ int hi16(unsigned v) { return (int)(v >> 16); }
enum { F_OG01, F_OG2, F_CGI, F_AB01, F_AB2, F_BMI, F_HXU, F_HUU, F_V0, F_H0, F_H1, F_H2, F_H3, F_BQ0, F_BQ1, F_BQ2,
       F_SPC0, F_SPC1, F_SPC2, F_SAB0, F_SAB1, F_SAB2, F_SK, F_SZ, F_SG, F_SKP, F_NFIELD };
__device__ __forceinline__ int fget(const FConst& f, int i) { return (i & 1) ? hi16(f.p[i >> 1]) : lo16(f.p[i >> 1]); }

__device__ __forceinline__ FConst fconst(int lane) {
    int v[F_NFIELD];
    const int g = lane >> 4, c = lane & 15;
    v[F_OG01] = c < 15 ? c * 10 + g : R_Z;
    v[F_OG2] = (c < 15 && g < 2) ? c * 10 + g + 8 : R_Z;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int a = g + 4 * r, lo = a < c ? a : c, hi = a < c ? c : a;
        v[F_H0 + r] = (a < 14 && c < 14) ? R_H + tri14(lo, hi) : (a < 14 && c == 14) ? R_G + a : R_Z;
    }
    v[F_CGI] = (c < NX && g < NS) ? R_CT + g * 10 + c : R_Z;
    const bool xcol = c < NX || c == 14;
    const int xo = c < NX ? c : 10;
    v[F_AB01] = xcol ? (c < NX ? c : 14) * 10 + g : R_Z;
    v[F_AB2] = (xcol && g < 2) ? (c < NX ? c : 14) * 10 + g + 8 : R_Z;
    v[F_BMI] = c < NX ? (NX + g) * 10 + c : R_Z;
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const int a = g + 4 * r;
        v[F_SPC0 + r] = (c == 14 && a < NX) ? 8 * (S_PC + a) : SJB;
        v[F_SAB0 + r] = (xcol && a < NX) ? 8 * (S_AB + a * FR + xo) : SJB;
    }
    v[F_SK] = xcol ? 8 * (S_K + g * FR + xo) : SJB;
    v[F_SZ] = c < NX ? 8 * (S_Z + 4 * c + g) : SJB;
    v[F_SG] = c < NX ? 8 * (S_G + 10 * g + c) : SJB;
    v[F_SKP] = c == 14 ? 8 * (S_K + g * FR + 11) : SJB;
    v[F_HXU] = c < NX ? R_H + tri14(c, NX + g) : R_Z;
    const int c3 = c & 3;
    v[F_HUU] = R_H + tri14(NX + (c3 < g ? c3 : g), NX + (c3 < g ? g : c3));
#pragma unroll
    for (int st = 0; st < 3; ++st) v[F_BQ0 + st] = 4 * st + g < NX ? (NX + c3) * 10 + 4 * st + g : R_Z;
    v[F_V0] = c < 14 ? R_H + tri14(c < NX + g ? c : NX + g, c < NX + g ? NX + g : c) : c == 14 ? R_G + NX + g : R_Z;
    FConst f;
#pragma unroll
    for (int i = 0; i < 13; ++i)
        f.p[i] = (unsigned)opaque((int)((unsigned)v[2 * i] | ((unsigned)(2 * i + 1 < F_NFIELD ? v[2 * i + 1] : 0) << 16)));
    return f;
}
static_assert(F_NFIELD <= 26 && 8 * FRECS < 65536, "packed lane constants");

}  // namespace

#ifdef SEG_STAMPS  // diagnostic build only: per-wave, per-phase cycle accounting into A.stamps [B][4][24]
#define SSTAMP_DECL long long st_t0 = clock64(), st_acc[24] = {}; int st_ph = 0;
#define SSTAMP_PHASE(i) st_ph = (i)
#define SSTAMP(i) do { const long long t1_ = clock64(); st_acc[i] += t1_ - st_t0; st_t0 = t1_; } while (0)
#define SSTAMP_ARRIVE(body) do { SSTAMP(st_ph); body; SSTAMP(15); } while (0)
#define SSTAMP_OUT if (lane == 0 && A.stamps) for (int i_ = 0; i_ < 24; ++i_) A.stamps[((size_t)b * NSEG_MAX + w) * 24 + i_] = (double)st_acc[i_];
#else
#define SSTAMP_DECL
#define SSTAMP_PHASE(i)
#define SSTAMP(i)
#define SSTAMP_ARRIVE(body) body
#define SSTAMP_OUT
#endif

template <int NSEG, int NMAX>
// occupancy targets: three or two (P = 2, 3) workgroups per CU; P = 4 at two (256 registers per lane: no
// spill at 223 VGPRs; the 128-register target of four per CU spilled, and without a target the compiler
// took 265 registers -- one workgroup per CU, half the instances of a B = 512 batch per round)
__global__ __launch_bounds__(64 * NSEG, NSEG == 4 ? 2 : NSEG) void rti_qp_seg_kernel(QpArgs A) {
    __shared__ __align__(16) double lds_q[SegLds<NSEG, NMAX>::TOTAL];
    SSTAMP_DECL
    const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63;
    // Stage code re-derives its lane index behind opaque() (`const int lane = opaque(lane_k)`): the lane
    // predicates are then recomputed per stage (a few VALU ops) instead of being hoisted to the prologue,
    // where each one held a 64-bit SGPR mask for the whole kernel and the masks spilled to VGPR lanes.
    const int lane_k = lane;
    const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
    // the row set (rti_qp.hip's, QpRows): nh (0..3) stage rows at nodes k < N, group j of a node reading column
    // h_col[j] of h / J_h, the last nhs of them hard (none at node 0); nhN terminal rows, the first nsN soft,
    // row j reading h[N][hN_col[j]] + hE[hE_col[j]]
    const int nh = A.nh, nss = nh - A.nhs;
    const int N = A.N, N1 = N + 1,
              m = 8 * N + 4 * (nss * N + A.nsN) + 2 * ((N - 1) * A.nhs + A.nhN - A.nsN);
    const SegSmem s = seg_carve<NSEG, NMAX>((ldsd*)lds_q, w);
    ldsd* const win = s.win;                                  // two windows; the coupling's scratch
    const int sa = w * N1 / NSEG, sb = (w + 1) * N1 / NSEG;  // this wave's nodes [sa, sb)
#ifdef SEGX_NO_AUG
    const bool aug = false;
#else
    const bool aug = w < NSEG - 1;                            // segments with a coupling (not the terminal one)
#endif
    double* const Rw = A.work + (size_t)b * qp_work_doubles(N);
    const double* R = Rw;
    double* F = Rw + (size_t)N1 * REC;
    double* CP = Rw + (size_t)N1 * (REC + FRECS) + (size_t)(w < NSEG - 1 ? w : 0) * CPL;
    double* PK = Rw + (size_t)N1 * (REC + FRECS) + (NSEG_MAX - 1) * (size_t)CPL + (size_t)w * QP_PARK;  // parked row state
    const __amdgpu_buffer_rsrc_t rsF = __builtin_amdgcn_make_buffer_rsrc(F, (short)0, N1 * FRECS * 8, 0x00020000);

    // ------------------------------------------------------------ constants, static record copies
    for (int e = tid; e < N1; e += 64 * NSEG) s.skv[e] = (A.cost_scaling && e < N) ? A.dt[e] : 1.0;
    if (tid < C_N) {  // constant indices: scalar loads of the kernel arguments
        double v = 0.0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (tid == i) v = A.lbu[i];
            if (tid == 4 + i) v = A.ubu[i];
        }
#pragma unroll
        for (int j = 0; j < 3; ++j) {
            if (tid == C_LO + j) v = A.lh[j];
            if (tid == C_HI + j) v = A.uh[j];
            if (tid == C_ZL + j) v = A.zl[j];
            if (tid == C_ZU + j) v = A.Zl[j];
        }
#pragma unroll
        for (int j = 0; j < QP_NHN; ++j) {
            if (tid == C_LO + 3 + j) v = A.lhN[j];
            if (tid == C_HI + 3 + j) v = A.uhN[j];
            if (tid == C_ZL + 3 + j) v = j < 3 ? A.zlN[j < 3 ? j : 0] : 0.0;
            if (tid == C_ZU + 3 + j) v = j < 3 ? A.ZlN[j < 3 ? j : 0] : 0.0;
        }
        s.cst[tid] = v;
    }
    // terminal rows j < nhN: C row j = J_h[N] column hN_col[j] + J_hE column hE_col[j] (rti_qp.hip's); rows
    // nhN .. QP_NHN - 1 zero, so the terminal stages run over all QP_NHN rows without a count (their folds
    // stay zero: no lane owns them)
    if (tid < 10 * QP_NHN) {
        const int e = tid, j = e / 10, l = e - 10 * j;
        const double* jr = A.Jh + ((size_t)b * N1 + N) * 30 + l * 3;
        const double j0 = jr[0], j1 = jr[1], j2 = jr[2];  // in flight while the columns are looked up
        int c1 = -1, c2 = -1;
#pragma unroll
        for (int q = 0; q < QP_NHN; ++q)
            if (q == j) { c1 = A.hN_col[q]; c2 = A.hE_col[q]; }
        double cv = 0.0;
        if (j < A.nhN) {
            if (c1 >= 0) cv += c1 == 0 ? j0 : c1 == 1 ? j1 : j2;
            if (c2 >= 0) cv += A.JhE[((size_t)b * 10 + l) * 6 + c2];  // rec_feas / stability rows only
        }
        s.ctn[e] = cv;
    }
    if (tid < 48) s.zero[tid] = 0.0;
    // folds of every group: the groups past nh keep (0, 0) (their C^T rows are zero rows of the record)
    for (int e = tid; e < N * NS + QP_NHN; e += 64 * NSEG) {
        s.fw[e] = 0.0;
        s.fg[e] = 0.0;
    }
    if (A.sdf_row_patch) {  // records packed beside the SDF kernel (pack_part 1): their sdf row of C^T
        for (int e = lane; e < (sb - sa) * NX; e += 64) {
            const int k = sa + e / NX, l = e % NX;
            Rw[(size_t)k * REC + R_CT + 10 * A.sdf_row + l] = A.Jh[((size_t)b * N1 + k) * 30 + l * 3 + 2];
        }
    }
    // [c | g | B | C^T] of the stage record into the factor record (R[100, 194) is [B | c | g | C^T])
    for (int e = lane; e < (sb - sa) * 94; e += 64) {
        const int k = sa + e / 94, q = e % 94;
        const int src = q < 10 ? R_C + q : q < 24 ? R_G + q - 10 : q < 64 ? 100 + q - 24 : R_CT + q - 64;
        F[(size_t)k * FRECS + S_C + q] = R[(size_t)k * REC + src];
    }
    // lane-owned rows: box pair (kb, ib) (rows 8 kb + ib, 8 kb + 4 + ib) of this wave's nodes; group (ks, js)
    // of a stage node (lanes 0..47: at most 15 stage nodes x 3), soft (its four rows in ts / ls) or hard
    // (lower, upper in ts[0..1] / ls[0..1]); in the last wave lanes 48 + j the terminal row j, soft or hard
    const bool last = w == NSEG - 1;
    const int jt = lane - 48;
    const bool tlane = last && jt >= 0 && jt < QP_NHN;
    const int kb = sa + (lane >> 2), ib = lane & 3, ks = tlane ? N : sa + lane / 3, js = tlane ? jt : lane % 3;
    const bool ownb = kb < (sb < N ? sb : N);
    const bool stg = !tlane && ks < (last ? N : sb) && js < nh;
    const bool owns = tlane ? jt < A.nsN : stg && js < nss;
    const bool ownh = tlane ? jt >= A.nsN && jt < A.nhN : stg && js >= nss && ks > 0;
    const int ci = tlane ? 3 + jt : js;  // the row kind in the constant table
    const int kbc = ownb ? kb : sa, ksc = (owns || ownh) ? ks : sa;
    const double ubv = ownb ? A.u[((size_t)b * N + kbc) * NU + ib] : 0.0;
    double hsv = 0.0;
    if (owns || ownh) {
        if (tlane) {
            int c1 = -1, c2 = -1;
#pragma unroll
            for (int q = 0; q < QP_NHN; ++q)
                if (q == jt) { c1 = A.hN_col[q]; c2 = A.hE_col[q]; }
            if (c1 >= 0) hsv += A.h[((size_t)b * N1 + N) * NS + c1];
            if (c2 >= 0) hsv += A.hE[(size_t)b * 6 + c2];
        } else {
            int hc = 0;
#pragma unroll
            for (int q = 0; q < 3; ++q)
                if (q == js) hc = A.h_col[q];
            hsv = A.h[((size_t)b * N1 + ksc) * NS + hc];
        }
    }
    if (tid < NX) s.dxc[tid] = A.x0[(size_t)b * 10 + tid] - A.x[(size_t)b * N1 * 10 + tid];
    // du of the start iterate into dua (free until the first forward sweep): 0, or on a primal warm start
    // the previous QP's du as found in A.du (qp_solver_warm_start, ocp.py:116)
    // (a du with a non-finite entry, a failed QP's output, gives a cold start: the failure does not stick)
    int nonfin = 0;
    for (int e = tid; e < N * NU; e += 64 * NSEG) {
        const double v = A.warm_start ? A.du[(size_t)b * N * NU + e] : 0.0;
        nonfin |= !__builtin_isfinite(v);
        s.dua[e] = v;
    }
    if (__syncthreads_or(nonfin))
        for (int e = tid; e < N * NU; e += 64 * NSEG) s.dua[e] = 0.0;
    wg_sync();
    // row constants: box rows at du = 0 (dlo, dup), soft rows at C dx = 0 (hl0, hu0), slack weights
    auto dlo = [&]() { return ubv - s.cst[ib]; };
    auto dup = [&]() { return s.cst[4 + ib] - ubv; };
    auto hl0 = [&]() { return hsv - s.cst[C_LO + ci]; };
    auto hu0 = [&]() { return s.cst[C_HI + ci] - hsv; };
    auto Zs = [&]() { return s.skv[ksc] * s.cst[C_ZU + ci]; };
    auto zs = [&]() { return s.skv[ksc] * s.cst[C_ZL + ci]; };
    double tb0 = 1.0, tb1 = 1.0, lb0 = 0.0, lb1 = 0.0;  // box rows (lower, upper); unowned: t = 1, lambda = 0
    double ts[4] = {1.0, 1.0, 1.0, 1.0}, ls[4] = {0.0, 0.0, 0.0, 0.0};
    // the row state parks in memory while the factor sweep and its coupling need the registers
    auto park = [&]() {
        const double v[12] = {tb0, tb1, lb0, lb1, ts[0], ts[1], ts[2], ts[3], ls[0], ls[1], ls[2], ls[3]};
#pragma unroll
        for (int j = 0; j < 12; ++j) PK[64 * j + lane] = v[j];
        asm volatile("" ::: "memory");
    };
    auto unpark = [&]() {
        asm volatile("" ::: "memory");
        double v[12];
#pragma unroll
        for (int j = 0; j < 12; ++j) v[j] = PK[64 * j + lane];
        tb0 = v[0]; tb1 = v[1]; lb0 = v[2]; lb1 = v[3];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            ts[q] = v[4 + q];
            ls[q] = v[8 + q];
        }
    };

    // ------------------------------------------------------------ workgroup reductions (fixed order)
    int rslot = 0;
    auto wg_red = [&](double v, auto op) -> double {  // v: this wave's (uniform) partial
        ldsd* r = s.red + 8 * (rslot & 7);
        ++rslot;
        if (lane == 0) r[w] = v;
        wg_sync();
        double t = r[0];
#pragma unroll
        for (int i = 1; i < NSEG; ++i) t = op(t, r[i]);
        return t;
    };
    auto opsum = [](double a_, double c_) { return a_ + c_; };
    auto opmax = [](double a_, double c_) { return fmax(a_, c_); };
    auto opmin = [](double a_, double c_) { return fmin(a_, c_); };

    // ------------------------------------------------------------ record stream (LDS-DMA, two windows)
    // A stage issues its global stores before its refill and nothing to global memory after it, so when
    // a stage starts, the only VMEM operations that may be newer than its window's DMA are the three of
    // the latest refill: s_waitcnt vmcnt(3) retires its window (VMEM operations of a wave complete in
    // order).  The compiler does not track LDS-DMA -> ds_read dependencies; these waits are the ordering.
    typedef __attribute__((address_space(3))) void ldsv;
    auto issue = [&](auto KIc, ldsd* dst, int k, const int* sg) {
        constexpr int KI = decltype(KIc)::value;
        const double* base = (KI == 0 || KI == 1) ? R + (size_t)k * REC : F + (size_t)k * FRECS;
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the window's previous reads are done
        __builtin_amdgcn_global_load_lds((const void*)(base + 2 * sg[0]), (ldsv*)dst, 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)(base + 2 * sg[1]), (ldsv*)(dst + 128), 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const void*)(base + 2 * sg[2]), (ldsv*)(dst + 256), 16, 0, 0);
        asm volatile("" ::: "memory");
    };
    auto arrived = [&]() { asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); };
    auto drained = [&]() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };
    // one sweep over n positions, node(q) the node of position q, positions alternating between the
    // two windows; a stage calls refill() after its last window read, which issues position q + 2 into
    // the window it has just read (lead: the rest of that stage plus the next one).  The loop body is
    // straight-line (refills past the end reload the last node), so the compiler counts the VMEM
    // operations in flight exactly and waits only for the token of the window a stage reads.
    auto sweep = [&](auto Kc, int n, auto node, auto stage) {
        constexpr int K = decltype(Kc)::value;
        int sg[3];
#pragma unroll
        for (int j = 0; j < 3; ++j) sg[j] = opaque(src_granule(K, 64 * j + lane));
        ldsd* const w0 = win;
        ldsd* const w1 = win + WIN;
        auto nd = [&](int q) { return node(q < n ? q : n - 1); };
        issue(Kc, w0, nd(0), sg);
        issue(Kc, w1, nd(1), sg);
        int q = 0;
        for (; q + 1 < n; q += 2) {
            SSTAMP_ARRIVE(arrived());
            stage(q, node(q), w0, [&]() { issue(Kc, w0, nd(q + 2), sg); });
            SSTAMP_ARRIVE(arrived());
            stage(q + 1, node(q + 1), w1, [&]() { issue(Kc, w1, nd(q + 3), sg); });
        }
        if (q < n) {
            SSTAMP_ARRIVE(arrived());
            stage(q, node(q), w0, [&]() {});
        }
        drained();
    };

    // ------------------------------------------------------------ forward stage
    // lane r < 10: x_{k+1}[r]; 10..13: u_k; 14..16: (C x_k)_{r-14}.  K == 0: the initial iterate
    // (rows of A x + c from the stage record).  LAM: the costate term -[B G; G] lam_b of segments 0..2.
    // TERM: the terminal node (its rows' C from ctn, lanes 14 .. 13 + QP_NHN), a separate instantiation so the
    // other stages keep their lane constants
    auto fw_stage = [&](auto Kc, auto LAMc, auto TERMc, int k, bool seg_end, const ldsd* cw, auto refill) {
        const int lane = opaque(lane_k);
        constexpr int K = decltype(Kc)::value;
        constexpr bool LAM = decltype(LAMc)::value;
        constexpr bool term = decltype(TERMc)::value;
        const bool fx = lane < NX, fu = lane >= NX && lane < 14, fc = lane >= 14 && lane < (term ? 14 + QP_NHN : 14 + NS);
        const int fcj = fc ? lane - 14 : 0;
        ldsd* const duo = K == 4 ? s.duc : s.dua;
        ldsd* const cxo = K == 4 ? s.cxc : s.cxa;
        double row[NX], off;
        if constexpr (K == 0) {
            const ldsd* rp = fx ? cw + R_AB + lane : fc ? (term ? s.ctn : cw + R_CT) + fcj * 10 : s.zero;
            const int str = fx ? 10 : 1;
#pragma unroll
            for (int l = 0; l < NX; ++l) row[l] = rp[l * str];
            off = *(fx ? cw + R_C + lane : s.zero);
            // + B du_k of the start iterate (dua; 0 on a cold start): B[r][j] at R_AB + 10 (NX + j) + r
            const int bx = fx ? lane : 0, ku = k < N ? k : N - 1;
            const double bdu = cw[R_AB + 100 + bx] * s.dua[ku * NU] + cw[R_AB + 110 + bx] * s.dua[ku * NU + 1] +
                               cw[R_AB + 120 + bx] * s.dua[ku * NU + 2] + cw[R_AB + 130 + bx] * s.dua[ku * NU + 3];
            off += (fx ? 1.0 : 0.0) * bdu;
        } else {
            const ldsd2* rp = (const ldsd2*)(lane < 14 ? cw + lane * FR : fc ? (term ? s.ctn : cw + WF_CT) + fcj * 10 : s.zero);
#pragma unroll
            for (int l = 0; l < NX / 2; ++l) {
                const d2 v = rp[l];
                row[2 * l] = v.x;
                row[2 * l + 1] = v.y;
            }
            off = *(lane < 14 ? cw + lane * FR + 10 : s.zero);
            if constexpr (LAM) {  // d = G lam_b (lanes 10..13), off -= [B d ; d]
                const ldsd2* gp = (const ldsd2*)(fu ? cw + WF_G + 10 * (lane - NX) : s.zero);
                const ldsd2* lp = (const ldsd2*)s.xlam;
                double dv = 0.0;
#pragma unroll
                for (int l = 0; l < NX / 2; ++l) {
                    const d2 gv = gp[l], lv = lp[l];
                    dv = fma(gv.x, lv.x, dv);
                    dv = fma(gv.y, lv.y, dv);
                }
                const double d0 = rdlane(dv, 10), d1 = rdlane(dv, 11), d2_ = rdlane(dv, 12), d3 = rdlane(dv, 13);
                const int bx = fx ? lane : 0;
                const double bdv = cw[WF_B + bx] * d0 + cw[WF_B + 10 + bx] * d1 + cw[WF_B + 20 + bx] * d2_ + cw[WF_B + 30 + bx] * d3;
                off -= (fx ? 1.0 : 0.0) * bdv + (fu ? 1.0 : 0.0) * dv;  // bdv used by every lane: its reads stay unconditional
            }
        }
        // x_k (the chain's LDS hand-off) is read before the refill, so the refill's lgkmcnt(0) covers it
        // together with the window reads: one LDS round trip on the chain instead of two
        const ldsd2* xp = (const ldsd2*)(s.dxc + k * NX);
        d2 xv[NX / 2];
#pragma unroll
        for (int l = 0; l < NX / 2; ++l) xv[l] = xp[l];
        refill();
        double a0 = off, a1 = 0.0;
#pragma unroll
        for (int l = 0; l < NX / 2; ++l) {
            a0 = fma(row[2 * l], xv[l].x, a0);
            a1 = fma(row[2 * l + 1], xv[l].y, a1);
        }
        const double z = a0 + a1;
        ldsd* dst = fc ? cxo + k * NS + fcj
                  : (k < N && fx && !seg_end) ? s.dxc + (k + 1) * NX + lane
                  : (K != 0 && k < N && fu) ? duo + k * NU + lane - NX : s.junk;
        *dst = z;
    };

    // ------------------------------------------------------------ backward stage, factor
#define FBST(v, off) bst(v, rsF, (unsigned)(off), sko)
    d4 Pa = {0.0, 0.0, 0.0, 0.0};   // [P | p] of the node ahead (segments 0..2: J | eta), accumulator layout
    d4 Psi = {0.0, 0.0, 0.0, 0.0};  // [Phi | beta]^T (rows 0..9: Phi^T, row 14: beta), segments 0..2
    d4 Cg = {0.0, 0.0, 0.0, 0.0};   // C, segments 0..2
    auto bf_stage = [&](auto Fc, auto AUGc, int k, const FConst& f, const ldsd* cw, auto refill) {
        const int lane = opaque(lane_k);
        constexpr bool FIRST = decltype(Fc)::value;  // the terminal node
        constexpr bool AUG = decltype(AUGc)::value;
        const int g = lane >> 4, c = lane & 15;
        const double m14 = c == 14 ? 1.0 : 0.0, mg3 = g < NS ? 1.0 : 0.0;
        const int gj = g < NS ? g : 0;
        const double cg = cw[fget(f, F_CGI)];
        const double fb = mg3 * fma(s.fw[k * NS + gj], cg, m14 * s.fg[k * NS + gj]);
        if constexpr (FIRST) {  // [P_N | p_N] = [H_N | g_N] + the folds of the nhN terminal rows (C rows in ctn)
            d4 T;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int a_ = g + 4 * r, lo = a_ < c ? a_ : c, hi = a_ < c ? c : a_;
                T[r] = cw[(a_ < NX && c < NX) ? R_H + tri10(lo, hi) : (a_ < NX && c == 14) ? R_G + a_ : R_Z];
            }
            // rows j = g and g + 4 (rows past nhN are zero rows with zero folds): lane (g, c) holds C[j][c] and
            // w_j C[j][c] + [c = 14] gamma_j
            auto tfold = [&](int j, d4 acc) {
                const double ct = ldsel(s.ctn, 10 * j + (c < NX ? c : 0), c < NX);
                return mfma(ct, fma(s.fw[N * NS + j], ct, m14 * s.fg[N * NS + j]), acc);
            };
            Pa = tfold(g, T);
            Pa = tfold(g + 4, Pa);
            refill();
            return;
        }
        const unsigned sko = (unsigned)k * (FRECS * 8u);
        // ---- region 1: W = P G (K = 10), rows 10..13 of M' = [H_u | g_u] + box terms + B^T W, B^T P, Z^T
        const int og01 = fget(f, F_OG01);
        const double og0 = cw[og01], og1 = cw[og01 + 4], og2v = cw[fget(f, F_OG2)];
        const double bq0 = cw[fget(f, F_BQ0)], bq1 = cw[fget(f, F_BQ1)], bq2 = cw[fget(f, F_BQ2)];
        // box folds: unconditional LDS reads scaled by 0 / 1 lane masks (a conditional read is a divergent
        // branch: exec save / restore around it, ten of them per stage before)
        const double bdg = s.bd[k * NU + g], bvg = s.bv[k * NU + g];
        const double hv0 = cw[fget(f, F_V0)] + (c == NX + g ? 1.0 : 0.0) * bdg + (c == 14 ? 1.0 : 0.0) * bvg;
        d4 W = {0.0, 0.0, 0.0, 0.0};
        W = mfma(Pa[0], og0, W);
        W = mfma(Pa[1], og1, W);
        W = mfma(Pa[2], og2v, W);
        FBST(W[0], fget(f, F_SPC0));
        FBST(W[1], fget(f, F_SPC1));
        FBST(W[2], fget(f, F_SPC2));
#pragma unroll
        for (int r = 0; r < 3; ++r) W[r] = fma(m14, Pa[r], W[r]);
        double Mu = mfma4(bq0, W[0], hv0);
        Mu = mfma4(bq1, W[1], Mu);
        Mu = mfma4(bq2, W[2], Mu);
        double Ub = mfma4(bq0, Pa[0], 0.0);
        Ub = mfma4(bq1, Pa[1], Ub);
        Ub = mfma4(bq2, Pa[2], Ub);
        double zt = 0.0;
        if constexpr (AUG) {  // Z^T = B^T Psi: lane (g, c) holds Z[c][g] = (Phi B)[c][g]
            zt = mfma4(bq0, Psi[0], 0.0);
            zt = mfma4(bq1, Psi[1], zt);
            zt = mfma4(bq2, Psi[2], zt);
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- region 2: L = chol(R^), [K | k_ff] = -L^-T L^-1 [S | m_u]; segments 0..2: G, C += Zh Zh^T
        double kg;
        {
            const double r00 = rdlane(Mu, 10), r10 = rdlane(Mu, 26), r20 = rdlane(Mu, 42), r30 = rdlane(Mu, 58);
            const double r11 = rdlane(Mu, 27), r21 = rdlane(Mu, 43), r31 = rdlane(Mu, 59);
            const double r22 = rdlane(Mu, 44), r32 = rdlane(Mu, 60), r33 = rdlane(Mu, 61);
            const double s0 = __shfl(Mu, c), s1 = __shfl(Mu, 16 + c), s2 = __shfl(Mu, 32 + c), s3 = __shfl(Mu, 48 + c);
            const double i0 = rsqrt_nr(r00);
            const double l10 = r10 * i0, l20 = r20 * i0, l30 = r30 * i0;
            const double i1 = rsqrt_nr(r11 - l10 * l10);
            const double l21 = (r21 - l20 * l10) * i1, l31 = (r31 - l30 * l10) * i1;
            const double i2 = rsqrt_nr(r22 - l20 * l20 - l21 * l21);
            const double l32 = (r32 - l30 * l20 - l31 * l21) * i2;
            const double i3 = rsqrt_nr(r33 - l30 * l30 - l31 * l31 - l32 * l32);
            const double y0 = s0 * i0;
            const double y1 = (s1 - l10 * y0) * i1;
            const double y2 = (s2 - l20 * y0 - l21 * y1) * i2;
            const double y3 = (s3 - l30 * y0 - l31 * y1 - l32 * y2) * i3;
            const double k3 = -y3 * i3;
            const double k2 = (-y2 - l32 * k3) * i2;
            const double k1 = (-y1 - l21 * k2 - l31 * k3) * i1;
            const double k0 = (-y0 - l10 * k1 - l20 * k2 - l30 * k3) * i0;
            kg = sel4(g, k0, k1, k2, k3);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (AUG) {
                const double z0 = __shfl(zt, c), z1 = __shfl(zt, 16 + c), z2 = __shfl(zt, 32 + c), z3 = __shfl(zt, 48 + c);
                // Zh^T = L^-1 Z^T (column c), G = L^-T Zh^T = R^-1 Z^T
                const double h0 = z0 * i0;
                const double h1 = (z1 - l10 * h0) * i1;
                const double h2 = (z2 - l20 * h0 - l21 * h1) * i2;
                const double h3 = (z3 - l30 * h0 - l31 * h1 - l32 * h2) * i3;
                const double g3 = h3 * i3;
                const double g2 = (h2 - l32 * g3) * i2;
                const double g1 = (h1 - l21 * g2 - l31 * g3) * i1;
                const double g0 = (h0 - l10 * g1 - l20 * g2 - l30 * g3) * i0;
                const double zsel = sel4(g, h0, h1, h2, h3);
                const double gsel = sel4(g, g0, g1, g2, g3);
                Cg = mfma(zsel, zsel, Cg);  // C += Zh Zh^T
                FBST(zt, fget(f, F_SZ));
                FBST(gsel, fget(f, F_SG));
                FBST(kg, fget(f, F_SKP));
            }
            // chol(R^) packed into column 11 of rows 0..9: i0 l10 i1 l20 l21 i2 l30 l31 l32 i3
            double lv = i3;  // selects, not a branch tree
            lv = lane == 8 ? l32 : lv;
            lv = lane == 7 ? l31 : lv;
            lv = lane == 6 ? l30 : lv;
            lv = lane == 5 ? i2 : lv;
            lv = lane == 4 ? l21 : lv;
            lv = lane == 3 ? l20 : lv;
            lv = lane == 2 ? i1 : lv;
            lv = lane == 1 ? l10 : lv;
            lv = lane == 0 ? i0 : lv;
            FBST(lv, lane < NX ? 8 * (lane * FR + 11) : SJB);
            FBST(kg, fget(f, F_SK));
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- region 3: Joseph form [P | p] <- T^T H^ T + A~^T [P A~ | P b~ + p], T = [I 0; K k_ff; 0 1],
        // with [P A~ | P b~ + p] = [P A | P c + p] + (P B) [K | k_ff]
        const double hua = cw[fget(f, F_HUU)] + ((c & 3) == g ? 1.0 : 0.0) * bdg;
        const double V = mfma4(hua, kg, hv0);  // rows 10..13 of H^ T
        const int ab01 = fget(f, F_AB01);
        d4 Ab;
        Ab[0] = cw[ab01];
        Ab[1] = cw[ab01 + 4];
        Ab[2] = cw[fget(f, F_AB2)];
        Ab[3] = 0.0;
        const double bm = cw[fget(f, F_BMI)];
        d4 Hh;
#pragma unroll
        for (int r = 0; r < 4; ++r) Hh[r] = cw[fget(f, F_H0 + r)];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int a_ = g + 4 * (2 + h);
            const bool in = a_ >= NX && a_ < 14;
            const int bi = in ? a_ - NX : 0;
            Hh[2 + h] += (in && c == a_ ? 1.0 : 0.0) * s.bd[k * NU + bi] + (in && c == 14 ? 1.0 : 0.0) * s.bv[k * NU + bi];
        }
        const double hxa = cw[fget(f, F_HXU)];
        Ab = mfma(bm, kg, Ab);                  // [A~ | b~] = [A | c] + B [K | k_ff]
        FBST(Ab[0], fget(f, F_SAB0));
        FBST(Ab[1], fget(f, F_SAB1));
        FBST(Ab[2], fget(f, F_SAB2));
        refill();                               // after the stage's last window read and last store
        const d4 W2 = mfma(Ub, kg, W);          // [P A~ | P b~ + p]
        Hh = mfma(cg, fb, Hh);                  // + C^T diag(w) [C | gamma]
        Hh = mfma(hxa, kg, Hh);                 // H^_x T
        Hh = mfma(kg, V, Hh);                   // + K^T (H^_u T)
        Pa = mfma(Ab[0], W2[0], Hh);
        Pa = mfma(Ab[1], W2[1], Pa);
        Pa = mfma(Ab[2], W2[2], Pa);
        if constexpr (AUG) {  // [Phi | beta] <- [Phi A~ | Phi b~ + beta]  (Psi <- T^T Psi, T = [A~ b~; 0 1])
            const double e14 = (g == 2 && c == 14) ? 1.0 : 0.0;
            d4 Pn = {0.0, 0.0, 0.0, 0.0};
            Pn = mfma(Ab[0], Psi[0], Pn);
            Pn = mfma(Ab[1], Psi[1], Pn);
            Pn = mfma(Ab[2], Psi[2], Pn);
            Pn = mfma(e14, Psi[3], Pn);
            Psi = Pn;
        }
    };

    // ------------------------------------------------------------ backward stage, corrector
    // v = P c + p_{k+1};  lane r < 10: p_k[r] = g~_x[r] + (K^T g~_u)[r] + (A~^T v)[r]   (the chain)
    //                     lane 10 + i: z_u[i] = g~_u[i] + (B^T v)[i]
    // then w = L^-1 z_u, k_ff = -L^-T w, b~ = c + B k_ff (off the chain).  g~ = g + fold | box.
    double chain = 0.0;  // p_{k+1} in lanes 0..9
    double bacc = 0.0;   // beta of the corrector (lanes 0..9, segments 0..2)
    double cfv = 0.0;    // the corrector's record row (b~ | k_ff) of node cpend, stored by the next stage
    int cpend = -1;
    auto bc_stage = [&](auto Fc, auto AUGc, int k, const ldsd* cw, auto refill) {
        const int lane = opaque(lane_k);
        constexpr bool FIRST = decltype(Fc)::value;
        constexpr bool AUG = decltype(AUGc)::value;
        const bool fx = lane < NX, fu = lane >= NX && lane < 14;
        const int bx = fx ? lane : 0;
        // ---- the chain's offset: g~_x + K^T g~_u (lanes 0..9), g~_u (lanes 10..13)
        double off = *(lane < 14 ? cw + S_GV + lane : s.zero);
        if constexpr (FIRST) {  // the terminal rows' C from ctn (rows past nhN: zero rows, zero gamma)
#pragma unroll
            for (int j = 0; j < QP_NHN; ++j) {
                const double t = s.fg[N * NS + j] * s.ctn[10 * j + bx];
                off += fx ? t : 0.0;
            }
        } else {
            const ldsd* bc_ct = fx ? cw + S_CT + lane : s.zero;
#pragma unroll
            for (int j = 0; j < NS; ++j) off += s.fg[k * NS + j] * bc_ct[10 * j];
        }
        if constexpr (FIRST) {  // p_N = g_N + sum_j gamma_j C_j^T
            chain = off;
            if (cpend >= 0) bst(cfv, rsF, 8u * (lane < 14 ? lane * FR + 10 : S_J), (unsigned)cpend * (FRECS * 8u));
            cpend = -1;
            refill();
            return;
        }
        {
            const ldsd* bc_k = fx ? cw + S_K + lane : s.zero;
            const ldsd2* bq = (const ldsd2*)(s.bv + k * NU);
            const ldsd2* gq = (const ldsd2*)(cw + S_GV + NX);
            const d2 b0 = bq[0], b1 = bq[1], g0 = gq[0], g1 = gq[1];
            const double bvv[NU] = {b0.x, b0.y, b1.x, b1.y}, guw[NU] = {g0.x, g0.y, g1.x, g1.y};
#pragma unroll
            for (int i = 0; i < NU; ++i) off += bc_k[FR * i] * (guw[i] + bvv[i]) + (lane == NX + i ? bvv[i] : 0.0);
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- the chain: lane r < 10: p_k[r] = off + (A~^T (P c + p_{k+1}))[r]; lane 10 + i: z_u[i] = off + (B^T (P c + p_{k+1}))[i]
        double z;
        {
            const ldsd* bc_row = fx ? cw + S_AB + lane : fu ? cw + S_B + 10 * (lane - NX) : s.zero;
            const int bc_str = fx ? FR : 1;
            double row[NX];
#pragma unroll
            for (int l = 0; l < NX; ++l) row[l] = bc_row[l * bc_str];
            const ldsd2* pc = (const ldsd2*)(cw + S_PC);
            d2 pcv[NX / 2];
#pragma unroll
            for (int l = 0; l < NX / 2; ++l) pcv[l] = pc[l];
            double a0 = off, a1 = 0.0;
#pragma unroll
            for (int l = 0; l < NX / 2; ++l) {
                a0 = fma(row[2 * l], pcv[l].x + rdlane(chain, 2 * l), a0);
                a1 = fma(row[2 * l + 1], pcv[l].y + rdlane(chain, 2 * l + 1), a1);
            }
            z = a0 + a1;
        }
        chain = z;
        __builtin_amdgcn_sched_barrier(0);
        // ---- off the chain: w = L^-1 z_u, k_ff = -L^-T w, b~ = c + B k_ff
        const double z0 = rdlane(z, 10), z1 = rdlane(z, 11), z2 = rdlane(z, 12), z3 = rdlane(z, 13);
        const double i0 = cw[11], l10 = cw[11 + FR], i1 = cw[11 + 2 * FR], l20 = cw[11 + 3 * FR], l21 = cw[11 + 4 * FR];
        const double i2 = cw[11 + 5 * FR], l30 = cw[11 + 6 * FR], l31 = cw[11 + 7 * FR], l32 = cw[11 + 8 * FR], i3 = cw[11 + 9 * FR];
        const double w0 = z0 * i0;
        const double w1 = (z1 - l10 * w0) * i1;
        const double w2 = (z2 - l20 * w0 - l21 * w1) * i2;
        const double w3 = (z3 - l30 * w0 - l31 * w1 - l32 * w2) * i3;
        const double k3 = -w3 * i3;
        const double k2 = (-w2 - l32 * k3) * i2;
        const double k1 = (-w1 - l21 * k2 - l31 * k3) * i1;
        const double k0 = (-w0 - l10 * k1 - l20 * k2 - l30 * k3) * i0;
        const double bb = cw[S_C + bx] + cw[S_B + bx] * k0 + cw[S_B + 10 + bx] * k1 + cw[S_B + 20 + bx] * k2 + cw[S_B + 30 + bx] * k3;
        double dz = 0.0;
        if constexpr (AUG) {  // beta += Z (kf - kf_pred)
            const ldsd2* zr = (const ldsd2*)(cw + S_Z + 4 * bx);
            const d2 q0 = zr[0], q1 = zr[1];
            const double p0 = cw[S_K + 11], p1 = cw[S_K + FR + 11], p2 = cw[S_K + 2 * FR + 11], p3 = cw[S_K + 3 * FR + 11];
            dz = q0.x * (k0 - p0) + q0.y * (k1 - p1) + q1.x * (k2 - p2) + q1.y * (k3 - p3);
        }
        // the previous stage's record row goes out now, ahead of this stage's refill; this one's waits
        if (cpend >= 0) bst(cfv, rsF, 8u * (lane < 14 ? lane * FR + 10 : S_J), (unsigned)cpend * (FRECS * 8u));
        refill();
        cfv = fx ? bb : sel4(lane - NX, k0, k1, k2, k3);
        cpend = k;
        if constexpr (AUG) bacc += fx ? dz : 0.0;
    };

    // ------------------------------------------------------------ soft groups and box pairs of this lane
    struct Grp {
        double s1, s2, s3, s4, v1, v2, v3, v4, iHl, iHu, gl, gu;
    };
    // phase 1 (corrector): the affine deltas of the four rows, from the affine solution (cxa)
    auto group = [&](int phase, double sigmu) -> Grp {
        Grp g;
        const double Zsv = Zs(), zsv = zs(), hl = hl0(), hu = hu0();
        const double it1 = rcp_nr(ts[0]), it2 = rcp_nr(ts[1]), it3 = rcp_nr(ts[2]), it4 = rcp_nr(ts[3]);
        g.s1 = ls[0] * it1; g.s3 = ls[1] * it2; g.s2 = ls[2] * it3; g.s4 = ls[3] * it4;
        g.v1 = g.s1 * (ts[0] - hl);
        g.v3 = g.s3 * (ts[1] - hu);
        g.v2 = g.s2 * ts[2];
        g.v4 = g.s4 * ts[3];
        g.iHl = rcp_nr(Zsv + g.s1 + g.s2);
        g.iHu = rcp_nr(Zsv + g.s3 + g.s4);
        if (phase) {
            const double cxa = s.cxa[ksc * NS + js];
            const double sla = -((zsv - g.v1 - g.v2) + g.s1 * cxa) * g.iHl;
            const double sua = -((zsv - g.v3 - g.v4) - g.s3 * cxa) * g.iHu;
            const double d1 = cxa + hl + sla - ts[0];
            const double d2 = -cxa + hu + sua - ts[1];
            const double d3 = sla - ts[2], d4 = sua - ts[3];
            g.v1 -= (d1 * (-g.s1 * d1 - ls[0]) - sigmu) * it1;
            g.v3 -= (d2 * (-g.s3 * d2 - ls[1]) - sigmu) * it2;
            g.v2 -= (d3 * (-g.s2 * d3 - ls[2]) - sigmu) * it3;
            g.v4 -= (d4 * (-g.s4 * d4 - ls[3]) - sigmu) * it4;
        }
        g.gl = zsv - g.v1 - g.v2;
        g.gu = zsv - g.v3 - g.v4;
        return g;
    };
    // row values of the soft group at an LQR solution with C dx = cxs (rows hl, hu, sl, su)
    auto soft_vals = [&](const Grp& g, double cxs, double* v) {
        const double sl = -(g.gl + g.s1 * cxs) * g.iHl, su = -(g.gu - g.s3 * cxs) * g.iHu;
        v[0] = cxs + hl0() + sl;
        v[1] = -cxs + hu0() + su;
        v[2] = sl;
        v[3] = su;
    };
    auto terms = [&](int phase, double sigmu) {
#ifdef SEGX_NO_TERMS
        return;
#endif
        if (owns) {
            const Grp g = group(phase, sigmu);
            const double Zsv = Zs(), zsv = zs();
            if (!phase) s.fw[ksc * NS + js] = g.s1 * (Zsv + g.s2) * g.iHl + g.s3 * (Zsv + g.s4) * g.iHu;
            s.fg[ksc * NS + js] = -(g.v1 * (Zsv + g.s2) + g.s1 * (zsv - g.v2)) * g.iHl + (g.v3 * (Zsv + g.s4) + g.s3 * (zsv - g.v4)) * g.iHu;
        }
        if (ownh) {  // a hard row folds like a box pair: w = sigma_l + sigma_u, gamma = -v_l + v_u (rti_qp.hip)
            const double d0 = hl0(), d1 = hu0();
            const double it0 = rcp_nr(ts[0]), it1 = rcp_nr(ts[1]), sg0 = ls[0] * it0, sg1 = ls[1] * it1;
            double v0 = sg0 * (ts[0] - d0), v1 = sg1 * (ts[1] - d1);
            if (phase) {
                const double cx = s.cxa[ksc * NS + js];
                const double da0 = cx + d0 - ts[0], da1 = -cx + d1 - ts[1];
                v0 -= (da0 * (-sg0 * da0 - ls[0]) - sigmu) * it0;
                v1 -= (da1 * (-sg1 * da1 - ls[1]) - sigmu) * it1;
            }
            if (!phase) s.fw[ksc * NS + js] = sg0 + sg1;
            s.fg[ksc * NS + js] = -v0 + v1;
        }
        if (ownb) {
            const double d0 = dlo(), d1 = dup();
            const double it0 = rcp_nr(tb0), it1 = rcp_nr(tb1), sg0 = lb0 * it0, sg1 = lb1 * it1;
            double v0 = sg0 * (tb0 - d0), v1 = sg1 * (tb1 - d1);
            if (phase) {
                const double du = s.dua[kbc * NU + ib];
                const double da0 = du + d0 - tb0, da1 = -du + d1 - tb1;
                v0 -= (da0 * (-sg0 * da0 - lb0) - sigmu) * it0;
                v1 -= (da1 * (-sg1 * da1 - lb1) - sigmu) * it1;
            }
            if (!phase) s.bd[kbc * NU + ib] = sg0 + sg1;
            s.bv[kbc * NU + ib] = -v0 + v1;
        }
        wave_sync();
    };

    // ------------------------------------------------------------ coupling of segment w < 3
    // matrix part: from P_b (slot w) and this wave's J | eta (Pa), Psi, Cg; scratch = the two windows
    auto mchain = [&]() {
        const int lane = opaque(lane_k);
        const int g = lane >> 4, c = lane & 15;
        const ldsd* Pb = s.slot + 112 * w;
        ldsd* vv = s.vec;
        double col[NX], inv[NX];
        // L = chol(P_b), one column per lane
        // column `lane` of the symmetric P_b read as its row: ten contiguous doubles, five 16-byte reads
        {
            const ldsd2* pr = (const ldsd2*)(Pb + (lane < NX ? lane : 0) * NX);
#pragma unroll
            for (int l = 0; l < NX / 2; ++l) {
                const d2 v = pr[l];
                col[2 * l] = lane < NX ? v.x : (2 * l == (lane & 7) ? 1.0 : 0.0);
                col[2 * l + 1] = lane < NX ? v.y : (2 * l + 1 == (lane & 7) ? 1.0 : 0.0);
            }
        }
        chol_cols(col, inv, lane);
        SSTAMP(16);
        if (lane < NX) {
#pragma unroll
            for (int i = 0; i < NX; ++i)
                if (i >= lane) win[CP_L + trl(i, lane)] = col[i];
        }
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < NX; ++j) vv[V_IL + j] = inv[j];
        }
        wave_sync();
        d4 Lt;  // L tile
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = g + 4 * r;
            const bool ok = row < NX && c < NX && row >= c;
            Lt[r] = ldsel(win, CP_L + trl(ok ? row : 0, ok ? c : 0), ok);
        }
        d4 T = {0.0, 0.0, 0.0, 0.0};
        T = mfma(Cg[0], Lt[0], T);
        T = mfma(Cg[1], Lt[1], T);
        T = mfma(Cg[2], Lt[2], T);
        d4 S;
#pragma unroll
        for (int r = 0; r < 4; ++r) S[r] = (g + 4 * r == c) ? 1.0 : 0.0;
        S = mfma(Lt[0], T[0], S);
        S = mfma(Lt[1], T[1], S);
        S = mfma(Lt[2], T[2], S);
        SSTAMP(17);
        // U = chol(S): S through the V area of the scratch
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = g + 4 * r;
            if (row < NX && c < NX) win[CP_V + row * NX + c] = S[r];
        }
        wave_sync();
        {  // column `lane` of the symmetric S read as its row (five 16-byte reads)
            const ldsd2* sr = (const ldsd2*)(win + CP_V + (lane < NX ? lane : 0) * NX);
#pragma unroll
            for (int l = 0; l < NX / 2; ++l) {
                const d2 v = sr[l];
                col[2 * l] = lane < NX ? v.x : (2 * l == (lane & 7) ? 1.0 : 0.0);
                col[2 * l + 1] = lane < NX ? v.y : (2 * l + 1 == (lane & 7) ? 1.0 : 0.0);
            }
        }
        chol_cols(col, inv, lane);
        SSTAMP(18);
        if (lane < NX) {
#pragma unroll
            for (int i = 0; i < NX; ++i)
                if (i >= lane) win[CP_U + trl(i, lane)] = col[i];
        }
        if (lane == 0) {
#pragma unroll
            for (int j = 0; j < NX; ++j) vv[V_IU + j] = inv[j];
        }
        // row c of V = L U^-T: U^-1 (row c of L)^T in lane c, U[i][j] broadcast from lane j's column
        double y[NX];
#pragma unroll
        for (int j = 0; j < NX; ++j) {
            const bool ok = lane < NX && j <= lane;
            y[j] = ldsel(win, CP_L + trl(ok ? lane : 0, ok ? j : 0), ok);
        }
#pragma unroll
        for (int j = 0; j < NX; ++j) {
            y[j] *= inv[j];
#pragma unroll
            for (int i = j + 1; i < NX; ++i) y[i] = fma(-rdlane(col[i], j), y[j], y[i]);
        }
        SSTAMP(19);
        // Psi (Phi^T) into the X area; beta into vec
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = g + 4 * r;
            if (row < NX && c < NX) win[CP_X + row * NX + c] = Psi[r];
            if (row == 14 && c < NX) vv[V_B + c] = Psi[r];
        }
        wave_sync();
        if (lane < NX) {
#pragma unroll
            for (int j = 0; j < NX; ++j) win[CP_V + lane * NX + j] = y[j];
        }
        wave_sync();
        d4 Ph, Vt, VTt;  // [Phi | beta], V, V^T tiles
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = g + 4 * r, rc = row < NX ? row : 0, cc = c < NX ? c : 0;
            const bool in = row < NX && c < NX;
            const double px = win[CP_X + cc * NX + rc], pbv = vv[V_B + rc];
            Ph[r] = in ? px : (c == 14 && row < NX) ? pbv : 0.0;
            Vt[r] = ldsel(win, CP_V + rc * NX + cc, in);
            VTt[r] = ldsel(win, CP_V + cc * NX + rc, in);
        }
        d4 X = {0.0, 0.0, 0.0, 0.0};
        X = mfma(Vt[0], Ph[0], X);
        X = mfma(Vt[1], Ph[1], X);
        X = mfma(Vt[2], Ph[2], X);
#pragma unroll
        for (int r = 0; r < 4; ++r) X[r] = c < NX ? X[r] : 0.0;
        wave_sync();
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = g + 4 * r;
            if (row < NX && c < NX) win[CP_X + row * NX + c] = X[r];
        }
        if (w > 0) {  // P_a = J + X^T X into the slot of segment w - 1
            d4 Pn = Pa;
            Pn = mfma(X[0], X[0], Pn);
            Pn = mfma(X[1], X[1], Pn);
            Pn = mfma(X[2], X[2], Pn);
            ldsd* Pd = s.slot + 112 * (w - 1);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int row = g + 4 * r;
                if (row < NX && c < NX) Pd[row * NX + c] = Pn[r];
            }
        }
        // [Phi | beta] for moff, in the second window (free during the coupling): rows 10..15 of the tile
        // are 0 (row < NX) -- 16 x 16 slots
#pragma unroll
        for (int r = 0; r < 4; ++r) win[CP_PHI + (g + 4 * r) * 16 + c] = Ph[r];
        SSTAMP(20);
    };
    // off the chain (runs while the next segment couples): Lam = V X, M = Phi - C Lam (rows to the
    // coupling block for the x chain), C and the scratch to the coupling block
    auto moff = [&]() {
        const int lane = opaque(lane_k);
        const int g = lane >> 4, c = lane & 15;
        d4 cPh, cVTt, cX;  // [Phi | beta], V^T and X tiles from the scratch
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = g + 4 * r, rc = row < NX ? row : 0, cc = c < NX ? c : 0;
            const bool in = row < NX && c < NX;
            cPh[r] = win[CP_PHI + row * 16 + c];
            cVTt[r] = ldsel(win, CP_V + cc * NX + rc, in);
            cX[r] = ldsel(win, CP_X + rc * NX + cc, in);
        }
        d4 Lm = {0.0, 0.0, 0.0, 0.0};
        Lm = mfma(cVTt[0], cX[0], Lm);
        Lm = mfma(cVTt[1], cX[1], Lm);
        Lm = mfma(cVTt[2], cX[2], Lm);
        d4 D = {0.0, 0.0, 0.0, 0.0};
        D = mfma(Cg[0], Lm[0], D);
        D = mfma(Cg[1], Lm[1], D);
        D = mfma(Cg[2], Lm[2], D);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int row = g + 4 * r;
            if (row < NX && c < NX) {
                CP[CP_M + row * NX + c] = cPh[r] - D[r];
                CP[CP_LM + row * NX + c] = Lm[r];
                if (row >= c) win[CP_C + trl(row, c)] = Cg[r];
            }
            if (row < NX && c == 14) CP[CP_B + row] = cPh[r];  // beta of [Phi | beta]
        }
        wave_sync();
        for (int e = lane; e < CP_SC; e += 64) CP[e] = win[e];
        SSTAMP(21);
    };
    // vector part: eta, beta (lanes 0..9), p_b (slot w) -> p_a (slot w - 1, if w > 0), lam0, m (lanes 0..9);
    // scratch holds L, U, V, X, C of this segment, vec the reciprocal diagonals
    double lam0 = 0.0, mvec = 0.0;
    auto vchain = [&](double eta, double beta) {
        const int lane = opaque(lane_k);
        const ldsd* pb = s.slot + 112 * w + 100;
        ldsd* vv = s.vec;
        if (lane < NX) vv[V_B + lane] = beta;
        // q = U^-1 L^-1 p_b: lane i holds q_i; step j scales q_j and broadcasts it
        const int r = lane < NX ? lane : 0;
        double qr = pb[r];
        const double il = vv[V_IL + r], iu = vv[V_IU + r];
#pragma unroll
        for (int j = 0; j < NX; ++j) {
            const double lij = ldsel(win, CP_L + trl(r, j), lane > j && lane < NX);
            qr = lane == j ? qr * il : qr;
            qr = fma(-lij, rdlane(qr, j), qr);
        }
#pragma unroll
        for (int j = 0; j < NX; ++j) {
            const double uij = ldsel(win, CP_U + trl(r, j), lane > j && lane < NX);
            qr = lane == j ? qr * iu : qr;
            qr = fma(-uij, rdlane(qr, j), qr);
        }
        wave_sync();
        double z = qr;  // z = V^T beta + q
#pragma unroll
        for (int k = 0; k < NX; ++k) z = fma(win[CP_V + k * NX + r], vv[V_B + k], z);
        if (lane < NX) vv[V_Z + lane] = z;
        wave_sync();
        double l0 = 0.0, pa = eta;
#pragma unroll
        for (int k = 0; k < NX; ++k) {
            const double zk = vv[V_Z + k];
            l0 = fma(win[CP_V + r * NX + k], zk, l0);
            pa = fma(win[CP_X + k * NX + r], zk, pa);
        }
        if (lane < NX) {
            vv[V_L0 + lane] = l0;
            if (w > 0) s.slot[112 * (w - 1) + 100 + lane] = pa;
        }
        lam0 = l0;
    };
    // off the chain: m = beta - C lam0 (needs C in the scratch: after moff)
    auto voff = [&](double beta) {
        const int lane = opaque(lane_k);
        const int r = lane < NX ? lane : 0;
        wave_sync();
        double mm = beta;
#pragma unroll
        for (int k = 0; k < NX; ++k) {
            const int lo = r < k ? r : k, hi = r < k ? k : r;
            mm = fma(-win[CP_C + trl(hi, lo)], s.vec[V_L0 + k], mm);
        }
        mvec = mm;
    };
    // x chain step of segment w: x_b = M x_a + m (lanes 0..9), lam_b = Lam x_a + lam0 (lanes 16..25)
    auto xload = [&](double (&xrow)[NX]) {  // issued before the chain wait
        const int lane = opaque(lane_k);
        const int r = lane & 15;
        const double* src = CP + ((lane >> 4) == 1 ? CP_LM : CP_M) + (r < NX ? r : 0) * NX;
#pragma unroll
        for (int l = 0; l < NX; ++l) xrow[l] = src[l];
    };
    auto xstep = [&](const double (&xrow)[NX]) {
        const int lane = opaque(lane_k);
        const int r = lane & 15, hi = lane >> 4;
        if (lane < NX) s.vec[V_M + lane] = mvec;
        if (lane < NX) s.vec[V_L0 + lane] = lam0;
        wave_sync();
        double v = (hi == 1 && r < NX) ? s.vec[V_L0 + r] : s.vec[V_M + (r < NX ? r : 0)];
        const ldsd* xa = s.dxc + sa * NX;
#pragma unroll
        for (int l = 0; l < NX; ++l) v = fma(xrow[l], xa[l], v);
        if (hi == 0 && r < NX) s.dxc[sb * NX + r] = v;
        if (hi == 1 && r < NX) s.xlam[r] = v;
        wave_sync();
    };

    // ------------------------------------------------------------ sweeps of this wave
    const int nn = sb - sa;
    const int nf = w == NSEG - 1 ? N1 - sa : nn;  // factor / corrector positions
    const int kb0 = w == NSEG - 1 ? N : sb - 1;   // first node of the backward sweeps
    auto node_bw = [&](int q) { return kb0 - q; };
    auto node_fw = [&](int q) { return sa + q; };
    auto factor_sweep = [&]() {
        const FConst f = fconst(opaque(lane));
        if (aug) {
            sweep(IC<1>{}, nf, node_bw, [&](int q, int k, const ldsd* cw, auto rf) { bf_stage(IC<0>{}, IC<1>{}, k, f, cw, rf); (void)q; });
        } else {
            sweep(IC<1>{}, nf, node_bw, [&](int q, int k, const ldsd* cw, auto rf) {
                if (q == 0) bf_stage(IC<1>{}, IC<0>{}, k, f, cw, rf);
                else bf_stage(IC<0>{}, IC<0>{}, k, f, cw, rf);
            });
        }
    };
    auto corr_sweep = [&]() {
        if (aug) {
            sweep(IC<3>{}, nf, node_bw, [&](int q, int k, const ldsd* cw, auto rf) { bc_stage(IC<0>{}, IC<1>{}, k, cw, rf); (void)q; });
        } else {
            sweep(IC<3>{}, nf, node_bw, [&](int q, int k, const ldsd* cw, auto rf) {
                if (q == 0) bc_stage(IC<1>{}, IC<0>{}, k, cw, rf);
                else bc_stage(IC<0>{}, IC<0>{}, k, cw, rf);
            });
        }
    };
    // the x chain, then every segment's forward pass
    auto forward = [&](auto Kc) {
        double xrow[NX];
        xload(xrow);
#pragma unroll 1
        for (int st = 0; st < NSEG - 1; ++st) {
            wg_sync();
            if (w == st) xstep(xrow);
        }
        wg_sync();
        SSTAMP(decltype(Kc)::value == 2 ? 4 : 9);
        SSTAMP_PHASE(decltype(Kc)::value == 2 ? 12 : 14);
        if (aug) {
            sweep(Kc, nn, node_fw, [&](int q, int k, const ldsd* cw, auto rf) { fw_stage(Kc, IC<1>{}, IC<0>{}, k, k == sb - 1, cw, rf); (void)q; });
        } else {
            sweep(Kc, nn, node_fw, [&](int q, int k, const ldsd* cw, auto rf) {
                if (k == N) fw_stage(Kc, IC<0>{}, IC<1>{}, k, false, cw, rf);
                else fw_stage(Kc, IC<0>{}, IC<0>{}, k, false, cw, rf);
                (void)q;
            });
        }
    };

    // ------------------------------------------------------------ initial iterate (wave 0, all nodes)
#ifndef SEGX_NO_INIT
    if (w == 0)
        sweep(IC<0>{}, N1, node_fw, [&](int q, int k, const ldsd* cw, auto rf) {
            if (k == N) fw_stage(IC<0>{}, IC<0>{}, IC<1>{}, k, false, cw, rf);
            else fw_stage(IC<0>{}, IC<0>{}, IC<0>{}, k, false, cw, rf);
            (void)q;
        });
#endif
    wg_sync();
    for (int e = lane; e < nn * NX; e += 64) A.dx[((size_t)b * N1 + sa) * NX + e] = s.dxc[sa * NX + e];
    const int nu_ = (sb < N ? sb : N) - sa;
    // the iterate's du lives in A.du: the start point (0 cold; the entry values on a warm start, unless
    // they held a non-finite entry)
    for (int e = lane; e < nu_ * NU; e += 64) A.du[((size_t)b * N + sa) * NU + e] = s.dua[sa * NU + e];
    double rp = 0.0;
    {
        double rl = 0.0;
        if (ownb) {
            const double du = s.dua[kbc * NU + ib];  // the start iterate's
            const double d0 = dlo() + du, d1 = dup() - du;
            tb0 = fmax(d0, T0); tb1 = fmax(d1, T0); lb0 = L0; lb1 = L0;
            rl = fmax(fabs(d0 - tb0), fabs(d1 - tb1));
        }
        if (owns) {
            const double cx = s.cxa[ksc * NS + js];
            const double v[4] = {cx + hl0(), -cx + hu0(), 0.0, 0.0};
            const double l0 = fmax(L0, LC * s.skv[ksc] * s.cst[C_ZL + ci]);
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                ts[q] = fmax(v[q], T0);
                ls[q] = l0;
                rl = fmax(rl, fabs(v[q] - ts[q]));
            }
        }
        if (ownh) {  // hard row: lower cx + (h - lo), upper -cx + (hi - h) (rti_qp.hip rows_init)
            const double cx = s.cxa[ksc * NS + js];
            const double v0 = cx + hl0(), v1 = -cx + hu0();
            ts[0] = fmax(v0, T0);
            ts[1] = fmax(v1, T0);
            ls[0] = L0;
            ls[1] = L0;
            rl = fmax(rl, fmax(fabs(v0 - ts[0]), fabs(v1 - ts[1])));
        }
        rp = wg_red(wmax(rl), opmax);
    }
    auto own_tl = [&](double& sum, double& mx) {
        sum = 0.0;
        mx = 0.0;
        if (ownb) {
            sum += tb0 * lb0 + tb1 * lb1;
            mx = fmax(tb0 * lb0, tb1 * lb1);
        }
        if (owns || ownh) {  // a hard row's unused ts[2..3] / ls[2..3] stay 1 / 0
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                sum += ts[q] * ls[q];
                mx = fmax(mx, ts[q] * ls[q]);
            }
        }
    };
    double mu, cm;
    {
        double ps, pm;
        own_tl(ps, pm);
        const double ws = wsum(ps), wm = wmax(pm);
        mu = wg_red(ws, opsum) / m;
        cm = wg_red(wm, opmax);
    }
    double gap = 1.0;
    int it = 0;
    SSTAMP(0);
    while (!(cm < A.tol && rp < A.tol && gap < A.tol) && it < A.max_iter && __builtin_isfinite(mu + rp)) {
        // ---------------- factorisation + predictor
        terms(0, 0.0);
        park();
        SSTAMP(1);
        Pa = d4{0.0, 0.0, 0.0, 0.0};
        Cg = d4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int r = 0; r < 4; ++r) Psi[r] = ((lane >> 4) + 4 * r == (lane & 15) && (lane & 15) < NX) ? 1.0 : 0.0;
        lam0 = 0.0;
        mvec = 0.0;
        SSTAMP_PHASE(2);
#ifndef SEGX_NO_FACTOR
        factor_sweep();
#endif
        SSTAMP(2);
        double eta = 0.0, beta = 0.0;
        {
            const int g = lane >> 4, c = lane & 15;
            if (!aug) {  // P | p at the last segment's first node into the slot of the segment before it
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = g + 4 * r;
                    if (row < NX && c < NX) s.slot[112 * (NSEG - 2) + row * NX + c] = Pa[r];
                    if (row < NX && c == 14) s.slot[112 * (NSEG - 2) + 100 + row] = Pa[r];
                }
            } else {  // eta = column 14 of J | eta, beta = row 14 of Psi, into lanes 0..9
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int row = g + 4 * r;
                    if (row < NX && c == 14) win[row] = Pa[r];
                    if (row == 14 && c < NX) win[16 + c] = Psi[r];
                }
                wave_sync();
                eta = win[lane < NX ? lane : 0];
                beta = win[16 + (lane < NX ? lane : 0)];
                wave_sync();
            }
        }
        // the chain hands P_a, p_a down segment by segment; each segment's off-chain part runs while the
        // segment before it couples (wave 0's after the loop)
#pragma unroll 1
        for (int st = NSEG - 2; st >= 0; --st) {
            wg_sync();
            if (w == st) {
                SSTAMP(3);
#ifndef SEGX_NO_COUPLE
                mchain();
                wave_sync();
                vchain(eta, beta);
#endif
                SSTAMP(11);
            }
#ifndef SEGX_NO_COUPLE
            if (w == st + 1 && st + 1 < NSEG - 1) {
                SSTAMP(3);
                moff();
                voff(beta);
                SSTAMP(11);
            }
#endif
        }
#ifndef SEGX_NO_COUPLE
        if (w == 0) {
            moff();
            voff(beta);
        }
#endif
        SSTAMP(3);
#ifndef SEGX_NO_FWD
        forward(IC<2>{});
#endif
        unpark();
        wg_sync();
        SSTAMP(12);
        // ---------------- predictor rows: affine step, mu_aff -> sigma mu
        double sigmu = 1e-10;
#ifndef SEGX_NO_ROWS
        {
            double sdt[4] = {0.0, 0.0, 0.0, 0.0}, sdl[4] = {0.0, 0.0, 0.0, 0.0};
            double amax = 1.0;
            auto bound = [&](double t, double l, double dt, double dl) {
                if (dt < 0.0) amax = fmin(amax, -t * rcp_nr(dt));
                if (dl < 0.0) amax = fmin(amax, -l * rcp_nr(dl));
            };
            double bdt0 = 0.0, bdt1 = 0.0, bdl0 = 0.0, bdl1 = 0.0;
            if (ownb) {
                const double du = s.dua[kbc * NU + ib];
                bdt0 = du + dlo() - tb0;
                bdt1 = -du + dup() - tb1;
                bdl0 = -(lb0 * rcp_nr(tb0)) * bdt0 - lb0;
                bdl1 = -(lb1 * rcp_nr(tb1)) * bdt1 - lb1;
                bound(tb0, lb0, bdt0, bdl0);
                bound(tb1, lb1, bdt1, bdl1);
            }
            if (owns) {
                const Grp g = group(0, 0.0);
                double v[4];
                soft_vals(g, s.cxa[ksc * NS + js], v);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    sdt[q] = v[q] - ts[q];
                    sdl[q] = -(ls[q] * rcp_nr(ts[q])) * sdt[q] - ls[q];
                    bound(ts[q], ls[q], sdt[q], sdl[q]);
                }
            }
            if (ownh) {
                const double cx = s.cxa[ksc * NS + js];
                sdt[0] = cx + hl0() - ts[0];
                sdt[1] = -cx + hu0() - ts[1];
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    sdl[q] = -(ls[q] * rcp_nr(ts[q])) * sdt[q] - ls[q];
                    bound(ts[q], ls[q], sdt[q], sdl[q]);
                }
            }
            const double aa = wg_red(wmin(amax), opmin);
            double lmua = 0.0;
            if (ownb) lmua += (tb0 + aa * bdt0) * (lb0 + aa * bdl0) + (tb1 + aa * bdt1) * (lb1 + aa * bdl1);
            if (owns || ownh) {
#pragma unroll
                for (int q = 0; q < 4; ++q) lmua += (ts[q] + aa * sdt[q]) * (ls[q] + aa * sdl[q]);
            }
            const double mua = wg_red(wsum(lmua), opsum) / m;
            const double sig = (mua / mu) * (mua / mu) * (mua / mu);
            sigmu = fmax(sig * mu, 1e-2 * A.tol);
        }
#endif
        SSTAMP(5);
        // ---------------- corrector
        terms(1, sigmu);
        park();
        bacc = aug ? CP[CP_B + (lane < NX ? lane : 0)] : 0.0;
        chain = 0.0;
        cpend = -1;
        SSTAMP(6);
        SSTAMP_PHASE(7);
#ifndef SEGX_NO_CORR
        corr_sweep();
#endif
        if (cpend >= 0) bst(cfv, rsF, 8u * (lane < 14 ? lane * FR + 10 : S_J), (unsigned)cpend * (FRECS * 8u));
        SSTAMP(7);
        if (!aug) {
            if (lane < NX) s.slot[112 * (NSEG - 2) + 100 + lane] = chain;
        } else {
            for (int e = lane; e < CP_SC; e += 64) win[e] = CP[e];
        }
        const double etac = chain, betac = bacc;
#pragma unroll 1
        for (int st = NSEG - 2; st >= 0; --st) {
            wg_sync();
            if (w == st) {
                SSTAMP(8);
#ifndef SEGX_NO_COUPLE
                vchain(etac, betac);
#endif
                SSTAMP(13);
            }
#ifndef SEGX_NO_COUPLE
            if (w == st + 1 && st + 1 < NSEG - 1) {
                SSTAMP(8);
                voff(betac);
                SSTAMP(13);
            }
#endif
        }
#ifndef SEGX_NO_COUPLE
        if (w == 0) voff(betac);
#endif
        SSTAMP(8);
#ifndef SEGX_NO_FWD
        forward(IC<4>{});
#endif
        unpark();
        wg_sync();
        SSTAMP(14);
        // ---------------- step length, update, mu
#ifdef SEGX_NO_ROWS
        mu *= 0.5; cm *= 0.5;
#else
        {
            double sdt[4] = {0.0, 0.0, 0.0, 0.0}, sdl[4] = {0.0, 0.0, 0.0, 0.0};
            double amax = 1.0;
            auto bound = [&](double t, double l, double dt, double dl) {
                if (dt < 0.0) amax = fmin(amax, -t * rcp_nr(dt));
                if (dl < 0.0) amax = fmin(amax, -l * rcp_nr(dl));
            };
            double bdt[2] = {0.0, 0.0}, bdl[2] = {0.0, 0.0};
            if (ownb) {
                const double duc = s.duc[kbc * NU + ib], dua = s.dua[kbc * NU + ib], d0 = dlo(), d1 = dup();
                const double dt0 = duc + d0 - tb0, dt1 = -duc + d1 - tb1;
                const double da0 = dua + d0 - tb0, da1 = -dua + d1 - tb1;
                const double it0 = rcp_nr(tb0), it1 = rcp_nr(tb1), sg0 = lb0 * it0, sg1 = lb1 * it1;
                bdt[0] = dt0;
                bdt[1] = dt1;
                bdl[0] = -sg0 * dt0 - lb0 - (da0 * (-sg0 * da0 - lb0) - sigmu) * it0;
                bdl[1] = -sg1 * dt1 - lb1 - (da1 * (-sg1 * da1 - lb1) - sigmu) * it1;
                bound(tb0, lb0, bdt[0], bdl[0]);
                bound(tb1, lb1, bdt[1], bdl[1]);
            }
            if (owns) {
                const Grp ga = group(0, 0.0), gc = group(1, sigmu);
                double va[4], vc[4];
                soft_vals(ga, s.cxa[ksc * NS + js], va);
                soft_vals(gc, s.cxc[ksc * NS + js], vc);
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const double dta = va[q] - ts[q];
                    sdt[q] = vc[q] - ts[q];
                    const double itq = rcp_nr(ts[q]), sg = ls[q] * itq;
                    sdl[q] = -sg * sdt[q] - ls[q] - (dta * (-sg * dta - ls[q]) - sigmu) * itq;
                    bound(ts[q], ls[q], sdt[q], sdl[q]);
                }
            }
            if (ownh) {
                const double cc = s.cxc[ksc * NS + js], ca = s.cxa[ksc * NS + js];
                const double dd[2] = {hl0(), hu0()};
#pragma unroll
                for (int q = 0; q < 2; ++q) {
                    const double dta = (q ? -ca : ca) + dd[q] - ts[q];
                    sdt[q] = (q ? -cc : cc) + dd[q] - ts[q];
                    const double itq = rcp_nr(ts[q]), sg = ls[q] * itq;
                    sdl[q] = -sg * sdt[q] - ls[q] - (dta * (-sg * dta - ls[q]) - sigmu) * itq;
                    bound(ts[q], ls[q], sdt[q], sdl[q]);
                }
            }
            const double tau = fmin(TAU_HI, fmax(TAU_LO, 1.0 - mu));
            const double al = fmin(1.0, tau * wg_red(wmin(amax), opmin));
            if (ownb) {
                tb0 += al * bdt[0]; lb0 += al * bdl[0];
                tb1 += al * bdt[1]; lb1 += al * bdl[1];
            }
            if (owns || ownh) {
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    ts[q] += al * sdt[q];
                    ls[q] += al * sdl[q];
                }
            }
            for (int e = lane; e < nn * NX; e += 64) {
                double* p = A.dx + ((size_t)b * N1 + sa) * NX + e;
                *p += al * (s.dxc[sa * NX + e] - *p);
            }
            for (int e = lane; e < nu_ * NU; e += 64) {
                double* p = A.du + ((size_t)b * N + sa) * NU + e;
                *p += al * (s.duc[sa * NU + e] - *p);
            }
            double ps, pm;
            own_tl(ps, pm);
            const double ws = wsum(ps), wm = wmax(pm);
            mu = wg_red(ws, opsum) / m;
            cm = wg_red(wm, opmax);
            rp *= (1.0 - al);
            gap *= (1.0 - al);
        }
#endif
        SSTAMP(10);
        ++it;
    }
    SSTAMP_OUT
    // ------------------------------------------------------------ outputs
    // slacks [N+1][3][2] (rti_qp.hip's layout): stage node k's soft row j, the terminal soft row j; zero past them
    if (A.slack && (tlane ? jt < 3 : ks < (last ? N : sb))) {
        A.slack[((size_t)b * N1 * NS + ks * NS + js) * 2] = owns ? ts[2] : 0.0;
        A.slack[((size_t)b * N1 * NS + ks * NS + js) * 2 + 1] = owns ? ts[3] : 0.0;
    }
    if (tid == 0) {
        A.iters[b] = it;
        A.status[b] = !__builtin_isfinite(mu + rp) ? 2 : (cm < A.tol && rp < A.tol && gap < A.tol) ? 0 : 1;
        A.res[b * 2] = cm;
        A.res[b * 2 + 1] = rp;
    }
}

// instantiations: (segments, largest horizon); a segment holds at most 16 nodes (a wave's box pairs, 4
// per node, within its 64 lanes) and at least 2
struct SegCfg {
    int P, NMAX;
};
constexpr SegCfg SEG_CFGS[] = {{2, 31}, {3, 47}, {4, 63}};
static size_t seg_lds_bytes(int P, int NMAX) {
    switch (P) {
        case 2: return sizeof(double) * SegLds<2, 31>::TOTAL;
        case 3: return sizeof(double) * SegLds<3, 47>::TOTAL;
        default: return sizeof(double) * SegLds<4, 63>::TOTAL;
    }
    (void)NMAX;
}
// segments per instance for horizon N (0: unsupported): four where they fit, else three, else two (the
// kernel serves latency-sized batches -- one workgroup per CU -- where more segments mean a shorter
// chain: B = 1 at N = 40 takes 0.583 ms with four, 0.599 ms with three; at N = 60 only four fit).  SDFNMPC_QP_NSEG = 2, 3, 4
// overrides (diagnostic).
int rti_qp_seg_count(int N) {
    auto fits = [&](int P) {
        for (const SegCfg& c : SEG_CFGS)
            if (c.P == P) return N <= c.NMAX && N + 1 >= 2 * P;
        return false;
    };
    if (const char* e = getenv("SDFNMPC_QP_NSEG")) {
        const int P = atoi(e);
        return fits(P) ? P : 0;
    }
    return fits(4) ? 4 : fits(3) ? 3 : fits(2) ? 2 : 0;
}

bool rti_qp_seg_supported(int N) { return rti_qp_seg_count(N) > 0; }

size_t qp_seg_lds_bytes(int N) {
    const int P = rti_qp_seg_count(N);
    for (const SegCfg& c : SEG_CFGS)
        if (c.P == P) return seg_lds_bytes(c.P, c.NMAX);
    return 0;
}

template <int P, int NMAX>
static int seg_blocks_per_cu() {
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, rti_qp_seg_kernel<P, NMAX>, 64 * P, 0) != hipSuccess) return 0;
    return n;
}

// workgroups (instances) per CU at horizon N: the minimum of the LDS, register (__launch_bounds__) and wave
// limits, as the runtime applies them
int rti_qp_seg_blocks_per_cu(int N) {
    switch (rti_qp_seg_count(N)) {
        case 2: return seg_blocks_per_cu<2, 31>();
        case 3: return seg_blocks_per_cu<3, 47>();
        case 4: return seg_blocks_per_cu<4, 63>();
        default: return 0;
    }
}

template <int P, int NMAX>
static hipError_t launch_seg(const QpArgs& a, hipStream_t s) {
    hipLaunchKernelGGL((rti_qp_seg_kernel<P, NMAX>), dim3(a.B), dim3(64 * P), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_rti_qp_seg(const QpArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    switch (rti_qp_seg_count(a.N)) {
        case 2: return launch_seg<2, 31>(a, s);
        case 3: return launch_seg<3, 47>(a, s);
        case 4: return launch_seg<4, 63>(a, s);
        default: return hipErrorInvalidValue;
    }
}

}  // namespace sdfn
