// Device helpers shared by the QP kernels (rti_qp.hip: one wavefront per instance; rti_qp_seg.hip: one
// workgroup of four wavefronts per instance, a partitioned Riccati).
#pragma once
#include <hip/hip_runtime.h>

#include <type_traits>

#include "qp_kernels.h"

namespace sdfn {
namespace qpd {

// LDS pointers must keep address space 3: a generic pointer compiles to flat_load/store, whose waits
// (vmcnt(0) AND lgkmcnt(0)) drain every global prefetch in flight at each LDS access.
typedef __attribute__((address_space(3))) double ldsd;
typedef double d2 __attribute__((ext_vector_type(2)));
typedef __attribute__((address_space(3))) d2 ldsd2;
typedef double d4 __attribute__((ext_vector_type(4)));
template <int V>
using IC = std::integral_constant<int, V>;

constexpr int NX = 10, NU = 4, NS = 3;
// stage record: [AB 140 (column j = d xn / d (x,u)_j) | c 10 | g 14 | C^T 30 (row j = d h_j / d x) | H 105 upper | 0]
constexpr int R_AB = 0, R_C = 140, R_G = 150, R_CT = 164, R_H = 194, R_Z = 299, REC = QP_REC;
constexpr int FR = 12;  // factor-record row stride (11 used: a forward stage reads its row with five 16-byte LDS reads)
// IPM starting point and step fraction (the kernel waits for its slowest instance, so these were
// chosen on the worst case over seeds / x0 spreads with the C restatement, oracle/qp_ipm.c):
// t = max(row value, T0); lambda = L0 on the box rows and max(L0, LC s_k zl_j) on the four rows of
// soft group (k, j) (the duals of the penalised slacks start near their optimal magnitude, and the
// slack rows' stationarity s_k zl - lambda_h - lambda_s starts at 0); step fraction
// tau = min(TAU_HI, max(TAU_LO, 1 - mu)).
#ifndef QP_T0
#define QP_T0 0.5
#endif
#ifndef QP_L0
#define QP_L0 1.0
#endif
#ifndef QP_LC
#define QP_LC 0.5
#endif
#ifndef QP_TAU_LO
#define QP_TAU_LO 0.995
#endif
#ifndef QP_TAU_HI
#define QP_TAU_HI 0.995
#endif
constexpr double T0 = QP_T0, L0 = QP_L0, LC = QP_LC, TAU_LO = QP_TAU_LO, TAU_HI = QP_TAU_HI;

__device__ __forceinline__ int tri10(int a, int c) { return a * 10 - a * (a - 1) / 2 + (c - a); }  // a <= c
__device__ __forceinline__ int tri14(int a, int c) { return a * 14 - a * (a - 1) / 2 + (c - a); }  // a <= c

// value of lane l (wave-uniform l) in every lane, via scalar registers
__device__ __forceinline__ double rdlane(double v, int l) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, l);
    const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), l);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// DPP move of a double (both halves with the same control); rows outside row_mask keep `old`
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp64(double x, double old) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(x);
    const unsigned long long o = (unsigned long long)__double_as_longlong(old);
    const unsigned lo = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)o, (int)(unsigned)u, CTRL, ROWS, 0xF, false);
    const unsigned hi = (unsigned)__builtin_amdgcn_update_dpp((int)(unsigned)(o >> 32), (int)(unsigned)(u >> 32), CTRL, ROWS,
                                                              0xF, false);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}
// wave reduction on DPP (quad xor 1, 2, half-row and row mirrors, then row_bcast15 / row_bcast31 into
// lane 63, read back through a scalar register): no LDS round trips, one fixed order in every lane
template <class Op>
__device__ __forceinline__ double wred(double v, double idn, Op op) {
    v = op(v, dpp64<0xB1, 0xF>(v, idn));   // quad_perm [1, 0, 3, 2]
    v = op(v, dpp64<0x4E, 0xF>(v, idn));   // quad_perm [2, 3, 0, 1]
    v = op(v, dpp64<0x141, 0xF>(v, idn));  // row_half_mirror
    v = op(v, dpp64<0x140, 0xF>(v, idn));  // row_mirror: every lane of a row holds the row's value
    v = op(v, dpp64<0x142, 0xA>(v, idn));  // row_bcast15: rows 1, 3 += rows 0, 2
    v = op(v, dpp64<0x143, 0xC>(v, idn));  // row_bcast31: rows 2, 3 += rows 0 + 1
    return rdlane(v, 63);
}
__device__ __forceinline__ double wsum(double v) {
    return wred(v, 0.0, [](double a, double b) { return a + b; });
}
__device__ __forceinline__ double wmax(double v) {
    return wred(v, -__builtin_inf(), [](double a, double b) { return fmax(a, b); });
}
__device__ __forceinline__ double wmin(double v) {
    return wred(v, __builtin_inf(), [](double a, double b) { return fmin(a, b); });
}
__device__ __forceinline__ d4 mfma(double a, double b, d4 c) {
    return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
// f64 4x4x4, four blocks: with the A block replicated over the blocks (lane (g, c) holds A[c & 3][g]) it is
// rows 0..3 of the 16x16x4 product in one accumulator register (lane (g, c): D[g][c]) at a quarter of
// the matrix-pipe time (16 cycles against 64, dependent latency ~21 against ~67 on gfx950)
__device__ __forceinline__ double mfma4(double a, double b, double c) {
    return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
// 1/x: hardware estimate + two Newton steps (the IPM's row updates; replaces IEEE division)
__device__ __forceinline__ double rcp_nr(double x) {
    double y = __builtin_amdgcn_rcp(x);
    double e = fma(-x, y, 1.0);
    y = fma(y, e, y);
    e = fma(-x, y, 1.0);
    return fma(y, e, y);
}
// 1/sqrt(v), v > 0: hardware estimate + one Newton step
__device__ __forceinline__ double rsqrt_nr(double v) {
    double y = __builtin_amdgcn_rsq(v);
    const double h = 0.5 * v;
    return y * fma(-h * y, y, 1.5);
}
// The QP kernel runs one wavefront per workgroup, and a wave's LDS operations complete in issue
// order: a stage hand-off only has to stop the compiler from moving LDS accesses across it (a
// workgroup barrier would also drain lgkmcnt at every stage).
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

typedef unsigned u2 __attribute__((ext_vector_type(2)));
// raw buffer store of one double: SGPR resource + 32-bit lane byte offset + uniform byte offset
__device__ __forceinline__ void bst(double v, __amdgpu_buffer_rsrc_t r, unsigned vo, unsigned so) {
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), r, vo, so, 0);
}

// a copy of v the compiler cannot see through (blocks hoisting of what is derived from it)
__device__ __forceinline__ int opaque(int v) {
    int r;
    asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
    return r;
}


}  // namespace qpd
}  // namespace sdfn
