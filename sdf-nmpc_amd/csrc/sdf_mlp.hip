// NeuralDF forward + position-Jacobian on gfx950 -- the compute-bound half of the hot path.
//
// Reference semantics (paths relative to /root/reference):
//   PositionEmbedding.forward  sdf_nmpc/utils/embeddings.py:106-111 (e = [x, sin(xb), sin(xb+pi/2)])
//   NeuralDF.forward           sdf_nmpc/network/neural_df.py:91-103 (res='full'), Sine activation.py:12
//   d df / d input             what L4CasADi's jac_sdf_l4c returns (gen_model.py:39, with_jacobian)
//
// Design:
//   * one workgroup = M rows (M = 32 or 64) of (instance, node) pairs, 4 waves, every layer an
//     exact-fp32 MFMA GEMM (v_mfma_f32_32x32x2_f32) OUT[M x N] = IN[M x K] . W^T with the
//     activations in LDS (row stride = 4 mod 8 floats: conflict-free ds_read_b128) and the weights
//     streamed from L2 straight into registers, pre-packed so each wave-instruction loads 1 KiB
//     contiguous (16 B per lane = 4 k-steps).
//   * the latent half of layers 1 and 3 (W1[:,83:] z + b1, W3[:,339:] z + b3) is hoisted per
//     instance by sdf_hoist_kernel and enters as the accumulator's initial value.
//   * reverse mode for d df / d pos: each wave owns the same output columns in the forward layer l
//     and in the backward GEMM producing d h_l, so the activation derivatives cos(w0 a_l) never
//     leave the wave's registers; only the activations/deltas of the current layer live in LDS.
//   * the embedding is built in the accumulator layout of the d e GEMM, so its derivative factors
//     (cos(xb), cos(xb + pi/2)) also stay in registers until the final contraction.
#include <hip/hip_runtime.h>

#include "sdf_kernels.h"
#include "sincos.h"

namespace sdfn {

typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
#ifdef SDF_NO_MFMA  // diagnostic build (tools/build_variant.sh): the kernel's time without its matrix work
    c[0] = fmaf(a, b, c[0]);
    return c;
#else
    return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
#endif
}

// weight prefetch depth of the GEMM loop, in groups of 4 k-steps
#ifndef SDF_PF
#define SDF_PF 3
#endif

#ifdef SDF_NO_SYNC  // diagnostic build: the kernel's time without its workgroup barriers (results invalid)
#define SDF_SYNC() __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup")
#else
#define SDF_SYNC() __syncthreads()
#endif

// Row held by accumulator register `reg` of lane half `h` (32x32 f32 MFMA C/D layout, gfx950).
__device__ __forceinline__ int acc_row(int reg, int h) { return (reg & 3) + 8 * (reg >> 2) + 4 * h; }

// acc[rb][c] += IN[rb*32 .. +32][0..K) . Wpk(cb = cb0 + 4c)  for every row block rb and the wave's
// column blocks.  Feature k of k-step s, lane half h is k = h*K/2 + s (any bijection works as long as
// A and B agree; this one makes both operands 16-B contiguous per lane over 4 k-steps).
// Weights (L2-resident) are prefetched PF groups ahead in a register ring, activations (LDS) one ahead.
// Only groups [G0, G1) of the K/8 groups of 4 k-steps are accumulated (K-split between waves).
template <int RB, int NCB, int K, int CBS = 4, int G0 = 0, int G1 = K / 8>
__device__ __forceinline__ void gemm(f32x16 (&acc)[RB][NCB], const float* lds, int stride,
                                     const float4* __restrict__ wpk, int cb0, int lane) {
    constexpr int G = K / 8;
    constexpr int NG = G1 - G0;
    constexpr int PF = (NG < SDF_PF) ? NG : SDF_PF;
    static_assert(0 <= G0 && G0 < G1 && G1 <= G, "group range");
    static_assert(K % 8 == 0, "K must be a multiple of 8");
#ifdef SDF_PRIO_GEMM  // diagnostic: raise the wave's issue priority over its matrix phase
    __builtin_amdgcn_s_setprio(2);
#endif
    const int r = lane & 31, h = lane >> 5;
    const float* abase = lds + r * stride + h * (K / 2);
    const float4* bbase = wpk + (size_t)cb0 * G * 64 + lane;
    float4 bring[PF][NCB];
    float4 a[RB];
#pragma unroll
    for (int q = 0; q < PF; ++q)
#pragma unroll
        for (int c = 0; c < NCB; ++c) bring[q][c] = bbase[(size_t)c * CBS * G * 64 + (G0 + q) * 64];
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) a[rb] = *(const float4*)(abase + rb * 32 * stride + 4 * G0);
#pragma unroll
    for (int q = 0; q < NG; ++q) {
        const int g = G0 + q;
        float4 b[NCB], an[RB];
#pragma unroll
        for (int c = 0; c < NCB; ++c) b[c] = bring[q % PF][c];
        if (q + PF < NG) {
#pragma unroll
            for (int c = 0; c < NCB; ++c) bring[q % PF][c] = bbase[(size_t)c * CBS * G * 64 + (g + PF) * 64];
        }
        if (q + 1 < NG) {
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) an[rb] = *(const float4*)(abase + rb * 32 * stride + 4 * (g + 1));
        }
        // keep the prefetches issued here: the scheduler would otherwise sink every load to just
        // before its first use (one MFMA group ahead), exposing the L2 latency
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int c = 0; c < NCB; ++c) {
                acc[rb][c] = mfma(a[rb].x, b[c].x, acc[rb][c]);
                acc[rb][c] = mfma(a[rb].y, b[c].y, acc[rb][c]);
                acc[rb][c] = mfma(a[rb].z, b[c].z, acc[rb][c]);
                acc[rb][c] = mfma(a[rb].w, b[c].w, acc[rb][c]);
            }
        __builtin_amdgcn_sched_barrier(0);
        if (q + 1 < NG) {
#pragma unroll
            for (int rb = 0; rb < RB; ++rb) a[rb] = an[rb];
        }
    }
#ifdef SDF_PRIO_GEMM
    __builtin_amdgcn_s_setprio(0);
#endif
}

template <int RB, int NCB>
__device__ __forceinline__ void zero(f32x16 (&acc)[RB][NCB]) {
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int c = 0; c < NCB; ++c)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[rb][c][i] = 0.0f;
}

// accumulator init from a per-column vector (bias)
template <int RB, int NCB, int CBS = 4>
__device__ __forceinline__ void init_bias(f32x16 (&acc)[RB][NCB], const float* __restrict__ v, int cb0, int lane) {
#pragma unroll
    for (int c = 0; c < NCB; ++c) {
        const float bv = v[(cb0 + CBS * c) * 32 + (lane & 31)];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int i = 0; i < 16; ++i) acc[rb][c][i] = bv;
    }
}

// accumulator init from the hoisted per-instance latent projection c[inst(row)][col]
template <int RB, int NCB>
__device__ __forceinline__ void init_hoisted(f32x16 (&acc)[RB][NCB], const float* __restrict__ c13, int c_off,
                                             const int* inst_lds, int cb0, int lane) {
    const int col = lane & 31, h = lane >> 5;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const float* crow = c13 + (size_t)inst_lds[rb * 32 + acc_row(i, h)] * C13_STRIDE + c_off + col;
#pragma unroll
            for (int c = 0; c < NCB; ++c) acc[rb][c][i] = crow[(cb0 + 4 * c) * 32];
        }
}

#ifdef SDF_CHEAP_SIN  // diagnostic build (tools/build_variant.sh): the kernel's time without its sine epilogues
__device__ __forceinline__ void act_sincos(float x, float* s, float* c) { *s = x * 0.01f; *c = 1.0f - x; }
#else
__device__ __forceinline__ void act_sincos(float x, float* s, float* c) { sdfn_sincosf(x, s, c); }
#endif

// sine activation epilogue: t = w0*acc, h = sin(t) -> LDS, keep cos(t) in `d`
template <int RB, int NCB>
__device__ __forceinline__ void act_fwd(f32x16 (&acc)[RB][NCB], f32x16 (&d)[RB][NCB], float* out, int stride,
                                        float w0, int cb0, int lane) {
    const int col = lane & 31, h = lane >> 5;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int c = 0; c < NCB; ++c)
#pragma unroll
            for (int i = 0; i < 16; i += 2) {
                float s0, c0, s1, c1;
#ifdef SDF_CHEAP_SIN
                act_sincos(w0 * acc[rb][c][i], &s0, &c0);
                act_sincos(w0 * acc[rb][c][i + 1], &s1, &c1);
#else
                sdfn_sincosf2(w0 * acc[rb][c][i], w0 * acc[rb][c][i + 1], &s0, &c0, &s1, &c1);  // packed fp32 pipe
#endif
                d[rb][c][i] = c0;
                d[rb][c][i + 1] = c1;
                out[(rb * 32 + acc_row(i, h)) * stride + (cb0 + 4 * c) * 32 + col] = s0;
                out[(rb * 32 + acc_row(i + 1, h)) * stride + (cb0 + 4 * c) * 32 + col] = s1;
            }
}

// backward epilogue: delta_a = (delta_h * cos(t)) * w0 -> LDS  (torch SinBackward then MulBackward)
template <int RB, int NCB>
__device__ __forceinline__ void act_bwd(const f32x16 (&acc)[RB][NCB], const f32x16 (&d)[RB][NCB], float* out,
                                        int stride, float w0, int cb0, int lane) {
    const int col = lane & 31, h = lane >> 5;
#pragma unroll
    for (int rb = 0; rb < RB; ++rb)
#pragma unroll
        for (int c = 0; c < NCB; ++c)
#pragma unroll
            for (int i = 0; i < 16; i += 2) {  // two elements per packed multiply (the same products)
                const sdfn_f2 a2 = {acc[rb][c][i], acc[rb][c][i + 1]}, d2 = {d[rb][c][i], d[rb][c][i + 1]};
                const sdfn_f2 v = (a2 * d2) * w0;
                out[(rb * 32 + acc_row(i, h)) * stride + (cb0 + 4 * c) * 32 + col] = v.x;
                out[(rb * 32 + acc_row(i + 1, h)) * stride + (cb0 + 4 * c) * 32 + col] = v.y;
            }
}

// ------------------------------------------------------------------------------------------------
template <int M, bool LATENT_GRAD>
__global__ __launch_bounds__(256, (M == 32) ? 2 : 1) void sdf_mlp_kernel(SdfArgs A) {
    constexpr int RB = M / 32;
    extern __shared__ __align__(16) float lds[];
    float* Abuf = lds;                       // [M][SA]
    float* Ebuf = Abuf + M * SA;             // [M][SE]  embedding e (fwd), h4 (after L3)
    float* Bbuf = Ebuf + M * SE;             // [M][SA]
    float* posb = Bbuf + M * SA;             // [M][4]   pos, later (df, g0, g1, g2)
    int* instb = (int*)(posb + M * 4);       // [M]      instance of each row

    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int col = lane & 31, hh = lane >> 5;
    const int row0 = blockIdx.x * M;
    const float w0 = A.w0;

    // ---- rows of this tile: position and instance index
    if (tid < M) {
        const int r = row0 + tid;
        const int rr = r < A.rows ? r : A.rows - 1;
        float4 p;
        if (A.x) {  // Co_p_B = W_R_Co^T (W_p_B - W_p_Co) in fp64, handed over as fp32 (gen_model.py:46-51)
            const double* xr = A.x + (size_t)rr * 10;
            const double* pr = A.p + (size_t)rr * A.np;
            const double* R = pr + 4;
            const double e0 = xr[0] - pr[1], e1 = xr[1] - pr[2], e2 = xr[2] - pr[3];
            p = make_float4((float)((e0 * R[0] + e1 * R[3]) + e2 * R[6]), (float)((e0 * R[1] + e1 * R[4]) + e2 * R[7]),
                            (float)((e0 * R[2] + e1 * R[5]) + e2 * R[8]), 0.0f);
        } else {
            p = A.pos[rr];
        }
        posb[tid * 4 + 0] = r < A.rows ? p.x : 0.0f;
        posb[tid * 4 + 1] = r < A.rows ? p.y : 0.0f;
        posb[tid * 4 + 2] = r < A.rows ? p.z : 0.0f;
        instb[tid] = rr / A.rows_per_inst;
    }
    SDF_SYNC();

    // ---- positional embedding in the (rb, cb = w) accumulator layout of the d e GEMM (waves 0..2)
    f32x16 gemb[RB][1];  // d e_m / d xb  (cos(xb) | cos(xb + pi/2) | 1 for m < 3 | 0 pad)
    const float4 ptab = (w < 3) ? A.emb_tab[w * 32 + col] : make_float4(0, 0, 0, 0);
    if (w < 3) {
        const int m = w * 32 + col;
        const float half_pi = 1.57079637050628662109375f;  // (float)(0.5 * np.pi)
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int row = rb * 32 + acc_row(i, hh);
                const float px = posb[row * 4], py = posb[row * 4 + 1], pz = posb[row * 4 + 2];
                float e, g;
                if (m < 3) {
                    e = (m == 0) ? px : (m == 1 ? py : pz);
                    g = 1.0f;
                } else if (m < 3 + 2 * EMB_NB) {
                    float xb = px * ptab.x + py * ptab.y + pz * ptab.z;  // proj * 2^f (exact scaling)
                    if (m >= 3 + EMB_NB) xb = xb + half_pi;
                    float s, c;
                    sdfn_sincosf(xb, &s, &c);
                    e = s;
                    g = c;
                } else {
                    e = 0.0f;
                    g = 0.0f;
                }
                gemb[rb][0][i] = g;
                if (m < KE) Ebuf[row * SE + m] = e;
            }
    }
    SDF_SYNC();

    // ---- L1: h1 = sin(w0 (W1e e + c1))                 [M x 256], wave cols {w, w+4}
    f32x16 d1[RB][2], acc2[RB][2];
    init_hoisted(acc2, A.c13, 0, instb, w, lane);
    gemm<RB, 2, KE>(acc2, Ebuf, SE, A.wF1, w, lane);
    act_fwd(acc2, d1, Abuf, SA, w0, w, lane);
    SDF_SYNC();
    // ---- L2: h2 = sin(w0 (W2 h1 + b2))                  [M x 256]
    f32x16 d2[RB][2];
    init_bias(acc2, A.b2, w, lane);
    gemm<RB, 2, N1>(acc2, Abuf, SA, A.wF2, w, lane);
    act_fwd(acc2, d2, Bbuf, SA, w0, w, lane);
    SDF_SYNC();
    // ---- L3: h3 = sin(w0 (W3h h2 + W3e e + c3))        [M x 128], wave col {w}
    f32x16 d3[RB][1], acc1[RB][1];
    init_hoisted(acc1, A.c13, N1, instb, w, lane);
    gemm<RB, 1, N2>(acc1, Bbuf, SA, A.wF3h, w, lane);
    gemm<RB, 1, KE>(acc1, Ebuf, SE, A.wF3e, w, lane);
    act_fwd(acc1, d3, Abuf, SA, w0, w, lane);
    SDF_SYNC();
    // ---- L4: h4 = sin(w0 (W4 h3 + b4))                  [M x 64], waves 2,3 (col block w-2)
    //      delta4 = (W5 * cos(t4)) * w0 -> Bbuf, h4 -> Ebuf
    if (w >= 2) {
        const int cb4 = w - 2;
        init_bias(acc1, A.b4, cb4, lane);
        gemm<RB, 1, N3>(acc1, Abuf, SA, A.wF4, cb4, lane);
        const float w5 = A.w5[cb4 * 32 + col];
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                float s, co;
                act_sincos(w0 * acc1[rb][0][i], &s, &co);
                const int row = rb * 32 + acc_row(i, hh);
                Ebuf[row * SE + cb4 * 32 + col] = s;
                Bbuf[row * SA + cb4 * 32 + col] = (w5 * co) * w0;
            }
    }
    SDF_SYNC();
    // ---- df = W5 h4 + b5 (one thread per row)
    float df = 0.0f;
    if (tid < M) {
        float acc = 0.0f;
        for (int n = 0; n < N4; ++n) acc += A.w5[n] * Ebuf[tid * SE + n];
        df = acc + A.b5;
    }
    // ---- b4: delta3 = ((delta4 W4) * cos t3) * w0        -> Abuf   [M x 128]
    zero(acc1);
    gemm<RB, 1, N4>(acc1, Bbuf, SA, A.wB4, w, lane);
    act_bwd(acc1, d3, Abuf, SA, w0, w, lane);
    SDF_SYNC();
    // ---- b3: delta2 = ((delta3 W3h) * cos t2) * w0     -> Bbuf   [M x 256]
    //          d e  (partial) = delta3 W3e                (regs, waves 0..2)
    //          d z  (partial) = delta3 W3z                (regs, optional)
    zero(acc2);
    gemm<RB, 2, N3>(acc2, Abuf, SA, A.wB3, w, lane);
    act_bwd(acc2, d2, Bbuf, SA, w0, w, lane);
    // d e = delta3 W3e (+ delta1 W1e below), [M x 96]: K-split so every wave does the same MFMA count:
    // waves 0..2 own column block w over groups [0, 3G/4), wave 3 all three blocks over [3G/4, G)
    f32x16 de[RB][1], de3[RB][3];
    zero(de);
    if (w < 3) {
        gemm<RB, 1, N3, 4, 0, 3 * N3 / 32>(de, Abuf, SA, A.wB3e, w, lane);
    } else {
        zero(de3);
        gemm<RB, 3, N3, 1, 3 * N3 / 32, N3 / 8>(de3, Abuf, SA, A.wB3e, 0, lane);
    }
    f32x16 dz[RB][1];
    if constexpr (LATENT_GRAD) {
        zero(dz);
        gemm<RB, 1, N3>(dz, Abuf, SA, A.wB3z, w, lane);
    }
    SDF_SYNC();
    // ---- b2: delta1 = ((delta2 W2) * cos t1) * w0      -> Abuf   [M x 256]
    zero(acc2);
    gemm<RB, 2, N2>(acc2, Bbuf, SA, A.wB2, w, lane);
    act_bwd(acc2, d1, Abuf, SA, w0, w, lane);
    SDF_SYNC();
    // ---- b1: d e += delta1 W1e (same K-split) ; d z += delta1 W1z
    if (w < 3) gemm<RB, 1, N1, 4, 0, 3 * N1 / 32>(de, Abuf, SA, A.wB1e, w, lane);
    else gemm<RB, 3, N1, 1, 3 * N1 / 32, N1 / 8>(de3, Abuf, SA, A.wB1e, 0, lane);
    if constexpr (LATENT_GRAD) {
        gemm<RB, 1, N1>(dz, Abuf, SA, A.wB1z, w, lane);
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int r = row0 + rb * 32 + acc_row(i, hh);
                if (r < A.rows) A.grad_latent[(size_t)r * L + w * 32 + col] = dz[rb][0][i];
            }
    }
    // ---- wave 3 hands its K-slice of d e to the owners of the column blocks (through Abuf)
    SDF_SYNC();  // everyone is done reading delta1 in Abuf
    if (w == 3) {
#pragma unroll
        for (int c = 0; c < 3; ++c)
#pragma unroll
            for (int rb = 0; rb < RB; ++rb)
#pragma unroll
                for (int i = 0; i < 16; ++i) Abuf[(rb * 32 + acc_row(i, hh)) * SA + c * 32 + col] = de3[rb][c][i];
    }
    SDF_SYNC();
    if (w < 3) {
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int i = 0; i < 16; ++i) de[rb][0][i] += Abuf[(rb * 32 + acc_row(i, hh)) * SA + w * 32 + col];
    }
    // ---- embedding backward: grad_c = sum_m (d e_m * g_m) * P[m][c]  (+ d e_c for m < 3)
    //      partials per (row, c, m) -> Ebuf..Bbuf (contiguous, both free), then one thread per
    //      (row, c) sums over m
    // rows of NE + 1 floats: the summing threads (one per (row, c), reading along m) then hit 32 distinct
    // banks; at NE = 96 = 0 mod 32 every lane of a read would share one bank (32-way)
    constexpr int NR = NE + 1;
    static_assert(SE + SA >= 3 * NR, "reduction area");
    float* red = Ebuf;  // [M][3][NR]
    if (w < 3) {
        const int m = w * 32 + col;
#pragma unroll
        for (int rb = 0; rb < RB; ++rb)
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                const int row = rb * 32 + acc_row(i, hh);
                const float u = de[rb][0][i] * gemb[rb][0][i];
                float v0, v1, v2;
                if (m < 3) {
                    v0 = (m == 0) ? u : 0.0f;
                    v1 = (m == 1) ? u : 0.0f;
                    v2 = (m == 2) ? u : 0.0f;
                } else {
                    v0 = u * ptab.x;
                    v1 = u * ptab.y;
                    v2 = u * ptab.z;
                }
                red[(row * 3 + 0) * NR + m] = v0;
                red[(row * 3 + 1) * NR + m] = v1;
                red[(row * 3 + 2) * NR + m] = v2;
            }
    }
    SDF_SYNC();
    if (tid < 3 * M) {
        const float* src = red + tid * NR;
        float s = 0.0f;
        for (int m = 0; m < NE; ++m) s += src[m];
        posb[(tid / 3) * 4 + 1 + tid % 3] = s;
    }
    SDF_SYNC();
    if (tid < M && row0 + tid < A.rows) {
        const int r = row0 + tid;
        const float g0 = posb[tid * 4 + 1], g1 = posb[tid * 4 + 2], g2 = posb[tid * 4 + 3];
        A.out[r] = make_float4(df, g0, g1, g2);
        if (A.h) {  // sdf row of the constraint vector and its Jacobian (gen_model.py:46-61)
            const double* pr = A.p + (size_t)r * A.np;
            const double flag = pr[0];
            const double* R = pr + 4;  // W_R_Co row-major (== casadi reshape((3,3)).T)
            A.h[(size_t)r * 3 + 2] = flag * (double)df + (1.0 - flag) * A.max_df;
            double* J = A.Jh + (size_t)r * 30 + 2;
#pragma unroll
            for (int j = 0; j < 10; ++j)
                J[j * 3] = (j < 3) ? flag * (((double)g0 * R[j * 3 + 0] + (double)g1 * R[j * 3 + 1]) + (double)g2 * R[j * 3 + 2])
                                   : 0.0;
        }
    }
}

// c13[i] = [W1[:, E:] z_i + b1 | W3[:, N2+E:] z_i + b3]   (latent hoisting, per instance)
// A [n_inst x L] . [L x C13_STRIDE] GEMM on the same fp32 MFMA: workgroup (ib, jb) = 32 instances x
// 128 output columns, one 32-column block per wave; bias as the initial accumulator.
// z_i = (float) latent source (fp64 stage parameters at a stride, or an fp32 array).
template <typename T>
__global__ __launch_bounds__(256) void sdf_hoist_kernel(HoistArgs<T> A) {
    __shared__ __align__(16) float z[HOIST_ROWS * SZ];
    const int i0 = blockIdx.x * HOIST_ROWS;
    for (int t = threadIdx.x; t < HOIST_ROWS * L; t += blockDim.x) {
        const int ii = t / L, k = t % L;
        const int inst = i0 + ii < A.n_inst ? i0 + ii : A.n_inst - 1;
        z[ii * SZ + k] = (float)A.latent[(size_t)inst * A.stride + k];
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int cb = blockIdx.y * (HOIST_COLS / 32) + w;  // global 32-column block
    f32x16 acc[1][1];
    init_bias<1, 1>(acc, A.bias, cb, lane);
    gemm<1, 1, L>(acc, z, SZ, A.wpk, cb, lane);
    const int col = cb * 32 + (lane & 31), hh = lane >> 5;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int inst = i0 + acc_row(i, hh);
        if (inst < A.n_inst) A.c13[(size_t)inst * C13_STRIDE + col] = acc[0][0][i];
    }
}

// ------------------------------------------------------------------------------------------------
size_t sdf_lds_bytes(int M) { return (size_t)M * (SE + 2 * SA + 4) * sizeof(float) + (size_t)M * sizeof(int); }

hipError_t launch_sdf_mlp(const SdfArgs& a, int M, bool latent_grad, hipStream_t s) {
    if (a.rows <= 0) return hipSuccess;
    const size_t lds = sdf_lds_bytes(M);
    const dim3 grid((a.rows + M - 1) / M), block(256);
    if (M == 32 && !latent_grad) hipLaunchKernelGGL((sdf_mlp_kernel<32, false>), grid, block, lds, s, a);
    else if (M == 32 && latent_grad) hipLaunchKernelGGL((sdf_mlp_kernel<32, true>), grid, block, lds, s, a);
    else if (M == 64 && !latent_grad) hipLaunchKernelGGL((sdf_mlp_kernel<64, false>), grid, block, lds, s, a);
    else if (M == 64 && latent_grad) hipLaunchKernelGGL((sdf_mlp_kernel<64, true>), grid, block, lds, s, a);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t sdf_set_lds_limits() {
    hipError_t e = hipSuccess;
    const void* ks[4] = {(const void*)sdf_mlp_kernel<32, false>, (const void*)sdf_mlp_kernel<32, true>,
                         (const void*)sdf_mlp_kernel<64, false>, (const void*)sdf_mlp_kernel<64, true>};
    const int Ms[4] = {32, 32, 64, 64};
    for (int i = 0; i < 4; ++i) {
        hipError_t r = hipFuncSetAttribute(ks[i], hipFuncAttributeMaxDynamicSharedMemorySize, (int)sdf_lds_bytes(Ms[i]));
        if (r != hipSuccess) e = r;
    }
    return e;
}

template <typename T>
hipError_t launch_hoist(const HoistArgs<T>& a, hipStream_t s) {
    if (a.n_inst <= 0) return hipSuccess;
    static_assert(C13_STRIDE % HOIST_COLS == 0, "hoist column split");
    hipLaunchKernelGGL((sdf_hoist_kernel<T>), dim3((a.n_inst + HOIST_ROWS - 1) / HOIST_ROWS, C13_STRIDE / HOIST_COLS),
                       dim3(256), 0, s, a);
    return hipGetLastError();
}
template hipError_t launch_hoist<float>(const HoistArgs<float>&, hipStream_t);
template hipError_t launch_hoist<double>(const HoistArgs<double>&, hipStream_t);

}  // namespace sdfn
