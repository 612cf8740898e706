// NeuralDF value + full 1x131 input gradient for a handful of rows: the latency path of the CasADi
// external (config C2: acados calls sdf_l4c / jac_sdf_l4c one shooting node at a time, gen_model.py:
// 39,60).  The batched kernel (sdf_mlp.hip) tiles 32 rows per workgroup and hoists the latent per
// instance -- at one row it is a single workgroup walking ~1.5 MB of weights through a 3-deep register
// ring, latency-bound at ~60 us.  Here one 512-thread workgroup per row keeps each layer's weights in
// flight at once:
//   forward  a = W in + b   threads own outputs and K-slices of the transposed weights W^T: coalesced
//                           loads, no cross-lane reduction;  h = sin(w0 a), cos(w0 a) kept in LDS
//   backward d_in = W^T d   waves own input rows j, lanes own columns k and accumulate over j, one LDS
//                           reduction over the 8 waves -- W read row-major (coalesced across lanes)
// At one row the kernel is a chain of 8 dependent layers, each a few L2 / MALL round trips: ~23 us on
// MI355X, against ~60 us for the batched kernel at one row.
// Reference semantics: PositionEmbedding (embeddings.py:106-111), NeuralDF.forward (neural_df.py:
// 91-103), Sine (activation.py:12-13) and the reverse-mode input gradient L4CasADi's jac_sdf_l4c
// returns; the arithmetic of the embedding and its derivative is sdf_mlp.hip's / sdf_wide.hip's.
#include <hip/hip_runtime.h>

#include "sdf_kernels.h"
#include "sincos.h"

namespace sdfn {

namespace {

constexpr int RW = 8;             // waves per row workgroup
constexpr int C1 = E + L;         // W1 row length (211)
constexpr int C3 = N2 + E + L;    // W3 row length (467)

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

// A layer at one row is a GEMV over ~0.25 MB of L2/MALL-resident weights: its time is the memory
// latency unless every load of the layer is in flight at once.  Both directions therefore give each
// thread one float4 column quad and a slice of the reduction dimension, issue the slice's loads
// back to back into registers (up to 32 float4 = 128 VGPRs), then reduce; the slices' partial sums
// meet in LDS (`part`).  Addresses are clamped and the padding multiplied by 0 (no divergent branch).

// out[j] = bias[j] + W[j][:K] . in  for j < J, from the transposed copy WT [K][J] (row k of WT: the
// k-th input's weights of every output, 16-byte aligned): thread t owns outputs 4q..4q+3, q = t % (J/4),
// over the K-slice t / (J/4)
template <int J, int K>
__device__ __forceinline__ void fwd(const float* __restrict__ WT, const float* __restrict__ bias, const float* in,
                                    float* part, float* out) {
    constexpr int Q = J / 4, S = 64 * RW / Q, KS = (K + S - 1) / S;
    static_assert(J % 4 == 0 && S >= 1 && S * Q == 64 * RW, "J / 4 must divide the workgroup");
    const int t = threadIdx.x, q = t % Q, s = t / Q, k0 = s * KS;
    const float4* W4 = (const float4*)WT;
    float4 w[KS];
#pragma unroll
    for (int i = 0; i < KS; ++i) {
        const int k = k0 + i < K ? k0 + i : K - 1;
        w[i] = W4[(size_t)k * Q + q];
    }
    float4 a = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int i = 0; i < KS; ++i) {
        const int k = k0 + i;
        const float x = (k < K ? 1.0f : 0.0f) * in[k < K ? k : 0];
        a.x = fmaf(w[i].x, x, a.x);
        a.y = fmaf(w[i].y, x, a.y);
        a.z = fmaf(w[i].z, x, a.z);
        a.w = fmaf(w[i].w, x, a.w);
    }
    *(float4*)(part + s * J + 4 * q) = a;
    __syncthreads();
    if (t < J) {
        float v = 0.0f;
#pragma unroll
        for (int r = 0; r < S; ++r) v += part[r * J + t];
        out[t] = v + bias[t];
    }
}

// out[k] = sum_j W[j][k] d[j]  for k < K (W row-major [J][K4], rows padded to K4 = 4 ceil(K / 4)):
// thread t owns columns 4q..4q+3, q = t % (K4/4), over the row slice t / (K4/4) (threads past the last
// whole slice idle)
template <int J, int K>
__device__ __forceinline__ void bwd(const float* __restrict__ W, const float* d, float* part, float* out) {
    constexpr int K4 = (K + 3) / 4 * 4, Q = K4 / 4, S = 64 * RW / Q, JS = (J + S - 1) / S;
    static_assert(S >= 1, "K too wide for the workgroup");
    const int t = threadIdx.x, q = t % Q, s = t / Q, j0 = s * JS;
    const bool act = s < S;
    const float4* W4 = (const float4*)W;
    float4 w[JS];
#pragma unroll
    for (int i = 0; i < JS; ++i) {
        const int j = (act && j0 + i < J) ? j0 + i : 0;
        w[i] = W4[(size_t)j * Q + q];
    }
    float4 a = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
    for (int i = 0; i < JS; ++i) {
        const int j = j0 + i;
        const bool in = act && j < J;
        const float x = (in ? 1.0f : 0.0f) * d[in ? j : 0];
        a.x = fmaf(w[i].x, x, a.x);
        a.y = fmaf(w[i].y, x, a.y);
        a.z = fmaf(w[i].z, x, a.z);
        a.w = fmaf(w[i].w, x, a.w);
    }
    if (act) *(float4*)(part + s * K4 + 4 * q) = a;
    __syncthreads();
    for (int k = t; k < K; k += 64 * RW) {
        float v = 0.0f;
#pragma unroll
        for (int r = 0; r < S; ++r) v += part[r * K4 + k];
        out[k] = v;
    }
    __syncthreads();
}

}  // namespace

__global__ __launch_bounds__(64 * RW) void sdf_row_kernel(SdfRowArgs A) {
    const int r = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __shared__ float in1[C1], in3[C3], gm[NE];             // [e | z], [h2 | e | z], d e / d xb
    __shared__ float a1[N1], c1[N1], a2[N2], c2[N2], a3[N3], c3[N3], a4[N4], c4[N4], h3[N3], h4[N4];
    __shared__ float g1[C1], g3[C3];
    __shared__ __align__(16) float part[RW * (C3 + 1)];
    __shared__ float red[4];
    const float w0 = A.w0;
    float4 p;
    if (A.x) {  // Co_p_B = W_R_Co^T (W_p_B - W_p_Co) in fp64, handed over as fp32 (sdf_mlp_kernel's)
        const double* xr = A.x + (size_t)r * 10;
        const double* pr = A.p + (size_t)r * A.np;
        const double* R = pr + 4;
        const double e0 = xr[0] - pr[1], e1 = xr[1] - pr[2], e2 = xr[2] - pr[3];
        p = make_float4((float)((e0 * R[0] + e1 * R[3]) + e2 * R[6]), (float)((e0 * R[1] + e1 * R[4]) + e2 * R[7]),
                        (float)((e0 * R[2] + e1 * R[5]) + e2 * R[8]), 0.0f);
    } else {
        p = A.pos[r];
    }
    // ---- embedding (e = [x, sin(xb), sin(xb + pi/2)], sdf_wide.hip's arithmetic) and the latent
    for (int m = threadIdx.x; m < NE; m += 64 * RW) {
        float e = 0.0f, g = 0.0f;
        if (m < 3) {
            e = m == 0 ? p.x : (m == 1 ? p.y : p.z);
            g = 1.0f;
        } else if (m < E) {
            const float4 t = A.emb_tab[m];
            float xb = p.x * t.x + p.y * t.y + p.z * t.z;
            if (m >= 3 + EMB_NB) xb = xb + 1.57079637050628662109375f;
            sdfn_sincosf(xb, &e, &g);
        }
        gm[m] = g;
        if (m < E) {
            in1[m] = e;
            in3[N2 + m] = e;
        }
    }
    for (int k = threadIdx.x; k < L; k += 64 * RW) {
        const float z = A.zd ? (float)A.zd[(size_t)(r / A.rows_per_inst) * A.zstride + k] : A.latent[(size_t)r * L + k];
        in1[E + k] = z;
        in3[N2 + E + k] = z;
    }
    __syncthreads();
    // ---- forward
    fwd<N1, C1>(A.W1T, A.b1, in1, part, a1);
    __syncthreads();
    for (int j = threadIdx.x; j < N1; j += 64 * RW) {
        float s, c;
        sdfn_sincosf(w0 * a1[j], &s, &c);
        a1[j] = s;  // h1
        c1[j] = c;
    }
    __syncthreads();
    fwd<N2, N1>(A.W2T, A.b2, a1, part, a2);
    __syncthreads();
    for (int j = threadIdx.x; j < N2; j += 64 * RW) {
        float s, c;
        sdfn_sincosf(w0 * a2[j], &s, &c);
        in3[j] = s;  // h2
        c2[j] = c;
    }
    __syncthreads();
    fwd<N3, C3>(A.W3T, A.b3, in3, part, a3);
    __syncthreads();
    for (int j = threadIdx.x; j < N3; j += 64 * RW) {
        float s, c;
        sdfn_sincosf(w0 * a3[j], &s, &c);
        h3[j] = s;
        c3[j] = c;
    }
    __syncthreads();
    fwd<N4, N3>(A.W4T, A.b4, h3, part, a4);
    __syncthreads();
    for (int j = threadIdx.x; j < N4; j += 64 * RW) {
        float s, c;
        sdfn_sincosf(w0 * a4[j], &s, &c);
        h4[j] = s;
        c4[j] = c;
    }
    __syncthreads();
    if (wave == 0) {
        const float v = wave_sum(lane < N4 ? A.w5[lane] * h4[lane] : 0.0f);
        if (lane == 0) red[0] = v + A.b5;
    }
    // ---- backward: delta_a = (delta_h * cos(w0 a)) * w0 (torch SinBackward then MulBackward)
    for (int j = threadIdx.x; j < N4; j += 64 * RW) a4[j] = (A.w5[j] * c4[j]) * w0;
    __syncthreads();
    bwd<N4, N3>(A.W4, a4, part, h3);             // d h3
    for (int j = threadIdx.x; j < N3; j += 64 * RW) a3[j] = (h3[j] * c3[j]) * w0;
    __syncthreads();
    bwd<N3, C3>(A.W3, a3, part, g3);             // [d h2 | d e | d z]
    for (int j = threadIdx.x; j < N2; j += 64 * RW) a2[j] = (g3[j] * c2[j]) * w0;
    __syncthreads();
    bwd<N2, N1>(A.W2, a2, part, a1);             // d h1
    for (int j = threadIdx.x; j < N1; j += 64 * RW) a1[j] = (a1[j] * c1[j]) * w0;
    __syncthreads();
    bwd<N1, C1>(A.W1, a1, part, g1);             // [d e | d z]
    // ---- outputs: df, d df / d pos (through the embedding), d df / d latent
    if (A.grad_latent)
        for (int k = threadIdx.x; k < L; k += 64 * RW) A.grad_latent[(size_t)r * L + k] = g3[N2 + E + k] + g1[E + k];
    if (wave == 0) {
        float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f;
        for (int m = lane; m < E; m += 64) {
            const float u = (g3[N2 + m] + g1[m]) * gm[m];
            if (m < 3) {
                s0 += m == 0 ? u : 0.0f;
                s1 += m == 1 ? u : 0.0f;
                s2 += m == 2 ? u : 0.0f;
            } else {
                const float4 t = A.emb_tab[m];
                s0 = fmaf(u, t.x, s0);
                s1 = fmaf(u, t.y, s1);
                s2 = fmaf(u, t.z, s2);
            }
        }
        s0 = wave_sum(s0);
        s1 = wave_sum(s1);
        s2 = wave_sum(s2);
        if (lane == 0) {
            const float df = red[0];
            A.out[r] = make_float4(df, s0, s1, s2);
            if (A.h) {  // sdf row of the constraint vector and its Jacobian (gen_model.py:46-61), as sdf_mlp_kernel
                const double* pr = A.p + (size_t)r * A.np;
                const double flag = pr[0];
                const double* R = pr + 4;  // W_R_Co row-major (== casadi reshape((3,3)).T)
                A.h[(size_t)r * 3 + 2] = flag * (double)df + (1.0 - flag) * A.max_df;
                double* J = A.Jh + (size_t)r * 30 + 2;
#pragma unroll
                for (int j = 0; j < 10; ++j)
                    J[j * 3] = (j < 3) ? flag * (((double)s0 * R[j * 3 + 0] + (double)s1 * R[j * 3 + 1]) +
                                                 (double)s2 * R[j * 3 + 2])
                                       : 0.0;
            }
        }
    }
}

hipError_t launch_sdf_row(const SdfRowArgs& a, hipStream_t s) {
    if (a.rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(sdf_row_kernel, dim3((unsigned)a.rows), dim3(64 * RW), 0, s, a);
    return hipGetLastError();
}

}  // namespace sdfn
