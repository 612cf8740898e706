// NeuralDF value + full 1x131 input gradient for a handful of rows: the latency path of the CasADi
// external (config C2: acados calls sdf_l4c / jac_sdf_l4c one shooting node at a time, gen_model.py:
// 39,60).  The batched kernel (sdf_mlp.hip) tiles 32 rows per workgroup and hoists the latent per
// instance -- at one row it is a single workgroup walking ~1.5 MB of weights through a 3-deep register
// ring, latency-bound at ~60 us.  Here one 512-thread workgroup per row keeps each layer's weights in
// flight at once:
//   forward  a = W in + b   threads own outputs and K-slices of the transposed weights W^T: coalesced
//                           loads, no cross-lane reduction;  h = sin(w0 a), cos(w0 a) kept in LDS
//   backward d_in = W^T d   from the same transposed copy: lanes split each row of W^T, a DPP group sum
//                           per row (each layer's weights are streamed once per call)
// At one row the kernel is a chain of 8 dependent layers, each a few L2 / MALL round trips: ~23 us on
// MI355X, against ~60 us for the batched kernel at one row.
// Reference semantics: PositionEmbedding (embeddings.py:106-111), NeuralDF.forward (neural_df.py:
// 91-103), Sine (activation.py:12-13) and the reverse-mode input gradient L4CasADi's jac_sdf_l4c
// returns; the arithmetic of the embedding and its derivative is sdf_mlp.hip's / sdf_wide.hip's.
#include <hip/hip_runtime.h>

#include <type_traits>

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
// The weight pointer of a layer is laundered at the layer: in the resident server's request loop the
// compiler would otherwise issue every layer's weight loads up front (or hoist them out of the loop)
// and spill them to scratch.
template <typename T>
__device__ __forceinline__ const T* launder(const T* p) {
    asm volatile("" : "+s"(p));
    return p;
}

// threadIdx.x behind an opaque copy: in the server's request loop the compiler would otherwise hoist
// every lane-dependent index and address of the evaluation out of the loop and spill them
__device__ __forceinline__ int tix() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

template <int J, int K>
__device__ __forceinline__ void fwd(const float* __restrict__ WT_, const float* __restrict__ bias, const float* in,
                                    float* part, float* out) {
    const float* __restrict__ WT = launder(WT_);
    constexpr int Q = J / 4, S = 64 * RW / Q, KS = (K + S - 1) / S;
    static_assert(J % 4 == 0 && S >= 1 && S * Q == 64 * RW, "J / 4 must divide the workgroup");
    const int t = tix(), q = t % Q, s = t / Q, k0 = s * KS;
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

// sum over aligned groups of QR lanes (QR = 4, 8 or 16, inside one DPP row), every lane of a group
// receiving the group's sum: quad butterflies, then the half-row and row mirrors
template <int QR>
__device__ __forceinline__ float group_sum(float v) {
    static_assert(QR == 4 || QR == 8 || QR == 16, "group of 4, 8 or 16 lanes");
    auto dpp = [](float x, auto ctrl) {
        constexpr int C = decltype(ctrl)::value;
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), C, 0xf, 0xf, false));
    };
    v += dpp(v, std::integral_constant<int, 0xB1>{});  // quad_perm [1, 0, 3, 2]
    v += dpp(v, std::integral_constant<int, 0x4E>{});  // quad_perm [2, 3, 0, 1]
    if constexpr (QR >= 8) v += dpp(v, std::integral_constant<int, 0x141>{});  // row_half_mirror
    if constexpr (QR >= 16) v += dpp(v, std::integral_constant<int, 0x140>{});  // row_mirror
    return v;
}

// out[k] = sum_j W[j][k] d[j] for k < K from the TRANSPOSED copy WT [K][J] (the forward's operand, so
// one copy of the weights serves both directions): QR = J / 16 lanes share row k of WT, lane q loading
// its float4 columns q, q + QR, q + 2 QR, q + 3 QR (each load instruction contiguous per row); a wave covers 64 / QR rows per group of loads and its
// ceil(K / RW) rows in NG groups, all loads in flight at once; the QR partial dot products meet in a
// DPP group sum.  d must be 16-byte aligned.
template <int J, int K>
__device__ __forceinline__ void bwd_t(const float* __restrict__ WT_, const float* d, float* out) {
    const float* __restrict__ WT = launder(WT_);
    constexpr int QR = J / 16, G = 64 / QR, RPW = (K + RW - 1) / RW, NG = (RPW + G - 1) / G;
    static_assert(J % 64 == 0, "J must be a multiple of 64");
    const int lane = tix() & 63, wave = tix() >> 6, sub = lane / QR, qq = lane % QR;
    const float4* W4 = (const float4*)WT;
    float4 w[NG][4];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const int i = g * G + sub, k = wave * RPW + i;
        const int kk = (i < RPW && k < K) ? k : K - 1;
#pragma unroll
        for (int c = 0; c < 4; ++c) w[g][c] = W4[(size_t)kk * (J / 4) + c * QR + qq];  // QR lanes: contiguous
    }
    float4 dv[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) dv[c] = *(const float4*)(d + 4 * (c * QR + qq));
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        float a = 0.0f;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
            a = fmaf(w[g][c].x, dv[c].x, a);
            a = fmaf(w[g][c].y, dv[c].y, a);
            a = fmaf(w[g][c].z, dv[c].z, a);
            a = fmaf(w[g][c].w, dv[c].w, a);
        }
        a = group_sum<QR>(a);
        const int i = g * G + sub, k = wave * RPW + i;
        if (qq == 0 && i < RPW && k < K) out[k] = a;
    }
    __syncthreads();
}

}  // namespace

// diagnostics: wall-clock stamp of phase i by thread 0 (after a barrier) when A.stamps is set (the server)
#define ROW_STAMP(i)                                                  \
    do {                                                              \
        if (A.stamps && tix() == 0)                                   \
            __hip_atomic_store(A.stamps + (i), (long long)wall_clock64(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); \
    } while (0)

// value + gradient of row r by the whole (64 RW)-thread workgroup; shared by the per-call kernel and the
// resident server (A.pos / A.latent may point into LDS there)
__device__ __forceinline__ void row_eval(const SdfRowArgs& A, const int r) {
    const int lane = tix() & 63, wave = tix() >> 6;
    __shared__ float in1[C1], in3[C3], gm[NE];             // [e | z], [h2 | e | z], d e / d xb
    __shared__ __align__(16) float a1[N1], a2[N2], a3[N3], a4[N4];  // 16-byte aligned: bwd_t reads float4
    __shared__ float c1[N1], c2[N2], c3[N3], c4[N4], h3[N3], h4[N4];
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
    for (int m = tix(); m < NE; m += 64 * RW) {
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
    for (int k = tix(); k < L; k += 64 * RW) {
        const float z = A.zd ? (float)A.zd[(size_t)(r / A.rows_per_inst) * A.zstride + k] : A.latent[(size_t)r * L + k];
        in1[E + k] = z;
        in3[N2 + E + k] = z;
    }
    __syncthreads();
    ROW_STAMP(0);
    // ---- forward
    fwd<N1, C1>(A.W1T, A.b1, in1, part, a1);
    __syncthreads();
    ROW_STAMP(1);
    for (int j = tix(); j < N1; j += 64 * RW) {
        float s, c;
        sdfn_sincosf(w0 * a1[j], &s, &c);
        a1[j] = s;  // h1
        c1[j] = c;
    }
    __syncthreads();
    ROW_STAMP(2);
    fwd<N2, N1>(A.W2T, A.b2, a1, part, a2);
    __syncthreads();
    ROW_STAMP(3);
    for (int j = tix(); j < N2; j += 64 * RW) {
        float s, c;
        sdfn_sincosf(w0 * a2[j], &s, &c);
        in3[j] = s;  // h2
        c2[j] = c;
    }
    __syncthreads();
    ROW_STAMP(4);
    fwd<N3, C3>(A.W3T, A.b3, in3, part, a3);
    __syncthreads();
    ROW_STAMP(5);
    for (int j = tix(); j < N3; j += 64 * RW) {
        float s, c;
        sdfn_sincosf(w0 * a3[j], &s, &c);
        h3[j] = s;
        c3[j] = c;
    }
    __syncthreads();
    ROW_STAMP(6);
    fwd<N4, N3>(A.W4T, A.b4, h3, part, a4);
    __syncthreads();
    ROW_STAMP(7);
    for (int j = tix(); j < N4; j += 64 * RW) {
        float s, c;
        sdfn_sincosf(w0 * a4[j], &s, &c);
        h4[j] = s;
        c4[j] = c;
    }
    __syncthreads();
    ROW_STAMP(8);
    if (wave == 0) {
        const float v = wave_sum(lane < N4 ? A.w5[lane] * h4[lane] : 0.0f);
        if (lane == 0) red[0] = v + A.b5;
    }
    // ---- backward: delta_a = (delta_h * cos(w0 a)) * w0 (torch SinBackward then MulBackward)
    for (int j = tix(); j < N4; j += 64 * RW) a4[j] = (A.w5[j] * c4[j]) * w0;
    __syncthreads();
    bwd_t<N4, N3>(A.W4T, a4, h3);             // d h3
    ROW_STAMP(9);
    for (int j = tix(); j < N3; j += 64 * RW) a3[j] = (h3[j] * c3[j]) * w0;
    __syncthreads();
    bwd_t<N3, C3>(A.W3T, a3, g3);             // [d h2 | d e | d z]
    ROW_STAMP(10);
    for (int j = tix(); j < N2; j += 64 * RW) a2[j] = (g3[j] * c2[j]) * w0;
    __syncthreads();
    bwd_t<N2, N1>(A.W2T, a2, a1);             // d h1
    ROW_STAMP(11);
    for (int j = tix(); j < N1; j += 64 * RW) a1[j] = (a1[j] * c1[j]) * w0;
    __syncthreads();
    bwd_t<N1, C1>(A.W1T, a1, g1);             // [d e | d z]
    ROW_STAMP(12);
    // ---- outputs: df, d df / d pos (through the embedding), d df / d latent
    if (A.grad_latent)
        for (int k = tix(); k < L; k += 64 * RW) A.grad_latent[(size_t)r * L + k] = g3[N2 + E + k] + g1[E + k];
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

__global__ __launch_bounds__(64 * RW) void sdf_row_kernel(SdfRowArgs A) { row_eval(A, blockIdx.x); }


// system-scope (host-coherent) accesses of the mailbox: vector loads / stores that bypass the GPU caches
__device__ __forceinline__ unsigned long long mb_load(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned int mb_load_u32(const unsigned int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void mb_store(long long* p, long long v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The resident server (SdfMbox, sdf_kernels.h): thread 0 polls seq_in; the request is staged into LDS
// with one PCIe read per word; the rows are evaluated by row_eval with the outputs written straight into
// the mailbox; after a system-scope fence seq_out publishes them.  Every exit path (stop, idle, life) is
// taken by the whole workgroup together (the decision goes through LDS behind a barrier), between
// requests, and ends with the launch's epoch stored to `gone`, so a caller that posted a request the
// leaving server did not see relaunches at once instead of waiting for the stream to drain.  The life
// bound (0.8 ms by default) is what a device-wide synchronisation elsewhere in the process can wait.
__global__ __launch_bounds__(64 * RW) void sdf_server_kernel(SdfRowArgs A, SdfMbox* mb, long long idle,
                                                              long long life, unsigned long long epoch) {
    __shared__ __align__(16) float s_in[SDF_ROW_MAX * (4 + L)], s_out[SDF_ROW_MAX * (4 + L)];
    __shared__ unsigned long long s_seq;
    __shared__ int s_go, s_rows, s_grad;
    const long long t0 = wall_clock64();
    long long last = t0;
    unsigned long long done = 0;
    if (threadIdx.x == 0) done = mb_load(&mb->seq_out);
    for (;;) {
        if (threadIdx.x == 0) {
            int go = 0;
            unsigned long long q = done;
            for (;;) {
                q = mb_load(&mb->seq_in);
                if (q != done) {
                    go = 1;
                    break;
                }
                const long long now = wall_clock64();
                if (mb_load(&mb->stop) || now - last > idle || now - t0 > life) break;
                __builtin_amdgcn_s_sleep(2);
            }
            s_go = go;
            s_seq = q;
            if (go) {
                const int rows = (int)mb_load_u32((const unsigned int*)&mb->rows);
                s_rows = rows < 1 ? 1 : (rows > SDF_ROW_MAX ? SDF_ROW_MAX : rows);
                s_grad = (int)mb_load_u32((const unsigned int*)&mb->grad);
            }
        }
        __syncthreads();
        if (!s_go) {
            if (threadIdx.x == 0) {
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __hip_atomic_store(&mb->gone, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            break;
        }
        const long long t_seen = wall_clock64();
        const int rows = s_rows;
        for (int i = threadIdx.x; i < rows * (4 + L); i += 64 * RW)
            s_in[i] = __uint_as_float(mb_load_u32((const unsigned int*)mb->in + i));
        __syncthreads();
        const long long t_staged = wall_clock64();
        SdfRowArgs B = A;
        B.pos = (const float4*)s_in;
        B.latent = s_in + rows * 4;
        B.out = (float4*)s_out;  // results go to LDS first, then to the mailbox with write-through stores
        B.grad_latent = s_grad ? s_out + rows * 4 : nullptr;
        B.rows = rows;
        B.x = nullptr;
        B.zd = nullptr;
        B.h = nullptr;
        B.stamps = mb->t_phase;
        for (int r = 0; r < rows; ++r) {
            row_eval(B, r);
            __syncthreads();  // row_eval's LDS is reused by the next row
        }
        const long long t_done = wall_clock64();
        // Publishing without an L2 write-back (__threadfence_system's buffer_wbl2, ~1.7 us each): the
        // results leave with system-scope stores, which write through the GPU caches to host memory; once
        // every wave's stores have completed (vmcnt(0)) and met at the barrier, one lane stores seq_out.
        // (Plain stores would stay in the L2 and the host would read stale results.)
        for (int i = threadIdx.x; i < rows * (s_grad ? 4 + L : 4); i += 64 * RW)
            __hip_atomic_store((unsigned int*)mb->out + i, __float_as_uint(s_out[i]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            mb_store(&mb->t_seen, t_seen);
            mb_store(&mb->t_staged, t_staged);
            mb_store(&mb->t_done, t_done);
            mb_store(&mb->t_phase[13], t_done);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&mb->seq_out, s_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            done = s_seq;
        }
        last = wall_clock64();
    }
}

hipError_t launch_sdf_server(const SdfRowArgs& a, SdfMbox* mb_dev, long long idle_ticks, long long life_ticks,
                             unsigned long long epoch, hipStream_t s) {
    hipLaunchKernelGGL(sdf_server_kernel, dim3(1), dim3(64 * RW), 0, s, a, mb_dev, idle_ticks, life_ticks, epoch);
    return hipGetLastError();
}

hipError_t launch_sdf_row(const SdfRowArgs& a, hipStream_t s) {
    if (a.rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(sdf_row_kernel, dim3((unsigned)a.rows), dim3(64 * RW), 0, s, a);
    return hipGetLastError();
}

}  // namespace sdfn
