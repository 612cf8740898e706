// NeuralDF value + full input gradient at a handful of rows for every network other than the deployed
// one (engine.cpp is_deployed): the CasADi external's latency path (config C2: acados calls sdf_l4c /
// jac_sdf_l4c one shooting node at a time, gen_model.py:39,60) for any layer sizes, embedding, res mode,
// activation and size_latent the reference's NeuralDF accepts (neural_df.py:13-103, embeddings.py:12-111,
// activation.py).  sdf_row.hip does this for the deployed architecture with compile-time shapes; here the
// shapes are the wide schedule's (sdf_wide.hip) and the operands are its row-major [N][K] matrices
// (engine.cpp upload_wide: layer widths padded to multiples of 128, padded units with zero weights).
//
// One 512-thread workgroup per row walks the layers as GEMVs.  Every operand is row-major with K
// contiguous, so a GEMV gives each output row a group of 16 lanes (one DPP row): lane q loads the row's
// float4 chunks q, q + 16, ... (each load instruction of a group contiguous), and a DPP group sum
// reduces them; 32 rows per pass of the workgroup, eight passes x four chunks per lane unrolled so a
// 256 x 256 layer's loads are all in flight at once (at one row a layer is a chain of L2 / MALL round
// trips, as sdf_row.hip explains).  The backward pass uses the transposed copies the wide schedule keeps
// (B4, B3h, B3e, B2, B1e, Bz), so it is the same GEMV.  Each GEMV's epilogue runs on lanes 0..7 of every
// group (its eight rows of the batch at once): the activation (sin(w0 .), ReLU, Softplus with threshold
// 20) and its torch backward factor, wide_gemm_kernel's epilogues element for element.
#include <hip/hip_runtime.h>

#include <atomic>
#include <type_traits>

#include "sdf_kernels.h"
#include "sincos.h"

namespace sdfn {

namespace {

constexpr int WR = 8;           // waves per row workgroup
constexpr int WT = 64 * WR;     // threads
constexpr int GRP = 16;         // lanes per GEMV row
constexpr int RPP = WT / GRP;   // rows per pass
constexpr int U = 8;            // passes whose loads are in flight together
constexpr int CI = 4;           // float4 chunks per lane per batch (U x CI float4 = 128 VGPRs of loads)

// threadIdx.x behind an opaque copy (the server's request loop would otherwise hoist and spill every
// lane-dependent address out of the loop, as in sdf_row.hip)
__device__ __forceinline__ int tix() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}
template <typename T>
__device__ __forceinline__ const T* launder(const T* p) {
    asm volatile("" : "+s"(p));
    return p;
}

// sum over the 16 lanes of a DPP row, every lane receiving it (quad butterflies, half-row and row mirrors)
__device__ __forceinline__ float row16_sum(float v) {
    auto dpp = [](float x, auto ctrl) {
        constexpr int C = decltype(ctrl)::value;
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), C, 0xf, 0xf, false));
    };
    v += dpp(v, std::integral_constant<int, 0xB1>{});
    v += dpp(v, std::integral_constant<int, 0x4E>{});
    v += dpp(v, std::integral_constant<int, 0x141>{});
    v += dpp(v, std::integral_constant<int, 0x140>{});
    return v;
}

__device__ __forceinline__ float dot4(float4 w, float4 x, float a) {
    a = fmaf(w.x, x.x, a);
    a = fmaf(w.y, x.y, a);
    a = fmaf(w.z, x.z, a);
    return fmaf(w.w, x.w, a);
}

// epi(j, W[j][:K1 + K2] . [x1 | x2]) for j < J, the U rows of a group's batch through the epilogue at once (on
// lanes 0..U-1 of the group); W row-major with row stride K1 + K2 (multiples of 4 floats), x1 / x2 16-byte
// aligned in LDS.  Ends with a workgroup barrier.
template <typename Epi>
__device__ __forceinline__ void gemv(const float* W_, int J, const float* x1, int K1, const float* x2, int K2,
                                     Epi&& epi) {
    const float* __restrict__ W = launder(W_);
    const int t = tix(), g = t / GRP, q = t % GRP;
    const int C1 = K1 / 4, C = (K1 + K2) / 4;
    const float4* xa = (const float4*)x1;
    const float4* xb = (const float4*)x2;
    for (int j0 = g; j0 < J; j0 += U * RPP) {
        float a[U];
#pragma unroll
        for (int u = 0; u < U; ++u) a[u] = 0.0f;
        for (int c0 = q; c0 < C; c0 += CI * GRP) {
            // U rows x CI chunks of loads issued back to back (clamped addresses, dead chunks times 0)
            float4 w[U][CI];
#pragma unroll
            for (int u = 0; u < U; ++u) {
                const int j = j0 + u * RPP, jj = j < J ? j : J - 1;  // a dead row re-reads a live one
                const float4* row = (const float4*)(W + (size_t)jj * (K1 + K2));
#pragma unroll
                for (int i = 0; i < CI; ++i) {
                    const int c = c0 + i * GRP;
                    w[u][i] = row[c < C ? c : C - 1];
                }
            }
#pragma unroll
            for (int i = 0; i < CI; ++i) {
                const int c = c0 + i * GRP;
                float4 x = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (c < C) x = c < C1 ? xa[c] : xb[c - C1];
#pragma unroll
                for (int u = 0; u < U; ++u) a[u] = dot4(w[u][i], x, a[u]);
            }
        }
        // every lane of a group gets the U sums; lane q < U takes row j0 + q RPP through the epilogue
        float mine = 0.0f;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const float v = row16_sum(a[u]);
            mine = q == u ? v : mine;
        }
        const int j = j0 + q * RPP;
        if (q < U && j < J) epi(j, mine);
    }
    __syncthreads();
}

// the activation of a pre-activation t and its derivative factor (wide_gemm_kernel's forward epilogue)
__device__ __forceinline__ void act_fd(int act, float w0, float t, float& h, float& d) {
    if (act == 0) {
        sdfn_sincosf(w0 * t, &h, &d);
    } else if (act == 1) {  // torch ReLU; ReluBackward passes where the output is > 0
        h = t > 0.0f ? t : 0.0f;
        d = h > 0.0f ? 1.0f : 0.0f;
    } else {  // torch Softplus(beta 1, threshold 20) and SoftplusBackward: z / (z + 1), z = exp(t)
        const float ez = expf(t);
        h = t > 20.0f ? t : log1pf(ez);
        d = t > 20.0f ? 1.0f : ez / (ez + 1.0f);
    }
}

// LDS layout of one row's evaluation (floats, every block a multiple of 4: 16-byte aligned)
struct RowLds {
    float *e, *gm, *z, *hz, *h1, *d1, *h2, *d2, *h3, *d3, *h4, *d4, *ge3, *ge1, *red;
};
__host__ __device__ inline int r4(int n) { return (n + 3) & ~3; }
__host__ __device__ inline size_t row_lds_floats(const WideRowArgs& a) {
    return 2 * (size_t)r4(a.NEK) + (size_t)a.LZ + (a.P1 + a.P3) + 2 * (size_t)(a.P1 + a.P2 + a.P3 + a.P4) +
           2 * (size_t)a.NEB + 8;
}
__device__ inline RowLds carve(float* q, const WideRowArgs& a) {
    RowLds s;
    auto take = [&](int n) { float* r = q; q += r4(n); return r; };
    s.e = take(a.NEK); s.gm = take(a.NEK); s.z = take(a.LZ); s.hz = take(a.P1 + a.P3);
    s.h1 = take(a.P1); s.d1 = take(a.P1); s.h2 = take(a.P2); s.d2 = take(a.P2);
    s.h3 = take(a.P3); s.d3 = take(a.P3); s.h4 = take(a.P4); s.d4 = take(a.P4);
    s.ge3 = take(a.NEB); s.ge1 = take(a.NEB); s.red = take(8);
    return s;
}

}  // namespace

// value + gradient of row r by the whole workgroup (A.pos / A.latent / A.out may point into LDS)
__device__ __forceinline__ void row_eval_wide(const WideRowArgs& A, const int r, float* lds) {
    const RowLds s = carve(lds, A);
    const int lane = tix() & 63, wave = tix() >> 6;
    const float w0 = A.w0;
    const int act = A.act;
    const float4 p = A.pos[r];
    // ---- embedding e = [x, sin(xb), sin(xb + pi/2)] and its derivative factors (wide_emb_kernel's arithmetic)
    for (int m = tix(); m < A.NEK; m += WT) {
        float e = 0.0f, g = 0.0f;
        if (m < 3) {
            e = m == 0 ? p.x : (m == 1 ? p.y : p.z);
            g = 1.0f;
        } else if (m < 3 + 2 * A.nb) {
            const float4 t = A.emb_tab[m];
            float xb = p.x * t.x + p.y * t.y + p.z * t.z;
            if (m >= 3 + A.nb) xb = xb + 1.57079637050628662109375f;
            sdfn_sincosf(xb, &e, &g);
        }
        s.e[m] = e;
        s.gm[m] = g;
    }
    for (int k = tix(); k < A.LZ; k += WT) s.z[k] = k < A.LH ? A.latent[(size_t)r * A.LH + k] : 0.0f;
    if (!A.e3)
        for (int m = tix(); m < A.NEB; m += WT) s.ge3[m] = 0.0f;
    __syncthreads();
    // ---- the latent's share of layers 1 and 3: hz = [W1z ; W3z] z + [b1 | b3] (the wide schedule's hoist:
    //      its STORE epilogue, acc + bias)
    gemv(A.Hz, A.P1 + A.P3, s.z, A.LZ, nullptr, 0, [&](int j, float v) { s.hz[j] = v + A.bz[j]; });
    // ---- forward, the activation (and its derivative factor) in each GEMV's epilogue
    gemv(A.F1, A.P1, s.e, A.NEK, nullptr, 0, [&](int j, float v) { act_fd(act, w0, v + s.hz[j], s.h1[j], s.d1[j]); });
    gemv(A.F2, A.P2, s.h1, A.P1, nullptr, 0, [&](int j, float v) { act_fd(act, w0, v + A.b2[j], s.h2[j], s.d2[j]); });
    gemv(A.F3, A.P3, s.h2, A.P2, A.e3 ? s.e : nullptr, A.e3 ? A.NEK : 0,
         [&](int j, float v) { act_fd(act, w0, v + s.hz[A.P1 + j], s.h3[j], s.d3[j]); });
    gemv(A.F4, A.P4, s.h3, A.P3, nullptr, 0, [&](int j, float v) {
        float h, d;
        act_fd(act, w0, v + A.b4[j], h, d);
        s.h4[j] = h;
        s.d4[j] = act == 0 ? (A.w5[j] * d) * w0 : A.w5[j] * d;  // delta4 (wide_gemm's SIN_L4 epilogue)
    });
    if (wave == 0) {  // df = w5 . h4 + b5
        float v = 0.0f;
        for (int n = lane; n < A.P4; n += 64) v = fmaf(A.w5[n], s.h4[n], v);
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
        if (lane == 0) s.red[0] = v + A.b5;
    }
    // ---- backward: delta_{l-1} = (W_l^T delta_l) * act'(a_{l-1}) (* w0 for sin): torch's SinBackward then
    //      MulBackward, as wide_gemm's BWD epilogue; deltas overwrite the consumed activations
    auto bwd = [&](float* dl, const float* dv) {
        return [=](int j, float v) {
            const float dd = v * dv[j];
            dl[j] = act == 0 ? dd * w0 : dd;
        };
    };
    gemv(A.B4, A.P3, s.d4, A.P4, nullptr, 0, bwd(s.h3, s.d3));
    gemv(A.B3h, A.P2, s.h3, A.P3, nullptr, 0, bwd(s.h2, s.d2));
    if (A.e3)  // res 'latent' / 'none': layer 3 does not see the embedding (ge3 zeroed with the embedding)
        gemv(A.B3e, A.NEB, s.h3, A.P3, nullptr, 0, [&](int j, float v) { s.ge3[j] = v; });
    gemv(A.B2, A.P1, s.h2, A.P2, nullptr, 0, bwd(s.h1, s.d1));
    gemv(A.B1e, A.NEB, s.h1, A.P1, nullptr, 0, [&](int j, float v) { s.ge1[j] = v; });
    if (A.grad_latent) {  // d df / d z = [delta1 | delta3] . [W1z ; W3z]
        float* gl = A.grad_latent + (size_t)r * A.LH;
        gemv(A.Bz, A.LH, s.h1, A.P1, s.h3, A.P3, [&](int j, float v) { gl[j] = v; });
    }
    // ---- d df / d pos through the embedding (wide_final_kernel's sums, by one wave)
    if (wave == 0) {
        float s0 = 0.0f, s1 = 0.0f, s2 = 0.0f;
        for (int m = lane; m < A.NEK; m += 64) {
            const float u = (s.ge3[m] + s.ge1[m]) * s.gm[m];
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
#pragma unroll
        for (int o = 32; o > 0; o >>= 1) {
            s0 += __shfl_xor(s0, o);
            s1 += __shfl_xor(s1, o);
            s2 += __shfl_xor(s2, o);
        }
        if (lane == 0) A.out[r] = make_float4(s.red[0], s0, s1, s2);
    }
    __syncthreads();
}

__global__ __launch_bounds__(WT) void sdf_row_wide_kernel(WideRowArgs A) {
    extern __shared__ __align__(16) float lds_w[];
    row_eval_wide(A, blockIdx.x, lds_w);
}

// system-scope (host-coherent) mailbox accesses, as sdf_row.hip's server
__device__ __forceinline__ unsigned long long mbw_load(const unsigned long long* p) {
    return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ unsigned int mbw_load_u32(const unsigned int* p) {
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The resident server for these networks: sdf_server_kernel's mailbox protocol (sdf_row.hip) -- poll seq_in,
// stage the request into LDS, evaluate, write the results through to the mailbox, publish seq_out; leave on
// stop, idle or life, storing the launch epoch to `gone` -- with the request in dynamic LDS after the
// evaluator's and at most wide_row_max_rows(LH) rows per request.
__global__ __launch_bounds__(WT) void sdf_server_wide_kernel(WideRowArgs A, SdfMbox* mb, long long idle, long long life,
                                                             unsigned long long epoch) {
    extern __shared__ __align__(16) float lds_w[];
    float* s_in = lds_w + row_lds_floats(A);
    float* s_out = s_in + SDF_MBOX_FLOATS;
    __shared__ unsigned long long s_seq;
    __shared__ int s_go, s_rows, s_grad;
    const long long t0 = wall_clock64();
    long long last = t0;
    unsigned long long done = 0;
    const int LH = A.LH, max_rows = SDF_MBOX_FLOATS / (4 + LH) < SDF_ROW_MAX ? SDF_MBOX_FLOATS / (4 + LH) : SDF_ROW_MAX;
    if (threadIdx.x == 0) done = mbw_load(&mb->seq_out);
    for (;;) {
        if (threadIdx.x == 0) {
            int go = 0;
            unsigned long long q = done;
            for (;;) {
                q = mbw_load(&mb->seq_in);
                if (q != done) {
                    go = 1;
                    break;
                }
                const long long now = wall_clock64();
                if (mbw_load(&mb->stop) || now - last > idle || now - t0 > life) break;
                __builtin_amdgcn_s_sleep(2);
            }
            s_go = go;
            s_seq = q;
            if (go) {
                const int rows = (int)mbw_load_u32((const unsigned int*)&mb->rows);
                s_rows = rows < 1 ? 1 : (rows > max_rows ? max_rows : rows);
                s_grad = (int)mbw_load_u32((const unsigned int*)&mb->grad);
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
        for (int i = threadIdx.x; i < rows * (4 + LH); i += WT)
            s_in[i] = __uint_as_float(mbw_load_u32((const unsigned int*)mb->in + i));
        __syncthreads();
        const long long t_staged = wall_clock64();
        WideRowArgs B = A;
        B.pos = (const float4*)s_in;
        B.latent = s_in + rows * 4;
        B.out = (float4*)s_out;
        B.grad_latent = s_grad ? s_out + rows * 4 : nullptr;
        B.rows = rows;
        for (int r = 0; r < rows; ++r) row_eval_wide(B, r, lds_w);
        const long long t_done = wall_clock64();
        for (int i = threadIdx.x; i < rows * (s_grad ? 4 + LH : 4); i += WT)
            __hip_atomic_store((unsigned int*)mb->out + i, __float_as_uint(s_out[i]), __ATOMIC_RELAXED,
                               __HIP_MEMORY_SCOPE_SYSTEM);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) {
            __hip_atomic_store(&mb->t_seen, t_seen, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&mb->t_staged, t_staged, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            __hip_atomic_store(&mb->t_done, t_done, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __hip_atomic_store(&mb->seq_out, s_seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
            done = s_seq;
        }
        last = wall_clock64();
    }
}

// the dynamic-LDS limit of a kernel, raised once to the largest size asked for so far (the launches on the
// host path are serialised by the context's lock; a race between contexts only repeats the call)
static std::atomic<size_t> lds_row_set{0}, lds_srv_set{0};
static hipError_t raise_lds(const void* k, size_t bytes, std::atomic<size_t>& set) {
    if (bytes <= 64 * 1024 || bytes <= set.load(std::memory_order_relaxed)) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) set.store(bytes, std::memory_order_relaxed);
    return e;
}

size_t wide_row_lds_bytes(const WideRowArgs& a) { return row_lds_floats(a) * sizeof(float); }

int wide_row_max_rows(int LH) {
    const int n = SDF_MBOX_FLOATS / (4 + LH);
    return n < SDF_ROW_MAX ? n : SDF_ROW_MAX;
}

hipError_t launch_sdf_row_wide(const WideRowArgs& a, hipStream_t s) {
    if (a.rows <= 0) return hipSuccess;
    const size_t lds = wide_row_lds_bytes(a);
    hipError_t e = raise_lds((const void*)sdf_row_wide_kernel, lds, lds_row_set);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(sdf_row_wide_kernel, dim3((unsigned)a.rows), dim3(WT), lds, s, a);
    return hipGetLastError();
}

hipError_t launch_sdf_server_wide(const WideRowArgs& a, SdfMbox* mb_dev, long long idle_ticks, long long life_ticks,
                                  unsigned long long epoch, hipStream_t s) {
    const size_t lds = wide_row_lds_bytes(a) + 2 * SDF_MBOX_FLOATS * sizeof(float);
    hipError_t e = raise_lds((const void*)sdf_server_wide_kernel, lds, lds_srv_set);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(sdf_server_wide_kernel, dim3(1), dim3(WT), lds, s, a, mb_dev, idle_ticks, life_ticks, epoch);
    return hipGetLastError();
}

}  // namespace sdfn
