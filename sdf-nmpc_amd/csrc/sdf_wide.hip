// NeuralDF forward + position-Jacobian for WIDE networks (config C5: layer_sizes [1024,1024,512,256]).
//
// Same semantics as sdf_mlp.hip (neural_df.py:91-103, embeddings.py:106-111, reverse mode for
// d df / d pos), different schedule: at these widths one row's activations (up to 2 x 4 KiB per layer)
// and the 8 MiB of weights cannot stay on chip, so the network runs layer by layer as large GEMMs
// over all B x (N+1) rows with the activations in HBM (~24 KB per row) and every weight matrix read
// from L2 once per group of 8 row tiles:
//   wide_latent  z (fp64 stage parameters) -> fp32 [n_inst][L]
//   wide_gemm    hoist  c13 = z [W1z | W3z]^T + [b1 | b3]            (per instance)
//   wide_emb     Co_p_B (fp64 -> fp32), e [R][nek], d e / d xb factors g [R][nek]
//   wide_gemm    L1..L4 forward: act(A W^T + bias / c13) -- sin(w0 .), relu or softplus -- keeping act'
//                for the backward pass
//   wide_gemm    backward: delta_{l-1} = (delta_l W_l) * act' (* w0 for sin), d e = delta3 W3e + delta1 W1e
// The same schedule serves every NeuralDF other than the deployed one (engine.cpp is_deployed): layer
// widths zero-padded to multiples of 128, any embedding (none / pos / cube / oct / dod / ico), res
// full / state / latent (neural_df.py:40-103).
//   wide_final   df = w5 h4 + b5, d df / d pos from d e, and the fused sdf constraint row h[2], J_h
// wide_gemm is an fp32 MFMA (v_mfma_f32_32x32x2_f32, exact fp32 products) GEMM: 128 x 128 tile per
// 256-thread workgroup (2 x 2 waves of 64 x 64), K staged 16 at a time through double-buffered LDS
// (rows padded to 20 floats: conflict-free ds_read_b128), tiles ordered in groups of 8 row tiles so
// the 8 XCDs each keep one row tile while the weight columns stream through their L2.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "sdf_kernels.h"
#include "sincos.h"

namespace sdfn {

typedef float wf32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 wbf16x8 __attribute__((ext_vector_type(8)));

constexpr int WG_BM = 128, WG_BN = 128, WG_BK = 16, WG_LD = 20, WG_GROUP = 8;

#ifndef WIDE_WGS
#define WIDE_WGS 4  // 119 VGPRs, 40 KB LDS: four 256-thread workgroups per CU (three: 2.88 vs 2.59 ms at C5)
#endif
// fp32 products on the bf16 matrix pipe (SPLIT, round 6; vae_enc.hip's scheme): each fp32 operand is split
// exactly into three bf16 x = hi + mid + lo (round-to-nearest of the remainders) as it is staged into LDS (three
// planes per operand, 32-byte rows with the halves of rows 8..15 of every 16 swapped: conflict-free
// ds_read_b128), and a 32 x 32 block takes six v_mfma_f32_32x32x16_bf16 per K-tile of 16 -- al.bh, ah.bl,
// am.bm, am.bh, ah.bm, ah.bh, smallest first, accumulated in fp32; the dropped products (am.bl, al.bm,
// al.bl) are <= 2^-27 relative, under the fp32 rounding level.  6 x 32 matrix-pipe cycles per block and K-tile
// against 8 x 64 for v_mfma_f32_32x32x2_f32.  48 KB of LDS: three workgroups per CU.
// Two values at a time, each rounded to nearest bf16 (v_cvt_pk_bf16_f32, the first value in the low half):
// x = hi + mid + lo exactly (the remainders of a round-to-nearest are exact fp32 and keep <= 16, then <= 8
// significant bits), and each remainder is at most half a bf16 ulp of the one before, so the three dropped
// products are <= 2^-27 relative (2^-24 with truncation, vae_enc.hip's split: too coarse for the deep
// ReLU variants' scale-free bar)
typedef __bf16 wbf16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned wpk(float a, float b) {
    const wbf16x2 t = {(__bf16)a, (__bf16)b};
    return __builtin_bit_cast(unsigned, t);
}
__device__ __forceinline__ void wsplit2(float a, float b, unsigned& h, unsigned& m, unsigned& l) {
    h = wpk(a, b);
    const float ra = a - __uint_as_float(h << 16), rb = b - __uint_as_float(h & 0xffff0000u);
    m = wpk(ra, rb);
    const float sa = ra - __uint_as_float(m << 16), sb = rb - __uint_as_float(m & 0xffff0000u);
    l = wpk(sa, sb);
}
__device__ __forceinline__ int wsw(int row, int half) { return row * 16 + 8 * (half ^ ((row >> 3) & 1)); }
constexpr int WS_PLANE = WG_BM * 16;  // bf16 per plane and operand (WG_BM == WG_BN)
constexpr int WS_LDS_FLOATS = 2 * 6 * WS_PLANE / 2;
static_assert(WG_BM == WG_BN && WS_LDS_FLOATS >= 4 * 64 * 33, "split staging / epilogue LDS");

template <int EPI, bool SPLIT>
__global__ __launch_bounds__(256, SPLIT ? 3 : WIDE_WGS) void wide_gemm_kernel(WideGemmArgs a) {
    constexpr int SMEM = SPLIT ? WS_LDS_FLOATS : 2 * (WG_BM + WG_BN) * WG_LD;
    __shared__ __align__(16) float smem[SMEM];
    float(*As)[WG_BM * WG_LD] = (float(*)[WG_BM * WG_LD])smem;
    float(*Bs)[WG_BN * WG_LD] = (float(*)[WG_BN * WG_LD])(smem + 2 * WG_BM * WG_LD);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1, lr = lane & 31, lh = lane >> 5;
    const int MT = (a.M + WG_BM - 1) / WG_BM, NT = a.N / WG_BN;
    // grouped tile order: WG_GROUP row tiles x all column tiles per group
    const int bid = blockIdx.x, per = WG_GROUP * NT, g = bid / per, r = bid - g * per;
    const int gm = min(WG_GROUP, MT - g * WG_GROUP);
    const int mt = g * WG_GROUP + r % gm, nt = r / gm;
    const int K = a.K1 + a.K2, KT1 = a.K1 / WG_BK, KT = K / WG_BK;
    const int kq = tid & 3;
    const int m0 = mt * WG_BM + (tid >> 2), m1 = m0 + 64;
    const bool v0 = m0 < a.M, v1 = m1 < a.M;
    const size_t q0 = v0 ? m0 : 0, q1 = v1 ? m1 : 0;
    const float* pa0 = a.A1 + q0 * a.lda1 + 4 * kq;
    const float* pa1 = a.A1 + q1 * a.lda1 + 4 * kq;
    const float* pc0 = a.A2 ? a.A2 + q0 * a.lda2 + 4 * kq : pa0;
    const float* pc1 = a.A2 ? a.A2 + q1 * a.lda2 + 4 * kq : pa1;
    const float* pb0 = a.W + (size_t)(nt * WG_BN + (tid >> 2)) * K + 4 * kq;
    const float* pb1 = pb0 + (size_t)64 * K;
    const int srow0 = (tid >> 2) * WG_LD + 4 * kq, srow1 = srow0 + 64 * WG_LD;
    float4 ra0, ra1, rb0, rb1;
#define WIDE_LOAD(kt)                                                                                   \
    do {                                                                                                \
        const bool seg2_ = (kt) >= KT1;                                                                 \
        const int ko_ = seg2_ ? ((kt) - KT1) * WG_BK : (kt) * WG_BK;                                    \
        /* rows past M read row 0 (q0, q1) unselected: they only feed accumulator rows that are never   \
           stored, and a select next to the load made the compiler wait for it at once */               \
        ra0 = *(const float4*)((seg2_ ? pc0 : pa0) + ko_);                                              \
        ra1 = *(const float4*)((seg2_ ? pc1 : pa1) + ko_);                                              \
        rb0 = *(const float4*)(pb0 + (size_t)(kt) * WG_BK);                                             \
        rb1 = *(const float4*)(pb1 + (size_t)(kt) * WG_BK);                                             \
    } while (0)
    unsigned short* const L16 = (unsigned short*)smem;  // SPLIT: [buf][A hi, mid, lo, B hi, mid, lo][row * 16]
    // SPLIT: a float4 (4 k of one row) into the three planes of operand `op` of buffer `buf`, row `row`
    auto split_stash = [&](int buf, int op, int row, float4 v) {
        unsigned h0, m0, l0, h1, m1, l1;
        wsplit2(v.x, v.y, h0, m0, l0);
        wsplit2(v.z, v.w, h1, m1, l1);
        unsigned short* base = L16 + (size_t)(buf * 6 + 3 * op) * WS_PLANE + wsw(row, kq >> 1) + 4 * (kq & 1);
        *(uint2*)base = make_uint2(h0, h1);
        *(uint2*)(base + WS_PLANE) = make_uint2(m0, m1);
        *(uint2*)(base + 2 * WS_PLANE) = make_uint2(l0, l1);
    };
#define WIDE_STASH(buf)                                    \
    do {                                                   \
        if constexpr (SPLIT) {                             \
            split_stash(buf, 0, tid >> 2, ra0);            \
            split_stash(buf, 0, (tid >> 2) + 64, ra1);     \
            split_stash(buf, 1, tid >> 2, rb0);            \
            split_stash(buf, 1, (tid >> 2) + 64, rb1);     \
        } else {                                           \
            *(float4*)(&As[buf][srow0]) = ra0;             \
            *(float4*)(&As[buf][srow1]) = ra1;             \
            *(float4*)(&Bs[buf][srow0]) = rb0;             \
            *(float4*)(&Bs[buf][srow1]) = rb1;             \
        }                                                  \
    } while (0)

    wf32x16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int q = 0; q < 16; ++q) acc[i][j][q] = 0.f;

    WIDE_LOAD(0);
    WIDE_STASH(0);
    __syncthreads();
    for (int kt = 0; kt < KT; ++kt) {
        const int buf = kt & 1;
        if (kt + 1 < KT) WIDE_LOAD(kt + 1);
        if constexpr (SPLIT) {
            const unsigned short* pa_ = L16 + (size_t)(buf * 6) * WS_PLANE;
            const unsigned short* pb_ = pa_ + 3 * WS_PLANE;
            wbf16x8 ah[2], am[2], al[2], bh[2], bm[2], bl[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                const int oa = wsw(wm * 64 + 32 * i + lr, lh), ob = wsw(wn * 64 + 32 * i + lr, lh);
                ah[i] = *(const wbf16x8*)(pa_ + oa);
                am[i] = *(const wbf16x8*)(pa_ + WS_PLANE + oa);
                al[i] = *(const wbf16x8*)(pa_ + 2 * WS_PLANE + oa);
                bh[i] = *(const wbf16x8*)(pb_ + ob);
                bm[i] = *(const wbf16x8*)(pb_ + WS_PLANE + ob);
                bl[i] = *(const wbf16x8*)(pb_ + 2 * WS_PLANE + ob);
            }
#define WIDE_MM(X, Y)                                                                                   \
    _Pragma("unroll") for (int i = 0; i < 2; ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j)         \
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(X[i], Y[j], acc[i][j], 0, 0, 0);
            WIDE_MM(al, bh)
            WIDE_MM(ah, bl)
            WIDE_MM(am, bm)
            WIDE_MM(am, bh)
            WIDE_MM(ah, bm)
            WIDE_MM(ah, bh)
#undef WIDE_MM
            if (kt + 1 < KT) WIDE_STASH(buf ^ 1);
            __syncthreads();
            continue;
        }
        float av[2][8], bv[2][8];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const float* ap = &As[buf][(wm * 64 + 32 * i + lr) * WG_LD + 8 * lh];
            const float* bp = &Bs[buf][(wn * 64 + 32 * i + lr) * WG_LD + 8 * lh];
            const float4 a0 = *(const float4*)ap, a1 = *(const float4*)(ap + 4);
            const float4 b0 = *(const float4*)bp, b1 = *(const float4*)(bp + 4);
            av[i][0] = a0.x; av[i][1] = a0.y; av[i][2] = a0.z; av[i][3] = a0.w;
            av[i][4] = a1.x; av[i][5] = a1.y; av[i][6] = a1.z; av[i][7] = a1.w;
            bv[i][0] = b0.x; bv[i][1] = b0.y; bv[i][2] = b0.z; bv[i][3] = b0.w;
            bv[i][4] = b1.x; bv[i][5] = b1.y; bv[i][6] = b1.z; bv[i][7] = b1.w;
        }
#pragma unroll
        for (int s = 0; s < 8; ++s)
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
                for (int j = 0; j < 2; ++j)
                    acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[i][s], bv[j][s], acc[i][j], 0, 0, 0);
        if (kt + 1 < KT) WIDE_STASH(buf ^ 1);
        __syncthreads();
    }
#undef WIDE_LOAD
#undef WIDE_STASH

    // epilogue, one 64 x 32 half of the wave tile at a time through LDS (the loop's last barrier freed
    // it): register q of lane (lr, lh) holds row 8(q/4) + 4 lh + q%4, column lr of its 32x32 block.
    // The element loop then runs rolled (the sincos is not replicated 64 times) with 128-B row stores.
    float* T = smem + wave * (64 * 33);
    const int mw = mt * WG_BM + wm * 64;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int q = 0; q < 16; ++q) T[(32 * i + 8 * (q >> 2) + 4 * lh + (q & 3)) * 33 + lr] = acc[i][j][q];
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        const int n = nt * WG_BN + wn * 64 + 32 * j + lr;
        const float bias = (EPI != WIDE_EPI_BWD && a.bias) ? a.bias[n] : 0.f;
        const float w5 = (EPI == WIDE_EPI_SIN_L4) ? a.w5[n] : 0.f;
        for (int it = 0; it < 32; ++it) {
            const int row = 2 * it + lh, m = mw + row;
            if (m >= a.M) break;
            const float v = T[row * 33 + lr];
            if constexpr (EPI == WIDE_EPI_BWD) {
                // torch's SinBackward then MulBackward: (delta_h * cos(t)) * w0; relu / softplus: delta_h * act'(t)
                const float dd = v * a.d[(size_t)m * a.ldd + n];
                a.out1[(size_t)m * a.ld1 + n] = a.act == 0 ? dd * a.w0 : dd;
            } else if constexpr (EPI == WIDE_EPI_STORE) {
                a.out1[(size_t)m * a.ld1 + n] = v + bias;
            } else {
                const float c0 = a.c ? a.c[(size_t)(m / a.rows_per_inst) * a.ldc + n] : bias;
                const float t = v + c0;
                float hv, dv;
                if (a.act == 0) {
                    sdfn_sincosf(a.w0 * t, &hv, &dv);
                } else if (a.act == 1) {  // torch ReLU; ReluBackward passes where the output is > 0
                    hv = t > 0.0f ? t : 0.0f;
                    dv = hv > 0.0f ? 1.0f : 0.0f;
                } else {  // torch Softplus(beta 1, threshold 20) and SoftplusBackward: z / (z + 1), z = exp(t)
                    const float ez = expf(t);
                    hv = t > 20.0f ? t : log1pf(ez);
                    dv = t > 20.0f ? 1.0f : ez / (ez + 1.0f);
                }
                a.out1[(size_t)m * a.ld1 + n] = hv;
                a.out2[(size_t)m * a.ld2 + n] = (EPI == WIDE_EPI_SIN_L4) ? (a.act == 0 ? (w5 * dv) * a.w0 : w5 * dv) : dv;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

hipError_t launch_wide_gemm(const WideGemmArgs& a, int epi, hipStream_t s) {
    if (a.M <= 0) return hipSuccess;
    if (a.N % WG_BN || a.K1 % WG_BK || a.K2 % WG_BK || a.K1 <= 0 || (a.K2 > 0 && !a.A2) || a.lda1 % 4 ||
        (a.A2 && a.lda2 % 4))
        return hipErrorInvalidValue;
    const long long MT = (a.M + WG_BM - 1) / WG_BM, grid = MT * (a.N / WG_BN);
    if (grid > 0x7fffffffLL) return hipErrorInvalidValue;
    // SDFNMPC_WIDE_F32=1: the exact-fp32 MFMA main loop (comparison builds of the same library)
    static const bool f32 = [] { const char* e = getenv("SDFNMPC_WIDE_F32"); return e && *e == '1'; }();
    auto go = [&](auto ec, auto sc) {
        hipLaunchKernelGGL((wide_gemm_kernel<decltype(ec)::value, decltype(sc)::value>), dim3((unsigned)grid), dim3(256),
                           0, s, a);
    };
    auto by_split = [&](auto ec) {
        if (f32) go(ec, std::false_type{});
        else go(ec, std::true_type{});
    };
    switch (epi) {
        case WIDE_EPI_SIN: by_split(std::integral_constant<int, WIDE_EPI_SIN>{}); break;
        case WIDE_EPI_SIN_L4: by_split(std::integral_constant<int, WIDE_EPI_SIN_L4>{}); break;
        case WIDE_EPI_BWD: by_split(std::integral_constant<int, WIDE_EPI_BWD>{}); break;
        case WIDE_EPI_STORE: by_split(std::integral_constant<int, WIDE_EPI_STORE>{}); break;
        default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// latent (fp64 stage parameters or fp32, strided, lh entries) -> fp32 [n_inst][lz], zero past lh: a
// size_latent below the GEMMs' 128-multiple K is zero-padded (the padded columns of Hz / rows of Bz are
// zero too, so they add exact zeros)
template <typename T>
__global__ void wide_latent_kernel(const T* lat, long long stride, int n_inst, int lh, int lz, float* z) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (long long)n_inst * lz) return;
    const long long inst = i / lz, k = i - inst * lz;
    z[i] = k < lh ? (float)lat[inst * stride + k] : 0.0f;
}

// positional embedding e (embeddings.py:106-111) and its derivative factors, nek features per row
// (m < 3: pos, then sin(xb), sin(xb + pi/2) over the nb projected frequencies, zero pad; embed 'none':
// nb = 0) -- the same arithmetic as sdf_mlp.hip
__global__ __launch_bounds__(256) void wide_emb_kernel(WideSdfArgs a) {
    const long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x;
    const int NEK = a.nek, NB = a.nb;
    if (i >= (long long)a.rows * NEK) return;
    const int r = (int)(i / NEK), m = (int)(i - (long long)r * NEK);
    float px, py, pz;
    if (a.x) {  // Co_p_B = W_R_Co^T (W_p_B - W_p_Co) in fp64, handed over as fp32 (gen_model.py:46-51)
        const double* xr = a.x + (size_t)r * 10;
        const double* pr = a.p + (size_t)r * a.np;
        const double* R = pr + 4;
        const double e0 = xr[0] - pr[1], e1 = xr[1] - pr[2], e2 = xr[2] - pr[3];
        px = (float)((e0 * R[0] + e1 * R[3]) + e2 * R[6]);
        py = (float)((e0 * R[1] + e1 * R[4]) + e2 * R[7]);
        pz = (float)((e0 * R[2] + e1 * R[5]) + e2 * R[8]);
    } else {
        const float4 p = a.pos[r];
        px = p.x; py = p.y; pz = p.z;
    }
    float e, g;
    if (m < 3) {
        e = (m == 0) ? px : (m == 1 ? py : pz);
        g = 1.0f;
    } else if (m < 3 + 2 * NB) {
        const float4 t = a.emb_tab[m];
        float xb = px * t.x + py * t.y + pz * t.z;
        if (m >= 3 + NB) xb = xb + 1.57079637050628662109375f;
        float s, c;
        sdfn_sincosf(xb, &s, &c);
        e = s;
        g = c;
    } else {
        e = 0.0f;
        g = 0.0f;
    }
    a.E[(size_t)r * NEK + m] = e;
    a.G[(size_t)r * NEK + m] = g;
}

// df, d df / d pos and the constraint epilogue, one thread per row (sequential sums: deterministic)
__global__ __launch_bounds__(256) void wide_final_kernel(WideSdfArgs a) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= a.rows) return;
    const float* h4 = a.H4 + (size_t)r * a.n4;
    float acc = 0.0f;
    for (int n = 0; n < a.n4; ++n) acc += a.w5[n] * h4[n];
    const float df = acc + a.b5;
    const float* ge3 = a.GE3 + (size_t)r * a.neb;
    const float* ge1 = a.GE1 + (size_t)r * a.neb;
    const float* gg = a.G + (size_t)r * a.nek;
    float s0 = 0.f, s1 = 0.f, s2 = 0.f;
    for (int m = 0; m < a.nek; ++m) {
        const float u = (ge3[m] + ge1[m]) * gg[m];
        if (m < 3) {
            s0 += (m == 0) ? u : 0.0f;
            s1 += (m == 1) ? u : 0.0f;
            s2 += (m == 2) ? u : 0.0f;
        } else {
            const float4 t = a.emb_tab[m];
            s0 += u * t.x;
            s1 += u * t.y;
            s2 += u * t.z;
        }
    }
    if (a.out) a.out[r] = make_float4(df, s0, s1, s2);
    if (a.h) {  // sdf row of the constraint vector and its Jacobian (gen_model.py:46-61)
        const double* pr = a.p + (size_t)r * a.np;
        const double flag = pr[0];
        const double* R = pr + 4;
        a.h[(size_t)r * 3 + 2] = flag * (double)df + (1.0 - flag) * a.max_df;
        double* J = a.Jh + (size_t)r * 30 + 2;
#pragma unroll
        for (int j = 0; j < 10; ++j)
            J[j * 3] = (j < 3) ? flag * (((double)s0 * R[j * 3 + 0] + (double)s1 * R[j * 3 + 1]) + (double)s2 * R[j * 3 + 2])
                               : 0.0;
    }
}

template <typename T>
hipError_t launch_wide_latent(const T* lat, long long stride, int n_inst, int lh, int lz, float* z, hipStream_t s) {
    if (n_inst <= 0) return hipSuccess;
    const long long n = (long long)n_inst * lz;
    hipLaunchKernelGGL(wide_latent_kernel<T>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, lat, stride, n_inst,
                       lh, lz, z);
    return hipGetLastError();
}
template hipError_t launch_wide_latent<double>(const double*, long long, int, int, int, float*, hipStream_t);
template hipError_t launch_wide_latent<float>(const float*, long long, int, int, int, float*, hipStream_t);

hipError_t launch_wide_emb(const WideSdfArgs& a, hipStream_t s) {
    if (a.rows <= 0) return hipSuccess;
    const long long n = (long long)a.rows * a.nek;
    hipLaunchKernelGGL(wide_emb_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, a);
    return hipGetLastError();
}

hipError_t launch_wide_final(const WideSdfArgs& a, hipStream_t s) {
    if (a.rows <= 0) return hipSuccess;
    hipLaunchKernelGGL(wide_final_kernel, dim3((a.rows + 255) / 256), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace sdfn
