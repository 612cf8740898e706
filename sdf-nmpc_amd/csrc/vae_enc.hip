// In-loop VAE encoder on gfx950: B depth images -> B latent means.
//
// Reference: sdf_nmpc/vae.py:15-40 (preprocessing + Encoder.forward), network/vae.py:6-46 (Encoder),
// network/resnet.py:5-56 (ResBlock), utils/preprocessing.py (Reshape, ClipDistance, Depth2Range).
// Inference semantics: dropout is the identity and every BatchNorm is folded into its convolution on
// the host (sdf-nmpc_amd/vae.py:_fold), so the network is a chain of biased convolutions.
//
// Kernels (activations NHWC fp32, resident in one workspace):
//   vae_pre_kernel   raw depth -> range image (resize, clip, depth->range), one thread per pixel
//   vae_stem_kernel  conv7x7/2 + ELU + maxpool3/2 fused per 7x8 pooled tile: an implicit GEMM (255 conv
//                    pixels x 64 channels x 49 taps) on the bf16 matrix pipe with fp32-exact split
//                    products, the conv tile in LDS for the pool
//   vae_conv_kernel  every ResBlock convolution as an implicit GEMM on f32 MFMA 32x32x2 (exact fp32
//                    products): 128x128 output tile per workgroup, K staged 16 at a time through
//                    double-buffered LDS, bias / residual / ReLU fused into the epilogue
//   vae_head_kernel  AdaptiveAvgPool2d((2,2)) + Flatten + mean Linear, 4 images per workgroup
#include <hip/hip_runtime.h>

#include <math.h>

#include "vae_kernels.h"

namespace sdfn {

typedef float floatx16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));



// ------------------------------------------------------------------------------------------------
// preprocessing: ToDevice (float32), Reshape (bilinear, align_corners=False), ClipDistance,
// Depth2Range -- fp32 in torch's operation order (oracle/vae.c:orc_vae_preprocess)
__global__ __launch_bounds__(256) void vae_pre_kernel(VaePreArgs a) {
#pragma clang fp contract(off)
    const int b = blockIdx.y;
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.H * a.W) return;
    const int y = i / a.W, x = i - y * a.W;
    const size_t ib = (size_t)b * a.Hi * a.Wi;
    auto px = [&](int yy, int xx) -> float {
        const size_t k = ib + (size_t)yy * a.Wi + xx;
        return a.dtype == 1 ? (float)((const unsigned short*)a.img)[k] : ((const float*)a.img)[k];
    };
    float v;
    if (a.Hi == a.H && a.Wi == a.W) {
        v = px(y, x);
    } else {
        const float sh = (float)a.Hi / (float)a.H, sw = (float)a.Wi / (float)a.W;
        float fy = sh * ((float)y + 0.5f) - 0.5f, fx = sw * ((float)x + 0.5f) - 0.5f;
        fy = fy < 0.f ? 0.f : fy;
        fx = fx < 0.f ? 0.f : fx;
        const int y0 = (int)fy, x0 = (int)fx;
        const int y1 = y0 + (y0 < a.Hi - 1), x1 = x0 + (x0 < a.Wi - 1);
        const float ly1 = fy - (float)y0, ly0 = 1.f - ly1, lx1 = fx - (float)x0, lx0 = 1.f - lx1;
        v = ly0 * (lx0 * px(y0, x0) + lx1 * px(y0, x1)) + ly1 * (lx0 * px(y1, x0) + lx1 * px(y1, x1));
    }
    v = v / a.clip;
    v = v < 0.f ? 0.f : (v > 1.f ? 1.f : v);
    if (a.yz) {
        v = v * a.yz[i];
        v = v < 0.f ? 0.f : (v > 1.f ? 1.f : v);
    }
    a.out[(size_t)b * a.H * a.W + i] = v;
}

hipError_t launch_vae_pre(const VaePreArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    hipLaunchKernelGGL(vae_pre_kernel, dim3((a.H * a.W + 255) / 256, a.B), dim3(256), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// stem: conv7x7/2 pad 3 (1 -> 64) + bias + ELU + maxpool3/2 pad 1 (vae.py:19-21), as an implicit GEMM on
// the bf16 matrix pipe with fp32-exact products (the split of the ResBlock convolutions below):
//   out[p][n] = sum_k A[p][k] W[k][n],  p = the 255 conv pixels of a 7 x 8 pooled tile (15 x 17, one slot of
//   padding: 8 pixel blocks of 32), n = 64 channels, k = 48 of the 49 taps (3 K-steps of 16, in the order
//   of vae_stem_slot_tap) + tap 48 as one fp32 fma per output on the vector ALU.  Each wave owns two pixel
//   blocks x two channel blocks.  The weights come split into hi / mid / lo bf16 planes (once at load,
//   sdfnmpc_vae_load) and sit in registers for the workgroup's life; the input patch is split likewise, once
//   per tile, into three bf16 planes in LDS, from which each lane gathers its pixel's taps (a horizontal tap
//   pair = one 32-bit read).  Six v_mfma_f32_32x32x16_bf16 per block and K-step (al.bh, ah.bl, am.bm, am.bh,
//   ah.bm, ah.bh) accumulate in fp32; the dropped products are <= 2^-24 relative.  conv + bias into the conv
//   tile in LDS (over the patch), then the maxpool and the ELU of the pooled values, four channels per
//   thread (16-byte LDS reads and global stores).  Persistent: two workgroups per CU walk the tiles, the next
//   tile's patch loads in flight in registers under the current tile's products.
constexpr int ST_PY = 7, ST_PX = 8;                        // pooled tile
constexpr int ST_CY = 2 * ST_PY + 1, ST_CX = 2 * ST_PX + 1;  // conv tile 15 x 17 = 255 pixels
constexpr int ST_IY = 2 * ST_CY + 5, ST_IX = 2 * ST_CX + 5;  // input patch 35 x 39
// patch row stride (bf16): even (32-bit aligned tap pairs) and 24 words, so one conv row further (two patch
// rows, 48 words = 16 banks) puts a lane group's second conv row on the other half of the banks: the 32
// lanes of a gather (17 + 15 pixels of two conv rows) hit distinct banks but one (40 bf16 rows: 2-way)
constexpr int ST_IXP = 48;
static_assert(ST_IXP >= ST_IX + 1 && ST_IXP % 2 == 0, "patch row");
constexpr int ST_CS = 68;                                  // conv tile row (floats): 16-byte rows for the pool
constexpr int ST_PATCH = ST_IY * ST_IXP;                   // values per patch plane (bf16)
constexpr int ST_CONV = ST_CY * ST_CX * ST_CS;             // floats
constexpr int ST_LDS = (3 * ST_PATCH * 2 > ST_CONV * 4 ? 3 * ST_PATCH * 2 : ST_CONV * 4);
static_assert(ST_IXP % 2 == 0 && ST_PATCH % 2 == 0, "32-bit tap-pair reads need even rows and planes");

// x = hi + mid + lo exactly, each a bf16 truncation of the remainder (the split of split3_store)
__device__ __forceinline__ void split3(float x, unsigned& h, unsigned& m, unsigned& l) {
    h = __float_as_uint(x) & 0xffff0000u;
    const float r1 = x - __uint_as_float(h);
    m = __float_as_uint(r1) & 0xffff0000u;
    const float r2 = r1 - __uint_as_float(m);
    l = __float_as_uint(r2) & 0xffff0000u;
}

// ELU(alpha = 1) = x for x > 0, expm1(x) otherwise (torch elu).  expm1 on x <= 0: the Taylor series to
// x^8 / 8! on (-0.35, 0] (truncation <= 2.3e-10 relative, Horner in fp32), exp(x) - 1 below, where exp(x)
// <= 0.71 leaves no cancellation; exp(x) as v_exp_f32(x log2 e): the rounding of the product costs at most
// |x| exp(x) log2(e) 2^-24 <= 3.2e-8 absolute, under the fp32 rounding of the result.  A NaN stays a NaN.
// ELU is increasing, so the kernel pools first and activates the pooled values only (4.6x fewer).  Two
// values at a time: the series on the packed fp32 pipe (v_pk_fma_f32).
typedef float float2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float2v elu2(float2v x) {
    float2v p = (float2v)(1.0f / 40320.0f);
    p = __builtin_elementwise_fma(p, x, (float2v)(1.0f / 5040.0f));
    p = __builtin_elementwise_fma(p, x, (float2v)(1.0f / 720.0f));
    p = __builtin_elementwise_fma(p, x, (float2v)(1.0f / 120.0f));
    p = __builtin_elementwise_fma(p, x, (float2v)(1.0f / 24.0f));
    p = __builtin_elementwise_fma(p, x, (float2v)(1.0f / 6.0f));
    p = __builtin_elementwise_fma(p, x, (float2v)(0.5f));
    const float2v taylor = __builtin_elementwise_fma(p * x, x, x);
    const float2v y = x * 1.44269504088896341f;
    const float2v viaexp = float2v{__builtin_amdgcn_exp2f(y.x), __builtin_amdgcn_exp2f(y.y)} - 1.0f;
    return float2v{!(x.x <= 0.f) ? x.x : (x.x > -0.35f ? taylor.x : viaexp.x),
                   !(x.y <= 0.f) ? x.y : (x.y > -0.35f ? taylor.y : viaexp.y)};
}

__device__ __forceinline__ float max9(const float4 (&v)[9], int f) {
    float m[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        const float a = (&v[3 * r].x)[f], b = (&v[3 * r + 1].x)[f], c = (&v[3 * r + 2].x)[f];
        m[r] = __builtin_elementwise_maximum(__builtin_elementwise_maximum(a, b), c);
    }
    return __builtin_elementwise_maximum(__builtin_elementwise_maximum(m[0], m[1]), m[2]);
}

constexpr int ST_PRE = (ST_IY * ST_IX + 255) / 256;  // patch values per thread

__global__ __launch_bounds__(256, 2) void vae_stem_kernel(VaeStemArgs a, int tiles_x, int tiles_img, int n_tiles) {
    __shared__ __align__(16) float smem[ST_LDS / 4];  // the split patch, then the conv tile
    __shared__ __align__(16) int poff[24];  // slot pair -> patch offset ky * ST_IXP + kx of its first tap from the
                                            // pixel's tap 0; general pairs: both offsets, the second << 16
    __shared__ __align__(16) float bias[64];
    __shared__ __align__(16) float w48[64];           // tap 48 = (6, 6) of each channel, fp32
    // [hi | mid | lo][row][column] bf16: a horizontal tap pair of a pixel is one aligned 32-bit word, and
    // the stride-2 pixels of a lane group read consecutive words (conflict-free)
    unsigned short* patch = (unsigned short*)smem;
    float* conv = smem;  // after the products
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, lr = lane & 31, lh = lane >> 5;
    // the weight fragments of the three K-steps, once per workgroup: channel n = 32 j + lr, taps
    // 16 s + 8 lh .. + 7 of each plane
    bf16x8 bw[3][3][2];
#pragma unroll
    for (int s = 0; s < 3; ++s)
#pragma unroll
        for (int pl = 0; pl < 3; ++pl)
#pragma unroll
            for (int j = 0; j < 2; ++j)
                bw[s][pl][j] = *(const bf16x8*)&a.wpl[pl * VAE_STEM_PLANE + (32 * j + lr) * 64 + 16 * s + 8 * lh];
    if (t < 24) {
        const int k0 = vae_stem_slot_tap(2 * t), k1 = vae_stem_slot_tap(2 * t + 1);
        const int o0 = (k0 / 7) * ST_IXP + k0 % 7, o1 = (k1 / 7) * ST_IXP + k1 % 7;
        poff[t] = vae_stem_general_pair(t) ? o0 | (o1 << 16) : o0;
    }
    if (t < 64) {
        bias[t] = a.b[t];
        // hi + mid + lo = the fp32 weight exactly
        w48[t] = (__uint_as_float((unsigned)a.wpl[t * 64 + 48] << 16) +
                  __uint_as_float((unsigned)a.wpl[VAE_STEM_PLANE + t * 64 + 48] << 16)) +
                 __uint_as_float((unsigned)a.wpl[2 * VAE_STEM_PLANE + t * 64 + 48] << 16);
    }
    // this lane's two pixels (pixel blocks i = 0, 1 of the wave): conv pixel q = 64 wave + 32 i + lr
    int pbase[2], pcy[2], pcx[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
        const int q = wave * 64 + 32 * i + lr, qq = q < ST_CY * ST_CX ? q : 0;
        pcy[i] = qq / ST_CX;
        pcx[i] = qq - pcy[i] * ST_CX;
        pbase[i] = (2 * pcy[i]) * ST_IXP + 2 * pcx[i];
    }
    // the next tile's input patch, in flight in registers while this tile computes
    float pre[ST_PRE];
    auto fetch = [&](int tile) {
        const int img = tile / tiles_img, tt = tile - img * tiles_img, ty = tt / tiles_x;
        const int gy0 = 4 * ty * ST_PY - 5, gx0 = 4 * (tt - ty * tiles_x) * ST_PX - 5;
        const float* in = a.in + (size_t)img * a.H * a.W;
#pragma unroll
        for (int u = 0; u < ST_PRE; ++u) {
            const int e = t + 256 * u, r = e / ST_IX, c = e - r * ST_IX, gy = gy0 + r, gx = gx0 + c;
            pre[u] = e < ST_IY * ST_IX && (unsigned)gy < (unsigned)a.H && (unsigned)gx < (unsigned)a.W
                         ? in[(size_t)gy * a.W + gx] : 0.f;
        }
    };
    fetch(blockIdx.x);  // the grid is at most n_tiles workgroups
    for (int tile = blockIdx.x; tile < n_tiles; tile += gridDim.x) {
        const int img = tile / tiles_img, tt = tile - img * tiles_img, ty = tt / tiles_x;
        const int py0 = ty * ST_PY, px0 = (tt - ty * tiles_x) * ST_PX;
#pragma unroll
        for (int u = 0; u < ST_PRE; ++u) {
            const int e = t + 256 * u, r = e / ST_IX, c = e - r * ST_IX;
            if (e < ST_IY * ST_IX) {
                unsigned h, m, l;
                split3(pre[u], h, m, l);
                const int o = r * ST_IXP + c;
                patch[o] = (unsigned short)(h >> 16);
                patch[ST_PATCH + o] = (unsigned short)(m >> 16);
                patch[2 * ST_PATCH + o] = (unsigned short)(l >> 16);
            }
        }
        __syncthreads();
        if (tile + (int)gridDim.x < n_tiles) fetch(tile + gridDim.x);
        // C^T = W^T A^T: rows = channels (the weight fragment is the first operand), columns = pixels, so
        // each lane ends with four consecutive channels of one pixel per register quad (16-byte LDS writes)
        floatx16 acc[2][2];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
#pragma unroll
        for (int s = 0; s < 3; ++s) {
            // A: slots k = 16 s + 8 lh + 2 jj (+1) of the lane's pixels, slot pair 8 s + 4 lh + jj (offsets
            // from the pair table: one 16-byte read), from the split planes: a horizontal pair is one 32-bit
            // read per plane, a general pair (K-step 2, jj >= 2, for both lane halves) two 16-bit reads
            const int4 of = *(const int4*)&poff[8 * s + 4 * lh];
            const int pof[4] = {of.x, of.y, of.z, of.w};
            bf16x8 ah[2], am[2], al[2];
#pragma unroll
            for (int i = 0; i < 2; ++i) {
                unsigned hp[4], mp[4], lp[4];
#pragma unroll
                for (int jj = 0; jj < 4; ++jj) {
                    if (s == 2 && jj >= 2) {
                        const unsigned short* p0 = patch + pbase[i] + (pof[jj] & 0xffff);
                        const unsigned short* p1 = patch + pbase[i] + (pof[jj] >> 16);
                        hp[jj] = p0[0] | ((unsigned)p1[0] << 16);
                        mp[jj] = p0[ST_PATCH] | ((unsigned)p1[ST_PATCH] << 16);
                        lp[jj] = p0[2 * ST_PATCH] | ((unsigned)p1[2 * ST_PATCH] << 16);
                    } else {
                        const unsigned* p0 = (const unsigned*)(patch + pbase[i] + pof[jj]);
                        hp[jj] = p0[0];
                        mp[jj] = p0[ST_PATCH / 2];
                        lp[jj] = p0[ST_PATCH];
                    }
                }
                ah[i] = __builtin_bit_cast(bf16x8, make_uint4(hp[0], hp[1], hp[2], hp[3]));
                am[i] = __builtin_bit_cast(bf16x8, make_uint4(mp[0], mp[1], mp[2], mp[3]));
                al[i] = __builtin_bit_cast(bf16x8, make_uint4(lp[0], lp[1], lp[2], lp[3]));
            }
#define ST_MM(X, PL)                                                                                    \
    _Pragma("unroll") for (int i = 0; i < 2; ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j)           \
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bw[s][PL][j], X[i], acc[i][j], 0, 0, 0);
            ST_MM(al, 0)
            ST_MM(ah, 2)
            ST_MM(am, 1)
            ST_MM(am, 0)
            ST_MM(ah, 1)
            ST_MM(ah, 0)
#undef ST_MM
        }
        // tap 48, the 49th, on the vector ALU (one fp32 fma per output) rather than a fourth K-step that
        // would be 15/16 padding: the lane's pixel value, hi + mid + lo = the fp32 input exactly
        float x48[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const unsigned short* p = patch + pbase[i] + 6 * ST_IXP + 6;  // (ky, kx) = (6, 6)
            x48[i] = (__uint_as_float((unsigned)p[0] << 16) + __uint_as_float((unsigned)p[ST_PATCH] << 16)) +
                     __uint_as_float((unsigned)p[2 * ST_PATCH] << 16);
        }
        __syncthreads();  // every wave is done with the patch: the conv tile takes its place
        // epilogue: conv + bias (pre-activation) into the tile; lane (lr, lh), register r holds channel
        // 32 j + 8 (r / 4) + 4 lh + r % 4 of pixel 64 wave + 32 i + lr.  Conv pixels outside the map (the
        // pool's padding, the map's far edge) get -inf: they never win the pool.
        const int cy0 = 2 * py0 - 1, cx0 = 2 * px0 - 1;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int q = wave * 64 + 32 * i + lr;
            if (q >= ST_CY * ST_CX) continue;
            if ((unsigned)(cy0 + pcy[i]) < (unsigned)a.Hc && (unsigned)(cx0 + pcx[i]) < (unsigned)a.Wc) {
                const float2v x2 = (float2v)(x48[i]);
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int g = 0; g < 4; ++g) {
                        const int c = 32 * j + 8 * g + 4 * lh;
                        const float4 b4 = *(const float4*)&bias[c], w4 = *(const float4*)&w48[c];
                        const float2v lo = __builtin_elementwise_fma(x2, float2v{w4.x, w4.y}, float2v{acc[i][j][4 * g], acc[i][j][4 * g + 1]}) + float2v{b4.x, b4.y};
                        const float2v hi = __builtin_elementwise_fma(x2, float2v{w4.z, w4.w}, float2v{acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]}) + float2v{b4.z, b4.w};
                        *(float4*)&conv[q * ST_CS + c] = make_float4(lo.x, lo.y, hi.x, hi.y);
                    }
            } else {
#pragma unroll
                for (int j = 0; j < 2; ++j)
#pragma unroll
                    for (int g = 0; g < 4; ++g)
                        *(float4*)&conv[q * ST_CS + 32 * j + 8 * g + 4 * lh] = make_float4(-INFINITY, -INFINITY, -INFINITY, -INFINITY);
            }
        }
        __syncthreads();
        // maxpool 3/2 of the pre-activations, then the ELU of the pooled value (ELU is increasing: the same
        // result as pooling the activations, vae.py:19-21); thread -> (pooled pixel, four channels).
        // NaN-sticky as torch's max_pool2d: IEEE 754-2019 maximum (v_maximum3_f32), which propagates a NaN
        // lane -> (pooled pixel, four channels) so that each 16-lane group of a ds_read_b128
        // ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and the same + 32) reads one pixel's 256 contiguous
        // bytes (conflict-free); with 16 consecutive lanes per pixel, the groups straddled two pixels
        // two conv columns (544 B) apart
        for (int e = t; e < ST_PY * ST_PX * 16; e += 256) {
            const int L = e & 31, g1 = L < 4 || (L >= 12 && L < 16) || (L >= 20 && L < 28);
            const int rk = g1 ? (L < 4 ? L : L < 16 ? L - 8 : L - 12) : (L < 12 ? L - 4 : L < 20 ? L - 8 : L - 16);
            const int q = 2 * (e >> 5) + (g1 ? 0 : 1), c4 = 4 * rk;
            const int pyl = q >> 3, pxl = q & 7;
            const int py = py0 + pyl, px = px0 + pxl;
            if (py >= a.Hp || px >= a.Wp) continue;
#ifdef STEM_DIAG_NOPOOL  // diagnostic builds only (tools/build_variant.sh)
            *(float4*)&a.out[((size_t)img * 64 + (c4 & ~15)) * a.Hp * a.Wp + (py * a.Wp + px) * 16 + (c4 & 15)] = *(const float4*)&conv[((2 * pyl + 1) * ST_CX + 2 * pxl + 1) * ST_CS + c4];
#else
            float4 v[9];
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx)
                    v[3 * dy + dx] = *(const float4*)&conv[((2 * pyl + dy) * ST_CX + 2 * pxl + dx) * ST_CS + c4];
#ifdef STEM_DIAG_NOELU
            *(float4*)&a.out[((size_t)img * 64 + (c4 & ~15)) * a.Hp * a.Wp + (py * a.Wp + px) * 16 + (c4 & 15)] =
                make_float4(max9(v, 0), max9(v, 1), max9(v, 2), max9(v, 3));
#else
            const float2v e0 = elu2(float2v{max9(v, 0), max9(v, 1)}), e1 = elu2(float2v{max9(v, 2), max9(v, 3)});
            // channel-blocked output [B][4][Hp][Wp][16] (the convolutions' layout)
            *(float4*)&a.out[((size_t)img * 64 + (c4 & ~15)) * a.Hp * a.Wp + (py * a.Wp + px) * 16 + (c4 & 15)] =
                make_float4(e0.x, e0.y, e1.x, e1.y);
#endif
#endif
        }
        __syncthreads();  // the pool is done with the conv tile: the next patch takes its place
    }
}

hipError_t launch_vae_stem(const VaeStemArgs& a, int n_cu, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    if (a.Hc != (a.H - 1) / 2 + 1 || a.Wc != (a.W - 1) / 2 + 1 || a.Hp != (a.Hc - 1) / 2 + 1 ||
        a.Wp != (a.Wc - 1) / 2 + 1)
        return hipErrorInvalidValue;
    const int tiles_x = (a.Wp + ST_PX - 1) / ST_PX, tiles_img = tiles_x * ((a.Hp + ST_PY - 1) / ST_PY);
    if ((long long)tiles_img * a.B > 0x7fffffff) return hipErrorInvalidValue;
    const int n_tiles = tiles_img * a.B;
    // persistent: two workgroups per CU (the 69 KB conv tile), each walking the tiles with a stride of
    // the grid, the next tile's patch loads in flight under the current tile's products
    if (n_cu <= 0) return hipErrorInvalidDevice;
    const int grid = n_tiles < 2 * n_cu ? n_tiles : 2 * n_cu;
    hipLaunchKernelGGL(vae_stem_kernel, dim3(grid), dim3(256), 0, s, a, tiles_x, tiles_img, n_tiles);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// implicit-GEMM convolution: out[m][n] = sum_k A[m][k] W[n][k], m = (image, oy, ox), n = channel,
// k = (ky, kx, ci).  Tile 128 x 128 x 16, 4 waves as 2 x 2 of 64 x 64 (four 32x32 MFMA blocks each).
// LDS rows are 16 k-values padded to 20 floats: the ds_read_b128 lane groups then hit 16 distinct
// 16-byte slots (conflict-free).  Within a K-tile, MFMA step s feeds lane half h with k = 8h + s
// (the same permutation for A and B), so each lane reads its 8 k-values with two ds_read_b128.
constexpr int CV_BM = 128, CV_BN = 128, CV_BK = 16;
#ifndef VAE_CONV_WGS
#define VAE_CONV_WGS 3
#endif
// bf16 plane rows of 16 k-values, 32 bytes, unpadded; the two 16-byte halves of rows 8..15 of every 16
// swapped (row bit 3), so the lane groups of the fragments' ds_read_b128 hit 16 distinct 16-byte slots
// and the staging stores stay contiguous.  Two stages x 3 planes x 256 rows = 48 KB: three workgroups
// per CU (the 48-byte padded rows took 72 KB, two per CU).
#if VAE_CONV_WGS == 3
constexpr int CV_SLD = 16;
__device__ __forceinline__ int cv_off(int row, int half) { return row * 16 + 8 * (half ^ ((row >> 3) & 1)); }
#else  // diagnostic build: the round-3 layout (48-byte rows, two workgroups per CU)
constexpr int CV_SLD = 24;
__device__ __forceinline__ int cv_off(int row, int half) { return row * 24 + 8 * half; }
#endif

// fp32 -> three bf16 by truncation: x = hi + mid + lo EXACTLY (each takes the next 8 significant bits of
// the 24; the remainders are exact fp32 differences).  A float4 of one row -> its 4-bf16 pieces of the
// hi / mid / lo planes (8-byte stores).
__device__ __forceinline__ void split3_store(float4 v, unsigned short* planes, int pstride, int off) {
#ifdef VAE_DIAG_NOSPLIT  // diagnostic build (tools/build_variant.sh): the time without the split's VALU work
    const uint2 q = make_uint2((__float_as_uint(v.x) >> 16) | (__float_as_uint(v.y) & 0xffff0000u),
                               (__float_as_uint(v.z) >> 16) | (__float_as_uint(v.w) & 0xffff0000u));
    *(uint2*)&planes[off] = q;
    *(uint2*)&planes[pstride + off] = q;
    *(uint2*)&planes[2 * pstride + off] = q;
    return;
#endif
    const float x[4] = {v.x, v.y, v.z, v.w};
    unsigned hb[4], mb[4], lb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        hb[q] = __float_as_uint(x[q]) & 0xffff0000u;
        const float r1 = x[q] - __uint_as_float(hb[q]);
        mb[q] = __float_as_uint(r1) & 0xffff0000u;
        const float r2 = r1 - __uint_as_float(mb[q]);
        lb[q] = __float_as_uint(r2) & 0xffff0000u;
    }
    *(uint2*)&planes[off] = make_uint2((hb[0] >> 16) | hb[1], (hb[2] >> 16) | hb[3]);
    *(uint2*)&planes[pstride + off] = make_uint2((mb[0] >> 16) | mb[1], (mb[2] >> 16) | mb[3]);
    *(uint2*)&planes[2 * pstride + off] = make_uint2((lb[0] >> 16) | lb[1], (lb[2] >> 16) | lb[3]);
}

// component-wise select (a ?: on the float4 struct goes through a stack slot)
__device__ __forceinline__ float4 sel4(bool ok, float4 v) {
    return make_float4(ok ? v.x : 0.f, ok ? v.y : 0.f, ok ? v.z : 0.f, ok ? v.w : 0.f);
}

#ifndef VAE_LOAD_DEPTH
#define VAE_LOAD_DEPTH 1
#endif
constexpr int CV_D = VAE_LOAD_DEPTH;  // K-tiles whose global loads are in flight in registers

template <int KS, int S>
__global__ __launch_bounds__(256, VAE_CONV_WGS) void vae_conv_kernel(VaeConvArgs a) {
    constexpr int P = KS / 2;
    // the K-tile split ONCE, by the thread that loads it, into bf16 hi / mid / lo planes: rows of 16 bf16
    // at a 24-bf16 (48-byte) stride, so the lane groups of a ds_read_b128 hit distinct 16-byte slots
    __shared__ __align__(16) unsigned short As3[2][3][CV_BM * CV_SLD];
    __shared__ __align__(16) unsigned short Bs3[2][3][CV_BN * CV_SLD];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1, lr = lane & 31, lh = lane >> 5;
    const int M = a.B * a.Ho * a.Wo, MT = (M + CV_BM - 1) / CV_BM;
    const int nt = blockIdx.x / MT, mt = blockIdx.x - nt * MT;
    const int Cin = a.Cin, K = KS * KS * Cin, KT = K / CV_BK;
    const int kq = tid & 3;

    // loader rows (A) and columns (B) of this thread (scalars, so nothing is indexed dynamically)
    const int HW = a.Ho * a.Wo;
    const int m0 = mt * CV_BM + (tid >> 2), m1 = m0 + 64;
    const bool v0 = m0 < M, v1 = m1 < M;
    const int q0 = v0 ? m0 : 0, q1 = v1 ? m1 : 0;
    const int im0 = q0 / HW, r0 = q0 - im0 * HW, oy0 = r0 / a.Wo, ox0 = r0 - oy0 * a.Wo;
    const int im1 = q1 / HW, r1 = q1 - im1 * HW, oy1 = r1 / a.Wo, ox1 = r1 - oy1 * a.Wo;
    const int iyA = oy0 * S - P, ixA = ox0 * S - P, iyB = oy1 * S - P, ixB = ox1 * S - P;
    // activations channel-blocked, [B][C / 16][H][W][16] (VaeConvArgs): a K-tile's 16 channels of
    // consecutive pixels are consecutive 64-byte pieces, so a load instruction's 16 rows x 4 quarters
    // read 1 KB of whole cache lines (NHWC spread them over 16 lines, half of each used)
    const size_t HWi = (size_t)a.Hi * a.Wi;
    const float* pa0 = a.in + (size_t)im0 * HWi * Cin + 4 * kq;
    const float* pa1 = a.in + (size_t)im1 * HWi * Cin + 4 * kq;
    // B from the weight planes split at load: column tid / 2, k-values 8 (tid % 2) .. + 7 (16 bytes) of
    // each plane
    const size_t wps = (size_t)a.Cout * K;
    const unsigned short* pb = a.wpl + (size_t)(nt * CV_BN + (tid >> 1)) * K + 8 * (tid & 1);
    const int brow = cv_off(tid >> 1, tid & 1);
    const int hrow0 = cv_off(tid >> 2, kq >> 1) + 4 * (kq & 1), hrow1 = cv_off((tid >> 2) + 64, kq >> 1) + 4 * (kq & 1);

    // a ring of CV_D register sets (A rows m0, m1; B columns n0, n1 of one K-tile): the loads of K-tile
    // kt + 1 + CV_D are issued when tile kt + 1 has been stashed.  Depth 2, 3 and 4 measure the same
    // (15.5 / 15.6 / 15.6 ms of convolutions per 512 images): the loop is not load-latency bound.
    struct Stage {
        float4 a0, a1;  // A rows m0, m1 (fp32, split at the stash)
        uint4 b[3];     // B: hi / mid / lo (split at load)
    };
    Stage ring[CV_D];
    int ky = 0, kx = 0, c0 = 0, kl = 0;  // the next K-tile to load: tap (ky, kx), channel block c0, index kl
    // the rows' pixel pointers for the current tap, recomputed only when the tap changes (every Cin / 16
    // K-tiles); a K-tile then adds c0 (H W) of the row's channel stride.  A pixel outside the map reads a
    // zeroed 64-byte block with stride 0 (a.zero16): the loaded value is the operand, no select.
    const float *ap0 = pa0, *ap1 = pa1;
    unsigned st0 = 0, st1 = 0;
    auto tap = [&]() {
        const int iy0 = iyA + ky, ix0 = ixA + kx, iy1 = iyB + ky, ix1 = ixB + kx;
        const bool ok0 = v0 && (unsigned)iy0 < (unsigned)a.Hi && (unsigned)ix0 < (unsigned)a.Wi;
        const bool ok1 = v1 && (unsigned)iy1 < (unsigned)a.Hi && (unsigned)ix1 < (unsigned)a.Wi;
        ap0 = ok0 ? pa0 + ((size_t)iy0 * a.Wi + ix0) * 16 : a.zero16 + 4 * kq;
        ap1 = ok1 ? pa1 + ((size_t)iy1 * a.Wi + ix1) * 16 : a.zero16 + 4 * kq;
        st0 = ok0 ? (unsigned)HWi : 0u;
        st1 = ok1 ? (unsigned)HWi : 0u;
    };
    tap();
    // Loads are unconditional and their values untouched until the stash (past the last K-tile they
    // re-read valid addresses: the last weight tile; A's channel offset stays inside the map, Cin (H W)
    // at most): a select or a branch next to a load makes the compiler wait for it at once (vmcnt),
    // which serialised every K-tile on its A loads.
    auto load = [&](Stage& r) {
#ifdef VAE_DIAG_NOALOAD  // diagnostic build: A from registers, not memory (results invalid)
        r.a0 = make_float4(1.f + c0, 2.f, 3.f, 4.f);
        r.a1 = make_float4(5.f, 6.f + kx, 7.f, 8.f);
#else
        r.a0 = *(const float4*)(ap0 + (size_t)c0 * st0);
        r.a1 = *(const float4*)(ap1 + (size_t)c0 * st1);
#endif
        const int klc = kl < KT ? kl : KT - 1;
#pragma unroll
        for (int p = 0; p < 3; ++p) r.b[p] = *(const uint4*)(pb + p * wps + (size_t)klc * CV_BK);
        c0 += CV_BK;
        if (c0 == Cin) {
            c0 = 0;
            if (++kx == KS) {
                kx = 0;
                ++ky;
            }
            tap();
        }
        ++kl;
    };
    auto stash = [&](int buf, const Stage& r) {
        split3_store(r.a0, As3[buf][0], CV_BM * CV_SLD, hrow0);
        split3_store(r.a1, As3[buf][0], CV_BM * CV_SLD, hrow1);
#pragma unroll
        for (int p = 0; p < 3; ++p) *(uint4*)&Bs3[buf][p][brow] = r.b[p];
    };

    floatx16 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    auto products = [&](int buf) {
        // fp32 products on the bf16 matrix pipe: a = ah + am + al, b = bh + bm + bl exactly, and the six
        // products down to 2^-16 relative (al.bh, ah.bl, am.bm, am.bh, ah.bm, ah.bh; smallest first)
        // are accumulated in fp32 -- the dropped ones (am.bl, al.bm, al.bl) are <= 2^-24 relative, the
        // fp32 rounding level.  One 32x32x16 K-step covers the K-tile (lane half h: k = 8h .. 8h + 7,
        // the same permutation for A and B).  6 x 32 cycles of the matrix pipe per block and K-tile.
        bf16x8 ah[2], am[2], al[2], bh[2], bm[2], bl[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const int ao = cv_off(wm * 64 + 32 * i + lr, lh), bo = cv_off(wn * 64 + 32 * i + lr, lh);
            ah[i] = *(const bf16x8*)&As3[buf][0][ao];
            am[i] = *(const bf16x8*)&As3[buf][1][ao];
            al[i] = *(const bf16x8*)&As3[buf][2][ao];
            bh[i] = *(const bf16x8*)&Bs3[buf][0][bo];
            bm[i] = *(const bf16x8*)&Bs3[buf][1][bo];
            bl[i] = *(const bf16x8*)&Bs3[buf][2][bo];
        }
#define VAE_MM(X, Y)                                                                                   \
    _Pragma("unroll") for (int i = 0; i < 2; ++i) _Pragma("unroll") for (int j = 0; j < 2; ++j)         \
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(X[i], Y[j], acc[i][j], 0, 0, 0);
#ifndef VAE_DIAG_ONEMM  // diagnostic build: one product per block and K-tile instead of six (results invalid)
        VAE_MM(al, bh)
        VAE_MM(ah, bl)
        VAE_MM(am, bm)
        VAE_MM(am, bh)
        VAE_MM(ah, bm)
#else
        (void)al; (void)bl; (void)am; (void)bm;
#endif
        VAE_MM(ah, bh)
#undef VAE_MM
    };

    // prologue: K-tiles 0 .. CV_D - 1 in flight, tile 0 stashed, slot 0 refilled with tile CV_D
#pragma unroll
    for (int d = 0; d < CV_D; ++d) load(ring[d]);
    stash(0, ring[0]);
    load(ring[0]);
    __syncthreads();
    // K-tile kt: products from LDS buffer kt & 1; then tile kt + 1 (ring slot (kt + 1) % CV_D) is split
    // into the other buffer and its slot refilled with tile kt + 1 + CV_D.  Unrolled by CV_D so that the
    // ring slots are static registers.
#ifdef VAE_DIAG_NOSYNC  // diagnostic build: no barrier per K-tile (results invalid)
#define CV_SYNC() __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup")
#else
#define CV_SYNC() __syncthreads()
#endif
    // main trips: CV_D K-tiles each, every one followed by a stash and a load (no conditions)
    int kt0 = 0;
    for (; kt0 + CV_D < KT; kt0 += CV_D) {
#pragma unroll
        for (int d = 0; d < CV_D; ++d) {
            products((kt0 + d) & 1);
            stash((kt0 + d + 1) & 1, ring[(d + 1) % CV_D]);
            load(ring[(d + 1) % CV_D]);
            CV_SYNC();
        }
    }
    // the last 1 .. CV_D K-tiles
#pragma unroll
    for (int d = 0; d < CV_D; ++d) {
        const int kt = kt0 + d;
        if (kt < KT) {
            products(kt & 1);
            if (kt + 1 < KT) stash((kt + 1) & 1, ring[(d + 1) % CV_D]);
            CV_SYNC();
        }
    }
#undef CV_SYNC

    // epilogue: lane (lr, lh), register r holds row 8(r/4) + 4 lh + r%4, column lr of each block
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        const int n = nt * CV_BN + wn * 64 + 32 * j + lr;
        const float bias = a.b[n];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                const int m = mt * CV_BM + wm * 64 + 32 * i + 8 * (r >> 2) + 4 * lh + (r & 3);
                if (m < M) {
                    const int img = m / HW, pix = m - img * HW;  // channel-blocked output
                    const size_t o = ((size_t)img * a.Cout + (n & ~15)) * HW + pix * 16 + (n & 15);
                    float v = acc[i][j][r] + bias;
                    if (a.resid) v += a.resid[o];
                    if (a.relu) v = v < 0.f ? 0.f : v;  // torch.relu keeps a NaN (fmaxf would drop it)
                    a.out[o] = v;
                }
            }
    }
}

hipError_t launch_vae_conv(const VaeConvArgs& a, int ks, int stride, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    const int p = ks / 2;
    if (a.Cin % CV_BK || a.Cout % CV_BN || a.Ho != (a.Hi + 2 * p - ks) / stride + 1 ||
        a.Wo != (a.Wi + 2 * p - ks) / stride + 1)
        return hipErrorInvalidValue;
    const long long M = (long long)a.B * a.Ho * a.Wo;
    const long long grid = ((M + CV_BM - 1) / CV_BM) * (a.Cout / CV_BN);
    if (grid > 0x7fffffffLL) return hipErrorInvalidValue;
    if (ks == 3 && stride == 1)
        hipLaunchKernelGGL((vae_conv_kernel<3, 1>), dim3((unsigned)grid), dim3(256), 0, s, a);
    else if (ks == 3 && stride == 2)
        hipLaunchKernelGGL((vae_conv_kernel<3, 2>), dim3((unsigned)grid), dim3(256), 0, s, a);
    else if (ks == 1 && stride == 2)
        hipLaunchKernelGGL((vae_conv_kernel<1, 2>), dim3((unsigned)grid), dim3(256), 0, s, a);
    else
        return hipErrorInvalidValue;
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------------
// head: AdaptiveAvgPool2d((2,2)) (bin i spans [floor(i h/2), ceil((i+1) h/2))), Flatten (c*4 + i*2 + j),
// mean Linear, as two launches spread over the chip:
//   vae_pool_kernel    one workgroup per (image, 256 channels), a thread per channel and its four bins
//                      (coalesced across channels) -> feat [B][2048]
//   vae_linear_kernel  one workgroup per (4 images, 32 outputs): eight K-slices of 256 features per output,
//                      summed in a fixed order (bias, then slices 0..7), so a latent does not depend on its
//                      batch neighbours.
// (Round 3 ran both in one workgroup per 4 images, 128 workgroups with a 2048-long serial loop: 0.59 ms
// per 512 images.)
__global__ __launch_bounds__(256) void vae_pool_kernel(VaeHeadArgs a) {
    const int b = blockIdx.x, c = blockIdx.y * 256 + threadIdx.x;
    const float* in = a.in + ((size_t)b * 512 + (c & ~15)) * a.h * a.w + (c & 15);  // channel-blocked
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int y0 = (i * a.h) / 2, y1 = ((i + 1) * a.h + 1) / 2;
            const int x0 = (j * a.w) / 2, x1 = ((j + 1) * a.w + 1) / 2;
            float s = 0.f;
            for (int y = y0; y < y1; ++y)
                for (int x = x0; x < x1; ++x) s += in[((size_t)y * a.w + x) * 16];
            a.feat[(size_t)b * 2048 + c * 4 + i * 2 + j] = s / (float)((y1 - y0) * (x1 - x0));
        }
}

constexpr int HD_IMG = 4, HD_OUT = 32, HD_KS = 8;

__global__ __launch_bounds__(256) void vae_linear_kernel(VaeHeadArgs a) {
    __shared__ float fs[HD_IMG][2048];
    __shared__ float red[HD_KS][HD_IMG][HD_OUT];
    const int t = threadIdx.x, b0 = blockIdx.x * HD_IMG;
    for (int e = t; e < HD_IMG * 2048; e += 256) {
        const int q = e >> 11, f = e & 2047;
        fs[q][f] = b0 + q < a.B ? a.feat[(size_t)(b0 + q) * 2048 + f] : 0.f;
    }
    __syncthreads();
    const int ks = t / HD_OUT, ol = t % HD_OUT, o = blockIdx.y * HD_OUT + ol;
    float p[HD_IMG] = {0.f, 0.f, 0.f, 0.f};
    if (o < a.L) {
        const float* w = a.wt + o;
#pragma unroll 8
        for (int f = ks * 256; f < ks * 256 + 256; ++f) {
            const float wv = w[(size_t)f * a.L];
#pragma unroll
            for (int q = 0; q < HD_IMG; ++q) p[q] = fmaf(wv, fs[q][f], p[q]);
        }
    }
#pragma unroll
    for (int q = 0; q < HD_IMG; ++q) red[ks][q][ol] = p[q];
    __syncthreads();
    if (t < HD_IMG * HD_OUT) {
        const int q = t / HD_OUT, b = b0 + q, oo = blockIdx.y * HD_OUT + (t % HD_OUT);
        if (b < a.B && oo < a.L) {
            float s = a.b[oo];
#pragma unroll
            for (int k = 0; k < HD_KS; ++k) s += red[k][q][t % HD_OUT];
            a.latent[(size_t)b * a.L + oo] = s;
            if (a.latent64) a.latent64[(size_t)b * a.L + oo] = (double)s;
        }
    }
}

hipError_t launch_vae_head(const VaeHeadArgs& a, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    hipLaunchKernelGGL(vae_pool_kernel, dim3(a.B, 2), dim3(256), 0, s, a);
    hipLaunchKernelGGL(vae_linear_kernel, dim3((a.B + HD_IMG - 1) / HD_IMG, (a.L + HD_OUT - 1) / HD_OUT), dim3(256), 0, s, a);
    return hipGetLastError();
}

}  // namespace sdfn
