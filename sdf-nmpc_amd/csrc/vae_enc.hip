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

#include <cstdint>
#include <numeric>
#include <type_traits>
#include <utility>

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

// x = hi + mid + lo exactly, each a bf16 truncation of the remainder
__device__ __forceinline__ void split3(float x, unsigned& h, unsigned& m, unsigned& l) {
    h = __float_as_uint(x) & 0xffff0000u;
    const float r1 = x - __uint_as_float(h);
    m = __float_as_uint(r1) & 0xffff0000u;
    const float r2 = r1 - __uint_as_float(m);
    l = __float_as_uint(r2) & 0xffff0000u;
}

// four consecutive channels of one pixel into the three planes (8-byte stores), and back: (hi + mid) + lo is
// the fp32 value exactly (hi + mid drops only the low 8 bits, representable)
__device__ __forceinline__ void store_planes4(unsigned short* pl, size_t ps, size_t o, float4 v) {
    unsigned h[4], m[4], l[4];
    split3(v.x, h[0], m[0], l[0]);
    split3(v.y, h[1], m[1], l[1]);
    split3(v.z, h[2], m[2], l[2]);
    split3(v.w, h[3], m[3], l[3]);
    *(uint2*)&pl[o] = make_uint2((h[0] >> 16) | h[1], (h[2] >> 16) | h[3]);
    *(uint2*)&pl[ps + o] = make_uint2((m[0] >> 16) | m[1], (m[2] >> 16) | m[3]);
    *(uint2*)&pl[2 * ps + o] = make_uint2((l[0] >> 16) | l[1], (l[2] >> 16) | l[3]);
}
__device__ __forceinline__ float bf_lo(unsigned u) { return __uint_as_float(u << 16); }
__device__ __forceinline__ float bf_hi(unsigned u) { return __uint_as_float(u & 0xffff0000u); }
__device__ __forceinline__ float4 load_planes4(const unsigned short* pl, size_t ps, size_t o) {
    const uint2 h = *(const uint2*)&pl[o], m = *(const uint2*)&pl[ps + o], l = *(const uint2*)&pl[2 * ps + o];
    return make_float4((bf_lo(h.x) + bf_lo(m.x)) + bf_lo(l.x), (bf_hi(h.x) + bf_hi(m.x)) + bf_hi(l.x),
                       (bf_lo(h.y) + bf_lo(m.y)) + bf_lo(l.y), (bf_hi(h.y) + bf_hi(m.y)) + bf_hi(l.y));
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
            const size_t oo = ((size_t)img * 64 + (c4 & ~15)) * a.Hp * a.Wp + (py * a.Wp + vae_col(px, a.Wp, a.out_ph)) * 16 + (c4 & 15);
#ifdef STEM_DIAG_NOPOOL  // diagnostic builds only (tools/build_variant.sh)
            store_planes4(a.out, a.ops, oo, *(const float4*)&conv[((2 * pyl + 1) * ST_CX + 2 * pxl + 1) * ST_CS + c4]);
#else
            float4 v[9];
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx)
                    v[3 * dy + dx] = *(const float4*)&conv[((2 * pyl + dy) * ST_CX + 2 * pxl + dx) * ST_CS + c4];
#ifdef STEM_DIAG_NOELU
            store_planes4(a.out, a.ops, oo, make_float4(max9(v, 0), max9(v, 1), max9(v, 2), max9(v, 3)));
#else
            const float2v e0 = elu2(float2v{max9(v, 0), max9(v, 1)}), e1 = elu2(float2v{max9(v, 2), max9(v, 3)});
            // channel-blocked output [B][4][Hp][Wp][16] (the convolutions' layout), as planes
            store_planes4(a.out, a.ops, oo, make_float4(e0.x, e0.y, e1.x, e1.y));
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
// k = (ci / 16, ky, kx, ci % 16).  Tile 128 x 128 x 16, 4 waves as 2 x 2 of 64 x 64 (four 32x32 MFMA blocks each).
// Both operands arrive split into bf16 planes -- the activations by the layer that produced them, the
// weights at load -- so a K-tile is staged from memory straight into LDS by LDS-DMA (global_load_lds, 16
// bytes per lane): three A and three B loads per thread, no vector-ALU work and no register staging.  Three
// LDS buffers: tiles kt + 1 and kt + 2 are in flight under the products of tile kt; one barrier per tile.
// LDS plane rows are 16 bf16 (32 B) with the two 16-byte halves of rows 8..15 of every 16 swapped (row bit
// 3), so the lane groups of the fragments' ds_read_b128 hit 16 distinct 16-byte slots.  LDS-DMA writes a
// wave's loads lane-linearly (base + 16 lane), so the swap is made on the SOURCE side: for A, lane 2 r + h
// of the wave's 32 rows loads half h ^ bit3(row) of its row; B is stored at load as the LDS image of each
// K-tile (4 KB slabs), so a wave's B load is 1 KB contiguous (8 cache lines, not 32 rows K apart: the
// texture-address unit's work per tile, which bounds this kernel, drops by half).  The reads apply the
// same involution (cv_off).
// Within a K-tile, MFMA step s feeds lane half h with k = 8h + s (the same permutation for A and B).
// The weight fragment is the MFMA's first operand, so the accumulator is C^T: a lane ends with four
// consecutive channels of one pixel per register quad (8-byte plane stores, 16-byte fp32 stores).
constexpr int CV_BK = 16;
__device__ __forceinline__ int cv_off(int row, int half) { return row * 16 + 8 * (half ^ ((row >> 3) & 1)); }
template <class T>
__device__ __forceinline__ void cv_tie(T& x) { asm volatile("" : "+v"(x)); }
// f(integral_constant<int, I>) for I = 0, 1, ... in order
template <class F, int... I>
__device__ __forceinline__ void cv_static_for(F&& f, std::integer_sequence<int, I...>) {
    (f(std::integral_constant<int, I>{}), ...);
}

// WM x WN 32x32 blocks per wave, 2 x 2 waves: a (64 WM) x (64 WN) workgroup tile; NB LDS buffers.
template <int KS, int S, int WM, int WN, int NB>
__global__ __launch_bounds__(256, 2) void vae_conv_kernel(VaeConvArgs a) {
    constexpr int P = KS / 2, BM = 64 * WM, BN = 64 * WN, RA = BM / 128, RB = BN / 128;
    constexpr int NV = 3 * (RA + RB);  // LDS-DMA loads per thread and K-tile
    typedef __attribute__((address_space(3))) void ldsv;
    // one LDS object per buffer and operand, each addressed with a compile-time buffer index: the compiler
    // then tells a buffer's fragment reads from the LDS-DMA into the other buffers (one shared object
    // indexed at run time makes every ds_read wait for all DMA in flight, vmcnt(0))
    __shared__ __align__(16) unsigned short A0[3][BM * 16], A1[3][BM * 16], A2[NB > 2 ? 3 : 1][BM * 16];
    __shared__ __align__(16) unsigned short B0[3][BN * 16], B1[3][BN * 16], B2[NB > 2 ? 3 : 1][BN * 16];
    auto As = [&](auto bc) -> unsigned short(*)[BM * 16] {
        constexpr int b = decltype(bc)::value;
        if constexpr (b == 0) return A0;
        else if constexpr (b == 1) return A1;
        else return A2;
    };
    auto Bs = [&](auto bc) -> unsigned short(*)[BN * 16] {
        constexpr int b = decltype(bc)::value;
        if constexpr (b == 0) return B0;
        else if constexpr (b == 1) return B1;
        else return B2;
    };
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1, lr = lane & 31, lh = lane >> 5;
    const int M = a.B * a.Ho * a.Wo, MT = (M + BM - 1) / BM;
    const int nt = blockIdx.x / MT, mt = blockIdx.x - nt * MT;
    const int Cin = a.Cin, K = KS * KS * Cin, KT = K / CV_BK;

    // the A rows this thread stages (pixels 128 r + 32 wave + lane / 2) and which half of them
    const int srow = 32 * wave + (lane >> 1), shalf = (lane & 1) ^ ((srow >> 3) & 1);
    const int HW = a.Ho * a.Wo;
    const size_t HWi = (size_t)a.Hi * a.Wi;
    int iy0[RA], ix0[RA];
    bool vm[RA];
    const unsigned short* pa[RA];
#pragma unroll
    for (int r = 0; r < RA; ++r) {
        const int m0 = mt * BM + 128 * r + srow;
        vm[r] = m0 < M;
        const int q0 = vm[r] ? m0 : 0;
        const int im = q0 / HW, r0 = q0 - im * HW, oy = r0 / a.Wo, ox = r0 - oy * a.Wo;
        iy0[r] = oy * S - P;
        ix0[r] = ox * S - P;
        pa[r] = a.in + (size_t)im * HWi * Cin + 8 * shalf;  // channel-blocked planes
    }
    const size_t wps = (size_t)a.Cout * K;
    // B: the weights' K-tile slabs (the LDS image of 128 channels x 16 k), loaded lane-linearly
    const unsigned short* pb = a.wpl + (size_t)nt * RB * KT * (128 * CV_BK) + 8 * tid;
    // the rows' nine tap pixels, once: element offset of tap t = ky KS + kx within the row's image plane
    // (channel block 0), or ~0u outside the map (the tile then reads the zero block with strides 0).  The
    // K loop is unrolled over a channel block's KS KS taps, so the tap index is a compile-time constant.
    constexpr int NT = KS * KS;
    unsigned toff[RA][NT];
#pragma unroll
    for (int r = 0; r < RA; ++r)
#pragma unroll
        for (int t = 0; t < NT; ++t) {
            const int iy = iy0[r] + t / KS, ix = ix0[r] + t % KS;
            const bool ok = vm[r] && (unsigned)iy < (unsigned)a.Hi && (unsigned)ix < (unsigned)a.Wi;
            toff[r][t] = ok ? (unsigned)((iy * a.Wi + vae_col(ix, a.Wi, a.in_ph)) * 16) : ~0u;
        }
    int kl = 0;                // next K-tile to stage
    size_t cofs = 0;           // its channel block's element offset (c0 H W)
    // K-tile kl (tap tc, K order (channel block, ky, kx)) into LDS buffer bc (per load, a wave's 32 rows of
    // a plane: 1 KB), then advance
    auto issue = [&](auto bc, auto tc) {
        constexpr int t = decltype(tc)::value;
        auto* LA = As(bc);
        auto* LB = Bs(bc);
        if (t == 0 && kl > 0) cofs += (size_t)CV_BK * HWi;  // the next channel block
#ifndef VAE_DIAG_NOISSUE  // diagnostic build: no staging loads at all (results invalid)
        const unsigned short* ap[RA];
        size_t pst[RA];
#pragma unroll
        for (int r = 0; r < RA; ++r) {
            const bool ok = toff[r][t] != ~0u;
            ap[r] = ok ? pa[r] + cofs + toff[r][t] : a.zero + 8 * shalf;
            pst[r] = ok ? a.ips : 0;
        }
#pragma unroll
        for (int p = 0; p < 3; ++p) {
#ifndef VAE_DIAG_NOA  // diagnostic build: no A staging loads (results invalid)
#pragma unroll
            for (int r = 0; r < RA; ++r)
                __builtin_amdgcn_global_load_lds((const void*)(ap[r] + p * pst[r]),
                                                 (ldsv*)&LA[p][2048 * r + 512 * wave], 16, 0, 0);
#endif
#ifndef VAE_DIAG_NOB  // diagnostic build: no B staging loads (results invalid)
#pragma unroll
            for (int r = 0; r < RB; ++r)
                __builtin_amdgcn_global_load_lds((const void*)(pb + ((size_t)r * KT + kl) * (128 * CV_BK) + p * wps),
                                                 (ldsv*)&LB[p][2048 * r + 512 * wave], 16, 0, 0);
#endif
        }
#else
        (void)LA; (void)LB;
#endif
        ++kl;
    };

    floatx16 acc[WM][WN];
#pragma unroll
    for (int i = 0; i < WM; ++i)
#pragma unroll
        for (int j = 0; j < WN; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

    auto products = [&](auto bc) {
        const auto* LA = As(bc);
        const auto* LB = Bs(bc);
        // fp32 products on the bf16 matrix pipe: a = ah + am + al, b = bh + bm + bl exactly, and the six
        // products down to 2^-16 relative (al.bh, ah.bl, am.bm, am.bh, ah.bm, ah.bh; smallest first)
        // are accumulated in fp32 -- the dropped ones (am.bl, al.bm, al.bl) are <= 2^-24 relative, the
        // fp32 rounding level.  One 32x32x16 K-step covers the K-tile.  6 x 32 cycles of the matrix pipe
        // per block and K-tile.
        // Fragment reads are inline ds_read_b128: the compiler cannot see their LDS access, so it adds no
        // wait for the LDS-DMA in flight (it would wait for all of it after every loop merge); the vmcnt +
        // barrier of the step order them after this tile's DMA.  Each lgkmcnt wait is followed by empty
        // asm "redefining" the fragments it covers, so no MFMA is scheduled above it.
        bf16x8 ah[WM], am[WM], al[WM], bh[WN], bm[WN], bl[WN];
        const unsigned la = (unsigned)(uintptr_t)(const ldsv*)&LA[0][0];
        const unsigned lb = (unsigned)(uintptr_t)(const ldsv*)&LB[0][0];
#define VAE_DSR(R, ADDR, OFF) asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(R) : "v"(ADDR), "i"(OFF))
        unsigned ao[WM], bo[WN];
#pragma unroll
        for (int i = 0; i < WM; ++i) {
            ao[i] = la + 2 * cv_off(wm * 32 * WM + 32 * i + lr, lh);
            VAE_DSR(ah[i], ao[i], 0);
            VAE_DSR(al[i], ao[i], 2 * BM * 16 * 2);
        }
#pragma unroll
        for (int j = 0; j < WN; ++j) {
            bo[j] = lb + 2 * cv_off(wn * 32 * WN + 32 * j + lr, lh);
            VAE_DSR(bh[j], bo[j], 0);
            VAE_DSR(bl[j], bo[j], 2 * BN * 16 * 2);
        }
#pragma unroll
        for (int i = 0; i < WM; ++i) VAE_DSR(am[i], ao[i], BM * 16 * 2);
#pragma unroll
        for (int j = 0; j < WN; ++j) VAE_DSR(bm[j], bo[j], BN * 16 * 2);
#undef VAE_DSR
        // the mid planes arrive under the first 2 WM WN MFMAs
        asm volatile("s_waitcnt lgkmcnt(%0)" ::"i"(WM + WN));
#pragma unroll
        for (int i = 0; i < WM; ++i) {
            cv_tie(ah[i]);
            cv_tie(al[i]);
        }
#pragma unroll
        for (int j = 0; j < WN; ++j) {
            cv_tie(bh[j]);
            cv_tie(bl[j]);
        }
#define VAE_MM(X, Y)                                                                                   \
    _Pragma("unroll") for (int i = 0; i < WM; ++i) _Pragma("unroll") for (int j = 0; j < WN; ++j)       \
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(Y[j], X[i], acc[i][j], 0, 0, 0);
        VAE_MM(al, bh)
        VAE_MM(ah, bl)
#pragma unroll
        for (int i = 0; i < WM; ++i)
#pragma unroll
            for (int j = 0; j < WN; ++j) cv_tie(acc[i][j]);  // those MFMAs stay above the second wait
        asm volatile("s_waitcnt lgkmcnt(0)");
#pragma unroll
        for (int i = 0; i < WM; ++i) cv_tie(am[i]);
#pragma unroll
        for (int j = 0; j < WN; ++j) cv_tie(bm[j]);
        VAE_MM(am, bm)
        VAE_MM(am, bh)
        VAE_MM(ah, bm)
        VAE_MM(ah, bh)
#undef VAE_MM
    };

    // K-tile kt (buffer kt % NB): wait for this thread's DMA of it (VMEM operations of a wave complete in
    // order, so the NV loads of the tile after it may stay in flight), then a barrier (every thread's DMA
    // of tile kt has landed; every wave's reads of the buffer about to be refilled are done), stage tile
    // kt + NB - 1, and the products of tile kt under the tiles in flight.
    // Steps are unrolled over L = lcm(NB, KS KS) K-tiles (9 for 3x3: a channel block; NB for 1x1), so
    // buffer and tap are compile-time constants; 3x3 layers have KT = 9 Cin / 16, a multiple of 9.
    constexpr int L = std::lcm(NB, KS > 1 ? NT : 1);
    auto stepc = [&](int kt, auto sc) {
        constexpr int s = decltype(sc)::value;
        using BC = std::integral_constant<int, s % NB>;
        using BN = std::integral_constant<int, (s + NB - 1) % NB>;
        using TN = std::integral_constant<int, (s + NB - 1) % (KS > 1 ? NT : 1)>;
        if constexpr (NB == 3) {
#ifdef VAE_DIAG_NOWAIT  // diagnostic build: the products do not wait for the DMA (results invalid)
            if (kt + 1 < KT) asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
#else
            if (kt + 1 < KT) asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::"i"(NV) : "memory");
#endif
            else asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        } else {
            asm volatile("s_waitcnt vmcnt(0)\n\ts_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
        }
        if (kt + NB - 1 < KT) issue(BN{}, TN{});
        products(BC{});
    };
    // prologue: tiles 0 .. NB - 2
    issue(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
    if constexpr (NB == 3)
        if (KT > 1) issue(std::integral_constant<int, 1>{}, std::integral_constant<int, (KS > 1 ? 1 : 0)>{});
    int kt = 0;
    for (; kt + L <= KT; kt += L)
        cv_static_for([&](auto sc) { stepc(kt + decltype(sc)::value, sc); }, std::make_integer_sequence<int, L>{});
    // the last KT % L tiles (none for the encoder's 3x3 layers)
    cv_static_for([&](auto sc) { if (kt + decltype(sc)::value < KT) stepc(kt + decltype(sc)::value, sc); },
                  std::make_integer_sequence<int, L - 1>{});

    // epilogue (C^T): lane (lr, lh) holds pixel 32 i + lr of the wave's rows and, in register quad g,
    // channels 32 j + 8 g + 4 lh .. + 3
#pragma unroll
    for (int i = 0; i < WM; ++i) {
        const int m = mt * BM + wm * 32 * WM + 32 * i + lr;
        if (m >= M) continue;
        const int img = m / HW, pix = m - img * HW, oy = pix / a.Wo, ox = pix - oy * a.Wo;
        const int po = oy * a.Wo + vae_col(ox, a.Wo, a.out_ph), pr = oy * a.Wo + vae_col(ox, a.Wo, a.res_ph);
#pragma unroll
        for (int j = 0; j < WN; ++j)
#pragma unroll
            for (int g = 0; g < 4; ++g) {
                const int n = nt * BN + wn * 32 * WN + 32 * j + 8 * g + 4 * lh;
                const size_t cb = ((size_t)img * a.Cout + (n & ~15)) * HW + (n & 15);
                const size_t o = cb + po * 16, orr = cb + pr * 16;
                const float4 bias = make_float4(a.b[n], a.b[n + 1], a.b[n + 2], a.b[n + 3]);
                float4 v = make_float4(acc[i][j][4 * g] + bias.x, acc[i][j][4 * g + 1] + bias.y,
                                       acc[i][j][4 * g + 2] + bias.z, acc[i][j][4 * g + 3] + bias.w);
                if (a.resid || a.resid_pl) {
                    const float4 rv = a.resid ? *(const float4*)&a.resid[orr] : load_planes4(a.resid_pl, a.rps, orr);
                    v = make_float4(v.x + rv.x, v.y + rv.y, v.z + rv.z, v.w + rv.w);
                }
                if (a.relu)  // torch.relu keeps a NaN (fmaxf would drop it)
                    v = make_float4(v.x < 0.f ? 0.f : v.x, v.y < 0.f ? 0.f : v.y, v.z < 0.f ? 0.f : v.z, v.w < 0.f ? 0.f : v.w);
                if (a.out_pl) store_planes4(a.out_pl, a.ops, o, v);
                else *(float4*)&a.out[o] = v;
            }
    }
}

// The product tile is 128 x 128 with three LDS buffers.  (Round 5 measured a 128 x 256 / 256 x 128 tile
// with two buffers -- 48 MFMAs per wave and barrier -- at 11.39-11.5 vs 11.26-11.31 ms per 512 images;
// the template keeps WM, WN, NB as parameters.)
template <int KS, int S>
static void cv_launch(const VaeConvArgs& a, long long M, hipStream_t s) {
    const long long g = ((M + 127) / 128) * (a.Cout / 128);
    hipLaunchKernelGGL((vae_conv_kernel<KS, S, 2, 2, 3>), dim3((unsigned)g), dim3(256), 0, s, a);
}

hipError_t launch_vae_conv(const VaeConvArgs& a, int ks, int stride, hipStream_t s) {
    if (a.B <= 0) return hipSuccess;
    const int p = ks / 2;
    if (a.Cin % CV_BK || a.Cout % 128 || a.Ho != (a.Hi + 2 * p - ks) / stride + 1 ||
        a.Wo != (a.Wi + 2 * p - ks) / stride + 1 || !a.in || !a.wpl || !a.zero || (!a.out && !a.out_pl) ||
        ((uintptr_t)a.in & 15) || (a.ips & 7) || ((uintptr_t)a.zero & 15))
        return hipErrorInvalidValue;
    const long long M = (long long)a.B * a.Ho * a.Wo;
    if ((M + 127) / 128 * (a.Cout / 128) > 0x7fffffffLL) return hipErrorInvalidValue;
    if (ks == 3 && stride == 1)
        cv_launch<3, 1>(a, M, s);
    else if (ks == 3 && stride == 2)
        cv_launch<3, 2>(a, M, s);
    else if (ks == 1 && stride == 2)
        cv_launch<1, 2>(a, M, s);
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
    const size_t ci = ((size_t)b * 512 + (c & ~15)) * a.h * a.w + (c & 15);  // channel-blocked planes
    const unsigned short *in = a.in + ci, *in1 = in + a.ips, *in2 = in + 2 * a.ips;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) {
            const int y0 = (i * a.h) / 2, y1 = ((i + 1) * a.h + 1) / 2;
            const int x0 = (j * a.w) / 2, x1 = ((j + 1) * a.w + 1) / 2;
            float s = 0.f;
            for (int y = y0; y < y1; ++y)
                for (int x = x0; x < x1; ++x) {
                    const size_t e = ((size_t)y * a.w + x) * 16;  // (hi + mid) + lo: the fp32 value
                    s += (__uint_as_float((unsigned)in[e] << 16) + __uint_as_float((unsigned)in1[e] << 16)) +
                         __uint_as_float((unsigned)in2[e] << 16);
                }
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
