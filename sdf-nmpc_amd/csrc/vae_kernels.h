// In-loop VAE encoder kernels: csrc/vae_enc.hip.
#pragma once
#include <hip/hip_runtime.h>

namespace sdfn {

// raw depth images -> preprocessed range images [B][H][W] fp32 (sdf_nmpc/vae.py:15-24)
struct VaePreArgs {
    const void* img;   // [B][Hi][Wi] fp32 (dtype 0) or uint16 (dtype 1)
    int dtype, B, Hi, Wi, H, W;
    float clip;        // ClipDistance.dmax (preprocessing.py:91)
    const float* yz;   // [H][W] Depth2Range.yz_sqrt or nullptr (is_depth false)
    float* out;        // [B][H][W]
};

// Activations between the stem and the head are stored pre-split: three bf16 planes (hi, mid, lo; x = hi + mid
// + lo exactly, each the bf16 truncation of the remainder), plane p at p * ps elements, each in the
// channel-blocked order [B][C/16][H][W][16].  A convolution then stages its operand tiles from memory
// straight into LDS (global_load_lds), with no split on the vector ALU.
// conv7x7/2 (+bias) + ELU + maxpool3/2 (vae.py:19-21), output as planes [3][B][64/16][Hp][Wp][16]
struct VaeStemArgs {
    const float* in;   // [B][H][W]
    const unsigned short* wpl;  // [3][64 n][64 k] bf16 bits: the weights split hi / mid / lo, slot k holding
                                // tap vae_stem_slot_tap(k)
    const float* b;    // [64]
    unsigned short* out;  // planes, plane stride ops
    size_t ops;
    int B, H, W, Hc, Wc, Hp, Wp;
    int out_ph;  // output columns in parity-phase order (vae_col): the next layer is a stride-2 convolution
};
constexpr int VAE_STEM_PLANE = 64 * 64;

// Parity-phase column order of a map of width W: the even columns first, then the odd ones.  A stride-2
// convolution's taps then read consecutive output columns from consecutive stored columns (32 B apart in
// a channel-blocked plane instead of 64), halving the cache lines its activation loads touch.  Maps read by
// a stride-2 convolution are stored in this order; the others in natural order.
__host__ __device__ inline int vae_col(int x, int W, int ph) { return ph ? ((x & 1) ? ((W + 1) >> 1) : 0) + (x >> 1) : x; }  // bf16 per plane of VaeStemArgs::wpl

// The stem's K order: slot k of a plane row holds tap vae_stem_slot_tap(k) = ky * 7 + kx (-1: zero).
// Slots pair up (2p, 2p + 1).  Pairs 0..17, 20, 21 are horizontal neighbours (ky, kx), (ky, kx + 1) with kx
// even, read from the patch as one 32-bit word; pairs 18, 19, 22 join two rows' kx = 6 taps and pair 23 is
// (6, 4), (6, 5), read as two 16-bit values (the "general" pairs: K-step 2, slots 2 and 3 of both lane
// halves).  Slot 48 is tap (6, 6), applied on the vector ALU; 49..63 are zero.
constexpr bool vae_stem_general_pair(int p) { return p == 18 || p == 19 || p == 22 || p == 23; }
constexpr int vae_stem_slot_tap(int k) {
    if (k == 48) return 48;
    if (k > 48 || k < 0) return -1;
    const int p = k / 2, h = k % 2;
    if (p == 18 || p == 19 || p == 22) {
        const int r = 2 * (p == 18 ? 0 : p == 19 ? 1 : 2) + h;  // rows 0..5, column 6
        return r * 7 + 6;
    }
    if (p == 23) return 6 * 7 + 4 + h;
    const int m = p < 18 ? p : p - 2;  // adjacent pairs 0..19
    return (m / 3) * 7 + 2 * (m % 3) + h;
}
constexpr bool vae_stem_order_ok() {  // every tap exactly once; horizontal pairs start at an even column
    int seen[49] = {};
    for (int k = 0; k < 64; ++k) {
        const int t = vae_stem_slot_tap(k);
        if (t < 0) continue;
        if (t > 48 || seen[t]++) return false;
        if (k < 48 && k % 2 == 0 && !vae_stem_general_pair(k / 2) &&
            (t % 7 % 2 != 0 || vae_stem_slot_tap(k + 1) != t + 1))
            return false;
    }
    for (int t = 0; t < 49; ++t)
        if (!seen[t]) return false;
    return true;
}
static_assert(vae_stem_order_ok(), "stem K order");

// implicit-GEMM convolution (BatchNorm folded) + bias (+ residual) (+ ReLU); activations channel-blocked,
// [B][C/16][H][W][16]
struct VaeConvArgs {
    const unsigned short* in;  // planes [3][B][Cin/16][Hi][Wi][16], plane stride ips
    size_t ips;
    const float* w;      // [Cout][KS][KS][Cin]
    const unsigned short* wpl;  // the same weights split into bf16 planes [3 hi/mid/lo][Cout/128][K/16][128][16]
                                // (K-tile slabs, row halves swapped on row bit 3; at load)
    const float* b;      // [Cout]
    const unsigned short* zero;  // 32 zero bytes (16-byte aligned): what a tap outside the map reads
    const float* resid;  // fp32 [B][Cout/16][Ho][Wo][16], or nullptr
    const unsigned short* resid_pl;  // or the residual as planes (plane stride rps), or nullptr
    size_t rps;
    float* out;          // fp32 [B][Cout/16][Ho][Wo][16], or nullptr
    unsigned short* out_pl;  // or the output as planes (plane stride ops), or nullptr
    size_t ops;
    int B, Hi, Wi, Cin, Ho, Wo, Cout, relu;
    int in_ph, out_ph, res_ph;  // which of in / out / resid keep their columns in parity-phase order (vae_col)
};

// AdaptiveAvgPool2d((2,2)) + Flatten + mean Linear (vae.py:26-30, 42-43)
struct VaeHeadArgs {
    const unsigned short* in;  // planes [3][B][512/16][h][w][16], plane stride ips
    size_t ips;
    float* feat;         // [B][2048] workspace: the pooled, flattened features
    const float* wt;     // [2048][L]  (transposed mean.weight)
    const float* b;      // [L]
    float* latent;       // [B][L]
    double* latent64;    // [B][L] or nullptr
    int B, h, w, L;
};

hipError_t launch_vae_pre(const VaePreArgs& a, hipStream_t s);
hipError_t launch_vae_stem(const VaeStemArgs& a, int n_cu, hipStream_t s);  // n_cu: the device's CUs (sdfnmpc_ctx::n_cu)
hipError_t launch_vae_conv(const VaeConvArgs& a, int ks, int stride, hipStream_t s);
hipError_t launch_vae_head(const VaeHeadArgs& a, hipStream_t s);

}  // namespace sdfn
