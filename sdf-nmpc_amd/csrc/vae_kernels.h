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

// conv7x7/2 (+bias) + ELU + maxpool3/2 (vae.py:19-21), channel-blocked output [B][64/16][Hp][Wp][16]
struct VaeStemArgs {
    const float* in;   // [B][H][W]
    const unsigned short* wpl;  // [3][64 n][64 k] bf16 bits: the weights split hi / mid / lo, slot k holding
                                // tap vae_stem_slot_tap(k)
    const float* b;    // [64]
    float* out;        // [B][4][Hp][Wp][16]
    int B, H, W, Hc, Wc, Hp, Wp;
};
constexpr int VAE_STEM_PLANE = 64 * 64;  // bf16 per plane of VaeStemArgs::wpl

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
    const float* in;     // [B][Cin/16][Hi][Wi][16]
    const float* w;      // [Cout][KS][KS][Cin]
    const unsigned short* wpl;  // the same weights split into bf16 planes [3 hi/mid/lo][Cout][KS KS Cin] (at load)
    const float* b;      // [Cout]
    const float* zero16; // 16 zero floats (64 B, 16-byte aligned): what a tap outside the map reads
    const float* resid;  // [B][Cout/16][Ho][Wo][16] or nullptr
    float* out;          // [B][Cout/16][Ho][Wo][16]
    int B, Hi, Wi, Cin, Ho, Wo, Cout, relu;
};

// AdaptiveAvgPool2d((2,2)) + Flatten + mean Linear (vae.py:26-30, 42-43)
struct VaeHeadArgs {
    const float* in;     // [B][512/16][h][w][16]
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
