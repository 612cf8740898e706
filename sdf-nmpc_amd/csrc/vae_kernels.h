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

// conv7x7/2 (+bias) + ELU + maxpool3/2 (vae.py:19-21), NHWC output [B][Hp][Wp][64]
struct VaeStemArgs {
    const float* in;   // [B][H][W]
    const float* w;    // [7][7][64]   (tap-major: one uniform 64-channel row per tap)
    const float* b;    // [64]
    float* out;        // [B][Hp][Wp][64]
    int B, H, W, Hc, Wc, Hp, Wp;
};

// implicit-GEMM convolution (BatchNorm folded) + bias (+ residual) (+ ReLU), NHWC
struct VaeConvArgs {
    const float* in;     // [B][Hi][Wi][Cin]
    const float* w;      // [Cout][KS][KS][Cin]
    const float* b;      // [Cout]
    const float* resid;  // [B][Ho][Wo][Cout] or nullptr
    float* out;          // [B][Ho][Wo][Cout]
    int B, Hi, Wi, Cin, Ho, Wo, Cout, relu;
};

// AdaptiveAvgPool2d((2,2)) + Flatten + mean Linear (vae.py:26-30, 42-43)
struct VaeHeadArgs {
    const float* in;     // [B][h][w][512]
    const float* wt;     // [2048][L]  (transposed mean.weight)
    const float* b;      // [L]
    float* latent;       // [B][L]
    double* latent64;    // [B][L] or nullptr
    int B, h, w, L;
};

hipError_t launch_vae_pre(const VaePreArgs& a, hipStream_t s);
hipError_t launch_vae_stem(const VaeStemArgs& a, hipStream_t s);
hipError_t launch_vae_conv(const VaeConvArgs& a, int ks, int stride, hipStream_t s);
hipError_t launch_vae_head(const VaeHeadArgs& a, hipStream_t s);

}  // namespace sdfn
