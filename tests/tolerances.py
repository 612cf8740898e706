"""Parity bars, written once and used by every test.

SDF (fp32 network; BASELINE north_star "SDF cost/gradient within 1e-5 rel fp32"):
  * df       |df - df_ref|          <= 1e-5 * max(|df_ref|, max_df)      max_df = 1 m, the truncation
                                                                         scale of the SDF (neural_df.py:18)
  * d df/dp  ||g - g_ref||_2        <= 1e-5 * max(||g_ref||_2, 1)        1 = eikonal scale |grad SDF|
  measured against BOTH the reference fp32 (torch CPU, what L4CasADi runs) and fp64 outputs.
  Rationale: the reference's own fp32 path differs from its fp64 evaluation by up to 1.3e-7 in df and
  1.2e-5 normwise-relative in the gradient on the same inputs, so a relative bar with a
  floor below fp32 resolution would reject the reference itself.
Ill-conditioned stress weights (x3 gain + biases, tests the sin range reduction): the kernel may be no
worse than STRESS_FACTOR x the reference fp32's own error vs fp64 on the same cases.
Linearisation (fp64): rtol 1e-9 / atol 1e-12 (x scale) against the fp64 oracle; entries fed by the fp32
network (h[2], J_h row 2) follow the SDF bar.
Shooting grid: bit-exact.
"""
import numpy as np

DF_RTOL = 1e-5
GRAD_RTOL = 1e-5
MAX_DF = 1.0
STRESS_FACTOR = 2.0
LIN_RTOL = 1e-9


def sdf_df_err(df, ref, max_df=MAX_DF):
    return np.max(np.abs(np.asarray(df, np.float64) - ref) / np.maximum(np.abs(ref), max_df))


def sdf_grad_err(g, ref):
    g = np.asarray(g, np.float64)
    return np.max(np.linalg.norm(g - ref, axis=-1) / np.maximum(np.linalg.norm(ref, axis=-1), 1.0))


def sdf_df_ok(df, ref, max_df=MAX_DF):
    return sdf_df_err(df, ref, max_df) <= DF_RTOL


def sdf_grad_ok(g, ref):
    return sdf_grad_err(g, ref) <= GRAD_RTOL


def lin_close(got, want, rtol=LIN_RTOL):
    scale = max(1.0, float(np.abs(want).max()))
    return float(np.abs(np.asarray(got) - want).max()) <= rtol * scale

# VAE encoder (fp32 network).  The reference's own fp32 torch encoder differs from
# its fp64 evaluation by 2.8e-7 x max|latent| on the golden images; the GPU kernels (exact-fp32 MFMA
# products, BatchNorm folded into the convolutions, a different summation order) are held to the
# north-star fp32 bar, 1e-5 relative to the latent's scale, against the fp64 reference outputs.
VAE_LATENT_RTOL = 1e-5
# preprocessing: torch's vectorised fp32 sqrt (Depth2Range table) is within 1 ulp of the correctly
# rounded one (values <= 1 after the clip: 1 ulp <= 1.2e-7); Reshape's bilinear resize in torch fp32
# is itself 1e-4 away from its fp64 evaluation on 0..6 m inputs, ours within 2e-5 m -> 4e-6 after /dmax.
VAE_PRE_ATOL = 1.2e-7
VAE_RESIZE_ATOL = 1e-5


def vae_latent_err(lat, ref):
    ref = np.asarray(ref, np.float64)
    return float(np.abs(np.asarray(lat, np.float64) - ref).max() / np.abs(ref).max())
