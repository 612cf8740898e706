"""Time the in-loop VAE encoder (csrc/vae_enc.hip) at batch B: ms per encode, TFLOP/s, per-kernel split."""
import sys
import time

import numpy as np
import torch

import os  # noqa: E402
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sdf_nmpc_amd import _lib, synth  # noqa: E402
from sdf_nmpc_amd import vae as V  # noqa: E402
from sdf_nmpc_amd.config import Config  # noqa: E402


def main(B=512, steps=10):
    if os.environ.get("SDFNMPC_LIB"):  # a diagnostic build (tools/build_variant.sh)
        _lib.LIB_PATH = os.environ["SDFNMPC_LIB"]
    cfg = Config()
    ctx = _lib.Context(0, stream=torch.cuda.current_stream().cuda_stream)
    spec = V.DEFAULT_ENCODER
    vae = _lib.Vae(ctx, V.pack(spec, V.synthetic_encoder(spec, 0)))
    imgs = torch.from_numpy(synth.depth_images(8, 270, 480, seed=1)).cuda().repeat(B // 8, 1, 1).contiguous()
    yz = torch.from_numpy(V.depth2range_table((270, 480), cfg.sensor.hfov, cfg.sensor.vfov)).cuda()
    lat = torch.empty(B, 128, device="cuda")
    opts = _lib.vae_opts(cfg, 5.0)
    for _ in range(2):
        _lib.vae_encode(ctx, vae, opts, imgs, yz, lat)
    torch.cuda.synchronize()
    ctx.enable_timing(True)
    ctx.reset_stats()
    t = time.perf_counter()
    for _ in range(steps):
        _lib.vae_encode(ctx, vae, opts, imgs, yz, lat)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    fl = spec.n_flops() * B
    print(f"{_lib.LIB_PATH[-32:]} B={B}: {dt*1e3:.3f} ms/encode  {fl/dt/1e12:.1f} TFLOP/s  ({B/dt:.0f} images/s)")
    for k in ("vae_pre", "vae_stem", "vae_conv", "vae_head"):
        ms, n = ctx.kernel_stats(k)
        print(f"  {k:10s} {ms/steps:.3f} ms/encode ({n//steps} launches)")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 512)
