"""Time the preparation phase with the C5 wide net ([1024,1024,512,256]) at B x N (default 512 x 60)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sdf_nmpc_amd import _lib, synth, weights as W  # noqa: E402
from sdf_nmpc_amd.config import Config  # noqa: E402


def main(B=512, N=60, steps=10):
    if os.environ.get("SDFNMPC_LIB"):  # a diagnostic build (tools/build_variant.sh)
        _lib.LIB_PATH = os.environ["SDFNMPC_LIB"]
    cfg = Config(mpc__N=N)
    ctx = _lib.Context(0, stream=torch.cuda.current_stream().cuda_stream)
    net = _lib.Net.from_blob(ctx, W.pack(W.WIDE_SPEC, W.siren_weights(W.WIDE_SPEC, 0)))
    prob = synth.make_problem(cfg, B, N, seed=0)
    dev = torch.device("cuda", 0)
    bufs = {k: torch.from_numpy(np.ascontiguousarray(prob[k])).to(dev) for k in ("x", "u", "p", "dt")}
    for k, s in {"xn": (B, N, 10), "AB": (B, N, 14, 10), "y": (B, N, 11), "Jy": (B, N, 14, 11), "yN": (B, 4),
                 "JyN": (B, 10, 4), "h": (B, N + 1, 3), "Jh": (B, N + 1, 10, 3)}.items():
        bufs[k] = torch.empty(s, dtype=torch.float64, device=dev)
    m = _lib.quad_model(cfg)
    for _ in range(2):
        _lib.linearize(ctx, net, m, B, N, prob["p"].shape[-1], bufs)
    torch.cuda.synchronize()
    ctx.enable_timing(True)
    ctx.reset_stats()
    t = time.perf_counter()
    for _ in range(steps):
        _lib.linearize(ctx, net, m, B, N, prob["p"].shape[-1], bufs)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    rows = B * (N + 1)
    fl = rows * 7_326_976 + B * 2 * 128 * (1024 + 512)
    print(f"B={B} N={N}: {dt*1e3:.3f} ms/prep  {fl/dt/1e12:.1f} TFLOP/s (SDF algorithmic)  {B/dt:.0f} inst-prep/s")
    for k in ("sdf_wide_hoist", "sdf_wide_emb", "sdf_wide_gemm", "sdf_wide_final", "linearize"):
        ms, n = ctx.kernel_stats(k)
        print(f"  {k:16s} {ms/steps:.3f} ms ({n//steps} launches)")
    print("finite h:", bool(torch.isfinite(bufs["h"]).all()))


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:3]))
