"""Time the C3 preparation phase (B x N, default 1024 x 40) and its kernels.  SDFNMPC_LIB=<path> loads
another build of libsdfnmpc.so (diagnostic variants, e.g. make -C sdf-nmpc_amd/csrc EXTRA=-DSDF_NO_MFMA)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from sdf_nmpc_amd import _lib, synth, weights as W  # noqa: E402
from sdf_nmpc_amd.config import Config  # noqa: E402


def main(B=1024, N=40, tile=32, steps=20):
    if os.environ.get("SDFNMPC_LIB"):
        _lib.LIB_PATH = os.environ["SDFNMPC_LIB"]
    cfg = Config(mpc__N=N)
    ctx = _lib.Context(0, stream=torch.cuda.current_stream().cuda_stream, tile_rows=tile)
    net = _lib.Net.siren(ctx, 0)
    prob = synth.make_problem(cfg, B, N, seed=0)
    dev = torch.device("cuda", 0)
    bufs = {k: torch.from_numpy(np.ascontiguousarray(prob[k])).to(dev) for k in ("x", "u", "p", "dt")}
    for k, s in {"xn": (B, N, 10), "AB": (B, N, 14, 10), "y": (B, N, 11), "Jy": (B, N, 14, 11), "yN": (B, 4),
                 "JyN": (B, 10, 4), "h": (B, N + 1, 3), "Jh": (B, N + 1, 10, 3)}.items():
        bufs[k] = torch.empty(s, dtype=torch.float64, device=dev)
    m = _lib.quad_model(cfg)
    for _ in range(3):
        _lib.linearize(ctx, net, m, B, N, prob["p"].shape[-1], bufs)
    torch.cuda.synchronize()
    ctx.enable_timing(True)
    ctx.reset_stats()
    t = time.perf_counter()
    for _ in range(steps):
        _lib.linearize(ctx, net, m, B, N, prob["p"].shape[-1], bufs)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    fl = B * (N + 1) * 553_984 + B * 98_304
    print(f"{_lib.LIB_PATH[-30:]} B={B} N={N} M={tile}: {dt*1e3:.3f} ms/prep  {fl/dt/1e12:.1f} TFLOP/s  ", end="")
    for k in ("sdf_hoist", "sdf_mlp", "linearize"):
        ms, n = ctx.kernel_stats(k)
        print(f"{k} {ms/steps:.4f} ms  ", end="")
    print()


if __name__ == "__main__":
    main(*(int(a) for a in sys.argv[1:4]))
