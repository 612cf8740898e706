#!/usr/bin/env python3
"""Probe: sdfnmpc_linearize alone at the C3 shape (B = 1024, N = 40, the default flag set), mean kernel
time over 50 launches from HIP events (the context's kernel stats).  SDFNMPC_LIB selects a diagnostic
build (tools/exp/exp_lin.sh)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import sdf_nmpc_amd  # noqa: E402,F401
from sdf_nmpc_amd import _lib, synth  # noqa: E402
from sdf_nmpc_amd.config import Config  # noqa: E402


def main():
    import torch
    B, N = int(os.environ.get("B", 1024)), int(os.environ.get("N", 40))
    os.environ["SDFNMPC_SERIAL_PREP"] = "1"
    cfg = Config()
    ctx = _lib.Context(0)
    net = _lib.Net.siren(ctx, 0)
    prob = synth.make_problem(cfg, B, N, seed=1)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)  # noqa: E731
    bufs = {k: t(prob[k]) for k in ("x", "u", "p", "dt")}
    shapes = {"xn": (B, N, 10), "AB": (B, N, 14, 10), "y": (B, N, 11), "Jy": (B, N, 14, 11), "yN": (B, 4),
              "JyN": (B, 10, 4), "h": (B, N + 1, 3), "Jh": (B, N + 1, 10, 3)}
    for k, s in shapes.items():
        bufs[k] = torch.zeros(s, dtype=torch.float64, device=dev)
    model = _lib.quad_model(cfg)
    for _ in range(5):
        _lib.linearize(ctx, net, model, B, N, prob["p"].shape[-1], bufs)
    ctx.synchronize()
    ctx.enable_timing(True)
    ctx.reset_stats()
    for _ in range(50):
        _lib.linearize(ctx, net, model, B, N, prob["p"].shape[-1], bufs)
    ctx.synchronize()
    v = ctx.kernel_stats("linearize")
    chk = float(bufs["AB"].double().abs().sum() + bufs["Jy"].double().abs().sum())
    print(f"linearize alone B={B} N={N}: {v[0] / v[1] * 1e3:.2f} us  (checksum {chk:.6e})", flush=True)


if __name__ == "__main__":
    main()
