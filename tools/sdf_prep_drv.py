"""Profiling driver: the preparation phase (sdf_hoist + sdf_mlp + linearize) at B x N, a few launches."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import sdf_nmpc_amd  # noqa: E402,F401
from sdf_nmpc_amd import _lib, synth  # noqa: E402
from sdf_nmpc_amd.config import Config  # noqa: E402

B, N = int(os.environ.get("B", 1024)), int(os.environ.get("N", 40))
tile = int(os.environ.get("TILE", 32))
cfg = Config()
ctx = _lib.Context(0, tile_rows=tile)
net = _lib.Net.siren(ctx, 0)
prob = synth.make_problem(cfg, B, N, seed=1000)
D = lambda a: _lib.DeviceArray.from_numpy(ctx, np.ascontiguousarray(a, dtype=np.float64))  # noqa: E731
bufs = {k: D(prob[k]) for k in ("x", "u", "p", "dt")}
for k, s in dict(xn=(B, N, 10), AB=(B, N, 14, 10), y=(B, N, 11), Jy=(B, N, 14, 11), yN=(B, 4), JyN=(B, 10, 4),
                 h=(B, N + 1, 3), Jh=(B, N + 1, 10, 3)).items():
    bufs[k] = _lib.DeviceArray(ctx, s)
for _ in range(int(os.environ.get("REPS", 5))):
    _lib.linearize(ctx, net, _lib.quad_model(cfg), B, N, prob["p"].shape[-1], bufs)
ctx.synchronize()
print("ok")
