"""CPU probe (oracle only, no GPU): the closed loop of tests/test_gpu_scene.py in the fitted obstacle scene
(tests/golden/scene.sdfw), to see when the SDF rows become active and release.  Prints, per RTI step and
instance: position, the smallest flagged SDF value h[2] over the horizon, the SDF slack of the QP
solution (active soft row when > 0) and the QP iterations.

    python tools/scene_probe.py [K] [warm]
"""
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import sdf_nmpc_amd  # noqa: E402,F401
from sdf_nmpc_amd import _lib, weights as W  # noqa: E402
from sdf_nmpc_amd.config import Config  # noqa: E402
from sdf_nmpc_amd.controller import Nmpc  # noqa: E402
import oracle as O  # noqa: E402
import scene_setup as S  # noqa: E402


def main(K=40, warm=False):
    O.build()
    cfg = Config(mpc__N=20)
    _, dt = _lib.shooting_grid(20, cfg.mpc.T)
    n = Nmpc(cfg, batch=S.B, ocp=types.SimpleNamespace(dt=dt))
    x0 = S.setup(n)
    with open(S.SCENE, "rb") as f:
        spec, params = W.unpack(f.read())
    onet = O.Net(spec, params)
    hist = S.oracle_loop(O, onet, n, cfg, x0, K, warm=warm)
    for k, h in enumerate(hist):
        row = "  ".join(f"x=({h['x0'][b, 0]:5.2f},{h['x0'][b, 1]:5.2f}) h2min={h['h2min'][b]:6.3f} "
                        f"sl={h['sdf_slack'][b]:.1e} it={h['iters'][b]:2d}" for b in range(S.B))
        print(f"step {k:2d}: {row}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 40, len(sys.argv) > 2 and sys.argv[2] == "warm")
