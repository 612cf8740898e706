"""CPU probe (oracle only): the obstacle-scene closed loop (tests/scene_setup.py) under a flag set of
tests/flag_sets.py at the reference's own bounds, with the braking polynomial of a physical braking law.
Reports per step the QP iterations / status and which hard rows bind.  Usage:
  python tools/scene_flags_probe.py <flag set> [N] [K] [x_start] [vx_start]"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle as O  # noqa: E402
import flag_sets as F  # noqa: E402
import scene_setup as S  # noqa: E402
from sdf_nmpc_amd import synth, weights as W  # noqa: E402
from sdf_nmpc_amd.controller import Nmpc  # noqa: E402
from sdf_nmpc_amd.model import Quad  # noqa: E402


def run(name, N=40, K=40, xs=1.0, ys=(0.25, 0.05, 0.55), vx=0.0, **over):
    cfg = F.config(name, mpc__N=N, **over)
    coeffs = None
    if cfg.flags.recursive_feasibility:
        coeffs = synth.braking_coeffs(int(cfg.mpc.braking_dist.degree), noise=0.0, a_brake=float(cfg.mpc.stability.a_b_min))
    q = Quad(cfg, braking_coeffs=coeffs)

    class StubOcp:
        model = q
        dt = np.full(N, cfg.mpc.T / N)

    n = Nmpc(cfg, batch=len(ys), ocp=StubOcp())
    x0 = S.setup(n, y0=np.asarray(ys, float))
    x0[:, 0] = xs
    x0[:, 7] = vx
    with open(S.SCENE, "rb") as f:
        onet = O.Net(*W.unpack(f.read()))
    hist = S.oracle_loop(O, onet, n, cfg, x0, K, strict=False)
    return q, hist


if __name__ == "__main__":
    name = sys.argv[1]
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 40
    xs = float(sys.argv[4]) if len(sys.argv) > 4 else 1.0
    vx = float(sys.argv[5]) if len(sys.argv) > 5 else 0.0
    over = {"mpc__bound_margin": 0.15}  # the reference's bound (flag_sets' hard_df moves it for the SIREN net)
    q, hist = run(name, N, K, xs, vx=vx, **over)
    for i, h in enumerate(hist):
        print(i, "x", np.round(h["x0"][:, :2], 2).tolist(), "it", h["iters"].tolist(), "st", h["status"].tolist(),
              "hard act", h["hard_active"].tolist(), "h2min", np.round(h["h2min"], 2).tolist())
