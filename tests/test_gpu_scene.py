"""A geometry-meaningful SDF.  Every other network here is the SIREN initialisation,
whose df is ~0 everywhere: every SDF row of every QP is active.  tests/golden/scene.sdfw is the deployed
NeuralDF architecture fitted offline (tools/fit_scene_sdf.py: the reference's NeuralDF, loss and
initialisation, torch CPU, seeded) to a pillar and a box (tests/scene_setup.py).

  * the network on the GPU against the reference's own NeuralDF on those weights (scene_golden.npz,
    make_golden.py scene), with the deployed net's bar;
  * the closed loop flying past the pillar, with and without HPIPM's primal warm start
    (qp_solver_warm_start = 1, ocp.py:116): the SDF rows become active as the pillar enters the horizon
    and release once it is passed, and every step's u_0 is pinned to the oracle pipeline (C linearisation
    + structured C IPM, run as the controller runs)."""
import os

import numpy as np
import pytest

from sdf_nmpc_amd import _lib
from sdf_nmpc_amd.config import Config
from sdf_nmpc_amd.controller import Nmpc
from sdf_nmpc_amd.model import Quad
from sdf_nmpc_amd.ocp import Ocp
from sdf_nmpc_amd import weights as W
from test_gpu_sdf import eval_device
from tolerances import STRESS_FACTOR
import scene_setup as S

pytestmark = pytest.mark.gpu

U0_ATOL = 2e-5
K = 40


@pytest.fixture(scope="module")
def sg():
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "scene_golden.npz"))


def test_scene_net_vs_reference_golden(gpu_ctx, sg):
    """The batched kernel (sdf_mlp) and the host path (jac_sdf_l4c's full 1 x 131 Jacobian) on the scene
    weights against the reference NeuralDF: error vs its fp64 at most 2x the reference fp32's own error
    (with a floor of 4 fp32 ulps of the scale), as for the deployed SIREN net."""
    import hashlib
    with open(S.SCENE, "rb") as f:
        blob = f.read()
    assert hashlib.sha256(blob).digest() == sg["sha256"].tobytes()
    net = _lib.Net.from_file(gpu_ctx, S.SCENE)
    try:
        o = eval_device(gpu_ctx, net, sg["input"]).astype(np.float64)
        df_h, g_h = net.eval_host(sg["input"].astype(np.float64))
    finally:
        net.close()
    eps = 4 * np.finfo(np.float32).eps
    d64, d32 = sg["df_f64"], sg["df_f32"].astype(np.float64)
    g64, g32 = sg["grad_f64"], sg["grad_f32"].astype(np.float64)
    ref_df, ref_g3 = np.abs(d32 - d64).max(), np.linalg.norm(g32[:, :3] - g64[:, :3], axis=1).max()
    ref_g = np.linalg.norm(g32 - g64, axis=1).max()
    for df, g3 in ((o[:, 0], o[:, 1:]), (df_h, g_h[:, :3])):
        assert np.abs(df - d64).max() <= max(STRESS_FACTOR * ref_df, eps * np.abs(d64).max())
        assert np.linalg.norm(g3 - g64[:, :3], axis=1).max() <= max(STRESS_FACTOR * ref_g3, eps * 4)
    assert np.linalg.norm(g_h - g64, axis=1).max() <= max(STRESS_FACTOR * ref_g, eps * 4)
    # what the fit is (not a parity bar): the network is the scene's distance to a few centimetres
    err = np.abs(d64 - sg["scene_df"])
    print(f"\nscene fit: |df - analytic sdf| mean {err.mean():.3f} m, p95 {np.quantile(err, 0.95):.3f} m")
    assert np.quantile(err, 0.95) < 0.1


@pytest.mark.parametrize("warm", [False, True])
def test_scene_closed_loop_sdf_rows_activate_and_release(oracle_lib, warm):
    O = oracle_lib
    cfg = Config(mpc__N=20)
    ocp = Ocp(Quad(cfg), batch=S.B, weights=S.SCENE, qp_warm_start=warm)
    n = Nmpc(cfg, batch=S.B, ocp=ocp)
    x0 = S.setup(n)
    with open(S.SCENE, "rb") as f:
        onet = O.Net(*W.unpack(f.read()))
    ug, xg, iters = [], x0.copy(), []
    for _ in range(K):
        n.set_x0(xg)
        assert n.solve() == 0 and (n.ocp.status == 0).all()
        ug.append(n.get_u().copy())
        iters.append(n.ocp.iters.copy())
        xg = S.plant(O, onet, cfg, xg, ug[-1], n.ocp.dt[0])
    hist = S.oracle_loop(O, onet, n, cfg, x0, K, warm=warm)
    ug = np.array(ug)
    uo = np.array([h["u0"] for h in hist])
    d = np.abs(ug - uo).max(axis=(1, 2))
    active = np.array([h["sdf_slack"] > 1e-6 for h in hist])  # [K, B]: the SDF soft row binds somewhere
    print(f"\nwarm={warm}: max |u0 - u0_oracle| per step {d.max():.2e}; SDF active steps per instance "
          f"{active.sum(0)}; QP iterations max {np.max(iters)}; final x {xg[:, 0]}")
    assert d.max() <= U0_ATOL, d
    # the SDF rows become active and release: the instance flying straight at the pillar is active at some
    # steps, every instance is released at the end, and the pillar was passed (x beyond it)
    assert active[:, 0].sum() >= 3
    assert not active[-5:].any()
    assert (xg[:, 0] > 3.6).all()
    ocp.close()


def test_scene_c3_full_size_active_rows_vs_oracle(oracle_lib):
    """C3's size (1024 instances x N = 40) on the scene net, where the SDF rows are active in a large share
    of the instances (the setup of bench.py's scene leg: starts spread over x in [0, 2.5] m and lateral
    offsets in [-1, 1.5] m, the loop closed with a perfect-model plant).  After six warm steps, at two
    steps, 24 instances with an active SDF soft row and 8 without are pinned to the oracle pipeline (the C
    linearisation and the structured C IPM at the iterate the GPU step linearised at): u_0 of the step."""
    O = oracle_lib
    B, N = 1024, 40
    cfg = Config(mpc__N=N)
    ocp = Ocp(Quad(cfg), batch=B, weights=S.SCENE)
    n = Nmpc(cfg, batch=B, ocp=ocp)
    rng = np.random.default_rng(77)
    x = S.setup(n, y0=rng.uniform(-1.0, 1.5, B))
    x[:, 0] = rng.uniform(0.0, 2.5, B)
    with open(S.SCENE, "rb") as f:
        onet = O.Net(*W.unpack(f.read()))
    try:
        for _ in range(6):
            n.set_x0(x)
            assert n.solve() == 0
            x = n.get_matrices()[0][:, 1].copy()
        for step in range(2):
            n.set_x0(x)
            xs, us = (a.copy() for a in n.get_matrices())  # the iterate this step linearises at (mpc.shift = 0)
            assert n.solve() == 0 and (ocp.status == 0).all()
            u0 = n.get_u().copy()
            act = (ocp.download("slack").reshape(B, N + 1, 3, 2)[:, :, 2, 0] > 1e-6).any(axis=1)
            pick = np.concatenate([np.flatnonzero(act)[:24], np.flatnonzero(~act)[:8]])
            xi, ui = xs[pick], us[pick]
            xi[:, 0] = x[pick]
            lin = O.linearize_batch(O.quad_model(cfg), onet, xi, ui, n.p[pick], ocp.dt)
            prob = {"yref": n.y[pick], "W": n.W[pick], "yN": n.yN[pick], "WN": n.WN[pick], "dt": ocp.dt, "x": xi,
                    "u": ui}
            r = O.qp_ipm_batch(lin, prob, x[pick], n.model, nthreads=8)
            assert (r["status"] == 0).all()
            d = np.abs(u0[pick] - (ui[:, 0] + r["du"][:, 0])).max(axis=1)
            oact = (r["slack"][:, :, 2, 0] > 1e-6).any(axis=1)
            print(f"\nstep {step}: SDF row active in {act.mean():.0%} of {B}; sample max |u0 - u0_oracle| "
                  f"{d.max():.2e}; oracle agrees on activity in {np.mean(oact == act[pick]):.0%}; GPU iterations "
                  f"max {ocp.iters.max()}")
            assert act.mean() >= 0.25 and len(pick) == 32
            assert d.max() <= U0_ATOL, d
            assert (oact == act[pick]).mean() >= 0.9
            x = n.get_matrices()[0][:, 1].copy()
    finally:
        ocp.close()
