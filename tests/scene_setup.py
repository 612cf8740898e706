"""TEST INFRASTRUCTURE: the obstacle-scene closed loop shared by tests/test_gpu_scene.py, bench.py's `scene`
leg and tools/scene_probe.py.

The scene network (tests/golden/scene.sdfw, tools/fit_scene_sdf.py) is the deployed NeuralDF architecture
fitted to a pillar of radius 0.4 m at (3.0, 0.3) and a box at x 5.0-5.6 m in the camera-origin frame, for the
scene latent stored in scene_golden.npz.  The depth image is taken once at the start: the camera pose is
the start pose (W_p_Bo = 0, W_R_Bo = I), so the scene is fixed in the world.  Every instance flies from x = 0
towards a waypoint beyond the pillar (x = 7) at a lateral offset; the SDF row (h[2] >= size.xy +
bound_margin = 0.37, gen_model.py:35, 58-61) becomes active as the pillar comes within the horizon and
releases once it is passed.  The oracle loop is the one of test_gpu_closed_loop.py: shift, x_0 = measured
state, oracle.linearize_batch, the structured C IPM, the update, the plant advanced by u_0 (RK4)."""
import os

import numpy as np

from sdf_nmpc_amd.reference import Ref, yaw2quat

HERE = os.path.dirname(os.path.abspath(__file__))
SCENE = os.path.join(HERE, "golden", "scene.sdfw")
B = 3
Y0 = np.array([0.25, 0.05, 0.55])  # lateral start offsets: straight at the pillar, left of it, right of it
GOAL = np.array([7.0, 0.3, 0.0])


def scene_latent():
    return np.load(os.path.join(HERE, "golden", "scene_golden.npz"))["latent"].astype(np.float64)


def setup(n, goal=GOAL, y0=Y0):
    """Flag on, the scene latent with the camera at the start pose, a waypoint reference; returns x0 [B, 10]."""
    Bn = max(n.B, 1)
    y0 = np.resize(y0, Bn)
    x0 = np.zeros((Bn, 10))
    x0[:, 1] = y0
    x0[:, 3] = 1.0  # identity attitude, at rest
    n.set_sdf_flag(1.0)
    n.set_latent(np.broadcast_to(scene_latent(), (Bn, 128)), np.zeros((Bn, 3)), np.stack([np.eye(3)] * Bn))
    r = Ref(n.cfg)
    r.p, r.q = np.asarray(goal, float), yaw2quat(0.0)
    r.use_weights(r.W_on)
    for k in range(n.N + 1):
        n.set_ref(r, k)
    return x0


def plant(O, onet, cfg, x, u, dt):
    """x_{t+1} = RK4(x_t, u_t, dt) of the model (the oracle's integrator, one instance per row)."""
    Bn = x.shape[0]
    lin = O.linearize_batch(O.quad_model(cfg), onet, np.stack([x, x], 1), u[:, None], np.zeros((Bn, 2, 145)),
                            np.array([dt]))
    return lin["xn"][:, 0]


def hard_rows_active(model, lin, r, tol=1e-6):
    """Per instance: how many hard constraint rows (stage rows with slack None at nodes 0 < k < N, hard
    terminal rows) and rec_feas braking rows (hard, or soft with slack_brake) bind at the QP solution r
    (the linearised row within tol of a bound, or beyond it on its slack), from the linearisation lin."""
    N = r["du"].shape[1]
    cnt = np.zeros(r["du"].shape[0], int)
    for j in range(model.nh - model.nhs, model.nh):
        c = model.h_cols[j]
        v = lin["h"][:, 1:N, c] + np.einsum("bki,bki->bk", lin["Jh"][:, 1:N, :, c], r["dx"][:, 1:N])
        cnt += ((v - model.lh[j] < tol) | (model.uh[j] - v < tol)).sum(axis=1)
    for j, (c1, c2, soft, lo, hi, _, _) in enumerate(model.term_rows):
        if soft and c2 != 0:
            continue
        v = np.zeros(len(cnt))
        g = np.zeros((len(cnt), 10))
        if c1 >= 0:
            v += lin["h"][:, N, c1]
            g += lin["Jh"][:, N, :, c1]
        if c2 >= 0:
            v += lin["hE"][:, c2]
            g += lin["JhE"][:, :, c2]
        v = v + np.einsum("bi,bi->b", g, r["dx"][:, N])
        cnt += (v - lo < tol) | (hi - v < tol)
    return cnt


def oracle_loop(O, onet, n, cfg, x0, K, warm=False, strict=True):
    """The oracle pipeline run as the controller runs it, with per-step diagnostics of the SDF rows:
    h2min = min over nodes of the flagged SDF value at the linearisation point, sdf_slack = max over nodes of
    the QP's SDF lower slack (> 0: the soft row is active), hard_active = binding hard rows
    (hard_rows_active), and the plant state before the step.  strict: every QP must converge."""
    Bn, N, dt, shift = x0.shape[0], n.N, n.ocp.dt, int(cfg.mpc.shift)
    xs = np.repeat(x0[:, None], N + 1, axis=1)
    us = np.broadcast_to(n.model.u_hover, (Bn, N, 4)).copy()
    prob = {"yref": n.y, "W": n.W, "yN": n.yN, "WN": n.WN, "dt": dt}
    xo, du, hist = x0.copy(), None, []
    for _ in range(K):
        if 0 < shift < N:
            xs[:, : N - shift] = xs[:, shift:N].copy()
            us[:, : N - shift] = us[:, shift:N].copy()
        xs[:, 0] = xo
        lin = O.linearize_batch(O.quad_model(cfg), onet, xs, us, n.p, dt, model=n.model)
        r = O.qp_ipm_batch(lin, dict(prob, x=xs, u=us), xo, n.model, nthreads=4,
                           du_ws=(np.zeros((Bn, N, 4)) if du is None else du) if warm else None)
        assert not strict or (r["status"] == 0).all()
        du = r["du"].copy()
        hist.append({"x0": xo.copy(), "h2min": lin["h"][..., 2].min(axis=1), "sdf_slack": r["slack"][:, :, 2, 0].max(axis=1),
                     "iters": r["iters"].copy(), "status": r["status"].copy(),
                     "hard_active": hard_rows_active(n.model, lin, r)})
        xs, us = xs + r["dx"], us + r["du"]
        hist[-1]["u0"] = us[:, 0].copy()
        xo = plant(O, onet, cfg, xo, us[:, 0], dt[0])
    return hist
