"""The flag space of default.yaml:16-23 on the CPU (gen_model.py:26-149): the constraint set the host builds
for every flag combination, the reference-pinned pieces of recursive_feasibility / stability, and the two
CPU QP checkers (oracle/qp_ipm.c, the structured Riccati IPM with the kernel's row semantics; oracle/
qp_oracle.py, the dense KKT IPM + active-set polish) against each other on every flag set.

Pins (tests/golden/flags_golden.npz, made by tests/golden/make_golden.py flags from the reference itself):
  * polynomial_3variate's term order and values (utils/math.py:294-321), degrees 0..6;
  * stability.get_r_tilde_max (utils/stability.py:44-75) under a seeded np.random;
  * Nmpc.set_ref at the terminal node with the stability row (nyN = 5: WN = W[:5], controller.py:141-142).
The row sets themselves (tests/flag_sets.py) restate gen_model.py:41-70,98-126 and cost_const_helpers.py:
70-102; acados is absent, so the QP they make is pinned to its exact solution, not to HPIPM.
"""
import os

import numpy as np
import pytest

import flag_sets as F
from sdf_nmpc_amd import synth, weights as W
from sdf_nmpc_amd.model import Quad, UnsupportedConfig, poly_eval, poly_terms, r_tilde_max

HERE = os.path.dirname(os.path.abspath(__file__))
QP_TOL = 1e-8
SOL_ATOL = 2e-6  # C IPM at QP_TOL vs the exact solution on well-posed instances (measured <= 4e-7)


@pytest.fixture(scope="module")
def fg():
    return np.load(os.path.join(HERE, "golden", "flags_golden.npz"))


@pytest.mark.parametrize("deg", range(7))
def test_poly_term_order_and_values_match_reference(fg, deg):
    np.testing.assert_array_equal(np.array(poly_terms(deg)), fg[f"poly/deg{deg}/exps"])
    val, grad = poly_eval(fg[f"poly/deg{deg}/coeffs"], deg, fg[f"poly/deg{deg}/v"])
    np.testing.assert_allclose(val, fg[f"poly/deg{deg}/val"], rtol=1e-12, atol=1e-12)
    # the gradient (the Jacobian the kernel forms with dual numbers) against central differences
    v = fg[f"poly/deg{deg}/v"]
    for i in range(3):
        d = np.zeros(3); d[i] = 1e-6
        fd = (poly_eval(fg[f"poly/deg{deg}/coeffs"], deg, v + d)[0] - poly_eval(fg[f"poly/deg{deg}/coeffs"], deg, v - d)[0]) / 2e-6
        np.testing.assert_allclose(grad[:, i], fd, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("N,T", [(20, 1.5), (40, 1.5), (30, 2.0)])
def test_r_tilde_matches_reference(fg, N, T):
    """get_r_tilde_max restated in closed form (the sympy solve is linear in r~) with the reference's SLSQP
    start drawn from np.random: the same seed gives the same maximum (SLSQP stops at ~1e-8 relative)."""
    from sdf_nmpc_amd.config import Config
    cfg = Config(mpc__N=N, mpc__T=T)
    for seed in (0, 1, 2):
        np.random.seed(seed)
        got = r_tilde_max(cfg)
        want = float(fg[f"rtilde/N{N}_T{T}/seed{seed}"])
        assert abs(got - want) <= 1e-6 * abs(want), (seed, got, want)


@pytest.mark.parametrize("name", list(F.FLAG_SETS))
def test_constraint_set_of_each_flag_set(name):
    cfg = F.config(name)
    q = F.quad(name, cfg)
    _, cols, rows = F.FLAG_SETS[name]
    assert q.h_cols == cols and q.nh == len(cols)
    assert [r[:3] for r in q.term_rows] == rows and q.nhN == len(rows)
    assert q.nsN == sum(1 for r in rows if r[2]) and all(r[2] for r in q.term_rows[:q.nsN])
    # hard stage rows: the columns whose slack weight is None (fov: 0, 1; sdf: 2), after the soft ones
    hard = {0: cfg.mpc.weights.slack_fov is None, 1: cfg.mpc.weights.slack_fov is None, 2: cfg.mpc.weights.slack_df is None}
    assert q.nhs == sum(hard[c] for c in cols) and all(hard[c] for c in cols[q.nh - q.nhs:])
    assert all((q.zl[j], q.Zl[j]) == (0.0, 0.0) for j in range(q.nh - q.nhs, q.nh))
    # bounds: fov rows +-fov_ratio fov, the sdf row [size.xy + bound_margin, max_df + 0.2] (gen_model.py:35),
    # the braking row [size.xy, max_df] (gen_model.py:118), the velocity bounds +-limits (add_vel_const)
    lims = {0: cfg.sensor.hfov * cfg.mpc.fov_ratio, 1: cfg.sensor.vfov * cfg.mpc.fov_ratio}
    for j, c in enumerate(cols):
        lo, hi = (-lims[c], lims[c]) if c < 2 else (cfg.robot.size.xy + cfg.mpc.bound_margin, q.max_df + 0.2)
        assert (q.lh[j], q.uh[j]) == pytest.approx((lo, hi))
    for (c1, c2, soft, lo, hi, zl, Zl) in q.term_rows:
        if c2 == 0:
            assert (lo, hi) == pytest.approx((cfg.robot.size.xy, q.max_df))
        elif c2 in (1, 2):
            assert (lo, hi) == pytest.approx((-lims[c2 - 1], lims[c2 - 1]))
        elif c2 >= 3:
            v = [cfg.robot.limits.vx, cfg.robot.limits.vy, cfg.robot.limits.vz][c2 - 3]
            assert (lo, hi) == (-v, v)
    assert q.nyN == (5 if cfg.flags.get("stability") and cfg.flags.get("recursive_feasibility") else 4)
    assert q.need_sdf == (2 in cols or q.sdf_cost or q.rec_feas)
    assert q.name.endswith("_sdf") == bool(cfg.flags.enable_sdf)


def test_unbuilt_models_are_refused():
    with pytest.raises(UnsupportedConfig):
        Quad(F.config("default", mpc__model="acc"))
    with pytest.raises(UnsupportedConfig):  # rec_feas without coefficients (no file in the cache dir)
        os.environ["SDFNMPC_CACHE"] = os.path.join(HERE, "_nonexistent_cache")
        try:
            Quad(F.config("rec_feas"))
        finally:
            os.environ.pop("SDFNMPC_CACHE")


def test_stability_terminal_reference_matches_reference(fg):
    """Nmpc.set_ref(ref, N) with the stability row: WN = W[:5], yN = y[:5] (controller.py:141-142) -- the 5th
    weight is the x velocity weight, not the reference's unused p_term (extra_WN, gen_model.py:149)."""
    from sdf_nmpc_amd.controller import Nmpc
    from sdf_nmpc_amd.reference import Ref

    cfg = F.config("stability", mpc__N=20)
    q = F.quad("stability", cfg)

    class StubOcp:
        model = q

    n = Nmpc(cfg, ocp=StubOcp())
    a = fg["setref5/ref"]
    r = Ref(cfg)
    r.p, r.q, r.v, r.wz = a[0:3], a[3:7], a[7:10], a[10]
    r.Wp, r.Wq, r.Wv, r.Ww, r.Wa = a[11:14], a[14:17], a[17:20], a[20:23], a[23]
    n.set_ref(r, cfg.mpc.N)
    np.testing.assert_array_equal(n.yN, fg["setref5/yN"])
    np.testing.assert_array_equal(n.WN, fg["setref5/WN"])
    assert q.extra_WN.shape == (1,) and q.extra_WN[0] > 0


def test_terminal_extras_oracle(oracle_lib):
    """orc_quad_term (the checker of the kernel's terminal extras): values against a numpy restatement of
    gen_model.py:81-121 built on the reference-pinned poly_eval, Jacobians against central differences."""
    cfg = F.config("stability")
    q = F.quad("stability", cfg)
    m = oracle_lib.quad_model(cfg)
    rng = np.random.default_rng(2)
    R_off = np.asarray(cfg.sensor.B_R_C).T @ np.asarray(cfg.sensor.B_p_C) + np.array([cfg.mpc.fov_const_offset, 0, 0])
    for _ in range(8):
        x = np.concatenate([rng.uniform(-2, 2, 3), synth.euler2quat(rng.uniform(-0.5, 0.5, 3)), rng.uniform(-3, 3, 3)])
        p = np.zeros(145)
        p[0] = rng.choice([0.0, 1.0, 0.3])
        R = synth.quat2rot(synth.euler2quat(rng.uniform(-1, 1, 3)))
        p[1:4], p[4:13] = rng.uniform(-1, 1, 3), R.ravel()
        hE, JhE, yN5, JyN5 = oracle_lib.term_extras(m, x, p, q)
        v = x[7:]
        pv, _ = poly_eval(q.poly, q.poly_deg, v)
        E = R.T @ (x[:3] + pv * v / np.sqrt(v @ v + 1e-4) - p[1:4]) + R_off
        want = [-p[0] * pv, p[0] * np.arctan2(E[1], E[0]), p[0] * np.arctan2(E[2], np.hypot(E[0], E[1])), *v]
        np.testing.assert_allclose(hE, want, rtol=1e-12, atol=1e-12)
        _, _, yN4, _ = oracle_lib.cost(m, x, np.zeros(4), p)
        np.testing.assert_allclose(yN5, p[0] * np.concatenate([yN4, [v @ v]]), rtol=1e-13, atol=1e-13)
        for j in range(10):
            d = np.zeros(10); d[j] = 1e-6
            hp, _, yp, _ = oracle_lib.term_extras(m, x + d, p, q)
            hm, _, ym, _ = oracle_lib.term_extras(m, x - d, p, q)
            np.testing.assert_allclose(JhE[:, j], (hp - hm) / 2e-6, rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(JyN5[:, j], (yp - ym) / 2e-6, rtol=1e-5, atol=1e-6)


def _net(oracle_lib, q):
    if F.uses_scene(q):
        import scene_setup as S
        with open(S.SCENE, "rb") as f:
            return oracle_lib.Net(*W.unpack(f.read()))
    return oracle_lib.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, 0))


def _problem(oracle_lib, name, B, N, seed, noise=0.05):
    cfg = F.config(name, mpc__N=N)
    q = F.quad(name, cfg)
    # the flight along the camera's view (hard fov rows: random v0 can leave the cone before any input acts,
    # which makes a hard row infeasible -- for the reference's HPIPM too); sets with hard rows on the scene net
    prob = F.problem(cfg, q, B, N, seed)
    x0 = prob["x"][:, 0] + np.random.default_rng(seed).normal(0, noise, (B, 10))
    net = _net(oracle_lib, q)
    lin = oracle_lib.linearize_batch(oracle_lib.quad_model(cfg), net, prob["x"], prob["u"], prob["p"], prob["dt"], model=q)
    return cfg, q, prob, x0, lin


@pytest.mark.parametrize("name", list(F.FLAG_SETS))
def test_riccati_ipm_matches_exact_solution_per_flag_set(oracle_lib, name):
    """The C restatement of the kernel's IPM (soft stage rows of the set, soft + hard terminal rows) against the
    exact QP solution: status 0; the objective within the duality gap m tol of F*; (dx, du) inside the
    strong-convexity ball sqrt(2 (F - F*) / mu); 2e-6 absolute where the instance is well posed (a hard
    terminal row far outside its bounds at the linearisation point -- the synthetic camera pose puts the
    braking point anywhere -- flattens the objective, as for the reference's HPIPM)."""
    import qp_oracle
    cfg, q, prob, x0, lin = _problem(oracle_lib, name, 3, 20, seed=3)
    r = oracle_lib.qp_ipm_batch(lin, prob, x0, q, tol=QP_TOL)
    assert (r["status"] == 0).all(), r["iters"]
    close = hard_active = 0
    for b in range(3):
        qq = qp_oracle.stage_qp({k: v[b] for k, v in lin.items() if k != "sdf"}, prob["x"][b], prob["u"][b], x0[b],
                                prob["yref"][b], prob["W"][b], prob["yN"][b], prob["WN"][b], prob["dt"], q, 10.0)
        H, g, E, e, G, d = qp_oracle.dense_problem(qq)
        ex = qp_oracle.polish_active_set(qq, qp_oracle.solve_dense(qq))
        assert ex["max_violation"] < 1e-9 and ex["min_dual"] > -1e-9
        sol = dict(dx=r["dx"][b], du=r["du"][b], sl=r["slack"][b][..., 0], su=r["slack"][b][..., 1])
        z, zs = qp_oracle.z_of(qq, sol), qp_oracle.z_of(qq, ex)
        Fz, Fs = 0.5 * z @ H @ z + g @ z, 0.5 * zs @ H @ zs + g @ zs
        assert (G @ z + d).min() > -1e-7 and np.abs(E @ z - e).max() < 1e-8  # feasible
        m = G.shape[0]
        assert Fz - Fs <= qp_oracle.objective_bound(m, QP_TOL, ex["lam_l1"], r["res"][b, 1]), (b, Fz - Fs)
        n_xu = 10 * (cfg.mpc.N + 1) + 4 * cfg.mpc.N
        mu = np.linalg.eigvalsh(H[:n_xu, :n_xu]).min()
        ball = np.sqrt(2 * max(Fz - Fs, 0.0) / mu) + 1e-6  # + the exact solution's own rounding level
        assert np.linalg.norm(z[:n_xu] - zs[:n_xu]) <= ball
        close += np.abs(sol["du"] - ex["du"]).max() <= SOL_ATOL
        if q.nhs:  # hard stage rows: some bind at the exact solution, none is violated by the C IPM's point
            nb = 8 * cfg.mpc.N + 4 * (cfg.mpc.N * (q.nh - q.nhs) + q.nsN)
            hard_active += int(((G @ zs + d)[nb:] < 1e-7).sum())
    assert close >= (1 if q.nhN > q.nsN else 2)
    if q.nhs:
        assert hard_active > 0


@pytest.mark.parametrize("name", ["no_vfov", "lidar_sdf_only", "rec_feas", "rec_feas_soft_brake", "hard_fov", "hard_df_rec_feas"])
def test_segments_match_serial_riccati(oracle_lib, name):
    """The C restatement's partitioned Riccati (P = 4) on the terminal rows of a flag set: the same iterates
    as the serial recursion (the terminal node is in the last, serial segment)."""
    cfg, q, prob, x0, lin = _problem(oracle_lib, name, 2, 40, seed=5)
    a = oracle_lib.qp_ipm_batch(lin, prob, x0, q, tol=QP_TOL)
    b = oracle_lib.qp_ipm_batch(lin, prob, x0, q, tol=QP_TOL, start=dict(seg=4))
    assert np.abs(a["iters"] - b["iters"]).max() <= 1
    np.testing.assert_allclose(a["du"], b["du"], rtol=0, atol=1e-6)  # rounding-level differences, amplified near tol
