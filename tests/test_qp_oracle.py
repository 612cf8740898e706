"""The two CPU QP checkers against each other: the structured Riccati IPM (oracle/qp_ipm.c, the
algorithm family of HPIPM and of csrc/rti_qp.hip) and the dense KKT Mehrotra IPM (oracle/qp_oracle.py).

The QP is strictly convex (lm > 0), so both must reach the same unique solution; they share no linear
algebra, so agreement pins the structured solver before it checks the GPU kernel (tests/test_gpu_qp.py)
and times the QP half of bench.py's cpu_baseline.  acados/HPIPM are absent: parity at the acados
boundary itself is unpinned.
"""
import numpy as np
import pytest

from sdf_nmpc_amd import synth, weights as W
from sdf_nmpc_amd.model import Quad

QP_TOL = 1e-8     # HPIPM's default stop tolerance (max complementarity / primal residual), the production value
SOL_ATOL = 2e-6   # Riccati IPM at QP_TOL vs the exact (active-set polished) solution: measured <= 3e-7
DENSE_ATOL = 1e-7  # dense IPM vs its own polished solution


def _with_flags(cfg, **flags):
    import copy
    c = copy.deepcopy(cfg)
    for k, v in flags.items():
        c.flags[k] = v
    return c


def _instance_set(oracle_lib, cfg, B, N, seed, noise, sdf_cost=False):
    prob = synth.make_problem(cfg, B, N, seed=seed, sdf_cost=sdf_cost)
    x0 = prob["x"][:, 0] + np.random.default_rng(seed).normal(0, noise, (B, 10))
    net = oracle_lib.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, 0))
    lin = oracle_lib.linearize_batch(oracle_lib.quad_model(cfg), net, prob["x"], prob["u"], prob["p"], prob["dt"])
    return prob, x0, lin


def _exact(q):
    """The unique solution of the QP, pinned two ways: the dense KKT IPM, and its active-set polish (one
    equality-constrained KKT solve on the IPM's active rows, no barrier ill-conditioning)."""
    import qp_oracle
    d = qp_oracle.solve_dense(q)
    p = qp_oracle.polish(q, d)
    assert p["max_violation"] < 1e-9 and p["min_dual"] > -1e-9  # a KKT point: feasible, duals >= 0
    for k in ("du", "dx", "sl", "su"):
        np.testing.assert_allclose(d[k], p[k], rtol=0, atol=DENSE_ATOL)
    return p


@pytest.mark.parametrize("B,N,seed,noise,sdf_cost,lm_scaling", [
    (3, 20, 1, 0.05, False, True), (2, 40, 2, 0.05, False, True), (2, 12, 7, 0.5, False, True),
    (2, 20, 4, 0.2, True, True), (3, 60, 5, 0.1, False, True), (2, 40, 2, 0.05, False, False)])
def test_riccati_ipm_matches_dense_ipm(oracle_lib, cfg, B, N, seed, noise, sdf_cost, lm_scaling):
    import qp_oracle
    model = Quad(_with_flags(cfg, sdf_cost=sdf_cost))
    assert model.ny == (12 if sdf_cost else 11)
    prob, x0, lin = _instance_set(oracle_lib, cfg, B, N, seed, noise, sdf_cost)
    r = oracle_lib.qp_ipm_batch(lin, prob, x0, model, tol=QP_TOL, lm_scaling=lm_scaling)
    assert (r["status"] == 0).all()
    assert (r["res"] < QP_TOL).all()
    for b in range(B):
        q = qp_oracle.stage_qp({k: v[b] for k, v in lin.items()}, prob["x"][b], prob["u"][b], x0[b], prob["yref"][b],
                               prob["W"][b], prob["yN"][b], prob["WN"][b], prob["dt"], model, 10.0,
                               lm_scaling=lm_scaling)
        ref = _exact(q)
        np.testing.assert_allclose(r["du"][b], ref["du"], rtol=0, atol=SOL_ATOL)
        np.testing.assert_allclose(r["dx"][b], ref["dx"], rtol=0, atol=SOL_ATOL)
        np.testing.assert_allclose(r["slack"][b][..., 0], ref["sl"], rtol=0, atol=SOL_ATOL)
        np.testing.assert_allclose(r["slack"][b][..., 1], ref["su"], rtol=0, atol=SOL_ATOL)


def test_lm_scaling_changes_the_qp(oracle_lib, cfg):
    """acados adds Ts_k * levenberg_marquardt at k < N and lm at N: the option is live in both oracles."""
    import qp_oracle
    model = Quad(cfg)
    prob, x0, lin = _instance_set(oracle_lib, cfg, 1, 20, 1, 0.05)
    a = oracle_lib.qp_ipm_batch(lin, prob, x0, model, tol=QP_TOL, lm_scaling=True)
    b = oracle_lib.qp_ipm_batch(lin, prob, x0, model, tol=QP_TOL, lm_scaling=False)
    assert np.abs(a["du"] - b["du"]).max() > 1e-3
    q = qp_oracle.stage_qp({k: v[0] for k, v in lin.items()}, prob["x"][0], prob["u"][0], x0[0], prob["yref"][0],
                           prob["W"][0], prob["yN"][0], prob["WN"][0], prob["dt"], model, 10.0)
    np.testing.assert_allclose(np.diag(q["H"][3]) - np.diag(qp_oracle.stage_qp(
        {k: v[0] for k, v in lin.items()}, prob["x"][0], prob["u"][0], x0[0], prob["yref"][0], prob["W"][0],
        prob["yN"][0], prob["WN"][0], prob["dt"], model, 10.0, lm_scaling=False)["H"][3]),
        10.0 * prob["dt"][3] - 10.0, rtol=1e-12)


def test_riccati_ipm_nan_instance_fails_alone(oracle_lib, cfg):
    """A NaN in one instance's linearisation: status 2 (QP failure) for it, the others unaffected."""
    model = Quad(cfg)
    prob, x0, lin = _instance_set(oracle_lib, cfg, 3, 20, 1, 0.05)
    good = oracle_lib.qp_ipm_batch(lin, prob, x0, model, tol=QP_TOL)
    lin["Jh"][1, 5, 2, 2] = np.nan
    bad = oracle_lib.qp_ipm_batch(lin, prob, x0, model, tol=QP_TOL)
    assert list(bad["status"]) == [0, 2, 0]
    assert bad["iters"][1] <= 1
    for b in (0, 2):
        assert np.array_equal(good["du"][b], bad["du"][b])


def test_riccati_ipm_threads_and_batch_invariance(oracle_lib, cfg):
    """One instance solved alone == the same instance inside an OpenMP batch (bitwise)."""
    model = Quad(cfg)
    prob, x0, lin = _instance_set(oracle_lib, cfg, 6, 20, 3, 0.05)
    full = oracle_lib.qp_ipm_batch(lin, prob, x0, model, nthreads=4)
    b = 4
    one = oracle_lib.qp_ipm_batch({k: v[b:b + 1] for k, v in lin.items()},
                                  {k: (v if k == "dt" else v[b:b + 1]) for k, v in prob.items()}, x0[b:b + 1], model)
    assert np.array_equal(full["du"][b], one["du"][0]) and np.array_equal(full["dx"][b], one["dx"][0])
    assert full["iters"][b] == one["iters"][0]


def test_riccati_ipm_warm_start(oracle_lib, cfg):
    """qp_solver_warm_start (ocp.py:116, HPIPM's primal warm start): the IPM started from a given du.  A
    zero du is the cold start bit for bit; a random one still reaches the unique solution (the exact one,
    to SOL_ATOL) along a different path; the input du is not modified."""
    import qp_oracle
    model = Quad(cfg)
    B, N = 4, 20
    prob, x0, lin = _instance_set(oracle_lib, cfg, B, N, 17, 0.2)
    cold = oracle_lib.qp_ipm_batch(lin, prob, x0, model, tol=QP_TOL)
    zero = oracle_lib.qp_ipm_batch(lin, prob, x0, model, tol=QP_TOL, du_ws=np.zeros((B, N, 4)))
    for k in ("du", "dx", "slack", "iters"):
        assert np.array_equal(cold[k], zero[k]), k
    du_ws = np.random.default_rng(18).normal(0, 0.1, (B, N, 4))
    keep = du_ws.copy()
    warm = oracle_lib.qp_ipm_batch(lin, prob, x0, model, tol=QP_TOL, du_ws=du_ws)
    assert np.array_equal(du_ws, keep)
    assert (warm["status"] == 0).all()
    # the start is live: one iteration from it lands elsewhere than one from the cold start
    one_c = oracle_lib.qp_ipm_batch(lin, prob, x0, model, tol=QP_TOL, max_iter=1)
    one_w = oracle_lib.qp_ipm_batch(lin, prob, x0, model, tol=QP_TOL, max_iter=1, du_ws=du_ws)
    assert np.abs(one_c["du"] - one_w["du"]).max() > 1e-3
    for b in range(B):
        q = qp_oracle.stage_qp({k: v[b] for k, v in lin.items()}, prob["x"][b], prob["u"][b], x0[b], prob["yref"][b],
                               prob["W"][b], prob["yN"][b], prob["WN"][b], prob["dt"], model, 10.0)
        ref = _exact(q)
        np.testing.assert_allclose(warm["du"][b], ref["du"], rtol=0, atol=SOL_ATOL)
        np.testing.assert_allclose(warm["dx"][b], ref["dx"], rtol=0, atol=SOL_ATOL)


def test_riccati_ipm_solution_is_feasible(oracle_lib, cfg):
    model = Quad(cfg)
    prob, x0, lin = _instance_set(oracle_lib, cfg, 4, 40, 11, 0.3)
    r = oracle_lib.qp_ipm_batch(lin, prob, x0, model, tol=QP_TOL)
    assert (r["status"] == 0).all()
    u = prob["u"] + r["du"]
    assert (u >= model.lbu - 1e-7).all() and (u <= model.ubu + 1e-7).all()
    np.testing.assert_allclose(r["dx"][:, 0], x0 - prob["x"][:, 0], atol=1e-12)
    A = np.transpose(lin["AB"][:, :, :10, :], (0, 1, 3, 2))
    Bm = np.transpose(lin["AB"][:, :, 10:, :], (0, 1, 3, 2))
    pred = np.einsum("bkij,bkj->bki", A, r["dx"][:, :-1]) + np.einsum("bkij,bkj->bki", Bm, r["du"]) + \
        lin["xn"] - prob["x"][:, 1:]
    np.testing.assert_allclose(r["dx"][:, 1:], pred, atol=1e-9)
    assert (r["slack"] >= -1e-8).all()


def test_c_ipm_against_exact_c3_fixture(oracle_lib):
    """The C restatement (the GPU kernels' algorithm) on the 64 C3 QPs of tests/golden/qp_exact_golden.npz:
    converged, feasible, within the duality-gap bound of F*, and (dx, du) inside the strong-convexity ball
    around the exact solution (the same checks tests/test_gpu_qp.py makes of the kernels)."""
    import os
    import sys
    import qp_oracle
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden"))
    import make_qp_exact as MX
    ex = np.load(os.path.join(os.path.dirname(__file__), "golden", "qp_exact_golden.npz"))
    cfg, model, prob, x0, lin = MX.problem()
    sel, N = ex["sel"], MX.N
    nv = (N + 1) * 10 + N * 4
    r = oracle_lib.qp_ipm_batch({k: v[sel] for k, v in lin.items()},
                                {k: (v if k == "dt" else v[sel]) for k, v in prob.items()}, x0[sel], model,
                                tol=1e-8, nthreads=8)
    assert (r["status"] == 0).all()
    for i, b in enumerate(sel):
        q = qp_oracle.stage_qp({k: v[b] for k, v in lin.items()}, prob["x"][b], prob["u"][b], x0[b], prob["yref"][b],
                               prob["W"][b], prob["yN"][b], prob["WN"][b], prob["dt"], model, 10.0)
        H, g, E, e, G, d = qp_oracle.dense_problem(q)
        z = np.concatenate([r["dx"][i].ravel(), r["du"][i].ravel(), r["slack"][i][..., 0].ravel(),
                            r["slack"][i][..., 1].ravel()])
        zs = np.concatenate([ex["dx"][i].ravel(), ex["du"][i].ravel(), ex["sl"][i].ravel(), ex["su"][i].ravel()])
        assert np.abs(E @ zs - e).max() < 1e-9 and (G @ zs + d).min() > -1e-9  # the fixture is feasible
        assert np.abs(E @ z - e).max() < 1e-9 and (G @ z + d).min() > -1e-8
        dF = 0.5 * z @ H @ z + g @ z - ex["F"][i]
        assert -1e-9 <= dF <= G.shape[0] * 1e-8
        assert np.linalg.norm((z - zs)[:nv]) <= np.sqrt(2.0 * (max(dF, 0.0) + 1e-9) / ex["mu"][i])
    assert np.abs(r["du"] - ex["du"]).max() <= 5e-5
