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

SOL_ATOL = 1e-6   # both IPMs stopped at tol 1e-10: solutions agree to ~sqrt(mu)


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


@pytest.mark.parametrize("B,N,seed,noise,sdf_cost", [(3, 20, 1, 0.05, False), (2, 40, 2, 0.05, False),
                                                     (2, 12, 7, 0.5, False), (2, 20, 4, 0.2, True)])
def test_riccati_ipm_matches_dense_ipm(oracle_lib, cfg, B, N, seed, noise, sdf_cost):
    import qp_oracle
    model = Quad(_with_flags(cfg, sdf_cost=sdf_cost))
    assert model.ny == (12 if sdf_cost else 11)
    prob, x0, lin = _instance_set(oracle_lib, cfg, B, N, seed, noise, sdf_cost)
    r = oracle_lib.qp_ipm_batch(lin, prob, x0, model, tol=1e-10)
    assert (r["status"] == 0).all()
    for b in range(B):
        q = qp_oracle.stage_qp({k: v[b] for k, v in lin.items()}, prob["x"][b], prob["u"][b], x0[b], prob["yref"][b],
                               prob["W"][b], prob["yN"][b], prob["WN"][b], prob["dt"], model, 10.0)
        ref = qp_oracle.solve_dense(q)
        np.testing.assert_allclose(r["du"][b], ref["du"], rtol=0, atol=SOL_ATOL)
        np.testing.assert_allclose(r["dx"][b], ref["dx"], rtol=0, atol=SOL_ATOL)
        np.testing.assert_allclose(r["slack"][b][..., 0], ref["sl"], rtol=0, atol=SOL_ATOL)
        np.testing.assert_allclose(r["slack"][b][..., 1], ref["su"], rtol=0, atol=SOL_ATOL)


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


def test_riccati_ipm_solution_is_feasible(oracle_lib, cfg):
    model = Quad(cfg)
    prob, x0, lin = _instance_set(oracle_lib, cfg, 4, 40, 11, 0.3)
    r = oracle_lib.qp_ipm_batch(lin, prob, x0, model, tol=1e-9)
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
