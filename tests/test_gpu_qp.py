"""Batched RTI QP (rti_qp.hip via sdfnmpc_qp_solve) vs the dense reference IPM (oracle/qp_oracle.py)."""
import numpy as np
import pytest

from sdf_nmpc_amd import _lib, synth
from sdf_nmpc_amd.model import Quad

pytestmark = pytest.mark.gpu

QP_TOL = 1e-10          # IPM stop tolerance used for the parity runs
SOL_ATOL = 1e-5         # |du - du_ref|, |dx - dx_ref| (IPM solutions agree to ~sqrt(mu) level)


def setup(gpu_ctx, cfg, B, N, seed, x0_noise=0.05, sdf_cost=False):
    import torch
    dev = torch.device("cuda", gpu_ctx.device)
    prob = synth.make_problem(cfg, B, N, seed=seed, sdf_cost=sdf_cost)
    rng = np.random.default_rng(seed)
    x0 = prob["x"][:, 0] + rng.normal(0, x0_noise, (B, 10))
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
         dict(x=prob["x"], u=prob["u"], p=prob["p"], dt=prob["dt"], x0=x0, yref=prob["yref"], W=prob["W"],
              yNref=prob["yN"], WN=prob["WN"]).items()}
    sh = dict(xn=(B, N, 10), AB=(B, N, 14, 10), y=(B, N, 11), Jy=(B, N, 14, 11), yN=(B, 4), JyN=(B, 10, 4),
              h=(B, N + 1, 3), Jh=(B, N + 1, 10, 3), dx=(B, N + 1, 10), du=(B, N, 4), slack=(B, N + 1, 3, 2),
              res=(B, 2))
    for k, s in sh.items():
        t[k] = torch.full(s, float("nan"), dtype=torch.float64, device=dev)
    t["status"] = torch.full((B,), -1, dtype=torch.int32, device=dev)
    t["iters"] = torch.full((B,), -1, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    net = _lib.Net.siren(gpu_ctx, 0)
    _lib.linearize(gpu_ctx, net, _lib.quad_model(cfg), B, N, prob["p"].shape[-1], t)
    return prob, x0, t


def solve(gpu_ctx, cfg, t, B, N, sdf_cost=False, **kw):
    import copy
    c = copy.deepcopy(cfg)
    c.flags["sdf_cost"] = sdf_cost
    model = Quad(c)
    _lib.qp_solve(gpu_ctx, _lib.qp_opts(model, **kw), B, N, t)
    gpu_ctx.synchronize()
    return model


@pytest.mark.parametrize("B,N,seed", [(3, 20, 1), (2, 40, 2)])
def test_qp_matches_dense_oracle(gpu_ctx, oracle_lib, cfg, B, N, seed):
    import qp_oracle
    prob, x0, t = setup(gpu_ctx, cfg, B, N, seed)
    model = solve(gpu_ctx, cfg, t, B, N, tol=QP_TOL)
    assert (t["status"].cpu().numpy() == 0).all()
    lin = {k: t[k].cpu().numpy() for k in ("xn", "AB", "y", "Jy", "yN", "JyN", "h", "Jh")}
    for b in range(B):
        q = qp_oracle.stage_qp({k: v[b] for k, v in lin.items()}, prob["x"][b], prob["u"][b], x0[b], prob["yref"][b],
                               prob["W"][b], prob["yN"][b], prob["WN"][b], prob["dt"], model, 10.0)
        ref = qp_oracle.solve_dense(q)
        np.testing.assert_allclose(t["du"][b].cpu().numpy(), ref["du"], rtol=0, atol=SOL_ATOL)
        np.testing.assert_allclose(t["dx"][b].cpu().numpy(), ref["dx"], rtol=0, atol=SOL_ATOL)
        sl = t["slack"][b].cpu().numpy()
        np.testing.assert_allclose(sl[..., 0], ref["sl"], rtol=0, atol=SOL_ATOL)
        np.testing.assert_allclose(sl[..., 1], ref["su"], rtol=0, atol=SOL_ATOL)


def test_qp_full_size_feasibility_and_determinism(gpu_ctx, cfg):
    """B=1024, N=40: every instance converges within qp_solver_iter_max = 100 (ocp.py:115); the solution
    satisfies the input boxes, x0 and the linearised dynamics; two solves agree bit for bit."""
    B, N = 1024, 40
    prob, x0, t = setup(gpu_ctx, cfg, B, N, seed=3)
    model = solve(gpu_ctx, cfg, t, B, N)
    st, it = t["status"].cpu().numpy(), t["iters"].cpu().numpy()
    assert (st == 0).all() and it.max() <= 100
    du, dx = t["du"].cpu().numpy(), t["dx"].cpu().numpy()
    u_new = prob["u"] + du
    assert (u_new >= model.lbu - 1e-7).all() and (u_new <= model.ubu + 1e-7).all()
    np.testing.assert_allclose(dx[:, 0], x0 - prob["x"][:, 0], atol=1e-12)
    AB = t["AB"].cpu().numpy()
    c = t["xn"].cpu().numpy() - prob["x"][:, 1:]
    pred = np.einsum("bkji,bkj->bki", AB[:, :, :10], dx[:, :-1]) + np.einsum("bkji,bkj->bki", AB[:, :, 10:], du) + c
    np.testing.assert_allclose(dx[:, 1:], pred, atol=1e-9)
    du1 = du.copy()
    solve(gpu_ctx, cfg, t, B, N)
    assert np.array_equal(du1, t["du"].cpu().numpy())


def test_rti_apply(gpu_ctx):
    import torch
    dev = torch.device("cuda", gpu_ctx.device)
    B, N = 5, 7
    g = torch.Generator().manual_seed(0)
    x, u = torch.randn(B, N + 1, 10, dtype=torch.float64), torch.randn(B, N, 4, dtype=torch.float64)
    dx, du = torch.randn(B, N + 1, 10, dtype=torch.float64), torch.randn(B, N, 4, dtype=torch.float64)
    xd, ud, dxd, dud = (a.to(dev) for a in (x, u, dx, du))
    u0 = torch.zeros(B, 4, dtype=torch.float64, device=dev)
    torch.cuda.synchronize()
    _lib.rti_apply(gpu_ctx, B, N, xd, ud, dxd, dud, u0)
    gpu_ctx.synchronize()
    assert torch.equal(xd.cpu(), x + dx) and torch.equal(ud.cpu(), u + du) and torch.equal(u0.cpu(), (u + du)[:, 0])


@pytest.mark.parametrize("B,N,seed,noise", [(64, 40, 3, 0.05), (32, 20, 9, 0.5)])
def test_qp_matches_riccati_oracle_batch(gpu_ctx, oracle_lib, cfg, B, N, seed, noise):
    """A wider batch against the structured C IPM (oracle/qp_ipm.c), itself pinned to the dense IPM."""
    prob, x0, t = setup(gpu_ctx, cfg, B, N, seed, x0_noise=noise)
    model = solve(gpu_ctx, cfg, t, B, N, tol=QP_TOL)
    assert (t["status"].cpu().numpy() == 0).all()
    lin = {k: t[k].cpu().numpy() for k in ("xn", "AB", "y", "Jy", "yN", "JyN", "h", "Jh")}
    ref = oracle_lib.qp_ipm_batch(lin, prob, x0, model, tol=QP_TOL, nthreads=8)
    assert (ref["status"] == 0).all()
    np.testing.assert_allclose(t["du"].cpu().numpy(), ref["du"], rtol=0, atol=SOL_ATOL)
    np.testing.assert_allclose(t["dx"].cpu().numpy(), ref["dx"], rtol=0, atol=SOL_ATOL)
    np.testing.assert_allclose(t["slack"].cpu().numpy(), ref["slack"], rtol=0, atol=SOL_ATOL)


def test_qp_sdf_cost_matches_riccati_oracle(gpu_ctx, oracle_lib, cfg):
    """flags.sdf_cost: the 12th residual (1 - s/2)^4 formed by the pack kernel from h[2], J_h[2]."""
    B, N = 16, 40
    prob, x0, t = setup(gpu_ctx, cfg, B, N, 21, x0_noise=0.2, sdf_cost=True)
    model = solve(gpu_ctx, cfg, t, B, N, sdf_cost=True, tol=QP_TOL)
    assert model.ny == 12 and (t["status"].cpu().numpy() == 0).all()
    lin = {k: t[k].cpu().numpy() for k in ("xn", "AB", "y", "Jy", "yN", "JyN", "h", "Jh")}
    ref = oracle_lib.qp_ipm_batch(lin, prob, x0, model, tol=QP_TOL, nthreads=8)
    assert (ref["status"] == 0).all()
    np.testing.assert_allclose(t["du"].cpu().numpy(), ref["du"], rtol=0, atol=SOL_ATOL)
    np.testing.assert_allclose(t["dx"].cpu().numpy(), ref["dx"], rtol=0, atol=SOL_ATOL)
    # and the residual changes the solution (the term is live)
    _, _, t2 = setup(gpu_ctx, cfg, B, N, 21, x0_noise=0.2)
    solve(gpu_ctx, cfg, t2, B, N, tol=QP_TOL)
    assert np.abs(t2["du"].cpu().numpy() - ref["du"]).max() > 1e-6
