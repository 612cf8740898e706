"""The acados-style phase split (include/sdfnmpc.h): sdfnmpc_rti_prepare (linearisation + the QP's stage
records, the record pack running beside the SDF kernel) followed by sdfnmpc_qp_feedback (the IPM) gives
bitwise the results of sdfnmpc_linearize + sdfnmpc_qp_solve, with and without flags.sdf_cost (whose pack
must wait for the SDF kernel), and for the wide network; feedback without a matching preparation fails
loudly.  rti_phase 1 / 2 split: ocp.py:110."""
import copy

import numpy as np
import pytest

from sdf_nmpc_amd import _lib, synth, weights as W
from sdf_nmpc_amd.model import Quad

pytestmark = pytest.mark.gpu

OUT = ("xn", "AB", "y", "Jy", "yN", "JyN", "h", "Jh", "dx", "du", "slack", "status", "iters", "res")


def _bufs(gpu_ctx, cfg, B, N, seed, sdf_cost):
    import torch
    dev = torch.device("cuda", gpu_ctx.device)
    prob = synth.make_problem(cfg, B, N, seed=seed, sdf_cost=sdf_cost)
    x0 = prob["x"][:, 0] + np.random.default_rng(seed).normal(0, 0.05, (B, 10))
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
    return prob, t


def _model(cfg, sdf_cost):
    c = copy.deepcopy(cfg)
    c.flags["sdf_cost"] = sdf_cost
    return Quad(c)


@pytest.mark.parametrize("B,N,sdf_cost,wide", [(64, 20, False, False), (33, 40, True, False), (16, 30, False, True)])
def test_prepare_feedback_bitwise_equals_linearize_qp_solve(gpu_ctx, cfg, B, N, sdf_cost, wide):
    net = (_lib.Net.from_blob(gpu_ctx, W.pack(W.WIDE_SPEC, W.siren_weights(W.WIDE_SPEC, 0))) if wide
           else _lib.Net.siren(gpu_ctx, 0))
    model = _model(cfg, sdf_cost)
    opts = _lib.qp_opts(model)
    qm = _lib.quad_model(cfg)
    prob, ta = _bufs(gpu_ctx, cfg, B, N, 7, sdf_cost)
    _, tb = _bufs(gpu_ctx, cfg, B, N, 7, sdf_cost)
    np_ = prob["p"].shape[-1]
    _lib.linearize(gpu_ctx, net, qm, B, N, np_, ta)
    _lib.qp_solve(gpu_ctx, opts, B, N, ta)
    _lib.rti_prepare(gpu_ctx, net, qm, opts, B, N, np_, tb)
    _lib.qp_feedback(gpu_ctx, opts, B, N, tb)
    gpu_ctx.synchronize()
    assert (ta["status"].cpu().numpy() == 0).all()
    for k in OUT:
        np.testing.assert_array_equal(ta[k].cpu().numpy(), tb[k].cpu().numpy(), err_msg=k)


def test_feedback_needs_a_matching_preparation(gpu_ctx, cfg):
    B, N = 4, 20
    net = _lib.Net.siren(gpu_ctx, 0)
    model = _model(cfg, False)
    opts = _lib.qp_opts(model)
    qm = _lib.quad_model(cfg)
    prob, t = _bufs(gpu_ctx, cfg, B, N, 3, False)
    np_ = prob["p"].shape[-1]
    _lib.linearize(gpu_ctx, net, qm, B, N, np_, t)
    with pytest.raises(_lib.SdfnmpcError, match="rti_prepare"):
        _lib.qp_feedback(gpu_ctx, opts, B, N, t)           # no preparation at all
    _lib.rti_prepare(gpu_ctx, net, qm, opts, B, N, np_, t)
    _lib.qp_feedback(gpu_ctx, opts, B, N, t)
    with pytest.raises(_lib.SdfnmpcError, match="rti_prepare"):
        _lib.qp_feedback(gpu_ctx, opts, B, N, t)           # one feedback per preparation
    _lib.rti_prepare(gpu_ctx, net, qm, opts, B, N, np_, t)
    with pytest.raises(_lib.SdfnmpcError, match="rti_prepare"):
        _lib.qp_feedback(gpu_ctx, opts, B - 1, N, t)       # another batch than the one prepared
    gpu_ctx.synchronize()


@pytest.mark.parametrize("B,N,graph", [(1, 40, False), (8, 20, False), (1, 40, True), (8, 20, True)])
def test_bound_rti_step_bitwise_equals_per_call_phases(gpu_ctx, cfg, B, N, graph):
    """_lib.RtiStep (argument blocks bound once; graph=True: the step captured into a HIP graph by
    sdfnmpc_step_create and replayed, the B = 1 latency leg of bench.py) runs the same three entry points
    as the per-call wrappers: closed-loop steps, bitwise the same iterates and outputs."""
    import torch
    net = _lib.Net.siren(gpu_ctx, 0)
    model = _model(cfg, False)
    opts = _lib.qp_opts(model)
    qm = _lib.quad_model(cfg)
    prob, ta = _bufs(gpu_ctx, cfg, B, N, 11, False)
    _, tb = _bufs(gpu_ctx, cfg, B, N, 11, False)
    np_ = prob["p"].shape[-1]
    ua = torch.empty((B, 4), dtype=torch.float64, device=ta["x"].device)
    ub = torch.empty_like(ua)
    if graph:  # create runs one step eagerly: the per-call side takes one step first
        _lib.rti_prepare(gpu_ctx, net, qm, opts, B, N, np_, ta)
        _lib.qp_feedback(gpu_ctx, opts, B, N, ta)
        _lib.rti_apply(gpu_ctx, B, N, ta["x"], ta["u"], ta["dx"], ta["du"], ua, ta["status"])
    step = _lib.RtiStep(gpu_ctx, net, qm, opts, B, N, np_, tb, u0=ub, graph=graph)
    for _ in range(2):
        _lib.rti_prepare(gpu_ctx, net, qm, opts, B, N, np_, ta)
        _lib.qp_feedback(gpu_ctx, opts, B, N, ta)
        _lib.rti_apply(gpu_ctx, B, N, ta["x"], ta["u"], ta["dx"], ta["du"], ua, ta["status"])
        step()
    gpu_ctx.synchronize()
    for k in OUT + ("x", "u"):
        np.testing.assert_array_equal(ta[k].cpu().numpy(), tb[k].cpu().numpy(), err_msg=k)
    np.testing.assert_array_equal(ua.cpu().numpy(), ub.cpu().numpy())


def test_graph_step_refuses_launch_after_workspace_growth(gpu_ctx, cfg):
    """a captured step addresses the context's workspaces; a later call with a larger batch grows
    (reallocates) them, and the launch then fails instead of running on freed device memory."""
    import torch
    B, N = 1, 40
    ctx = _lib.Context(gpu_ctx.device)  # a fresh context: its workspaces are sized by this test's calls only
    net = _lib.Net.siren(ctx, 0)
    qm = _lib.quad_model(cfg)
    opts = _lib.qp_opts(Quad(cfg))
    prob, tb = _bufs(ctx, cfg, B, N, 11, False)
    ub = torch.empty((B, 4), dtype=torch.float64, device=tb["x"].device)
    step = _lib.RtiStep(ctx, net, qm, opts, B, N, prob["p"].shape[-1], tb, u0=ub, graph=True)
    step()
    ctx.synchronize()
    prob2, t2 = _bufs(ctx, cfg, 64, N, 11, False)  # grows the QP workspace and the SDF buffers
    _lib.rti_prepare(ctx, net, qm, opts, 64, N, prob2["p"].shape[-1], t2)
    _lib.qp_feedback(ctx, opts, 64, N, t2)
    ctx.synchronize()
    with pytest.raises(_lib.SdfnmpcError, match="reallocated"):
        step()
    del step
    net.close()
    ctx.close()
