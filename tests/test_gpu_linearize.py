"""HIP preparation phase (sdfnmpc_linearize) vs the fp64 oracle, the reference-helper fixtures, and
size-independent properties at the full benchmark size (B=1024, N=40)."""
import numpy as np
import pytest

from sdf_nmpc_amd import _lib, synth, weights as W
from tolerances import lin_close, sdf_df_ok, sdf_grad_ok

pytestmark = pytest.mark.gpu

OUTS = ("xn", "AB", "y", "Jy", "yN", "JyN", "h", "Jh")


def run_gpu(ctx, net, cfg, prob, latent_mode=0):
    import torch
    dev = torch.device("cuda", ctx.device)
    B, N1, _ = prob["x"].shape
    N = N1 - 1
    bufs = {k: torch.from_numpy(np.ascontiguousarray(prob[k])).to(dev) for k in ("x", "u", "p", "dt")}
    shapes = dict(xn=(B, N, 10), AB=(B, N, 14, 10), y=(B, N, 11), Jy=(B, N, 14, 11), yN=(B, 4), JyN=(B, 10, 4),
                  h=(B, N1, 3), Jh=(B, N1, 10, 3))
    for k, s in shapes.items():
        bufs[k] = torch.full(s, float("nan"), dtype=torch.float64, device=dev)
    bufs["sdf"] = torch.full((B, N1, 4), float("nan"), dtype=torch.float32, device=dev)
    torch.cuda.synchronize()
    _lib.linearize(ctx, net, _lib.quad_model(cfg), B, N, prob["p"].shape[-1], bufs, latent_mode)
    ctx.synchronize()
    return {k: bufs[k].cpu().numpy() for k in OUTS + ("sdf",)}


def check_vs_oracle(got, ref, prob, oracle_lib):
    for k in ("xn", "AB", "y", "Jy", "yN", "JyN"):
        assert lin_close(got[k], ref[k]), (k, np.abs(got[k] - ref[k]).max())
    # h[0:2], J_h rows 0,1 (FOV) are pure fp64
    assert lin_close(got["h"][..., :2], ref["h"][..., :2]) and lin_close(got["Jh"][..., :2], ref["Jh"][..., :2])
    # sdf entries: network outputs vs the fp64 oracle evaluated at the same inputs
    flag = prob["p"][..., 0]
    s = got["sdf"].reshape(-1, 4)
    cpb = np.empty((s.shape[0], 3))
    m = oracle_lib.quad_model(_cfg())
    X, P = prob["x"].reshape(-1, 10), prob["p"].reshape(-1, prob["p"].shape[-1])
    for r in range(s.shape[0]):
        cpb[r] = oracle_lib.constr(m, X[r], P[r], 0.0, np.zeros(3))[2]
    inp = np.concatenate([cpb.astype(np.float32).astype(np.float64), P[:, 17:17 + 128].astype(np.float32)], 1)
    net = oracle_lib.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, 0))
    df64, g64, _ = net.f64(inp)
    assert sdf_df_ok(s[:, 0], df64) and sdf_grad_ok(s[:, 1:], g64)
    # h[2] = flag * df + (1 - flag) * max_df, J_h[2] = flag * g W_R_Co^T, composed in fp64 from the fp32 net
    fl = flag.reshape(-1)
    h2 = fl * s[:, 0].astype(np.float64) + (1 - fl) * 1.0
    assert np.array_equal(got["h"].reshape(-1, 3)[:, 2], h2)
    R = P[:, 4:13].reshape(-1, 3, 3)
    J2 = fl[:, None] * np.einsum("rc,rjc->rj", s[:, 1:].astype(np.float64), R)
    np.testing.assert_allclose(got["Jh"].reshape(-1, 10, 3)[:, :3, 2], J2, rtol=1e-12, atol=1e-15)
    assert np.all(got["Jh"].reshape(-1, 10, 3)[:, 3:, 2] == 0)


def _cfg():
    from sdf_nmpc_amd.config import Config
    return Config()


@pytest.mark.parametrize("B,N,tile,mode", [(1, 20, 32, 0), (1, 40, 32, 1), (7, 40, 64, 0), (16, 40, 32, 1), (3, 60, 32, 0)])
def test_linearize_vs_oracle(gpu_ctx, oracle_lib, cfg, B, N, tile, mode):
    prob = synth.make_problem(cfg, B, N, seed=B * 100 + N)
    prob["p"][:, ::3, 0] = 0.0  # flag off at some nodes (gen_model.py:58-61)
    if mode == 1:  # per-node latents (not what set_latent produces, but legal OCP parameters)
        prob["p"][..., 17:] += np.random.default_rng(1).normal(0, 0.3, prob["p"][..., 17:].shape)
    gpu_ctx.set_tile_rows(tile)
    net = _lib.Net.siren(gpu_ctx, 0)
    got = run_gpu(gpu_ctx, net, cfg, prob, mode)
    gpu_ctx.set_tile_rows(32)
    onet = oracle_lib.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, 0))
    ref = oracle_lib.linearize_batch(oracle_lib.quad_model(cfg), onet, prob["x"], prob["u"], prob["p"], prob["dt"], 4)
    for k in OUTS:
        assert np.isfinite(got[k]).all(), k
    check_vs_oracle(got, ref, prob, oracle_lib)


def test_linearize_vs_reference_helper_fixtures(golden, gpu_ctx, cfg):
    """The 64 lin_golden cases (values from the reference's numpy helpers, Jacobians FD-pinned)."""
    L = golden["lin"]
    net = _lib.Net.siren(gpu_ctx, 0)
    for dtv in np.unique(L["dt"]):
        idx = np.nonzero(L["dt"] == dtv)[0]
        B = len(idx)
        prob = {"x": np.repeat(L["x"][idx][:, None], 2, 1), "u": L["u"][idx][:, None].copy(),
                "p": np.repeat(L["p"][idx][:, None], 2, 1), "dt": np.array([dtv])}
        got = run_gpu(gpu_ctx, net, cfg, prob, latent_mode=1)
        assert lin_close(got["xn"][:, 0], L["xn"][idx])
        assert lin_close(got["AB"][:, 0].transpose(0, 2, 1), np.concatenate([L["A"][idx], L["B"][idx]], 2))
        assert lin_close(got["y"][:, 0], L["y"][idx])
        assert lin_close(got["Jy"][:, 0].transpose(0, 2, 1), L["Jy"][idx])
        assert lin_close(got["yN"], L["yN"][idx]) and lin_close(got["JyN"].transpose(0, 2, 1), L["JyN"][idx])
        assert lin_close(got["h"][:, 0, :2], L["h"][idx][:, :2])
        assert lin_close(got["Jh"][:, 0, :, :2].transpose(0, 2, 1), L["Jh"][idx][:, :2])
        # the sdf row compares the HIP fp32 net with the reference fp32 net (torch) at the same input
        assert sdf_df_ok(got["h"][:, 0, 2], L["h"][idx][:, 2])
        assert sdf_grad_ok(got["Jh"][:, 0, :3, 2], L["Jh"][idx][:, 2, :3])


def test_linearize_full_size_properties(gpu_ctx, oracle_lib, cfg):
    """B=1024, N=40 (config C3): deterministic, instance-permutation equivariant (bitwise), flag=0 rows
    exact, and a sampled subset equal to the oracle."""
    B, N = 1024, 40
    prob = synth.make_problem(cfg, B, N, seed=7)
    prob["p"][::5, :, 0] = 0.0
    net = _lib.Net.siren(gpu_ctx, 0)
    a = run_gpu(gpu_ctx, net, cfg, prob)
    b = run_gpu(gpu_ctx, net, cfg, prob)
    for k in OUTS:
        assert np.array_equal(a[k], b[k]), k
        assert np.isfinite(a[k]).all(), k
    perm = np.random.default_rng(0).permutation(B)
    pp = {k: (prob[k][perm] if k in ("x", "u", "p") else prob[k]) for k in ("x", "u", "p", "dt")}
    c = run_gpu(gpu_ctx, net, cfg, pp)
    for k in OUTS:
        assert np.array_equal(a[k][perm], c[k]), k
    off = prob["p"][..., 0] == 0
    assert np.all(a["h"][..., 2][off] == 1.0) and np.all(a["h"][..., :2][off] == 0.0)
    assert np.all(a["Jh"][off] == 0.0)
    sub = np.arange(0, B, 97)
    sp = {k: (prob[k][sub] if k in ("x", "u", "p") else prob[k]) for k in ("x", "u", "p", "dt")}
    onet = oracle_lib.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, 0))
    ref = oracle_lib.linearize_batch(oracle_lib.quad_model(cfg), onet, sp["x"], sp["u"], sp["p"], sp["dt"], 4)
    check_vs_oracle({k: a[k][sub] for k in OUTS + ("sdf",)}, ref, sp, oracle_lib)


def test_split_batch_equals_full_batch_bitwise(gpu_ctx, cfg):
    """Sharding instances (what each rank does at N>1 GPUs) changes nothing, bit for bit."""
    B, N = 64, 40
    prob = synth.make_problem(cfg, B, N, seed=9)
    net = _lib.Net.siren(gpu_ctx, 0)
    full = run_gpu(gpu_ctx, net, cfg, prob)
    for lo, hi in ((0, 23), (23, 64)):
        part = run_gpu(gpu_ctx, net, cfg, {k: (prob[k][lo:hi] if k in ("x", "u", "p") else prob[k])
                                           for k in ("x", "u", "p", "dt")})
        for k in OUTS:
            assert np.array_equal(full[k][lo:hi], part[k]), k
