"""Wide NeuralDF (config C5: layer_sizes [1024,1024,512,256]) on the layer-by-layer GEMM schedule
(csrc/sdf_wide.hip) against the reference's own NeuralDF at those widths (tests/golden/wide_golden.npz)
and the fp64 C oracle; the same parity bar as the deployed net (tests/tolerances.py)."""
import os

import numpy as np
import pytest

from sdf_nmpc_amd import _lib, weights as W
from test_gpu_sdf import eval_device
from tolerances import sdf_df_err, sdf_df_ok, sdf_grad_err, sdf_grad_ok

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wg():
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "wide_golden.npz"))


@pytest.fixture(scope="module")
def wide_net(gpu_ctx):
    net = _lib.Net.from_blob(gpu_ctx, W.pack(W.WIDE_SPEC, W.siren_weights(W.WIDE_SPEC, 0)))
    yield net
    net.close()


def test_wide_vs_reference_golden(gpu_ctx, wide_net, wg):
    o = eval_device(gpu_ctx, wide_net, wg["input"])
    for tag in ("f32", "f64"):
        assert sdf_df_ok(o[:, 0], wg[f"df_{tag}"]), sdf_df_err(o[:, 0], wg[f"df_{tag}"])
        assert sdf_grad_ok(o[:, 1:], wg[f"grad_{tag}"]), sdf_grad_err(o[:, 1:], wg[f"grad_{tag}"])


@pytest.mark.parametrize("rows,rpi", [(1, 1), (129, 1), (300, 61), (1000, 41)])
def test_wide_ragged_rows_vs_oracle(gpu_ctx, wide_net, oracle_lib, rows, rpi):
    """Row counts that are not GEMM-tile multiples, shared latents (hoisted once per instance)."""
    rng = np.random.default_rng(rows + 7)
    n_inst = (rows + rpi - 1) // rpi
    lat = rng.normal(size=(n_inst, 128)).astype(np.float32)
    pos = rng.uniform(-4, 4, (rows, 3)).astype(np.float32)
    inp = np.concatenate([pos, lat[np.arange(rows) // rpi]], 1)
    o = eval_device(gpu_ctx, wide_net, inp, rpi, latent=lat)
    onet = oracle_lib.Net(W.WIDE_SPEC, W.siren_weights(W.WIDE_SPEC, 0))
    df64, gp64, _ = onet.f64(inp.astype(np.float64))
    assert np.isfinite(o).all()
    assert sdf_df_ok(o[:, 0], df64), sdf_df_err(o[:, 0], df64)
    assert sdf_grad_ok(o[:, 1:], gp64), sdf_grad_err(o[:, 1:], gp64)


def test_wide_rows_independent_bitwise(gpu_ctx, wide_net):
    rng = np.random.default_rng(5)
    inp = np.concatenate([rng.uniform(-3, 3, (300, 3)), rng.normal(size=(300, 128))], 1).astype(np.float32)
    a = eval_device(gpu_ctx, wide_net, inp)
    perm = rng.permutation(300)
    b = eval_device(gpu_ctx, wide_net, inp[perm])
    assert np.array_equal(a[perm], b)


def test_wide_full_jacobian_vs_oracle(gpu_ctx, wide_net, oracle_lib, wg):
    """The 1 x 131 Jacobian (jac_sdf_l4c's latent columns included) of the C5 net through the host path,
    against the fp64 C oracle."""
    inp = wg["input"][:40].astype(np.float64)
    df, gr = wide_net.eval_host(inp, want_grad=True)
    onet = oracle_lib.Net(W.WIDE_SPEC, W.siren_weights(W.WIDE_SPEC, 0))
    df64, _, g64 = onet.f64(inp)
    assert sdf_df_ok(df, df64), sdf_df_err(df, df64)
    assert sdf_grad_ok(gr[:, :3], g64[:, :3]), sdf_grad_err(gr[:, :3], g64[:, :3])
    assert np.abs(gr[:, 3:] - g64[:, 3:]).max() <= 1e-5 * max(1.0, np.abs(g64[:, 3:]).max())


def test_wide_linearize_matches_oracle(gpu_ctx, cfg, oracle_lib):
    """sdfnmpc_linearize with the wide net: h[2] / J_h row 2 from the fused final kernel vs the oracle."""
    import torch
    from sdf_nmpc_amd import synth
    from sdf_nmpc_amd.model import Quad

    B, N = 3, 20
    prob = synth.make_problem(cfg, B, N, seed=2)
    net = _lib.Net.from_blob(gpu_ctx, W.pack(W.WIDE_SPEC, W.siren_weights(W.WIDE_SPEC, 0)))
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)  # noqa: E731
    bufs = {k: t(prob[k]) for k in ("x", "u", "p", "dt")}
    shapes = {"xn": (B, N, 10), "AB": (B, N, 14, 10), "y": (B, N, 11), "Jy": (B, N, 14, 11), "yN": (B, 4),
              "JyN": (B, 10, 4), "h": (B, N + 1, 3), "Jh": (B, N + 1, 10, 3)}
    for k, s in shapes.items():
        bufs[k] = torch.full(s, float("nan"), dtype=torch.float64, device=dev)
    _lib.linearize(gpu_ctx, net, _lib.quad_model(cfg), B, N, prob["p"].shape[-1], bufs)
    torch.cuda.synchronize()
    onet = oracle_lib.Net(W.WIDE_SPEC, W.siren_weights(W.WIDE_SPEC, 0))
    m = oracle_lib.quad_model(cfg, 1.0)
    ref = oracle_lib.linearize_batch(m, onet, prob["x"], prob["u"], prob["p"], prob["dt"])
    h = bufs["h"].cpu().numpy()
    assert np.abs(h[..., 2] - ref["h"][..., 2]).max() <= 1e-5
    assert np.abs(bufs["Jh"].cpu().numpy()[..., 2] - ref["Jh"][..., 2]).max() <= 1e-5 * max(1.0, np.abs(ref["Jh"]).max())
    assert np.abs(h[..., :2] - ref["h"][..., :2]).max() <= 1e-9
