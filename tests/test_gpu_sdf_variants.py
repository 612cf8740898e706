"""NeuralDF variants beyond the deployed net (sdf_nmpc/network/neural_df.py:13-103) on the padded
layer-by-layer schedule (csrc/sdf_wide.hip): activation relu / softplus / sin, embeddings none / pos /
cube / oct / dod / ico with any frequency count, res full / state / latent, layer sizes that are not
multiples of 128.  Checked against the reference's own NeuralDF outputs on the same weights and inputs
(tests/golden/variants_golden.npz, make_golden.py variants) and, in the RTI preparation phase, against the
numpy restatement oracle/neural_df_np.py (pinned to those fixtures by tests/test_oracle.py)."""
import numpy as np
import pytest

from sdf_nmpc_amd import _lib, weights as W
from test_gpu_sdf import eval_device
from variant_specs import BIAS_GAIN, NET_VARIANTS, SEED

pytestmark = pytest.mark.gpu


def _bar(ref64, ref32, scale_floor=1.0):
    """|GPU - ref fp64| allowed: 3x the reference fp32's own error on the case, at least 1e-5 relative to
    the case's magnitude (the north-star bar)."""
    return max(3.0 * np.abs(ref32 - ref64).max(), 1e-5 * max(scale_floor, np.abs(ref64).max()))


@pytest.mark.parametrize("name", sorted(NET_VARIANTS))
def test_variant_vs_reference_golden(gpu_ctx, golden, name):
    g, spec = golden["variants"], NET_VARIANTS[name]
    net = _lib.Net.from_blob(gpu_ctx, W.pack(spec, W.siren_weights(spec, SEED, bias_gain=BIAS_GAIN)))
    try:
        o = eval_device(gpu_ctx, net, g["input"])
    finally:
        net.close()
    assert np.isfinite(o).all()
    df64, df32 = g[f"{name}/df_f64"], g[f"{name}/df_f32"]
    g64, g32 = g[f"{name}/grad_f64"][:, :3], g[f"{name}/grad_f32"][:, :3]
    err_df, err_g = np.abs(o[:, 0] - df64).max(), np.abs(o[:, 1:] - g64).max()
    assert err_df <= _bar(df64, df32), (err_df, np.abs(df32 - df64).max())
    assert err_g <= _bar(g64, g32), (err_g, np.abs(g32 - g64).max())


@pytest.mark.parametrize("name", ["relu_none_state", "softplus_cube_state", "sin_dod_latent"])
def test_variant_in_the_preparation_phase(gpu_ctx, cfg, name):
    """sdfnmpc_linearize with a variant network: the fused sdf row h[2] = flag df + (1 - flag) max_df and
    J_h row 2 = flag (d df / d Co_p_B) W_R_Co^T (gen_model.py:46-61) against the numpy oracle evaluated at
    Co_p_B = W_R_Co^T (x[0:3] - W_p_Co) of every node."""
    import torch
    import neural_df_np
    from sdf_nmpc_amd import synth

    spec = NET_VARIANTS[name]
    params = W.siren_weights(spec, SEED, bias_gain=BIAS_GAIN)
    B, N = 3, 20
    prob = synth.make_problem(cfg, B, N, seed=4)
    net = _lib.Net.from_blob(gpu_ctx, W.pack(spec, params))
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.float64)).to(dev)  # noqa: E731
    bufs = {k: t(prob[k]) for k in ("x", "u", "p", "dt")}
    shapes = {"xn": (B, N, 10), "AB": (B, N, 14, 10), "y": (B, N, 11), "Jy": (B, N, 14, 11), "yN": (B, 4),
              "JyN": (B, 10, 4), "h": (B, N + 1, 3), "Jh": (B, N + 1, 10, 3)}
    for k, s in shapes.items():
        bufs[k] = torch.full(s, float("nan"), dtype=torch.float64, device=dev)
    try:
        _lib.linearize(gpu_ctx, net, _lib.quad_model(cfg), B, N, prob["p"].shape[-1], bufs)
        torch.cuda.synchronize()
    finally:
        net.close()
    x, p = prob["x"].reshape(-1, 10), prob["p"].reshape(-1, prob["p"].shape[-1])
    R = p[:, 4:13].reshape(-1, 3, 3)
    co = np.einsum("nji,nj->ni", R, x[:, :3] - p[:, 1:4])  # W_R_Co^T (x - W_p_Co)
    inp = np.concatenate([co.astype(np.float32), p[:, 17:].astype(np.float32)], 1)
    df, gp = neural_df_np.forward_grad(spec, params, inp)
    flag = p[:, 0]
    h_ref = flag * df + (1.0 - flag) * spec.max_df
    J_ref = flag[:, None] * np.einsum("nc,njc->nj", gp, R)
    h = bufs["h"].cpu().numpy().reshape(-1, 3)
    J = bufs["Jh"].cpu().numpy().reshape(-1, 10, 3)
    scale = max(1.0, np.abs(df).max())
    assert np.abs(h[:, 2] - h_ref).max() <= 1e-5 * scale
    assert np.abs(J[:, :3, 2] - J_ref).max() <= 1e-5 * max(1.0, np.abs(J_ref).max())
    assert np.all(J[:, 3:, 2] == 0.0)


@pytest.mark.parametrize("name", sorted(NET_VARIANTS))
def test_variant_full_jacobian_host_path(gpu_ctx, golden, name):
    """sdfnmpc_sdf_eval_host on a variant net: the full 1 x 131 Jacobian L4CasADi's jac_sdf_l4c returns
    (position and latent columns) against the reference's own autograd Jacobian, and through the CasADi
    external ABI's rows (one row per call, as acados calls it)."""
    g, spec = golden["variants"], NET_VARIANTS[name]
    net = _lib.Net.from_blob(gpu_ctx, W.pack(spec, W.siren_weights(spec, SEED, bias_gain=BIAS_GAIN)))
    try:
        inp = g["input"].astype(np.float64)
        df, gr = net.eval_host(inp)
        df1, gr1 = net.eval_host(inp[5:6])
    finally:
        net.close()
    g64, g32 = g[f"{name}/grad_f64"], g[f"{name}/grad_f32"]
    assert np.abs(df - g[f"{name}/df_f64"]).max() <= _bar(g[f"{name}/df_f64"], g[f"{name}/df_f32"])
    assert np.abs(gr - g64).max() <= _bar(g64, g32), (np.abs(gr - g64).max(), np.abs(g32 - g64).max())
    assert np.abs(gr1[0] - g64[5]).max() <= _bar(g64, g32)
    assert abs(df1[0] - g[f"{name}/df_f64"][5]) <= _bar(g[f"{name}/df_f64"], g[f"{name}/df_f32"])
