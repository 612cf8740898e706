"""The CPU oracle against the fixtures generated from the reference itself (tests/golden/make_golden.py).

These pin the oracle before it is trusted as the checker of the HIP path (tests/test_gpu_*.py).
"""
import hashlib

import numpy as np
import pytest

from sdf_nmpc_amd import weights as W
from tolerances import sdf_df_ok, sdf_grad_ok


@pytest.mark.parametrize("variant", ["siren", "stress"])
def test_weights_prng_and_packing_match_golden(golden, oracle_lib, variant):
    g = golden["sdf"]
    seed, wg, bg = g[f"{variant}/spec"]
    params = W.siren_weights(W.DEFAULT_SPEC, seed=int(seed), weight_gain=wg, bias_gain=bg)
    blob = W.pack(W.DEFAULT_SPEC, params)
    assert hashlib.sha256(blob).digest() == g[f"{variant}/sha256"].tobytes()
    # the C PRNG (mirrored in csrc/engine.cpp) is bit-identical to the numpy one
    for stream in (0, 1, 4, 9):
        assert np.array_equal(oracle_lib.prng_uniform(int(seed), stream, 4096),
                              W.prng_uniform(int(seed), stream, 4096))
    spec2, params2 = W.unpack(blob)
    assert spec2 == W.DEFAULT_SPEC
    for k in params:
        assert np.array_equal(params[k], params2[k])


@pytest.mark.parametrize("variant", ["siren", "stress"])
def test_oracle_f64_equals_reference_f64(golden, oracle_lib, variant):
    """fp64 restatement == the reference NeuralDF in fp64 (same algorithm, ~1 ulp of fp64)."""
    g = golden["sdf"]
    seed, wg, bg = g[f"{variant}/spec"]
    net = oracle_lib.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, int(seed), wg, bg))
    df, gp, gf = net.f64(g["input"].astype(np.float64))
    scale = max(1.0, np.abs(g[f"{variant}/grad_f64"]).max())
    assert np.abs(df - g[f"{variant}/df_f64"]).max() < 1e-12
    assert np.abs(gf - g[f"{variant}/grad_f64"]).max() < 1e-12 * scale
    assert np.array_equal(gp, gf[:, :3])


def test_oracle_f64_equals_reference_f64_on_c3_rows(golden, oracle_lib, cfg):
    """The C3-row fixture (every 32nd SDF row of the bench workload): its inputs are the rows the bench
    builds (camera-frame body positions from the synthetic iterate, the instance latents), and the fp64
    restatement reproduces the reference's fp64 outputs on them."""
    from sdf_nmpc_amd import _lib, synth
    g = golden["sdfc3"]
    params = W.siren_weights(W.DEFAULT_SPEC, 0)
    assert hashlib.sha256(W.pack(W.DEFAULT_SPEC, params)).digest() == g["sha256"].tobytes()
    _, dt = _lib.shooting_grid(40, cfg.mpc.T)
    prob = synth.make_problem(cfg, 1024, 40, seed=1000, dt=dt)
    rows = g["rows"]
    x, p = prob["x"].reshape(-1, 10)[rows], prob["p"].reshape(1024 * 41, -1)[rows]
    pos = np.einsum("nji,nj->ni", p[:, 4:13].reshape(-1, 3, 3), x[:, :3] - p[:, 1:4])
    np.testing.assert_array_equal(g["input"][:, :3], pos.astype(np.float32))
    np.testing.assert_array_equal(g["input"][:, 3:], p[:, 17:].astype(np.float32))
    net = oracle_lib.Net(W.DEFAULT_SPEC, params)
    df, gp, _ = net.f64(g["input"].astype(np.float64))
    assert np.abs(df - g["df_f64"]).max() < 1e-12
    assert np.abs(gp - g["grad_f64"]).max() < 1e-12


def test_oracle_f32_within_parity_bar(golden, oracle_lib):
    """fp32 restatement vs the reference fp32 / fp64 on deployed-scale (SIREN-init) weights."""
    g = golden["sdf"]
    net = oracle_lib.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, 0))
    df, gp, gf = net.f32(g["input"])
    assert sdf_df_ok(df, g["siren/df_f64"])
    assert sdf_grad_ok(gp, g["siren/grad_f64"][:, :3])
    assert sdf_df_ok(df, g["siren/df_f32"])


def test_oracle_linearisation_matches_golden(golden, oracle_lib, cfg):
    """Dynamics/cost/constraints vs values from the reference's numpy helpers (+ FD-pinned Jacobians)."""
    L = golden["lin"]
    m = oracle_lib.quad_model(cfg)
    n = L["x"].shape[0]
    for i in range(n):
        x, u, p, dt = L["x"][i], L["u"][i], L["p"][i], float(L["dt"][i])
        xn, AB = oracle_lib.rk4(m, x, u, dt)
        np.testing.assert_allclose(xn, L["xn"][i], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(AB[:, :10], L["A"][i], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(AB[:, 10:], L["B"][i], rtol=1e-10, atol=1e-12)
        y, Jy, yN, JyN = oracle_lib.cost(m, x, u, p)
        np.testing.assert_allclose(y, L["y"][i], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(Jy, L["Jy"][i], rtol=1e-10, atol=1e-12)
        np.testing.assert_allclose(yN, L["yN"][i], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(JyN, L["JyN"][i], rtol=1e-10, atol=1e-12)
        h, Jh, _ = oracle_lib.constr(m, x, p, float(L["df"][i]), L["gdf"][i])
        np.testing.assert_allclose(h, L["h"][i], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(Jh, L["Jh"][i], rtol=1e-10, atol=1e-12)


def test_oracle_shooting_grid_bit_exact(golden, oracle_lib, cfg):
    """ocp.py:21-27: numpy linspace/hstack/diff reproduced bit for bit."""
    G = golden["grid"]
    for N in (20, 40, 60):
        nodes, dt = oracle_lib.shooting_grid(N, cfg.mpc.T, True)
        assert np.array_equal(nodes, G[f"N{N}/uniform/nodes"]) and np.array_equal(dt, G[f"N{N}/uniform/dt"])
        nodes, dt = oracle_lib.shooting_grid(N, cfg.mpc.T, False, cfg.mpc.nb_short_nodes,
                                             cfg.mpc.control_loop_time * 1e-3)
        assert np.array_equal(nodes, G[f"N{N}/nonuniform/nodes"])
        assert np.array_equal(dt, G[f"N{N}/nonuniform/dt"])


def test_oracle_batch_equals_per_node_calls(oracle_lib, cfg):
    """orc_linearize_batch (the CPU baseline) == per-node oracle calls, incl. the terminal node."""
    from sdf_nmpc_amd import synth
    B, N = 3, 5
    prob = synth.make_problem(cfg, B, N, seed=5)
    net = oracle_lib.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, 0))
    m = oracle_lib.quad_model(cfg)
    out = oracle_lib.linearize_batch(m, net, prob["x"], prob["u"], prob["p"], prob["dt"], nthreads=2)
    for b in range(B):
        for k in range(N + 1):
            x, p = prob["x"][b, k], prob["p"][b, k]
            _, _, cpb = oracle_lib.constr(m, x, p, 0.0, np.zeros(3))
            inp = np.concatenate([cpb, p[17:]]).astype(np.float32)[None]
            df, gp, _ = net.f32(inp, full_grad=False)
            h, Jh, _ = oracle_lib.constr(m, x, p, float(df[0]), gp[0].astype(np.float64))
            assert np.array_equal(out["h"][b, k], h) and np.array_equal(out["Jh"][b, k], Jh.T)
            if k < N:
                xn, AB = oracle_lib.rk4(m, x, prob["u"][b, k], prob["dt"][k])
                assert np.array_equal(out["xn"][b, k], xn) and np.array_equal(out["AB"][b, k], AB.T)


# ---- NeuralDF variants (neural_df.py:13-103): act / embed / res / layer sizes / frequencies
from variant_specs import BIAS_GAIN, NET_VARIANTS, SEED, variant_input  # noqa: E402


@pytest.mark.parametrize("name", sorted(NET_VARIANTS))
def test_neural_df_np_matches_reference_variants(golden, name):
    """oracle/neural_df_np.py (the variants' checker) against the reference's own NeuralDF in fp64 on the
    same weights and inputs; the blob round trip and the embedding directions, bit for bit."""
    import neural_df_np
    g, spec = golden["variants"], NET_VARIANTS[name]
    params = W.siren_weights(spec, seed=SEED, bias_gain=BIAS_GAIN)
    blob = W.pack(spec, params)
    assert hashlib.sha256(blob).digest() == g[f"{name}/sha256"].tobytes()
    spec2, params2 = W.unpack(blob)
    assert spec2 == spec and all(np.array_equal(params[k], params2[k]) for k in params)
    if f"{name}/dirs" in g.files:  # weights.embedding_dirs == the buffer the reference builds
        assert np.array_equal(W.embedding_dirs(spec.embed), g[f"{name}/dirs"])
    df, gr, gz = neural_df_np.forward_grad(spec, params, variant_input(g, name), latent_grad=True)
    ref_df, ref_g = g[f"{name}/df_f64"], g[f"{name}/grad_f64"]
    assert np.abs(df - ref_df).max() <= 1e-12 * max(1.0, np.abs(ref_df).max())
    assert np.abs(gr - ref_g[:, :3]).max() <= 1e-12 * max(1.0, np.abs(ref_g).max())
    assert np.abs(gz - ref_g[:, 3:]).max() <= 1e-12 * max(1.0, np.abs(ref_g).max())


def test_oracle_pinned_on_the_scene_net(golden, oracle_lib):
    """The scene-fitted weights (tests/golden/scene.sdfw, tools/fit_scene_sdf.py): the fp64 C restatement
    reproduces the reference NeuralDF's fp64 outputs (df and the full 1 x 131 Jacobian), and the fit is the
    analytic scene to a few centimetres (tests/scene_setup.py)."""
    import os
    g = golden["scene"]
    with open(os.path.join(os.path.dirname(__file__), "golden", "scene.sdfw"), "rb") as f:
        blob = f.read()
    assert hashlib.sha256(blob).digest() == g["sha256"].tobytes()
    spec, params = W.unpack(blob)
    assert spec == W.DEFAULT_SPEC  # the deployed architecture: the fused kernels serve it
    net = oracle_lib.Net(spec, params)
    df, gp, gf = net.f64(g["input"].astype(np.float64))
    scale = max(1.0, np.abs(g["grad_f64"]).max())
    assert np.abs(df - g["df_f64"]).max() < 1e-12 * max(1.0, np.abs(g["df_f64"]).max())
    assert np.abs(gf - g["grad_f64"]).max() < 1e-12 * scale
    assert np.quantile(np.abs(g["df_f64"] - g["scene_df"]), 0.95) < 0.1
