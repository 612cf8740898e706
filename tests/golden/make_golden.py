#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

Run in the build container only (``/root/reference`` does not exist on the GPU box):

    python tests/golden/make_golden.py

What is pinned to what:
  * sdf_golden.npz     -- the reference's own ``NeuralDF`` (sdf_nmpc/network/neural_df.py:7-103),
                          imported from /root/reference with a no-op ``casadi`` module (embeddings.py:3
                          imports casadi without using it), weights from our seeded PRNG
                          (sdf-nmpc_amd/weights.py) loaded through ``load_state_dict``.  fp32 and fp64
                          forward, d df/d pos and d df/d input(131) by torch autograd (what L4CasADi's
                          ``jac_sdf_l4c`` returns, gen_model.py:39).
  * lin_golden.npz     -- dynamics / cost / constraint values computed with the reference's own numpy
                          helpers (utils/math.py: quat2rot :7, euler2rot :26, hamilton_prod :177,
                          invert :169) assembled as in model/quad_rollpitchyawrate.py:19-55 and
                          model/cost_const_helpers.py:48-75 / gen_model.py:46-61; RK4 (acados ERK,
                          ocp.py:106) on top; Jacobians by torch autograd of an fp64 restatement that
                          is asserted equal (values) to the helper-based version and to central
                          finite differences of it (derivatives).  CasADi/acados are not installed,
                          so this is the strongest pin available here.
  * grid_golden.npz    -- ocp.py:21-27 shooting grid (numpy linspace/hstack/diff, bit-exact target).
  * ts_golden.npz      -- the state_dict layout (names, shapes, embedding buffers) and the w0 / max_df
                          attributes of ``torch.jit.script(NeuralDF(...))`` -- what df_train.py saves and
                          gen_model.py:32 loads -- pinning weights.from_torchscript (data only: no
                          TorchScript archive, which would carry the reference's code, is committed).
  * refgen_golden.npz  -- the reference's own ``RefGen`` (ref_gen.py:7-130): gen_ref_list_wps over random
                          paths for every yaw mode, stop-and-turn on/off, gen_ref_joystick, from_x0.
  * vae_golden.npz     -- the reference's own ``Encoder`` (network/vae.py:6-46, resnet.py:5-56) in eval
                          mode and its preprocessing chain (vae.py:15-24: Reshape, ClipDistance,
                          Depth2Range from utils/preprocessing.py), weights from
                          sdf_nmpc_amd.vae.synthetic_encoder, images from synth.depth_images: latent
                          means in fp32 and fp64, sampled preprocessed pixels, per-stage channel sums.
  * wide_golden.npz    -- the reference's own ``NeuralDF`` at config C5's widths [1024,1024,512,256]
                          (SIREN-init seed 0): df and d df / d pos in fp32 and fp64.
  * flags_golden.npz   -- the flag space (flags_golden below): polynomial_3variate's term order / values,
                          stability.get_r_tilde_max, set_ref with the stability terminal row.
  * params_golden.npz  -- the reference's own ``Nmpc.set_latent`` / ``Nmpc.set_ref`` /
                          ``Quad.formate_ref`` (controller.py:50-54,133-142, quad_rollpitchyawrate.py:
                          62-65) called unbound on small stand-in objects; ``Config`` from the
                          reference's default.yaml (utils/config.py:32-44).
"""
import hashlib
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, ROOT)

import sdf_nmpc_amd  # noqa: E402
from sdf_nmpc_amd import weights as W  # noqa: E402

# -- the reference imports third-party modules that are absent here; none of them is used by the
#    functions exercised below (casadi only at import time in embeddings.py:3 / math.py:3 /
#    config.py:3; acados_template/l4casadi only by ocp.py / gen_model.py class bodies we never run).
for name in ("casadi", "acados_template", "l4casadi"):
    mod = types.ModuleType(name)
    if name == "acados_template":
        mod.AcadosOcp = mod.AcadosOcpSolver = mod.AcadosModel = object
    sys.modules.setdefault(name, mod)
sys.path.insert(0, REF)
from sdf_nmpc.network.neural_df import NeuralDF  # noqa: E402
from sdf_nmpc.utils import math as rmath  # noqa: E402
from sdf_nmpc.utils.config import Config  # noqa: E402

torch.set_num_threads(1)
CFG = Config(os.path.join(REF, "sdf_nmpc/config/default.yaml"))

VARIANTS = {  # name -> (seed, weight_gain, bias_gain)
    "siren": (0, 1.0, 0.0),
    "stress": (1, 3.0, 1.0),
}


def ref_net(spec, params, dtype):
    net = NeuralDF(nb_states=3, size_latent=spec.size_latent, signed=True, max_df=spec.max_df,
                   res=spec.res, w0=spec.w0, embed=spec.embed, act=spec.act,
                   layer_sizes=list(spec.layer_sizes), dropout_rate=0.1, nb_freqs=spec.nb_freqs)
    sd = net.state_dict()
    for k, v in params.items():
        assert sd[k].shape == v.shape, k
        sd[k] = torch.from_numpy(v.copy())
    net.load_state_dict(sd)
    net.eval()  # dropout = identity (gen_model.py:34)
    return net.to(dtype)


def sample_inputs(rng, n, L):
    """Body positions in the camera-origin frame (the SDF input Co_p_B, gen_model.py:50)."""
    hf, vf = CFG.sensor.hfov, CFG.sensor.vfov
    pos = []
    k = n // 2
    d = rng.uniform(0.05, 6.0, k)
    az = rng.uniform(-hf, hf, k)
    el = rng.uniform(-vf, vf, k)
    pos.append(np.stack([d * np.cos(el) * np.cos(az), d * np.cos(el) * np.sin(az), d * np.sin(el)], 1))
    k2 = n // 4
    v = rng.normal(size=(k2, 3))
    pos.append(v / np.linalg.norm(v, axis=1, keepdims=True) * rng.uniform(0, 1, (k2, 1)))
    k3 = n - k - k2 - 8
    pos.append(rng.uniform(-6, 6, (k3, 3)))
    pos.append(np.array([[0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, -1], [10, 0, 0], [-10, 10, 0],
                         [10, -10, 10], [1e-3, -1e-3, 2e-3]], dtype=np.float64))
    pos = np.concatenate(pos, 0).astype(np.float32)
    lat = rng.normal(size=(n, L)).astype(np.float32)
    lat[-16:] *= 3.0
    return np.concatenate([pos, lat], 1)


def sdf_golden(n=256):
    out = {}
    rng = np.random.default_rng(1234)
    spec = W.DEFAULT_SPEC
    inp = sample_inputs(rng, n, spec.size_latent)
    out["input"] = inp
    for name, (seed, wg, bg) in VARIANTS.items():
        params = W.siren_weights(spec, seed=seed, weight_gain=wg, bias_gain=bg)
        blob = W.pack(spec, params)
        out[f"{name}/spec"] = np.array([seed, wg, bg])
        out[f"{name}/sha256"] = np.frombuffer(hashlib.sha256(blob).digest(), dtype=np.uint8)
        for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
            net = ref_net(spec, params, dt)
            if tag == "f32":  # embedding directions: reference buffer == our fp32 construction
                assert np.array_equal(net.embed.dirs.numpy(), W.embedding_dirs(spec.embed))
                assert np.array_equal(net.embed.freq_bands.numpy(),
                                      (2.0 ** np.arange(spec.nb_freqs)).astype(np.float32))
            x = torch.from_numpy(inp).to(dt).requires_grad_(True)
            df = net(x)
            (g,) = torch.autograd.grad(df.sum(), x)
            out[f"{name}/df_{tag}"] = df.detach().numpy()[:, 0]
            out[f"{name}/grad_{tag}"] = g.numpy()  # [n,131]; [:, :3] = d df / d Co_p_B
            if tag == "f64":  # per-layer pre-activations for 8 cases (debug aid)
                with torch.no_grad():
                    xs = x[:8]
                    e = net.layers["embeddings"](xs[:, :3])
                    z = xs[:, 3:]
                    m1, m2 = net.layers["main1"], net.layers["main2"]
                    a1 = m1[0](torch.cat([e, z], 1)); h1 = m1[1](a1)
                    a2 = m1[3](h1); h2 = m1[4](a2)
                    a3 = m2[0](torch.cat([h2, e, z], 1)); h3 = m2[1](a3)
                    a4 = m2[3](h3); h4 = m2[4](a4)
                    for k_, v_ in (("e", e), ("a1", a1), ("a2", a2), ("a3", a3), ("a4", a4)):
                        out[f"{name}/act_{k_}"] = v_.numpy()
    np.savez_compressed(os.path.join(HERE, "sdf_golden.npz"), **out)
    print("sdf_golden.npz", {k: v.shape for k, v in out.items() if "act" not in k})


# ---------------------------------------------------------------------------------------------
# dynamics / cost / constraints of the default 'att' model
# ---------------------------------------------------------------------------------------------
G = 9.81
LIM = CFG.robot.limits
P_IDX = CFG.mpc.p_idx


def f_expl_np(x, u):
    """quad_rollpitchyawrate.py:19-42 with the reference's numpy helpers."""
    q = x[3:7] / np.linalg.norm(x[3:7])
    th = np.arctan2(q[3], q[0])
    qyaw = np.array([np.cos(th), 0, 0, np.sin(th)])
    gamma, roll, pitch, wz = u[0] * LIM.gamma, u[1] * LIM.roll, u[2] * LIM.pitch, u[3] * LIM.wz
    V_R_B = rmath.euler2rot(np.array([roll, pitch, 0.0]))
    W_R_V = rmath.quat2rot(qyaw)
    W_a = (W_R_V @ V_R_B) @ np.array([0, 0, gamma]) + np.array([0, 0, -G])
    dq = rmath.hamilton_prod(q, np.array([0, 0, 0, wz])) / 2
    return np.concatenate([x[7:10], dq, W_a]), W_a


def y_np(x, u, p):
    """quad_rollpitchyawrate.py:48-55 (stage/terminal NONLINEAR_LS residual)."""
    q = x[3:7] / np.linalg.norm(x[3:7])
    q_d = p[P_IDX.q_d]
    q_e = rmath.hamilton_prod(q_d, rmath.invert(q))
    _, W_a = f_expl_np(x, u)
    y = np.concatenate([x[:3], [q_e[3]], x[7:10], [u[1] * LIM.roll, u[2] * LIM.pitch, u[3] * LIM.wz, W_a[2]]])
    return y, np.concatenate([x[:3], [q_e[3]]])


def h_np(x, p, df, max_df=1.0):
    """cost_const_helpers.py:48-75 (FOV, trigo form) + gen_model.py:46-61 (sdf, flag)."""
    W_R_Co = p[P_IDX.W_R_Co].reshape(3, 3)  # == casadi reshape((3,3)).T
    W_p_Co = p[P_IDX.W_p_Co]
    flag = p[P_IDX.flag]
    Co_p_B = W_R_Co.T @ (x[:3] - W_p_Co)
    Co_p_C = Co_p_B + CFG.sensor.B_R_C.T @ np.array(CFG.sensor.B_p_C) + np.array([CFG.mpc.fov_const_offset, 0, 0])
    hfov = flag * np.arctan2(Co_p_C[1], Co_p_C[0])
    vfov = flag * np.arctan2(Co_p_C[2], np.linalg.norm(Co_p_C[:2]))
    s = flag * df + (1 - flag) * max_df
    return np.array([hfov, vfov, s]), Co_p_B


def rk4_np(x, u, dt):
    f = lambda z: f_expl_np(z, u)[0]
    k1 = f(x); k2 = f(x + dt / 2 * k1); k3 = f(x + dt / 2 * k2); k4 = f(x + dt * k3)
    return x + dt / 6 * (k1 + 2 * k2 + 2 * k3 + k4)


def _t_hprod(a, b):
    return torch.stack([a[0]*b[0] - a[1]*b[1] - a[2]*b[2] - a[3]*b[3],
                        a[0]*b[1] + a[1]*b[0] + a[2]*b[3] - a[3]*b[2],
                        a[0]*b[2] - a[1]*b[3] + a[2]*b[0] + a[3]*b[1],
                        a[0]*b[3] + a[1]*b[2] - a[2]*b[1] + a[3]*b[0]])


def f_t(x, u):
    q = x[3:7] / torch.linalg.norm(x[3:7])
    th = torch.atan2(q[3], q[0])
    c, s = torch.cos(th), torch.sin(th)
    gamma, roll, pitch, wz = u[0] * LIM.gamma, u[1] * LIM.roll, u[2] * LIM.pitch, u[3] * LIM.wz
    sr, cr, sp, cp = torch.sin(roll), torch.cos(roll), torch.sin(pitch), torch.cos(pitch)
    b = torch.stack([cr * sp, -sr, cr * cp]) * gamma  # V_R_B @ [0,0,gamma]
    # W_R_V = quat2rot([c,0,0,s]) (math.py:11-19): rotation by 2*theta about z
    r11, r12, r33 = c * c - s * s, -2 * c * s, c * c + s * s
    W_a = torch.stack([r11 * b[0] + r12 * b[1], -r12 * b[0] + r11 * b[1], r33 * b[2] - G])
    z = torch.zeros((), dtype=x.dtype)
    dq = _t_hprod(q, torch.stack([z, z, z, wz])) / 2
    return torch.cat([x[7:10], dq, W_a]), W_a


def rk4_t(xu, dt):
    x, u = xu[:10], xu[10:]
    f = lambda z: f_t(z, u)[0]
    k1 = f(x); k2 = f(x + dt / 2 * k1); k3 = f(x + dt / 2 * k2); k4 = f(x + dt * k3)
    return x + dt / 6 * (k1 + 2 * k2 + 2 * k3 + k4)


def y_t(xu, qd):
    x, u = xu[:10], xu[10:]
    q = x[3:7] / torch.linalg.norm(x[3:7])
    qi = torch.stack([q[0], -q[1], -q[2], -q[3]]) / torch.linalg.norm(q)
    q_e = _t_hprod(qd, qi)
    _, W_a = f_t(x, u)
    return torch.cat([x[:3], q_e[3:4], x[7:10], (u[1:4] * torch.tensor([LIM.roll, LIM.pitch, LIM.wz], dtype=x.dtype)), W_a[2:3]])


def hfov_t(x, p):
    W_R_Co = p[4:13].reshape(3, 3)
    C = W_R_Co.T @ (x[:3] - p[1:4]) + torch.tensor(CFG.sensor.B_R_C.T @ np.array(CFG.sensor.B_p_C)) \
        + torch.tensor([CFG.mpc.fov_const_offset, 0, 0], dtype=torch.float64)
    return p[0] * torch.stack([torch.atan2(C[1], C[0]), torch.atan2(C[2], torch.linalg.norm(C[:2]))])


def random_state(rng):
    p0 = rng.uniform([-2, -2, 0.5], [2, 2, 3])
    eul = np.array([rng.uniform(-0.3, 0.3), rng.uniform(-0.3, 0.3), rng.uniform(-np.pi, np.pi)])
    q = rmath.euler2quat(eul) * rng.uniform(0.9, 1.1)  # not unit: exercises the q/|q| in the model
    v = rng.uniform(-3, 3, 3)
    return np.concatenate([p0, q, v])


def lin_golden(n=64):
    rng = np.random.default_rng(4321)
    spec = W.DEFAULT_SPEC
    params = W.siren_weights(spec, seed=0)
    net32 = ref_net(spec, params, torch.float32)
    rec = {k: [] for k in ("x", "u", "p", "dt", "f", "xn", "A", "B", "y", "Jy", "yN", "JyN", "h", "Jh",
                           "df", "gdf")}
    B_p_C = np.array(CFG.sensor.B_p_C)
    for i in range(n):
        x = random_state(rng)
        u = rng.uniform([0, -1, -1, -1], [1, 1, 1, 1])
        cam = random_state(rng)  # camera pose near the body (controller.py:50-54 semantics)
        cam[:3] = x[:3] + rng.uniform(-1.5, 0.5, 3)
        W_R_Bo = rmath.quat2rot(cam[3:7] / np.linalg.norm(cam[3:7]))
        p = np.zeros(145)
        p[0] = 1.0 if i % 8 else 0.0  # flag off for every 8th case (gen_model.py:58-61)
        p[1:4] = W_R_Bo @ B_p_C + cam[:3]
        p[4:13] = (W_R_Bo @ CFG.sensor.B_R_C).reshape(9)
        p[13:17] = rmath.euler2quat(np.array([0, 0, rng.uniform(-np.pi, np.pi)]))
        p[17:] = rng.normal(size=128)
        dt = [0.075, 0.0375, 0.025, 0.01][i % 4]
        f, _ = f_expl_np(x, u)
        y, yN = y_np(x, u, p)
        # the network sees the fp32 cast of Co_p_B (L4CasADi passes float tensors)
        W_R_Co = p[4:13].reshape(3, 3)
        Co_p_B = W_R_Co.T @ (x[:3] - p[1:4])
        xin = torch.from_numpy(np.concatenate([Co_p_B, p[17:]]).astype(np.float32)[None]).requires_grad_(True)
        dfv = net32(xin)
        (g,) = torch.autograd.grad(dfv.sum(), xin)
        df = float(dfv.item())
        gpos = g.numpy()[0, :3].astype(np.float64)
        h, _ = h_np(x, p, df, spec.max_df)
        # Jacobians (torch fp64 autograd) + pins
        xu = torch.from_numpy(np.concatenate([x, u]))
        xn_t = rk4_t(xu, dt)
        AB = torch.autograd.functional.jacobian(lambda z: rk4_t(z, dt), xu).numpy()
        qd = torch.from_numpy(p[13:17])
        y_tv = y_t(xu, qd).detach().numpy()
        Jy = torch.autograd.functional.jacobian(lambda z: y_t(z, qd), xu).numpy()
        pt = torch.from_numpy(p)
        Jfov = torch.autograd.functional.jacobian(lambda z: hfov_t(z, pt), torch.from_numpy(x)).numpy()
        Jh = np.zeros((3, 10))
        Jh[:2] = Jfov
        Jh[2, :3] = p[0] * (gpos @ W_R_Co.T)
        # value pins: torch restatement == reference helpers
        assert np.allclose(xn_t.detach().numpy(), rk4_np(x, u, dt), rtol=0, atol=1e-13)
        assert np.allclose(y_tv, y, rtol=0, atol=1e-13)
        assert np.allclose(hfov_t(torch.from_numpy(x), pt).numpy(), h[:2], rtol=0, atol=1e-13), (i, hfov_t(torch.from_numpy(x), pt).numpy() - h[:2], h)
        # derivative pins: central finite differences of the reference-helper functions
        eps = 1e-6
        for j in range(14):
            d = np.zeros(14); d[j] = eps
            xp, up = (np.concatenate([x, u]) + d)[:10], (np.concatenate([x, u]) + d)[10:]
            xm, um = (np.concatenate([x, u]) - d)[:10], (np.concatenate([x, u]) - d)[10:]
            fd = (rk4_np(xp, up, dt) - rk4_np(xm, um, dt)) / (2 * eps)
            assert np.allclose(fd, AB[:, j], atol=2e-7 * max(1, np.abs(AB).max())), (i, j)
            fdy = (y_np(xp, up, p)[0] - y_np(xm, um, p)[0]) / (2 * eps)
            assert np.allclose(fdy, Jy[:, j], atol=2e-6 * max(1, np.abs(Jy).max())), (i, j)
            if j < 10:
                fdh = (h_np(xp, p, 0.0)[0][:2] - h_np(xm, p, 0.0)[0][:2]) / (2 * eps)
                assert np.allclose(fdh, Jfov[:, j], atol=2e-6 * max(1, np.abs(Jfov).max())), (i, j)
        for k_, v_ in (("x", x), ("u", u), ("p", p), ("dt", dt), ("f", f), ("xn", xn_t.detach().numpy()),
                       ("A", AB[:, :10]), ("B", AB[:, 10:]), ("y", y), ("Jy", Jy), ("yN", yN),
                       ("JyN", Jy[[0, 1, 2, 3], :10]), ("h", h), ("Jh", Jh), ("df", df), ("gdf", gpos)):
            rec[k_].append(v_)
    out = {k: np.array(v) for k, v in rec.items()}
    np.savez_compressed(os.path.join(HERE, "lin_golden.npz"), **out)
    print("lin_golden.npz", {k: v.shape for k, v in out.items()})


def grid_golden():
    """ocp.py:21-27 verbatim semantics (numpy linspace/hstack/diff)."""
    out = {}
    for N in (20, 40, 60):
        T = CFG.mpc.T
        nodes_u = np.linspace(0, T, N + 1)
        n_short = CFG.mpc.nb_short_nodes
        dt_short = CFG.mpc.control_loop_time * 1e-3
        nodes_n = np.hstack([np.linspace(0, dt_short * (n_short - 1), n_short),
                             np.linspace(dt_short * n_short, T, N - n_short + 1)])
        out[f"N{N}/uniform/nodes"] = nodes_u
        out[f"N{N}/uniform/dt"] = np.diff(nodes_u)
        out[f"N{N}/nonuniform/nodes"] = nodes_n
        out[f"N{N}/nonuniform/dt"] = np.diff(nodes_n)
    np.savez_compressed(os.path.join(HERE, "grid_golden.npz"), **out)
    print("grid_golden.npz", len(out))


def params_golden():
    """controller.py:50-54 (set_latent), :133-142 (set_ref), quad_rollpitchyawrate.py:62-65."""
    from sdf_nmpc.controller import Nmpc
    from sdf_nmpc.model.quad_rollpitchyawrate import Quad
    from sdf_nmpc.utils.reference import Ref

    rng = np.random.default_rng(77)
    out = {}
    N = 40
    for case in range(4):
        st = types.SimpleNamespace(cfg=CFG, N=N, p=np.zeros((N + 1, 145)), y=np.zeros((N, 11)),
                                   W=np.zeros((N, 11)), yN=np.zeros(4), WN=np.zeros(4),
                                   model=types.SimpleNamespace(nyN=4, extra_W=np.array([])))
        st.model.formate_ref = types.MethodType(Quad.formate_ref, st.model)
        latent = rng.normal(size=128)
        W_p_Bo = rng.uniform(-3, 3, 3)
        W_R_Bo = rmath.quat2rot(rmath.euler2quat(rng.uniform(-0.5, 0.5, 3) * [1, 1, 6]))
        Nmpc.set_sdf_flag(st, bool(case % 2 == 0))
        Nmpc.set_latent(st, latent, W_p_Bo, W_R_Bo)
        refs = []
        for k in range(N + 1):
            r = Ref(CFG)
            r.p = rng.uniform(-5, 5, 3)
            r.q = rmath.euler2quat(np.array([0, 0, rng.uniform(-np.pi, np.pi)]))
            r.v = rng.uniform(-3, 3, 3)
            r.wz = rng.uniform(-1, 1)
            ws = r.W_on if k % 3 else r.W_off  # note Ref's W_on/W_off swap, reference.py:15-28
            r.Wp, r.Wq, r.Wv, r.Ww, r.Wa = ws.Wp, ws.Wq, ws.Wv, ws.Ww, ws.Wa
            Nmpc.set_ref(st, r, k)
            refs.append(np.concatenate([r.p, r.q, r.v, [r.wz], ws.Wp, ws.Wq, ws.Wv, ws.Ww, [ws.Wa]]))
        out[f"c{case}/latent"] = latent
        out[f"c{case}/W_p_Bo"] = W_p_Bo
        out[f"c{case}/W_R_Bo"] = W_R_Bo
        out[f"c{case}/flag"] = np.array(float(case % 2 == 0))
        out[f"c{case}/refs"] = np.array(refs)  # p3 q4 v3 wz1 Wp3 Wq3 Wv3 Ww3 Wa1 = 24
        for k_ in ("p", "y", "W", "yN", "WN"):
            out[f"c{case}/{k_}"] = getattr(st, k_).copy()
    np.savez_compressed(os.path.join(HERE, "params_golden.npz"), **out)
    print("params_golden.npz", len(out))


def refgen_golden():
    """ref_gen.py:7-130 on random paths.  Each case stores x0, waypoints, the config knobs and the
    returned trajectory as rows [p3 q4 v3 wz1] (N or N+1 rows; NaN-padded to N+1)."""
    import copy as _copy
    from sdf_nmpc.ref_gen import RefGen
    from sdf_nmpc.utils.math import euler2quat

    rng = np.random.default_rng(91)
    out = {}
    N = int(CFG.mpc.N)
    case = 0
    modes = ["align", "ref", "current", "zero", "curent"]
    for mode in modes:
        for st_on in (False, True):
            for rep in range(4):
                cfg = _copy.deepcopy(CFG)
                cfg.ref.yaw_mode = mode
                cfg.ref.stop_and_turn.enable = st_on
                cfg.ref.stop_and_turn.dang_min = float(rng.uniform(0.3, 1.5))
                cfg.ref.align_yaw_offset = float(rng.choice([0.0, 0.2]))
                cfg.ref.vref = float(rng.choice([1.0, 3.0]))
                g = RefGen(cfg)
                x0 = np.zeros(13)
                x0[:3] = rng.uniform(-2, 2, 3)
                x0[3:7] = euler2quat(np.array([0.1, -0.1, rng.uniform(-np.pi, np.pi)]))
                x0[7:10] = rng.normal(0, 1, 3)
                nwp = int(rng.integers(1, 5))
                kind = rep % 4
                wps = []
                for w in range(nwp):
                    wp = types.SimpleNamespace()
                    # kind 2: a short path (total < vref * T: padded tail), kind 3: first waypoint on x0 (align dmin)
                    scale = 0.3 if kind == 2 else 4.0
                    wp.p = x0[:3] + rng.uniform(-scale, scale, 3) * (w + 1)
                    if kind == 3 and w == 0:
                        wp.p = x0[:3] + np.array([0.01, 0.0, 0.5])
                    wp.q = euler2quat(np.array([0.0, 0.0, rng.uniform(-np.pi, np.pi)]))
                    wps.append(wp)
                g.x0 = x0
                traj = g.gen_ref_list_wps(wps)
                rows = np.full((N + 1, 11), np.nan)
                for k, r in enumerate(traj):
                    rows[k] = np.concatenate([np.asarray(r.p, float), np.asarray(r.q, float), np.asarray(r.v, float),
                                              [float(r.wz)]])
                out[f"w{case}/x0"] = x0
                out[f"w{case}/wp_p"] = np.array([w.p for w in wps])
                out[f"w{case}/wp_q"] = np.array([w.q for w in wps])
                out[f"w{case}/knobs"] = np.array([modes.index(mode), float(st_on), cfg.ref.stop_and_turn.dang_min,
                                                  cfg.ref.align_yaw_offset, cfg.ref.vref, cfg.ref.yaw_align_dmin,
                                                  cfg.mpc.T, N])
                out[f"w{case}/traj"] = rows
                out[f"w{case}/len"] = np.array(len(traj))
                case += 1
    out["n_wps_cases"] = np.array(case)
    jc = 0
    for mode in ("align", "ref", "curent"):
        for rep in range(3):
            cfg = _copy.deepcopy(CFG)
            cfg.ref.yaw_mode = mode
            g = RefGen(cfg)
            x0 = np.zeros(10)
            x0[:3] = rng.uniform(-2, 2, 3)
            x0[3:7] = euler2quat(np.array([0.0, 0.0, rng.uniform(-np.pi, np.pi)]))
            vw = rng.uniform(-1, 1, 4) * (0.0 if rep == 2 else 1.0)
            g.x0 = x0
            traj = g.gen_ref_joystick(vw)
            out[f"j{jc}/x0"] = x0
            out[f"j{jc}/vw"] = vw
            out[f"j{jc}/mode"] = np.array(["align", "ref", "curent"].index(mode))
            out[f"j{jc}/traj"] = np.array([np.concatenate([np.asarray(r.p, float), np.asarray(r.q, float),
                                                           np.asarray(r.v, float), [float(r.wz)]]) for r in traj])
            out[f"j{jc}/Wp"] = np.array(traj[0].Wp, float)
            jc += 1
    out["n_joy_cases"] = np.array(jc)
    g = RefGen(CFG)
    g.x0 = np.array([0.5, -1, 2, *euler2quat(np.array([0, 0, 1.2])), 0, 0, 0])
    out["from_x0/x0"] = g.x0
    out["from_x0/traj"] = np.array([np.concatenate([np.asarray(r.p, float), np.asarray(r.q, float),
                                                    np.asarray(r.v, float), [float(r.wz)]]) for r in g.from_x0()])
    np.savez_compressed(os.path.join(HERE, "refgen_golden.npz"), **out)
    print("refgen_golden.npz", len(out))


def ts_golden():
    spec = W.DEFAULT_SPEC
    net = ref_net(spec, W.siren_weights(spec, 0), torch.float32)
    sm = torch.jit.script(net)
    sd = sm.state_dict()
    out = {"keys": np.array(list(sd.keys())), "w0": np.float64(sm.w0), "max_df": np.float64(sm.max_df)}
    for k, v in sd.items():
        out[f"shape/{k}"] = np.array(v.shape, dtype=np.int64)
        if "embed" in k:  # the embedding buffers are data the loader checks
            out[f"buf/{k}"] = v.detach().numpy()
    np.savez_compressed(os.path.join(HERE, "ts_golden.npz"), **out)
    print("ts_golden.npz", len(out))


def wide_golden(n=128):
    """The reference's own NeuralDF at config C5's widths [1024,1024,512,256] (SIREN-init, seed 0)."""
    out = {}
    rng = np.random.default_rng(4321)
    spec = W.WIDE_SPEC
    inp = sample_inputs(rng, n, spec.size_latent)
    params = W.siren_weights(spec, seed=0)
    out["input"] = inp
    out["sha256"] = np.frombuffer(hashlib.sha256(W.pack(spec, params)).digest(), dtype=np.uint8)
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        net = ref_net(spec, params, dt)
        x = torch.from_numpy(inp).to(dt).requires_grad_(True)
        df = net(x)
        (g,) = torch.autograd.grad(df.sum(), x)
        out[f"df_{tag}"] = df.detach().numpy()[:, 0]
        out[f"grad_{tag}"] = g.numpy()[:, :3]
    np.savez_compressed(os.path.join(HERE, "wide_golden.npz"), **out)
    print("wide_golden.npz", {k: v.shape for k, v in out.items()})


from variant_specs import BIAS_GAIN, NET_VARIANTS, SEED  # noqa: E402


def variants_golden(n=32):
    """The reference's own NeuralDF for each NET_VARIANTS spec (variant_specs.py; SIREN-init weights from
    our PRNG, biases drawn so the bias path is live): df and d df / d pos in fp32 and fp64, plus the embedding
    directions the reference builds (pins weights.embedding_dirs for every projection)."""
    out = {}
    rng = np.random.default_rng(777)
    inp = sample_inputs(rng, n, 128)
    out["input"] = inp
    for name, spec in NET_VARIANTS.items():
        params = W.siren_weights(spec, seed=SEED, bias_gain=BIAS_GAIN)
        out[f"{name}/sha256"] = np.frombuffer(hashlib.sha256(W.pack(spec, params)).digest(), dtype=np.uint8)
        vin = inp
        if spec.size_latent != 128:  # its own inputs (3 + size_latent columns), the shared positions
            vin = np.concatenate([inp[:, :3], np.random.default_rng(778 + spec.size_latent).normal(
                size=(n, spec.size_latent)).astype(np.float32)], 1)
            out[f"{name}/input"] = vin
        for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
            net = ref_net(spec, params, dt)
            x = torch.from_numpy(vin).to(dt).requires_grad_(True)
            df = net(x)
            (g,) = torch.autograd.grad(df.sum(), x)
            out[f"{name}/df_{tag}"] = df.detach().numpy()[:, 0]
            out[f"{name}/grad_{tag}"] = g.numpy()  # the full 1 x 131 Jacobian (jac_sdf_l4c)
        if spec.embed != "none":
            out[f"{name}/dirs"] = ref_net(spec, params, torch.float32).embed.dirs.numpy()
    np.savez_compressed(os.path.join(HERE, "variants_golden.npz"), **out)
    print("variants_golden.npz", len(out))


def sdfc3_golden(stride=32):
    """The reference's own NeuralDF (SIREN-init, seed 0) in fp32 and fp64 on every `stride`-th SDF row of
    the bench workload C3 (1024 instances x 41 nodes, synthetic seed 1000): body positions in the
    camera-origin frame (gen_model.py:50, as h_np) from the synthetic iterate and camera poses, and each
    instance's latent -- the rows sdf_mlp sees in bench.py."""
    from sdf_nmpc_amd import synth, _lib
    from sdf_nmpc_amd.config import Config as AmdConfig
    cfg = AmdConfig()
    B, N = 1024, 40
    _, dt = _lib.shooting_grid(N, cfg.mpc.T)  # as bench.py
    prob = synth.make_problem(cfg, B, N, seed=1000, dt=dt)
    x, pp = prob["x"].reshape(-1, 10), prob["p"].reshape(B * (N + 1), -1)
    rows = np.arange(0, B * (N + 1), stride)
    W_R_Co = pp[rows][:, P_IDX.W_R_Co].reshape(-1, 3, 3)
    W_p_Co = pp[rows][:, P_IDX.W_p_Co]
    pos = np.einsum("nji,nj->ni", W_R_Co, x[rows, :3] - W_p_Co)
    lat = pp[rows][:, P_IDX.latent:P_IDX.latent + W.DEFAULT_SPEC.size_latent]
    inp = np.concatenate([pos, lat], 1).astype(np.float32)
    params = W.siren_weights(W.DEFAULT_SPEC, seed=0)
    out = {"input": inp, "rows": rows, "sha256": np.frombuffer(hashlib.sha256(W.pack(W.DEFAULT_SPEC, params)).digest(),
                                                                  dtype=np.uint8)}
    for dtp, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        net = ref_net(W.DEFAULT_SPEC, params, dtp)
        xx = torch.from_numpy(inp).to(dtp).requires_grad_(True)
        df = net(xx)
        (g,) = torch.autograd.grad(df.sum(), xx)
        out[f"df_{tag}"] = df.detach().numpy()[:, 0]
        out[f"grad_{tag}"] = g.numpy()[:, :3]
    np.savez_compressed(os.path.join(HERE, "sdfc3_golden.npz"), **out)
    print("sdfc3_golden.npz", {k: v.shape for k, v in out.items()})


def vae_golden():
    import copy as _copy
    from sdf_nmpc.network.vae import Encoder
    from sdf_nmpc.utils import preprocessing as P
    from sdf_nmpc_amd import synth
    from sdf_nmpc_amd import vae as V

    spec = V.DEFAULT_ENCODER
    enc = Encoder(spec.nb_chan, spec.size_latent, dropout_rate=0.1, batchnorm=spec.batchnorm).eval()
    sd = enc.state_dict()
    names = [k for k in sd.keys() if not k.endswith("num_batches_tracked")]
    assert names == [n for n, _ in spec.param_shapes()], "param order"
    params = V.synthetic_encoder(spec, 0)
    for k, shape in spec.param_shapes():
        assert tuple(sd[k].shape) == shape, k
        sd[k] = torch.from_numpy(params[k].copy())
    enc.load_state_dict(sd)
    enc64 = _copy.deepcopy(enc).double()
    shape = list(CFG.sensor.shape_imgs)
    d2r = P.Depth2Range(shape, CFG.sensor.hfov, CFG.sensor.vfov)
    cases = [  # (image, mm_resolution)
        (synth.depth_images(1, 270, 480, seed=0)[0], 1000),
        (synth.depth_images(1, 270, 480, seed=1)[0], 1000),
        (synth.depth_images(1, 270, 480, seed=2, kind="mm")[0], 1),
        (synth.depth_images(1, 240, 424, seed=3)[0], 1000),  # Reshape's bilinear resize path
    ]
    rng = np.random.default_rng(5)
    out = {"names": np.array(names), "n_cases": np.array(len(cases)),
           "yz_sqrt_sample": d2r.yz_sqrt.numpy()[::7, ::11].copy(), "flops": np.int64(spec.n_flops())}
    for c, (img, mmr) in enumerate(cases):
        pre = torch.nn.Sequential(P.ToDevice("cpu"), torch.jit.script(P.Reshape(shape)),
                                  torch.jit.script(P.ClipDistance(CFG.sensor.dmax, mmr)),
                                  torch.jit.script(P.Depth2Range(shape, CFG.sensor.hfov, CFG.sensor.vfov, "cpu")))
        x = pre(img)
        with torch.no_grad():
            lat = enc(x).numpy()[0]
            lat64 = enc64(x.double()).numpy()[0]
        iy = rng.integers(0, shape[1], 4096)
        ix = rng.integers(0, shape[2], 4096)
        out[f"c{c}/seed"] = np.array([c, 2 if mmr == 1 else 0])
        out[f"c{c}/in_shape"] = np.array(img.shape)
        out[f"c{c}/mm_resolution"] = np.float64(mmr)
        out[f"c{c}/pre_idx"] = np.stack([iy, ix])
        out[f"c{c}/pre_val"] = x.numpy()[0, 0, iy, ix]
        out[f"c{c}/latent"] = lat
        out[f"c{c}/latent64"] = lat64
        if c == 0:  # per-stage channel sums of the fp64 run (debugging aid for the oracle / kernels)
            h = x.double()
            with torch.no_grad():
                for i, m in enumerate(enc64.layers["resnet"]):
                    h = m(h)
                    if i in (2, 3, 4, 5, 6):
                        out[f"c0/stage{i}"] = h.sum(dim=(0, 2, 3)).numpy()
    np.savez_compressed(os.path.join(HERE, "vae_golden.npz"), **out)
    print("vae_golden.npz", len(out))


def scene_golden(n=256):
    """The reference's own NeuralDF on the scene-fitted weights (tests/golden/scene.sdfw, written by
    tools/fit_scene_sdf.py) and the scene latent, in fp32 and fp64: df and the full 1 x 131 Jacobian on
    points along the corridor the closed-loop test flies (camera-origin frame), plus the analytic scene
    distance the weights were fitted to (what the fit is, not a parity bar)."""
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import fit_scene_sdf as FS
    with open(os.path.join(HERE, "scene.sdfw"), "rb") as f:
        blob = f.read()
    spec, params = W.unpack(blob)
    rng = np.random.default_rng(4242)
    pos = np.stack([rng.uniform(-0.5, 7.0, n), rng.uniform(-2.5, 2.5, n), rng.uniform(-1.0, 1.0, n)], 1)
    z = FS.scene_latent()
    inp = np.concatenate([pos.astype(np.float32), np.broadcast_to(z, (n, len(z)))], 1).astype(np.float32)
    out = {"input": inp, "latent": z, "sha256": np.frombuffer(hashlib.sha256(blob).digest(), dtype=np.uint8),
           "scene_df": FS.scene_sdf(pos)[0]}
    for dt, tag in ((torch.float32, "f32"), (torch.float64, "f64")):
        net = ref_net(spec, params, dt)
        x = torch.from_numpy(inp).to(dt).requires_grad_(True)
        df = net(x)
        (g,) = torch.autograd.grad(df.sum(), x)
        out[f"df_{tag}"] = df.detach().numpy()[:, 0]
        out[f"grad_{tag}"] = g.numpy()
    np.savez_compressed(os.path.join(HERE, "scene_golden.npz"), **out)
    print("scene_golden.npz", {k: v.shape for k, v in out.items()})


def flags_golden():
    """The flag space of default.yaml:16-23 (gen_model.py:26-149):
      * poly/*      -- polynomial_3variate (utils/math.py:294-321) run from the reference with casadi replaced
                       by a numeric stand-in: SX.sym('x') is a fixed numeric point, vertcat concatenates,
                       sum1 sums (and records its argument, the term vector), Function is inert.  At the
                       point (2, 3, 5) the terms 2^a 3^b 5^c give the exponents of every term in the
                       reference's order; with given coefficients, the polynomial's values at sample v.
      * rtilde/*    -- stability.get_r_tilde_max (utils/stability.py:44-75: sympy solve + scipy SLSQP) itself,
                       np.random seeded before each call (its start point is np.random.uniform), on the
                       reference Config with the weights it reads (mpc.weights.{acc, att}) set to set_const_on's.
      * setref5/*   -- Nmpc.set_ref at the terminal node with nyN = 5 (flags.stability adds a terminal cost
                       row, gen_model.py:149): WN = W[:5], yN = y[:5] (controller.py:141-142).
    """
    from sdf_nmpc.controller import Nmpc
    from sdf_nmpc.model.quad_rollpitchyawrate import Quad as RQuad
    from sdf_nmpc.utils import stability as rstab
    from sdf_nmpc.utils.reference import Ref
    out = {}
    cs = rmath.cs
    state = {"point": None, "terms": None}

    class _SX:
        @staticmethod
        def sym(name, n, m=1):
            return np.array(state["point"], float) if name == "x" else np.ones(n)

    def _sum1(v):
        state["terms"] = np.asarray(v, float).copy()
        return float(np.sum(v))

    saved = {k: getattr(cs, k, None) for k in ("SX", "vertcat", "sum1", "Function")}
    cs.SX = _SX
    cs.vertcat = lambda *a: np.concatenate([np.atleast_1d(np.asarray(v, float)) for v in a])
    cs.sum1 = _sum1
    cs.Function = lambda *a, **k: None
    try:
        rng = np.random.default_rng(5)
        for deg in (0, 1, 2, 3, 4, 5, 6):
            state["point"] = [2.0, 3.0, 5.0]
            rmath.polynomial_3variate(deg, np.ones((deg + 1) * (deg + 2) * (deg + 3) // 6))
            t = state["terms"]
            exps = []
            for v in t:
                e = []
                for pr in (2, 3, 5):
                    c = 0
                    while round(v) % pr == 0:
                        v /= pr
                        c += 1
                    e.append(c)
                exps.append(e)
            out[f"poly/deg{deg}/exps"] = np.array(exps, np.int64)
            coeffs = rng.normal(size=len(t))
            vs = rng.uniform(-4, 4, (16, 3))
            vals = []
            for v in vs:
                state["point"] = v
                rmath.polynomial_3variate(deg, coeffs)
                vals.append(float(np.sum(state["terms"])))
            out[f"poly/deg{deg}/coeffs"] = coeffs
            out[f"poly/deg{deg}/v"] = vs
            out[f"poly/deg{deg}/val"] = np.array(vals)
    finally:
        for k, v in saved.items():
            if v is None:
                delattr(cs, k)
            else:
                setattr(cs, k, v)
    cfg = Config(os.path.join(REF, "sdf_nmpc/config/default.yaml"))
    on = cfg.mpc.weights.set_const_on
    cfg.mpc.weights.acc, cfg.mpc.weights.att = on.acc, list(on.att)
    for i, (N, T) in enumerate(((20, 1.5), (40, 1.5), (30, 2.0))):
        cfg.mpc.N, cfg.mpc.T = N, T
        for seed in (0, 1, 2):
            np.random.seed(seed)
            out[f"rtilde/N{N}_T{T}/seed{seed}"] = np.array(float(rstab.get_r_tilde_max(cfg)))
    # set_ref with nyN = 5
    N = 20
    st = types.SimpleNamespace(cfg=CFG, N=N, p=np.zeros((N + 1, 145)), y=np.zeros((N, 11)), W=np.zeros((N, 11)),
                               yN=np.zeros(5), WN=np.zeros(5), model=types.SimpleNamespace(nyN=5, extra_W=np.array([])))
    st.model.formate_ref = types.MethodType(RQuad.formate_ref, st.model)
    r = Ref(CFG)
    r.p, r.q, r.v, r.wz = np.array([1.0, -2.0, 3.0]), rmath.euler2quat(np.array([0, 0, 0.7])), np.array([0.5, -1.0, 2.0]), 0.3
    ws = r.W_on
    r.Wp, r.Wq, r.Wv, r.Ww, r.Wa = ws.Wp, ws.Wq, ws.Wv, ws.Ww, ws.Wa
    Nmpc.set_ref(st, r, N)
    out["setref5/yN"], out["setref5/WN"] = st.yN.copy(), st.WN.copy()
    out["setref5/ref"] = np.concatenate([r.p, r.q, r.v, [r.wz], ws.Wp, ws.Wq, ws.Wv, ws.Ww, [ws.Wa]])
    np.savez_compressed(os.path.join(HERE, "flags_golden.npz"), **out)
    print("flags_golden.npz", len(out))


if __name__ == "__main__":
    only = sys.argv[1:]
    for name, fn in (("sdf", sdf_golden), ("lin", lin_golden), ("grid", grid_golden), ("params", params_golden),
                     ("ts", ts_golden), ("refgen", refgen_golden), ("vae", vae_golden), ("wide", wide_golden), ("sdfc3", sdfc3_golden),
                     ("variants", variants_golden), ("scene", scene_golden), ("flags", flags_golden)):
        if not only or name in only:
            fn()
