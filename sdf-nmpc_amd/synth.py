"""Seeded synthetic NMPC problems (BASELINE.json configs; SURVEY.md §8(d) "Synthetic inputs").

Host-side numpy only (input generation for tests and the benchmark, not a compute path).
Per instance: x0 with p0 ~ U([-2,2]^2 x [0.5,3]) m, roll/pitch ~ U(+-0.3), yaw ~ U(-pi, pi) (euler2quat,
reference utils/math.py:110-139), v0 ~ U(+-3)^3 m/s; latent z ~ N(0,1)^128 (the VAE prior); flag = 1;
camera pose from x0 with the sensor extrinsics (Nmpc.set_latent, controller.py:50-54); q_d = yaw
aligned toward a waypoint p0 + U(ball 5 m) (ref yaw_mode 'align'); y/W in formate_ref layout
(quad_rollpitchyawrate.py:62-65) with the set_const_on weights.  The current iterate (x, u) is a
hover-ish input sequence rolled out with the same RK4 the OCP uses.
"""
from __future__ import annotations

import numpy as np

G = 9.81


def euler2quat(e):
    """[roll, pitch, yaw] (..., 3) -> [qw, qx, qy, qz] (reference utils/math.py:110-139, numpy)."""
    cr, sr = np.cos(e[..., 0] * 0.5), np.sin(e[..., 0] * 0.5)
    cp, sp = np.cos(e[..., 1] * 0.5), np.sin(e[..., 1] * 0.5)
    cy, sy = np.cos(e[..., 2] * 0.5), np.sin(e[..., 2] * 0.5)
    return np.stack([cr * cp * cy + sr * sp * sy, sr * cp * cy - cr * sp * sy,
                     cr * sp * cy + sr * cp * sy, cr * cp * sy - sr * sp * cy], -1)


def quat2rot(q):
    """(..., 4) -> (..., 3, 3) (reference utils/math.py:7-23)."""
    w, x, y, z = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    return np.stack([
        np.stack([w * w + x * x - y * y - z * z, 2 * (x * y - w * z), 2 * (x * z + w * y)], -1),
        np.stack([2 * (x * y + w * z), w * w - x * x + y * y - z * z, 2 * (y * z - w * x)], -1),
        np.stack([2 * (x * z - w * y), 2 * (y * z + w * x), w * w - x * x - y * y + z * z], -1)], -2)


def f_expl(x, u, lim):
    """Vectorised 'att' dynamics (quad_rollpitchyawrate.py:19-42), (..., 10), (..., 4) -> (..., 10)."""
    q = x[..., 3:7] / np.linalg.norm(x[..., 3:7], axis=-1, keepdims=True)
    th = np.arctan2(q[..., 3], q[..., 0])
    c, s = np.cos(th), np.sin(th)
    gam, roll, pitch, wz = u[..., 0] * lim.gamma, u[..., 1] * lim.roll, u[..., 2] * lim.pitch, u[..., 3] * lim.wz
    b0, b1, b2 = np.cos(roll) * np.sin(pitch) * gam, -np.sin(roll) * gam, np.cos(roll) * np.cos(pitch) * gam
    r11, r21, r33 = c * c - s * s, 2 * c * s, c * c + s * s
    return np.concatenate([x[..., 7:10], np.stack([-q[..., 3] * wz, q[..., 2] * wz, -q[..., 1] * wz, q[..., 0] * wz], -1) / 2,
                           np.stack([r11 * b0 - r21 * b1, r21 * b0 + r11 * b1, r33 * b2 - G], -1)], -1)


def rk4(x, u, dt, lim):
    k1 = f_expl(x, u, lim)
    k2 = f_expl(x + dt / 2 * k1, u, lim)
    k3 = f_expl(x + dt / 2 * k2, u, lim)
    k4 = f_expl(x + dt * k3, u, lim)
    return x + dt / 6 * (k1 + 2 * k2 + 2 * k3 + k4)


def make_problem(cfg, B: int, N: int, seed: int = 0, np_: int = 145, dt=None, sdf_cost: bool = False, nyN: int = 4,
                 v_forward: bool = False):
    """v_forward: v0 along the camera's view (the body yaw) instead of U(+-3)^3, so the braking point of
    flags.recursive_feasibility (gen_model.py:106-112) lies in the field of view, as in flight."""
    rng = np.random.default_rng(seed)
    lim = cfg.robot.limits
    L = int(cfg.nn.size_latent)
    if dt is None:
        dt = np.full(N, cfg.mpc.T / N)
    p0 = rng.uniform([-2, -2, 0.5], [2, 2, 3], (B, 3))
    eul = np.stack([rng.uniform(-0.3, 0.3, B), rng.uniform(-0.3, 0.3, B), rng.uniform(-np.pi, np.pi, B)], -1)
    q0 = euler2quat(eul)
    v0 = rng.uniform(-3, 3, (B, 3))
    if v_forward:
        vb = np.stack([rng.uniform(0.5, 2.5, B), rng.uniform(-0.4, 0.4, B), rng.uniform(-0.3, 0.3, B)], -1)
        cy, sy = np.cos(eul[:, 2]), np.sin(eul[:, 2])
        v0 = np.stack([cy * vb[:, 0] - sy * vb[:, 1], sy * vb[:, 0] + cy * vb[:, 1], vb[:, 2]], -1)
    x0 = np.concatenate([p0, q0, v0], -1)
    latent = rng.normal(size=(B, L))
    # current iterate: hover thrust + small perturbations, rolled out
    u = np.empty((B, N, 4))
    u[..., 0] = np.clip(G / lim.gamma + rng.normal(0, 0.05, (B, N)), 0, 1)
    u[..., 1:] = np.clip(rng.normal(0, 0.15, (B, N, 3)), -1, 1)
    x = np.empty((B, N + 1, 10))
    x[:, 0] = x0
    for k in range(N):
        x[:, k + 1] = rk4(x[:, k], u[:, k], dt[k], lim)
    # parameters (Nmpc.set_sdf_flag / set_latent / set_ref)
    p = np.zeros((B, N + 1, np_))
    p[..., 0] = 1.0
    W_R_Bo = quat2rot(q0)
    p[..., 1:4] = (np.einsum("bij,j->bi", W_R_Bo, np.asarray(cfg.sensor.B_p_C, float)) + p0)[:, None, :]
    p[..., 4:13] = (W_R_Bo @ np.asarray(cfg.sensor.B_R_C))[:, None, :, :].reshape(B, 1, 9)
    v = rng.normal(size=(B, 3))
    wp = p0 + v / np.linalg.norm(v, axis=1, keepdims=True) * 5.0 * rng.uniform(0, 1, (B, 1)) ** (1 / 3)
    yaw = np.arctan2(wp[:, 1] - p0[:, 1], wp[:, 0] - p0[:, 0])
    qd = euler2quat(np.stack([np.zeros(B), np.zeros(B), yaw], -1))
    p[..., 13:17] = qd[:, None, :]
    p[..., 17:17 + L] = latent[:, None, :]
    # references (formate_ref layout) with set_const_on weights
    w = cfg.mpc.weights.set_const_on
    vref = (wp - p0) / np.maximum(np.linalg.norm(wp - p0, axis=1, keepdims=True), 1e-9) * float(cfg.get("ref", {}).get("vref", 3) if hasattr(cfg, "get") else 3)
    yref = np.zeros((B, N, 11))
    yref[..., 0:3] = wp[:, None, :]
    yref[..., 4:7] = vref[:, None, :]
    Wrow = np.concatenate([w.pos, [w.att[2]], w.vel, w.att[:2], w.rates[2:], [w.acc]]).astype(float)
    W = np.broadcast_to(Wrow, (B, N, 11)).copy()
    yN = yref[:, -1, :nyN].copy()  # Nmpc.set_ref at the last node: y[:nyN], W[:nyN] (controller.py:141-142)
    WN = W[:, -1, :nyN].copy()
    if sdf_cost:  # flags.sdf_cost: 12th residual (1 - s/2)^4 with reference 0 and weight 20 (model.Quad.extra_W)
        yref = np.concatenate([yref, np.zeros((B, N, 1))], axis=-1)
        W = np.concatenate([W, np.full((B, N, 1), 20.0)], axis=-1)
    return dict(x=x, u=u, p=p, dt=np.asarray(dt, float), yref=yref, W=W, yN=yN, WN=WN, x0=x0, latent=latent)


def depth_images(B: int, H: int = 270, W: int = 480, seed: int = 0, kind: str = "m") -> np.ndarray:
    """Seeded synthetic depth images [B, H, W] for the VAE path (1x270x480 ~ U(0, 5 m)).

    A smooth scene (two walls + a box) plus uniform noise, with ~5 % invalid (zero) pixels and ~5 %
    beyond dmax.  kind 'm': float32 metres; 'mm': uint16 millimetres (mm_resolution = 1 sensors).
    """
    from .weights import prng_uniform

    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    out = np.empty((B, H, W), np.float64)
    for b in range(B):
        u = prng_uniform(seed * 7919 + b, 40, 3 * H * W).reshape(3, H, W)
        ph = prng_uniform(seed * 7919 + b, 41, 6)
        wall = 1.0 + 3.0 * (0.5 + 0.5 * np.sin(xx / (20 + 40 * ph[0]) + 6.3 * ph[1])) * (0.6 + 0.4 * np.cos(yy / (15 + 30 * ph[2])))
        box = (np.abs(xx - W * ph[3]) < W * 0.15) & (np.abs(yy - H * ph[4]) < H * 0.2)
        d = np.where(box, 0.6 + 0.8 * ph[5], wall) + 0.3 * u[0]
        d = np.where(u[1] < 0.05, 0.0, d)
        d = np.where(u[2] < 0.05, 6.0 + 2.0 * u[0], d)
        out[b] = d
    if kind == "mm":
        return np.round(out * 1000.0).astype(np.uint16)
    return out.astype(np.float32)


def braking_coeffs(deg: int = 4, seed: int = 0, a_brake: float = 6.32, d0: float = 0.05, noise: float = 2e-3):
    """Synthetic braking-distance polynomial in polynomial_3variate's term order (utils/math.py:307-314):
    d(v) = d0 + |v|^2 / (2 a_brake) plus seeded small terms on every monomial, so every coefficient is
    exercised (the reference loads a fitted file, default.yaml:70-72, which is absent here)."""
    from .model import poly_terms
    rng = np.random.default_rng(seed)
    t = poly_terms(deg)
    c = rng.normal(0, noise, len(t))
    for i, (a, b, e) in enumerate(t):
        if (a, b, e) == (0, 0, 0):
            c[i] += d0
        if sorted((a, b, e)) == [0, 0, 2]:
            c[i] += 0.5 / a_brake
    return c
