"""The default 'att' (roll/pitch/yaw-rate) quadrotor OCP: dimensions, bounds, reference layout.

Host-side description only -- the arithmetic (dynamics, residuals, constraints and their Jacobians)
runs in csrc/linearize.hip and csrc/sdf_mlp.hip.  Mirrors (paths relative to the reference checkout):
  * dimensions / bounds / hover input ... sdf_nmpc/model/quad_rollpitchyawrate.py:12-17, 366, 380-381
  * formate_ref ........................ sdf_nmpc/model/quad_rollpitchyawrate.py:62-65
  * constraint set (every flag) ........ sdf_nmpc/gen_model.py:26-149, model/cost_const_helpers.py:48-102
  * braking polynomial / stability ..... utils/math.py:294-321, utils/stability.py:6-75
  * slack weights ...................... model/base_model.py:63-71,142-168, ocp.py:85-92
"""
from __future__ import annotations

import numpy as np

G = 9.81  # model/base_model.py:10


class UnsupportedConfig(ValueError):
    pass


def quat2rot(q):
    """[qw qx qy qz] -> rotation matrix, batched over leading dims (reference utils/math.py:7-23)."""
    q = np.asarray(q, dtype=float)
    w, x, y, z = q[..., 0], q[..., 1], q[..., 2], q[..., 3]
    R = np.stack([w * w + x * x - y * y - z * z, 2 * (x * y - w * z), 2 * (x * z + w * y),
                  2 * (x * y + w * z), w * w - x * x + y * y - z * z, 2 * (y * z - w * x),
                  2 * (x * z - w * y), 2 * (y * z + w * x), w * w - x * x - y * y + z * z], axis=-1)
    return R.reshape(q.shape[:-1] + (3, 3))


def euler2rot_b(roll, pitch, yaw):
    """Z1Y2X3 euler angles -> rotation matrix, batched (reference utils/math.py:26-54)."""
    sr, cr, sp, cp, sy, cy = np.sin(roll), np.cos(roll), np.sin(pitch), np.cos(pitch), np.sin(yaw), np.cos(yaw)
    R = np.stack([cp * cy, sr * sp * cy - cr * sy, cr * sp * cy + sr * sy,
                  cp * sy, sr * sp * sy + cr * cy, cr * sp * sy - sr * cy,
                  -sp, sr * cp, cr * cp], axis=-1)
    return R.reshape(np.shape(roll) + (3, 3))


def poly_terms(deg: int):
    """Monomial exponents (a, b, c) of polynomial_3variate in its term order (utils/math.py:307-314):
    total degree 0..deg, then the x exponent a, then the y exponent b (c = the rest)."""
    return [(a, b, d - a - b) for d in range(deg + 1) for a in range(d + 1) for b in range(d + 1 - a)]


def poly_eval(coeffs, deg: int, v):
    """poly_c(v) and its gradient for v [..., 3] (the braking distance of gen_model.py:76-78)."""
    v = np.asarray(v, dtype=float)
    val = np.zeros(v.shape[:-1])
    grad = np.zeros(v.shape)
    for c, (a, b, e) in zip(np.asarray(coeffs, float), poly_terms(deg)):
        px, py, pz = v[..., 0] ** a, v[..., 1] ** b, v[..., 2] ** e
        val = val + c * px * py * pz
        if a: grad[..., 0] += c * a * v[..., 0] ** (a - 1) * py * pz
        if b: grad[..., 1] += c * b * px * v[..., 1] ** (b - 1) * pz
        if e: grad[..., 2] += c * e * px * py * v[..., 2] ** (e - 1)
    return val, grad


def r_tilde_max(cfg, weights=None):
    """get_r_tilde_max (utils/stability.py:44-75): the largest r~ over thrust / roll / pitch in their limits
    such that the bounded input cost dominates the stage input cost.  The symbolic solve of
    stability.py:6-41 is linear in r~ and has the closed form r~ = (r1 (T - g)^2 + r2 phi^2 + r3 theta^2) /
    (dt^2 |T R e3 - g e3|^2) with psi = 0; the maximisation is the reference's: SLSQP from a start drawn
    with numpy's global generator (np.random.uniform, stability.py:72), so a seeded np.random reproduces
    the reference's start."""
    from scipy.optimize import minimize
    w = weights or _stab_weights(cfg)
    g = 9.81
    dt = cfg.mpc.T / cfg.mpc.N
    r1, r2, r3 = w["acc"], w["att"][0], w["att"][1]
    lim = cfg.robot.limits
    T_range, phi_range, th_range = [0, lim.gamma], [-lim.roll, lim.roll], [-lim.pitch, lim.pitch]

    def objective(z):
        T, phi, th = z
        den = dt * dt * (T * T - 2.0 * g * T * np.cos(th) * np.cos(phi) + g * g)
        return -(r1 * (T - g) ** 2 + r2 * phi ** 2 + r3 * th ** 2) / den

    cons = [{"type": "ineq", "fun": lambda z: z[0] - T_range[0]}, {"type": "ineq", "fun": lambda z: T_range[1] - z[0]},
            {"type": "ineq", "fun": lambda z: z[1] - phi_range[0]}, {"type": "ineq", "fun": lambda z: phi_range[1] - z[1]},
            {"type": "ineq", "fun": lambda z: z[2] - th_range[0]}, {"type": "ineq", "fun": lambda z: th_range[1] - z[2]}]
    z0 = [np.random.uniform(*T_range), np.random.uniform(*phi_range), np.random.uniform(*th_range)]
    return float(-minimize(objective, z0, constraints=cons, method="SLSQP").fun)


def _stab_weights(cfg):
    """The cost weights gen_model.py:129-133 / stability.py:52 read as cfg.mpc.weights.{vel, att, rates,
    acc}.  The reference's default.yaml keeps its weights under set_const_off / set_const_on only, so there
    those reads raise AttributeError; a config that defines them is used as is, otherwise set_const_on
    (the set the controller applies with constraints on)."""
    w = cfg.mpc.weights
    src = w if all(k in w for k in ("vel", "att", "rates", "acc")) else w.set_const_on
    return {k: (np.asarray(src[k], float) if k != "acc" else float(src[k])) for k in ("vel", "att", "rates", "acc")}


def _slack(v):
    """A slack-weight entry of the config: [L1, L2], or None / the YAML string 'None' for a hard row
    (default.yaml:51 writes `slack_brake: None`, which YAML reads as the string 'None' -- truthy, so the
    reference would index its characters as weights; the evident intent, a hard row, is taken)."""
    if v is None or (isinstance(v, str) and v.strip().lower() in ("none", "null", "")):
        return None
    return [float(v[0]), float(v[1])]


class Quad:
    """'att' model + the constraint set gen_model.get_model_from_cfg builds from the flags
    (gen_model.py:26-149, cost_const_helpers.py:48-102, quad_rollpitchyawrate.py:48-55).

    Node functions (fixed columns of the preparation phase's h / J_h): 0 hfov, 1 vfov, 2 sdf.
    Stage rows (in the order the reference adds them): hfov if sensor.hfov < 3.14, vfov if
    flags.vfov_constraint, sdf if flags.sdf_constraint -- all only with flags.enable_sdf; soft with the
    slack weights mpc.weights.slack_fov / slack_df, hard where that weight is None (base_model.py:142-155),
    and then ordered soft first (h_cols; nhs = the hard ones at the end).
    Terminal rows: the same fov rows, the sdf row unless recursive_feasibility; with
    recursive_feasibility the braking row sdf - flag poly(v) in [size.xy, max_df] (soft with
    slack_brake, else hard) and the hard fov rows at Co_p_E; with stability the hard terminal velocity
    bounds (add_vel_const, kept as unit rows on v_N) and the terminal cost row flag |v|^2."""

    nx, nu = 10, 4

    def __init__(self, cfg, max_df: float = 1.0, braking_coeffs=None):
        self.cfg = cfg
        self.name = "quad_rollpitchyawrate"
        fl = cfg.flags
        if cfg.mpc.model != "att":
            # gen_model.py:74 asserts on cfg.control_mode (undefined in Config); this build
            # is the 'att' model only (default model)
            raise UnsupportedConfig(f"mpc.model '{cfg.mpc.model}': only 'att' is built (SURVEY.md §8: default model)")
        E = bool(fl.get("enable_sdf"))
        H = E and cfg.sensor.hfov < 3.14
        V = E and bool(fl.get("vfov_constraint"))
        S = E and bool(fl.get("sdf_constraint"))
        RF = E and bool(fl.get("recursive_feasibility"))
        ST = RF and bool(fl.get("stability"))  # gen_model.py:124: inside the rec_feas block
        self.enable_sdf, self.rec_feas, self.stability = E, RF, ST
        if E:
            self.name += "_sdf"  # gen_model.py:29
        self.max_df = float(max_df)
        self.p_idx = cfg.mpc.p_idx
        self.np = int(cfg.mpc.p_idx.latent) + int(cfg.nn.size_latent)
        lim = cfg.robot.limits
        self.g = G
        self.lbu = np.array([0.0, -1.0, -1.0, -1.0])
        self.ubu = np.array([1.0, 1.0, 1.0, 1.0])
        self.u_hover = np.array([G / lim.gamma, 0.0, 0.0, 0.0])
        # the three node functions: bounds and slack weights (cost_const_helpers.py:67-75, gen_model.py:35,68)
        hfov_lim = cfg.sensor.hfov * cfg.mpc.fov_ratio
        vfov_lim = cfg.sensor.vfov * cfg.mpc.fov_ratio
        sf, sd = _slack(cfg.mpc.weights.slack_fov), _slack(cfg.mpc.weights.slack_df)
        fun_l = [-hfov_lim, -vfov_lim, cfg.robot.size.xy + cfg.mpc.bound_margin]
        fun_u = [hfov_lim, vfov_lim, self.max_df + 0.2]
        fun_w = [sf, sf, sd]  # None: a hard row (add_const_stage / add_const_term soften only `if slack_weights`)
        # stage rows: the soft ones first, then the hard ones (slack weight None), each kind in the reference's
        # order -- the QP's row order does not change its solution, and the kernels fold the hard rows like
        # box rows after the soft groups (rti_qp.hip)
        on = [c for c, f in ((0, H), (1, V), (2, S)) if f]
        self.h_cols = [c for c in on if fun_w[c] is not None] + [c for c in on if fun_w[c] is None]
        self.nh = len(self.h_cols)
        self.nhs = sum(1 for c in on if fun_w[c] is None)  # hard stage rows (the last nhs of h_cols)
        self.lh = np.array([fun_l[c] for c in self.h_cols], dtype=float)
        self.uh = np.array([fun_u[c] for c in self.h_cols], dtype=float)
        self.zl = np.array([(fun_w[c] or (0.0, 0.0))[0] for c in self.h_cols], dtype=float)
        self.Zl = np.array([(fun_w[c] or (0.0, 0.0))[1] for c in self.h_cols], dtype=float)
        # terminal rows (hN_col, hE_col, soft, lh, uh, zl, Zl), soft ones first (as the reference adds them)
        rows = [(c, -1, fun_w[c] is not None, fun_l[c], fun_u[c], *(fun_w[c] or (0.0, 0.0)))
                for c in on if not (c == 2 and RF)]
        if RF:
            sb = _slack(cfg.mpc.weights.get("slack_brake"))
            rows.append((2, 0, sb is not None, float(cfg.robot.size.xy), self.max_df, *(sb or (0.0, 0.0))))
            rows.append((-1, 1, False, -hfov_lim, hfov_lim, 0.0, 0.0))
            if V:
                rows.append((-1, 2, False, -vfov_lim, vfov_lim, 0.0, 0.0))
        if ST:  # add_vel_const(stage=False, term=True) (cost_const_helpers.py:79-102): hard bounds on v_N
            vb = [float(lim.vx), float(lim.vy), float(lim.vz)]
            rows += [(-1, 3 + i, False, -vb[i], vb[i], 0.0, 0.0) for i in range(3)]
        rows.sort(key=lambda r: not r[2])  # soft first (stable: the reference's order within each kind)
        self.term_rows = rows
        self.nhN = len(rows)
        self.nsN = sum(1 for r in rows if r[2])
        self.lhN = np.array([r[3] for r in rows], dtype=float)
        self.uhN = np.array([r[4] for r in rows], dtype=float)
        self.zlN = np.array([r[5] for r in rows if r[2]], dtype=float)
        self.ZlN = np.array([r[6] for r in rows if r[2]], dtype=float)
        # flags.sdf_cost: stage residual (1 - s/2)^4 of the flagged SDF value, weight 20
        # (gen_model.py:65-66, base_model.py:add_cost_stage); the QP forms it from h[2], J_h[2]
        self.sdf_cost = E and bool(fl.get("sdf_cost"))
        self.extra_W = np.array([20.0]) if self.sdf_cost else np.array([])
        self.ny = 11 + len(self.extra_W)
        # the network is evaluated only where a row or the cost reads it
        self.need_sdf = 2 in self.h_cols or self.sdf_cost or RF
        # braking-distance polynomial (gen_model.py:76-78): user-supplied coefficients
        self.poly_deg = int(cfg.mpc.braking_dist.degree) if RF else 0
        self.poly = np.zeros(0)
        if RF:
            if braking_coeffs is None:
                braking_coeffs = load_braking_coeffs(cfg)
            self.poly = np.asarray(braking_coeffs, dtype=float).ravel()
            n = len(poly_terms(self.poly_deg))
            if self.poly_deg > 6 or self.poly.size != n:
                raise UnsupportedConfig(f"braking polynomial: degree {self.poly_deg} needs {n} coefficients "
                                        f"(got {self.poly.size}); degrees up to 6 are built")
        # terminal cost: stability scales y_N by the flag and adds flag |v|^2 (quad_rollpitchyawrate.py:52-55,
        # gen_model.py:142-149); its weight p_term is the reference's extra_WN, which Nmpc.set_ref never
        # applies (it writes WN = W[:nyN], controller.py:141) -- kept here for a caller that wants it
        self.nyN = 5 if ST else 4
        self.extra_WN = np.array([stability_p_term(cfg)]) if ST else np.array([])

    # ---- input -> command maps (quad_rollpitchyawrate.py:37-45): batched over leading dims of x, u
    def _att(self, u):
        lim = self.cfg.robot.limits
        u = np.asarray(u, dtype=float)
        return u[..., 0] * lim.gamma, u[..., 1] * lim.roll, u[..., 2] * lim.pitch, u[..., 3] * lim.wz

    def u_to_TRPYr(self, x, u, p=None):
        """[thrust, roll, pitch, yaw rate] (quad_rollpitchyawrate.py:45)."""
        gamma, roll, pitch, wz = self._att(u)
        return np.stack([gamma * self.cfg.robot.mass, roll, pitch, wz], axis=-1)

    def u_to_acc(self, x, u, p=None):
        """[W_R_B^T W_a, wz] (quad_rollpitchyawrate.py:44): body-frame acceleration and yaw rate."""
        x = np.asarray(x, dtype=float)
        gamma, roll, pitch, wz = self._att(u)
        q = x[..., 3:7] / np.linalg.norm(x[..., 3:7], axis=-1, keepdims=True)
        th = np.arctan2(q[..., 3], q[..., 0])
        W_R_V = quat2rot(np.stack([np.cos(th), 0 * th, 0 * th, np.sin(th)], axis=-1))
        V_R_B = euler2rot_b(roll, pitch, 0 * roll)
        W_R_B = W_R_V @ V_R_B
        W_a = W_R_B[..., :, 2] * gamma[..., None] - np.array([0.0, 0.0, self.g])
        acc = np.einsum("...ji,...j->...i", W_R_B, W_a)
        return np.concatenate([acc, wz[..., None]], axis=-1)

    def weight_row(self, weights) -> np.ndarray:
        """The W row formate_ref builds from a weight set (Ref.W_on / W_off), as one array: what the
        device-side reference packing (csrc/ref_pack.hip) writes for every node."""
        w = weights
        return np.concatenate([w.Wp, [w.Wq[2]], w.Wv, w.Wq[:2], w.Ww[2:], [w.Wa], self.extra_W]).astype(np.float64)

    def formate_ref(self, ref):
        """(y_ref, W) in the residual layout y = [p, q_e[3], v, roll, pitch, wz, W_a[2]]."""
        yr = np.concatenate([ref.p, [0], ref.v, [0, 0], [ref.wz], [0], np.zeros_like(self.extra_W)])
        W = np.concatenate([ref.Wp, [ref.Wq[2]], ref.Wv, ref.Wq[:2], ref.Ww[2:], [ref.Wa], self.extra_W])
        return yr, W


def load_braking_coeffs(cfg):
    """np.load(cache_dir() / mpc.braking_dist.coeff_file) as gen_model.py:76-77 does (no pickles)."""
    import os
    from .ocp import cache_dir
    path = os.path.join(cache_dir(), cfg.mpc.braking_dist.coeff_file)
    if not os.path.exists(path):
        raise UnsupportedConfig(f"flags.recursive_feasibility needs the braking-distance coefficients {path} "
                                "(gen_model.py:76-77; pass braking_coeffs= to Quad to give them directly)")
    return np.load(path, allow_pickle=False)


def stability_p_term(cfg):
    """The terminal-cost weight of gen_model.py:128-148: max(r~ + max_vel_error, sc_max / a_b_min^2 / dt^2)."""
    w = _stab_weights(cfg)
    lim = cfg.robot.limits
    max_vel_error = (2 * cfg.ref.vref) ** 2 * float(np.max(w["vel"]))
    max_att = np.array([lim.roll, lim.pitch, lim.wz])
    max_att_error = max_att @ np.diag(np.concatenate([w["att"][:2], w["rates"][2:]])) @ max_att
    max_thrust_error = max(w["acc"] * (lim.gamma - G) ** 2, w["acc"] * G ** 2)
    sc_max = max_vel_error + max_att_error + max_thrust_error
    dt = cfg.mpc.T / cfg.mpc.N
    r_tilde = r_tilde_max(cfg, w)
    return float(max(r_tilde + max_vel_error, sc_max / cfg.mpc.stability.a_b_min ** 2 / dt ** 2))
