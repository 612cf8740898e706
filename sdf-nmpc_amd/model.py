"""The default 'att' (roll/pitch/yaw-rate) quadrotor OCP: dimensions, bounds, reference layout.

Host-side description only -- the arithmetic (dynamics, residuals, constraints and their Jacobians)
runs in csrc/linearize.hip and csrc/sdf_mlp.hip.  Mirrors (paths relative to the reference checkout):
  * dimensions / bounds / hover input ... sdf_nmpc/model/quad_rollpitchyawrate.py:12-17, 366, 380-381
  * formate_ref ........................ sdf_nmpc/model/quad_rollpitchyawrate.py:62-65
  * constraint set (default flags) ..... sdf_nmpc/gen_model.py:35,41-70, model/cost_const_helpers.py:48-75
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


class Quad:
    """'att' model + the SDF/FOV constraint set of gen_model.get_model_from_cfg (default flags)."""

    nx, nu, ny, nyN = 10, 4, 11, 4

    def __init__(self, cfg, max_df: float = 1.0):
        self.cfg = cfg
        self.name = "quad_rollpitchyawrate"
        fl = cfg.flags
        if cfg.mpc.model != "att":
            raise UnsupportedConfig(f"mpc.model '{cfg.mpc.model}': only 'att' is built (SURVEY.md §8: default model)")
        if fl.get("recursive_feasibility") or fl.get("stability"):
            # the reference itself cannot build these: gen_model.py:74 asserts on a non-existent
            # cfg.control_mode (AttributeError) -- SURVEY.md Appendix A
            raise UnsupportedConfig("flags recursive_feasibility / stability are broken in the reference "
                                    "(gen_model.py:74 reads cfg.control_mode, which Config does not define)")
        if not (fl.get("enable_sdf") and fl.get("sdf_constraint") and fl.get("vfov_constraint")):
            raise UnsupportedConfig("this build evaluates h = [hfov, vfov, sdf]: enable_sdf, sdf_constraint and "
                                    "vfov_constraint must be True")
        if not cfg.sensor.hfov < 3.14:
            raise UnsupportedConfig("hfov >= 3.14 drops the hfov constraint (gen_model.py:42); not built")
        self.name += "_sdf"  # gen_model.py:29
        self.max_df = float(max_df)
        self.p_idx = cfg.mpc.p_idx
        self.np = int(cfg.mpc.p_idx.latent) + int(cfg.nn.size_latent)
        lim = cfg.robot.limits
        self.g = G
        self.lbu = np.array([0.0, -1.0, -1.0, -1.0])
        self.ubu = np.array([1.0, 1.0, 1.0, 1.0])
        self.u_hover = np.array([G / lim.gamma, 0.0, 0.0, 0.0])
        # h = [hfov, vfov, sdf]; bounds (cost_const_helpers.py:66-75, gen_model.py:35)
        hfov_lim = cfg.sensor.hfov * cfg.mpc.fov_ratio
        vfov_lim = cfg.sensor.vfov * cfg.mpc.fov_ratio
        self.lh = np.array([-hfov_lim, -vfov_lim, cfg.robot.size.xy + cfg.mpc.bound_margin])
        self.uh = np.array([hfov_lim, vfov_lim, self.max_df + 0.2])
        self.nh = self.nhN = 3
        # every h row is soft (slack weights L1, L2): fov rows slack_fov, sdf row slack_df
        sf, sd = cfg.mpc.weights.slack_fov, cfg.mpc.weights.slack_df
        self.zl = np.array([sf[0], sf[0], sd[0]], dtype=float)
        self.Zl = np.array([sf[1], sf[1], sd[1]], dtype=float)
        # flags.sdf_cost: stage residual (1 - s/2)^4 of the flagged SDF value, weight 20
        # (gen_model.py:65-66, base_model.py:add_cost_stage); the QP forms it from h[2], J_h[2]
        self.sdf_cost = bool(fl.get("sdf_cost"))
        self.extra_W = np.array([20.0]) if self.sdf_cost else np.array([])
        self.ny = 11 + len(self.extra_W)

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
