"""The default 'att' (roll/pitch/yaw-rate) quadrotor OCP: dimensions, bounds, reference layout.

Host-side description only -- the arithmetic (dynamics, residuals, constraints and their Jacobians)
runs in csrc/linearize.hip and csrc/sdf_mlp.hip.  Mirrors (paths relative to the reference checkout):
  * dimensions / bounds / hover input ... sdf_nmpc/model/quad_rollpitchyawrate.py:12-17, 366, 380-381
  * formate_ref ........................ sdf_nmpc/model/quad_rollpitchyawrate.py:384-387
  * constraint set (default flags) ..... sdf_nmpc/gen_model.py:35,41-70, model/cost_const_helpers.py:435-462
  * slack weights ...................... model/base_model.py:296-322, ocp.py:85-92
"""
from __future__ import annotations

import numpy as np

G = 9.81  # model/base_model.py:10


class UnsupportedConfig(ValueError):
    pass


class Quad:
    """'att' model + the SDF/FOV constraint set of gen_model.get_model_from_cfg (default flags)."""

    nx, nu, ny, nyN = 10, 4, 11, 4

    def __init__(self, cfg, max_df: float = 1.0):
        self.cfg = cfg
        self.name = "quad_rollpitchyawrate"
        fl = cfg.flags
        if cfg.mpc.model != "att":
            raise UnsupportedConfig(f"mpc.model '{cfg.mpc.model}': only 'att' is built (SURVEY.md §8: default model)")
        if fl.get("recursive_feasibility") or fl.get("stability") or fl.get("sdf_cost"):
            raise UnsupportedConfig("flags recursive_feasibility / stability / sdf_cost are not built "
                                    "(SURVEY.md §8(f) rank 4)")
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
        # h = [hfov, vfov, sdf]; bounds (cost_const_helpers.py:454-462, gen_model.py:35)
        hfov_lim = cfg.sensor.hfov * cfg.mpc.fov_ratio
        vfov_lim = cfg.sensor.vfov * cfg.mpc.fov_ratio
        self.lh = np.array([-hfov_lim, -vfov_lim, cfg.robot.size.xy + cfg.mpc.bound_margin])
        self.uh = np.array([hfov_lim, vfov_lim, self.max_df + 0.2])
        self.nh = self.nhN = 3
        # every h row is soft (slack weights L1, L2): fov rows slack_fov, sdf row slack_df
        sf, sd = cfg.mpc.weights.slack_fov, cfg.mpc.weights.slack_df
        self.zl = np.array([sf[0], sf[0], sd[0]], dtype=float)
        self.Zl = np.array([sf[1], sf[1], sd[1]], dtype=float)
        self.extra_W = np.array([])

    def formate_ref(self, ref):
        """(y_ref, W) in the residual layout y = [p, q_e[3], v, roll, pitch, wz, W_a[2]]."""
        yr = np.concatenate([ref.p, [0], ref.v, [0, 0], [ref.wz], [0], np.zeros_like(self.extra_W)])
        W = np.concatenate([ref.Wp, [ref.Wq[2]], ref.Wv, ref.Wq[:2], ref.Ww[2:], [ref.Wa], self.extra_W])
        return yr, W
