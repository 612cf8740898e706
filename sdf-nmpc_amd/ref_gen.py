"""Reference trajectory generation (mirror of sdf_nmpc/ref_gen.py:7-130) and its batched device form.

``RefGen`` keeps the reference's per-instance host API (``from_x0``, ``gen_ref_list_wps``,
``gen_ref_joystick``) in numpy with the same arithmetic order, so its outputs are pinned bit for bit
to the reference's own (tests/golden/refgen_golden.npz).  Quirks kept on purpose:
``force_yaw_current`` compares ``yaw_mode`` with the misspelt ``'curent'`` (ref_gen.py:12), so mode
``'current'`` falls through to the identity quaternion in ``gen_ref_list_wps``; ``from_x0`` and the
stop-and-turn early return produce N (not N+1) references.

``pack_refs`` is SURVEY.md §8(f) rank 3: waypoint resampling + ``formate_ref`` + ``Nmpc.set_ref`` /
``set_latent`` for B instances x (N+1) nodes in one kernel launch (csrc/ref_pack.hip), writing the
OCP's device buffers (p, yref, W, yNref, WN) instead of 3 (N+1) host setter calls per instance.
"""
from __future__ import annotations

import copy

import numpy as np

from .reference import Ref, quat2yaw, yaw2quat

YAW_MODES = {"ref": 0, "align": 1, "current": 2, "zero": 3, "curent": 4}


class RefGen:
    def __init__(self, cfg):
        self.cfg = cfg
        self.x0 = None
        self.ref = Ref(cfg)
        self.force_yaw_current = (self.cfg.ref.yaw_mode == "curent")  # ref_gen.py:12 (sic)

    def _reset(self):
        self.ref = Ref(self.cfg)

    def from_x0(self):
        """ref_gen.py:17-23: hover at the current state (N references)."""
        ref = copy.copy(self.ref)
        ref.p = self.x0[:3]
        ref.q = yaw2quat(quat2yaw(self.x0[3:7]))
        ref.v = [0., 0., 0.]
        ref.wz = 0.
        return [ref] * self.cfg.mpc.N

    def gen_ref_list_wps(self, wps):
        """ref_gen.py:25-99: resample the path x0 -> waypoints at vref * T / N (N+1 references)."""
        self._reset()
        cfg = self.cfg
        trajectory = []
        path_p = np.vstack([self.x0[:3], [wp.p for wp in wps]])
        path_q = np.vstack([self.x0[3:7], [wp.q for wp in wps]])
        path_yaw = list(map(quat2yaw, path_q))

        if cfg.ref.stop_and_turn.enable:  # ref_gen.py:35-53
            yaw_curr = path_yaw[0]
            yaw_r = yaw_curr
            if cfg.ref.yaw_mode == "topic":
                yaw_r = quat2yaw(path_q[1])
            elif cfg.ref.yaw_mode == "align":
                dxy = path_p[1][:2] - self.x0[:2]
                if np.linalg.norm(dxy) > cfg.ref.yaw_align_dmin:
                    yaw_r = np.arctan2(dxy[1], dxy[0])
                yaw_r += cfg.ref.align_yaw_offset
            if abs(yaw_curr - yaw_r) > cfg.ref.stop_and_turn.dang_min:
                ref = copy.copy(self.ref)
                ref.p = self.x0[:3]
                ref.v = [0, 0, 0]
                ref.q = yaw2quat(yaw_r)
                return [ref] * cfg.mpc.N

        distances = np.linalg.norm(np.diff(path_p, axis=0), axis=1)
        cumulative_distances = np.cumsum(distances)
        cumulative_distances = np.insert(cumulative_distances, 0, 0)
        total_distance = cumulative_distances[-1]
        if total_distance / 1e-3:
            vref = min(cfg.ref.vref, total_distance)
            even_distances = np.arange(0, total_distance, cfg.mpc.T / cfg.mpc.N * vref)
            for d in even_distances:
                segment_index = np.searchsorted(cumulative_distances, d) - 1
                segment_index = max(0, min(segment_index, len(distances) - 1))
                direction = (path_p[segment_index + 1] - path_p[segment_index]) / distances[segment_index]
                delta_dist = (d - cumulative_distances[segment_index])
                ref = copy.copy(self.ref)
                ref.p = path_p[segment_index] + direction * delta_dist
                ref.v = direction * vref
                if self.force_yaw_current:
                    ref.q = path_q[0]
                elif cfg.ref.yaw_mode == "ref":
                    ref.q = yaw2quat(path_yaw[segment_index + 1])
                elif cfg.ref.yaw_mode == "align":
                    dxy = path_p[1][:2] - self.x0[:2]
                    if np.linalg.norm(dxy) > cfg.ref.yaw_align_dmin:
                        yaw_r = np.arctan2(ref.v[1], ref.v[0])
                        yaw_r += cfg.ref.align_yaw_offset
                        ref.q = yaw2quat(yaw_r)
                    else:
                        ref.q = path_q[0]
                else:
                    ref.q = [1, 0, 0, 0]
                trajectory.append(ref)
                if len(trajectory) > cfg.mpc.N:
                    break

        while len(trajectory) <= cfg.mpc.N:
            ref = copy.copy(self.ref)
            ref.p = trajectory[-1].p if trajectory else path_p[-1]
            ref.q = trajectory[-1].q if trajectory else path_q[-1]
            trajectory.append(ref)
        return trajectory

    def gen_ref_joystick(self, vwref):
        """ref_gen.py:101-130: constant (vx, vy, vz, wz) command integrated from x0 (N+1 references)."""
        cfg = self.cfg
        ref = copy.copy(self.ref)
        ref.v = np.array(vwref[:3]) * cfg.ref.vref
        ref.wz = np.array(vwref[3]) * cfg.ref.wzref
        if self.force_yaw_current:
            ref.q = yaw2quat(quat2yaw(self.x0[3:7]))
        elif cfg.ref.yaw_mode == "align":
            vxy = ref.v[:2]
            if np.linalg.norm(vxy) > cfg.ref.yaw_align_dmin:
                ref.q = yaw2quat(np.arctan2(vxy[1], vxy[0]))
            else:
                ref.q = yaw2quat(quat2yaw(self.x0[3:7]))
        else:
            ref.q = [1, 0, 0, 0]
        ref.Wp = [0, 0, 0]
        trajectory = []
        for i in range(cfg.mpc.N + 1):
            trajectory.append(copy.copy(ref))
            trajectory[-1].p = self.x0[:3] + (ref.v * i * cfg.mpc.T / cfg.mpc.N)
        return trajectory


def weight_row(model, weights) -> np.ndarray:
    """The W row formate_ref builds from a weight set (Ref.W_on / W_off, quad_rollpitchyawrate.py:62-65)."""
    w = weights
    return np.concatenate([w.Wp, [w.Wq[2]], w.Wv, w.Wq[:2], w.Ww[2:], [w.Wa], model.extra_W]).astype(np.float64)
