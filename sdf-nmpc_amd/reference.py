"""Reference / waypoint containers (mirror of sdf_nmpc/utils/reference.py:6-53).

Kept bit-compatible with the reference, including its known quirk:
``Ref.W_on`` is filled from ``set_const_off`` and ``W_off`` from ``set_const_on`` (reference.py:15-28).
``Quad.formate_ref`` reads ``ref.Wp/Wq/Wv/Ww/Wa``, which the caller (the external ROS node, or
``Ref.use_weights``) must set.
"""
import numpy as np

from .config import AttrDict


def quat2yaw(q):
    """reference utils/math.py:73-82 (numpy branch)."""
    return np.arctan2(2 * (q[0] * q[3] + q[1] * q[2]), 1 - 2 * (q[2] * q[2] + q[3] * q[3]))


def yaw2quat(yaw):
    """reference utils/math.py:142-166 (numpy branch)."""
    h = yaw * 0.5
    return np.array([np.cos(h), 0.0, 0.0, np.sin(h)])


class Ref:
    def __init__(self, cfg):
        self.cfg = cfg
        self.p = [0., 0., 0.]
        self.q = [1., 0., 0., 0.]
        self.v = [0., 0., 0.]
        self.wz = 0.
        w = cfg.mpc.weights
        self.W_on = AttrDict({"Wp": w.set_const_off.pos, "Wq": w.set_const_off.att, "Wv": w.set_const_off.vel,
                              "Ww": w.set_const_off.rates, "Wa": w.set_const_off.acc})
        self.W_off = AttrDict({"Wp": w.set_const_on.pos, "Wq": w.set_const_on.att, "Wv": w.set_const_on.vel,
                               "Ww": w.set_const_on.rates, "Wa": w.set_const_on.acc})

    def use_weights(self, ws):
        """Copy one weight set onto the attributes formate_ref reads (what the ROS wrapper does)."""
        self.Wp, self.Wq, self.Wv, self.Ww, self.Wa = ws.Wp, ws.Wq, ws.Wv, ws.Ww, ws.Wa
        return self

    def hover_at_state(self, x):
        self.p = x[:3]
        self.q = yaw2quat(quat2yaw(x[3:7]))
        self.v = [0., 0., 0.]
        self.wz = 0.


class Waypoint:
    def __init__(self, p, q=(1, 0, 0, 0)):
        self.p = np.array(p, dtype=float)
        self.q = np.array(q, dtype=float)
