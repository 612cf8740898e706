"""Configuration: YAML -> attribute dict with the reference's derived fields.

Mirrors ``sdf_nmpc/utils/config.py:9-44`` (``AttrDict``, ``Config``): same schema, same derived
``sensor.B_p_C`` / ``sensor.B_R_C`` (config.py:43-44) and the same FOV consistency assertion
(config.py:39-41).  Reference YAML files load unchanged.  Uses ``yaml.safe_load``.
"""
import os

import numpy as np
import yaml

DEFAULT_CONFIG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "config", "default.yaml")


class AttrDict(dict):
    """dict with attribute access, recursively (reference config.py:9-27)."""

    def __init__(self, d=None):
        super().__init__()
        for k, v in (d or {}).items():
            self[k] = v

    def __setitem__(self, key, value):
        if isinstance(value, dict) and not isinstance(value, AttrDict):
            value = AttrDict(value)
        elif isinstance(value, list):
            value = [AttrDict(v) if isinstance(v, dict) else v for v in value]
        super().__setitem__(key, value)

    def __getattr__(self, key):
        try:
            return self[key]
        except KeyError as e:
            raise AttributeError(key) from e

    def __setattr__(self, key, value):
        self[key] = value


def euler2rot(e):
    """Z1Y2X3 euler [roll, pitch, yaw] -> rotation matrix (reference utils/math.py:26-54, numpy)."""
    r, p, y = e
    sr, cr, sp, cp, sy, cy = np.sin(r), np.cos(r), np.sin(p), np.cos(p), np.sin(y), np.cos(y)
    return np.array([[cp * cy, sr * sp * cy - cr * sy, cr * sp * cy + sr * sy],
                     [cp * sy, sr * sp * sy + cr * cy, cr * sp * sy - sr * cy],
                     [-sp, sr * cp, cr * cp]])


def get_vfov(hfov, aspect_ratio, is_spherical):
    """reference utils/math.py:286-291."""
    return hfov / aspect_ratio if is_spherical else np.arctan(np.tan(hfov) / aspect_ratio)


class Config(AttrDict):
    def __init__(self, config_file=DEFAULT_CONFIG, **overrides):
        with open(config_file, "r") as f:
            d = yaml.safe_load(f)
        super().__init__(d)
        for path, v in overrides.items():  # e.g. Config(mpc__N=40)
            node = self
            keys = path.split("__")
            for k in keys[:-1]:
                node = node[k]
            node[keys[-1]] = v
        vfov_cpt = get_vfov(self.sensor.hfov, self.sensor.aspect_ratio, self.sensor.is_spherical)
        assert abs(vfov_cpt - self.sensor.vfov) < 0.1, "check sensor fov in config file"
        self.sensor.B_p_C = self.robot.sensor_extrinsics.position
        self.sensor.B_R_C = euler2rot(self.robot.sensor_extrinsics.orientation)
