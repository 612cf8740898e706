"""TEST INFRASTRUCTURE: the flag sets of default.yaml:16-23 the parity tests run (gen_model.py:26-149).

Each entry: name -> (Config overrides, expected stage columns, expected terminal rows as (hN_col, hE_col,
soft)).  'lidar' is sensor.hfov >= 3.14 (gen_model.py:42: no hfov row), with a spherical sensor so that
Config's fov consistency check (utils/config.py:39-41) holds."""
import numpy as np

LIDAR = dict(sensor__hfov=3.1416, sensor__is_spherical=True, sensor__aspect_ratio=3.1416 / 0.4903)
RF = dict(flags__recursive_feasibility=True)
ST = dict(flags__recursive_feasibility=True, flags__stability=True)

FLAG_SETS = {
    "default": ({}, [0, 1, 2], [(0, -1, True), (1, -1, True), (2, -1, True)]),
    "no_sdf": (dict(flags__enable_sdf=False), [], []),
    "no_sdf_constraint": (dict(flags__sdf_constraint=False), [0, 1], [(0, -1, True), (1, -1, True)]),
    "sdf_cost_only": (dict(flags__sdf_constraint=False, flags__sdf_cost=True), [0, 1], [(0, -1, True), (1, -1, True)]),
    "no_vfov": (dict(flags__vfov_constraint=False), [0, 2], [(0, -1, True), (2, -1, True)]),
    "lidar": (LIDAR, [1, 2], [(1, -1, True), (2, -1, True)]),
    "lidar_sdf_only": (dict(LIDAR, flags__vfov_constraint=False), [2], [(2, -1, True)]),
    "rec_feas": (RF, [0, 1, 2], [(0, -1, True), (1, -1, True), (2, 0, False), (-1, 1, False), (-1, 2, False)]),
    "rec_feas_soft_brake": (dict(RF, mpc__weights__slack_brake=[50.0, 10.0]), [0, 1, 2],
                            [(0, -1, True), (1, -1, True), (2, 0, True), (-1, 1, False), (-1, 2, False)]),
    "stability": (ST, [0, 1, 2], [(0, -1, True), (1, -1, True), (2, 0, False), (-1, 1, False), (-1, 2, False),
                                  (-1, 3, False), (-1, 4, False), (-1, 5, False)]),
    "stability_lidar_no_vfov": (dict(ST, **LIDAR, flags__vfov_constraint=False), [2],
                                [(2, 0, False), (-1, 1, False), (-1, 3, False), (-1, 4, False), (-1, 5, False)]),
}


def config(name, **more):
    from sdf_nmpc_amd.config import Config
    over, _, _ = FLAG_SETS[name]
    return Config(**over, **more)


def quad(name, cfg=None, seed=0):
    from sdf_nmpc_amd import synth
    from sdf_nmpc_amd.model import Quad
    cfg = cfg or config(name)
    coeffs = synth.braking_coeffs(int(cfg.mpc.braking_dist.degree), seed) if cfg.flags.recursive_feasibility else None
    return Quad(cfg, braking_coeffs=coeffs)
