"""TEST INFRASTRUCTURE: the flag sets of default.yaml:16-23 the parity tests run (gen_model.py:26-149).

Each entry: name -> (Config overrides, expected stage columns, expected terminal rows as (hN_col, hE_col,
soft)).  'lidar' is sensor.hfov >= 3.14 (gen_model.py:42: no hfov row), with a spherical sensor so that
Config's fov consistency check (utils/config.py:39-41) holds."""
import numpy as np

LIDAR = dict(sensor__hfov=3.1416, sensor__is_spherical=True, sensor__aspect_ratio=3.1416 / 0.4903)
RF = dict(flags__recursive_feasibility=True)
ST = dict(flags__recursive_feasibility=True, flags__stability=True)
# hard stage rows (slack weight None: add_const_stage / add_const_term without slack, base_model.py:142-168)
HARD_FOV = dict(mpc__weights__slack_fov=None)
HARD_DF = dict(mpc__weights__slack_df=None)

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
    # stage rows ordered soft first (model.Quad.h_cols), terminal rows soft first
    "hard_fov": (HARD_FOV, [2, 0, 1], [(2, -1, True), (0, -1, False), (1, -1, False)]),
    "hard_df": (HARD_DF, [0, 1, 2], [(0, -1, True), (1, -1, True), (2, -1, False)]),
    "hard_all": (dict(HARD_FOV, **HARD_DF), [0, 1, 2], [(0, -1, False), (1, -1, False), (2, -1, False)]),
    "hard_fov_lidar": (dict(LIDAR, **HARD_FOV), [2, 1], [(2, -1, True), (1, -1, False)]),
    "hard_df_rec_feas": (dict(RF, **HARD_DF), [0, 1, 2],
                         [(0, -1, True), (1, -1, True), (2, 0, False), (-1, 1, False), (-1, 2, False)]),
}
HARD_SETS = [n for n in FLAG_SETS if n.startswith("hard")]


def config(name, **more):
    from sdf_nmpc_amd.config import Config
    over, _, _ = FLAG_SETS[name]
    return Config(**{**over, **more})


def quad(name, cfg=None, seed=0):
    from sdf_nmpc_amd import synth
    from sdf_nmpc_amd.model import Quad
    cfg = cfg or config(name)
    coeffs = braking(cfg) if cfg.flags.recursive_feasibility else None
    return Quad(cfg, braking_coeffs=coeffs)


def uses_scene(q):
    """Sets with a hard row (stage rows with slack None, the rec_feas braking / Co_p_E rows, stability's
    velocity box) are run on the fitted obstacle-scene network (tests/golden/scene.sdfw, scene_setup.py) at
    the reference's own bounds: on the SIREN initialisation (df ~ 0 everywhere, every point inside an
    obstacle) a hard sdf or braking row demands moves no input sequence gives, and the QP is infeasible
    or degenerate -- for the reference's HPIPM as much as here."""
    return q.nhN > q.nsN or q.nhs > 0


def braking(cfg):
    """The braking polynomial of a physical braking law: d(v) = 0.05 + |v|^2 / (2 a_b_min) in the basis of
    polynomial_3variate (utils/math.py:307-314), a_b_min = mpc.stability.a_b_min (default.yaml:73-74)."""
    from sdf_nmpc_amd import synth
    return synth.braking_coeffs(int(cfg.mpc.braking_dist.degree), noise=0.0, a_brake=float(cfg.mpc.stability.a_b_min))


def problem(cfg, q, B, N, seed):
    """The synthetic problem of a set (synth.make_problem), its velocity along the camera's view (the braking
    point and the trajectory inside the field of view), and with uses_scene the scene latent in p."""
    from sdf_nmpc_amd import synth
    prob = synth.make_problem(cfg, B, N, seed=seed, sdf_cost=q.sdf_cost, nyN=q.nyN, v_forward=True)
    if uses_scene(q):
        import scene_setup as S
        prob["p"][..., 17:17 + 128] = S.scene_latent()
        # the image taken 1 m behind the start (camera moved back along the body's x axis): the start lies
        # inside the field of view, not at the camera's origin where the fov functions (atan2 of a few
        # centimetres) swing through the whole range -- a hard fov row would be infeasible at node 1
        fwd = synth.quat2rot(prob["x"][:, 0, 3:7])[:, :, 0]
        prob["p"][..., 1:4] -= fwd[:, None, :]
    return prob
