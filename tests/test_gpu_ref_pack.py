"""Device-side reference / parameter packing (csrc/ref_pack.hip), pinned directly
to the reference's own RefGen outputs (tests/golden/refgen_golden.npz, made by tests/golden/make_golden.py
from sdf_nmpc/ref_gen.py:7-130 over every yaw mode, stop-and-turn on/off, joystick and from_x0) through
formate_ref -> set_ref (quad_rollpitchyawrate.py:62-65, controller.py:133-142).  Exact except the
quaternions (atan2 / sin / cos of the device libm, within an ulp or two of glibc) and the rotated camera
pose (3-term dot products vs numpy's BLAS matmul)."""
import os

import numpy as np
import pytest

from sdf_nmpc_amd import _lib
from sdf_nmpc_amd.config import Config
from sdf_nmpc_amd.controller import Nmpc
from sdf_nmpc_amd.model import Quad
from sdf_nmpc_amd.reference import Ref, yaw2quat

pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("ignore:no SDF weights")]

Q_ATOL = 4e-16     # quaternion entries (|q| <= 1): an ulp or two of the trig functions
POSE_RTOL = 1e-15  # W_R_Bo @ B_p_C etc. vs numpy matmul
MODES = ["align", "ref", "current", "zero", "curent"]
SENTINEL = -7.0


@pytest.fixture(scope="module")
def rg():
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "refgen_golden.npz"))


def _expected(model, traj, n, ws, Wp=None):
    """q_d rows and the formate_ref outputs of the golden trajectory rows [p3 q4 v3 wz1]."""
    N = traj.shape[0] - 1
    qd, y, W = np.full((N + 1, 4), SENTINEL), np.full((N, model.ny), SENTINEL), np.full((N, model.ny), SENTINEL)
    yN, WN = np.full(4, SENTINEL), np.full(4, SENTINEL)
    for k in range(n):
        r = Ref(model.cfg)
        r.p, r.q, r.v, r.wz = traj[k, 0:3], traj[k, 3:7], traj[k, 7:10], traj[k, 10]
        r.use_weights(ws)
        if Wp is not None:
            r.Wp = Wp
        qd[k] = r.q
        yr, wr = model.formate_ref(r)
        if k < N:
            y[k], W[k] = yr, wr
        else:
            yN, WN = yr[:4], wr[:4]
    return qd, y, W, yN, WN


def _pack(ctx, cfg, model, kind, x0, wp_p=None, wp_q=None, vw=None, wrow=None):
    B, N = x0.shape[0], int(cfg.mpc.N)
    D = lambda a: _lib.DeviceArray.from_numpy(ctx, np.asarray(a, dtype=np.float64))  # noqa: E731
    bufs = dict(x0=D(x0), wrow=D(wrow), p=D(np.full((B, N + 1, model.np), SENTINEL)),
                yref=D(np.full((B, N, model.ny), SENTINEL)), W=D(np.full((B, N, model.ny), SENTINEL)),
                yNref=D(np.full((B, 4), SENTINEL)), WN=D(np.full((B, 4), SENTINEL)))
    n_wp = 0
    if kind == 0:
        bufs.update(wp_p=D(wp_p), wp_q=D(wp_q))
        n_wp = wp_p.shape[1]
    elif kind == 1:
        bufs["vw"] = D(vw)
    _lib.pack_refs(ctx, _lib.ref_opts(cfg, kind), B, N, model.np, model.ny, bufs, n_wp=n_wp)
    ctx.synchronize()
    return {k: v.numpy() for k, v in bufs.items()}


def _check(got, b, model, exp):
    qd, y, W, yN, WN = exp
    np.testing.assert_allclose(got["p"][b, :, 13:17], qd, rtol=0, atol=Q_ATOL)
    np.testing.assert_array_equal(got["p"][b, :, :13], SENTINEL)  # parameters other than q_d untouched
    np.testing.assert_array_equal(got["p"][b, :, 17:], SENTINEL)
    np.testing.assert_array_equal(got["yref"][b], y)
    np.testing.assert_array_equal(got["W"][b], W)
    np.testing.assert_array_equal(got["yNref"][b], yN)  # N references (from_x0, stop-and-turn): node N unset
    np.testing.assert_array_equal(got["WN"][b], WN)


def test_pack_refs_waypoints_vs_reference_refgen(gpu_ctx, rg):
    """gen_ref_list_wps: the 40 golden cases, each knob set (yaw mode incl. the reference's 'curent',
    stop-and-turn, dang_min, align offset, vref, T, N) one batch of the cases that share it."""
    for c in range(int(rg["n_wps_cases"])):
        mode, st_on, dang, off, vref, dmin, T, N = rg[f"w{c}/knobs"]
        cfg = Config(mpc__N=int(N), mpc__T=float(T))
        cfg.ref.yaw_mode = MODES[int(mode)]
        cfg.ref.stop_and_turn.enable = bool(st_on)
        cfg.ref.stop_and_turn.dang_min = float(dang)
        cfg.ref.align_yaw_offset = float(off)
        cfg.ref.vref = float(vref)
        cfg.ref.yaw_align_dmin = float(dmin)
        model = Quad(cfg)
        ws = Ref(cfg).W_on
        x0 = rg[f"w{c}/x0"][None]
        got = _pack(gpu_ctx, cfg, model, 0, x0, rg[f"w{c}/wp_p"][None], rg[f"w{c}/wp_q"][None],
                    wrow=model.weight_row(ws))
        _check(got, 0, model, _expected(model, rg[f"w{c}/traj"], int(rg[f"w{c}/len"]), ws))


def test_pack_refs_joystick_and_hover_vs_reference_refgen(gpu_ctx, rg):
    """gen_ref_joystick (position weights zeroed, ref_gen.py:122) and from_x0 (N references), batched:
    every joystick case of a yaw mode in one launch."""
    for mode in range(3):
        cs = [c for c in range(int(rg["n_joy_cases"])) if int(rg[f"j{c}/mode"]) == mode]
        if not cs:
            continue
        cfg = Config()
        cfg.ref.yaw_mode = ["align", "ref", "curent"][mode]
        model = Quad(cfg)
        ws = Ref(cfg).W_on
        wrow = model.weight_row(ws)
        wrow[:3] = 0.0
        got = _pack(gpu_ctx, cfg, model, 1, np.stack([rg[f"j{c}/x0"] for c in cs]),
                    vw=np.stack([rg[f"j{c}/vw"] for c in cs]), wrow=wrow)
        for i, c in enumerate(cs):
            traj = rg[f"j{c}/traj"]
            _check(got, i, model, _expected(model, traj, traj.shape[0], ws, Wp=rg[f"j{c}/Wp"]))
    cfg = Config()
    model = Quad(cfg)
    ws = Ref(cfg).W_on
    got = _pack(gpu_ctx, cfg, model, 2, rg["from_x0/x0"][None], wrow=model.weight_row(ws))
    traj = rg["from_x0/traj"]
    full = np.full((int(cfg.mpc.N) + 1, 11), np.nan)
    full[: traj.shape[0]] = traj
    _check(got, 0, model, _expected(model, full, traj.shape[0], ws))


def test_pack_latent_matches_set_latent(gpu_ctx):
    cfg = Config(mpc__N=20)
    B, N = 5, 20
    rng = np.random.default_rng(3)
    n = Nmpc(cfg, batch=B)
    lat = rng.normal(0, 1, (B, 128))
    pos = rng.uniform(-3, 3, (B, 3))
    R = np.stack([np.linalg.qr(rng.normal(size=(3, 3)))[0] for _ in range(B)])
    flag = (np.arange(B) % 2).astype(float)
    n.set_sdf_flag(flag)
    n.set_latent(lat, pos, R)
    host_p = n.p.copy()
    n.set_latent_device(lat, pos, R, flag=flag)
    dp = n.ocp.download("p")
    np.testing.assert_array_equal(dp[..., 0], host_p[..., 0])
    np.testing.assert_allclose(dp[..., 1:13], host_p[..., 1:13], rtol=POSE_RTOL, atol=1e-15)
    np.testing.assert_array_equal(dp[..., 17:], host_p[..., 17:])
    n.ocp.close()


def test_nmpc_device_refs_solve_equals_host_path(gpu_ctx):
    """Nmpc.gen_refs_device + set_latent_device + solve == the same parameters set from the host."""
    cfg = Config()
    B = 4
    rng = np.random.default_rng(8)
    x0 = np.zeros((B, 10))
    x0[:, :3] = rng.uniform(-1, 1, (B, 3))
    x0[:, 3:7] = np.stack([yaw2quat(y) for y in rng.uniform(-np.pi, np.pi, B)])
    lat = rng.normal(0, 1, (B, 128))
    R = np.stack([np.eye(3)] * B)
    wp_p = x0[:, None, :3] + rng.uniform(-3, 3, (B, 2, 3))
    wp_q = np.stack([[yaw2quat(0.4), yaw2quat(-0.2)]] * B)
    ws = Ref(cfg).W_on
    # device path
    nd = Nmpc(cfg, batch=B)
    nd.set_x0(x0)
    nd.set_latent_device(lat, x0[:, :3], R, flag=1.0)
    nd.gen_refs_device("wps", wps=(wp_p, wp_q), weights=ws)
    assert nd.solve() == 0
    # the host path with the same parameters / references: set through the Ocp with host arrays
    nh = Nmpc(cfg, batch=B)
    nh.set_x0(x0)
    nh.ocp.solve(x0, nd.ocp.download("yref"), nd.ocp.download("yNref")[:, 0], nd.ocp.download("W"),
                 nd.ocp.download("WN")[:, 0], nd.ocp.download("p"))
    np.testing.assert_array_equal(nd.get_u(), nh.get_u())
    # and the device-written references are the ones formate_ref gives for the device's own q_d rows
    qd = nd.ocp.download("p")[:, :, 13:17]
    assert np.isfinite(qd).all() and np.allclose(np.linalg.norm(qd, axis=-1), 1.0, atol=1e-12)
    nh.ocp.close()
    nd.ocp.close()
