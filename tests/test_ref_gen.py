"""RefGen mirror (sdf-nmpc_amd/ref_gen.py) against the reference's own RefGen outputs
(tests/golden/refgen_golden.npz, tests/golden/make_golden.py::refgen_golden): bit-exact."""
import copy

import numpy as np
import pytest

from sdf_nmpc_amd.config import Config
from sdf_nmpc_amd.ref_gen import RefGen
from sdf_nmpc_amd.reference import Waypoint

MODES = ["align", "ref", "current", "zero", "curent"]


def _cfg(knobs):
    mode, st_on, dang, off, vref, dmin, T, N = knobs
    cfg = Config(mpc__N=int(N), mpc__T=float(T))
    cfg.ref.yaw_mode = MODES[int(mode)]
    cfg.ref.stop_and_turn.enable = bool(st_on)
    cfg.ref.stop_and_turn.dang_min = float(dang)
    cfg.ref.align_yaw_offset = float(off)
    cfg.ref.vref = float(vref)
    cfg.ref.yaw_align_dmin = float(dmin)
    return cfg


def _rows(traj, N):
    rows = np.full((N + 1, 11), np.nan)
    for k, r in enumerate(traj):
        rows[k] = np.concatenate([np.asarray(r.p, float), np.asarray(r.q, float), np.asarray(r.v, float), [float(r.wz)]])
    return rows


def test_gen_ref_list_wps_bit_exact(golden_refgen):
    g = golden_refgen
    for c in range(int(g["n_wps_cases"])):
        cfg = _cfg(g[f"w{c}/knobs"])
        N = int(cfg.mpc.N)
        rg = RefGen(cfg)
        rg.x0 = g[f"w{c}/x0"]
        wps = [Waypoint(p, q) for p, q in zip(g[f"w{c}/wp_p"], g[f"w{c}/wp_q"])]
        traj = rg.gen_ref_list_wps(wps)
        assert len(traj) == int(g[f"w{c}/len"]), c
        np.testing.assert_array_equal(_rows(traj, N), g[f"w{c}/traj"], err_msg=f"case {c}")


def test_gen_ref_joystick_and_from_x0_bit_exact(golden_refgen):
    g = golden_refgen
    for c in range(int(g["n_joy_cases"])):
        cfg = Config()
        cfg.ref.yaw_mode = ["align", "ref", "curent"][int(g[f"j{c}/mode"])]
        rg = RefGen(cfg)
        rg.x0 = g[f"j{c}/x0"]
        traj = rg.gen_ref_joystick(g[f"j{c}/vw"])
        got = np.array([np.concatenate([np.asarray(r.p, float), np.asarray(r.q, float), np.asarray(r.v, float),
                                        [float(r.wz)]]) for r in traj])
        np.testing.assert_array_equal(got, g[f"j{c}/traj"])
        np.testing.assert_array_equal(np.asarray(traj[0].Wp, float), g[f"j{c}/Wp"])
    rg = RefGen(Config())
    rg.x0 = g["from_x0/x0"]
    got = np.array([np.concatenate([np.asarray(r.p, float), np.asarray(r.q, float), np.asarray(r.v, float),
                                    [float(r.wz)]]) for r in rg.from_x0()])
    np.testing.assert_array_equal(got, g["from_x0/traj"])


@pytest.fixture(scope="module")
def golden_refgen():
    import os
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "refgen_golden.npz"))
