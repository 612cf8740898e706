"""Which closed-loop scenarios with the SDF flag on are contractive?  For each config override, the
oracle pipeline (tests/test_gpu_closed_loop.py::_oracle_loop) is run twice -- latents as given and
x (1 + 1e-7) -- and the per-step |u - u'| printed, next to the GPU controller's distance to the oracle.
Diagnostic only (GPU box: the controller needs a device)."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import oracle as O
from sdf_nmpc_amd import weights as W
from sdf_nmpc_amd.config import Config
from sdf_nmpc_amd.controller import Nmpc
from test_gpu_controller import scenario
from test_gpu_closed_loop import _oracle_loop, _plant

O.build()
onet = O.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=0))
K = 10
for name, over in [("default", {}), ("margin-0.6", dict(mpc__bound_margin=-0.6)),
                   ("margin-0.6 fov3", dict(mpc__bound_margin=-0.6, mpc__fov_ratio=3.0)),
                   ("margin-1.2 fov3", dict(mpc__bound_margin=-1.2, mpc__fov_ratio=3.0))]:
    for shift in (0, 1):
        cfg = Config(mpc__N=20, mpc__shift=shift, **over)
        n = Nmpc(cfg, batch=4)
        x0 = scenario(n, np.random.default_rng(31))
        n.set_sdf_flag(1.0)
        ug, xg = [], x0.copy()
        for _ in range(K):
            n.set_x0(xg)
            assert n.solve() == 0
            ug.append(n.get_u().copy())
            xg = _plant(O, onet, cfg, xg, ug[-1], n.ocp.dt[0])
        uo, _, _ = _oracle_loop(O, onet, n, cfg, x0, n.p, K)
        p = n.p.copy()
        p[..., 17:] *= 1 + 1e-7
        up, _, _ = _oracle_loop(O, onet, n, cfg, x0, p, K)
        env = np.abs(up - uo).max(axis=(1, 2))
        d = np.abs(np.array(ug) - uo).max(axis=(1, 2))
        h = n.ocp.download("h") if hasattr(n.ocp, "download") else None
        print(f"{name:18s} shift {shift}: env {' '.join(f'{v:.0e}' for v in env)}")
        print(f"{'':18s}          gpu {' '.join(f'{v:.0e}' for v in d)}")
        n.ocp.close()
        sys.stdout.flush()
