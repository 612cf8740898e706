"""Batched GPU counterpart of the reference OCP object (sdf_nmpc/ocp.py).

The reference builds an acados OCP (NONLINEAR_LS cost, ERK, SQP_RTI, FULL_CONDENSING_HPIPM, soft h
constraints, input boxes; ocp.py:17-128) for ONE quadrotor and calls ``solve_for_x0`` per control
step.  Here the same iteration -- preparation phase (csrc/sdf_mlp.hip + csrc/linearize.hip),
feedback QP (csrc/rti_qp.hip) and the full-step iterate update -- runs for ``batch`` independent
instances at once on one GPU, through the C ABI of include/sdfnmpc.h.  The method names, argument
meaning and array layouts are the reference's (plus an optional leading batch dimension):

  Ocp(model, build)                   ocp.py:17    shooting grid, solver buffers
  init(x0)                            ocp.py:148   x_k = x0, u_k = u_hover
  shift(k)                            ocp.py:156   x_{i-k} = x_i, u_{i-k} = u_i for i = k..N-1
  solve(x0, y, yN, W, WN, p)          ocp.py:163   one SQP-RTI iteration, u = u_0
  get_u(), get_t()                    ocp.py:175   last u_0, solve wall time [s]
  solver.get(k, 'x' | 'u'), solver.set(k, ...), solver.reset(), solver.get_stats('time_tot')

``build_solver`` (ocp.py:9) installs what an acados user links instead of the L4CasADi library: the
CasADi external-function shim ``libsdf_l4c.so`` (include/sdf_l4c.h) and its weights, in
``<cache>/codegen/<cfg.name>/`` -- the directory ocp.py:103-105 names as
``model_external_shared_lib_dir``.

There is no CPU fallback: a missing HIP library or GPU raises (``_lib.SdfnmpcError`` / OSError).
"""
from __future__ import annotations

import os
import shutil
import time
import warnings

import numpy as np

from . import _lib
from . import weights as Wt
from .config import Config
from .model import Quad


def cache_dir() -> str:
    """Counterpart of sdf_nmpc.cache_dir() (sdf_nmpc/__init__.py): $SDFNMPC_CACHE or ~/.cache/sdf_nmpc_amd."""
    d = os.environ.get("SDFNMPC_CACHE") or os.path.join(os.path.expanduser("~"), ".cache", "sdf_nmpc_amd")
    os.makedirs(d, exist_ok=True)
    return d


def load_net(ctx, cfg, weights=None):
    """The SDF network: a packed ``.sdfw`` file (weights.pack; weights.from_torchscript converts the
    reference's TorchScript offline), ``$SDFNMPC_WEIGHTS``, or -- when neither is given -- the
    seeded SIREN initialisation (synthetic; the reference's weight files are LFS pointers here)."""
    path = weights or os.environ.get("SDFNMPC_WEIGHTS")
    if path:
        return _lib.Net.from_file(ctx, path)
    warnings.warn("no SDF weights given: using the seeded SIREN initialisation (synthetic network)")
    return _lib.Net.siren(ctx, 0)


def build_solver(cfg_file=None, weights=None) -> str:
    """Install the external-function shim + weights for an acados build (ocp.py:9-13).  Returns the dir."""
    cfg = Config(cfg_file) if cfg_file else Config()
    Quad(cfg)  # validates the configuration this build supports
    out = os.path.join(cache_dir(), "codegen", cfg.name)
    os.makedirs(out, exist_ok=True)
    shutil.copy2(_lib.l4c_path(), os.path.join(out, "libsdf_l4c.so"))
    dst = os.path.join(out, "sdf_l4c.sdfw")
    if weights:
        shutil.copy2(weights, dst)
    else:
        with open(dst, "wb") as f:
            f.write(Wt.pack(Wt.DEFAULT_SPEC, Wt.siren_weights(Wt.DEFAULT_SPEC, seed=0)))
    return out


class _SolverView:
    """The subset of AcadosOcpSolver the reference's controller/ocp use (get/set/reset/get_stats)."""

    def __init__(self, ocp: "Ocp"):
        self.ocp = ocp

    def _buf(self, field):
        if field not in ("x", "u"):
            raise KeyError(f"field {field!r}: only 'x' and 'u' are exposed")
        return self.ocp.bufs[field]

    def get(self, k, field):
        v = self._buf(field)[:, k].cpu().numpy()
        return v[0] if self.ocp.B == 1 else v

    def set(self, k, field, value):
        import torch
        buf = self._buf(field)
        buf[:, k] = torch.as_tensor(np.asarray(value, dtype=np.float64), device=buf.device).expand_as(buf[:, k])

    def reset(self):
        for k in ("x", "u", "dx", "du"):
            self.ocp.bufs[k].zero_()

    def get_stats(self, name):
        if name == "time_tot":
            return self.ocp.t
        if name == "qp_iter":
            return self.ocp.bufs["iters"].cpu().numpy()
        raise KeyError(name)


class Ocp:
    def __init__(self, model: Quad, build=False, batch: int = 1, device: int = 0, net=None, ctx=None,
                 weights=None, lm=None, qp_tol=1e-8, qp_iter_max=100):
        import torch

        self.model = model
        cfg = model.cfg
        self.T = cfg.mpc.T
        self.N = N = int(cfg.mpc.N)
        self.B = B = int(batch)
        # shooting grid (ocp.py:21-28) from the C ABI (bit-exact numpy.linspace semantics)
        self.shooting_nodes, self.dt = _lib.shooting_grid(N, self.T, bool(cfg.mpc.uniform_dt),
                                                          int(cfg.mpc.nb_short_nodes),
                                                          cfg.mpc.control_loop_time * 1e-3)
        if build:
            build_solver(weights=weights)
        self.device = torch.device("cuda", device)
        self.ctx = ctx or _lib.Context(device, stream=torch.cuda.current_stream(self.device).cuda_stream)
        self.net = net or load_net(self.ctx, cfg, weights)
        self.cmodel = _lib.quad_model(cfg)
        # QP data of the model + solver options (ocp.py:113-120: LM regularisation, <= 100 iterations)
        self.qp_opts = _lib.qp_opts(model, lm=float(cfg.mpc.lm_reg if lm is None else lm), max_iter=qp_iter_max,
                                    tol=qp_tol)
        f64 = dict(dtype=torch.float64, device=self.device)
        sh = dict(x=(B, N + 1, 10), u=(B, N, 4), p=(B, N + 1, model.np), x0=(B, 10), yref=(B, N, model.ny), W=(B, N, model.ny),
                  yNref=(B, 4), WN=(B, 4), xn=(B, N, 10), AB=(B, N, 14, 10), y=(B, N, 11), Jy=(B, N, 14, 11),
                  yN=(B, 4), JyN=(B, 10, 4), h=(B, N + 1, 3), Jh=(B, N + 1, 10, 3), dx=(B, N + 1, 10), du=(B, N, 4),
                  slack=(B, N + 1, 3, 2), res=(B, 2), u0=(B, 4))
        self.bufs = {k: torch.zeros(s, **f64) for k, s in sh.items()}
        self.bufs["dt"] = torch.as_tensor(self.dt, **f64)
        self.bufs["sdf"] = torch.zeros((B, N + 1, 4), dtype=torch.float32, device=self.device)
        self.bufs["status"] = torch.zeros(B, dtype=torch.int32, device=self.device)
        self.bufs["iters"] = torch.zeros(B, dtype=torch.int32, device=self.device)
        self.solver = _SolverView(self)
        self.u = np.zeros((B, model.nu)) if B > 1 else np.zeros(model.nu)
        self.t = 0.0
        self.status = np.zeros(B, dtype=np.int32)

    # ---- helpers
    def _put(self, name, value, shape):
        """Copy host (numpy) or device (torch) data into the named buffer; a missing batch dim broadcasts."""
        import torch
        buf = self.bufs[name]
        if isinstance(value, torch.Tensor):
            v = value.to(device=buf.device, dtype=buf.dtype)
        else:
            v = torch.as_tensor(np.array(value, dtype=np.float64), device=buf.device)
        if tuple(v.shape) == tuple(shape):
            v = v.unsqueeze(0)
        buf.copy_(v.expand_as(buf))

    # ---- the reference API
    def init(self, x0):
        """ocp.py:148-153: reset, x_k = x0 for k = 0..N, u_k = u_hover."""
        self.solver.reset()
        self._put("x0", x0, (10,))
        self.bufs["x"].copy_(self.bufs["x0"].unsqueeze(1).expand_as(self.bufs["x"]))
        self._put("u", np.broadcast_to(self.model.u_hover, (self.N, 4)), (self.N, 4))

    def shift(self, k=1):
        """ocp.py:156-160: x_{i-k} = x_i, u_{i-k} = u_i for i = k..N-1 (x_N and the tail keep their values)."""
        k = int(k)
        if k > 0 and k < self.N:
            x, u = self.bufs["x"], self.bufs["u"]
            x[:, : self.N - k] = x[:, k: self.N].clone()
            u[:, : self.N - k] = u[:, k: self.N].clone()

    def solve(self, x0, y, yN, W, WN, p):
        """ocp.py:163-172: set x0 / references / weights (diagonals) / parameters, one SQP-RTI iteration.
        An argument given as None keeps the device buffer as it is (written by ref_gen.pack_refs)."""
        N, m = self.N, self.model
        for name, v, shape in (("x0", x0, (m.nx,)), ("yref", y, (N, m.ny)), ("W", W, (N, m.ny)),
                               ("yNref", yN, (m.nyN,)), ("WN", WN, (m.nyN,)), ("p", p, (N + 1, m.np))):
            if v is not None:
                self._put(name, v, shape)
        b = self.bufs
        b["x"][:, 0] = b["x0"]
        t0 = time.perf_counter()
        _lib.linearize(self.ctx, self.net, self.cmodel, self.B, N, m.np, b)
        _lib.qp_solve(self.ctx, self.qp_opts, self.B, N, b)
        _lib.rti_apply(self.ctx, self.B, N, b["x"], b["u"], b["dx"], b["du"], b["u0"], status=b["status"])
        self.ctx.synchronize()
        self.t = time.perf_counter() - t0
        self.status = b["status"].cpu().numpy()
        u0 = b["u0"].cpu().numpy()
        self.u = u0[0] if self.B == 1 else u0
        if (self.status == 1).any():  # acados status 2 (QP max_iter): solve_for_x0 warns, keeps the step
            warnings.warn(f"QP reached qp_solver_iter_max on {(self.status == 1).sum()} of {self.B} instances")
        if (self.status >= 2).any():  # acados QP failure (status 4): solve_for_x0 raises; the iterate is kept
            raise _lib.SdfnmpcError(f"QP failure (non-finite data) on instances {np.flatnonzero(self.status >= 2)[:8]}"
                                    f" ({(self.status >= 2).sum()} of {self.B}); their iterate is unchanged")
        return self.u

    def get_u(self):
        return np.array(self.u)

    def get_t(self):
        return float(self.t)

    def close(self):
        self.net.close()
        self.ctx.close()
