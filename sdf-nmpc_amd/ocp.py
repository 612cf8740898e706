"""Batched GPU counterpart of the reference OCP object (sdf_nmpc/ocp.py).

The reference builds an acados OCP (NONLINEAR_LS cost, ERK, SQP_RTI, FULL_CONDENSING_HPIPM, soft h
constraints, input boxes; ocp.py:17-128) for ONE quadrotor and calls ``solve_for_x0`` per control
step.  Here the same iteration -- preparation phase (csrc/sdf_mlp.hip + csrc/linearize.hip),
feedback QP (csrc/rti_qp.hip) and the full-step iterate update -- runs for ``batch`` independent
instances at once, through the solver object of include/sdfnmpc.h (``sdfnmpc_solver``, which owns the
device workspace: no tensor library is involved).  The method names, argument meaning and array
layouts are the reference's (plus an optional leading batch dimension):

  Ocp(model, build)                   ocp.py:17    shooting grid, solver buffers
  init(x0)                            ocp.py:144   x_k = x0, u_k = u_hover
  shift(k)                            ocp.py:152   x_{i-k} = x_i, u_{i-k} = u_i for i = k..N-1
  solve(x0, y, yN, W, WN, p)          ocp.py:159   one SQP-RTI iteration, u = u_0
  get_u(), get_t()                    ocp.py:173   last u_0, solve wall time [s]
  solver.get(k, 'x' | 'u'), solver.set(k, ...), solver.reset(), solver.get_stats('time_tot')

Occupancy gate (north_star): with several ``devices`` the batch is split over as
many GPUs as it needs to fill (``shard.plan``: one GPU runs up to ``Context.qp_capacity(N)`` instances
concurrently -- 1024 at N = 40), each part a contiguous instance range with its own context, network
copy and solver; a step enqueues every part before waiting on any.

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
from . import shard
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

    @staticmethod
    def _field(field):
        if field not in ("x", "u"):
            raise KeyError(f"field {field!r}: only 'x' and 'u' are exposed")
        return field

    def get(self, k, field):
        v = self.ocp.download(self._field(field))[:, k]
        return v[0] if self.ocp.B == 1 else v

    def set(self, k, field, value):
        name = self._field(field)
        nodes = self.ocp.N + 1 if name == "x" else self.ocp.N
        full = np.zeros((self.ocp.B, nodes, 10 if name == "x" else 4))
        full[:, k] = np.asarray(value, dtype=np.float64)
        mask = np.zeros((self.ocp.B, nodes), bool)
        mask[:, k] = True
        self.ocp.upload(name, full, mask=mask)

    def reset(self):
        for name in ("x", "u", "dx", "du"):
            self.ocp.upload(name, 0.0)

    def get_stats(self, name):
        if name == "time_tot":
            return self.ocp.t
        if name == "qp_iter":
            return self.ocp.iters
        if name == "status":
            return self.ocp.status
        raise KeyError(name)


class _Part:
    """One device's share of the batch: instances [lo, hi) on their own context / network / solver."""

    def __init__(self, lo, hi, ctx, net, solver, own_ctx, own_net):
        self.lo, self.hi, self.ctx, self.net, self.solver = lo, hi, ctx, net, solver
        self.own_ctx, self.own_net = own_ctx, own_net


class Ocp:
    def __init__(self, model: Quad, build=False, batch: int = 1, device: int = 0, net=None, ctx=None,
                 weights=None, lm=None, qp_tol=1e-8, qp_iter_max=100, devices=None, lm_scaling=True,
                 qp_warm_start=True):
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
        self.cmodel = _lib.quad_model(cfg, model)
        # QP data of the model + solver options (ocp.py:113-120: LM regularisation, <= 100 iterations)
        # qp_warm_start: HPIPM's primal warm start, on by default as the reference configures its solver
        # (ocp.py:116 sets qp_solver_warm_start = 1): each QP starts from the previous one's du (the solver
        # object keeps it; zero after init).  The solution is unique (lm > 0), so the start changes iteration
        # counts, not the step beyond the QP tolerance (tools/ws_probe.py)
        self.qp_opts = _lib.qp_opts(model, lm=float(cfg.mpc.lm_reg if lm is None else lm), max_iter=qp_iter_max,
                                    tol=qp_tol, lm_scaling=lm_scaling, warm_start=qp_warm_start)
        devs = list(devices) if devices else [device]
        if ctx is None:  # the first device's context sizes the plan (sdfnmpc_qp_capacity_for: this constraint set)
            c0 = _lib.Context(devs[0])
            self.plan = shard.plan(B, c0.qp_capacity(N, self.qp_opts), len(devs))
        else:
            c0, self.plan = ctx, [(0, 0, B)]
        # one QP kernel for the whole batch (AUTO picks by batch size: include/sdfnmpc.h), so the split over
        # devices never changes a result -- every part runs what one part of B instances would
        qp_kind = c0.qp_kernel(N, B) if len(self.plan) > 1 else None
        self.parts = []
        for slot, lo, hi in self.plan:
            c = c0 if slot == 0 else _lib.Context(devs[slot])
            if qp_kind is not None:
                c.set_qp_kernel(qp_kind)
            # the network only with flags.enable_sdf (gen_model.py:26-39); the solver evaluates it only where a
            # constraint row or the cost reads it (Nmpc.eval reads it too)
            n = (net if (net is not None and slot == 0) else load_net(c, cfg, weights)) if model.enable_sdf else None
            s = _lib.Solver(c, n, self.cmodel, self.qp_opts, hi - lo, N, model.np, model.ny, self.dt)
            self.parts.append(_Part(lo, hi, c, n, s, ctx is None, n is not net))
        self.ctx, self.net = self.parts[0].ctx, self.parts[0].net
        self.solver = _SolverView(self)
        self.u = np.zeros((B, model.nu)) if B > 1 else np.zeros(model.nu)
        self.t = 0.0
        self.status = np.zeros(B, dtype=np.int32)
        self.iters = np.zeros(B, dtype=np.int32)

    # ---- device buffers (host views through the solver object)
    def upload(self, name, host, col0=0, ncol=None, mask=None):
        """host / mask: full-batch arrays [B][nodes][width] / [B][nodes] (a missing batch dim broadcasts);
        each part uploads its own instance rows."""
        shp = self.parts[0].solver.shape(name)
        full = np.broadcast_to(np.asarray(host, dtype=np.float64), (self.B,) + shp[1:])
        m = None if mask is None else np.broadcast_to(np.asarray(mask, bool), (self.B, shp[1]))
        for p in self.parts:
            p.solver.upload(name, full[p.lo:p.hi], col0, ncol, None if m is None else m[p.lo:p.hi])

    def download(self, name):
        return np.concatenate([p.solver.download(name) for p in self.parts])

    def field(self, name):
        """Device memory of a field (single-part Ocp): a view for the device-side setters."""
        if len(self.parts) != 1:
            raise ValueError("field(): the batch is split over several devices; use each part's solver")
        return self.parts[0].solver.field(name)

    # ---- the reference API
    def init(self, x0):
        """ocp.py:144-149: reset, x_k = x0 for k = 0..N, u_k = u_hover."""
        x0 = np.broadcast_to(np.asarray(x0, dtype=np.float64), (self.B, 10))
        for p in self.parts:
            p.solver.init(x0[p.lo:p.hi], self.model.u_hover)

    def shift(self, k=1):
        """ocp.py:152-156: x_{i-k} = x_i, u_{i-k} = u_i for i = k..N-1 (x_N and the tail keep their values)."""
        for p in self.parts:
            p.solver.shift(int(k))

    def solve(self, x0, y, yN, W, WN, p):
        """ocp.py:159-170: set x0 / references / weights (diagonals) / parameters, one SQP-RTI iteration.
        An argument given as None keeps the device buffer as it is (uploaded by Nmpc or written by a
        device-side setter)."""
        N, m = self.N, self.model
        for name, v, shape in (("x0", x0, (1, m.nx)), ("yref", y, (N, m.ny)), ("W", W, (N, m.ny)),
                               ("yNref", yN, (1, m.nyN)), ("WN", WN, (1, m.nyN)), ("p", p, (N + 1, m.np))):
            if v is not None:
                self.upload(name, np.reshape(np.asarray(v, dtype=np.float64), (-1,) + shape))
        t0 = time.perf_counter()
        for part in self.parts:  # every device busy before the host waits on any
            part.solver.step()
        u0 = np.concatenate([part.solver.wait().copy() for part in self.parts])
        self.t = time.perf_counter() - t0
        self.status = np.concatenate([part.solver.status for part in self.parts])
        self.iters = np.concatenate([part.solver.iters for part in self.parts])
        failed = self.status >= 2
        if failed.any() and getattr(self, "u", None) is not None:  # as solve_for_x0 raising before `self.u = ...`
            u0[failed] = np.reshape(self.u, u0.shape)[failed]   # (ocp.py:169): a failed instance keeps its last u_0
        self.fail_mask = failed
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
        for p in self.parts:
            p.solver.close()
            if p.own_net and p.net is not None:
                p.net.close()
            if p.own_ctx:
                p.ctx.close()
        self.parts = []
