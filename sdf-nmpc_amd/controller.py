"""Batched GPU counterpart of the reference controller (sdf_nmpc/controller.py:Nmpc).

Same methods, argument meaning and array layouts as the reference; every per-instance array gains
an optional leading batch dimension (``batch`` instances solved together, one SQP-RTI iteration per
``solve``).  With ``batch=1`` the shapes are exactly the reference's.

  reset()                              controller.py:35    p, y, yN, W, WN zeroed, flag off, latent reset
  set_sdf_flag(flag)                   controller.py:45
  set_latent(latent, W_p_Bo, W_R_Bo)   controller.py:50    W_p_Co, W_R_Co (row-major 3x3), latent in p
  reset_latent()                       controller.py:57
  set_x0(x0)                           controller.py:65    first call initialises the OCP
  solve()                              controller.py:72    shift + one RTI iteration; returns fail_count
  get_matrices(), get_u(), get_cmd_acc(), get_cmd_TRPYr(), get_openloop_traj(), eval(k), set_ref(ref, k)

Host setters write the host arrays (``p``, ``y``, ``W``, ``yN``, ``WN``) and mark the rows and columns
they touched; ``solve`` uploads exactly those regions.  Device-side setters (``gen_refs_device``,
``set_latent_device``, ``VaeWrapper.encode_to``) write the solver's device buffers directly and clear
the host marks of what they wrote.  The last writer of a region wins, whichever side it is on.
No tensor library is used on this path.

``get_cmd_props`` exists in the reference only for the 'props' model; this build is the 'att' model
(model.Quad), where the reference raises AttributeError too.
"""
from __future__ import annotations

import numpy as np

from .model import Quad


class Nmpc:
    """Wrapper around the NMPC controller with range image-based collision prediction (batched)."""

    def __init__(self, cfg, rebuild=False, batch: int = 1, device: int = 0, weights=None, ocp=None,
                 braking_coeffs=None):
        """braking_coeffs: the braking-distance polynomial of flags.recursive_feasibility (default: the
        config's mpc.braking_dist.coeff_file under the cache dir, as gen_model.py:76-77 loads it)."""
        from .ocp import Ocp

        self.cfg = cfg
        self.model = getattr(ocp, "model", None) or Quad(cfg, braking_coeffs=braking_coeffs)
        self.T = cfg.mpc.T
        self.N = int(cfg.mpc.N)
        self.B = int(batch)
        self.ocp = ocp if ocp is not None else Ocp(self.model, build=rebuild, batch=batch, device=device,
                                                  weights=weights)
        lim = cfg.robot.limits
        self.cmd_acc_hover = np.array([0, 0, 0, 0])
        self.cmd_acc_min = [-lim.ax, -lim.ay, -lim.az, -lim.wz]
        self.cmd_acc_max = [lim.ax, lim.ay, lim.az, lim.wz]
        self.cmd_TRPYr_hover = np.array([cfg.robot.mass * self.model.g, 0, 0, 0])
        self.cmd_TRPYr_min = [0, -lim.roll, -lim.pitch, -lim.wz]
        self.cmd_TRPYr_max = [lim.gamma, lim.roll, lim.pitch, lim.wz]
        self.reset()

    # ---- state of the controller (host arrays, batch-leading; B == 1 keeps the reference's shapes)
    def _shape(self, *s):
        return s if self.B == 1 else (self.B,) + s

    # ---- dirty regions of the host arrays: (field, col0, ncol) -> row mask [B][nodes]
    def _groups(self):
        idx, m = self.cfg.mpc.p_idx, self.model
        return {"flag": ("p", int(idx.flag), 1), "pose": ("p", int(idx.W_p_Co[0]), 12),
                "q_d": ("p", int(idx.q_d[0]), 4), "latent": ("p", int(idx.latent), m.np - int(idx.latent)),
                "yref": ("yref", 0, m.ny), "W": ("W", 0, m.ny), "yNref": ("yNref", 0, m.nyN), "WN": ("WN", 0, m.nyN)}

    def _mark(self, group, b=None, k=None):
        """Mark rows (instance b or all, node k or all) of a column group dirty."""
        field, _, _ = self._groups()[group]
        nodes = {"p": self.N + 1, "yref": self.N, "W": self.N}.get(field, 1)
        m = self._dirty.setdefault(group, np.zeros((max(self.B, 1), nodes), bool))
        m[(slice(None) if b is None else b), (slice(None) if k is None else k)] = True

    def _flush(self):
        """Upload the dirty host regions into the solver's device buffers."""
        host = {"p": self.p, "yref": self.y, "W": self.W, "yNref": self.yN, "WN": self.WN}
        groups = self._groups()
        for g, mask in self._dirty.items():
            field, col0, ncol = groups[g]
            a = host[field]
            a = a[None] if self.B == 1 else a
            if field in ("yNref", "WN"):
                a = a[:, None]
            self.ocp.upload(field, a, col0, ncol, mask)
        self._dirty = {}

    def _clean(self, *groups):
        for g in groups:
            self._dirty.pop(g, None)

    def reset(self):
        """Reset internal matrices to default values (controller.py:35-44)."""
        m = self.model
        self._dirty = {}
        self.x0 = None
        self.p = np.zeros(self._shape(self.N + 1, m.np))
        self.y = np.zeros(self._shape(self.N, m.ny))
        self.yN = np.zeros(self._shape(m.nyN))
        self.W = np.zeros(self._shape(self.N, m.ny))
        self.WN = np.zeros(self._shape(m.nyN))
        self.fail_count = 0
        self.fail_counts = np.zeros(self.B, dtype=int)  # per-instance consecutive QP failures
        self.set_sdf_flag(False)
        self.reset_latent()
        for g in ("q_d", "yref", "W", "yNref", "WN"):
            self._mark(g)

    # ---- parameter setters
    def set_sdf_flag(self, flag):
        """Enable/disable the sdf constraint (controller.py:47-49); flag: scalar or [B]."""
        f = np.asarray(flag, dtype=float)
        self.p[..., self.cfg.mpc.p_idx.flag] = f[..., None] if f.ndim else f
        self._mark("flag")

    def set_latent(self, latent, W_p_Bo, W_R_Bo):
        """Latent and camera pose at the time of the image (controller.py:50-54), batched over a leading dim."""
        idx = self.cfg.mpc.p_idx
        W_R_Bo = np.asarray(W_R_Bo, dtype=float)
        W_p_Co = W_R_Bo @ np.asarray(self.cfg.sensor.B_p_C, dtype=float).ravel() + W_p_Bo
        W_R_Co = (W_R_Bo @ np.asarray(self.cfg.sensor.B_R_C, dtype=float)).reshape(W_R_Bo.shape[:-2] + (9,))
        self.p[..., idx.W_p_Co] = np.asarray(W_p_Co)[..., None, :]
        self.p[..., idx.W_R_Co] = W_R_Co[..., None, :]
        self.p[..., idx.latent:] = np.asarray(latent, dtype=float)[..., None, :]
        self._mark("pose")
        self._mark("latent")

    def reset_latent(self):
        """controller.py:59-63."""
        idx = self.cfg.mpc.p_idx
        self.p[..., idx.W_p_Co] = 0
        self.p[..., idx.W_R_Co] = 0
        self.p[..., idx.latent:] = 0
        self._mark("pose")
        self._mark("latent")

    # ---- control iteration
    def set_x0(self, x0):
        """Current state feedback (controller.py:67-71); the first call initialises the OCP iterate."""
        x0 = np.asarray(x0, dtype=float)[..., : self.model.nx]
        if self.x0 is None:
            self.ocp.init(x0)
        self.x0 = x0

    def solve(self):
        """One SQP-RTI iteration for every instance (controller.py:72-81)."""
        try:
            self.ocp.shift(self.cfg.mpc.shift)
            self._flush()  # host-set regions; device-set regions are already in place
            self.ocp.solve(self.x0, None, None, None, None, None)
            self.fail_count = 0
        except Exception as e:  # same contract as the reference: report, count, keep running
            print("solver failed:", e)
            self.fail_count += 1
        # fail_count is batch-wide (any failed instance counts, as one reference solver per instance would
        # for that instance); fail_counts holds the per-instance consecutive failures
        mask = getattr(self.ocp, "fail_mask", None)
        if mask is not None:
            self.fail_counts = np.where(mask, getattr(self, "fail_counts", 0) + 1, 0)
        return self.fail_count

    # ---- getters
    def get_matrices(self):
        """x [.., N+1, nx], u [.., N, nu] of the current iterate (controller.py:87-96)."""
        x = self.ocp.download("x")
        u = self.ocp.download("u")
        return (x[0], u[0]) if self.B == 1 else (x, u)

    def get_u(self):
        """Last computed MPC inputs (controller.py:99-101)."""
        return self.ocp.get_u()

    def get_cmd_acc(self):
        """controller.py:104-106."""
        return np.clip(self.model.u_to_acc(self.x0, self.get_u()), self.cmd_acc_min, self.cmd_acc_max)

    def get_cmd_TRPYr(self):
        """controller.py:109-111."""
        return np.clip(self.model.u_to_TRPYr(self.x0, self.get_u()), self.cmd_TRPYr_min, self.cmd_TRPYr_max)

    def get_openloop_traj(self):
        """Predicted (position, quaternion) path, node 0 = x0 (controller.py:119-125); batched: per instance."""
        x, _ = self.get_matrices()
        x = x if self.B > 1 else x[None]
        x0 = self.x0 if self.B > 1 else self.x0[None]
        paths = []
        for b in range(x.shape[0]):
            path = [(x0[b][[0, 1, 2]], x0[b][[3, 4, 5, 6]])]
            for k in range(1, self.N + 1):
                path.append((x[b, k][[0, 1, 2]], x[b, k][[3, 4, 5, 6]]))
            paths.append(path)
        return paths[0] if self.B == 1 else paths

    def eval(self, k):
        """The model's evaluation vector at node k (controller.py:125-130, base_model.py:119-125): [0] without
        flags.enable_sdf; else the SDF value with flag = 1 (gen_model.py:64, computed by the HIP SDF kernel),
        and with recursive_feasibility the braking distance poly(v) and sdf - poly(v), flag = 1
        (gen_model.py:116-117)."""
        m = self.model
        if not m.enable_sdf:
            return [0] if self.B == 1 else np.zeros((self.B, 1))
        from .model import poly_eval
        idx = self.cfg.mpc.p_idx
        x = self.ocp.download("x")[:, k]
        p = self.p if self.B > 1 else self.p[None]
        pk = p[:, k]
        W_R_Co = pk[:, idx.W_R_Co].reshape(-1, 3, 3)
        Co_p_B = np.einsum("bji,bj->bi", W_R_Co, x[:, :3] - pk[:, idx.W_p_Co])
        df, _ = self.ocp.net.eval_host(np.concatenate([Co_p_B, pk[:, idx.latent:]], axis=1), want_grad=False)
        out = df[:, None]
        if m.rec_feas:
            bd, _ = poly_eval(m.poly, m.poly_deg, x[:, 7:10])
            out = np.concatenate([out, bd[:, None], (df - bd)[:, None]], axis=1)
        return out[0] if self.B == 1 else out

    # ---- device-side parameter packing (csrc/ref_pack.hip)
    def _dev(self, a):
        """Host array -> device (fp64); a device array (DeviceArray / FieldView / torch tensor) passes through."""
        from . import _lib
        if hasattr(a, "data_ptr"):
            if np.dtype(str(a.dtype).replace("torch.", "")) != np.float64:
                raise TypeError(f"device input must be float64, got {a.dtype}")
            return _lib.sync_producer(a)  # a torch tensor may still be in flight on torch's stream
        return _lib.DeviceArray.from_numpy(self.ocp.ctx, np.asarray(a, dtype=np.float64))

    def gen_refs_device(self, mode="wps", wps=None, vw=None, weights=None):
        """RefGen + formate_ref + set_ref for every instance and node in one kernel launch, written straight
        into the solver's device buffers (p[:, :, q_d], y, W, yN, WN).

        mode 'wps': ``RefGen.gen_ref_list_wps`` (ref_gen.py:25-99) from x0 (``set_x0``) through the
        waypoints ``wps = (p [B][n][3], q [B][n][4])`` (or a list of ``Waypoint`` for B = 1); 'joystick':
        ``gen_ref_joystick(vw)`` (ref_gen.py:101-130), vw [B][4]; 'hover': ``from_x0`` (ref_gen.py:17-23).
        ``weights`` is the weight set formate_ref reads (e.g. ``Ref(cfg).W_on``); the joystick mode zeroes
        its position weights as gen_ref_joystick does.  The host arrays of these regions are not updated;
        a later host setter of a region (e.g. set_ref at one node) overrides it at the next ``solve``.
        """
        from . import _lib
        from .reference import Ref
        if self.x0 is None:
            raise ValueError("set_x0 before gen_refs_device (the references start at the current state)")
        Bn = max(self.B, 1)
        ws = weights if weights is not None else Ref(self.cfg).W_on
        wrow = self.model.weight_row(ws)
        code = {"wps": 0, "joystick": 1, "hover": 2}[mode]
        if code == 1:
            wrow[:3] = 0.0  # ref.Wp = [0, 0, 0] (ref_gen.py:122)
        args = {"x0": self._dev(np.reshape(self.x0, (Bn, -1))), "wrow": self._dev(wrow)}
        n_wp = 0
        if code == 0:
            if isinstance(wps, (list, tuple)) and len(wps) and hasattr(wps[0], "p"):
                wps = (np.array([w.p for w in wps])[None], np.array([w.q for w in wps])[None])
            wp_p = np.reshape(np.asarray(wps[0], float), (Bn, -1, 3))
            wp_q = np.reshape(np.asarray(wps[1], float), (Bn, -1, 4))
            n_wp = wp_p.shape[1]
            args.update(wp_p=self._dev(wp_p), wp_q=self._dev(wp_q))
        elif code == 1:
            args["vw"] = self._dev(np.reshape(np.asarray(vw, float), (Bn, 4)))
        for k in ("p", "yref", "W", "yNref", "WN"):
            args[k] = self.ocp.field(k)
        _lib.pack_refs(self.ocp.ctx, _lib.ref_opts(self.cfg, code), Bn, self.N, self.model.np, self.model.ny, args,
                       n_wp=n_wp, nyN=self.model.nyN)
        self.ocp.ctx.synchronize()  # the temporary inputs are freed on return
        self._clean("q_d", "yref", "W", "yNref", "WN")

    def set_latent_device(self, latent, W_p_Bo, W_R_Bo, flag=None):
        """set_latent (+ set_sdf_flag) on the device buffers for every instance (controller.py:45-54);
        latent: host array or a device array [B][L] fp64 (e.g. VaeWrapper's latents, no host round trip).
        With the batch split over devices (Ocp(devices=...), shard.plan) each part packs its own instance
        rows on its own device: a device array on that device is read in place (a view at the part's first
        row), one on another device goes through the host once."""
        from . import _lib
        Bn = max(self.B, 1)
        L = int(self.cfg.nn.size_latent)
        cols = {"latent": L, "W_p_Bo": 3, "W_R_Bo": 9, "flag": 1}
        given = {"latent": latent, "W_p_Bo": W_p_Bo, "W_R_Bo": W_R_Bo}
        if flag is not None:
            given["flag"] = flag if hasattr(flag, "data_ptr") else np.broadcast_to(np.asarray(flag, float), (Bn,))
        host = {}
        for k, v in given.items():
            if not hasattr(v, "data_ptr"):
                host[k] = np.reshape(np.asarray(v, dtype=np.float64), (Bn, cols[k]))
            elif np.dtype(str(v.dtype).replace("torch.", "")) != np.float64:
                raise TypeError(f"device input must be float64, got {v.dtype}")
        parts = self.ocp.parts
        synced = set()
        for part in parts:
            lo, nb = part.lo, part.hi - part.lo
            args = {"p": part.solver.field("p")}
            for k, v in given.items():
                if k in host:
                    args[k] = _lib.DeviceArray.from_numpy(part.ctx, np.ascontiguousarray(host[k][lo:part.hi]))
                elif len(parts) == 1:
                    args[k] = _producer_done(v, part.ctx, synced)
                elif _device_of(v) == part.ctx.device:  # a view of the part's rows, in place
                    v = given[k] = _producer_done(v, part.ctx, synced)
                    args[k] = _lib.FieldView(v.data_ptr() + lo * cols[k] * 8, (nb, cols[k]), np.float64, part.ctx)
                else:  # another device: through the host, once per array
                    host[k] = _download(v, Bn, cols[k])
                    args[k] = _lib.DeviceArray.from_numpy(part.ctx, np.ascontiguousarray(host[k][lo:part.hi]))
            _lib.pack_refs(part.ctx, _lib.ref_opts(self.cfg, -1), nb, self.N, self.model.np, self.model.ny, args, L=L,
                           nyN=self.model.nyN)
        for part in parts:
            part.ctx.synchronize()
        self._clean("pose", "latent", *(("flag",) if flag is not None else ()))

    def set_ref(self, ref, k, b=None):
        """y, W and q_d of node k from a reference object (controller.py:136-142); b selects one instance
        of a batch (None: all)."""
        sel = () if self.B == 1 else (slice(None),) if b is None else (b,)
        self.p[sel + (k, self.cfg.mpc.p_idx.q_d)] = ref.q
        self._mark("q_d", b, k)
        y, W = self.model.formate_ref(ref)
        if k < self.N:
            self.y[sel + (k,)] = y
            self.W[sel + (k,)] = W
            self._mark("yref", b, k)
            self._mark("W", b, k)
        else:
            self.WN[sel] = W[: self.model.nyN]
            self.yN[sel] = y[: self.model.nyN]
            self._mark("yNref", b)
            self._mark("WN", b)


def _producer_done(a, ctx, synced: set):
    """A device array about to be read in place by a kernel on ``ctx``'s stream, once everything that
    produces it has finished: a torch tensor waits for torch's current stream (made contiguous first: the
    in-place views assume row-major [B][cols]); an array owned by another context (a DeviceArray or solver
    FieldView, e.g. VaeWrapper.latent64 written by the encoder's stream) waits for that context's stream.
    Each array is synchronised once per call (``synced``)."""
    from . import _lib
    if type(a).__module__.split(".")[0] == "torch":
        if not a.is_contiguous():
            a = a.contiguous()
        return _lib.sync_producer(a)
    owner = getattr(a, "ctx", None)
    if owner is not None and owner is not ctx and id(a) not in synced:
        owner.synchronize()
        synced.add(id(a))
    return a


def _device_of(a) -> int:
    """HIP device of a device array: DeviceArray / FieldView (its context's), torch tensor (its own)."""
    ctx = getattr(a, "ctx", None)
    if ctx is not None:
        return int(ctx.device)
    if type(a).__module__.split(".")[0] == "torch":
        return int(a.device.index or 0)
    raise TypeError(f"device of {type(a).__name__} unknown (expected a DeviceArray, FieldView or torch tensor)")


def _download(a, rows, cols):
    """Host copy [rows][cols] fp64 of a device array (DeviceArray or torch tensor)."""
    if hasattr(a, "numpy") and not type(a).__module__.startswith("torch"):
        return np.reshape(a.numpy(), (rows, cols))
    return np.reshape(a.detach().cpu().numpy(), (rows, cols))
