"""ctypes front-end of the C oracle (oracle.c).  TEST INFRASTRUCTURE ONLY.

Importable by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg -- as the checker /
the timed CPU baseline, never as a product path.  ``build()`` compiles ``_build/liboracle.so`` with
the Makefile next to this file.
"""
import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "_build", "liboracle.so")


class Spec(C.Structure):
    _fields_ = [("L", C.c_int), ("n1", C.c_int), ("n2", C.c_int), ("n3", C.c_int), ("n4", C.c_int),
                ("nf", C.c_int), ("nd", C.c_int), ("w0", C.c_float), ("max_df", C.c_float)]


class Quad(C.Structure):
    _fields_ = [("gamma", C.c_double), ("roll", C.c_double), ("pitch", C.c_double), ("wz", C.c_double),
                ("g", C.c_double), ("B_p_C", C.c_double * 3), ("B_R_C", C.c_double * 9),
                ("fov_offset", C.c_double), ("max_df", C.c_double)]


def build(force=False):
    if force or not os.path.exists(LIB) or os.path.getmtime(LIB) < max(
            os.path.getmtime(os.path.join(HERE, f)) for f in ("oracle.c", "sdf_net.inc", "qp_ipm.c", "vae.c", "Makefile")):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        P = C.POINTER
        f, d, i64 = C.c_float, C.c_double, C.c_int64
        _lib.orc_prng_uniform.argtypes = [C.c_uint64, C.c_uint64, i64, P(d)]
        _lib.orc_sdf_f32.argtypes = [P(Spec), P(f), P(f), P(f), i64, P(f), P(f), P(f), P(f), C.c_int]
        _lib.orc_sdf_f64.argtypes = [P(Spec), P(f), P(f), P(f), i64, P(d), P(d), P(d), P(d)]
        _lib.orc_quad_rk4.argtypes = [P(Quad), P(d), P(d), d, P(d), P(d)]
        _lib.orc_quad_cost.argtypes = [P(Quad), P(d), P(d), P(d), P(d), P(d), P(d), P(d)]
        _lib.orc_quad_constr.argtypes = [P(Quad), P(d), P(d), d, P(d), P(d), P(d), P(d)]
        _lib.orc_shooting_grid.argtypes = [C.c_int, d, C.c_int, C.c_int, d, P(d), P(d)]
        _lib.orc_quad_term.argtypes = [P(Quad), P(d), P(d), C.c_int, P(d), C.c_int, C.c_int, P(d), P(d), P(d), P(d)]
        _lib.orc_linearize_batch.argtypes = [P(Quad), P(Spec), P(f), P(f), P(f), C.c_int, C.c_int, C.c_int,
                                             P(d), P(d), P(d), P(d), P(d), P(d), P(d), P(d), P(d), P(d),
                                             P(d), P(d), P(f), C.c_int]
        _lib.orc_max_threads.restype = C.c_int
        _lib.orc_qp_ipm_batch.argtypes = [C.c_int, C.c_int] + [P(d)] * 19 + [C.c_int, C.c_int, C.c_int, P(d), P(d),
                                                                             P(d), P(C.c_int), P(C.c_int), P(d),
                                                                             C.c_int]
        _lib.orc_vae_preprocess.argtypes = [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int, C.c_float,
                                            P(f), P(f)]
        _lib.orc_vae_encode.argtypes = [P(f), C.c_int, C.c_int, C.c_int, P(f), C.c_int, C.c_int, P(d), P(d)]
        _lib.orc_vae_set_threads.argtypes = [C.c_int]
        _lib.orc_qp_trace.argtypes = [C.c_void_p, C.c_int]
    return _lib


def _p(a, t):
    return None if a is None else a.ctypes.data_as(C.POINTER(t))


class Net:
    """A network held as flat fp32 params in torch order (weights.param_shapes)."""

    def __init__(self, spec, params):
        from sdf_nmpc_amd import weights as W
        self.spec = spec
        self.flat = np.ascontiguousarray(np.concatenate([params[k].ravel() for k, _ in spec.param_shapes()]),
                                         dtype=np.float32)
        self.dirs = np.ascontiguousarray(W.embedding_dirs(spec.embed), dtype=np.float32)
        self.freqs = (2.0 ** np.arange(spec.nb_freqs)).astype(np.float32)
        n1, n2, n3, n4 = spec.layer_sizes
        self.cs = Spec(spec.size_latent, n1, n2, n3, n4, spec.nb_freqs, self.dirs.shape[1], spec.w0, spec.max_df)

    def f32(self, inp, nthreads=1, full_grad=True):
        inp = np.ascontiguousarray(inp, dtype=np.float32)
        n = inp.shape[0]
        df = np.empty(n, np.float32)
        g = np.empty_like(inp) if full_grad else None
        gp = np.empty((n, 3), np.float32)
        lib().orc_sdf_f32(C.byref(self.cs), _p(self.dirs, C.c_float), _p(self.freqs, C.c_float),
                          _p(self.flat, C.c_float), n, _p(inp, C.c_float), _p(df, C.c_float),
                          _p(g, C.c_float), _p(gp, C.c_float), nthreads)
        return df, gp, g

    def f64(self, inp):
        inp = np.ascontiguousarray(inp, dtype=np.float64)
        n = inp.shape[0]
        df = np.empty(n)
        g = np.empty_like(inp)
        gp = np.empty((n, 3))
        lib().orc_sdf_f64(C.byref(self.cs), _p(self.dirs, C.c_float), _p(self.freqs, C.c_float),
                          _p(self.flat, C.c_float), n, _p(inp, C.c_double), _p(df, C.c_double),
                          _p(g, C.c_double), _p(gp, C.c_double))
        return df, gp, g


def quad_model(cfg, max_df=1.0):
    L = cfg.robot.limits
    R = np.asarray(cfg.sensor.B_R_C, dtype=np.float64).ravel()
    return Quad(L.gamma, L.roll, L.pitch, L.wz, 9.81, (C.c_double * 3)(*cfg.sensor.B_p_C),
                (C.c_double * 9)(*R), cfg.mpc.fov_const_offset, max_df)


def rk4(m, x, u, dt):
    x = np.ascontiguousarray(x, np.float64); u = np.ascontiguousarray(u, np.float64)
    xn = np.empty(10); AB = np.empty((14, 10))
    lib().orc_quad_rk4(C.byref(m), _p(x, C.c_double), _p(u, C.c_double), dt, _p(xn, C.c_double), _p(AB, C.c_double))
    return xn, AB.T.copy()  # AB.T: [10][14]


def cost(m, x, u, p):
    x = np.ascontiguousarray(x, np.float64); u = np.ascontiguousarray(u, np.float64)
    p = np.ascontiguousarray(p, np.float64)
    y = np.empty(11); Jy = np.empty((14, 11)); yN = np.empty(4); JyN = np.empty((10, 4))
    lib().orc_quad_cost(C.byref(m), _p(x, C.c_double), _p(u, C.c_double), _p(p, C.c_double), _p(y, C.c_double),
                        _p(Jy, C.c_double), _p(yN, C.c_double), _p(JyN, C.c_double))
    return y, Jy.T.copy(), yN, JyN.T.copy()


def constr(m, x, p, df, gdf):
    x = np.ascontiguousarray(x, np.float64); p = np.ascontiguousarray(p, np.float64)
    g = np.ascontiguousarray(gdf, np.float64)
    h = np.empty(3); Jh = np.empty((10, 3)); cpb = np.empty(3)
    lib().orc_quad_constr(C.byref(m), _p(x, C.c_double), _p(p, C.c_double), float(df), _p(g, C.c_double),
                          _p(h, C.c_double), _p(Jh, C.c_double), _p(cpb, C.c_double))
    return h, Jh.T.copy(), cpb


def term_extras(m, x, p, model):
    """Terminal extras of a model.Quad with recursive_feasibility / stability at one node (orc_quad_term):
    hE [6], JhE [6][10] (row-major), and with stability yN [5], JyN [5][10]."""
    x = np.ascontiguousarray(x, np.float64); p = np.ascontiguousarray(p, np.float64)
    poly = np.ascontiguousarray(np.concatenate([model.poly, [0.0]]), np.float64)
    hE = np.empty(6); JhE = np.empty((10, 6)); yN = np.empty(5); JyN = np.empty((10, 5))
    lib().orc_quad_term(C.byref(m), _p(x, C.c_double), _p(p, C.c_double), int(model.poly_deg), _p(poly, C.c_double),
                        int(model.rec_feas), int(model.stability), _p(hE, C.c_double), _p(JhE, C.c_double),
                        _p(yN, C.c_double), _p(JyN, C.c_double))
    return hE, JhE.T.copy(), yN, JyN.T.copy()


def shooting_grid(N, T, uniform=True, n_short=2, dt_short=0.01):
    nodes = np.empty(N + 1); dt = np.empty(N)
    rc = lib().orc_shooting_grid(N, T, int(uniform), n_short, dt_short, _p(nodes, C.c_double), _p(dt, C.c_double))
    if rc != 0:
        raise ValueError("bad grid arguments")
    return nodes, dt


def prng_uniform(seed, stream, n):
    out = np.empty(n)
    lib().orc_prng_uniform(seed, stream, n, _p(out, C.c_double))
    return out


def linearize_batch(m, net, x, u, p, dt, nthreads=1, model=None):
    """Whole preparation phase on the CPU; layouts match include/sdfnmpc.h outputs.  model (model.Quad)
    with recursive_feasibility / stability adds hE [B][6], JhE [B][10][6] and the nyN = 5 terminal
    residual (yN [B][5], JyN [B][10][5])."""
    out = _linearize_batch(m, net, x, u, p, dt, nthreads)
    if model is not None and (model.rec_feas or model.stability):
        B, N = out["xn"].shape[:2]
        out["hE"], out["JhE"] = np.zeros((B, 6)), np.zeros((B, 10, 6))
        yN5, JyN5 = np.zeros((B, 5)), np.zeros((B, 10, 5))
        for b in range(B):
            hE, JhE, y5, J5 = term_extras(m, x[b, N], p[b, N], model)
            out["hE"][b], out["JhE"][b] = hE, JhE.T
            yN5[b], JyN5[b] = y5, J5.T
        if model.stability:
            out["yN"], out["JyN"] = yN5, JyN5
    return out


def _linearize_batch(m, net, x, u, p, dt, nthreads=1):
    B, N1, _ = x.shape
    N = N1 - 1
    x = np.ascontiguousarray(x, np.float64); u = np.ascontiguousarray(u, np.float64)
    p = np.ascontiguousarray(p, np.float64); dt = np.ascontiguousarray(dt, np.float64)
    out = dict(xn=np.empty((B, N, 10)), AB=np.empty((B, N, 14, 10)), y=np.empty((B, N, 11)),
               Jy=np.empty((B, N, 14, 11)), yN=np.empty((B, 4)), JyN=np.empty((B, 10, 4)),
               h=np.empty((B, N1, 3)), Jh=np.empty((B, N1, 10, 3)), sdf=np.empty((B, N1, 4), np.float32))
    lib().orc_linearize_batch(C.byref(m), C.byref(net.cs), _p(net.dirs, C.c_float), _p(net.freqs, C.c_float),
                              _p(net.flat, C.c_float), B, N, p.shape[-1], _p(x, C.c_double), _p(u, C.c_double),
                              _p(p, C.c_double), _p(dt, C.c_double), *(_p(out[k], C.c_double) for k in
                              ("xn", "AB", "y", "Jy", "yN", "JyN", "h", "Jh")), _p(out["sdf"], C.c_float), nthreads)
    return out


QP_IN = ("xn", "AB", "y", "Jy", "yN", "JyN", "h", "Jh", "hE", "JhE", "x", "u", "x0", "yref", "W", "yNref", "WN")


# IPM starting point / step fraction of csrc/rti_qp.hip (QP_T0, QP_L0, QP_LC, QP_TAU_LO, QP_TAU_HI)
QP_START = dict(t0=0.5, l0=1.0, lc=0.5, tau_lo=0.995, tau_hi=0.995, seg=1, gk=0, ga=1.0, gd=0.1, gbmin=0.1, gbmax=10.0, ws=0)


def qp_ipm_batch(lin, prob, x0, model, lm=10.0, tol=1e-8, max_iter=100, cost_scaling=True, nthreads=1, lm_scaling=True,
                 start=None, du_ws=None):
    """Structured Riccati IPM (qp_ipm.c) over a batch: the CPU restatement of the feedback-phase QP.

    lin: linearisation outputs (xn, AB, y, Jy, yN, JyN, h, Jh) with a leading batch dimension;
    prob: x, u, yref, W, yN (reference), WN, dt.  Returns dict(dx, du, slack, iters, status, res).
    du_ws: primal warm start (B, N, 4), the previous QP's du (HPIPM's qp_solver_warm_start = 1, ocp.py:116).
    """
    B, N = lin["xn"].shape[0], lin["xn"].shape[1]
    arrs = dict(lin)
    arrs.setdefault("hE", np.zeros((B, 6)))
    arrs.setdefault("JhE", np.zeros((B, 10, 6)))
    arrs.update(x=prob["x"], u=prob["u"], x0=x0, yref=prob["yref"], W=prob["W"], yNref=prob["yN"], WN=prob["WN"])
    arrs = {k: np.ascontiguousarray(arrs[k], dtype=np.float64) for k in QP_IN}
    dt = np.ascontiguousarray(prob["dt"], dtype=np.float64)
    pad = lambda a, n, v=0.0: list(np.asarray(a, float)) + [v] * (n - len(a))
    h_cols = list(getattr(model, "h_cols", [0, 1, 2]))
    rows = getattr(model, "term_rows", [(c, -1, True, model.lh[i], model.uh[i], model.zl[i], model.Zl[i])
                                        for i, c in enumerate(h_cols)])
    cset = ([len(h_cols)] + pad(h_cols, 3) + [len(rows), sum(1 for r in rows if r[2])] + pad([r[0] for r in rows], 8, -1)
            + pad([r[1] for r in rows], 8, -1) + pad([r[3] for r in rows], 8) + pad([r[4] for r in rows], 8)
            + pad([r[5] for r in rows if r[2]], 3) + pad([r[6] for r in rows if r[2]], 3) + [arrs["WN"].shape[-1]]
            + [int(getattr(model, "nhs", 0))])
    opts = np.concatenate([model.lbu, model.ubu, pad(model.lh, 3), pad(model.uh, 3), pad(model.zl, 3), pad(model.Zl, 3),
                           [lm, tol, float(bool(lm_scaling))],
                           [v for v in {**QP_START, **(start or {}), "ws": float(du_ws is not None)}.values()],
                           cset]).astype(np.float64)
    du0 = np.zeros((B, N, 4)) if du_ws is None else np.array(du_ws, dtype=np.float64).reshape(B, N, 4)
    out = dict(dx=np.zeros((B, N + 1, 10)), du=du0, slack=np.zeros((B, N + 1, 3, 2)),
               iters=np.zeros(B, np.int32), status=np.zeros(B, np.int32), res=np.zeros((B, 4)))
    d = C.c_double
    ny = arrs["W"].shape[-1]
    lib().orc_qp_ipm_batch(B, N, *[_p(arrs[k], d) for k in QP_IN], _p(dt, d), _p(opts, d), max_iter,
                           int(bool(cost_scaling)), ny, _p(out["dx"], d), _p(out["du"], d), _p(out["slack"], d),
                           _p(out["iters"], C.c_int), _p(out["status"], C.c_int), _p(out["res"], d), nthreads)
    out["seg_dev"] = out["res"][:, 2].copy()  # segmented solve: gap between a segment's own x_b and the coupled one
    out["gondzio"] = out["res"][:, 3].astype(np.int32)  # Gondzio correctors kept
    out["res"] = np.ascontiguousarray(out["res"][:, :2])
    return out


def vae_preprocess(img, shape, clip_scale, yz=None):
    """vae.py:15-24 preprocessing of one raw image [Hi, Wi] (float32 or uint16) -> fp32 [H, W]."""
    img = np.ascontiguousarray(img)
    dtype = 1 if img.dtype == np.uint16 else 0
    if dtype == 0:
        img = np.ascontiguousarray(img, dtype=np.float32)
    H, W = shape
    out = np.empty((H, W), np.float32)
    yzp = None if yz is None else _p(np.ascontiguousarray(yz, dtype=np.float32), C.c_float)
    lib().orc_vae_preprocess(img.ctypes.data, dtype, img.shape[0], img.shape[1], H, W, float(clip_scale), yzp,
                             _p(out, C.c_float))
    return out


def vae_encode(pre, flat_params, L=128, bn=True, stage_sums=False, nthreads=0):
    """Encoder.forward (network/vae.py:39-43) in fp64 on preprocessed images [B, H, W]
    (nthreads: OpenMP threads of the conv layers, 0 = the OpenMP default)."""
    lib().orc_vae_set_threads(int(nthreads))
    pre = np.ascontiguousarray(pre, dtype=np.float32)
    if pre.ndim == 2:
        pre = pre[None]
    B, H, W = pre.shape
    lat = np.empty((B, L), np.float64)
    ss = np.empty(64 + 128 + 256 + 512 + 512, np.float64) if stage_sums else None
    flat = np.ascontiguousarray(flat_params, dtype=np.float32)
    lib().orc_vae_encode(_p(pre, C.c_float), B, H, W, _p(flat, C.c_float), L, int(bn), _p(lat, C.c_double),
                         None if ss is None else _p(ss, C.c_double))
    return (lat, ss) if stage_sums else lat
