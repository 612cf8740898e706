"""ctypes binding of libsdfnmpc.so (include/sdfnmpc.h).

This is the only way Python reaches the hot path: every compute call goes through the C ABI into
the HIP kernels.  There is deliberately no CPU fallback -- if the library is missing, or no gfx950
device is visible, construction raises.

Device buffers are plain device pointers (ints).  Callers normally pass torch CUDA(HIP) tensors,
which are used for allocation and streams only (``tensor.data_ptr()``).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(PKG_DIR, "lib")
# SDFNMPC_LIB: a diagnostic build of the same library (tools/build_variant.sh, tools/exp/*.sh)
LIB_PATH = os.environ.get("SDFNMPC_LIB") or os.path.join(LIB_DIR, "libsdfnmpc.so")
L4C_PATH = os.path.join(LIB_DIR, "libsdf_l4c.so")

# exported symbols declared in include/sdfnmpc.h (checked by tests/test_abi.py)
SYMBOLS = [
    "sdfnmpc_abi_version", "sdfnmpc_last_error", "sdfnmpc_ctx_create", "sdfnmpc_ctx_destroy",
    "sdfnmpc_ctx_set_stream", "sdfnmpc_ctx_use_null_stream", "sdfnmpc_ctx_stream", "sdfnmpc_ctx_synchronize", "sdfnmpc_ctx_set_tile_rows",
    "sdfnmpc_ctx_set_qp_kernel", "sdfnmpc_ctx_set_sdf_server", "sdfnmpc_ctx_sdf_server_stats", "sdfnmpc_ctx_qp_kernel", "sdfnmpc_ctx_qp_kernel_for", "sdfnmpc_qp_lds_bytes", "sdfnmpc_qp_capacity", "sdfnmpc_qp_capacity_for",
    "sdfnmpc_ctx_enable_timing", "sdfnmpc_ctx_kernel_stats", "sdfnmpc_ctx_reset_stats", "sdfnmpc_net_load",
    "sdfnmpc_net_load_file", "sdfnmpc_net_siren", "sdfnmpc_net_free", "sdfnmpc_net_max_df",
    "sdfnmpc_net_size_latent", "sdfnmpc_net_fingerprint", "sdfnmpc_sdf_eval", "sdfnmpc_sdf_eval_host",
    "sdfnmpc_linearize", "sdfnmpc_shooting_grid", "sdfnmpc_qp_solve", "sdfnmpc_rti_prepare", "sdfnmpc_qp_feedback",
    "sdfnmpc_rti_apply", "sdfnmpc_step_create", "sdfnmpc_step_launch", "sdfnmpc_step_destroy", "sdfnmpc_pack_refs",
    "sdfnmpc_vae_load", "sdfnmpc_vae_free", "sdfnmpc_vae_size_latent", "sdfnmpc_vae_encode",
    "sdfnmpc_ctx_device", "sdfnmpc_dev_alloc", "sdfnmpc_dev_free", "sdfnmpc_memcpy",
    "sdfnmpc_solver_create", "sdfnmpc_solver_destroy", "sdfnmpc_solver_field", "sdfnmpc_solver_upload",
    "sdfnmpc_solver_download", "sdfnmpc_solver_init", "sdfnmpc_solver_shift", "sdfnmpc_solver_step",
    "sdfnmpc_solver_wait",
]
L4C_SYMBOLS = [
    f"{p}sdf_l4c{s}" for p in ("", "jac_", "adj1_")
    for s in ("", "_n_in", "_n_out", "_sparsity_in", "_sparsity_out", "_work")
] + ["sdf_l4c_name_in", "sdf_l4c_name_out", "sdf_l4c_checkout", "sdf_l4c_release", "sdf_l4c_incref",
     "sdf_l4c_decref", "sdf_l4c_configure", "sdf_l4c_last_error"]


class SdfnmpcError(RuntimeError):
    pass


POLY_MAX, NHN_MAX = 84, 8  # SDFNMPC_POLY_MAX, SDFNMPC_NHN_MAX


class QuadModelC(C.Structure):
    _fields_ = [("gamma", C.c_double), ("roll", C.c_double), ("pitch", C.c_double), ("wz", C.c_double),
                ("g", C.c_double), ("B_p_C", C.c_double * 3), ("B_R_C", C.c_double * 9),
                ("fov_const_offset", C.c_double), ("rec_feas", C.c_int), ("stability", C.c_int),
                ("poly_deg", C.c_int), ("poly", C.c_double * POLY_MAX)]


LIN_PTRS = ("x", "u", "p", "dt", "xn", "AB", "y", "Jy", "yN", "JyN", "h", "Jh", "sdf")


class LinArgsC(C.Structure):
    _fields_ = [("B", C.c_int), ("N", C.c_int), ("np", C.c_int), ("latent_mode", C.c_int)] + [
        (n, C.c_void_p) for n in LIN_PTRS] + [("nyN", C.c_int), ("no_sdf", C.c_int), ("hE", C.c_void_p),
                                             ("JhE", C.c_void_p)]


class QpOptsC(C.Structure):
    _fields_ = [("lbu", C.c_double * 4), ("ubu", C.c_double * 4), ("lh", C.c_double * 3), ("uh", C.c_double * 3),
                ("zl", C.c_double * 3), ("Zl", C.c_double * 3), ("lm", C.c_double), ("cost_scaling", C.c_int),
                ("max_iter", C.c_int), ("tol", C.c_double), ("ny", C.c_int), ("lm_scaling", C.c_int),
                ("warm_start", C.c_int), ("nh", C.c_int), ("h_col", C.c_int * 3), ("nhN", C.c_int), ("nsN", C.c_int),
                ("hN_col", C.c_int * NHN_MAX), ("hE_col", C.c_int * NHN_MAX), ("lhN", C.c_double * NHN_MAX),
                ("uhN", C.c_double * NHN_MAX), ("zlN", C.c_double * 3), ("ZlN", C.c_double * 3), ("nyN", C.c_int),
                ("nhs", C.c_int)]


class RefOptsC(C.Structure):
    _fields_ = [("mode", C.c_int), ("yaw_mode", C.c_int), ("st_enable", C.c_int), ("st_mode", C.c_int),
                ("st_dang", C.c_double), ("align_off", C.c_double), ("dmin", C.c_double), ("vref", C.c_double),
                ("wzref", C.c_double), ("T", C.c_double), ("B_p_C", C.c_double * 3), ("B_R_C", C.c_double * 9)]


REF_IN = ("wp_p", "wp_q", "vw", "wrow", "latent", "W_p_Bo", "W_R_Bo", "flag")
REF_OUT = ("p", "yref", "W", "yNref", "WN")


class RefArgsC(C.Structure):
    _fields_ = [("B", C.c_int), ("N", C.c_int), ("np", C.c_int), ("ny", C.c_int), ("n_wp", C.c_int),
                ("L", C.c_int), ("x0", C.c_void_p), ("x0_stride", C.c_int)] + [
        (n, C.c_void_p) for n in REF_IN + REF_OUT] + [("nyN", C.c_int)]


QP_IN = ("xn", "AB", "y", "Jy", "yN", "JyN", "h", "Jh", "hE", "JhE", "x", "u", "x0", "yref", "W", "yNref", "WN", "dt")
QP_OUT = ("dx", "du", "slack", "status", "iters", "res")


class VaeOptsC(C.Structure):
    _fields_ = [("B", C.c_int), ("in_h", C.c_int), ("in_w", C.c_int), ("dtype", C.c_int), ("clip", C.c_float),
                ("yz", C.c_void_p)]


class SolverOptsC(C.Structure):
    _fields_ = [("B", C.c_int), ("N", C.c_int), ("np", C.c_int), ("ny", C.c_int), ("latent_mode", C.c_int),
                ("dt", C.POINTER(C.c_double)), ("model", QuadModelC), ("qp", QpOptsC)]


class QpArgsC(C.Structure):
    _fields_ = [("B", C.c_int), ("N", C.c_int)] + [(n, C.c_void_p) for n in QP_IN + QP_OUT]


_lib = None


def load():
    """Load libsdfnmpc.so (raises if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise SdfnmpcError(f"{LIB_PATH} not built: run `python -c 'import __graft_entry__ as g; g.build()'` "
                           "(the HIP extension is the only compute path)")
    lib = C.CDLL(LIB_PATH)
    vp, i, f, d, ll, sz = C.c_void_p, C.c_int, C.c_float, C.c_double, C.c_longlong, C.c_size_t
    P = C.POINTER
    sig = {
        "sdfnmpc_abi_version": (i, []),
        "sdfnmpc_last_error": (C.c_char_p, []),
        "sdfnmpc_ctx_create": (i, [i, vp, P(vp)]),
        "sdfnmpc_ctx_destroy": (None, [vp]),
        "sdfnmpc_ctx_set_stream": (i, [vp, vp]),
        "sdfnmpc_ctx_use_null_stream": (i, [vp]),
        "sdfnmpc_ctx_stream": (vp, [vp]),
        "sdfnmpc_ctx_synchronize": (i, [vp]),
        "sdfnmpc_ctx_set_tile_rows": (i, [vp, i]),
        "sdfnmpc_ctx_set_qp_kernel": (i, [vp, i]),
        "sdfnmpc_ctx_set_sdf_server": (i, [vp, i]),
        "sdfnmpc_ctx_sdf_server_stats": (i, [vp, P(d)]),
        "sdfnmpc_ctx_qp_kernel": (i, [vp, i, i]),
        "sdfnmpc_ctx_qp_kernel_for": (i, [vp, i, i, P(QpOptsC)]),
        "sdfnmpc_qp_lds_bytes": (C.c_longlong, [i]),
        "sdfnmpc_qp_capacity": (C.c_longlong, [vp, i]),
        "sdfnmpc_qp_capacity_for": (C.c_longlong, [vp, i, P(QpOptsC)]),
        "sdfnmpc_ctx_enable_timing": (i, [vp, i]),
        "sdfnmpc_ctx_kernel_stats": (i, [vp, C.c_char_p, P(d), P(ll)]),
        "sdfnmpc_ctx_reset_stats": (i, [vp]),
        "sdfnmpc_net_load": (i, [vp, vp, sz, P(vp)]),
        "sdfnmpc_net_load_file": (i, [vp, C.c_char_p, P(vp)]),
        "sdfnmpc_net_siren": (i, [vp, C.c_uint64, f, f, P(vp)]),
        "sdfnmpc_net_free": (None, [vp]),
        "sdfnmpc_net_max_df": (f, [vp]),
        "sdfnmpc_net_size_latent": (i, [vp]),
        "sdfnmpc_net_fingerprint": (C.c_uint64, [vp]),
        "sdfnmpc_sdf_eval": (i, [vp, vp, ll, vp, vp, i, vp, vp]),
        "sdfnmpc_sdf_eval_host": (i, [vp, vp, i, P(d), P(d), P(d)]),
        "sdfnmpc_linearize": (i, [vp, vp, P(QuadModelC), P(LinArgsC)]),
        "sdfnmpc_shooting_grid": (i, [i, d, i, i, d, P(d), P(d)]),
        "sdfnmpc_qp_solve": (i, [vp, P(QpOptsC), P(QpArgsC)]),
        "sdfnmpc_rti_prepare": (i, [vp, vp, P(QuadModelC), P(LinArgsC), P(QpOptsC), P(QpArgsC)]),
        "sdfnmpc_qp_feedback": (i, [vp, P(QpOptsC), P(QpArgsC)]),
        "sdfnmpc_rti_apply": (i, [vp, i, i, vp, vp, vp, vp, vp, vp]),
        "sdfnmpc_step_create": (i, [vp, vp, P(QuadModelC), P(LinArgsC), P(QpOptsC), P(QpArgsC), vp, vp, P(vp)]),
        "sdfnmpc_step_launch": (i, [vp, vp]),
        "sdfnmpc_step_destroy": (None, [vp]),
        "sdfnmpc_pack_refs": (i, [vp, P(RefOptsC), P(RefArgsC)]),
        "sdfnmpc_vae_load": (i, [vp, vp, sz, P(vp)]),
        "sdfnmpc_vae_free": (None, [vp]),
        "sdfnmpc_vae_size_latent": (i, [vp]),
        "sdfnmpc_vae_encode": (i, [vp, vp, P(VaeOptsC), vp, vp, vp]),
        "sdfnmpc_ctx_device": (i, [vp]),
        "sdfnmpc_dev_alloc": (i, [vp, sz, P(vp)]),
        "sdfnmpc_dev_free": (None, [vp, vp]),
        "sdfnmpc_memcpy": (i, [vp, vp, vp, sz, i]),
        "sdfnmpc_solver_create": (i, [vp, vp, P(SolverOptsC), P(vp)]),
        "sdfnmpc_solver_destroy": (None, [vp]),
        "sdfnmpc_solver_field": (i, [vp, C.c_char_p, P(vp), P(i), P(i)]),
        "sdfnmpc_solver_upload": (i, [vp, C.c_char_p, i, i, vp, vp]),
        "sdfnmpc_solver_download": (i, [vp, C.c_char_p, vp]),
        "sdfnmpc_solver_init": (i, [vp, vp, vp]),
        "sdfnmpc_solver_shift": (i, [vp, i]),
        "sdfnmpc_solver_step": (i, [vp]),
        "sdfnmpc_solver_wait": (i, [vp, vp, vp, vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    if lib.sdfnmpc_abi_version() != 6:
        raise SdfnmpcError("libsdfnmpc.so ABI version mismatch")
    _lib = lib
    return lib


def l4c_path() -> str:
    """Path of the CasADi external-function shim (include/sdf_l4c.h); raises if it has not been built."""
    if not os.path.exists(L4C_PATH):
        raise SdfnmpcError(f"{L4C_PATH} not built")
    return L4C_PATH


def _check(rc):
    if rc != 0:
        raise SdfnmpcError(f"sdfnmpc error {rc}: {load().sdfnmpc_last_error().decode()}")


def _ptr(t):
    if t is None:
        return None
    if isinstance(t, int):
        return t
    return t.data_ptr()


def sync_producer(a):
    """A torch CUDA tensor handed to a kernel of ours (which runs on a context stream, not torch's): wait
    until torch's current stream on its device -- where a producing kernel or non_blocking copy was queued --
    has finished.  DeviceArray / FieldView / host arrays need nothing.  torch is imported only here."""
    if type(a).__module__.split(".")[0] == "torch" and getattr(a, "is_cuda", False):
        import torch
        torch.cuda.current_stream(a.device).synchronize()
    return a


class Context:
    """One HIP device + stream (sdfnmpc_ctx)."""

    def __init__(self, device: int = 0, stream=None, tile_rows: int = 32):
        """stream: None -> a private non-blocking stream; a HIP stream handle (int) -> that stream, where
        0 is the legacy null stream (PyTorch's default stream), so the kernels are ordered with torch's."""
        lib = load()
        h = C.c_void_p()
        _check(lib.sdfnmpc_ctx_create(device, stream or None, C.byref(h)))
        self.h = h
        if stream is not None and int(stream) == 0:
            _check(lib.sdfnmpc_ctx_use_null_stream(h))
        self.device = device
        self.set_tile_rows(tile_rows)

    def set_tile_rows(self, rows: int):
        _check(load().sdfnmpc_ctx_set_tile_rows(self.h, rows))

    QP_KERNELS = {"auto": 0, "serial": 1, "segmented": 2}

    def set_qp_kernel(self, kind: str):
        """'auto' (segmented for B <= 256 -- 512 from N = 48 -- at 36 <= N <= 63, else serial), 'serial' or
        'segmented' (include/sdfnmpc.h)."""
        _check(load().sdfnmpc_ctx_set_qp_kernel(self.h, self.QP_KERNELS[kind]))

    def set_sdf_server(self, on: bool):
        """Serve the host-pointer SDF path (sdf_eval_host, <= 16 rows) from the resident server kernel
        (default) or with one launch per call (include/sdfnmpc.h)."""
        _check(load().sdfnmpc_ctx_set_sdf_server(self.h, int(bool(on))))

    def sdf_server_stats(self) -> dict:
        """Mean microseconds per served request since the last call (diagnostics)."""
        o = (C.c_double * 18)()
        _check(load().sdfnmpc_ctx_sdf_server_stats(self.h, o))
        return {"stage_us": o[0], "eval_us": o[1], "wait_us": o[2], "requests": int(o[3]),
                "phases_us": [round(v, 2) for v in o[4:18]]}

    def qp_kernel(self, N: int, B: int, opts: "QpOptsC" = None) -> str:
        """The kernel a QP batch of B instances at horizon N runs ('serial' or 'segmented'); with opts: for that
        constraint set (sdfnmpc_ctx_qp_kernel_for)."""
        lib = load()
        k = lib.sdfnmpc_ctx_qp_kernel(self.h, N, B) if opts is None else lib.sdfnmpc_ctx_qp_kernel_for(self.h, N, B, C.byref(opts))
        return {1: "serial", 2: "segmented"}.get(k, "invalid")

    def qp_capacity(self, N: int, opts: "QpOptsC" = None) -> int:
        """Instances this device solves in one wave of QP workgroups at horizon N (sdfnmpc_qp_capacity; with
        opts: for that constraint set, sdfnmpc_qp_capacity_for)."""
        lib = load()
        n = int(lib.sdfnmpc_qp_capacity(self.h, N) if opts is None else lib.sdfnmpc_qp_capacity_for(self.h, N, C.byref(opts)))
        if n < 0:
            raise SdfnmpcError(f"sdfnmpc_qp_capacity: bad arguments (N={N})")
        return n

    def set_stream(self, stream):
        if stream is not None and int(stream) == 0:
            _check(load().sdfnmpc_ctx_use_null_stream(self.h))
        else:
            _check(load().sdfnmpc_ctx_set_stream(self.h, stream))

    def synchronize(self):
        _check(load().sdfnmpc_ctx_synchronize(self.h))

    @property
    def stream(self) -> int:
        return load().sdfnmpc_ctx_stream(self.h)

    @property
    def device_index(self) -> int:
        return int(load().sdfnmpc_ctx_device(self.h))

    def enable_timing(self, on=True):
        _check(load().sdfnmpc_ctx_enable_timing(self.h, int(on)))

    def kernel_stats(self, name: str):
        ms, n = C.c_double(), C.c_longlong()
        _check(load().sdfnmpc_ctx_kernel_stats(self.h, name.encode(), C.byref(ms), C.byref(n)))
        return ms.value, n.value

    def reset_stats(self):
        _check(load().sdfnmpc_ctx_reset_stats(self.h))

    def close(self):
        if getattr(self, "h", None):
            load().sdfnmpc_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Net:
    """Device-resident packed NeuralDF (sdfnmpc_net)."""

    def __init__(self, ctx: Context, handle):
        self.ctx, self.h = ctx, handle

    @classmethod
    def siren(cls, ctx: Context, seed: int = 0, weight_gain: float = 1.0, bias_gain: float = 0.0):
        h = C.c_void_p()
        _check(load().sdfnmpc_net_siren(ctx.h, seed, weight_gain, bias_gain, C.byref(h)))
        return cls(ctx, h)

    @classmethod
    def from_blob(cls, ctx: Context, blob: bytes):
        h = C.c_void_p()
        buf = C.create_string_buffer(blob, len(blob))
        _check(load().sdfnmpc_net_load(ctx.h, buf, len(blob), C.byref(h)))
        return cls(ctx, h)

    @classmethod
    def from_file(cls, ctx: Context, path: str):
        h = C.c_void_p()
        _check(load().sdfnmpc_net_load_file(ctx.h, path.encode(), C.byref(h)))
        return cls(ctx, h)

    @property
    def max_df(self) -> float:
        return float(load().sdfnmpc_net_max_df(self.h))

    @property
    def size_latent(self) -> int:
        return int(load().sdfnmpc_net_size_latent(self.h))

    @property
    def fingerprint(self) -> int:
        return int(load().sdfnmpc_net_fingerprint(self.h))

    def eval(self, rows, pos4, latent, rows_per_inst, out4, grad_latent=None):
        """Device-pointer SDF evaluation (asynchronous on the context stream)."""
        _check(load().sdfnmpc_sdf_eval(self.ctx.h, self.h, rows, _ptr(pos4), _ptr(latent), rows_per_inst,
                                       _ptr(out4), _ptr(grad_latent)))

    def eval_host(self, inp: np.ndarray, want_grad=True):
        """Host-pointer synchronous evaluation: inp [rows, 3 + L] fp64 -> (df [rows], grad [rows, 3 + L])
        (L = size_latent, 128 for the deployed net: the 131 of jac_sdf_l4c)."""
        inp = np.ascontiguousarray(inp, dtype=np.float64)
        rows = inp.shape[0]
        df = np.empty(rows)
        g = np.empty_like(inp) if want_grad else None
        P = C.POINTER(C.c_double)
        _check(load().sdfnmpc_sdf_eval_host(self.ctx.h, self.h, rows, inp.ctypes.data_as(P), df.ctypes.data_as(P),
                                            None if g is None else g.ctypes.data_as(P)))
        return df, g

    def close(self):
        if getattr(self, "h", None):
            load().sdfnmpc_net_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def quad_model(cfg, model=None) -> QuadModelC:
    """Model constants of a config; ``model`` (model.Quad) adds the terminal extras of its flags
    (recursive_feasibility: the braking polynomial; stability)."""
    lim = cfg.robot.limits
    R = np.asarray(cfg.sensor.B_R_C, dtype=np.float64).ravel()
    m = QuadModelC(float(lim.gamma), float(lim.roll), float(lim.pitch), float(lim.wz), 9.81,
                   (C.c_double * 3)(*[float(v) for v in cfg.sensor.B_p_C]), (C.c_double * 9)(*R),
                   float(cfg.mpc.fov_const_offset))
    if model is not None:
        m.rec_feas, m.stability = int(model.rec_feas), int(model.stability)
        m.poly_deg = int(model.poly_deg)
        for i, c in enumerate(model.poly):
            m.poly[i] = float(c)
    return m


def lin_args(B: int, N: int, np_: int, bufs: dict, latent_mode=0, nyN=4, no_sdf=False) -> LinArgsC:
    return LinArgsC(B, N, np_, latent_mode, *[_ptr(bufs.get(k)) for k in LIN_PTRS], int(nyN), int(bool(no_sdf)),
                    _ptr(bufs.get("hE")), _ptr(bufs.get("JhE")))


def linearize(ctx: Context, net, model: QuadModelC, B: int, N: int, np_: int, bufs: dict, latent_mode=0, nyN=4,
              no_sdf=False):
    """Enqueue the batched preparation phase.  bufs: device tensors named as sdfnmpc_lin_args (net may be
    None with no_sdf)."""
    a = lin_args(B, N, np_, bufs, latent_mode, nyN, no_sdf)
    _check(load().sdfnmpc_linearize(ctx.h, None if net is None else net.h, C.byref(model), C.byref(a)))


def qp_opts(model, lm=10.0, cost_scaling=True, max_iter=100, tol=1e-8, lm_scaling=True, warm_start=False) -> QpOptsC:
    """QP data of the 'att' model (model.Quad: bounds, the constraint set of its flags) + solver options
    (ocp.py:113-120 defaults).  lm_scaling: the Levenberg-Marquardt term is lm dt_k at stages k < N and lm at
    N (acados' Ts-scaled term).  warm_start: HPIPM's primal warm start (ocp.py:116) -- the IPM starts from
    the du buffer's entry values."""
    v = lambda a, n: (C.c_double * n)(*([float(x) for x in a] + [0.0] * (n - len(a))))
    iv = lambda a, n: (C.c_int * n)(*([int(x) for x in a] + [-1] * (n - len(a))))
    rows = model.term_rows
    return QpOptsC(v(model.lbu, 4), v(model.ubu, 4), v(model.lh, 3), v(model.uh, 3), v(model.zl, 3),
                   v(model.Zl, 3), float(lm), int(bool(cost_scaling)), int(max_iter), float(tol), int(model.ny),
                   int(bool(lm_scaling)), int(bool(warm_start)), int(model.nh), iv(model.h_cols, 3), int(model.nhN),
                   int(model.nsN), iv([r[0] for r in rows], NHN_MAX), iv([r[1] for r in rows], NHN_MAX),
                   v(model.lhN, NHN_MAX), v(model.uhN, NHN_MAX), v(model.zlN, 3), v(model.ZlN, 3), int(model.nyN),
                   int(getattr(model, "nhs", 0)))


def qp_solve(ctx: Context, opts: QpOptsC, B: int, N: int, bufs: dict):
    """Enqueue the batched feedback-phase QP.  bufs: device tensors named as sdfnmpc_qp_args."""
    a = QpArgsC(B, N, *[_ptr(bufs.get(k)) for k in QP_IN + QP_OUT])
    _check(load().sdfnmpc_qp_solve(ctx.h, C.byref(opts), C.byref(a)))


def rti_prepare(ctx: Context, net, model: QuadModelC, opts: QpOptsC, B: int, N: int, np_: int, bufs: dict,
                latent_mode=0, no_sdf=False):
    """Enqueue the RTI preparation phase acados-style: linearisation + the QP's stage records (everything
    but x0).  bufs: device tensors named as sdfnmpc_lin_args and sdfnmpc_qp_args."""
    la = lin_args(B, N, np_, bufs, latent_mode, opts.nyN, no_sdf)
    qa = QpArgsC(B, N, *[_ptr(bufs.get(k)) for k in QP_IN + QP_OUT])
    _check(load().sdfnmpc_rti_prepare(ctx.h, None if net is None else net.h, C.byref(model), C.byref(la),
                                      C.byref(opts), C.byref(qa)))


def qp_feedback(ctx: Context, opts: QpOptsC, B: int, N: int, bufs: dict):
    """Enqueue the RTI feedback phase: the IPM on the records of the last rti_prepare."""
    a = QpArgsC(B, N, *[_ptr(bufs.get(k)) for k in QP_IN + QP_OUT])
    _check(load().sdfnmpc_qp_feedback(ctx.h, C.byref(opts), C.byref(a)))


class RtiStep:
    """One SQP-RTI control step (rti_prepare + qp_feedback + rti_apply) over buffers bound once: the ctypes
    argument blocks are built here, not per call (the per-call form spends ~15 us of Python per phase
    building them, on the B = 1 latency path).  graph=True: the step is captured into a HIP graph
    (sdfnmpc_step_create, which runs it once eagerly) and a call is one graph launch.  The bound tensors
    must stay alive and at the same addresses."""

    def __init__(self, ctx: Context, net, model: QuadModelC, opts: QpOptsC, B: int, N: int, np_: int, bufs: dict,
                 u0=None, latent_mode=0, no_sdf=False, graph=False):
        self._lib = load()
        self._ctx, self._net = ctx.h, None if net is None else net.h
        self._model, self._opts, self._B, self._N = model, opts, B, N
        self._la = lin_args(B, N, np_, bufs, latent_mode, opts.nyN, no_sdf)
        self._qa = QpArgsC(B, N, *[_ptr(bufs.get(k)) for k in QP_IN + QP_OUT])
        self._apply = (_ptr(bufs["x"]), _ptr(bufs["u"]), _ptr(bufs["dx"]), _ptr(bufs["du"]), _ptr(u0),
                       _ptr(bufs.get("status")))
        self._keep = (bufs, u0, ctx, net)
        self._step = None
        if graph:
            for t in list(bufs.values()) + [u0]:
                sync_producer(t)
            h = C.c_void_p()
            _check(self._lib.sdfnmpc_step_create(self._ctx, self._net, C.byref(model), C.byref(self._la),
                                                 C.byref(opts), C.byref(self._qa), self._apply[4], self._apply[5],
                                                 C.byref(h)))
            self._step = h

    def __call__(self):
        lib, r = self._lib, C.byref
        if self._step is not None:
            _check(lib.sdfnmpc_step_launch(self._ctx, self._step))
            return
        _check(lib.sdfnmpc_rti_prepare(self._ctx, self._net, r(self._model), r(self._la), r(self._opts), r(self._qa)))
        _check(lib.sdfnmpc_qp_feedback(self._ctx, r(self._opts), r(self._qa)))
        _check(lib.sdfnmpc_rti_apply(self._ctx, self._B, self._N, *self._apply))

    def __del__(self):
        if getattr(self, "_step", None) is not None:
            self._lib.sdfnmpc_step_destroy(self._step)
            self._step = None


def rti_apply(ctx: Context, B: int, N: int, x, u, dx, du, u0=None, status=None):
    """x += dx, u += du, u0 = u[:, 0]; instances whose QP status is >= 2 (numerical failure) keep x, u."""
    _check(load().sdfnmpc_rti_apply(ctx.h, B, N, _ptr(x), _ptr(u), _ptr(dx), _ptr(du), _ptr(u0), _ptr(status)))


def shooting_grid(N: int, T: float, uniform=True, nb_short_nodes=2, dt_short=0.01):
    nodes, dt = np.empty(N + 1), np.empty(N)
    P = C.POINTER(C.c_double)
    _check(load().sdfnmpc_shooting_grid(N, T, int(bool(uniform)), nb_short_nodes, dt_short, nodes.ctypes.data_as(P),
                                        dt.ctypes.data_as(P)))
    return nodes, dt


def ref_opts(cfg, mode: int) -> RefOptsC:
    """RefGen knobs of a config (ref_gen.py) for sdfnmpc_pack_refs; mode 0 waypoints, 1 joystick, 2 from_x0,
    -1 latent / flag only."""
    r = cfg.ref
    ym = str(r.yaw_mode)
    yaw_mode = {"ref": 1, "align": 2, "curent": 3}.get(ym, 0)  # 'current' / 'zero': identity (ref_gen.py:12, sic)
    st_mode = {"topic": 1, "align": 2}.get(ym, 0)
    v = lambda a, n: (C.c_double * n)(*[float(x) for x in np.asarray(a, dtype=float).ravel()])
    return RefOptsC(int(mode), yaw_mode, int(bool(r.stop_and_turn.enable)), st_mode, float(r.stop_and_turn.dang_min),
                    float(r.align_yaw_offset), float(r.yaw_align_dmin), float(r.vref), float(r.wzref), float(cfg.mpc.T),
                    v(cfg.sensor.B_p_C, 3), v(cfg.sensor.B_R_C, 9))


def pack_refs(ctx: Context, opts: RefOptsC, B: int, N: int, np_: int, ny: int, bufs: dict, n_wp: int = 0, L: int = 0,
              nyN: int = 4):
    """Enqueue sdfnmpc_pack_refs.  bufs: device tensors named as sdfnmpc_ref_args (x0 [B][stride])."""
    x0 = bufs.get("x0")
    stride = int(x0.shape[-1]) if x0 is not None else 0
    a = RefArgsC(B, N, np_, ny, n_wp, L, _ptr(x0), stride, *[_ptr(bufs.get(k)) for k in REF_IN + REF_OUT], int(nyN))
    _check(load().sdfnmpc_pack_refs(ctx.h, C.byref(opts), C.byref(a)))


class Vae:
    """Device-resident VAE encoder (sdfnmpc_vae) from a `.vaew` blob (sdf_nmpc_amd.vae.pack)."""

    def __init__(self, ctx: Context, blob: bytes, batch: int = 1):
        self.ctx = ctx
        h = C.c_void_p()
        buf = C.create_string_buffer(blob, len(blob))
        _check(load().sdfnmpc_vae_load(ctx.h, buf, len(blob), C.byref(h)))
        self.h = h
        self.batch = batch

    @property
    def size_latent(self) -> int:
        return int(load().sdfnmpc_vae_size_latent(self.h))

    def close(self):
        if getattr(self, "h", None):
            load().sdfnmpc_vae_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def vae_opts(cfg, clip: float) -> VaeOptsC:
    """Per-call options from the config (sensor.dmax / mm_resolution, is_depth); B / size / dtype / yz per call."""
    o = VaeOptsC()
    o.clip = float(clip)
    o.dtype = 0
    return o


def vae_encode(ctx: Context, vae: Vae, opts: VaeOptsC, img, yz, latent, latent64=None, depth2range=True):
    """Enqueue sdfnmpc_vae_encode: img device array [B][H][W] (float32 or uint16; a DeviceArray or a torch
    tensor), latent [B][L] fp32."""
    o = VaeOptsC(int(img.shape[0]), int(img.shape[-2]), int(img.shape[-1]), 1 if "uint16" in str(img.dtype) else 0,
                 float(opts.clip), _ptr(yz) if depth2range else None)
    _check(load().sdfnmpc_vae_encode(ctx.h, vae.h, C.byref(o), _ptr(img), _ptr(latent), _ptr(latent64)))


class DeviceArray:
    """A device buffer on a context, with numpy-style shape / dtype (the tensor-free way to hand device
    inputs to the entry points).  ``data_ptr()`` makes it usable wherever a torch tensor is accepted."""

    def __init__(self, ctx: Context, shape, dtype=np.float64):
        self.ctx, self.shape, self.dtype = ctx, tuple(int(v) for v in shape), np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape, dtype=np.int64)) * self.dtype.itemsize
        p = C.c_void_p()
        _check(load().sdfnmpc_dev_alloc(ctx.h, self.nbytes, C.byref(p)))
        self.ptr = p.value

    @classmethod
    def from_numpy(cls, ctx: Context, a, dtype=None):
        a = np.ascontiguousarray(a, dtype=dtype)
        d = cls(ctx, a.shape, a.dtype)
        d.upload(a)
        return d

    def data_ptr(self) -> int:
        return self.ptr

    def upload(self, a):
        a = np.ascontiguousarray(a, dtype=self.dtype)
        if a.nbytes != self.nbytes:
            raise ValueError(f"upload of {a.nbytes} bytes into a {self.nbytes}-byte device array")
        _check(load().sdfnmpc_memcpy(self.ctx.h, self.ptr, a.ctypes.data, self.nbytes, 1))

    def numpy(self) -> np.ndarray:
        out = np.empty(self.shape, self.dtype)
        _check(load().sdfnmpc_memcpy(self.ctx.h, out.ctypes.data, self.ptr, self.nbytes, 2))
        return out

    def close(self):
        if getattr(self, "ptr", None):
            load().sdfnmpc_dev_free(self.ctx.h, self.ptr)
            self.ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class FieldView:
    """A solver field's device memory (borrowed: owned by the Solver) -- data_ptr() / shape for the
    lower-level entry points that write it in place (sdfnmpc_pack_refs, sdfnmpc_vae_encode)."""

    def __init__(self, ptr: int, shape, dtype, ctx: "Context" = None):
        self.ptr, self.shape, self.dtype, self.ctx = ptr, tuple(shape), np.dtype(dtype), ctx

    def data_ptr(self) -> int:
        return self.ptr

    @property
    def device(self) -> int:
        if self.ctx is None:
            raise SdfnmpcError("FieldView without a context: its device is unknown")
        return int(self.ctx.device)

    def numpy(self) -> np.ndarray:
        """Host copy (synchronous, ordered on the owning context's stream)."""
        if self.ctx is None:
            raise SdfnmpcError("FieldView without a context cannot be downloaded")
        out = np.empty(self.shape, self.dtype)
        _check(load().sdfnmpc_memcpy(self.ctx.h, out.ctypes.data, self.ptr, out.nbytes, 2))
        return out


class Solver:
    """sdfnmpc_solver: B instances' SQP-RTI workspace on one context, driven with host arrays."""

    INT_FIELDS = ("status", "iters")

    def __init__(self, ctx: Context, net, model: QuadModelC, qp: QpOptsC, B: int, N: int, np_: int, ny: int,
                 dt, latent_mode: int = 0):
        """net may be None when the constraint set and the cost never read the SDF (model.Quad.need_sdf)."""
        self.ctx, self.net, self.B, self.N, self.np, self.ny = ctx, net, int(B), int(N), int(np_), int(ny)
        self._dt = np.ascontiguousarray(dt, dtype=np.float64)
        o = SolverOptsC(self.B, self.N, self.np, self.ny, int(latent_mode),
                        self._dt.ctypes.data_as(C.POINTER(C.c_double)), model, qp)
        h = C.c_void_p()
        _check(load().sdfnmpc_solver_create(ctx.h, None if net is None else net.h, C.byref(o), C.byref(h)))
        self.h = h
        self._shapes = {}
        self.u0 = np.zeros((self.B, 4))
        self.status = np.zeros(self.B, np.int32)
        self.iters = np.zeros(self.B, np.int32)

    def shape(self, name: str):
        shp = self._shapes.get(name)  # fixed at creation: cached (the per-step upload path asks for it)
        if shp is None:
            nodes, width = C.c_int(), C.c_int()
            _check(load().sdfnmpc_solver_field(self.h, name.encode(), None, C.byref(nodes), C.byref(width)))
            shp = self._shapes[name] = (self.B, nodes.value, width.value)
        return shp

    def field(self, name: str) -> FieldView:
        p, nodes, width = C.c_void_p(), C.c_int(), C.c_int()
        _check(load().sdfnmpc_solver_field(self.h, name.encode(), C.byref(p), C.byref(nodes), C.byref(width)))
        return FieldView(p.value, (self.B, nodes.value, width.value), np.int32 if name in self.INT_FIELDS else np.float64,
                         self.ctx)

    def upload(self, name: str, host, col0: int = 0, ncol=None, mask=None):
        """host: the full [B][nodes][width] mirror (or anything broadcastable to it); mask [B][nodes] of rows."""
        shp = self.shape(name)
        a = np.ascontiguousarray(np.broadcast_to(np.asarray(host, dtype=np.float64), shp))
        ncol = shp[2] - col0 if ncol is None else int(ncol)
        m = None
        if mask is not None:
            m = np.ascontiguousarray(np.broadcast_to(np.asarray(mask, dtype=bool), shp[:2]), dtype=np.uint8)
            if not m.any():
                return
        _check(load().sdfnmpc_solver_upload(self.h, name.encode(), int(col0), ncol,
                                             None if m is None else m.ctypes.data, a.ctypes.data))

    def download(self, name: str) -> np.ndarray:
        shp = self.shape(name)
        out = np.empty(shp, np.int32 if name in self.INT_FIELDS else np.float64)
        _check(load().sdfnmpc_solver_download(self.h, name.encode(), out.ctypes.data))
        return out

    def init(self, x0, u_init):
        x0 = np.ascontiguousarray(np.broadcast_to(np.asarray(x0, dtype=np.float64), (self.B, 10)))
        u = np.ascontiguousarray(u_init, dtype=np.float64)
        _check(load().sdfnmpc_solver_init(self.h, x0.ctypes.data, u.ctypes.data))

    def shift(self, k: int):
        _check(load().sdfnmpc_solver_shift(self.h, int(k)))

    def step(self):
        _check(load().sdfnmpc_solver_step(self.h))

    def wait(self):
        _check(load().sdfnmpc_solver_wait(self.h, self.u0.ctypes.data, self.status.ctypes.data, self.iters.ctypes.data))
        return self.u0

    def close(self):
        if getattr(self, "h", None):
            load().sdfnmpc_solver_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
