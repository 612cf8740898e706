"""B = 1 step (rti_prepare + qp_feedback + rti_apply at N, bench.py's p50_step_ms_b1 leg) for a kernel trace:
per-kernel GPU durations and the gaps between consecutive kernels of one step (diagnostic)."""
import os, sys, time
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sdf_nmpc_amd import _lib, synth
from sdf_nmpc_amd.config import Config
from sdf_nmpc_amd.model import Quad
N = int(os.environ.get("N", 40))
cfg = Config(mpc__N=N)
dev = torch.device("cuda:0")
ctx = _lib.Context(0, stream=torch.cuda.current_stream().cuda_stream)
net = _lib.Net.siren(ctx, 0)
model = Quad(cfg)
prob = synth.make_problem(cfg, 1, N, seed=0)
b1 = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
      dict(x=prob["x"], u=prob["u"], p=prob["p"], dt=prob["dt"], x0=prob["x"][:, 0], yref=prob["yref"], W=prob["W"],
           yNref=prob["yN"], WN=prob["WN"]).items()}
for k, s in dict(xn=(1, N, 10), AB=(1, N, 14, 10), y=(1, N, 11), Jy=(1, N, 14, 11), yN=(1, 4), JyN=(1, 10, 4),
                 h=(1, N + 1, 3), Jh=(1, N + 1, 10, 3), hE=(1, 6), JhE=(1, 10, 6), dx=(1, N + 1, 10), du=(1, N, 4),
                 res=(1, 2)).items():
    b1[k] = torch.zeros(s, dtype=torch.float64, device=dev)
b1["status"] = torch.zeros(1, dtype=torch.int32, device=dev)
b1["iters"] = torch.zeros(1, dtype=torch.int32, device=dev)
qopts = _lib.qp_opts(model, tol=1e-8)
cmodel = _lib.quad_model(cfg, model)
x1, u1, u0 = b1["x"].clone(), b1["u"].clone(), torch.empty((1, 4), dtype=torch.float64, device=dev)
np_ = prob["p"].shape[-1]
print("QP kernel:", ctx.qp_kernel(N, 1))

rti1 = (_lib.RtiStep(ctx, net, cmodel, qopts, 1, N, np_, b1, u0=u0, graph=bool(os.environ.get("B1_GRAPH")))
        if hasattr(_lib, "RtiStep") else None)


def step():
    b1["x"].copy_(x1)
    b1["u"].copy_(u1)
    if rti1 is not None and not os.environ.get("B1_PERCALL"):
        rti1()
        return
    _lib.rti_prepare(ctx, net, cmodel, qopts, 1, N, np_, b1)
    _lib.qp_feedback(ctx, qopts, 1, N, b1)
    _lib.rti_apply(ctx, 1, N, b1["x"], b1["u"], b1["dx"], b1["du"], u0)

for _ in range(10):
    step()
lat = []
for _ in range(int(os.environ.get("STEPS", 50))):
    torch.cuda.synchronize()
    t = time.perf_counter()
    step()
    torch.cuda.synchronize()
    lat.append((time.perf_counter() - t) * 1e3)
print(f"B=1 N={N}: p50 {np.median(lat):.3f} ms, min {np.min(lat):.3f} ms, iters {int(b1['iters'][0])}")

if os.environ.get("B1_HOSTTIME"):  # host time of each call of the (per-call) step, GPU running behind
    la = _lib.lin_args(1, N, np_, b1, 0, qopts.nyN, False)
    qa = _lib.QpArgsC(1, N, *[_lib._ptr(b1.get(k)) for k in _lib.QP_IN + _lib.QP_OUT])
    lib = _lib.load()
    import ctypes as C
    ts = {k: [] for k in ("copies", "prepare", "feedback", "apply", "sync")}
    for _ in range(50):
        t0 = time.perf_counter()
        b1["x"].copy_(x1)
        b1["u"].copy_(u1)
        t1 = time.perf_counter()
        lib.sdfnmpc_rti_prepare(ctx.h, net.h, C.byref(cmodel), C.byref(la), C.byref(qopts), C.byref(qa))
        t2 = time.perf_counter()
        lib.sdfnmpc_qp_feedback(ctx.h, C.byref(qopts), C.byref(qa))
        t3 = time.perf_counter()
        lib.sdfnmpc_rti_apply(ctx.h, 1, N, b1["x"].data_ptr(), b1["u"].data_ptr(), b1["dx"].data_ptr(),
                              b1["du"].data_ptr(), u0.data_ptr(), b1["status"].data_ptr())
        t4 = time.perf_counter()
        torch.cuda.synchronize()
        t5 = time.perf_counter()
        for k, a, b in (("copies", t0, t1), ("prepare", t1, t2), ("feedback", t2, t3), ("apply", t3, t4), ("sync", t4, t5)):
            ts[k].append((b - a) * 1e6)
    print("host us (median):", {k: round(float(np.median(v)), 1) for k, v in ts.items()})
