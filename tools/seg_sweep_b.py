"""rti_qp time of the serial and segmented kernels over the batch size (N = 40, HIP events; diagnostic)."""
import os, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
from sdf_nmpc_amd import _lib, synth
from sdf_nmpc_amd.config import Config
if os.environ.get("SDFNMPC_LIB"):  # a diagnostic build (tools/build_variant.sh)
    _lib.LIB_PATH = os.environ["SDFNMPC_LIB"]
from sdf_nmpc_amd.model import Quad
cfg = Config(); model = Quad(cfg)
dev = torch.device("cuda:0")
ctx = _lib.Context(0)
net = _lib.Net.siren(ctx, 0)
N = int(os.environ.get("N", 40))
for B in [int(v) for v in (sys.argv[1:] or ["1", "8", "64", "256", "1024"])]:
    prob = synth.make_problem(cfg, B, N, seed=5)
    x0 = prob["x"][:, 0] + np.random.default_rng(6).normal(0, 0.05, (B, 10))
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
         dict(x=prob["x"], u=prob["u"], p=prob["p"], dt=prob["dt"], x0=x0, yref=prob["yref"], W=prob["W"],
              yNref=prob["yN"], WN=prob["WN"]).items()}
    sh = dict(xn=(B, N, 10), AB=(B, N, 14, 10), y=(B, N, 11), Jy=(B, N, 14, 11), yN=(B, 4), JyN=(B, 10, 4),
              h=(B, N + 1, 3), Jh=(B, N + 1, 10, 3), dx=(B, N + 1, 10), du=(B, N, 4), slack=(B, N + 1, 3, 2), res=(B, 2))
    for k, s in sh.items():
        t[k] = torch.zeros(s, dtype=torch.float64, device=dev)
    t["status"] = torch.zeros(B, dtype=torch.int32, device=dev)
    t["iters"] = torch.zeros(B, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    _lib.linearize(ctx, net, _lib.quad_model(cfg), B, N, prob["p"].shape[-1], t)
    ctx.synchronize()
    row = f"B={B:5d}"
    for kind in ("serial", "segmented"):
        ctx.set_qp_kernel(kind)
        _lib.qp_solve(ctx, _lib.qp_opts(model), B, N, t)
        ctx.enable_timing(True); ctx.reset_stats()
        for _ in range(10):
            _lib.qp_solve(ctx, _lib.qp_opts(model), B, N, t)
        ctx.synchronize()
        row += f"  {kind} {ctx.kernel_stats('rti_qp')[0] / 10:.3f} ms (iters max {int(t['iters'].max())})"
        ctx.enable_timing(False)
    print(row, flush=True)
