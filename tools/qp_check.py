"""GPU QP vs the dense oracle on a few instances (diagnostic)."""
import os, sys, time
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O, qp_oracle as Q
from sdf_nmpc_amd import _lib, synth, weights as W
from sdf_nmpc_amd.config import Config
from sdf_nmpc_amd.model import Quad
cfg = Config(); model = Quad(cfg)
dev = torch.device("cuda:0")
ctx = _lib.Context(0, stream=torch.cuda.current_stream().cuda_stream)
net = _lib.Net.siren(ctx, 0)
for B, N in ((4, 20), (1024, 40)):
    prob = synth.make_problem(cfg, B, N, seed=5)
    rng = np.random.default_rng(1)
    x0 = prob["x"][:, 0] + rng.normal(0, 0.05, (B, 10))
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
         dict(x=prob["x"], u=prob["u"], p=prob["p"], dt=prob["dt"], x0=x0, yref=prob["yref"], W=prob["W"],
              yNref=prob["yN"], WN=prob["WN"]).items()}
    sh = dict(xn=(B, N, 10), AB=(B, N, 14, 10), y=(B, N, 11), Jy=(B, N, 14, 11), yN=(B, 4), JyN=(B, 10, 4),
              h=(B, N + 1, 3), Jh=(B, N + 1, 10, 3), dx=(B, N + 1, 10), du=(B, N, 4), slack=(B, N + 1, 3, 2), res=(B, 2))
    for k, s in sh.items():
        t[k] = torch.zeros(s, dtype=torch.float64, device=dev)
    t["status"] = torch.zeros(B, dtype=torch.int32, device=dev); t["iters"] = torch.zeros(B, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    _lib.linearize(ctx, net, _lib.quad_model(cfg), B, N, 145, t)
    opts = _lib.qp_opts(model, tol=1e-10)
    _lib.qp_solve(ctx, opts, B, N, t)
    ctx.synchronize()
    print(f"B={B} N={N}: status {np.bincount(t['status'].cpu().numpy())} iters min/max {t['iters'].min().item()}/{t['iters'].max().item()} res max {t['res'].max(0).values.cpu().numpy()}")
    lin = {k: t[k].cpu().numpy() for k in ("xn", "AB", "y", "Jy", "yN", "JyN", "h", "Jh")}
    for b in range(min(B, 3)):
        lb = {k: lin[k][b] for k in lin}
        q = Q.stage_qp(lb, prob["x"][b], prob["u"][b], x0[b], prob["yref"][b], prob["W"][b], prob["yN"][b], prob["WN"][b], prob["dt"], model, 10.0)
        ref = Q.solve_dense(q)
        du, dx = t["du"][b].cpu().numpy(), t["dx"][b].cpu().numpy()
        print(f"  inst {b}: oracle iters {ref['iters']}, |du-ref| {np.abs(du-ref['du']).max():.3e} |dx-ref| {np.abs(dx-ref['dx']).max():.3e} |du| {np.abs(ref['du']).max():.3e}")
    if B > 100:
        ctx.enable_timing(True); ctx.reset_stats()
        for _ in range(5):
            _lib.qp_solve(ctx, _lib.qp_opts(model), B, N, t)
        print("  qp ms", ctx.kernel_stats("rti_qp")[0] / 5, "iters", t["iters"].float().mean().item())
        ctx.enable_timing(False)
