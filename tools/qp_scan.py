"""QP kernel time per IPM iteration vs batch size (diagnostic).

The kernel waits for its slowest instance (one wavefront per instance), so the figure of merit is
kernel time / max iterations.  Small batches keep the stage/factor record stream L2-resident; a
flat per-iteration time across B says the sweeps are not waiting on memory.
Usage: python tools/qp_scan.py [B ...]   (LIB=<path> overrides the product library)
"""
import os, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sdf_nmpc_amd import _lib, synth
from sdf_nmpc_amd.config import Config
from sdf_nmpc_amd.model import Quad

cfg = Config(); model = Quad(cfg)
dev = torch.device("cuda:0")
ctx = _lib.Context(0, stream=torch.cuda.current_stream().cuda_stream)
net = _lib.Net.siren(ctx, 0)
N = int(os.environ.get("N", 40))
for B in [int(a) for a in sys.argv[1:]] or [32, 128, 256, 512, 1024, 2048]:
    prob = synth.make_problem(cfg, B, N, seed=1000)
    x0 = prob["x"][:, 0] + np.random.default_rng(2000).normal(0, 0.05, (B, 10))
    t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
         dict(x=prob["x"], u=prob["u"], p=prob["p"], dt=prob["dt"], x0=x0, yref=prob["yref"], W=prob["W"],
              yNref=prob["yN"], WN=prob["WN"]).items()}
    sh = dict(xn=(B, N, 10), AB=(B, N, 14, 10), y=(B, N, 11), Jy=(B, N, 14, 11), yN=(B, 4), JyN=(B, 10, 4),
              h=(B, N + 1, 3), Jh=(B, N + 1, 10, 3), dx=(B, N + 1, 10), du=(B, N, 4), res=(B, 2))
    for k, s in sh.items():
        t[k] = torch.zeros(s, dtype=torch.float64, device=dev)
    t["status"] = torch.zeros(B, dtype=torch.int32, device=dev)
    t["iters"] = torch.zeros(B, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    _lib.linearize(ctx, net, _lib.quad_model(cfg), B, N, prob["p"].shape[-1], t)
    opts = _lib.qp_opts(model)
    _lib.qp_solve(ctx, opts, B, N, t)
    ctx.synchronize()
    ctx.enable_timing(True); ctx.reset_stats()
    R = 10
    for _ in range(R):
        _lib.qp_solve(ctx, opts, B, N, t)
    ctx.synchronize()
    ms = ctx.kernel_stats("rti_qp")[0] / R
    ctx.enable_timing(False)
    it = t["iters"].cpu().numpy()
    print(f"B={B:5d} N={N}: rti_qp {ms * 1e3:8.1f} us  iters mean {it.mean():.2f} max {it.max()}  "
          f"{ms * 1e3 / it.max():6.2f} us per max-iteration  status!=0 {(t['status'] != 0).sum().item()}", flush=True)
