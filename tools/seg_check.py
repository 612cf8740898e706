"""Segmented QP kernel (rti_qp_seg.hip) vs the serial kernel (rti_qp.hip) and the C restatement of the
partitioned solve (oracle/qp_ipm.c lqr_seg, seg=4): iterations, status, solution gaps, and the kernel
time of both at C3 (diagnostic)."""
import os, sys, time
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle as O
from sdf_nmpc_amd import _lib, synth, weights as W
from sdf_nmpc_amd.config import Config
from sdf_nmpc_amd.model import Quad

cfg = Config(); model = Quad(cfg)
dev = torch.device("cuda:0")
ctx = _lib.Context(0)
net = _lib.Net.siren(ctx, 0)
onet = O.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=0))
cases = [(4, 20, 1), (8, 40, 2), (4, 60, 3), (1024, 40, 5)]
if len(sys.argv) > 1:
    cases = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]]
for B, N, seed in cases:
    prob = synth.make_problem(cfg, B, N, seed=seed)
    rng = np.random.default_rng(seed)
    x0 = prob["x"][:, 0] + rng.normal(0, 0.05, (B, 10))
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
    lin = {k: t[k].cpu().numpy() for k in ("xn", "AB", "y", "Jy", "yN", "JyN", "h", "Jh")}
    out = {}
    for kind in ("serial", "segmented"):
        for mi in (1, 100):
            ctx.set_qp_kernel(kind)
            t["dx"].zero_(); t["du"].zero_()
            _lib.qp_solve(ctx, _lib.qp_opts(model, max_iter=mi), B, N, t)
            ctx.synchronize()
            out[kind, mi] = {k: t[k].cpu().numpy().copy() for k in ("dx", "du", "iters", "status", "res")}
    nb = min(B, 16)
    sub = {k: v[:nb] for k, v in lin.items()}
    pr = dict(prob, x=prob["x"][:nb], u=prob["u"][:nb], yref=prob["yref"][:nb], W=prob["W"][:nb], yN=prob["yN"][:nb],
              WN=prob["WN"][:nb])
    cs = {mi: O.qp_ipm_batch(sub, pr, x0[:nb], model, nthreads=8, max_iter=mi, start=dict(seg=4)) for mi in (1, 100)}
    c1 = {mi: O.qp_ipm_batch(sub, pr, x0[:nb], model, nthreads=8, max_iter=mi) for mi in (1, 100)}
    print(f"--- B={B} N={N} seed={seed}  auto kernel: {ctx.qp_kernel(N, B)}")
    for kind in ("serial", "segmented"):
        o = out[kind, 100]
        print(f"  {kind:10s} status {np.bincount(o['status'], minlength=3)} iters max {o['iters'].max()} mean {o['iters'].mean():.2f}")
    for mi in (1, 100):
        g, s_ = out["segmented", mi], out["serial", mi]
        print(f"  max_iter={mi}: |seg-serial| du {np.abs(g['du'] - s_['du']).max():.2e} dx {np.abs(g['dx'] - s_['dx']).max():.2e}"
              f" | seg vs C-seg du {np.abs(g['du'][:nb] - cs[mi]['du']).max():.2e} dx {np.abs(g['dx'][:nb] - cs[mi]['dx']).max():.2e}"
              f" | serial vs C du {np.abs(s_['du'][:nb] - c1[mi]['du']).max():.2e}"
              f" | iters seg {g['iters'][:nb].tolist()[:8]} C-seg {cs[mi]['iters'].tolist()[:8]}")
    if B >= 256:
        for kind in ("serial", "segmented"):
            ctx.set_qp_kernel(kind)
            ctx.enable_timing(True); ctx.reset_stats()
            for _ in range(5):
                _lib.qp_solve(ctx, _lib.qp_opts(model), B, N, t)
            ctx.synchronize()
            print(f"  {kind:10s} rti_qp {ctx.kernel_stats('rti_qp')[0] / 5:.3f} ms  pack {ctx.kernel_stats('rti_qp_pack')[0] / 5:.3f} ms")
            ctx.enable_timing(False)
    sys.stdout.flush()
