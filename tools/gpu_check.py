"""First-contact GPU diagnostic: parity stats of the HIP path vs the oracle/golden + rough timing."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402
import sdf_nmpc_amd  # noqa: E402
from sdf_nmpc_amd import _lib, synth, weights as W  # noqa: E402
from sdf_nmpc_amd.config import Config  # noqa: E402

dev = torch.device("cuda:0")
ctx = _lib.Context(0, stream=torch.cuda.current_stream().cuda_stream)
g = np.load(os.path.join(ROOT, "tests/golden/sdf_golden.npz"))
inp = g["input"]
n = inp.shape[0]
for v in ("siren", "stress"):
    seed, wg, bg = g[v + "/spec"]
    net = _lib.Net.siren(ctx, int(seed), float(wg), float(bg))
    for M in (32, 64):
        ctx.set_tile_rows(M)
        pos4 = torch.zeros(n, 4, device=dev)
        pos4[:, :3] = torch.from_numpy(inp[:, :3]).to(dev)
        lat = torch.from_numpy(inp[:, 3:]).contiguous().to(dev)
        out = torch.empty(n, 4, device=dev)
        net.eval(n, pos4, lat, 1, out)
        ctx.synchronize()
        o = out.cpu().numpy()
        r32, r64 = g[v + "/df_f32"], g[v + "/df_f64"]
        G32, G64 = g[v + "/grad_f32"][:, :3], g[v + "/grad_f64"][:, :3]
        nrm = np.linalg.norm(G64, axis=1)
        print(f"{v} M={M}: df |gpu-ref32| max {np.abs(o[:,0]-r32).max():.3e} |gpu-ref64| {np.abs(o[:,0]-r64).max():.3e}"
              f" (ref32-ref64 {np.abs(r32-r64).max():.3e}); grad normwise gpu-ref64 "
              f"{(np.linalg.norm(o[:,1:]-G64,axis=1)/nrm).max():.3e} gpu-ref32 {(np.linalg.norm(o[:,1:]-G32,axis=1)/nrm).max():.3e}"
              f" (ref32-ref64 {(np.linalg.norm(G32-G64,axis=1)/nrm).max():.3e}) abs {np.abs(o[:,1:]-G32).max():.3e}")
    # latent grad via host path
    df, gr = net.eval_host(inp[:64].astype(np.float64))
    G32f = g[v + "/grad_f32"][:64]
    print(f"{v} host path: df max {np.abs(df-g[v+'/df_f32'][:64]).max():.3e}, full grad max abs {np.abs(gr-G32f).max():.3e}"
          f" rel {np.abs(gr-G32f).max()/np.abs(G32f).max():.3e}")
    net.close()

# linearize vs oracle
cfg = Config()
B, N = 64, 40
prob = synth.make_problem(cfg, B, N, seed=3)
net = _lib.Net.siren(ctx, 0)
model = _lib.quad_model(cfg)
t = {k: torch.from_numpy(np.ascontiguousarray(prob[k])).to(dev) for k in ("x", "u", "p", "dt")}
outs = dict(xn=(B, N, 10), AB=(B, N, 14, 10), y=(B, N, 11), Jy=(B, N, 14, 11), yN=(B, 4), JyN=(B, 10, 4),
            h=(B, N + 1, 3), Jh=(B, N + 1, 10, 3))
bufs = {k: torch.full(s, float("nan"), dtype=torch.float64, device=dev) for k, s in outs.items()}
bufs["sdf"] = torch.empty(B, N + 1, 4, device=dev)
bufs.update(t)
ctx.set_tile_rows(32)
torch.cuda.synchronize()
_lib.linearize(ctx, net, model, B, N, 145, bufs)
ctx.synchronize()
onet = O.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, 0))
ref = O.linearize_batch(O.quad_model(cfg), onet, prob["x"], prob["u"], prob["p"], prob["dt"], nthreads=8)
for k in ("xn", "AB", "y", "Jy", "yN", "JyN", "h", "Jh"):
    a, b = bufs[k].cpu().numpy(), ref[k]
    print(f"lin {k}: max abs {np.nanmax(np.abs(a-b)):.3e} max|ref| {np.abs(b).max():.3e} nan {np.isnan(a).sum()}")
s = bufs["sdf"].cpu().numpy()
print("sdf df gpu-oracle32", np.abs(s[..., 0] - ref["sdf"][..., 0]).max(), "grad", np.abs(s[..., 1:] - ref["sdf"][..., 1:]).max())

# timing C3: B=1024, N=40
B, N = 1024, 40
prob = synth.make_problem(cfg, B, N, seed=0)
t = {k: torch.from_numpy(np.ascontiguousarray(prob[k])).to(dev) for k in ("x", "u", "p", "dt")}
outs = dict(xn=(B, N, 10), AB=(B, N, 14, 10), y=(B, N, 11), Jy=(B, N, 14, 11), yN=(B, 4), JyN=(B, 10, 4),
            h=(B, N + 1, 3), Jh=(B, N + 1, 10, 3))
bufs = {k: torch.empty(s, dtype=torch.float64, device=dev) for k, s in outs.items()}
bufs.update(t)
for M in (32, 64):
    ctx.set_tile_rows(M)
    for _ in range(3):
        _lib.linearize(ctx, net, model, B, N, 145, bufs)
    ctx.synchronize()
    ctx.enable_timing(True)
    ctx.reset_stats()
    K = 20
    t0 = time.perf_counter()
    for _ in range(K):
        _lib.linearize(ctx, net, model, B, N, 145, bufs)
    ctx.synchronize()
    wall = (time.perf_counter() - t0) / K
    st = {k: ctx.kernel_stats(k) for k in ("sdf_hoist", "sdf_mlp", "linearize")}
    ctx.enable_timing(False)
    sdf_ms = st["sdf_mlp"][0] / st["sdf_mlp"][1]
    flops = (B * (N + 1) * 553984) / (sdf_ms * 1e-3)
    print(f"M={M}: wall {wall*1e3:.3f} ms/step -> {B/wall:.0f} inst-steps/s; kernels(ms): " +
          ", ".join(f"{k} {v[0]/max(v[1],1):.4f}" for k, v in st.items()) + f"; sdf {flops/1e12:.1f} TFLOP/s")
