"""Diagnostic: GPU QP vs the C restatement vs the exact solution on a batch (per-instance errors, iterations)."""
import sys, os
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "oracle")); sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch
import oracle as O, qp_oracle
import sdf_nmpc_amd
from sdf_nmpc_amd import _lib
from sdf_nmpc_amd.config import Config
import test_gpu_qp as T

B, N, seed, noise = [float(a) if "." in a else int(a) for a in sys.argv[1:5]]
tol = float(sys.argv[5]) if len(sys.argv) > 5 else 1e-8
cfg = Config()
ctx = _lib.Context(0, stream=torch.cuda.current_stream().cuda_stream)
prob, x0, t = T.setup(ctx, cfg, B, N, seed, x0_noise=noise)
model = T.solve(ctx, cfg, t, B, N, tol=tol)
lin = {k: t[k].cpu().numpy() for k in ("xn", "AB", "y", "Jy", "yN", "JyN", "h", "Jh")}
ref = O.qp_ipm_batch(lin, prob, x0, model, tol=tol, nthreads=8)
du, it, res = t["du"].cpu().numpy(), t["iters"].cpu().numpy(), t["res"].cpu().numpy()
d = np.abs(du - ref["du"]).max(axis=(1, 2))
print("iters gpu max/mean", it.max(), it.mean(), " C", ref["iters"].max(), ref["iters"].mean(), " iters differ:", (it != ref["iters"]).sum())
for b in np.argsort(-d)[:6]:
    q = qp_oracle.stage_qp({k: v[b] for k, v in lin.items()}, prob["x"][b], prob["u"][b], x0[b], prob["yref"][b],
                           prob["W"][b], prob["yN"][b], prob["WN"][b], prob["dt"], model, 10.0)
    ex = qp_oracle.polish(q, qp_oracle.solve_dense(q))
    print(f"b={b} gpu-C {d[b]:.2e}  gpu-exact {np.abs(du[b]-ex['du']).max():.2e}  C-exact {np.abs(ref['du'][b]-ex['du']).max():.2e}"
          f"  iters gpu {it[b]} C {ref['iters'][b]}  res gpu {res[b]} C {ref['res'][b]}")
