"""Per-phase cycle accounting of the RTI QP kernel (diagnostic).

Linearises a B=1024, N=40 problem on the GPU, dumps the QP inputs and runs tools/_qp_stamps_drv
(rti_qp.hip built with -DQP_STAMPS; build line in tools/qp_stamps_drv.hip's header) as a child process.
"""
import os, subprocess, sys
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from sdf_nmpc_amd import _lib, synth
from sdf_nmpc_amd.config import Config
from sdf_nmpc_amd.model import Quad

B, N = int(os.environ.get("B", 1024)), int(os.environ.get("N", 40))
cfg = Config(); model = Quad(cfg)
dev = torch.device("cuda:0")
ctx = _lib.Context(0, stream=torch.cuda.current_stream().cuda_stream)
net = _lib.Net.siren(ctx, 0)
SEED, NOISE = int(os.environ.get("SEED", 5)), float(os.environ.get("NOISE", 0.05))
prob = synth.make_problem(cfg, B, N, seed=SEED)
x0 = prob["x"][:, 0] + np.random.default_rng(SEED + 1).normal(0, NOISE, (B, 10))
t = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in
     dict(x=prob["x"], u=prob["u"], p=prob["p"], dt=prob["dt"], x0=x0, yref=prob["yref"], W=prob["W"],
          yNref=prob["yN"], WN=prob["WN"]).items()}
sh = dict(xn=(B, N, 10), AB=(B, N, 14, 10), y=(B, N, 11), Jy=(B, N, 14, 11), yN=(B, 4), JyN=(B, 10, 4),
          h=(B, N + 1, 3), Jh=(B, N + 1, 10, 3), hE=(B, 6), JhE=(B, 10, 6))
for k, s in sh.items():
    t[k] = torch.zeros(s, dtype=torch.float64, device=dev)
torch.cuda.synchronize()
_lib.linearize(ctx, net, _lib.quad_model(cfg), B, N, prob["p"].shape[-1], t)
ctx.synchronize()
path = os.path.join(os.environ.get("TMPDIR", "/tmp"), "qp_in.bin")
os.makedirs(os.path.dirname(path), exist_ok=True)
with open(path, "wb") as f:
    f.write(np.array([B, N], np.int32).tobytes())
    for k in ("xn", "AB", "y", "Jy", "yN", "JyN", "h", "Jh", "x", "u", "x0", "yref", "W", "yNref", "WN", "dt"):  # the driver's order
        f.write(np.ascontiguousarray(t[k].double().cpu().numpy()).tobytes())
    f.write(np.concatenate([model.lbu, model.ubu, model.lh, model.uh, model.zl, model.Zl, [10.0, 1e-8]]).astype(np.float64).tobytes())
del t; torch.cuda.synchronize()
sys.exit(subprocess.call([os.path.join(ROOT, "tools", "_qp_stamps_drv" + os.environ.get("DRV", "")), path]))
