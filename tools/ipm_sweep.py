"""IPM parameter sweep on the CPU restatement (oracle/qp_ipm.c): max / mean QP iterations over consecutive
RTI steps of the bench problem (synthetic, seed 1000 + s).  Diagnostic only -- the kernel's defaults
live in csrc/rti_qp.hip (QP_T0 ...), the oracle's in oracle.QP_START.
Usage: python tools/ipm_sweep.py B STEPS SEEDS 'name:{"tau_hi":0.999}' ..."""
import json, os, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle as O
from sdf_nmpc_amd import synth, weights as W, _lib
from sdf_nmpc_amd.config import Config
from sdf_nmpc_amd.model import Quad

B, STEPS, SEEDS = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
GC = float(os.environ.get("GONDZIO_COST", 0.4))
variants = [("base", {})] + [(a.split(":", 1)[0], json.loads(a.split(":", 1)[1])) for a in sys.argv[4:]]
cfg = Config(); model = Quad(cfg); N = int(os.environ.get("HORIZON", 40))
onet = O.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=0))
m = O.quad_model(cfg)
_, dt = _lib.shooting_grid(N, cfg.mpc.T)
# linearisations of each variant's own trajectory: cache per (variant, seed, step)
res = {n: [] for n, _ in variants}
for seed in range(SEEDS):
    prob0 = synth.make_problem(cfg, B, N, seed=1000 + seed, dt=dt)
    x0 = prob0["x"][:, 0] + np.random.default_rng(2000 + seed).normal(0, 0.05, (B, 10))
    for name, start in variants:
        prob = {k: v.copy() for k, v in prob0.items()}
        for st in range(STEPS):
            x = prob["x"].copy()
            if os.environ.get("X0_NODE0", "1") == "1":
                x[:, 0] = x0  # solver semantics (ocp.py:161): node 0 of the iterate is the measured state
            t0 = time.time()
            lin = O.linearize_batch(m, onet, x, prob["u"], prob["p"], dt, nthreads=8)
            q = O.qp_ipm_batch(lin, dict(prob, x=x), x0, model, nthreads=8, start=start)
            cost = q["iters"] + GC * q["gondzio"]  # corrector solve ~ GC of an iteration in the kernel
            res[name].append((seed, st, int(q["iters"].max()), float(q["iters"].mean()), int((q["status"] != 0).sum()),
                              float(cost.max()), float(cost.mean()), float(q["gondzio"].mean())))
            prob["x"] = x + q["dx"]; prob["u"] = prob["u"] + q["du"]
for name, _ in variants:
    r = np.array(res[name])
    print(f"{name:12s} max {int(r[:, 2].max()):3d}  mean-of-max {r[:, 2].mean():6.2f}  mean {r[:, 3].mean():5.2f}  "
          f"fail {int(r[:, 4].sum())}  cost max {r[:, 5].max():5.1f} mean-of-max {r[:, 5].mean():5.2f} mean {r[:, 6].mean():5.2f} "
          f"gondzio/inst {r[:, 7].mean():4.2f}  per-step max {list(r[:, 2].astype(int))}")
