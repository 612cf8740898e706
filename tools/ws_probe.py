"""Does HPIPM's primal warm start (qp_solver_warm_start = 1, ocp.py:116) shorten the QPs of a closed
RTI loop?  CPU only: the C restatement (oracle/qp_ipm.c) runs the bench problem (synth.make_problem)
as the controller runs it -- x_0 = the plant state, linearise, QP, full step, plant advanced by u_0 --
once cold-started and once started from the previous QP's du, and prints the per-step mean / max
iteration counts and the largest |u_0| difference between the two loops (the QP is strictly convex, so
the start changes only the iteration count, to the QP tolerance).  Diagnostic."""
import os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle as O
from sdf_nmpc_amd import synth, weights as W
from sdf_nmpc_amd.config import Config
from sdf_nmpc_amd.model import Quad

B = int(os.environ.get("B", 64))
K = int(os.environ.get("K", 12))
O.build()
onet = O.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=0))
for N in [int(v) for v in (sys.argv[1:] or ["20", "40"])]:
    for shift in (0, 1):
        cfg = Config(mpc__N=N, mpc__shift=shift)
        model, om = Quad(cfg), O.quad_model(cfg)
        prob = synth.make_problem(cfg, B, N, seed=5)
        dt = prob["dt"]
        runs = {}
        for ws in (False, True):
            xs, us, xo = prob["x"].copy(), prob["u"].copy(), prob["x"][:, 0].copy()
            du_prev, its, u0s = None, [], []
            for _ in range(K):
                if 0 < shift < N:
                    xs[:, : N - shift] = xs[:, shift:N].copy()
                    us[:, : N - shift] = us[:, shift:N].copy()
                xs[:, 0] = xo
                lin = O.linearize_batch(om, onet, xs, us, prob["p"], dt, nthreads=8)
                q = O.qp_ipm_batch(lin, dict(prob, x=xs, u=us), xo, model, nthreads=8,
                                   du_ws=du_prev if ws else None)
                du_prev = q["du"].copy()
                xs, us = xs + q["dx"], us + q["du"]
                its.append(q["iters"].copy())
                u0s.append(us[:, 0].copy())
                # plant: the model's RK4 over dt[0] under u_0
                pl = O.linearize_batch(om, onet, np.stack([xo, xo], 1), us[:, :1], np.zeros((B, 2, prob["p"].shape[-1])),
                                       dt[:1], nthreads=8)
                xo = pl["xn"][:, 0]
            runs[ws] = (np.array(its), np.array(u0s))
        (ic, uc), (iw, uw) = runs[False], runs[True]
        print(f"N={N} shift={shift}  cold mean/max per step: " + " ".join(f"{a.mean():.1f}/{a.max()}" for a in ic))
        print(f"{'':16s}warm mean/max per step: " + " ".join(f"{a.mean():.1f}/{a.max()}" for a in iw))
        print(f"{'':16s}max |u0 cold - u0 warm| = {np.abs(uc - uw).max():.2e}", flush=True)
