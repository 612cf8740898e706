"""Per-iteration trace of the C IPM restatement (oracle/qp_ipm.c, orc_qp_trace) on the slowest instances of
the bench problem (synthetic seed 1000 + s, node 0 of the iterate = x0): alpha_aff, alpha, mean / max
complementarity, the row holding the max.  Diagnostic only.
Usage: python tools/ipm_trace.py SEED [NWORST] ['{"start": ...}']"""
import ctypes as C, json, os, sys
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
import oracle as O
from sdf_nmpc_amd import synth, weights as W, _lib
from sdf_nmpc_amd.config import Config
from sdf_nmpc_amd.model import Quad

seed = int(sys.argv[1]); nw = int(sys.argv[2]) if len(sys.argv) > 2 else 4
start = json.loads(sys.argv[3]) if len(sys.argv) > 3 else {}
cfg = Config(); model = Quad(cfg); N = int(os.environ.get("HORIZON", 40)); B = 1024
onet = O.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=0))
m = O.quad_model(cfg)
_, dt = _lib.shooting_grid(N, cfg.mpc.T)
prob = synth.make_problem(cfg, B, N, seed=1000 + seed, dt=dt)
x0 = prob["x"][:, 0] + np.random.default_rng(2000 + seed).normal(0, 0.05, (B, 10))
prob["x"][:, 0] = x0
lin = O.linearize_batch(m, onet, prob["x"], prob["u"], prob["p"], dt, nthreads=8)
q = O.qp_ipm_batch(lin, prob, x0, model, nthreads=8, start=start)
it = q["iters"]
print("iters histogram", np.bincount(it).tolist())
worst = np.argsort(-it, kind="stable")[:nw]
lib = O.lib()
for b in worst:
    tr = np.zeros((100, 9))
    lib.orc_qp_trace(tr.ctypes.data, 100)
    sub = {k: v[b:b + 1] for k, v in lin.items()}
    pb = {k: (v if k == "dt" else v[b:b + 1]) for k, v in prob.items()}
    r = O.qp_ipm_batch(sub, pb, x0[b:b + 1], model, nthreads=1, start=start)
    lib.orc_qp_trace(None, 0)
    n = int(r["iters"][0])
    print(f"--- instance {b}: {n} iterations, status {r['status'][0]}")
    for i in range(n):
        a = tr[i]
        row = int(a[6]); kind = "box" if row < 8 * N else "soft"
        kk = row // 8 if row < 8 * N else (row - 8 * N) // 12
        print(f"  it {i + 1:2d} a_aff {a[0]:.3f} a {a[1]:.3f} mu {a[2]:.2e} max {a[3]:.2e} rp {a[4]:.1e} "
              f"sigmu {a[5]:.1e} row {row} ({kind} k={kk} r={(row % 8) if row < 8 * N else (row - 8 * N) % 12}) t {a[7]:.2e} l {a[8]:.2e}")
