"""Exact solutions of 64 QPs of the bench workload C3 (qp_exact_golden.npz) -- test infrastructure.

The QPs: synthetic seed 1000, B = 1024, N = 40, x0 = x_0 + N(0, 0.05) (rng 2000), node 0 of the iterate
set to x0 (the solver object's ocp.py:161 semantics, as bench.py), linearised by the C oracle
(oracle/oracle.c).  The 64 instances: every 32nd, plus the 32 most degenerate of the rest -- those whose
C-IPM solution (oracle/qp_ipm.c, the GPU kernel's algorithm) moves most between the production stop
tolerance 1e-8 and 1e-13 (a flat direction at a near-degenerate vertex).  Each is solved by the dense
Mehrotra IPM on the full KKT system and polished on its active set (oracle/qp_oracle.py), KKT-checked,
and stored with its objective F* and the strong-convexity modulus mu of the objective in (dx, du)
(the smallest eigenvalue of its (dx, du) Hessian block: the Levenberg-Marquardt term makes it > 0).
Run: python tests/golden/make_qp_exact.py  (about a minute on 8 cores)."""
import os
import sys
from multiprocessing import Pool

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle")]
os.environ.setdefault("OMP_NUM_THREADS", "1")
os.environ.setdefault("OPENBLAS_NUM_THREADS", "1")
os.environ.setdefault("MKL_NUM_THREADS", "1")
import numpy as np  # noqa: E402

B, N, SEED, NSEL = 1024, 40, 1000, 64


def problem():
    """The workload and its C-oracle linearisation (shared with tests/test_gpu_qp.py)."""
    import oracle as O
    from sdf_nmpc_amd import _lib, synth, weights as W
    from sdf_nmpc_amd.config import Config
    from sdf_nmpc_amd.model import Quad
    cfg = Config()
    model = Quad(cfg)
    _, dt = _lib.shooting_grid(N, cfg.mpc.T)
    prob = synth.make_problem(cfg, B, N, seed=SEED, dt=dt)
    x0 = prob["x"][:, 0] + np.random.default_rng(2000).normal(0, 0.05, (B, 10))
    prob["x"][:, 0] = x0
    O.build()
    onet = O.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=0))
    lin = O.linearize_batch(O.quad_model(cfg), onet, prob["x"], prob["u"], prob["p"], dt, nthreads=8)
    return cfg, model, prob, x0, lin


def _exact(args):
    import qp_oracle
    b, lin_b, prob_b, x0_b, model, hi_b = args
    q = qp_oracle.stage_qp(lin_b, prob_b["x"], prob_b["u"], x0_b, prob_b["yref"], prob_b["W"], prob_b["yN"],
                           prob_b["WN"], prob_b["dt"], model, 10.0)
    # polish on the dense IPM's active set, corrected row by row until the KKT conditions hold
    # (oracle/qp_oracle.py polish_active_set); the C IPM's tol-1e-13 point is the second start
    ref = None
    for st in (qp_oracle.solve_dense(q), hi_b):
        ref = qp_oracle.polish_active_set(q, st)
        if ref["max_violation"] < 1e-9 and ref["min_dual"] > -1e-9:
            break
    H, g, E, e, G, d = qp_oracle.dense_problem(q)
    z = np.concatenate([ref["dx"].ravel(), ref["du"].ravel(), ref["sl"].ravel(), ref["su"].ravel()])
    nv = (N + 1) * 10 + N * 4
    mu = np.linalg.eigvalsh(H[:nv, :nv])[0]
    return b, ref, 0.5 * z @ H @ z + g @ z, mu


def main():
    import oracle as O
    cfg, model, prob, x0, lin = problem()
    lo = O.qp_ipm_batch(lin, prob, x0, model, tol=1e-8, nthreads=8)
    hi = O.qp_ipm_batch(lin, prob, x0, model, tol=1e-13, max_iter=200, nthreads=8)
    score = np.abs(lo["du"] - hi["du"]).max(axis=(1, 2))
    strided = np.arange(0, B, B // (NSEL // 2))
    rest = np.setdiff1d(np.arange(B), strided)
    worst = rest[np.argsort(-score[rest], kind="stable")[:NSEL // 2]]
    sel = np.sort(np.concatenate([strided, worst]))
    jobs = [(int(b), {k: v[b] for k, v in lin.items()},
             {k: (v if k == "dt" else v[b]) for k, v in prob.items()}, x0[b], model,
             {"dx": hi["dx"][b], "du": hi["du"][b], "sl": hi["slack"][b][..., 0], "su": hi["slack"][b][..., 1]})
            for b in sel]
    with Pool(8) as pool:
        res = sorted(pool.map(_exact, jobs), key=lambda r: r[0])
    out = {"sel": sel, "score": score[sel]}
    for key in ("dx", "du", "sl", "su"):
        out[key] = np.stack([r[1][key] for r in res])
    out["F"] = np.array([r[2] for r in res])
    out["mu"] = np.array([r[3] for r in res])
    out["max_violation"] = np.array([r[1]["max_violation"] for r in res])
    out["min_dual"] = np.array([r[1]["min_dual"] for r in res])
    print("kkt", out["max_violation"].max(), out["min_dual"].min(), np.argsort(out["min_dual"])[:5], np.sort(out["min_dual"])[:5])
    assert (out["max_violation"] < 1e-9).all() and (out["min_dual"] > -1e-9).all()
    np.savez_compressed(os.path.join(HERE, "qp_exact_golden.npz"), **out)
    d_lo = np.abs(lo["du"][sel] - out["du"]).max(axis=(1, 2))
    print("qp_exact_golden.npz", {k: v.shape for k, v in out.items()})
    print(f"C IPM at tol 1e-8 vs exact: max |du| err {d_lo.max():.2e}, median {np.median(d_lo):.2e}, "
          f"> 5e-6 on {(d_lo > 5e-6).sum()} of {len(sel)}; mu in [{out['mu'].min():.3f}, {out['mu'].max():.3f}]")


if __name__ == "__main__":
    main()
