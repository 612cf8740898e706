#!/usr/bin/env python3
"""Probe: one flag set's QP at (B, N) on the serial and the segmented kernel beside the C IPM's serial and
segmented recursions (oracle/qp_ipm.c): per instance |du| differences, iterations, status, objective gap to
the exact solution.  python3 tools/seg_flag_probe.py hard_df_rec_feas 16 40"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle")]
import sdf_nmpc_amd  # noqa: E402,F401
from sdf_nmpc_amd import _lib  # noqa: E402


def main():
    import oracle as O
    import qp_oracle
    import test_gpu_flags as T
    name, B, N = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    import torch
    O.build()
    assert torch.cuda.is_available()  # torch's HIP runtime first, as the tests' gpu_ctx fixture does
    ctx = _lib.Context(0, stream=torch.cuda.current_stream().cuda_stream)
    res = {}
    for kernel in ("serial", "segmented"):
        cfg, q, prob, x0, t = T._setup(ctx, name, B, N, seed=12)
        _lib.linearize(ctx, T._net(ctx, q), _lib.quad_model(cfg, q), B, N, q.np, t, nyN=q.nyN, no_sdf=not q.need_sdf)
        opts = _lib.qp_opts(q, tol=T.QP_TOL)
        ctx.set_qp_kernel(kernel)
        _lib.qp_solve(ctx, opts, B, N, t)
        ctx.synchronize()
        res[kernel] = T._np(t, T.OUT)
    lin = {k: res["serial"][k] for k in T.LIN}
    c1 = O.qp_ipm_batch(lin, prob, x0, q, tol=T.QP_TOL)
    c4 = O.qp_ipm_batch(lin, prob, x0, q, tol=T.QP_TOL, start=dict(seg=4))
    for b in range(B):
        qq = qp_oracle.stage_qp({k: v[b] for k, v in lin.items()}, prob["x"][b], prob["u"][b], x0[b], prob["yref"][b],
                                prob["W"][b], prob["yN"][b], prob["WN"][b], prob["dt"], q, 10.0)
        ex = qp_oracle.polish_active_set(qq, qp_oracle.solve_dense(qq))
        H, g, E, e, G, d = qp_oracle.dense_problem(qq)
        zs = qp_oracle.z_of(qq, ex)
        Fs = 0.5 * zs @ H @ zs + g @ zs
        line = [f"b={b:2d}"]
        for lab, o in (("gpu_ser", res["serial"]), ("gpu_seg", res["segmented"]), ("c_ser", c1), ("c_seg", c4)):
            sol = dict(dx=o["dx"][b], du=o["du"][b], sl=o["slack"][b][..., 0], su=o["slack"][b][..., 1])
            z = qp_oracle.z_of(qq, sol)
            F = 0.5 * z @ H @ z + g @ z
            line.append(f"{lab}: it {int(o['iters'][b])} st {int(o['status'][b])} dF {F - Fs:+.1e} "
                        f"|du-ex| {np.abs(o['du'][b] - ex['du']).max():.1e}")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main()
