#!/usr/bin/env python3
"""Probe: C3 RTI throughput with the per-GPU batch split into L lanes, each lane a context on its own
stream solving B/L instances step after step, the lanes' steps free to overlap (a lane's preparation
phase beside another lane's latency-bound QP).  Prints one line per configuration.

    python tools/pipe_probe.py --lanes 1 2 4 --steps 30
"""
import argparse
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import sdf_nmpc_amd  # noqa: E402,F401
from sdf_nmpc_amd import _lib, synth, weights as W  # noqa: E402
from sdf_nmpc_amd.config import Config  # noqa: E402
from sdf_nmpc_amd.model import Quad  # noqa: E402


def make_lane(cfg, blob, prob, x0, lo, hi, N, dev, priority=0):
    B = hi - lo
    s = torch.cuda.Stream(dev, priority=priority)
    ctx = _lib.Context(dev.index, stream=s.cuda_stream)
    ctx.set_qp_kernel("serial")
    net = _lib.Net.from_blob(ctx, blob)
    bufs = {k: torch.from_numpy(np.ascontiguousarray(prob[k][lo:hi])).to(dev) for k in ("x", "u", "p")}
    bufs["dt"] = torch.from_numpy(np.ascontiguousarray(prob["dt"])).to(dev)
    shapes = dict(xn=(B, N, 10), AB=(B, N, 14, 10), y=(B, N, 11), Jy=(B, N, 14, 11), yN=(B, 4),
                  JyN=(B, 10, 4), h=(B, N + 1, 3), Jh=(B, N + 1, 10, 3))
    for k, sh in shapes.items():
        bufs[k] = torch.empty(sh, dtype=torch.float64, device=dev)
    bufs["sdf"] = torch.empty((B, N + 1, 4), dtype=torch.float32, device=dev)
    for k, v in dict(x0=x0[lo:hi], yref=prob["yref"][lo:hi], W=prob["W"][lo:hi], yNref=prob["yN"][lo:hi],
                     WN=prob["WN"][lo:hi]).items():
        bufs[k] = torch.from_numpy(np.ascontiguousarray(v)).to(dev)
    for k, sh in dict(dx=(B, N + 1, 10), du=(B, N, 4), res=(B, 2)).items():
        bufs[k] = torch.empty(sh, dtype=torch.float64, device=dev)
    bufs["status"] = torch.empty(B, dtype=torch.int32, device=dev)
    bufs["iters"] = torch.empty(B, dtype=torch.int32, device=dev)
    u0 = torch.empty((B, 4), dtype=torch.float64, device=dev)
    x_init, u_init = bufs["x"].clone(), bufs["u"].clone()
    x_init[:, 0].copy_(bufs["x0"])
    return dict(B=B, s=s, ctx=ctx, net=net, bufs=bufs, u0=u0, x_init=x_init, u_init=u_init)


def lane_step(L, model, qopts, N, np_, wait=None, record=None):
    b = L["bufs"]
    if wait is not None:
        L["s"].wait_event(wait)
    with torch.cuda.stream(L["s"]):
        b["x"].copy_(L["x_init"])
        b["u"].copy_(L["u_init"])
    _lib.rti_prepare(L["ctx"], L["net"], model, qopts, L["B"], N, np_, b)
    if record is not None:
        record.record(L["s"])
    _lib.qp_feedback(L["ctx"], qopts, L["B"], N, b)
    _lib.rti_apply(L["ctx"], L["B"], N, b["x"], b["u"], b["dx"], b["du"], L["u0"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lanes", type=int, nargs="+", default=[1, 2, 4])
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--batch", type=int, default=1024)
    ap.add_argument("--horizon", type=int, default=40)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    cfg = Config()
    N, B = args.horizon, args.batch
    blob = W.pack(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=0))
    _, dt = _lib.shooting_grid(N, cfg.mpc.T)
    prob = synth.make_problem(cfg, B, N, seed=1000, dt=dt)
    x0 = prob["x"][:, 0] + np.random.default_rng(2000).normal(0, 0.05, (B, 10))
    model = _lib.quad_model(cfg)
    qopts = _lib.qp_opts(Quad(cfg))
    np_ = prob["p"].shape[-1]
    for nl in args.lanes:
        for stagger in ((False, True) if nl > 1 else (False,)):
            edges = np.linspace(0, B, nl + 1).astype(int)
            lanes = [make_lane(cfg, blob, prob, x0, edges[i], edges[i + 1], N, dev) for i in range(nl)]
            for _ in range(3):
                for L in lanes:
                    lane_step(L, model, qopts, N, np_)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if stagger:  # lane i's first step waits for lane i-1's first preparation phase
                ev = [torch.cuda.Event() for _ in lanes]
                for i, L in enumerate(lanes):
                    lane_step(L, model, qopts, N, np_, wait=ev[i - 1] if i else None, record=ev[i])
            for k in range(args.steps - (1 if stagger else 0)):
                for L in lanes:
                    lane_step(L, model, qopts, N, np_)
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            it = np.concatenate([L["bufs"]["iters"].cpu().numpy() for L in lanes])
            st = np.concatenate([L["bufs"]["status"].cpu().numpy() for L in lanes])
            print(f"lanes={nl} stagger={stagger}: {B * args.steps / el:,.0f} instance-RTI-solves/s "
                  f"({el / args.steps * 1e3:.3f} ms/step)  iters max {it.max()} mean {it.mean():.2f} "
                  f"status max {st.max()}", flush=True)
            del lanes
            torch.cuda.synchronize()


if __name__ == "__main__":
    main()
