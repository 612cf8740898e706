#!/usr/bin/env python3
"""Probe: one CasADi-external call (config C2, one row per call) on variant networks -- the resident server
(sdf_row_wide.hip), one sdf_row_wide launch per call, and the layer-by-layer schedule (sdf_wide.hip, the
path above the row evaluator's weight cap) -- mean wall time per call over 2000 calls, python ctypes."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import sdf_nmpc_amd  # noqa: E402,F401
from sdf_nmpc_amd import _lib, weights as W  # noqa: E402

SPECS = {
    "deployed": W.DEFAULT_SPEC,
    "sin_oct_L64": W.NetSpec(size_latent=64),
    "softplus_cube_L200": W.NetSpec(act="softplus", embed="cube", res="latent", size_latent=200, w0=1.0),
    "relu_pos_full_256": W.NetSpec(act="relu", embed="pos", res="full", layer_sizes=(256, 256, 256, 256), w0=1.0),
    "c5_wide": W.WIDE_SPEC,
}


def per_call(ctx, net, xs, server, n=2000):
    ctx.set_sdf_server(server)
    for x in xs:
        net.eval_host(x)
    t0 = time.perf_counter()
    for i in range(n):
        net.eval_host(xs[i % len(xs)])
    return (time.perf_counter() - t0) / n * 1e6


def main():
    ctx = _lib.Context(0)
    rng = np.random.default_rng(0)
    for name, spec in SPECS.items():
        blob = W.pack(spec, W.siren_weights(spec, 0))
        xs = [np.concatenate([rng.uniform(-2, 2, 3), rng.normal(size=spec.size_latent)])[None] for _ in range(41)]
        net = _lib.Net.from_blob(ctx, blob)
        os.environ["SDFNMPC_WIDE_ROW_MAX_MB"] = "0"
        net_l = _lib.Net.from_blob(ctx, blob)
        del os.environ["SDFNMPC_WIDE_ROW_MAX_MB"]
        ctx.sdf_server_stats()
        srv = per_call(ctx, net, xs, True)
        st = ctx.sdf_server_stats()
        launch = per_call(ctx, net, xs, False)
        layers = per_call(ctx, net_l, xs, False, n=500)
        print(f"{name}: server {srv:.2f} us, row launch {launch:.2f} us, layer-by-layer {layers:.2f} us per call; "
              f"server evaluation {st['eval_us']:.2f} us, staging {st['stage_us']:.2f} us, wait {st['wait_us']:.2f} us",
              flush=True)
        net.close()
        net_l.close()


if __name__ == "__main__":
    main()
