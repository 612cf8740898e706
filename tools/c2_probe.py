"""Diagnostic: where the per-call time of the host-pointer SDF path (the CasADi external, config C2) goes."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import sdf_nmpc_amd  # noqa: E402,F401
from sdf_nmpc_amd import _lib  # noqa: E402

if os.environ.get("SDFNMPC_LIB"):  # a diagnostic build (tools/build_variant.sh)
    _lib.LIB_PATH = os.environ["SDFNMPC_LIB"]
ctx = _lib.Context(0)
net = _lib.Net.siren(ctx, 0)
rng = np.random.default_rng(0)
x = np.concatenate([rng.uniform(-2, 2, (41, 3)), np.repeat(rng.normal(size=(1, 128)), 41, 0)], 1)
for grad in (True, False):
    for _ in range(20):
        net.eval_host(x[:1], want_grad=grad)
    ctx.enable_timing(True)
    ctx.reset_stats()
    t0 = time.perf_counter()
    n = 400
    for i in range(n):
        net.eval_host(x[i % 41: i % 41 + 1], want_grad=grad)
    wall = (time.perf_counter() - t0) / n * 1e6
    ks = {k: ctx.kernel_stats(k) for k in ("sdf_hoist", "sdf_mlp", "sdf_row")}
    ctx.enable_timing(False)
    print(f"grad={grad}: wall {wall:.1f} us/call; " + ", ".join(f"{k} {v[0] / max(v[1], 1) * 1e3:.1f} us x{v[1]}" for k, v in ks.items()))
    t0 = time.perf_counter()
    for i in range(n):
        net.eval_host(x[i % 41: i % 41 + 1], want_grad=grad)
    print(f"   untimed wall {(time.perf_counter() - t0) / n * 1e6:.1f} us/call")
