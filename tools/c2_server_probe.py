#!/usr/bin/env python3
"""Probe: where the time of one CasADi-external call goes (config C2, one row per call).  Calls
sdfnmpc_sdf_eval_host 2000 times with the resident server and with one launch per call; prints the
mean wall time per call and the server's own phase stamps (staging, evaluation, caller's wait)."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import sdf_nmpc_amd  # noqa: E402,F401
from sdf_nmpc_amd import _lib  # noqa: E402


def main():
    ctx = _lib.Context(0)
    net = _lib.Net.siren(ctx, 0)
    rng = np.random.default_rng(0)
    xs = [np.concatenate([rng.uniform(-2, 2, 3), rng.normal(size=128)])[None] for _ in range(41)]
    for server in (True, False, True):
        ctx.set_sdf_server(server)
        for x in xs:
            net.eval_host(x)
        ctx.sdf_server_stats() if server else None
        t0 = time.perf_counter()
        n = 2000
        for i in range(n):
            net.eval_host(xs[i % 41])
        us = (time.perf_counter() - t0) / n * 1e6
        st = ctx.sdf_server_stats() if server else {}
        print(f"server={server}: {us:.2f} us per call (python ctypes)  {st}", flush=True)


if __name__ == "__main__":
    main()
