#!/usr/bin/env python3
"""Benchmark: NMPC RTI throughput at batch x N = 1024 x 40 per GPU (BASELINE.json config C3/C4).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A "step" is one pass of the hot path over one batch: for every one of the B instances on this GPU,
the SQP-RTI preparation phase over all N+1 shooting nodes (SDF forward + position-Jacobian,
ERK4 + forward sensitivities, NONLINEAR_LS residual/Jacobian, h = [hfov, vfov, sdf] and its
Jacobian) -- SURVEY.md §8(d)'s unit of work.  Inputs are resident in HBM before the timed region.
value = instances x steps / time over ALL ranks (weak scaling: B instances per GPU).  The full RTI
iteration (preparation + batched QP feedback phase + iterate update, i.e. one acados SQP_RTI
solve) is timed in its own loop with the same barrier / max-over-ranks protocol and reported in
"full_rti".  One process per GPU; instances never interact, so there is no data-path collective;
RCCL broadcasts the packed weights once at init.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SDF_FLOP_PER_ROW = 553_984      # fwd 138,456 MAC + d/dpos 138,536 MAC, x2
SDF_FLOP_PER_INST = 98_304      # hoisted latent GEMVs per instance
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: Peak FP32 (matrix)
HBM_PEAK_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E peak (spec)


def lin_bytes_per_instance(N, np_=145):
    """Algorithmic HBM bytes of the linearize kernel per instance (inputs read once + outputs)."""
    reads = 8 * ((N + 1) * 10 + N * 4 + (N + 1) * 17 + N) + 16 * (N + 1)   # x, u, p[0:17], dt, sdf
    writes = 8 * (N * (10 + 140 + 11 + 154) + 4 + 40 + (N + 1) * (3 + 30))
    return reads + writes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=1024, help="instances per GPU (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=0,
                    help="if > 0: this many instances in total, split by shard.instance_range (strong scaling)")
    ap.add_argument("--horizon", type=int, default=40)
    ap.add_argument("--tile-rows", type=int, default=32)
    ap.add_argument("--cpu-sample", type=int, default=64, help="instances in the CPU-baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--rti-steps", type=int, default=10, help="timed full-RTI steps (0: skip)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=dev)

    import sdf_nmpc_amd  # noqa: F401
    from sdf_nmpc_amd import _lib, shard, synth, weights as W
    from sdf_nmpc_amd.config import Config

    cfg = Config()
    N = args.horizon
    if args.global_batch > 0:
        lo, hi = shard.instance_range(args.global_batch, world, rank)
        B = hi - lo
    else:
        B = args.batch
    stream = torch.cuda.current_stream(dev).cuda_stream
    ctx = _lib.Context(local, stream=stream, tile_rows=args.tile_rows)

    # weights: rank 0 packs the SIREN-init network; RCCL broadcasts the blob (init-time collective)
    blob = W.pack(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=0)) if rank == 0 else None
    if world > 1:
        blob = shard.broadcast_blob(blob, dev)
    net = _lib.Net.from_blob(ctx, blob)
    model = _lib.quad_model(cfg)

    # synthetic problem for this rank's instance shard (seed = rank: distinct instances per GPU)
    nodes, dt = _lib.shooting_grid(N, cfg.mpc.T)
    prob = synth.make_problem(cfg, B, N, seed=1000 + rank, dt=dt)
    bufs = {k: torch.from_numpy(np.ascontiguousarray(prob[k])).to(dev) for k in ("x", "u", "p", "dt")}
    shapes = dict(xn=(B, N, 10), AB=(B, N, 14, 10), y=(B, N, 11), Jy=(B, N, 14, 11), yN=(B, 4), JyN=(B, 10, 4),
                  h=(B, N + 1, 3), Jh=(B, N + 1, 10, 3))
    for k, s in shapes.items():
        bufs[k] = torch.empty(s, dtype=torch.float64, device=dev)
    bufs["sdf"] = torch.empty((B, N + 1, 4), dtype=torch.float32, device=dev)
    np_ = prob["p"].shape[-1]
    # feedback-phase (QP) inputs/outputs: x0 near the first node, references, weights
    from sdf_nmpc_amd.model import Quad
    quad = Quad(cfg)
    x0 = prob["x"][:, 0] + np.random.default_rng(2000 + rank).normal(0, 0.05, (B, 10))
    for k, v in dict(x0=x0, yref=prob["yref"], W=prob["W"], yNref=prob["yN"], WN=prob["WN"]).items():
        bufs[k] = torch.from_numpy(np.ascontiguousarray(v)).to(dev)
    for k, sh in dict(dx=(B, N + 1, 10), du=(B, N, 4), res=(B, 2)).items():
        bufs[k] = torch.empty(sh, dtype=torch.float64, device=dev)
    bufs["status"] = torch.empty(B, dtype=torch.int32, device=dev)
    bufs["iters"] = torch.empty(B, dtype=torch.int32, device=dev)
    u0 = torch.empty((B, 4), dtype=torch.float64, device=dev)
    qopts = _lib.qp_opts(quad)

    def step():
        _lib.linearize(ctx, net, model, B, N, np_, bufs)

    def rti_step():  # one SQP-RTI solve: preparation, feedback (QP), iterate update + u_0
        _lib.linearize(ctx, net, model, B, N, np_, bufs)
        _lib.qp_solve(ctx, qopts, B, N, bufs)
        _lib.rti_apply(ctx, B, N, bufs["x"], bufs["u"], bufs["dx"], bufs["du"], u0)

    def barrier():
        if world > 1:
            dist.barrier()

    def timed(fn, k):
        torch.cuda.synchronize(dev)
        barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize(dev)
        barrier()
        el = time.perf_counter() - t0
        return shard.max_over_ranks(el, dev) if world > 1 else el

    for _ in range(args.warmup):
        step()
    elapsed = timed(step, args.steps)
    ms_per_step = elapsed / args.steps * 1e3
    total = args.global_batch if args.global_batch > 0 else world * B
    value = total * args.steps / elapsed

    # per-step latency distribution (each step synchronised on its own) and B=1 latency (config C2)
    lat = []
    for _ in range(min(args.steps, 50)):
        s0 = time.perf_counter()
        step()
        torch.cuda.synchronize(dev)
        lat.append((time.perf_counter() - s0) * 1e3)
    p50 = float(np.median(lat))

    # kernel durations by HIP events on the context stream (separate, untimed pass)
    ctx.enable_timing(True)
    ctx.reset_stats()
    reps = max(10, min(args.steps, 50))
    for _ in range(reps):
        step()
    kst = {k: ctx.kernel_stats(k) for k in ("sdf_hoist", "sdf_mlp", "linearize")}
    ctx.enable_timing(False)
    kms = {k: (v[0] / v[1] if v[1] else None) for k, v in kst.items()}
    rows = B * (N + 1)
    sdf_flop = rows * SDF_FLOP_PER_ROW
    achieved = sdf_flop / (kms["sdf_mlp"] * 1e-3) / 1e12
    lin_b = B * lin_bytes_per_instance(N)
    lin_gbs = lin_b / (kms["linearize"] * 1e-3) / 1e9

    # full SQP-RTI iteration (preparation + QP + update); the iterate evolves step to step
    full = None
    if args.rti_steps > 0:
        for _ in range(2):
            rti_step()
        rel = timed(rti_step, args.rti_steps)
        ctx.enable_timing(True)
        ctx.reset_stats()
        rti_step()
        qst = ctx.kernel_stats("rti_qp")
        ctx.enable_timing(False)
        it = bufs["iters"].cpu().numpy()
        st = bufs["status"].cpu().numpy()
        full = {"value": total * args.rti_steps / rel, "unit": "instance-RTI-solves/s (prep + QP + update)",
                "ms_per_step": rel / args.rti_steps * 1e3, "steps": args.rti_steps,
                "qp_kernel_ms": qst[0] / qst[1] if qst[1] else None,
                "qp_iters_mean": float(it.mean()), "qp_iters_max": int(it.max()),
                "qp_converged_frac": float((st == 0).mean()),
                "qp": "batched Riccati IPM, one wavefront per instance (rti_qp.hip); tol 1e-8, max_iter 100"}

    # traffic from the committed PMC profile of this same command (profiles/)
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            if pmc.get("B") == B and pmc.get("N") == N and pmc.get("tile_rows") == args.tile_rows:
                traffic = pmc["kernels"]["sdf_mlp"]["hbm_bytes_per_launch"]
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU baseline leg only (the "port")
        O.build()
        threads = min(16, os.cpu_count() or 1)
        S = min(args.cpu_sample, B)
        onet = O.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=0))
        om = O.quad_model(cfg)
        sub = {k: np.ascontiguousarray(prob[k][:S]) for k in ("x", "u", "p")}
        O.linearize_batch(om, onet, sub["x"][:2], sub["u"][:2], sub["p"][:2], dt, nthreads=threads)  # warm
        c0 = time.perf_counter()
        O.linearize_batch(om, onet, sub["x"], sub["u"], sub["p"], dt, nthreads=threads)
        cpu_s = time.perf_counter() - c0
        S1 = max(2, S // 16)
        c0 = time.perf_counter()
        O.linearize_batch(om, onet, sub["x"][:S1], sub["u"][:S1], sub["p"][:S1], dt, nthreads=1)
        cpu1_s = time.perf_counter() - c0
        cpu = {"value": S / cpu_s, "unit": "instance-RTI-steps/s (preparation phase)", "cores": threads,
               "kind": "port",
               "sample": f"{S} of the {B} instances x {N + 1} nodes, C oracle (oracle/oracle.c, fp32 MLP + fp64 "
                         f"linearisation, OpenMP over rows); 1-thread rate on {S1} instances = "
                         f"{S1 / cpu1_s:.1f}/s",
               "value_1thread": S1 / cpu1_s}

    out = {
        "metric": "NMPC solves/sec at batch×N=1024×40 on 1/2/4/8 GPUs; p50 control-step latency",
        "value": value,
        "unit": "instance-RTI-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if args.global_batch > 0 else "weak",
        "vs_baseline": None,
        "dtype": "f32 (SDF MLP, MFMA) + f64 (linearisation)",
        "data": "synthetic (seeded x0/latent/waypoints, SIREN-init weights seed 0; real weights are LFS pointers)",
        "config": {"workload": f"C3/C4: batch={B} instances per GPU x N={N}, RTI preparation phase "
                               "(SDF fwd+d/dpos, ERK4+sens, NLS, h+J_h), 'att' model, default flags",
                   "phase": "preparation (acados rti_phase=1 semantics); full RTI with the QP in full_rti",
                   "global_batch": total, "horizon": N, "parallelism": f"instances sharded over {world} GPU(s)",
                   "tile_rows": args.tile_rows},
        "p50_step_ms": p50,
        "kernel_ms": kms,
        "roofline": {"bound": "mfma", "kernel": "sdf_mlp", "achieved": achieved, "peak": FP32_MFMA_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": achieved / FP32_MFMA_PEAK_TFLOPS, "traffic": traffic,
                     "flop_per_launch": sdf_flop},
        "roofline_linearize": {"bound": "hbm", "achieved": lin_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": lin_gbs / HBM_PEAK_GBS, "bytes_per_launch": lin_b},
        "cpu_baseline": cpu,
        "full_rti": full,
    }
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
