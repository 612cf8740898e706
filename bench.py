#!/usr/bin/env python3
"""Benchmark: NMPC RTI throughput at batch x N = 1024 x 40 per GPU (BASELINE.json config C3/C4).

    python bench.py --gpus N --steps K --warmup W
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A "step" is one SQP-RTI solve (acados SQP_RTI, sdf_nmpc/ocp.py:110) for every one of the B instances
on this GPU: the preparation phase over all N+1 shooting nodes (SDF forward + position-Jacobian, ERK4 +
forward sensitivities, NONLINEAR_LS residual/Jacobian, h = [hfov, vfov, sdf] and its Jacobian --
SURVEY.md §8(d)'s unit of work), the feedback phase (the batched QP, rti_qp.hip) and the iterate
update with u_0.  Every step starts from the same initial iterate (a device copy inside the timed
region), so each one is a fresh solve of the same synthetic batch.  Inputs are resident in HBM before
the timed region.  value = instances x steps / time over ALL ranks (weak scaling: B instances per GPU).
The preparation phase alone is timed in its own loop ("prep").  One process per GPU; instances never
interact, so there is no data-path collective; RCCL broadcasts the packed weights once at init.
"""
import argparse
import json
import os
import sys
import time

import numpy as np


def host_cpus():
    """The host CPUs the CPU-baseline leg runs on: every CPU this process may be scheduled on
    (sched_getaffinity), with nproc, the cgroup CPU quota and the CPU model recorded beside it."""
    import subprocess
    info = {"nproc": os.cpu_count() or 1}
    try:
        info["affinity"] = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        info["affinity"] = info["nproc"]
    quota = None
    try:  # cgroup v2: "max 100000" or "<quota> <period>"
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            quota = None if q == "max" else round(int(q) / int(per), 2)
    except (OSError, ValueError):
        pass
    info["cgroup_cpu_quota"] = quota
    # threads that can run at once: the affinity set, capped by the cgroup's CPU quota (oversubscribing a
    # 16-CPU quota with 256 threads measured 2.4x slower on the GPU box than 16 threads)
    usable = info["affinity"] if quota is None else max(1, min(info["affinity"], int(quota + 0.5)))
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        for line in out.splitlines():
            k, _, v = line.partition(":")
            if k.strip() in ("Model name", "Socket(s)", "Core(s) per socket", "Thread(s) per core"):
                info[k.strip()] = v.strip()
    except (OSError, subprocess.SubprocessError):
        pass
    try:
        info["physical_cores"] = int(info["Core(s) per socket"]) * int(info["Socket(s)"])
    except (KeyError, ValueError):
        info["physical_cores"] = None
    return usable, info

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

SDF_FLOP_PER_ROW = 553_984      # fwd 138,456 MAC + d/dpos 138,536 MAC, x2
SDF_FLOP_PER_INST = 98_304      # hoisted latent GEMVs per instance
FP32_MFMA_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: Peak FP32 (matrix)
BF16_MFMA_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: Peak BF16 MFMA, dense (~2.5 PF)
FP64_PEAK_TFLOPS = 78.6         # AMD MI355X spec: FP64 vector = FP64 matrix (not in the guide's table)
# QP algorithmic FLOP per node per IPM iteration (rti_qp.hip): factor stage
# W = P G 1500 + M' = G_ab^T W 2100 + fold 330 + chol/solves 240 + Y^T Y 484 + A~ = A + B K 440 FMA,
# two forward matvecs 2 x 170, corrector 270 FMA (5,704 FMA), ~200 FLOP of row updates
QP_FLOP_PER_NODE_ITER = 11_608
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
    ap.add_argument("--cpu-sample", type=int, default=0,
                    help="instances in the CPU-baseline sample (0: the whole per-GPU batch)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--quiet", action="store_true")
    ap.add_argument("--prep-steps", type=int, default=50, help="timed preparation-only steps (0: skip)")
    ap.add_argument("--no-b1", action="store_true", help="skip the B=1 latency probe (profiling runs)")
    ap.add_argument("--no-c2", action="store_true", help="skip the CasADi-external (libsdf_l4c.so) call leg")
    ap.add_argument("--no-c1", action="store_true", help="skip the B=1, N=20 controller-step leg (config C1)")
    ap.add_argument("--no-scene", action="store_true", help="skip the obstacle-scene SDF side leg")
    ap.add_argument("--no-c5", action="store_true", help="skip the config-C5 sub-block of the default line")
    ap.add_argument("--config", choices=("c3", "c5"), default="c3",
                    help="c3: the headline 1024 x 40 RTI (default); c5: 4x-wide SDF MLP + in-loop VAE encode, "
                         "N = 60, 4096 instances over 8 GPUs (512 per GPU)")
    args = ap.parse_args()
    if args.config == "c5":
        return main_c5(args)

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    # SDFNMPC_DIST_BACKEND=gloo rehearses the multi-rank path with several ranks on one GPU (the 1-GPU
    # test box); the product run is one rank per GPU over RCCL ("nccl")
    backend = os.environ.get("SDFNMPC_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

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

    x_init, u_init = bufs["x"].clone(), bufs["u"].clone()
    # the solver object writes the measured state into node 0 of the iterate before every step
    # (Ocp.solve: solver.set(0, 'x', x0), ocp.py:161; sdfnmpc_solver_step, csrc/solver.hip): the
    # restored initial iterate carries it, so every timed step linearises node 0 at x0 as the controller does
    x_init[:, 0].copy_(bufs["x0"])

    def prep():  # preparation phase only (linearisation + the QP's stage records)
        _lib.rti_prepare(ctx, net, model, qopts, B, N, np_, bufs)

    def step():  # one SQP-RTI solve from the initial iterate: preparation, feedback (QP), update + u_0
        bufs["x"].copy_(x_init)
        bufs["u"].copy_(u_init)
        _lib.rti_prepare(ctx, net, model, qopts, B, N, np_, bufs)  # preparation: linearisation + QP records
        _lib.qp_feedback(ctx, qopts, B, N, bufs)                     # feedback: the IPM
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
    it = bufs["iters"].cpu().numpy()
    st = bufs["status"].cpu().numpy()

    # control-step latency: each step synchronised on its own
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
    reps = max(5, min(args.steps, 20))
    for _ in range(reps):
        step()
    names = ("sdf_hoist", "sdf_mlp", "linearize", "rti_qp_pack", "rti_qp", "rti_apply")
    kst = {k: ctx.kernel_stats(k) for k in names}
    ctx.enable_timing(False)
    kms = {k: (v[0] / v[1] if v[1] else None) for k, v in kst.items()}
    rows = B * (N + 1)
    sdf_flop = rows * SDF_FLOP_PER_ROW
    sdf_tf = sdf_flop / (kms["sdf_mlp"] * 1e-3) / 1e12
    lin_b = B * lin_bytes_per_instance(N)
    lin_gbs = lin_b / (kms["linearize"] * 1e-3) / 1e9  # beside sdf_mlp, as the step runs it
    # linearize alone: a second context with the serial preparation (SDFNMPC_SERIAL_PREP is read at context
    # creation), the same buffers, HIP events around the kernel (untimed diagnostic pass)
    lin_alone_ms = lin_events_ms = None
    if rank == 0:
        prev_sp = os.environ.get("SDFNMPC_SERIAL_PREP")
        os.environ["SDFNMPC_SERIAL_PREP"] = "1"
        try:
            ctx_s = _lib.Context(local, stream=stream, tile_rows=args.tile_rows)
        finally:
            if prev_sp is None:
                del os.environ["SDFNMPC_SERIAL_PREP"]
            else:
                os.environ["SDFNMPC_SERIAL_PREP"] = prev_sp
        _lib.linearize(ctx_s, net, model, B, N, np_, bufs)
        ctx_s.enable_timing(True)
        ctx_s.reset_stats()
        for _ in range(5):
            _lib.linearize(ctx_s, net, model, B, N, np_, bufs)
        v = ctx_s.kernel_stats("linearize")
        ctx_s.synchronize()
        lin_events_ms = v[0] / v[1] if v[1] else None  # an event pair around each launch (adds its own gap)
        # the kernel alone: 20 back-to-back launches without the SDF kernels (no_sdf: the sdf row is not
        # written; linearize's work does not depend on it) between one event pair -- rocprofv3's per-launch
        # mean is the same figure (profiles/r06/kernel_stats_bench.csv)
        ctx_s.enable_timing(False)
        reps = 20
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            _lib.linearize(ctx_s, None, model, B, N, np_, bufs, no_sdf=True)
        e1.record()
        e1.synchronize()
        lin_alone_ms = e0.elapsed_time(e1) / reps
        _lib.linearize(ctx_s, net, model, B, N, np_, bufs)  # the sdf rows back for the steps after
        ctx_s.synchronize()
        del ctx_s
    qp_flop = float(it.sum()) * (N + 1) * QP_FLOP_PER_NODE_ITER
    qp_tf = qp_flop / (kms["rti_qp"] * 1e-3) / 1e12

    # preparation phase alone (acados rti_phase=1), same protocol
    prep_out = None
    if args.prep_steps > 0:
        for _ in range(3):
            prep()
        pel = timed(prep, args.prep_steps)
        prep_out = {"value": total * args.prep_steps / pel, "unit": "instance-RTI-preparations/s",
                    "ms_per_step": pel / args.prep_steps * 1e3, "steps": args.prep_steps}

    # B = 1, N = horizon: the single-instance control-step latency (BASELINE.json config C2)
    lat1 = None
    if rank == 0 and not args.no_b1:
        b1 = {k: (v[:1].clone() if v.dim() > 0 and v.shape[0] == B else v) for k, v in bufs.items()}
        b1["dt"] = bufs["dt"]
        x1, u1_, u01 = b1["x"].clone(), b1["u"].clone(), torch.empty((1, 4), dtype=torch.float64, device=dev)
        x1[:, 0].copy_(b1["x0"])  # ocp.py:161, as above

        rti1 = _lib.RtiStep(ctx, net, model, qopts, 1, N, np_, b1, u0=u01)  # argument blocks bound once

        def step1():
            b1["x"].copy_(x1)
            b1["u"].copy_(u1_)
            rti1()
        for _ in range(5):
            step1()
        l1 = []
        for _ in range(30):
            torch.cuda.synchronize(dev)
            s0 = time.perf_counter()
            step1()
            torch.cuda.synchronize(dev)
            l1.append((time.perf_counter() - s0) * 1e3)
        lat1 = float(np.median(l1))

    # config C2 as acados drives it: the CasADi external functions of libsdf_l4c.so, called per shooting
    # node (sdf_l4c, then jac_sdf_l4c on the same input; gen_model.py:39,60), N + 1 nodes per RTI
    c2 = None
    if rank == 0 and not args.no_c2:
        c2 = bench_c2(local, N, W, args.no_cpu_baseline)
    # config C1 (B = 1, N = 20) through the controller API
    c1 = None
    if rank == 0 and not args.no_c1:
        c1 = bench_c1(local, args.no_cpu_baseline)

    # the headline workload's size on the obstacle-scene SDF net (active / releasing SDF rows)
    scene = None
    if rank == 0 and not args.no_scene:
        scene = bench_scene(local, B, N)
    # config C5 at its per-GPU size (512 instances x N = 60, VAE encode + 4x-wide SDF + RTI), under the
    # driver's clock: the same leg as `bench.py --config c5` (c5_leg), 10 timed steps
    c5 = None
    if rank == 0 and world == 1 and not args.no_c5:
        c5 = c5_leg(local, dev, 1, 0, 512, 60, 10, 3, args.no_cpu_baseline)
        for k in ("metric", "n_gpus", "higher_is_better", "vs_baseline", "data"):
            c5.pop(k, None)
    # traffic from the committed PMC profile of this same command (profiles/)
    traffic = None
    pmc_path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if os.path.exists(pmc_path):
        try:
            with open(pmc_path) as f:
                pmc = json.load(f)
            if pmc.get("B") == B and pmc.get("N") == N and pmc.get("tile_rows") == args.tile_rows:
                traffic = {k: pmc["kernels"][k]["hbm_bytes_per_launch"] for k in ("rti_qp", "sdf_mlp")}
                sys.path.insert(0, os.path.join(ROOT, "tools"))
                from pmc_summary import kernel_sources_sha16
                traffic["source"] = {"file": "profiles/pmc_summary.json", "commit": pmc.get("commit"),
                                     "kernel_sources_match": pmc.get("kernel_sources_sha16") == kernel_sources_sha16(ROOT)}
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU baseline leg only (the "port")
        O.build()
        threads, host = host_cpus()
        S = B if args.cpu_sample <= 0 else min(args.cpu_sample, B)
        onet = O.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=0))
        om = O.quad_model(cfg)
        sub = {k: np.ascontiguousarray(prob[k][:S]) for k in ("x", "u", "p", "yref", "W", "yN", "WN")}
        sub["dt"] = prob["dt"]

        def cpu_rti(n, nth):  # one SQP-RTI solve of n instances on the host: preparation + QP
            sl = {k: (v if k == "dt" else v[:n]) for k, v in sub.items()}
            lin = O.linearize_batch(om, onet, sl["x"], sl["u"], sl["p"], dt, nthreads=nth)
            return O.qp_ipm_batch(lin, sl, x0[:n], quad, nthreads=nth)
        cpu_rti(2, threads)  # warm
        reps = []
        for _ in range(2):  # the whole sample twice: the better pass is the rate
            c0 = time.perf_counter()
            cpu_rti(S, threads)
            reps.append(time.perf_counter() - c0)
        cpu_s = min(reps)
        S1 = 32
        c0 = time.perf_counter()
        cpu_rti(S1, 1)
        cpu1_s = time.perf_counter() - c0
        cpu = {"value": S / cpu_s, "unit": "instance-RTI-solves/s (prep + QP)", "cores": threads, "kind": "port",
               "sample": f"{S} of the {B} instances x {N + 1} nodes, best of 2 passes ({reps[0]:.2f} s, {reps[1]:.2f} s "
                         f"wall on {threads} threads): C oracle preparation (oracle/oracle.c, fp32 MLP + fp64 "
                         f"linearisation) + structured Riccati IPM QP (oracle/qp_ipm.c), OpenMP over instances on "
                         f"every CPU the process may use at once (affinity set capped by the cgroup CPU quota); 1-thread rate on {S1} instances = {S1 / cpu1_s:.1f}/s",
               "value_1thread": S1 / cpu1_s, "host": host,
               # not measured: the whole host is not this process's to use (cgroup quota); the 1-thread rate
               # x the host's physical cores is the ideal-scaling bound of an all-core run
               "projected_all_cores": (S1 / cpu1_s * host["physical_cores"]) if host.get("physical_cores") else None}

    out = {
        "metric": "NMPC solves/sec at batch×N=1024×40 on 1/2/4/8 GPUs; p50 control-step latency",
        "value": value,
        "unit": "instance-RTI-solves/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong" if args.global_batch > 0 else "weak",
        "vs_baseline": None,
        "dtype": "f64 (QP, linearisation) + f32 (SDF MLP on MFMA)",
        "data": "synthetic (seeded x0/latent/waypoints, SIREN-init weights seed 0; real weights are LFS pointers)",
        "config": {"workload": f"C3/C4: batch={B} instances per GPU x N={N}, one SQP-RTI solve per step "
                               "(preparation: SDF fwd+d/dpos, ERK4+sens, NLS, h+J_h; feedback: batched Riccati IPM "
                               "QP to tol 1e-8; iterate update), 'att' model, default flags",
                   "global_batch": total, "horizon": N, "parallelism": f"instances sharded over {world} GPU(s)",
                   "tile_rows": args.tile_rows},
        "p50_step_ms": p50,
        "p50_step_ms_b1": lat1,
        "qp_iters_mean": float(it.mean()), "qp_iters_max": int(it.max()), "qp_converged_frac": float((st == 0).mean()),
        "kernel_ms": kms,
        "roofline": {"bound": "mfma", "kernel": "rti_qp", "achieved": qp_tf, "peak": FP64_PEAK_TFLOPS,
                     "unit": "TFLOP/s", "frac": qp_tf / FP64_PEAK_TFLOPS,
                     "traffic": traffic["rti_qp"] if traffic else None, "flop_per_launch": qp_flop,
                     "traffic_source": traffic["source"] if traffic else None,
                     "note": "latency-bound serial Riccati recursion (one wavefront per instance); f64 peak"},
        "roofline_sdf": {"bound": "mfma", "kernel": "sdf_mlp", "achieved": sdf_tf, "peak": FP32_MFMA_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": sdf_tf / FP32_MFMA_PEAK_TFLOPS,
                         "traffic": traffic["sdf_mlp"] if traffic else None, "flop_per_launch": sdf_flop},
        "roofline_linearize": {"bound": "hbm", "achieved": lin_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": lin_gbs / HBM_PEAK_GBS, "bytes_per_launch": lin_b,
                               "note": "achieved over the kernel's duration beside sdf_mlp (the step's schedule)",
                               "alone": None if lin_alone_ms is None else {
                                   "ms": lin_alone_ms, "achieved": lin_b / (lin_alone_ms * 1e-3) / 1e9,
                                   "frac": lin_b / (lin_alone_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                   "timing": "20 back-to-back launches between one event pair",
                                   "ms_event_pair_per_launch": lin_events_ms}},
        "cpu_baseline": cpu,
        "prep": prep_out,
        "c2": c2,
        "c1": c1,
        "scene": scene,
        "c5": c5,
    }
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def bench_c1(device, no_cpu, steps=200):
    """BASELINE.json configs[0] (C1): one quadrotor, N = 20, the controller's own control step
    (Nmpc.set_x0 + Nmpc.solve: host arrays in, u_0 out, controller.py:72-81) repeated with the iterate
    carried, p50 / p99 wall time per step.  Beside it the same closed loop on the host (the C oracle's
    preparation phase and structured IPM, one thread), the CPU plumbing C1 names."""
    from sdf_nmpc_amd.config import Config
    from sdf_nmpc_amd.controller import Nmpc
    from sdf_nmpc_amd.reference import Ref, yaw2quat
    N = 20
    cfg = Config(mpc__N=N)
    n = Nmpc(cfg, batch=1, device=device)
    rng = np.random.default_rng(11)
    x0 = np.zeros(10)
    x0[:3] = rng.uniform(-1, 1, 3)
    x0[3:7] = yaw2quat(0.2)
    n.set_sdf_flag(1.0)
    n.set_latent(rng.normal(0, 1, 128), x0[:3] + 0.1, np.eye(3))
    r = Ref(cfg)
    r.p, r.q = x0[:3] + np.array([2.0, -1.0, 0.5]), yaw2quat(0.3)
    r.use_weights(r.W_on)
    for k in range(N + 1):
        n.set_ref(r, k)
    ts = []
    for i in range(steps + 10):
        t0 = time.perf_counter()
        n.set_x0(x0)
        n.solve()
        t1 = time.perf_counter()
        if i >= 10:
            ts.append((t1 - t0) * 1e3)
    res = {"p50_step_ms": float(np.percentile(ts, 50)), "p99_step_ms": float(np.percentile(ts, 99)), "steps": steps,
           "path": "Nmpc.set_x0 + Nmpc.solve (host arrays, solver object, one SQP-RTI iteration), B=1, N=20"}
    if not no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU baseline leg only (the "port")
        O.build()
        from sdf_nmpc_amd import weights as W
        onet = O.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=0))
        om = O.quad_model(cfg)
        dt = n.ocp.dt
        xs = np.repeat(x0[None, None], N + 1, axis=1)
        us = np.broadcast_to(n.model.u_hover, (1, N, 4)).copy()
        p = n.p.reshape(1, N + 1, -1)
        prob = {"yref": n.y.reshape(1, N, -1), "W": n.W.reshape(1, N, -1), "yN": n.yN.reshape(1, -1),
                "WN": n.WN.reshape(1, -1), "dt": dt}
        cs = []
        for i in range(steps + 5):
            t0 = time.perf_counter()
            xs[:, 0] = x0
            lin = O.linearize_batch(om, onet, xs, us, p, dt, nthreads=1)
            q = O.qp_ipm_batch(lin, dict(prob, x=xs, u=us), x0[None], n.model, nthreads=1)
            xs, us = xs + q["dx"], us + q["du"]
            t1 = time.perf_counter()
            if i >= 5:
                cs.append((t1 - t0) * 1e3)
        res["cpu_baseline"] = {"p50_step_ms": float(np.percentile(cs, 50)), "p99_step_ms": float(np.percentile(cs, 99)),
                               "cores": 1, "kind": "port",
                               "sample": f"{steps} closed-loop steps of the same problem: C oracle preparation "
                                         "(oracle/oracle.c) + structured Riccati IPM (oracle/qp_ipm.c), one thread"}
    n.ocp.close()
    return res


def bench_scene(device, B=1024, N=40, warm_steps=6, steps=10):
    """Side leg (not the headline): the headline's batch and horizon with the SDF network fitted to an obstacle
    scene (tests/golden/scene.sdfw, tools/fit_scene_sdf.py; tests/scene_setup.py) instead of the SIREN
    initialisation, whose df ~ 0 makes every SDF row of every QP active.  B instances start at x in [0, 2.5] m
    and lateral offsets in [-1, 1.5] m and fly towards a waypoint beyond the pillar; the loop is closed with a
    perfect-model plant (x_0 of the next step = node 1 of the updated iterate).  After `warm_steps` steps
    (the pillar inside most horizons), `steps` further steps are timed per kernel (HIP events): the rti_qp
    time and IPM iterations on this net, and how many instances have an active SDF soft row."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import scene_setup as S
    from sdf_nmpc_amd.config import Config
    from sdf_nmpc_amd.controller import Nmpc
    from sdf_nmpc_amd.model import Quad
    from sdf_nmpc_amd.ocp import Ocp
    cfg = Config(mpc__N=N)
    o = Ocp(Quad(cfg), batch=B, device=device, weights=S.SCENE)
    n = Nmpc(cfg, batch=B, ocp=o)
    rng = np.random.default_rng(77)
    x = S.setup(n, y0=rng.uniform(-1.0, 1.5, B))
    x[:, 0] = rng.uniform(0.0, 2.5, B)
    for _ in range(warm_steps):
        n.set_x0(x)
        n.solve()
        x = n.get_matrices()[0][:, 1].copy()
    o.ctx.enable_timing(True)
    o.ctx.reset_stats()
    iters, active, wall = [], [], []
    for _ in range(steps):
        n.set_x0(x)
        t0 = time.perf_counter()
        n.solve()
        wall.append(time.perf_counter() - t0)
        iters.append(o.iters.copy())
        sl = o.download("slack").reshape(B, N + 1, 3, 2)
        active.append((sl[:, :, 2, 0] > 1e-6).any(axis=1))
        x = n.get_matrices()[0][:, 1].copy()
    kms = {k: (v[0] / v[1] if v[1] else None) for k, v in
           ((k, o.ctx.kernel_stats(k)) for k in ("sdf_mlp", "linearize", "rti_qp", "rti_qp_pack"))}
    o.ctx.enable_timing(False)
    it = np.array(iters)
    res = {"workload": f"{B} instances x N={N}, obstacle-scene SDF net (deployed architecture fitted to a pillar "
                       f"and a box), closed loop past the pillar, timed steps {warm_steps}..{warm_steps + steps - 1}",
           "kernel_ms": kms, "qp_iters_max": int(it.max()), "qp_iters_mean": float(it.mean()),
           "qp_iters_max_per_step": [int(v) for v in it.max(axis=1)],
           "sdf_active_frac": float(np.mean(active)), "instances_with_active_sdf_row_per_step":
               [int(v) for v in np.sum(active, axis=1)],
           "solve_wall_ms_p50": float(np.median(wall) * 1e3)}
    o.close()
    return res


def bench_c2(device, N, W, no_cpu, rtis=30):
    """Per-call latency of the acados drop-in (include/sdf_l4c.h) through ctypes: every RTI evaluates
    sdf_l4c and jac_sdf_l4c (1 x 131 Jacobian) at each of the N + 1 nodes, one instance, one latent.
    Beside it: the same value + 131-gradient from the C oracle's fp32 network on one host thread."""
    import ctypes as C
    import tempfile
    from sdf_nmpc_amd import _lib
    lib = C.CDLL(_lib.l4c_path())
    D = 131
    with tempfile.NamedTemporaryFile(suffix=".sdfw", delete=False) as f:
        f.write(W.pack(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=0)))
        wpath = f.name
    lib.sdf_l4c_configure.argtypes = [C.c_char_p, C.c_int]
    if lib.sdf_l4c_configure(wpath.encode(), device) != 0:
        raise RuntimeError("sdf_l4c_configure failed")
    os.unlink(wpath)
    rng = np.random.default_rng(5)
    lat = rng.normal(size=128)
    inp = np.empty((N + 1, D))
    inp[:, :3] = rng.uniform(-2, 2, (N + 1, 3))
    inp[:, 3:] = lat
    out = np.empty(N + 1)
    jac = np.empty((N + 1, D))
    PD = C.POINTER(C.c_double)
    a1 = [(PD * 1)(inp[k].ctypes.data_as(PD)) for k in range(N + 1)]
    a2 = [(PD * 2)(inp[k].ctypes.data_as(PD), out[k:k + 1].ctypes.data_as(PD)) for k in range(N + 1)]
    r1 = [(PD * 1)(out[k:k + 1].ctypes.data_as(PD)) for k in range(N + 1)]
    r2 = [(PD * 1)(jac[k].ctypes.data_as(PD)) for k in range(N + 1)]
    f, jf = lib.sdf_l4c, lib.jac_sdf_l4c

    def rti():
        for k in range(N + 1):
            if f(a1[k], r1[k], None, None, 0) or jf(a2[k], r2[k], None, None, 0):
                raise RuntimeError("sdf_l4c call failed")
    for _ in range(3):
        rti()
    ts = []
    for _ in range(rtis):
        t0 = time.perf_counter()
        rti()
        ts.append(time.perf_counter() - t0)
    per_rti = float(np.median(ts))
    res = {"us_per_node": per_rti / (N + 1) * 1e6, "ms_per_rti": per_rti * 1e3, "nodes_per_rti": N + 1,
           "calls": "sdf_l4c + jac_sdf_l4c per node (ctypes, fp64 in/out, value and 1x131 Jacobian)"}
    # the same calls from C (tools/c2_driver.c, a child process): acados's own call path, no Python per call
    drv = os.path.join(ROOT, "tools", "_c2_driver")
    if os.path.exists(drv):
        import subprocess
        with tempfile.NamedTemporaryFile(suffix=".sdfw", delete=False) as f:
            f.write(W.pack(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=0)))
            wpath2 = f.name
        try:
            r = subprocess.run([drv, _lib.l4c_path(), wpath2, str(device), str(N + 1), str(rtis)],
                               capture_output=True, text=True, timeout=120)
            if r.returncode == 0:
                res["c_driver"] = json.loads(r.stdout.strip().splitlines()[-1])
        finally:
            os.unlink(wpath2)
    if not no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        O.build()
        onet = O.Net(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, seed=0))
        onet.f32(inp[:1])
        t0 = time.perf_counter()
        reps = 200
        for k in range(reps):
            onet.f32(inp[k % (N + 1):k % (N + 1) + 1], nthreads=1)
        cpu_us = (time.perf_counter() - t0) / reps * 1e6
        res["cpu_baseline"] = {"us_per_node": cpu_us, "cores": 1, "kind": "port",
                               "sample": f"{reps} single-row fp32 value + 131-gradient evaluations, C oracle "
                                         "(oracle/sdf_net.inc) on one host thread, as L4CasADi runs torch with "
                                         "set_num_threads(1) (gen_model.py:27)"}
    return res


def main_c5(args):
    """BASELINE.json configs[4]: per control step and instance, a new 1x270x480 depth image is encoded by
    the VAE (sdf_nmpc/vae.py:37-40) into the latent that parameterises the 4x-wide SDF
    (set_latent, controller.py:50-54), then one SQP-RTI solve at N = 60 runs with that SDF.  Weak scaling:
    512 instances per GPU (4096 over 8 GPUs)."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run")
    backend = os.environ.get("SDFNMPC_DIST_BACKEND", "nccl")  # gloo: rehearsal with ranks sharing a GPU
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
    from sdf_nmpc_amd import shard
    N = args.horizon if args.horizon != 40 else 60
    B = args.batch if args.batch != 1024 else 512
    if args.global_batch > 0:
        lo, hi = shard.instance_range(args.global_batch, world, rank)
        B = hi - lo
    steps = args.steps if args.steps != 50 else 10
    warm = args.warmup if args.warmup != 10 else 3
    out = c5_leg(local, dev, world, rank, B, N, steps, warm, args.no_cpu_baseline, args.global_batch)
    if rank == 0:
        print(json.dumps(out))
    if world > 1:
        dist.destroy_process_group()


def c5_leg(local, dev, world, rank, B, N, steps, warm, no_cpu, global_batch=0):
    """Config C5 on this GPU (main_c5, and the c5 sub-block of the default line): B instances at horizon N,
    per step the VAE encode of B depth images, the latents packed into p on the device, one SQP-RTI solve
    with the 4x-wide SDF.  Returns the C5 result dict (value over all ranks)."""
    import torch
    import torch.distributed as dist
    from sdf_nmpc_amd import _lib, shard, synth, vae as V, weights as W
    from sdf_nmpc_amd.config import Config
    from sdf_nmpc_amd.model import Quad
    cfg = Config(mpc__N=N)
    ctx = _lib.Context(local, stream=torch.cuda.current_stream(dev).cuda_stream)
    blob = W.pack(W.WIDE_SPEC, W.siren_weights(W.WIDE_SPEC, seed=0)) if rank == 0 else None
    vblob = V.pack(V.DEFAULT_ENCODER, V.synthetic_encoder(V.DEFAULT_ENCODER, 0)) if rank == 0 else None
    if world > 1:
        blob = shard.broadcast_blob(blob, dev)
        vblob = shard.broadcast_blob(vblob, dev)
    net = _lib.Net.from_blob(ctx, blob)
    vae = _lib.Vae(ctx, vblob)
    model = _lib.quad_model(cfg)
    quad = Quad(cfg)
    nodes, dt = _lib.shooting_grid(N, cfg.mpc.T)
    prob = synth.make_problem(cfg, B, N, seed=1000 + rank, dt=dt)
    bufs = {k: torch.from_numpy(np.ascontiguousarray(prob[k])).to(dev) for k in ("x", "u", "p", "dt")}
    for k, sh in dict(xn=(B, N, 10), AB=(B, N, 14, 10), y=(B, N, 11), Jy=(B, N, 14, 11), yN=(B, 4),
                      JyN=(B, 10, 4), h=(B, N + 1, 3), Jh=(B, N + 1, 10, 3)).items():
        bufs[k] = torch.empty(sh, dtype=torch.float64, device=dev)
    np_ = prob["p"].shape[-1]
    x0 = prob["x"][:, 0] + np.random.default_rng(2000 + rank).normal(0, 0.05, (B, 10))
    for k, v in dict(x0=x0, yref=prob["yref"], W=prob["W"], yNref=prob["yN"], WN=prob["WN"]).items():
        bufs[k] = torch.from_numpy(np.ascontiguousarray(v)).to(dev)
    for k, sh in dict(dx=(B, N + 1, 10), du=(B, N, 4), res=(B, 2)).items():
        bufs[k] = torch.empty(sh, dtype=torch.float64, device=dev)
    bufs["status"] = torch.empty(B, dtype=torch.int32, device=dev)
    bufs["iters"] = torch.empty(B, dtype=torch.int32, device=dev)
    u0 = torch.empty((B, 4), dtype=torch.float64, device=dev)
    qopts = _lib.qp_opts(quad)
    # depth images (resident in HBM), Depth2Range table, latents, camera pose at image time
    imgs = torch.from_numpy(synth.depth_images(min(B, 16), 270, 480, seed=rank)).to(dev)
    imgs = imgs.repeat((B + 15) // 16, 1, 1)[:B].contiguous()
    yz = torch.from_numpy(V.depth2range_table(cfg.sensor.shape_imgs, cfg.sensor.hfov, cfg.sensor.vfov)).to(dev)
    vopts = _lib.vae_opts(cfg, V.clip_scale(cfg))
    lat32 = torch.empty((B, 128), dtype=torch.float32, device=dev)
    lat64 = torch.empty((B, 128), dtype=torch.float64, device=dev)
    W_p_Bo = torch.from_numpy(np.ascontiguousarray(prob["x"][:, 0, :3])).to(dev)
    from sdf_nmpc_amd.model import quat2rot
    W_R_Bo = torch.from_numpy(np.ascontiguousarray(quat2rot(prob["x"][:, 0, 3:7]).reshape(B, 9))).to(dev)
    ropts = _lib.ref_opts(cfg, -1)
    rargs = {"latent": lat64, "W_p_Bo": W_p_Bo, "W_R_Bo": W_R_Bo, "p": bufs["p"]}
    x_init, u_init = bufs["x"].clone(), bufs["u"].clone()
    x_init[:, 0].copy_(bufs["x0"])  # ocp.py:161: node 0 of the iterate = the measured state

    def step():  # image -> latent -> p (set_latent) -> SQP-RTI solve from the initial iterate
        _lib.vae_encode(ctx, vae, vopts, imgs, yz, lat32, lat64)
        _lib.pack_refs(ctx, ropts, B, N, np_, 11, rargs, L=128)
        bufs["x"].copy_(x_init)
        bufs["u"].copy_(u_init)
        _lib.rti_prepare(ctx, net, model, qopts, B, N, np_, bufs)  # preparation: linearisation + QP records
        _lib.qp_feedback(ctx, qopts, B, N, bufs)                     # feedback: the IPM
        _lib.rti_apply(ctx, B, N, bufs["x"], bufs["u"], bufs["dx"], bufs["du"], u0)

    def timed(fn, k):
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for _ in range(k):
            fn()
        torch.cuda.synchronize(dev)
        if world > 1:
            dist.barrier()
        el = time.perf_counter() - t0
        return shard.max_over_ranks(el, dev) if world > 1 else el

    for _ in range(warm):
        step()
    el = timed(step, steps)
    total = global_batch if global_batch > 0 else world * B
    it = bufs["iters"].cpu().numpy()
    st = bufs["status"].cpu().numpy()
    ctx.enable_timing(True)
    ctx.reset_stats()
    reps = 5
    for _ in range(reps):
        step()
    names = ("vae_pre", "vae_stem", "vae_conv", "vae_head", "sdf_wide_hoist", "sdf_wide_emb", "sdf_wide_gemm",
             "sdf_wide_final", "linearize", "ref_pack", "rti_qp_pack", "rti_qp", "rti_apply")
    kms = {k: ctx.kernel_stats(k)[0] / reps for k in names}  # ms per step (all launches of that name)
    ctx.enable_timing(False)
    spec = V.DEFAULT_ENCODER
    vae_flop = spec.n_flops() * B
    conv_flop = vae_flop - 2 * B * (135 * 240 * 64 * 49 + 2048 * 128)
    rows = B * (N + 1)
    wide_flop = rows * 7_326_976 + B * 2 * 128 * (1024 + 512)
    vae_ms = sum(kms[k] for k in ("vae_pre", "vae_stem", "vae_conv", "vae_head"))
    wide_ms = sum(kms[k] for k in ("sdf_wide_hoist", "sdf_wide_emb", "sdf_wide_gemm", "sdf_wide_final"))
    conv_tf = conv_flop / (kms["vae_conv"] * 1e-3) / 1e12
    wide_tf = (wide_flop - B * 2 * 128 * 1536) / (kms["sdf_wide_gemm"] * 1e-3) / 1e12
    out = {
        "metric": "NMPC solves/sec, config C5: 4x-wide SDF MLP + in-loop VAE encode, N=60, batch 4096 over 8 GPUs",
        "value": total * steps / el,
        "unit": "instance-RTI-solves/s (incl. VAE encode)",
        "n_gpus": world, "steps": steps, "warmup": warm, "ms_per_step": el / steps * 1e3,
        "higher_is_better": True, "scaling": "strong" if global_batch > 0 else "weak", "vs_baseline": None,
        "dtype": "f32 (VAE convs as fp32-exact bf16 splits on the bf16 MFMA; wide SDF MLP on the f32 MFMA) + f64 "
                 "(linearisation, QP)",
        "data": "synthetic depth images (seeded scenes + noise), synthetic VAE weights, SIREN-init wide SDF seed 0",
        "config": {"workload": f"C5: batch={B} instances per GPU x N={N}; per step: VAE encode of B 1x270x480 depth "
                               "images -> latent -> p, then one SQP-RTI solve with the [1024,1024,512,256] SDF",
                   "global_batch": total, "horizon": N, "parallelism": f"instances sharded over {world} GPU(s)"},
        "qp_iters_mean": float(it.mean()), "qp_iters_max": int(it.max()), "qp_converged_frac": float((st == 0).mean()),
        "kernel_ms_per_step": kms,
        # the convolutions run each fp32 product as six bf16 products (csrc/vae_enc.hip): the matrix pipe they
        # load is the bf16 one, so the fraction is of the dense bf16 peak at 6 pipe FLOP per fp32 FLOP;
        # conv_tf (fp32-equivalent work per second) is given beside it
        "roofline": {"bound": "mfma", "kernel": "vae_conv (11 launches, bf16 pipe)", "achieved": 6.0 * conv_tf,
                     "peak": BF16_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": 6.0 * conv_tf / BF16_MFMA_PEAK_TFLOPS,
                     "traffic": None, "flop_per_step": conv_flop, "fp32_equivalent_tflops": conv_tf,
                     "fp32_equivalent_frac_of_f32_mfma_peak": conv_tf / FP32_MFMA_PEAK_TFLOPS},
        "roofline_wide_sdf": {"bound": "mfma", "kernel": "sdf_wide_gemm (9 launches)", "achieved": wide_tf,
                              "peak": FP32_MFMA_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": wide_tf / FP32_MFMA_PEAK_TFLOPS,
                              "note": "fp32 GEMM FLOPs over the f32 MFMA peak; the products run fp32-exact as three-way "
                                      "bf16 splits on the bf16 pipe (sdf_wide.hip SPLIT; SDFNMPC_WIDE_F32=1: f32 MFMA)"},
        "vae_ms": vae_ms, "wide_sdf_ms": wide_ms,
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not no_cpu:
        # the same per-instance work on the host: fp64 C encoder (oracle/vae.c) of the instance's image,
        # the wide network's preparation phase (oracle/oracle.c) and the structured C IPM, a bounded sample
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O  # CPU baseline leg only (the "port")
        O.build()
        S = 4
        threads, host = host_cpus()
        spec = V.DEFAULT_ENCODER
        flat = np.concatenate([V.synthetic_encoder(spec, 0)[n].ravel() for n, _ in spec.param_shapes()])
        yzh = V.depth2range_table(cfg.sensor.shape_imgs, cfg.sensor.hfov, cfg.sensor.vfov)
        img_h = synth.depth_images(S, 270, 480, seed=rank)
        onet = O.Net(W.WIDE_SPEC, W.siren_weights(W.WIDE_SPEC, seed=0))
        om = O.quad_model(cfg)
        sub = {k: np.ascontiguousarray(prob[k][:S]) for k in ("x", "u", "p", "yref", "W", "yN", "WN")}
        sub["dt"] = prob["dt"]
        c0 = time.perf_counter()
        pre = np.stack([O.vae_preprocess(im, (270, 480), V.clip_scale(cfg), yzh) for im in img_h])
        lat = O.vae_encode(pre, flat, nthreads=threads)
        sub["p"][:, :, 17:] = lat[:, None, :]
        lin = O.linearize_batch(om, onet, sub["x"], sub["u"], sub["p"], sub["dt"], nthreads=threads)
        O.qp_ipm_batch(lin, sub, x0[:S], quad, nthreads=threads)
        cpu_s = time.perf_counter() - c0
        out["cpu_baseline"] = {"value": S / cpu_s, "unit": "instance-RTI-solves/s (incl. VAE encode)",
                               "cores": threads, "kind": "port", "host": host,
                               "sample": f"{S} instances: fp64 C encoder (oracle/vae.c, OpenMP) of one 270x480 image "
                                         f"each, the wide network's preparation phase at N={N} and the structured "
                                         "C IPM (oracle/oracle.c, oracle/qp_ipm.c)"}
    ctx.synchronize()
    vae.close()
    net.close()
    ctx.close()
    return out


if __name__ == "__main__":
    main()
