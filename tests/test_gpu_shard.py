"""The sharded RTI of config C4 (BASELINE.json configs[3]) with world_size 2 on one GPU: two processes
over gloo, each solving its shard.instance_range of the batch with the solver object on cuda:0, u_0
gathered to rank 0 -- bitwise equal to one process solving the whole batch (instances never interact,
SURVEY.md §8(e)); and the in-process occupancy gate (Ocp over several device slots) the same way."""
import os
import socket

import numpy as np
import pytest

pytestmark = [pytest.mark.gpu, pytest.mark.filterwarnings("ignore:no SDF weights")]

TOTAL, N = 96, 40


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _solve(lo, hi, ctx):
    """One SQP-RTI step for instances [lo, hi) of the seeded C4-style batch (solver object, no torch)."""
    from sdf_nmpc_amd import _lib, synth, weights as W
    from sdf_nmpc_amd.config import Config
    from sdf_nmpc_amd.model import Quad
    cfg = Config(mpc__N=N)
    model = Quad(cfg)
    _, dt = _lib.shooting_grid(N, cfg.mpc.T)
    prob = synth.make_problem(cfg, TOTAL, N, seed=77, dt=dt)
    x0 = prob["x"][:, 0] + np.random.default_rng(78).normal(0, 0.05, (TOTAL, 10))
    net = _lib.Net.from_blob(ctx, W.pack(W.DEFAULT_SPEC, W.siren_weights(W.DEFAULT_SPEC, 0)))
    s = _lib.Solver(ctx, net, _lib.quad_model(cfg), _lib.qp_opts(model), hi - lo, N, model.np, model.ny, dt)
    sl = slice(lo, hi)
    for name, v in (("x", prob["x"][sl]), ("u", prob["u"][sl]), ("p", prob["p"][sl]), ("x0", x0[sl, None]),
                    ("yref", prob["yref"][sl]), ("W", prob["W"][sl]), ("yNref", prob["yN"][sl, None]),
                    ("WN", prob["WN"][sl, None])):
        s.upload(name, v)
    s.step()
    u0 = s.wait().copy()
    st = s.status.copy()
    s.close()
    net.close()
    return u0, st


def _rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from sdf_nmpc_amd import _lib, shard
        ctx = _lib.Context(0)  # both ranks on the one GPU of the box
        lo, hi = shard.instance_range(TOTAL, world, rank)
        u0, st = _solve(lo, hi, ctx)
        full = shard.gather_rows(torch.from_numpy(u0), TOTAL)
        stat = shard.gather_rows(torch.from_numpy(st.astype(np.int64)[:, None]), TOTAL)
        if rank == 0:
            ref, ref_st = _solve(0, TOTAL, ctx)  # the whole batch in one process
            q.put((full.numpy(), stat.numpy()[:, 0], ref, ref_st))
        ctx.close()
    finally:
        dist.destroy_process_group()


def test_two_rank_sharded_rti_equals_single_process():
    import torch.multiprocessing as mp
    mpc = mp.get_context("spawn")
    q = mpc.Queue()
    port = _free_port()
    procs = [mpc.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    full, st, ref, ref_st = q.get(timeout=240)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert (st == 0).all() and (ref_st == 0).all()
    np.testing.assert_array_equal(full, ref)


def test_qp_capacity_from_the_library():
    """The occupancy gate's capacity comes from the C ABI (sdfnmpc_qp_capacity: device CUs x min(LDS per
    CU // the kernel's LDS per instance, the runtime's occupancy of the kernel -- registers included)) at N
    in {20, 40, 60, 80}.  The serial kernel holds 375 registers, one wave per SIMD: four instances per CU
    even where the LDS would admit seven (N = 20); 1024 instances at N = 20 and 40 on an MI355X."""
    import torch
    from sdf_nmpc_amd import _lib
    ctx = _lib.Context(0)
    prop = torch.cuda.get_device_properties(0)
    cus = prop.multi_processor_count
    lds = 160 * 1024  # gfx950 LDS per CU
    caps = {}
    for N in (20, 40, 60, 80):
        per = int(_lib.load().sdfnmpc_qp_lds_bytes(N))
        assert per > 0
        caps[N] = ctx.qp_capacity(N)
        assert 0 < caps[N] <= cus * min(4, lds // per), (N, caps[N], cus, per)
        if lds // per <= 4:
            assert caps[N] == cus * (lds // per), (N, caps[N], cus, per)
    assert caps[20] == caps[40] == 1024 and caps[40] >= caps[60] >= caps[80] > 0
    assert ctx.qp_capacity(400) == 0  # no instance of that horizon fits one CU's LDS
    with pytest.raises(_lib.SdfnmpcError):
        ctx.qp_capacity(0)


def test_qp_kernel_auto_policy():
    """AUTO (include/sdfnmpc.h): segmented at 36 <= N <= 63 for B <= 256 (512 from N = 48), serial
    otherwise; an explicit choice overrides it; the capacity uses the kernel of a full batch."""
    from sdf_nmpc_amd import _lib
    ctx = _lib.Context(0)
    assert ctx.qp_kernel(40, 1) == "segmented" and ctx.qp_kernel(40, 256) == "segmented"
    assert ctx.qp_kernel(40, 257) == "serial" and ctx.qp_kernel(40, 1024) == "serial"
    assert ctx.qp_kernel(60, 512) == "segmented" and ctx.qp_kernel(60, 513) == "serial"
    assert ctx.qp_kernel(20, 1) == "serial" and ctx.qp_kernel(35, 1) == "serial" and ctx.qp_kernel(36, 1) == "segmented"
    assert ctx.qp_kernel(64, 1) == "serial"  # beyond the segmented kernel's horizon
    ctx.set_qp_kernel("serial")
    assert ctx.qp_kernel(40, 1) == "serial"
    ctx.set_qp_kernel("segmented")
    assert ctx.qp_kernel(40, 1024) == "segmented" and ctx.qp_kernel(20, 1) == "segmented"
    assert ctx.qp_kernel(80, 1) == "serial"  # unsupported horizon: serial whatever is asked
    # the P = 4 segmented kernel's registers (__launch_bounds__(256, 2)) allow two workgroups per CU, fewer
    # than its LDS would (three): the capacity follows the registers
    assert ctx.qp_capacity(40) == 2 * 256
    ctx.set_qp_kernel("auto")
    assert ctx.qp_capacity(40) == 1024


def test_ocp_occupancy_gate_parts_equal_one_part():
    """Ocp over two device slots (both cuda:0 here): a batch above one GPU's capacity at N = 60 (512
    instances) is split into two parts by shard.plan; the result equals a single-part solve bitwise."""
    from sdf_nmpc_amd import shard
    from sdf_nmpc_amd.config import Config
    from sdf_nmpc_amd.controller import Nmpc
    from sdf_nmpc_amd.model import Quad
    from sdf_nmpc_amd.ocp import Ocp
    from sdf_nmpc_amd.reference import Ref, yaw2quat
    Bt, cfg = 600, Config(mpc__N=60)
    from sdf_nmpc_amd import _lib
    cap = _lib.Context(0).qp_capacity(60)
    assert cap == 512 and len(shard.plan(Bt, cap, 2)) == 2 and len(shard.plan(512, cap, 8)) == 1
    rng = np.random.default_rng(4)
    x0 = np.zeros((Bt, 10))
    x0[:, :3] = rng.uniform(-1, 1, (Bt, 3))
    x0[:, 3:7] = np.stack([yaw2quat(y) for y in rng.uniform(-np.pi, np.pi, Bt)])
    lat = rng.normal(size=(Bt, 128))
    r = Ref(cfg)
    r.p, r.q = np.array([1.0, 2.0, 1.5]), yaw2quat(0.3)
    r.use_weights(r.W_on)
    res = []
    for devs in ([0, 0], [0]):
        o = Ocp(Quad(cfg), batch=Bt, devices=devs)
        assert len(o.parts) == len(devs)
        n = Nmpc(cfg, batch=Bt, ocp=o)
        n.set_sdf_flag(1.0)
        n.set_latent(lat, x0[:, :3], np.stack([np.eye(3)] * Bt))
        for k in range(61):
            n.set_ref(r, k)
        n.set_x0(x0)
        assert n.solve() == 0 and n.solve() == 0  # two steps: the carried iterate too
        res.append(n.get_u())
        o.close()
    np.testing.assert_array_equal(res[0], res[1])


def _c4_inputs(cfg, Bt, seed):
    from sdf_nmpc_amd.reference import Ref, yaw2quat
    rng = np.random.default_rng(seed)
    x0 = np.zeros((Bt, 10))
    x0[:, :3] = rng.uniform(-2, 2, (Bt, 3))
    x0[:, 3:7] = np.stack([yaw2quat(y) for y in rng.uniform(-np.pi, np.pi, Bt)])
    x0[:, 7:] = rng.uniform(-1, 1, (Bt, 3))
    lat = rng.normal(size=(Bt, 128))
    r = Ref(cfg)
    r.p, r.q = np.array([1.0, 2.0, 1.5]), yaw2quat(0.3)
    r.use_weights(r.W_on)
    return x0, lat, r


def _c4_run(cfg, x0, lat, r, devices, kernel=None, steps=2):
    from sdf_nmpc_amd.controller import Nmpc
    from sdf_nmpc_amd.model import Quad
    from sdf_nmpc_amd.ocp import Ocp
    Bt = x0.shape[0]
    o = Ocp(Quad(cfg), batch=Bt, devices=devices)
    if kernel is not None:
        for p in o.parts:
            p.ctx.set_qp_kernel(kernel)
    n = Nmpc(cfg, batch=Bt, ocp=o)
    n.set_sdf_flag(1.0)
    n.set_latent(lat, x0[:, :3], np.stack([np.eye(3)] * Bt))
    for k in range(cfg.mpc.N + 1):
        n.set_ref(r, k)
    n.set_x0(x0)
    for _ in range(steps):  # the carried iterate too
        assert n.solve() == 0
    out = dict(u0=n.get_u(), status=o.status.copy(), iters=o.iters.copy(), u=o.download("u"), n_parts=len(o.parts))
    o.close()
    return out


def test_c4_full_batch_through_the_occupancy_gate():
    """BASELINE.json configs[3] (C4) at its real batch: 8192 instances at N = 40 through
    Ocp(devices=[0] * 8) -- the eight device slots of an 8-GPU node, all on the one GPU here.  shard.plan
    splits the batch into eight 1024-instance parts (the occupancy gate, sdfnmpc_qp_capacity); two RTI steps
    converge on every instance, the iterate respects the input boxes, and each part equals the same
    instances solved alone, bit for bit (a part never sees its neighbours)."""
    from sdf_nmpc_amd import _lib, shard
    from sdf_nmpc_amd.config import Config
    from sdf_nmpc_amd.model import Quad
    cfg = Config()
    Bt = 8192
    assert shard.plan(Bt, _lib.Context(0).qp_capacity(40), 8) == [(g, 1024 * g, 1024 * (g + 1)) for g in range(8)]
    x0, lat, r = _c4_inputs(cfg, Bt, 40)
    full = _c4_run(cfg, x0, lat, r, [0] * 8)
    assert full["n_parts"] == 8
    assert (full["status"] == 0).all() and full["iters"].max() < 100
    m = Quad(cfg)
    assert (full["u"] >= m.lbu - 1e-9).all() and (full["u"] <= m.ubu + 1e-9).all()
    for g in (0, 5, 7):  # parts solved alone (the same QP kernel the split pinned: serial at B = 8192)
        sl = slice(1024 * g, 1024 * (g + 1))
        alone = _c4_run(cfg, x0[sl], lat[sl], r, [0], kernel="serial")
        np.testing.assert_array_equal(alone["u0"], full["u0"][sl])
        np.testing.assert_array_equal(alone["iters"], full["iters"][sl])


def test_set_latent_device_multi_part_inputs_from_another_stream():
    """with the batch split into parts, every part after the first reads a device latent in place
    (a view at its first row).  Here latent, W_p_Bo and W_R_Bo are all device arrays of a third context whose
    values are still being written by a kernel on that context's stream (rti_apply: x += dx) when
    set_latent_device is called, and no flag is passed (no host temporary whose free would drain the device).
    The packed parameters and the RTI step must equal those of the host-array path bit for bit."""
    from sdf_nmpc_amd import _lib
    from sdf_nmpc_amd.config import Config
    from sdf_nmpc_amd.controller import Nmpc
    from sdf_nmpc_amd.model import Quad
    from sdf_nmpc_amd.ocp import Ocp
    from sdf_nmpc_amd.reference import Ref, yaw2quat
    Bt, cfg = 600, Config(mpc__N=60)
    rng = np.random.default_rng(9)
    x0 = np.zeros((Bt, 10))
    x0[:, :3] = rng.uniform(-1, 1, (Bt, 3))
    x0[:, 3:7] = np.stack([yaw2quat(y) for y in rng.uniform(-np.pi, np.pi, Bt)])
    lat = rng.normal(size=(Bt, 128))
    R = np.stack([np.eye(3)] * Bt)
    r = Ref(cfg)
    r.p, r.q = np.array([1.0, 2.0, 1.5]), yaw2quat(0.3)
    r.use_weights(r.W_on)
    prod = _lib.Context(0)  # the producer: its own stream

    def produced(a, nb, n1):  # device array whose final values an async kernel on prod's stream writes
        a = np.ascontiguousarray(a, dtype=np.float64).reshape(nb, n1, 10)
        out = _lib.DeviceArray.from_numpy(prod, np.zeros_like(a))
        d = _lib.DeviceArray.from_numpy(prod, a)
        uu = _lib.DeviceArray.from_numpy(prod, np.zeros((nb, n1 - 1, 4)))
        du = _lib.DeviceArray.from_numpy(prod, np.zeros((nb, n1 - 1, 4)))
        _lib.rti_apply(prod, nb, n1 - 1, out, uu, d, du)  # asynchronous: out = 0 + a
        out.keep = (d, uu, du)
        out.shape = (Bt, a.size // Bt)
        return out

    res = []
    for dev_inputs in (False, True):
        o = Ocp(Quad(cfg), batch=Bt, devices=[0, 0])
        assert len(o.parts) == 2
        n = Nmpc(cfg, batch=Bt, ocp=o)
        n.set_sdf_flag(1.0)
        for k in range(61):
            n.set_ref(r, k)
        n.set_x0(x0)
        n._flush()
        if dev_inputs:
            n.set_latent_device(produced(lat, 120, 64), produced(x0[:, :3], 1, 180), produced(R.reshape(Bt, 9), 1, 540))
        else:
            n.set_latent_device(lat, x0[:, :3], R)
        p = o.download("p")
        assert n.solve() == 0
        res.append((p, n.get_u()))
        o.close()
    np.testing.assert_array_equal(res[0][0], res[1][0])
    np.testing.assert_array_equal(res[0][1], res[1][1])
    prod.close()
