"""Config C5 at its per-GPU size (BASELINE.json configs[4]: 4096 instances over 8 GPUs -> 512 per GPU,
N = 60, the 4x-wide SDF [1024,1024,512,256], in-loop VAE encode) through the product path:
VaeWrapper-equivalent encode of 512 depth images -> set_latent on the device -> the solver object's
SQP-RTI step (wide preparation phase, QP at N = 60, update).

Full-size properties: every QP converges, the step satisfies the input boxes, x_0 and the linearised
dynamics, runs are bitwise repeatable and permuting the instances permutes the results bitwise.
Oracle spot checks on a strided subset: VAE latents vs the fp64 C encoder (oracle/vae.c), the wide
linearisation vs oracle.linearize_batch, the QP vs the structured C IPM (oracle/qp_ipm.c)."""
import numpy as np
import pytest

from sdf_nmpc_amd import _lib, synth, vae as V, weights as W
from sdf_nmpc_amd.config import Config
from sdf_nmpc_amd.model import Quad, quat2rot
from tolerances import VAE_LATENT_RTOL, vae_latent_err

pytestmark = pytest.mark.gpu

B, N, N_IMG = 512, 60, 32   # per-GPU share of C5; 32 distinct images, each used by 16 instances


class C5:
    def __init__(self, ctx, perm=None):
        cfg = Config(mpc__N=N)
        self.cfg, self.model = cfg, Quad(cfg)
        self.net = _lib.Net.from_blob(ctx, W.pack(W.WIDE_SPEC, W.siren_weights(W.WIDE_SPEC, 0)))
        spec = V.DEFAULT_ENCODER
        self.vparams = V.synthetic_encoder(spec, 0)
        self.vae = _lib.Vae(ctx, V.pack(spec, self.vparams), B)
        _, dt = _lib.shooting_grid(N, cfg.mpc.T)
        prob = synth.make_problem(cfg, B, N, seed=1000, dt=dt)
        x0 = prob["x"][:, 0] + np.random.default_rng(2000).normal(0, 0.05, (B, 10))
        self.imgs = synth.depth_images(N_IMG, 270, 480, seed=5)[np.arange(B) % N_IMG]
        perm = np.arange(B) if perm is None else perm
        self.prob = {k: (v if k == "dt" else v[perm]) for k, v in prob.items()}
        self.x0, self.imgs = x0[perm], self.imgs[perm]
        self.solver = _lib.Solver(ctx, self.net, _lib.quad_model(cfg), _lib.qp_opts(self.model), B, N,
                                  self.model.np, self.model.ny, dt)
        self.ctx = ctx
        self.yz = _lib.DeviceArray.from_numpy(ctx, V.depth2range_table(cfg.sensor.shape_imgs, cfg.sensor.hfov,
                                                                       cfg.sensor.vfov))
        self.img = _lib.DeviceArray.from_numpy(ctx, self.imgs.astype(np.float32))
        self.lat32 = _lib.DeviceArray(ctx, (B, 128), np.float32)
        self.lat64 = _lib.DeviceArray(ctx, (B, 128), np.float64)
        xs = self.prob["x"]
        self.pose = (_lib.DeviceArray.from_numpy(ctx, xs[:, 0, :3]),
                     _lib.DeviceArray.from_numpy(ctx, quat2rot(xs[:, 0, 3:7]).reshape(B, 9)))

    def step(self):
        """image -> latent -> p (set_latent on the device) -> one SQP-RTI step from the initial iterate."""
        s, pr = self.solver, self.prob
        for name, v in (("x", pr["x"]), ("u", pr["u"]), ("p", pr["p"]), ("x0", self.x0[:, None]),
                        ("yref", pr["yref"]), ("W", pr["W"]), ("yNref", pr["yN"][:, None]), ("WN", pr["WN"][:, None])):
            s.upload(name, v)
        _lib.vae_encode(self.ctx, self.vae, _lib.vae_opts(self.cfg, V.clip_scale(self.cfg)), self.img, self.yz,
                        self.lat32, self.lat64)
        _lib.pack_refs(self.ctx, _lib.ref_opts(self.cfg, -1), B, N, self.model.np, self.model.ny,
                       {"latent": self.lat64, "W_p_Bo": self.pose[0], "W_R_Bo": self.pose[1], "p": s.field("p")},
                       L=128)
        s.step()
        return s.wait().copy()


@pytest.fixture(scope="module")
def run(gpu_ctx):
    gpu_ctx.synchronize()
    c5 = C5(gpu_ctx)
    u0 = c5.step()
    shapes = dict(x=(B, N + 1, 10), u=(B, N, 4), p=(B, N + 1, -1), dx=(B, N + 1, 10), du=(B, N, 4), xn=(B, N, 10),
                  AB=(B, N, 14, 10), y=(B, N, 11), Jy=(B, N, 14, 11), yN=(B, 4), JyN=(B, 10, 4), h=(B, N + 1, 3),
                  Jh=(B, N + 1, 10, 3), slack=(B, N + 1, 3, 2), status=(B,), iters=(B,))
    out = {k: c5.solver.download(k).reshape(sh) for k, sh in shapes.items()}
    return c5, u0, out


def test_c5_vae_latents_vs_fp64_oracle(run, oracle_lib, cfg):
    c5, _, out = run
    lat = c5.lat32.numpy()
    yz = V.depth2range_table(cfg.sensor.shape_imgs, cfg.sensor.hfov, cfg.sensor.vfov)
    flat = np.concatenate([c5.vparams[n].ravel() for n, _ in V.DEFAULT_ENCODER.param_shapes()])
    for b in (0, 301):
        pre = oracle_lib.vae_preprocess(c5.imgs[b], (270, 480), V.clip_scale(cfg), yz)
        ref = oracle_lib.vae_encode(pre[None], flat)[0]
        assert vae_latent_err(lat[b], ref) <= VAE_LATENT_RTOL, b
    # instances sharing an image get the same latent, bit for bit (batch independence of the encoder)
    np.testing.assert_array_equal(lat[5], lat[5 + N_IMG])
    # set_latent on the device: every node of p carries the fp64 latent
    np.testing.assert_array_equal(out["p"][..., 17:], np.broadcast_to(c5.lat64.numpy()[:, None], (B, N + 1, 128)))


def test_c5_wide_linearisation_vs_oracle(run, oracle_lib):
    c5, _, out = run
    sel = np.array([0, 171, 342, 511])
    onet = oracle_lib.Net(W.WIDE_SPEC, W.siren_weights(W.WIDE_SPEC, 0))
    x = c5.prob["x"][sel].copy()
    x[:, 0] = c5.x0[sel]
    ref = oracle_lib.linearize_batch(oracle_lib.quad_model(c5.cfg), onet, x, c5.prob["u"][sel], out["p"][sel],
                                     c5.prob["dt"])
    for k in ("xn", "AB", "y", "Jy", "yN", "JyN"):
        np.testing.assert_allclose(out[k][sel], ref[k], rtol=1e-9, atol=1e-12 * max(1.0, np.abs(ref[k]).max()))
    np.testing.assert_allclose(out["h"][sel][..., :2], ref["h"][..., :2], rtol=1e-9, atol=1e-12)
    assert np.abs(out["h"][sel][..., 2] - ref["h"][..., 2]).max() <= 1e-5
    assert np.abs(out["Jh"][sel][..., 2] - ref["Jh"][..., 2]).max() <= 1e-5 * max(1.0, np.abs(ref["Jh"]).max())


def test_c5_qp_full_size_properties_and_oracle(run, oracle_lib):
    from test_gpu_qp import _agree
    c5, u0, out = run
    assert (out["status"] == 0).all() and out["iters"].max() <= 100
    m = c5.model
    du, dx = out["du"], out["dx"]
    u_new = c5.prob["u"] + du
    assert (u_new >= m.lbu - 1e-7).all() and (u_new <= m.ubu + 1e-7).all()
    np.testing.assert_array_equal(u0, out["u"][:, 0])
    assert not dx[:, 0].any()  # the step sets x_0 = x0 before linearising (Ocp.solve, ocp.py:161)
    AB, c = out["AB"], out["xn"] - c5.prob["x"][:, 1:]
    pred = np.einsum("bkji,bkj->bki", AB[:, :, :10], dx[:, :-1]) + np.einsum("bkji,bkj->bki", AB[:, :, 10:], du) + c
    np.testing.assert_allclose(dx[:, 1:], pred, atol=1e-9)
    sel = np.arange(0, B, 32)
    x = c5.prob["x"][sel].copy()
    x[:, 0] = c5.x0[sel]
    lin = {k: out[k][sel] for k in ("xn", "AB", "y", "Jy", "yN", "JyN", "h", "Jh")}
    prob = {k: (v if k == "dt" else v[sel]) for k, v in c5.prob.items()}
    prob["x"] = x
    ref = oracle_lib.qp_ipm_batch(lin, prob, c5.x0[sel], m, nthreads=8)
    assert (ref["status"] == 0).all()
    got = {"du": du[sel], "dx": dx[sel], "slack": out["slack"][sel]}
    _agree(prob, c5.x0[sel], lin, m, got, ref)


def test_c5_deterministic_and_permutation_equivariant(run, gpu_ctx):
    c5, u0, _ = run
    np.testing.assert_array_equal(c5.step(), u0)  # bitwise repeatable
    perm = np.random.default_rng(7).permutation(B)
    cp = C5(gpu_ctx, perm=perm)
    np.testing.assert_array_equal(cp.step(), u0[perm])
    np.testing.assert_array_equal(cp.solver.download("iters").ravel(), c5.solver.download("iters").ravel()[perm])


def test_c5_full_batch_through_shard_plan(tmp_path):
    """BASELINE.json configs[4] (C5) at its real batch: 4096 instances at N = 60 with the 4x-wide SDF and the
    in-loop VAE, through Ocp(devices=[0] * 8) -- shard.plan gives eight 512-instance parts (the N = 60
    capacity) -- and VaeWrapper(batch=4096).encode_to, which packs each part's latents on its own device.
    One RTI step converges on every instance inside the input boxes, and two parts solved alone (their own
    512 images through their own VaeWrapper, the same QP kernel) agree bit for bit."""
    from sdf_nmpc_amd import shard
    from sdf_nmpc_amd.controller import Nmpc
    from sdf_nmpc_amd.ocp import Ocp
    from sdf_nmpc_amd.reference import Ref, yaw2quat
    cfg = Config(mpc__N=N)
    Bt, n_img = 4096, 64
    wpath = str(tmp_path / "c5.sdfw")
    with open(wpath, "wb") as f:
        f.write(W.pack(W.WIDE_SPEC, W.siren_weights(W.WIDE_SPEC, 0)))
    assert shard.plan(Bt, _lib.Context(0).qp_capacity(N), 8) == [(g, 512 * g, 512 * (g + 1)) for g in range(8)]
    rng = np.random.default_rng(45)
    x0 = np.zeros((Bt, 10))
    x0[:, :3] = rng.uniform(-2, 2, (Bt, 3))
    x0[:, 3:7] = np.stack([yaw2quat(y) for y in rng.uniform(-np.pi, np.pi, Bt)])
    imgs = synth.depth_images(n_img, 270, 480, seed=46)
    sel_img = rng.integers(0, n_img, Bt)
    r = Ref(cfg)
    r.p, r.q = np.array([1.0, 2.0, 1.5]), yaw2quat(0.3)
    r.use_weights(r.W_on)
    W_R = quat2rot(x0[:, 3:7]).reshape(Bt, 3, 3)

    def run(lo, hi, devices, kernel=None):
        nb = hi - lo
        o = Ocp(Quad(cfg), batch=nb, devices=devices, weights=wpath)
        if kernel is not None:
            for p in o.parts:
                p.ctx.set_qp_kernel(kernel)
        n = Nmpc(cfg, batch=nb, ocp=o)
        vw = V.VaeWrapper(cfg, batch=nb, ctx=o.ctx)
        vw.set_img(imgs[sel_img[lo:hi]])
        vw.encode_to(n, x0[lo:hi, :3], W_R[lo:hi], flag=1.0)
        for k in range(N + 1):
            n.set_ref(r, k)
        n.set_x0(x0[lo:hi])
        assert n.solve() == 0
        out = dict(u0=n.get_u(), status=o.status.copy(), iters=o.iters.copy(), u=o.download("u"),
                   p=o.download("p"), parts=len(o.parts), kind=o.parts[0].ctx.qp_kernel(N, nb))
        o.close()
        return out

    full = run(0, Bt, [0] * 8)
    assert full["parts"] == 8
    assert (full["status"] == 0).all() and full["iters"].max() < 100
    m = Quad(cfg)
    assert (full["u"] >= m.lbu - 1e-9).all() and (full["u"] <= m.ubu + 1e-9).all()
    # the latents every part packed: instances sharing an image carry the same latent at every node
    b0 = np.flatnonzero(sel_img == sel_img[0])
    assert len(b0) > 8 and (b0 // 512).min() != (b0 // 512).max()  # shared across parts
    np.testing.assert_array_equal(full["p"][b0][:, :, 17:], np.broadcast_to(full["p"][b0[0], 0, 17:], (len(b0), N + 1, 128)))
    for g in (0, 6):
        lo, hi = 512 * g, 512 * (g + 1)
        alone = run(lo, hi, [0], kernel=full["kind"])
        np.testing.assert_array_equal(alone["u0"], full["u0"][lo:hi])
        np.testing.assert_array_equal(alone["iters"], full["iters"][lo:hi])
