"""In-loop VAE encoder on the GPU (csrc/vae_enc.hip) through the C ABI, against the
reference's own Encoder outputs (tests/golden/vae_golden.npz) and the C oracle (oracle/vae.c)."""
import os

import numpy as np
import pytest

from sdf_nmpc_amd import _lib, synth
from sdf_nmpc_amd import vae as V
from tolerances import VAE_LATENT_RTOL, vae_latent_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def vg():
    return np.load(os.path.join(os.path.dirname(__file__), "golden", "vae_golden.npz"))


@pytest.fixture(scope="module")
def dev_vae(gpu_ctx):
    spec = V.DEFAULT_ENCODER
    params = V.synthetic_encoder(spec, 0)
    vae = _lib.Vae(gpu_ctx, V.pack(spec, params))
    flat = np.concatenate([params[n].ravel() for n, _ in spec.param_shapes()])
    yield spec, vae, flat
    vae.close()


def _encode(gpu_ctx, vae, cfg, imgs, clip, yz=True):
    import torch
    t = torch.from_numpy(np.ascontiguousarray(imgs)).cuda()
    table = V.depth2range_table(cfg.sensor.shape_imgs, cfg.sensor.hfov, cfg.sensor.vfov)
    yzt = torch.from_numpy(table).cuda()
    B = t.shape[0]
    lat = torch.empty(B, 128, dtype=torch.float32, device="cuda")
    lat64 = torch.empty(B, 128, dtype=torch.float64, device="cuda")
    _lib.vae_encode(gpu_ctx, vae, _lib.vae_opts(cfg, clip), t, yzt, lat, lat64, depth2range=yz)
    torch.cuda.synchronize()
    return lat.cpu().numpy(), lat64.cpu().numpy()


def _case(vg, c):
    seed, kind = (int(v) for v in vg[f"c{c}/seed"])
    H, W = (int(v) for v in vg[f"c{c}/in_shape"])
    return synth.depth_images(1, H, W, seed=seed, kind="mm" if kind == 2 else "m")[0]


def test_encoder_vs_reference_golden(gpu_ctx, dev_vae, cfg, vg):
    _, vae, _ = dev_vae
    for c in range(int(vg["n_cases"])):
        clip = cfg.sensor.dmax / float(vg[f"c{c}/mm_resolution"]) * 1000
        lat, lat64 = _encode(gpu_ctx, vae, cfg, _case(vg, c)[None], clip)
        err = vae_latent_err(lat[0], vg[f"c{c}/latent64"])
        assert err <= VAE_LATENT_RTOL, (c, err)
        assert np.array_equal(lat64[0], lat[0].astype(np.float64))


def test_encoder_vs_oracle_batch(gpu_ctx, dev_vae, cfg, oracle_lib):
    """A batch of 6 images (float32) against the fp64 C oracle on the same preprocessed pixels."""
    _, vae, flat = dev_vae
    imgs = synth.depth_images(6, 270, 480, seed=11)
    lat, _ = _encode(gpu_ctx, vae, cfg, imgs, 5.0)
    yz = V.depth2range_table(cfg.sensor.shape_imgs, cfg.sensor.hfov, cfg.sensor.vfov)
    pre = np.stack([oracle_lib.vae_preprocess(im, (270, 480), 5.0, yz) for im in imgs])
    ref = oracle_lib.vae_encode(pre, flat)
    for b in range(6):
        assert vae_latent_err(lat[b], ref[b]) <= VAE_LATENT_RTOL, b


def test_encoder_non_finite_pixels(gpu_ctx, dev_vae, cfg, oracle_lib):
    """ADVICE r3 (split-bf16 exactness): the convolutions see only preprocessed pixels, and ClipDistance /
    Depth2Range clip to [0, 1] (utils/preprocessing.py:30-31, 78-79) -- an Inf depth pixel reaches them as
    1.0, where the split is exact, and the latent matches the fp64 oracle as for any image.  A NaN pixel
    passes the clips as NaN (torch.clip and the kernel's compare-selects both keep it) and poisons the
    latent, as in the reference: NaN in, NaN out, never a silently finite latent."""
    _, vae, flat = dev_vae
    imgs = synth.depth_images(2, 270, 480, seed=29)
    imgs[0, 100, 200] = np.inf
    imgs[0, 0, 0] = np.inf
    imgs[1, 135, 240] = np.nan
    lat, _ = _encode(gpu_ctx, vae, cfg, imgs, 5.0)
    yz = V.depth2range_table(cfg.sensor.shape_imgs, cfg.sensor.hfov, cfg.sensor.vfov)
    pre = oracle_lib.vae_preprocess(imgs[0], (270, 480), 5.0, yz)
    assert pre[100, 200] == 1.0 and np.isfinite(pre).all()
    ref = oracle_lib.vae_encode(pre[None], flat)
    assert np.isfinite(lat[0]).all() and vae_latent_err(lat[0], ref[0]) <= VAE_LATENT_RTOL
    assert np.isnan(lat[1]).any()


def test_batch_invariance_and_determinism(gpu_ctx, dev_vae, cfg):
    """Each image's latent is independent of its batch neighbours (bitwise) and runs are bitwise repeatable;
    37 images leave a ragged last GEMM row tile in every layer."""
    _, vae, _ = dev_vae
    imgs = synth.depth_images(37, 270, 480, seed=3)
    a, _ = _encode(gpu_ctx, vae, cfg, imgs, 5.0)
    b, _ = _encode(gpu_ctx, vae, cfg, imgs, 5.0)
    assert np.array_equal(a, b)
    for i in (0, 17, 36):
        s, _ = _encode(gpu_ctx, vae, cfg, imgs[i:i + 1], 5.0)
        assert np.array_equal(s[0], a[i]), i


def test_uint16_and_no_depth2range(gpu_ctx, dev_vae, cfg, oracle_lib):
    """uint16 millimetre input (mm_resolution = 1) and sensor.is_depth = False (no Depth2Range)."""
    _, vae, flat = dev_vae
    mm = synth.depth_images(2, 270, 480, seed=8, kind="mm")
    lat, _ = _encode(gpu_ctx, vae, cfg, mm, 5000.0, yz=False)
    pre = np.stack([oracle_lib.vae_preprocess(im, (270, 480), 5000.0, None) for im in mm])
    ref = oracle_lib.vae_encode(pre, flat)
    for b in range(2):
        assert vae_latent_err(lat[b], ref[b]) <= VAE_LATENT_RTOL, b


def test_vae_wrapper_feeds_controller(gpu_ctx, cfg):
    """VaeWrapper (sdf_nmpc/vae.py:7-50 mirror) -> encode_to(Nmpc) equals encode() -> host set_latent."""
    from sdf_nmpc_amd.controller import Nmpc

    B = 4
    w = V.VaeWrapper(cfg, batch=B, ctx=gpu_ctx)
    imgs = synth.depth_images(B, 270, 480, seed=21)
    w.set_img(imgs)
    lat = w.encode()
    assert lat.shape == (B, 128) and np.isfinite(lat).all()
    rng = np.random.default_rng(0)
    W_p_Bo = rng.normal(size=(B, 3))
    W_R_Bo = np.stack([np.eye(3)] * B)
    m1 = Nmpc(cfg, batch=B)
    m2 = Nmpc(cfg, batch=B)
    m1.set_latent(lat.astype(np.float64), W_p_Bo, W_R_Bo)
    w.encode_to(m2, W_p_Bo, W_R_Bo)
    p2 = m2.ocp.download("p").reshape(m1.p.shape)
    np.testing.assert_array_equal(p2[..., 17:], m1.p[..., 17:])
