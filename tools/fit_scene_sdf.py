"""Offline (CPU, seeded): fit the reference-architecture NeuralDF to an analytic obstacle scene, so that
the SDF constraint of the NMPC becomes active and releases along a trajectory.

Every other network in this repository is the SIREN initialisation, whose df is ~0 everywhere (so every
SDF row of every QP is active).  This script trains the deployed architecture (network/neural_df.py:
[256, 256, 128, 64], 'oct' x 5 frequencies, sin w0 = 20, res 'full', latent 128,
scripts/neural_nets/df_train.py:96-103) with the reference's own loss (utils/losses.py:68-96, weights
(50, 0, 1/60, 5) as df_train.py:73) and initialisation (utils/layer_init.py:15-25), AdamW with a cosine
learning rate, on points sampled around an analytic scene in the camera-origin frame (x forward, y left,
z up: the frame of Co_p_B, gen_model.py:46-51), for ONE fixed latent (SCENE_LATENT_SEED): the network is a
stand-in for "the SDF of the scene this depth image's latent encodes".

Scene (metres, camera-origin frame): a vertical pillar of radius 0.4 at (3.0, 0.3), z in [-3, 3], and a
box x in [5.0, 5.6], y in [-2.5, -0.8], z in [-3, 3]; the truncated signed distance min(sdf, max_df = 1)
(df_train.py:50-52).  Output: tests/golden/scene.sdfw (weights.pack) and its training record.

The reference checkout is needed (this container only): run as
    python tools/fit_scene_sdf.py [steps]
"""
import os
import sys
import time
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT]
REF = "/root/reference"
sys.modules.setdefault("casadi", types.ModuleType("casadi"))  # utils/embeddings.py imports it unused
sys.path.insert(0, REF)
from sdf_nmpc.network.neural_df import NeuralDF  # noqa: E402
from sdf_nmpc.utils.layer_init import init_linear_layer_sine  # noqa: E402
from sdf_nmpc.utils.losses import loss_sdf  # noqa: E402

import sdf_nmpc_amd  # noqa: E402,F401
from sdf_nmpc_amd import weights as W  # noqa: E402

SCENE_LATENT_SEED = 2024
PILLAR = (3.0, 0.3, 0.4)                      # x, y, radius
BOX = ((5.0, 5.6), (-2.5, -0.8), (-3.0, 3.0))  # x, y, z ranges
MAX_DF = 1.0
OUT = os.path.join(ROOT, "tests", "golden", "scene.sdfw")


def scene_latent():
    return np.random.default_rng(SCENE_LATENT_SEED).normal(size=W.DEFAULT_SPEC.size_latent).astype(np.float32)


def scene_sdf(p):
    """Signed distance to the scene and its gradient (numpy or torch [n, 3] fp64 -> [n], [n, 3])."""
    x, y, z = p[:, 0], p[:, 1], p[:, 2]
    lib = torch if isinstance(p, torch.Tensor) else np
    # pillar: distance to the vertical axis minus the radius (its z extent covers the sampled range)
    dxp, dyp = x - PILLAR[0], y - PILLAR[1]
    rxy = lib.sqrt(dxp * dxp + dyp * dyp) + 1e-12
    d1 = rxy - PILLAR[2]
    g1 = lib.stack([dxp / rxy, dyp / rxy, 0 * z], 1)
    # box: the exact signed distance of an axis-aligned box
    c = [0.5 * (a + b) for a, b in BOX]
    h = [0.5 * (b - a) for a, b in BOX]
    q = lib.stack([lib.abs(x - c[0]) - h[0], lib.abs(y - c[1]) - h[1], lib.abs(z - c[2]) - h[2]], 1)
    sgn = lib.stack([lib.sign(x - c[0]), lib.sign(y - c[1]), lib.sign(z - c[2])], 1)
    qp = lib.clip(q, 0, None) if lib is np else torch.clamp(q, min=0)
    out = lib.sqrt((qp * qp).sum(1)) + 1e-12
    inside = q.max(1) if lib is np else q.max(1).values
    d2 = out + (lib.minimum(inside, 0 * inside) if lib is np else torch.clamp(inside, max=0))
    g_out = qp / out[:, None] * sgn
    am = q.argmax(1)
    g_in = (lib.arange(3)[None, :] == am[:, None]) * sgn
    g_in = g_in.astype(np.float64) if lib is np else g_in.to(p.dtype)
    g2 = lib.where((inside > 0)[:, None], g_out, g_in)
    use1 = d1 <= d2
    d = lib.where(use1, d1, d2)
    g = lib.where(use1[:, None], g1, g2)
    # truncation (df_train.py:50): beyond max_df the target is max_df with a zero gradient
    tr = d >= MAX_DF
    d = lib.where(tr, MAX_DF + 0 * d, d)
    g = lib.where(tr[:, None], 0 * g, g)
    return d, g


def sample(rng, n):
    """Points of the camera-origin frame: the frustum box, a ball at the origin, shells around the obstacles
    (df_train.py:61-71 samples frustum / origin ball / obstacle neighbourhood the same way)."""
    k1, k2 = n // 2, n // 8
    k3 = n - k1 - k2
    a = np.stack([rng.uniform(-1.0, 7.0, k1), rng.uniform(-4.0, 4.0, k1), rng.uniform(-2.0, 2.0, k1)], 1)
    v = rng.normal(size=(k2, 3))
    b = v / np.linalg.norm(v, axis=1, keepdims=True) * rng.uniform(0, 0.75, (k2, 1))
    # near the surfaces: pillar shell and box shell
    t = rng.uniform(0, 2 * np.pi, k3 // 2)
    r = PILLAR[2] + rng.uniform(-0.2, 1.2, k3 // 2)
    c = np.stack([PILLAR[0] + r * np.cos(t), PILLAR[1] + r * np.sin(t), rng.uniform(-2, 2, k3 // 2)], 1)
    m = k3 - k3 // 2
    d = np.stack([rng.uniform(BOX[0][0] - 1.2, BOX[0][1] + 1.2, m), rng.uniform(BOX[1][0] - 1.2, BOX[1][1] + 1.2, m),
                  rng.uniform(-2, 2, m)], 1)
    return np.concatenate([a, b, c, d]).astype(np.float32)


def main(steps=3000, batch=4096, seed=0):
    torch.manual_seed(seed)
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    rng = np.random.default_rng(seed)
    spec = W.DEFAULT_SPEC
    net = NeuralDF(nb_states=3, size_latent=spec.size_latent, signed=True, max_df=MAX_DF, res="full", w0=spec.w0,
                   embed="oct", act="sin", layer_sizes=list(spec.layer_sizes), dropout_rate=0.1, nb_freqs=spec.nb_freqs)
    init_linear_layer_sine(net.layers, net.w0)
    net.train()
    z = torch.from_numpy(scene_latent())[None, :]
    opt = torch.optim.AdamW(net.parameters(), lr=3e-4, weight_decay=1e-5)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=steps, eta_min=1e-5)
    wts = (50, 0, 1 / 60, 5)  # df_train.py:73
    tic = time.time()
    for it in range(steps):
        pts = torch.from_numpy(sample(rng, batch))
        d, g = scene_sdf(pts.double())
        pts.requires_grad_(True)
        out = net(torch.hstack([pts, z.expand(batch, -1)]))
        losses = loss_sdf(out, pts, g.float(), d.float())
        loss = sum(w * l for l, w in zip(losses, wts))
        opt.zero_grad()
        loss.backward()
        opt.step()
        sched.step()
        if it % 250 == 0 or it == steps - 1:
            print(f"step {it}: loss {loss.item():.4f} regression {losses[0].item():.2e} dir {losses[2].item():.2f} deg "
                  f"eikonal {losses[3].item():.2e} ({time.time() - tic:.0f} s)", flush=True)
    net.eval()
    params = {k: v.detach().numpy().astype(np.float32) for k, v in net.state_dict().items() if k in
              dict(spec.param_shapes())}
    # held-out error of the fit
    pts = sample(np.random.default_rng(seed + 1), 20000)
    d, _ = scene_sdf(pts.astype(np.float64))
    with torch.no_grad():
        pred = net(torch.hstack([torch.from_numpy(pts), z.expand(len(pts), -1)])).numpy()[:, 0]
    err = np.abs(pred - d)
    print(f"held-out |df - sdf|: mean {err.mean():.3f} m, p95 {np.quantile(err, 0.95):.3f} m, max {err.max():.3f} m")
    with open(OUT, "wb") as f:
        f.write(W.pack(spec, params))
    print("wrote", OUT)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3000)
