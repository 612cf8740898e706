"""In-loop VAE encoder: depth image -> latent, on the device, for config C5.

Host-side plumbing: architecture spec, deterministic synthetic weights, BatchNorm folding into the
packed `.vaew` layout that ``csrc/vae_enc.hip`` consumes through the C ABI (``include/sdfnmpc.h``),
the Depth2Range table, and ``VaeWrapper`` -- the mirror of the reference's ``sdf_nmpc/vae.py``
``VaeWrapper`` (set_img / set_latent / encode) whose encode runs on the GPU.

Reference anchors (``/root/reference``):
  * encoder architecture ........ ``sdf_nmpc/network/vae.py:6-46`` (``Encoder``; ``forward`` = mean head)
  * residual block .............. ``sdf_nmpc/network/resnet.py:5-56`` (``ResBlock``, non-bottleneck)
  * preprocessing ............... ``sdf_nmpc/vae.py:15-24`` -> ``utils/preprocessing.py``
                                  ``ToDevice`` :263-276, ``Reshape`` :99-112, ``ClipDistance`` :84-96,
                                  ``Depth2Range`` :5-30
  * wrapper API ................. ``sdf_nmpc/vae.py:7-50``

Inference semantics (``model.eval()``): Dropout / Dropout2d are identities and BatchNorm uses its
running statistics, so every BatchNorm folds into the preceding convolution:
``w' = w * g / sqrt(v + eps)``, ``b' = (b - m) * g / sqrt(v + eps) + beta`` (fp64, rounded once to fp32).

The real ``vae.pt`` is a git-LFS pointer in the reference checkout, so tests use weights from the
counter-based PRNG of ``weights.py`` (``synthetic_encoder``); ``from_state_dict`` / ``from_torchscript``
convert a real checkpoint offline.
"""
from __future__ import annotations

import dataclasses
import struct
from typing import Dict, List, Tuple

import numpy as np

from .weights import prng_uniform

MAGIC = b"SDFNVAEW"
VERSION = 1
BN_EPS = 1e-5  # torch.nn.BatchNorm2d default (resnet.py:32-37)
_HDR = struct.Struct("<8s8I")  # magic, version, nb_chan, size_latent, H, W, n_convs, n_floats, reserved


@dataclasses.dataclass(frozen=True)
class EncoderSpec:
    """``Encoder(nb_chan, size_latent, batchnorm)`` (vae.py:11) on ``shape_imgs`` (default.yaml sensor)."""
    nb_chan: int = 1
    size_latent: int = 128
    shape: Tuple[int, int] = (270, 480)
    batchnorm: bool = True
    widths: Tuple[int, ...] = (64, 128, 256, 512)  # ResBlock inputs (vae.py:22-25), strides 2,2,2,1

    def blocks(self):
        """(size_in, stride) of the four ResBlocks."""
        return [(64, 2), (128, 2), (256, 2), (512, 1)]

    def maps(self):
        """Spatial sizes: stem conv, maxpool, then each block output."""
        H, W = self.shape
        conv = lambda n, k, s, p: (n + 2 * p - k) // s + 1  # noqa: E731
        h, w = conv(H, 7, 2, 3), conv(W, 7, 2, 3)
        out = [(h, w)]
        h, w = conv(h, 3, 2, 1), conv(w, 3, 2, 1)
        out.append((h, w))
        for _, s in self.blocks():
            h, w = conv(h, 3, s, 1), conv(w, 3, s, 1)
            out.append((h, w))
        return out

    def param_shapes(self) -> List[Tuple[str, Tuple[int, ...]]]:
        """``Encoder.state_dict()`` names and shapes in order (num_batches_tracked omitted)."""
        bn = self.batchnorm
        out = [("layers.resnet.0.weight", (64, self.nb_chan, 7, 7)), ("layers.resnet.0.bias", (64,))]

        def conv(prefix, cin, cout, k):
            out.append((prefix + ".weight", (cout, cin, k, k)))
            if not bn:
                out.append((prefix + ".bias", (cout,)))

        def norm(prefix, c):
            if bn:
                out.extend([(prefix + s, (c,)) for s in (".weight", ".bias", ".running_mean", ".running_var")])

        for i, (cin, s) in enumerate(self.blocks()):
            p = f"layers.resnet.{3 + i}"
            cout = cin * s
            conv(p + ".layers.0", cin, cout, 3)
            norm(p + ".layers.1", cout)
            conv(p + ".layers.3", cout, cout, 3)
            norm(p + ".layers.4", cout)
            if s != 1:
                conv(p + ".shortcut.0", cin, cout, 1)
                norm(p + ".shortcut.1", cout)
        F = 512 * 2 * 2
        out += [("layers.mean.weight", (self.size_latent, F)), ("layers.mean.bias", (self.size_latent,)),
                ("layers.logvar.weight", (self.size_latent, F)), ("layers.logvar.bias", (self.size_latent,))]
        return out

    def n_flops(self) -> int:
        """Algorithmic FLOPs of one encode (2 x MAC of every conv / linear, mean head only)."""
        (h0, w0), (hp, wp), *blk = self.maps()
        mac = h0 * w0 * 64 * 49 * self.nb_chan
        h, w = hp, wp
        for (cin, s), (ho, wo) in zip(self.blocks(), blk):
            cout = cin * s
            mac += ho * wo * cout * 9 * cin + ho * wo * cout * 9 * cout
            if s != 1:
                mac += ho * wo * cout * cin
            h, w = ho, wo
        mac += 2048 * self.size_latent
        return 2 * mac


DEFAULT_ENCODER = EncoderSpec()


def synthetic_encoder(spec: EncoderSpec = DEFAULT_ENCODER, seed: int = 0) -> Dict[str, np.ndarray]:
    """Deterministic encoder parameters (stream t = position in ``param_shapes``).

    Conv weights He-uniform U(+-sqrt(6/fan_in)) so activations stay O(1) through the ReLU stack, biases
    U(+-1/sqrt(fan_in)) (torch's default bias init), BatchNorm gamma U(0.5,1.5), beta U(-0.2,0.2),
    running_mean U(-0.2,0.2), running_var U(0.5,1.5) so the folding is exercised, linear weights
    U(+-1/sqrt(fan_in)).  Values are rounded once from double to fp32.
    """
    out = {}
    for t, (name, shape) in enumerate(spec.param_shapes()):
        n = int(np.prod(shape))
        u = prng_uniform(seed + 1000, t, n)
        kind = name.rsplit(".", 1)[1]
        is_bn = ("layers.resnet." in name and len(shape) == 1 and not name.endswith(".0.bias")
                 and spec.batchnorm)
        if is_bn:
            lo, hi = {"weight": (0.5, 1.5), "bias": (-0.2, 0.2), "running_mean": (-0.2, 0.2),
                      "running_var": (0.5, 1.5)}[kind]
            v = lo + (hi - lo) * u
        elif len(shape) == 4:
            fan_in = int(np.prod(shape[1:]))
            v = (2.0 * u - 1.0) * np.sqrt(6.0 / fan_in)
        else:  # linear weight / any bias
            fan_in = shape[1] if len(shape) == 2 else _fan_in_of_bias(spec, name)
            v = (2.0 * u - 1.0) / np.sqrt(fan_in)
        out[name] = v.astype(np.float32).reshape(shape)
    return out


def _fan_in_of_bias(spec, name):
    shapes = dict(spec.param_shapes())
    w = shapes[name[: -len("bias")] + "weight"]
    return int(np.prod(w[1:]))


# ---------------------------------------------------------------------------------------------
# folding + packing: the device layout
# ---------------------------------------------------------------------------------------------
def _fold(params, conv, norm, bn):
    """(w [Cout][KH][KW][Cin] fp32, b [Cout] fp32) of conv (+ BatchNorm), folded in fp64."""
    w = params[conv + ".weight"].astype(np.float64)
    b = params[conv + ".bias"].astype(np.float64) if (conv + ".bias") in params else np.zeros(w.shape[0])
    if bn:
        g, beta = params[norm + ".weight"].astype(np.float64), params[norm + ".bias"].astype(np.float64)
        m, v = params[norm + ".running_mean"].astype(np.float64), params[norm + ".running_var"].astype(np.float64)
        sc = g / np.sqrt(v + BN_EPS)
        w = w * sc[:, None, None, None]
        b = (b - m) * sc + beta
    return (np.ascontiguousarray(w.transpose(0, 2, 3, 1)).astype(np.float32), b.astype(np.float32))


def device_layers(spec: EncoderSpec, params: Dict[str, np.ndarray]):
    """The packed conv list in launch order: stem, then per block (conv_a, [shortcut], conv_b), head.

    Each entry is (name, w, b); w is [Cout][KH][KW][Cin] (K contiguous per output channel, the GEMM's
    B-operand layout), the head is the mean Linear as a [L][2048] matrix.
    """
    bn = spec.batchnorm
    layers = [("stem",) + _fold(params, "layers.resnet.0", None, False)]
    for i, (cin, s) in enumerate(spec.blocks()):
        p = f"layers.resnet.{3 + i}"
        layers.append((f"b{i}a",) + _fold(params, p + ".layers.0", p + ".layers.1", bn))
        if s != 1:
            layers.append((f"b{i}s",) + _fold(params, p + ".shortcut.0", p + ".shortcut.1", bn))
        layers.append((f"b{i}b",) + _fold(params, p + ".layers.3", p + ".layers.4", bn))
    layers.append(("head", params["layers.mean.weight"].astype(np.float32),
                   params["layers.mean.bias"].astype(np.float32)))
    return layers


def pack(spec: EncoderSpec, params: Dict[str, np.ndarray]) -> bytes:
    """Serialise to the `.vaew` layout read by ``sdfnmpc_vae_load`` (include/sdfnmpc.h)."""
    if spec.nb_chan != 1 or tuple(spec.widths) != (64, 128, 256, 512):
        raise ValueError("only the reference encoder (1 channel, widths 64..512) is built")
    body = []
    for _, w, b in device_layers(spec, params):
        body += [np.ascontiguousarray(w, dtype="<f4").tobytes(), np.ascontiguousarray(b, dtype="<f4").tobytes()]
    blob = b"".join(body)
    hdr = _HDR.pack(MAGIC, VERSION, spec.nb_chan, spec.size_latent, spec.shape[0], spec.shape[1],
                    len(body) // 2, len(blob) // 4, 0)
    return hdr + blob


def save(path: str, spec: EncoderSpec, params: Dict[str, np.ndarray]) -> None:
    with open(path, "wb") as f:
        f.write(pack(spec, params))


def from_state_dict(sd, spec: EncoderSpec = None) -> Tuple[EncoderSpec, Dict[str, np.ndarray]]:
    """An ``Encoder`` (or whole ``Vae``: keys under ``encoder.``) state_dict -> (spec, params)."""
    sd = {k: (v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)) for k, v in sd.items()}
    if any(k.startswith("encoder.") for k in sd):
        sd = {k[len("encoder."):]: v for k, v in sd.items() if k.startswith("encoder.")}
    L = sd["layers.mean.weight"].shape[0]
    bn = "layers.resnet.3.layers.1.running_mean" in sd
    spec = spec or EncoderSpec(size_latent=L, batchnorm=bn)
    params = {}
    for name, shape in spec.param_shapes():
        a = np.asarray(sd[name], dtype=np.float32)
        if a.shape != shape:
            raise ValueError(f"{name}: shape {a.shape} != {shape}")
        params[name] = a
    return spec, params


def from_torchscript(path: str, shape=(270, 480)) -> Tuple[EncoderSpec, Dict[str, np.ndarray]]:
    """Convert a VAE TorchScript archive of YOUR OWN (what ``sdf_nmpc/vae.py:11`` loads) offline."""
    import torch  # offline only

    m = torch.jit.load(path, map_location="cpu")
    sd = m.state_dict()
    spec, params = from_state_dict(sd)
    return dataclasses.replace(spec, shape=tuple(shape)), params


# ---------------------------------------------------------------------------------------------
# preprocessing constants (utils/preprocessing.py)
# ---------------------------------------------------------------------------------------------
def depth2range_table(shape, hfov, vfov) -> np.ndarray:
    """``Depth2Range.yz_sqrt`` (preprocessing.py:16-27) in fp32 with correctly rounded operations.

    torch's scalar ``tan`` is correctly rounded (numpy's fp32 ``tan`` is not, so it is taken in fp64 and
    rounded once); torch's vectorised fp32 ``sqrt`` is within 1 ulp of the correctly rounded one used here
    (tests/test_vae.py pins the table and the preprocessed pixels to the golden file at that bar).
    """
    H, W = int(shape[-2]), int(shape[-1])
    u, v = np.meshgrid(np.arange(W, dtype=np.float32), np.arange(H, dtype=np.float32), indexing="xy")
    th = np.float32(np.tan(np.float64(np.float32(hfov))))
    tv = np.float32(np.tan(np.float64(np.float32(vfov))))
    a = th * (np.float32(1) - np.float32(2) * u / np.float32(W))
    b = tv * (np.float32(1) - np.float32(2) * v / np.float32(H))
    return np.sqrt(np.float32(1) + a * a + b * b).astype(np.float32)


def clip_scale(cfg) -> float:
    """``ClipDistance.dmax`` (preprocessing.py:91): dmax / mm_resolution * 1000."""
    return cfg.sensor.dmax / cfg.sensor.mm_resolution * 1000


class VaeWrapper:
    """Mirror of the reference's ``VaeWrapper`` (sdf_nmpc/vae.py:7-50) over a batch of B images.

    ``set_img(img)`` takes one raw image [H, W] (B = 1, as the reference) or a batch [B, H, W] (numpy
    float32 / uint16, or a device array -- ``_lib.DeviceArray`` or a torch tensor, used in place);
    ``encode()`` runs preprocessing + the encoder on the GPU and returns the latent means [L] / [B, L] as
    numpy.  ``encode_to(nmpc)`` writes them straight into an ``Nmpc``'s device parameters (set_latent on
    the device, no host round trip).  ``decode`` is not provided: the decoder is only used for
    visualisation (out of scope).  No tensor library is needed.
    """

    def __init__(self, cfg, weights=None, batch: int = 1, device: int = 0, ctx=None, seed: int = 0):
        from . import _lib

        self.cfg = cfg
        self.B = int(batch)
        self._own_ctx = ctx is None
        self.ctx = ctx if ctx is not None else _lib.Context(device)
        spec = EncoderSpec(size_latent=int(cfg.nn.size_latent), shape=tuple(cfg.sensor.shape_imgs[-2:]))
        if weights is None:
            weights = cfg.nn.get("vae_weights")
            seed = int(cfg.nn.get("vae_seed", seed))
        if weights is None:
            params = synthetic_encoder(spec, seed)
        elif isinstance(weights, str):
            spec, params = from_torchscript(weights, spec.shape)
        else:
            spec, params = weights
        self.spec = spec
        self.vae = _lib.Vae(self.ctx, pack(spec, params), self.B)
        yz = depth2range_table(spec.shape, cfg.sensor.hfov, cfg.sensor.vfov)
        self.yz = _lib.DeviceArray.from_numpy(self.ctx, yz)
        self.opts = _lib.vae_opts(cfg, clip_scale(cfg) if not cfg.sensor.get("is_normalized", False) else 1.0)
        self.depth2range = bool(cfg.sensor.get("is_depth", True))
        self.img = None
        self.latent = _lib.DeviceArray.from_numpy(self.ctx, np.zeros((self.B, spec.size_latent), np.float32))
        self.latent64 = _lib.DeviceArray.from_numpy(self.ctx, np.zeros((self.B, spec.size_latent), np.float64))

    def set_img(self, img):
        from . import _lib

        if hasattr(img, "data_ptr"):  # already on the device: [B][H][W] float32 / uint16, used in place
            if tuple(img.shape)[0] != self.B or len(img.shape) != 3:
                raise ValueError(f"expected a device array [{self.B}, H, W], got {tuple(img.shape)}")
            self.img = _lib.sync_producer(img)  # a torch tensor may still be in flight on torch's stream
            return
        a = np.asarray(img)
        if a.dtype != np.uint16:
            a = a.astype(np.float32)
        if a.ndim == 2:
            a = a[None]
        if a.shape[0] != self.B:
            raise ValueError(f"expected {self.B} images, got {a.shape[0]}")
        if self.img is None or not isinstance(self.img, _lib.DeviceArray) or self.img.shape != a.shape or \
                self.img.dtype != a.dtype:
            self.img = _lib.DeviceArray(self.ctx, a.shape, a.dtype)
        self.img.upload(a)

    def set_latent(self, latent):
        self.latent.upload(np.reshape(np.asarray(latent, dtype=np.float32), (self.B, -1)))

    def encode(self):
        self._run()
        out = self.latent.numpy()
        return out[0] if self.B == 1 else out

    def _run(self):
        if self.img is None:
            raise ValueError("set_img before encode")
        from . import _lib
        _lib.vae_encode(self.ctx, self.vae, self.opts, self.img, self.yz, self.latent, self.latent64,
                        depth2range=self.depth2range)

    def encode_to(self, nmpc, W_p_Bo, W_R_Bo, flag=None):
        """encode + ``nmpc.set_latent_device`` with the fp64 latents (no host round trip).  The encoder and
        the controller's parts may use other streams: set_latent_device drains the encoder's stream before
        any part on another context reads latent64 in place (controller._producer_done)."""
        self._run()
        nmpc.set_latent_device(self.latent64, W_p_Bo, W_R_Bo, flag)
