"""NeuralDF weights: architecture spec, deterministic SIREN-init generator, packed `.sdfw` format.

This module is host-side plumbing for the hot path: it produces the fp32 parameter set that the
HIP kernels (``csrc/sdf_mlp.hip``) consume through the C ABI (``include/sdfnmpc.h``).

Reference anchors (``/root/reference``):
  * architecture / parameter order ... ``sdf_nmpc/network/neural_df.py:61-89`` (``layers`` ModuleDict)
  * forward semantics ................ ``sdf_nmpc/network/neural_df.py:91-103``
  * positional embedding ............. ``sdf_nmpc/utils/embeddings.py:12-111`` ('octohedron' dirs :37-51)
  * SIREN init ....................... ``sdf_nmpc/utils/layer_init.py:15-25``
  * deployed hyper-parameters ........ ``scripts/neural_nets/df_train.py:98-102``
    (``layer_sizes=[256,256,128,64]``, ``embed='oct'``, ``nb_freqs=5``, ``w0=20``, ``res='full'``)

The real trained weights (``sdf_nmpc/data/sdf_90_25664.pt``) are git-LFS pointers that are absent
from the reference checkout, so every test and benchmark uses weights regenerated from a seed by
the counter-based PRNG below. The same PRNG is implemented in C (``csrc/engine.cpp:prng_fill``) and in the
oracle, so weights never need to be committed.
"""
from __future__ import annotations

import dataclasses
import struct
from typing import Dict, List, Tuple

import numpy as np

MAGIC = b"SDFNMPCW"
VERSION = 1  # res='full', act='sin' networks (every deployed / C5 blob); version 2 adds the activation
_HDR = struct.Struct("<8s10I2f")  # magic, version, nb_states, L, n1..n4, nb_freqs, n_dirs, res, w0, max_df
_HDR2 = struct.Struct("<8s11I2f")  # version 2: ... n_dirs, res, act, w0, max_df
# neural_df.py:76-78, 97-100: layer 3 sees [h2 | e | z] ('full'), [h2 | e] ('state'), [h2 | z] ('latent');
# any other value of `res` gives a plain MLP (layer 3 sees h2 only), stored as 'none'
RES_CODES = {"full": 0, "state": 1, "latent": 2, "none": 3}


def norm_res(res) -> str:
    """The reference's `res` argument as this build names it: 'full' / 'state' / 'latent', anything else
    (None, 'none', False, ...) 'none' -- neural_df.py only tests membership in those three."""
    return res if res in ("full", "state", "latent") else "none"
ACT_CODES = {"sin": 0, "relu": 1, "softplus": 2}   # neural_df.py:40-47

# embedding projection directions, one row per direction (embeddings.py:20-100)
_OCT = [(-1, -1, -1), (-1, -1, +1), (-1, +1, -1), (-1, +1, +1),
        (+1, -1, -1), (+1, -1, +1), (+1, +1, -1), (+1, +1, +1)]
_CUBE = [(-1, 0, 0), (+1, 0, 0), (0, -1, 0), (0, +1, 0), (0, 0, -1), (0, 0, +1)]
_PHI = (1 + np.sqrt(5)) / 2
_DOD = [(0, -1, -_PHI), (0, +1, -_PHI), (0, -1, +_PHI), (0, +1, +_PHI), (-1, 0, -_PHI), (+1, 0, -_PHI),
        (-1, 0, +_PHI), (+1, 0, +_PHI), (-1, -_PHI, 0), (+1, -_PHI, 0), (-1, +_PHI, 0), (+1, +_PHI, 0)]
_H = 1 / _PHI
_ICO = [(+1, +1, +1), (+1, +1, -1), (+1, -1, +1), (+1, -1, -1), (-1, +1, +1), (-1, +1, -1), (-1, -1, +1),
        (-1, -1, -1), (0, +_PHI, +_H), (0, +_PHI, -_H), (0, -_PHI, +_H), (0, -_PHI, -_H), (+_H, 0, +_PHI),
        (+_H, 0, -_PHI), (-_H, 0, +_PHI), (-_H, 0, -_PHI), (+_PHI, +_H, 0), (+_PHI, -_H, 0), (-_PHI, +_H, 0),
        (-_PHI, -_H, 0)]
EMBED_BY_DIRS = {0: "none", 3: "pos", 6: "cube", 8: "oct", 12: "dod", 20: "ico"}


def embedding_dirs(embed: str) -> np.ndarray:
    """fp32 [3, n_dirs] projection matrix exactly as torch builds it (embeddings.py:20-100); 'none' (no
    embedding, neural_df.py:50-52) has no directions.

    The reference lists the directions as Python floats and builds an fp32 tensor (each value rounded
    once), then normalises each column with ``vector_norm`` in fp32: torch accumulates the squares with
    fused multiply-adds (acc = fma(x, x, acc), one rounding per component -- the dod / ico columns with a
    zero in the middle tell it from a sum of rounded squares), takes an fp32 sqrt and divides with one
    rounding; numpy reproduces that bit for bit (fp32 products are exact in fp64).
    """
    if embed == "none":
        return np.zeros((3, 0), dtype=np.float32)
    if embed == "pos":
        return np.eye(3, dtype=np.float32)
    if embed == "cube":  # not normalised in the reference (embeddings.py:26-36)
        return np.array(_CUBE, dtype=np.float32).T.copy()
    tab = {"oct": _OCT, "dod": _DOD, "ico": _ICO}.get(embed)
    if tab is None:
        raise ValueError(f"unknown embedding '{embed}' (none, pos, cube, oct, dod, ico)")
    d = np.array(tab, dtype=np.float64).astype(np.float32).T.copy()
    acc = np.zeros(d.shape[1], dtype=np.float32)
    for c in range(3):
        acc = (d[c].astype(np.float64) * d[c].astype(np.float64) + acc.astype(np.float64)).astype(np.float32)
    n = np.sqrt(acc).astype(np.float32)
    return (d / n[None, :]).astype(np.float32)


@dataclasses.dataclass(frozen=True)
class NetSpec:
    """Architecture of one NeuralDF (neural_df.py:13-26 constructor arguments)."""
    size_latent: int = 128
    layer_sizes: Tuple[int, int, int, int] = (256, 256, 128, 64)
    nb_freqs: int = 5
    embed: str = "oct"
    w0: float = 20.0
    max_df: float = 1.0
    nb_states: int = 3
    act: str = "sin"    # 'sin' | 'relu' | 'softplus' (neural_df.py:40-47)
    res: str = "full"   # 'full' | 'state' | 'latent' | 'none': what layer 3 sees besides h2 (neural_df.py:76-78)

    def __post_init__(self):
        object.__setattr__(self, "res", norm_res(self.res))

    @property
    def n_dirs(self) -> int:
        return embedding_dirs(self.embed).shape[1]

    @property
    def n_embed(self) -> int:  # embeddings.py:104
        return self.nb_freqs * self.n_dirs * 2 + 3

    def param_shapes(self) -> List[Tuple[str, Tuple[int, ...]]]:
        """Parameter names/shapes in torch ``state_dict`` order (neural_df.py:61-89)."""
        E, L = self.n_embed, self.size_latent
        n1, n2, n3, n4 = self.layer_sizes
        c3 = n2 + {"full": E + L, "state": E, "latent": L, "none": 0}[self.res]
        return [
            ("layers.main1.0.weight", (n1, E + L)), ("layers.main1.0.bias", (n1,)),
            ("layers.main1.3.weight", (n2, n1)), ("layers.main1.3.bias", (n2,)),
            ("layers.main2.0.weight", (n3, c3)), ("layers.main2.0.bias", (n3,)),
            ("layers.main2.3.weight", (n4, n3)), ("layers.main2.3.bias", (n4,)),
            ("layers.df.0.weight", (1, n4)), ("layers.df.0.bias", (1,)),
        ]

    def n_params(self) -> int:
        return int(sum(np.prod(s) for _, s in self.param_shapes()))


DEFAULT_SPEC = NetSpec()
WIDE_SPEC = NetSpec(layer_sizes=(1024, 1024, 512, 256))  # BASELINE config 5


# ---------------------------------------------------------------------------------------------
# counter-based PRNG (splitmix64 finaliser); mirrored in csrc/engine.cpp (prng_fill) and oracle/oracle.c
# ---------------------------------------------------------------------------------------------
_M64 = (1 << 64) - 1
_GOLD = 0x9E3779B97F4A7C15
_TSTEP = 0xD1B54A32D192ED03


def _mix64_int(z: int) -> int:
    z &= _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def _mix64_np(z: np.ndarray) -> np.ndarray:
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def prng_uniform(seed: int, stream: int, n: int) -> np.ndarray:
    """n doubles in [0,1) with 24 random bits each; element i depends only on (seed, stream, i)."""
    key = _mix64_int(seed * _GOLD + stream * _TSTEP + 1)
    i = np.arange(1, n + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = _mix64_np(np.uint64(key) + i * np.uint64(_GOLD))
    return (x >> np.uint64(40)).astype(np.float64) * (2.0 ** -24)


def siren_weights(spec: NetSpec = DEFAULT_SPEC, seed: int = 0, weight_gain: float = 1.0,
                  bias_gain: float = 0.0) -> Dict[str, np.ndarray]:
    """SIREN-initialised parameters (layer_init.py:15-25): W ~ U(+-sqrt(6/n_in)/w0), b = 0.

    ``weight_gain`` scales the weight range (x2..x4 stresses the sin range reduction: trained nets
    need not stay inside the init range); ``bias_gain`` > 0 draws biases from
    U(+-bias_gain*sqrt(6/n_in)/w0) so the bias path is exercised (the reference init zeroes them).
    Values are rounded once from double to fp32, identically in the C generator.
    """
    out = {}
    shapes = spec.param_shapes()
    for t in range(0, len(shapes), 2):
        (wn, ws), (bn, bs) = shapes[t], shapes[t + 1]
        bound = np.sqrt(6.0 / ws[-1]) / spec.w0
        u = prng_uniform(seed, t, int(np.prod(ws)))
        out[wn] = ((2.0 * u - 1.0) * (bound * weight_gain)).astype(np.float32).reshape(ws)
        if bias_gain > 0.0:
            ub = prng_uniform(seed, t + 1, int(np.prod(bs)))
            out[bn] = ((2.0 * ub - 1.0) * (bound * bias_gain)).astype(np.float32).reshape(bs)
        else:
            out[bn] = np.zeros(bs, dtype=np.float32)
    return out


# ---------------------------------------------------------------------------------------------
# packed binary format
# ---------------------------------------------------------------------------------------------
def pack(spec: NetSpec, params: Dict[str, np.ndarray]) -> bytes:
    """Serialise to the `.sdfw` layout read by ``sdfnmpc_net_load_file`` (include/sdfnmpc.h)."""
    dirs = embedding_dirs(spec.embed)
    nf = spec.nb_freqs if dirs.shape[1] else 0  # embed 'none': no frequencies
    freqs = (2.0 ** np.linspace(0, nf - 1, nf)).astype(np.float32)
    if spec.act == "sin" and spec.res == "full":  # version 1: byte-identical to every earlier blob
        hdr = _HDR.pack(MAGIC, VERSION, spec.nb_states, spec.size_latent, *spec.layer_sizes,
                        nf, dirs.shape[1], 0, spec.w0, spec.max_df)
    else:
        hdr = _HDR2.pack(MAGIC, 2, spec.nb_states, spec.size_latent, *spec.layer_sizes, nf, dirs.shape[1],
                         RES_CODES[spec.res], ACT_CODES[spec.act], spec.w0, spec.max_df)
    body = [dirs.astype("<f4").tobytes(), freqs.astype("<f4").tobytes()]
    for name, shape in spec.param_shapes():
        a = np.asarray(params[name], dtype=np.float32)
        if a.shape != shape:
            raise ValueError(f"{name}: shape {a.shape} != {shape}")
        body.append(a.astype("<f4").tobytes())
    return hdr + b"".join(body)


def unpack(blob: bytes) -> Tuple[NetSpec, Dict[str, np.ndarray]]:
    magic, ver = struct.unpack_from("<8sI", blob, 0)
    if magic != MAGIC or ver not in (1, 2):
        raise ValueError("not a version-1/2 .sdfw blob")
    if ver == 1:
        _, _, ns, L, n1, n2, n3, n4, nf, nd, res, w0, max_df = _HDR.unpack_from(blob, 0)
        act, hsize = 0, _HDR.size
        if res != 0:
            raise ValueError("version-1 .sdfw blobs are res='full'")
    else:
        _, _, ns, L, n1, n2, n3, n4, nf, nd, res, act, w0, max_df = _HDR2.unpack_from(blob, 0)
        hsize = _HDR2.size
    spec = NetSpec(size_latent=L, layer_sizes=(n1, n2, n3, n4), nb_freqs=nf if nd else 5, embed=EMBED_BY_DIRS[nd],
                   w0=float(w0), max_df=float(max_df), nb_states=ns,
                   act={v: k for k, v in ACT_CODES.items()}[act], res={v: k for k, v in RES_CODES.items()}[res])
    off = hsize + 4 * (3 * nd + nf)
    params = {}
    for name, shape in spec.param_shapes():
        n = int(np.prod(shape))
        params[name] = np.frombuffer(blob, dtype="<f4", count=n, offset=off).reshape(shape).copy()
        off += 4 * n
    if off != len(blob):
        raise ValueError("trailing bytes in .sdfw blob")
    return spec, params


def save(path: str, spec: NetSpec, params: Dict[str, np.ndarray]) -> None:
    with open(path, "wb") as f:
        f.write(pack(spec, params))


def load(path: str) -> Tuple[NetSpec, Dict[str, np.ndarray]]:
    with open(path, "rb") as f:
        return unpack(f.read())


def from_torchscript(path: str) -> Tuple[NetSpec, Dict[str, np.ndarray]]:
    """Convert a NeuralDF TorchScript archive of YOUR OWN (e.g. a df_train.py output,
    ``df_train.py:250-253``) to (spec, params). Offline tool; the product never calls it.
    The reference's ``sdf_nmpc/data/*.pt`` are LFS pointers in this checkout and are not read.
    """
    import torch  # offline only

    m = torch.jit.load(path, map_location="cpu")
    sd = {k: v.detach().cpu().numpy() for k, v in m.state_dict().items()}
    n1 = sd["layers.main1.0.weight"].shape[0]
    n2 = sd["layers.main1.3.weight"].shape[0]
    n3 = sd["layers.main2.0.weight"].shape[0]
    n4 = sd["layers.main2.3.weight"].shape[0]
    nd = sd["embed.dirs"].shape[1] if "embed.dirs" in sd else 0
    nf = sd["embed.freq_bands"].shape[0] if nd else 5
    E = 3 + 2 * nf * nd
    L = sd["layers.main1.0.weight"].shape[1] - E
    embed = EMBED_BY_DIRS[nd]
    spec = NetSpec(size_latent=L, layer_sizes=(n1, n2, n3, n4), nb_freqs=nf, embed=embed,
                   w0=float(m.w0), max_df=float(m.max_df), act=str(getattr(m, "activation", "sin")),
                   res=norm_res(getattr(m, "res", "full")))
    if nd and not np.array_equal(sd["embed.dirs"], embedding_dirs(embed)):
        raise ValueError("unexpected embedding directions")
    return spec, {k: sd[k] for k, _ in spec.param_shapes()}


if __name__ == "__main__":  # offline converter: python -m sdf_nmpc_amd.weights model.pt model.sdfw
    import sys

    if len(sys.argv) != 3:
        raise SystemExit("usage: python -m sdf_nmpc_amd.weights <neural_df TorchScript .pt> <out .sdfw>")
    _spec, _params = from_torchscript(sys.argv[1])
    save(sys.argv[2], _spec, _params)
    print(f"{sys.argv[2]}: {_spec} ({_spec.n_params()} parameters)")
