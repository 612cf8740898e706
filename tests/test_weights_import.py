"""weights.from_torchscript (the offline TorchScript -> .sdfw converter) against the
state_dict layout of the reference's own scripted NeuralDF (tests/golden/ts_golden.npz, made by
tests/golden/make_golden.py from torch.jit.script(NeuralDF(...)) -- names, shapes, embedding buffers,
w0 / max_df; the reference's trained .pt files are LFS pointers and are not read).
"""
import numpy as np
import pytest

from sdf_nmpc_amd import weights as W

torch = pytest.importorskip("torch")


def _scripted_like_reference(ts, params):
    """A TorchScript module with the reference's state_dict layout, filled with `params`."""
    class Node(torch.nn.Module):
        def forward(self, x):
            return x

    root = Node()
    shared = {}
    for key in ts["keys"]:
        key = str(key)
        *path, leaf = key.split(".")
        mod = root
        for i, part in enumerate(path):
            sub = getattr(mod, part, None) if part in mod._modules else None
            if sub is None:
                # `embed` and `layers.embeddings.0` are one module object in NeuralDF (neural_df.py:53-58)
                full = ".".join(path[: i + 1])
                sub = shared.get("embed") if full in ("embed", "layers.embeddings.0") and "embed" in shared else Node()
                if full in ("embed", "layers.embeddings.0"):
                    shared["embed"] = sub
                mod.add_module(part, sub)
            mod = sub
        if "embed" in key:
            if leaf not in mod._buffers:
                mod.register_buffer(leaf, torch.from_numpy(ts[f"buf/{key}"].copy()))
        else:
            mod.register_parameter(leaf, torch.nn.Parameter(torch.from_numpy(params[key].copy())))
    root.w0 = float(ts["w0"])
    root.max_df = float(ts["max_df"])
    return torch.jit.script(root)


def test_from_torchscript_reads_the_reference_layout(tmp_path):
    import os
    ts = np.load(os.path.join(os.path.dirname(__file__), "golden", "ts_golden.npz"))
    spec = W.DEFAULT_SPEC
    params = W.siren_weights(spec, seed=7, weight_gain=2.0, bias_gain=1.0)
    for k, shape in spec.param_shapes():  # our names / shapes are the reference's
        assert tuple(ts[f"shape/{k}"]) == shape
    m = _scripted_like_reference(ts, params)
    path = str(tmp_path / "sdf.pt")
    m.save(path)
    spec2, params2 = W.from_torchscript(path)
    assert spec2 == spec
    for k in params:
        assert np.array_equal(params[k], params2[k])
    # round trip into the packed format the HIP library loads
    spec3, params3 = W.unpack(W.pack(spec2, params2))
    assert spec3 == spec and all(np.array_equal(params[k], params3[k]) for k in params)
