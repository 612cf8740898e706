"""NeuralDF variants beyond the deployed net (sdf_nmpc/network/neural_df.py:13-103): activation, embedding,
residual input of layer 3, layer sizes (non-multiples of 128 exercise the padded schedule) and frequency
count.  Shared by make_golden.py (variants_golden.npz, from the reference's own NeuralDF) and the tests."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import sdf_nmpc_amd  # noqa: E402,F401
from sdf_nmpc_amd import weights as W  # noqa: E402

NET_VARIANTS = {
    "relu_pos_full": W.NetSpec(act="relu", embed="pos", res="full", layer_sizes=(256, 256, 256, 256), w0=1.0),
    "softplus_cube_state": W.NetSpec(act="softplus", embed="cube", res="state", w0=1.0),
    "sin_dod_latent": W.NetSpec(act="sin", embed="dod", res="latent"),
    "sin_ico_full": W.NetSpec(act="sin", embed="ico", res="full", layer_sizes=(128, 128, 128, 128)),
    "relu_none_state": W.NetSpec(act="relu", embed="none", res="state", layer_sizes=(192, 160, 100, 50), w0=1.0),
    "sin_oct6_full": W.NetSpec(act="sin", embed="oct", res="full", nb_freqs=6, w0=30.0),
    # round 4: a plain MLP (any `res` outside full / state / latent, neural_df.py:76-78, 97-100) and latent
    # sizes other than 128 (neural_df.py:16): 64 and 200 (zero-padded to 256 on the GEMMs)
    "relu_pos_none": W.NetSpec(act="relu", embed="pos", res="none", layer_sizes=(256, 192, 128, 64), w0=1.0),
    "sin_oct_full_L64": W.NetSpec(act="sin", embed="oct", res="full", size_latent=64),
    "softplus_cube_latent_L200": W.NetSpec(act="softplus", embed="cube", res="latent", size_latent=200, w0=1.0),
}
SEED, BIAS_GAIN = 7, 0.5  # variants_golden.npz weights: W.siren_weights(spec, SEED, bias_gain=BIAS_GAIN)


def variant_input(g, name):
    """The fixture inputs of variant `name`: its own ([n, 3 + size_latent]) when its latent is not 128."""
    return g[f"{name}/input"] if f"{name}/input" in g.files else g["input"]
