"""The C-ABI libraries load on a CPU-only host and export every symbol the headers declare.

No compute calls here (no GPU in the build container); host-only entry points (shooting grid, error
reporting) are exercised.
"""
import ctypes
import os
import re

import numpy as np
import pytest

import sdf_nmpc_amd
from sdf_nmpc_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions(name):
    src = open(os.path.join(ROOT, "include", name)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b([a-z_][a-z0-9_]*)\s*\([^;{]*\)\s*;", src)))


@pytest.fixture(scope="module")
def libs():
    if not os.path.exists(_lib.LIB_PATH):
        import __graft_entry__
        __graft_entry__.build()
    return ctypes.CDLL(_lib.LIB_PATH), ctypes.CDLL(_lib.L4C_PATH)


def test_sdfnmpc_exports_header(libs):
    lib, _ = libs
    fns = header_functions("sdfnmpc.h")
    assert len(fns) >= 20
    missing = [f for f in fns if not hasattr(lib, f)]
    assert not missing, missing
    assert sorted(_lib.SYMBOLS) == fns


def test_sdf_l4c_exports_header(libs):
    _, l4c = libs
    fns = header_functions("sdf_l4c.h")
    missing = [f for f in fns if not hasattr(l4c, f)]
    assert not missing, missing
    assert set(_lib.L4C_SYMBOLS) <= set(fns)


def test_l4c_casadi_metadata(libs):
    """CasADi external protocol metadata: 1 in (131x1 dense) / 1 out (1x1); jac: 2 in / 1 out (1x131)."""
    _, l4c = libs
    for fn in ("sdf_l4c_n_in", "sdf_l4c_n_out", "jac_sdf_l4c_n_in", "jac_sdf_l4c_n_out", "adj1_sdf_l4c_n_in"):
        getattr(l4c, fn).restype = ctypes.c_longlong
    assert (l4c.sdf_l4c_n_in(), l4c.sdf_l4c_n_out()) == (1, 1)
    assert (l4c.jac_sdf_l4c_n_in(), l4c.jac_sdf_l4c_n_out()) == (2, 1)
    assert l4c.adj1_sdf_l4c_n_in() == 3
    P = ctypes.POINTER(ctypes.c_longlong)
    for fn in ("sdf_l4c_sparsity_in", "sdf_l4c_sparsity_out", "jac_sdf_l4c_sparsity_out"):
        getattr(l4c, fn).restype = P
        getattr(l4c, fn).argtypes = [ctypes.c_longlong]
    sp = l4c.sdf_l4c_sparsity_in(0)
    assert (sp[0], sp[1], sp[2], sp[3]) == (131, 1, 0, 131) and [sp[4 + i] for i in range(131)] == list(range(131))
    so = l4c.sdf_l4c_sparsity_out(0)
    assert [so[i] for i in range(5)] == [1, 1, 0, 1, 0]
    sj = l4c.jac_sdf_l4c_sparsity_out(0)
    assert (sj[0], sj[1]) == (1, 131)
    assert [sj[2 + j] for j in range(132)] == list(range(132))
    assert all(sj[2 + 132 + j] == 0 for j in range(131))
    assert not l4c.sdf_l4c_sparsity_in(1)


def test_shooting_grid_bit_exact_via_abi(golden, cfg):
    """a13: ocp.py:21-27 shooting nodes and dt, bit for bit, through the product C ABI."""
    G = golden["grid"]
    for N in (20, 40, 60):
        nodes, dt = _lib.shooting_grid(N, cfg.mpc.T)
        assert np.array_equal(nodes, G[f"N{N}/uniform/nodes"]) and np.array_equal(dt, G[f"N{N}/uniform/dt"])
        nodes, dt = _lib.shooting_grid(N, cfg.mpc.T, False, cfg.mpc.nb_short_nodes, cfg.mpc.control_loop_time * 1e-3)
        assert np.array_equal(nodes, G[f"N{N}/nonuniform/nodes"]) and np.array_equal(dt, G[f"N{N}/nonuniform/dt"])
    for N, ns in ((5, 1), (7, 7), (1, 1)):  # edge cases vs numpy itself
        nodes, dt = _lib.shooting_grid(N, 1.5, False, ns, 0.01)
        ref = np.hstack([np.linspace(0, 0.01 * (ns - 1), ns), np.linspace(0.01 * ns, 1.5, N - ns + 1)])
        assert np.array_equal(nodes, ref) and np.array_equal(dt, np.diff(ref))
    with pytest.raises(_lib.SdfnmpcError):
        _lib.shooting_grid(0, 1.5)


def test_no_cpu_fallback_without_gpu():
    """The product path fails loudly (no silent CPU fallback) when no HIP device is visible."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is visible")
    with pytest.raises(_lib.SdfnmpcError, match="no HIP device"):
        _lib.Context(0)
