"""Host side of the controller mirror (sdf-nmpc_amd/controller.py) against the reference's own
Nmpc.set_latent / set_sdf_flag / set_ref outputs (tests/golden/params_golden.npz, made by
tests/golden/make_golden.py from sdf_nmpc/controller.py:47-56,136-142).  No GPU: the OCP is a stub."""
import numpy as np
import pytest

from sdf_nmpc_amd.config import Config
from sdf_nmpc_amd.controller import Nmpc
from sdf_nmpc_amd.reference import Ref


class StubOcp:
    """Records the calls Nmpc makes (no device)."""

    def __init__(self):
        self.calls = []

    def init(self, x0):
        self.calls.append(("init", np.array(x0)))

    def shift(self, k):
        self.calls.append(("shift", k))

    def solve(self, *a):
        self.calls.append(("solve",) + tuple(np.array(v) for v in a))

    def upload(self, name, host, col0=0, ncol=None, mask=None):
        self.calls.append(("upload", name, col0, ncol, None if mask is None else np.array(mask), np.array(host)))

    def get_u(self):
        return np.zeros(4)


def make(batch=1, N=40):
    return Nmpc(Config(mpc__N=N), batch=batch, ocp=StubOcp())


def ref_from_row(cfg, row):
    r = Ref(cfg)
    r.p, r.q, r.v, r.wz = row[0:3], row[3:7], row[7:10], row[10]
    r.Wp, r.Wq, r.Wv, r.Ww, r.Wa = row[11:14], row[14:17], row[17:20], row[20:23], row[23]
    return r


@pytest.mark.parametrize("case", range(4))
def test_params_match_reference(golden, case):
    g = golden["params"]
    c = f"c{case}/"
    n = make()
    n.set_sdf_flag(bool(g[c + "flag"]))
    n.set_latent(g[c + "latent"], g[c + "W_p_Bo"], g[c + "W_R_Bo"])
    for k, row in enumerate(g[c + "refs"]):
        n.set_ref(ref_from_row(n.cfg, row), k)
    for key in ("p", "y", "W", "yN", "WN"):
        np.testing.assert_array_equal(getattr(n, key), g[c + key], err_msg=key)


def test_batched_params_equal_per_instance(golden):
    g = golden["params"]
    B = 4
    nb = make(batch=B)
    nb.set_sdf_flag(np.array([bool(g[f"c{c}/flag"]) for c in range(B)]))
    nb.set_latent(np.stack([g[f"c{c}/latent"] for c in range(B)]), np.stack([g[f"c{c}/W_p_Bo"] for c in range(B)]),
                  np.stack([g[f"c{c}/W_R_Bo"] for c in range(B)]))
    for c in range(B):
        for k, row in enumerate(g[f"c{c}/refs"]):
            nb.set_ref(ref_from_row(nb.cfg, row), k, b=c)
    for c in range(B):
        for key in ("p", "y", "W", "yN", "WN"):
            np.testing.assert_array_equal(getattr(nb, key)[c], g[f"c{c}/{key}"], err_msg=key)


def test_reset_and_control_iteration_calls():
    n = make(N=20)
    n.set_latent(np.ones(128), np.ones(3), np.eye(3))
    n.set_sdf_flag(True)
    n.reset()
    assert not n.p.any() and n.x0 is None and n.fail_count == 0
    x0 = np.arange(12.0)
    n.set_x0(x0)
    n.set_x0(x0 + 1)  # only the first feedback initialises the OCP (controller.py:67-71)
    assert [c[0] for c in n.ocp.calls] == ["init"]
    np.testing.assert_array_equal(n.ocp.calls[0][1], x0[:10])
    assert n.solve() == 0
    kinds = [c[0] for c in n.ocp.calls]
    assert kinds[:2] == ["init", "shift"] and kinds[-1] == "solve" and set(kinds[2:-1]) == {"upload"}
    assert n.ocp.calls[1][1] == n.cfg.mpc.shift
    np.testing.assert_array_equal(n.ocp.calls[-1][1], x0[:10] + 1)
    # reset() marked everything: every column group of p and every reference field went up whole
    up = {(c[1], c[2]) for c in n.ocp.calls if c[0] == "upload"}
    assert up == {("p", 0), ("p", 1), ("p", 13), ("p", 17), ("yref", 0), ("W", 0), ("yNref", 0), ("WN", 0)}


def test_solve_uploads_only_dirty_regions():
    """host setters mark what they wrote; solve uploads exactly that (device-side writes of
    other regions survive), and nothing twice."""
    n = make(N=20)
    n.set_x0(np.zeros(10))
    n.solve()
    n.ocp.calls.clear()
    n.solve()
    assert [c[0] for c in n.ocp.calls] == ["shift", "solve"]  # nothing dirty
    n.ocp.calls.clear()
    r = Ref(n.cfg)
    r.p, r.q = np.ones(3), np.array([1.0, 0, 0, 0])
    r.use_weights(r.W_on)
    n.set_ref(r, 3)
    n.solve()
    ups = [c for c in n.ocp.calls if c[0] == "upload"]
    assert sorted((c[1], c[2]) for c in ups) == [("W", 0), ("p", 13), ("yref", 0)]
    for c in ups:
        rows = np.flatnonzero(c[4].ravel())
        assert list(rows) == [3], (c[1], rows)
    # a device-side setter clears the host marks of the regions it wrote
    n.ocp.calls.clear()
    n.set_ref(r, 5)
    n._clean("q_d", "yref", "W", "yNref", "WN")
    n.solve()
    assert [c[0] for c in n.ocp.calls] == ["shift", "solve"]


def test_solver_failure_counts():
    n = make(N=20)

    def boom(*a):
        raise RuntimeError("qp")
    n.ocp.solve = boom
    n.set_x0(np.zeros(10))
    assert n.solve() == 1 and n.solve() == 2


def test_commands_at_hover(cfg):
    n = make(N=20)
    x = np.zeros(10)
    x[3] = 1.0
    n.x0 = x
    n.ocp.get_u = lambda: n.model.u_hover
    np.testing.assert_allclose(n.get_cmd_acc(), [0, 0, 0, 0], atol=1e-12)
    np.testing.assert_allclose(n.get_cmd_TRPYr(), n.cmd_TRPYr_hover, rtol=1e-12)
