"""Dense reference solver for the SQP-RTI QP -- TEST INFRASTRUCTURE ONLY (the checker of csrc/rti_qp.hip).

The QP is the one acados builds in the RTI preparation phase and HPIPM solves in the feedback phase
(sdf_nmpc/ocp.py:54-120: NONLINEAR_LS + GAUSS_NEWTON, levenberg_marquardt = mpc.lm_reg, ERK, soft
nonlinear constraints idxsh with L1/L2 slack penalties, input box constraints, x_0 fixed):

  min  sum_{k<N} s_k [ 1/2 |J_y,k w_k + r_k|^2_{W_k} ] + 1/2 lm_k |w_k|^2   (lm_k = lm dt_k, see stage_qp)
     + s_N 1/2 |J_yN dx_N + r_N|^2_{W_N} + 1/2 lm |dx_N|^2
     + sum_{k<=N} s_k (zl.sl_k + 1/2 Zl.sl_k^2 + zu.su_k + 1/2 Zu.su_k^2)
  s.t. dx_0 = x0 - xbar_0,  dx_{k+1} = A_k dx_k + B_k du_k + (xn_k - xbar_{k+1})
       lbu - ubar_k <= du_k <= ubu - ubar_k
       lh - h_k - sl_k <= J_h,k dx_k <= uh - h_k + su_k,  sl_k, su_k >= 0   (the soft rows of the constraint set)
       lh - h_k <= J_h,k dx_k <= uh - h_k              (hard rows: slack weight None, base_model.py:142-168;
                                                          rec_feas / stability terminal rows)
  w_k = [dx_k; du_k], r_k = y_k - yref_k, s_k = cost scaling (acados default: dt_k for k < N, 1 at N)

HPIPM's algorithm (Riccati-based IPM) is not reproducible here (acados is absent; parity at the
acados boundary is unpinned); the QP is strictly convex (lm > 0) so its solution is
unique, and this solver -- a textbook Mehrotra predictor-corrector on the full dense KKT system --
pins it independently of the GPU solver's structure.
"""
import numpy as np


def stage_qp(lin, xbar, ubar, x0, yref, W, yNref, WN, dt, model, lm, scaling=None, lm_scaling=True):
    """Assemble the per-stage QP data of ONE instance from the linearisation outputs.

    lin: dict with xn [N,10], AB [N,14,10], y [N,11], Jy [N,14,11], yN [nyN], JyN [10,nyN], h [N+1,3],
    Jh [N+1,10,3] (+ hE [6], JhE [10,6] when a terminal row reads them) -- the sdfnmpc_linearize layouts,
    column-major blocks.  The constraint set is model's (model.Quad: h_cols, nhs, term_rows): stage k < N has
    the rows h[k][h_cols], the last nhs of them hard; the terminal node the rows of term_rows (soft first,
    then hard), each the sum of an h[N] column and an hE column (gen_model.py:26-149).
    """
    N = xbar.shape[0] - 1
    s = np.concatenate([dt, [1.0]]) if scaling is None else np.asarray(scaling, float)
    q = {"N": N, "s": s}
    q["A"] = np.transpose(lin["AB"][:, :10, :], (0, 2, 1))    # [N,10,10] A[i][j]
    q["B"] = np.transpose(lin["AB"][:, 10:, :], (0, 2, 1))    # [N,10,4]
    q["c"] = lin["xn"] - xbar[1:]
    Jy = np.transpose(lin["Jy"], (0, 2, 1))                   # [N,11,14]
    r = lin["y"] - yref[:, :11]
    if W.shape[-1] == 12:  # flags.sdf_cost (gen_model.py:65-66): residual (1 - s/2)^4 of s = h[2]
        t = 1.0 - 0.5 * lin["h"][:N, 2]
        j = np.zeros((N, 1, 14))
        j[:, 0, :10] = (-2.0 * t ** 3)[:, None] * lin["Jh"][:N, :, 2]
        Jy = np.concatenate([Jy, j], axis=1)
        r = np.concatenate([r, (t ** 4 - yref[:, 11])[:, None]], axis=1)
    # Levenberg-Marquardt term: lm dt_k at k < N with lm_scaling (acados: Ts[k] * levenberg_marquardt), lm at N
    lmk = lm * np.asarray(dt, float)[:N] if lm_scaling else np.full(N, float(lm))
    q["H"] = np.einsum("kai,ka,kaj->kij", Jy, W, Jy) * s[:N, None, None] + lmk[:, None, None] * np.eye(14)
    q["g"] = np.einsum("kai,ka,ka->ki", Jy, W, r) * s[:N, None]
    JyN = np.asarray(lin["JyN"]).T                             # [nyN,10]
    rN = lin["yN"] - yNref
    q["HN"] = JyN.T @ np.diag(WN) @ JyN * s[N] + lm * np.eye(10)
    q["gN"] = JyN.T @ (WN * rN) * s[N]
    # stage rows: the first ns soft, the last nhs hard
    hc = list(getattr(model, "h_cols", [0, 1, 2]))
    q["nhs"] = int(getattr(model, "nhs", 0))
    q["ns"] = len(hc) - q["nhs"]
    q["C"] = np.transpose(lin["Jh"][:N][:, :, hc], (0, 2, 1))  # [N,nh,10]
    q["hl"] = lin["h"][:N][:, hc] - np.asarray(model.lh)      # constant of the lower soft row
    q["hu"] = np.asarray(model.uh) - lin["h"][:N][:, hc]
    q["zl"], q["Zl"] = np.asarray(model.zl, float), np.asarray(model.Zl, float)
    # terminal rows
    rows = getattr(model, "term_rows", None)
    if rows is None:
        rows = [(c, -1, True, model.lh[i], model.uh[i], model.zl[i], model.Zl[i]) for i, c in enumerate(hc)]
    CN, hN = [], []
    for c1, c2, soft, lo, hi, zl, Zl in rows:
        cr, hv = np.zeros(10), 0.0
        if c1 >= 0:
            cr = cr + lin["Jh"][N][:, c1]
            hv += lin["h"][N][c1]
        if c2 >= 0:
            cr = cr + lin["JhE"][:, c2]
            hv += lin["hE"][c2]
        CN.append(cr)
        hN.append(hv)
    q["nhN"] = len(rows)
    q["nsN"] = sum(1 for r_ in rows if r_[2])
    q["CN"] = np.array(CN).reshape(len(rows), 10)
    q["hlN"] = np.array(hN) - np.array([r_[3] for r_ in rows])
    q["huN"] = np.array([r_[4] for r_ in rows]) - np.array(hN)
    q["zlN"] = np.array([r_[5] for r_ in rows if r_[2]], float)
    q["ZlN"] = np.array([r_[6] for r_ in rows if r_[2]], float)
    q["ulo"] = model.lbu - ubar                                # du >= ulo
    q["uhi"] = model.ubu - ubar
    q["x0"] = x0 - xbar[0]
    return q


def _layout(q):
    """Variable offsets: z = [dx_0..dx_N, du_0..du_{N-1}, sl (stage groups k ns + j, then terminal soft rows),
    su (same)].  With the default set (3 soft rows everywhere) sl / su are the [N+1][3] arrays."""
    N, nx, nu = q["N"], 10, 4
    nsl = N * q["ns"] + q["nsN"]
    o_du = (N + 1) * nx
    o_sl = o_du + N * nu
    o_su = o_sl + nsl
    return dict(N=N, nsl=nsl, o_du=o_du, o_sl=o_sl, o_su=o_su, nz=o_su + nsl)


def dense_problem(q):
    """The QP of stage_qp as one dense problem: min 1/2 z'Hz + g'z s.t. E z = e, G z + d >= 0 (z: _layout)."""
    L = _layout(q)
    N, nx, nu, ns = q["N"], 10, 4, q["ns"]
    ix = lambda k: k * nx
    iu = lambda k: L["o_du"] + k * nu
    nz = L["nz"]
    H = np.zeros((nz, nz)); g = np.zeros(nz)
    s = q["s"]
    for k in range(N):
        idx = np.r_[ix(k):ix(k) + nx, iu(k):iu(k) + nu]
        H[np.ix_(idx, idx)] += q["H"][k]
        g[idx] += q["g"][k]
    H[ix(N):ix(N) + nx, ix(N):ix(N) + nx] += q["HN"]
    g[ix(N):ix(N) + nx] += q["gN"]
    # soft groups: (node, C row, hl, hu, zl, Zl)
    groups = [(k, q["C"][k, j], q["hl"][k, j], q["hu"][k, j], q["zl"][j], q["Zl"][j]) for k in range(N) for j in range(ns)]
    groups += [(N, q["CN"][j], q["hlN"][j], q["huN"][j], q["zlN"][j], q["ZlN"][j]) for j in range(q["nsN"])]
    for e, (k, C, hl, hu, zl, Zl) in enumerate(groups):
        for o in (L["o_sl"] + e, L["o_su"] + e):
            H[o, o] += s[k] * Zl
            g[o] += s[k] * zl
    # equalities E z = e
    ne = (N + 1) * nx
    E = np.zeros((ne, nz)); e = np.zeros(ne)
    E[0:nx, ix(0):ix(0) + nx] = np.eye(nx); e[0:nx] = q["x0"]
    for k in range(N):
        r0 = (k + 1) * nx
        E[r0:r0 + nx, ix(k + 1):ix(k + 1) + nx] = np.eye(nx)
        E[r0:r0 + nx, ix(k):ix(k) + nx] = -q["A"][k]
        E[r0:r0 + nx, iu(k):iu(k) + nu] = -q["B"][k]
        e[r0:r0 + nx] = q["c"][k]
    # inequalities G z + d >= 0
    rows, d = [], []
    for k in range(N):
        for i in range(nu):
            a = np.zeros(nz); a[iu(k) + i] = 1.0; rows.append(a); d.append(-q["ulo"][k, i])
            a = np.zeros(nz); a[iu(k) + i] = -1.0; rows.append(a); d.append(q["uhi"][k, i])
    for e_, (k, C, hl, hu, zl, Zl) in enumerate(groups):
        a = np.zeros(nz); a[ix(k):ix(k) + nx] = C; a[L["o_sl"] + e_] = 1.0; rows.append(a); d.append(hl)
        a = np.zeros(nz); a[ix(k):ix(k) + nx] = -C; a[L["o_su"] + e_] = 1.0; rows.append(a); d.append(hu)
        a = np.zeros(nz); a[L["o_sl"] + e_] = 1.0; rows.append(a); d.append(0.0)
        a = np.zeros(nz); a[L["o_su"] + e_] = 1.0; rows.append(a); d.append(0.0)
    for k in range(1, N):  # hard stage rows: none at node 0 (acados 0.3.1: initial-node h rows come only
        for j in range(ns, ns + q["nhs"]):  # from con_h_expr_0, which the reference's ocp.py never sets)
            a = np.zeros(nz); a[ix(k):ix(k) + nx] = q["C"][k, j]; rows.append(a); d.append(q["hl"][k, j])
            a = np.zeros(nz); a[ix(k):ix(k) + nx] = -q["C"][k, j]; rows.append(a); d.append(q["hu"][k, j])
    for j in range(q["nsN"], q["nhN"]):  # hard terminal rows
        a = np.zeros(nz); a[ix(N):ix(N) + nx] = q["CN"][j]; rows.append(a); d.append(q["hlN"][j])
        a = np.zeros(nz); a[ix(N):ix(N) + nx] = -q["CN"][j]; rows.append(a); d.append(q["huN"][j])
    G = np.array(rows).reshape(len(rows), nz); d = np.array(d)
    return H, g, E, e, G, d


def _slack_nodes(q, v):
    """Soft-slack vector (group order) -> [N+1][3] by (node, row) (zeros where a node has fewer rows)."""
    N, ns = q["N"], q["ns"]
    out = np.zeros((N + 1, 3))
    out[:N, :ns] = v[:N * ns].reshape(N, ns)
    out[N, :q["nsN"]] = v[N * ns:]
    return out


def z_of(q, sol):
    """The dense variable vector of a solution dict (dx, du, sl / su as [N+1][3] by node and row)."""
    N, ns = q["N"], q["ns"]
    def flat(a):
        a = np.asarray(a)
        return np.concatenate([a[:N, :ns].ravel(), a[N, :q["nsN"]]])
    return np.concatenate([np.asarray(sol["dx"]).ravel(), np.asarray(sol["du"]).ravel(), flat(sol["sl"]), flat(sol["su"])])


def _unpack(q, z):
    L = _layout(q)
    N, nx, nu = q["N"], 10, 4
    return {"dx": z[:L["o_du"]].reshape(N + 1, nx), "du": z[L["o_du"]:L["o_sl"]].reshape(N, nu),
            "sl": _slack_nodes(q, z[L["o_sl"]:L["o_su"]]), "su": _slack_nodes(q, z[L["o_su"]:])}


def polish(q, sol, act_tol=1e-7):
    """Active-set polish of an IPM solution: the rows with G z + d < act_tol become equalities and the
    equality-constrained QP is solved directly (one dense KKT solve, no barrier terms, so no late-IPM
    ill-conditioning).  Returns the polished solution and the KKT check (min dual, max row violation)."""
    H, g, E, e, G, d = dense_problem(q)
    z0 = z_of(q, sol)
    act = (G @ z0 + d) < act_tol
    Ga, da = G[act], d[act]
    nz, ne, na = H.shape[0], E.shape[0], Ga.shape[0]
    K = np.block([[H, E.T, -Ga.T], [E, np.zeros((ne, ne)), np.zeros((ne, na))], [Ga, np.zeros((na, ne + na))]])
    sol_ = np.linalg.lstsq(K, np.concatenate([-g, e, -da]), rcond=None)[0]
    z, lam = sol_[:nz], sol_[nz + ne:]
    out = _unpack(q, z)
    out["min_dual"] = lam.min() if na else 0.0
    out["max_violation"] = max(0.0, -(G @ z + d).min())
    return out


def polish_active_set(q, sol, act_tol=1e-7, max_swaps=200):
    """polish() followed by active-set corrections until the KKT conditions hold: a violated row joins
    the active set, an active row with a negative multiplier leaves it (one change per solve, the worst
    first).  For a strictly convex QP the point that passes is its unique solution; near-degenerate
    vertices (weakly active rows the IPM leaves at slack ~1e-6) need this where a single threshold cut
    of the IPM point picks a wrong set."""
    H, g, E, e, G, d = dense_problem(q)
    z0 = z_of(q, sol)
    act = (G @ z0 + d) < act_tol
    nz, ne = H.shape[0], E.shape[0]
    for _ in range(max_swaps):
        Ga, da = G[act], d[act]
        na = Ga.shape[0]
        K = np.block([[H, E.T, -Ga.T], [E, np.zeros((ne, ne)), np.zeros((ne, na))], [Ga, np.zeros((na, ne + na))]])
        x = np.linalg.lstsq(K, np.concatenate([-g, e, -da]), rcond=None)[0]
        z, lam = x[:nz], x[nz + ne:]
        viol = G @ z + d
        iv = int(np.argmin(viol))
        il = int(np.argmin(lam)) if na else -1
        if viol[iv] < -1e-10 and (na == 0 or -viol[iv] >= -lam[il]):
            act[iv] = True
        elif na and lam[il] < -1e-10:
            act[np.flatnonzero(act)[il]] = False
        else:
            break
    out = _unpack(q, z)
    out["min_dual"] = lam.min() if na else 0.0
    out["max_violation"] = max(0.0, -viol.min())
    out["lam_l1"] = float(np.abs(lam).sum()) if na else 0.0  # |lambda*|_1: prices a primal residual (objective_bound)
    return out


def objective_bound(m, tol, lam_l1, rp):
    """How far above the optimum F* an IPM point stopped at max_i t_i lambda_i < tol with primal residual rp
    (max abs) may lie: F(z) - F* <= lambda' (G z + d) + r_d' (z - z*) (convexity, E z = e exactly), and
    lambda' (G z + d) = lambda' t + lambda' r_p <= m tol + |lambda|_1 rp.  The stationarity residual r_d
    decays with the step lengths (the stop test's gap term) and is left out; |lambda|_1 is the exact
    solution's (the IPM's multipliers converge to it).  On hard rows with large multipliers the second
    term is the larger."""
    return m * tol + lam_l1 * max(rp, tol)


def solve_dense(q, tol=1e-11, max_iter=100):
    """Mehrotra IPM on the full KKT system.  Returns dict(dx [N+1,10], du [N,4], sl, su [N+1,3], iters)."""
    L = _layout(q)
    nz, ne = L["nz"], (q["N"] + 1) * 10
    H, g, E, e, G, d = dense_problem(q)
    m = G.shape[0]
    z = np.zeros(nz)
    z = np.linalg.lstsq(E, e, rcond=None)[0]
    t = np.maximum(G @ z + d, 1.0)
    lam = np.ones(m)
    y = np.zeros(ne)
    it = 0
    # stationarity is measured relative to the data scale: at tight tolerances the dense LU solve of the
    # (ill-conditioned, late-IPM) KKT system cannot push |rd| below ~1e-11 absolute, and iterating on
    # then degrades the iterate -- so stop there, and otherwise return the best iterate seen
    sd = max(1.0, np.abs(g).max(), np.abs(H).max())
    best = None
    for it in range(1, max_iter + 1):
        rd = H @ z + g - G.T @ lam + E.T @ y
        rp = G @ z + d - t
        re = E @ z - e
        mu = t @ lam / m
        merit = max(np.abs(rd).max() / sd, np.abs(rp).max(), np.abs(re).max(), mu)
        if best is None or merit < best[0]:
            best = (merit, z.copy(), t.copy(), lam.copy(), it)
        if merit < tol:
            best = None
            break
        Sig = lam / t
        K = np.block([[H + G.T @ (Sig[:, None] * G), E.T], [E, np.zeros((ne, ne))]])

        def solve(rc):
            rhs1 = -rd - G.T @ (Sig * rp + rc / t)
            sol = np.linalg.solve(K, np.concatenate([rhs1, -re]))
            dz, dy = sol[:nz], sol[nz:]
            dt_ = G @ dz + rp
            dl = -(rc + lam * dt_) / t
            return dz, dy, dt_, dl

        def step(x, dx):
            neg = dx < 0
            return min(1.0, np.min(-x[neg] / dx[neg])) if neg.any() else 1.0

        dz, dy, dt_, dl = solve(t * lam)
        a = min(step(t, dt_), step(lam, dl))
        mu_aff = (t + a * dt_) @ (lam + a * dl) / m
        sig = (mu_aff / mu) ** 3
        dz, dy, dt_, dl = solve(t * lam + dt_ * dl - sig * mu)
        a = min(1.0, 0.995 * min(step(t, dt_), step(lam, dl)))
        z += a * dz; y += a * dy; t += a * dt_; lam += a * dl
    if best is not None:  # max_iter without meeting tol: the best iterate seen
        _, z, t, lam, it = best
    out = _unpack(q, z)
    out.update(iters=it, mu=t @ lam / m, obj=0.5 * z @ H @ z + g @ z)
    return out
