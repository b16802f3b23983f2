"""Test infrastructure (never imported by the product path): the box
geometric multigrid V-cycle of csrc/tv_mgsolve.cpp / tv_mgdist.cpp restated in
numpy on the oracle's assembled Jacobians, for tests/test_multigrid.py and
tests/vcycle_part_check.py.

    vcycle_reference(axes, T, mp, dt, levels)            one partition / GLOBAL coupling
    vcycle_reference(..., n_parts=P, part=p)             LOCAL coupling: partition p's
                                                          block of the block-Jacobi V-cycle

The hierarchy: every other node plus the last one along each axis with >= 2
cells, P = linear interpolation (kron of the per-axis maps), R = P^T, coarse
J(T) re-assembled with T injected, damped Jacobi (weight 2 / (1.1 b), b the
Gershgorin bound) before and after the coarse correction, one Jacobi step on
the coarsest level.  LOCAL coupling restricts every level to the planes
(storage axis 2) the partition owns -- level 0: part_planes(N2, P, p); a coarse
plane belongs to the owner of the fine plane it coincides with -- i.e. the
principal blocks of J and the matching blocks of P (tv_mgdist.cpp).
"""
import numpy as np
import scipy.sparse as sp

from oracle import tv_oracle as O


def axis_mats(x):
    """assembled 1D P1 mass / stiffness on nodes x (a single node: M = 1, K = 0)"""
    n = len(x)
    if n == 1:
        return sp.csr_matrix(np.ones((1, 1))), sp.csr_matrix((1, 1))
    h = np.diff(x)
    M = np.zeros((n, n))
    K = np.zeros((n, n))
    for e in range(n - 1):
        M[e:e + 2, e:e + 2] += h[e] * np.array([[1.0 / 3.0, 1.0 / 6.0], [1.0 / 6.0, 1.0 / 3.0]])
        K[e:e + 2, e:e + 2] += np.array([[1.0, -1.0], [-1.0, 1.0]]) / h[e]
    return sp.csr_matrix(M), sp.csr_matrix(K)


def kron3(z, y, x):
    return sp.kron(z, sp.kron(y, x, format="csr"), format="csr")  # node i + n0 (j + n1 k)


def omega(axes, da):
    """2 / (1.1 b), b = the Gershgorin bound of D^-1 (M + da K) (rows of the cell
    operator, floor 2.25 for the Robin facet masses, x 1.05) -- mg_gershgorin"""
    (Mx, Kx), (My, Ky), (Mz, Kz) = [axis_mats(a) for a in axes]
    A = kron3(Mz, My, Mx) + da * (kron3(Mz, My, Kx) + kron3(Mz, Ky, Mx) + kron3(Kz, My, Mx))
    b = float(np.max(np.asarray(abs(A).sum(axis=1)).ravel() / A.diagonal()))
    return 2.0 / (1.1 * (max(b, 2.25) * 1.05))


def auto_levels(axes, dt, alpha):
    """the automatic depth of mg_setup: coarsen until dt alpha / h^2 <= 0.5"""
    da, nlev, Xp = dt * alpha, 1, [np.asarray(a) for a in axes]
    while True:
        cells = [len(a) - 1 for a in Xp]
        h = min((a[-1] - a[0]) / c for a, c in zip(Xp, cells) if c >= 1)
        if not any(c >= 2 for c in cells) or da / (h * h) <= 0.5:
            return nlev
        Xp = [a[(np.arange(len(a)) % 2 == 0) | (np.arange(len(a)) == len(a) - 1)] if len(a) >= 3 else a
              for a in Xp]
        nlev += 1


def part_planes(N2, P, p):
    return (N2 * p) // P, (N2 * (p + 1)) // P


def vcycle_reference(axes, T, mp, dt, levels, n_parts=1, part=0):
    da = dt * mp["alpha"]
    prm = O.ThermalParams.from_dict(mp)
    lev = []
    Xp = [np.asarray(a, dtype=float) for a in axes]
    Tp = T
    owner = np.zeros(len(Xp[2]), dtype=np.int64)
    for q in range(n_parts):
        b0, b1 = part_planes(len(Xp[2]), n_parts, q)
        owner[b0:b1] = q
    while True:
        mesh = O.rectilinear_mesh(Xp)
        J = O.HeatForm(O.Space(mesh, "CG", 1), dt, prm).jacobian(Tp).tocsr()
        n = [len(a) for a in Xp]
        sel = np.repeat(owner == part, n[0] * n[1]) if n_parts > 1 else np.ones(J.shape[0], dtype=bool)
        lev.append({"J": J, "d": J.diagonal(), "omega": omega(Xp, da), "sel": sel})
        if len(lev) == levels:
            break
        keep, Ps = [], []
        for a in Xp:
            nf = len(a)
            k = np.ones(nf, dtype=bool)
            if nf - 1 >= 2:
                k = (np.arange(nf) % 2 == 0) | (np.arange(nf) == nf - 1)
            cpos = np.cumsum(k) - 1
            P = np.zeros((nf, int(k.sum())))
            for i in range(nf):
                if k[i]:
                    P[i, cpos[i]] = 1.0
                else:
                    wl = (a[i + 1] - a[i]) / (a[i + 1] - a[i - 1])
                    P[i, cpos[i - 1]] = wl
                    P[i, cpos[i + 1]] = 1.0 - wl
            keep.append(k)
            Ps.append(sp.csr_matrix(P))
        lev[-1]["P_to_coarse"] = kron3(Ps[2], Ps[1], Ps[0])
        Tp = Tp.reshape(n[2], n[1], n[0])[np.ix_(keep[2], keep[1], keep[0])].ravel()
        Xp = [a[k] for a, k in zip(Xp, keep)]
        owner = owner[keep[2]]
    # the partition's blocks (the whole operators on one partition)
    for l, L in enumerate(lev):
        s = L["sel"]
        L["J"] = L["J"][s][:, s]
        L["d"] = L["d"][s]
        if "P_to_coarse" in L:
            L["P_to_coarse"] = L["P_to_coarse"][s][:, lev[l + 1]["sel"]]

    def cycle(l, b):
        L = lev[l]
        x = L["omega"] * b / L["d"]  # the pre-smoothing step from 0
        if l + 1 < len(lev):
            P = L["P_to_coarse"]
            x = x + P @ cycle(l + 1, P.T @ (b - L["J"] @ x))
            x = x + L["omega"] * (b - L["J"] @ x) / L["d"]
        return x
    return lambda r: cycle(0, r)
