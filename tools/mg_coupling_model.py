"""Krylov counts of the partitioned multigrid preconditioners, modelled in
numpy (scipy sparse) on the C4 cell sizes: GLOBAL coupling (the V-cycle of the
whole box, what tv_mgdist.cpp distributes) against LOCAL coupling (block
Jacobi: each slab's own V-cycle, the principal blocks of every level) for P
slabs along y.

The operator is the cell part of the heat Jacobian, M + dt alpha K, on a
rectilinear Q1 grid (Kronecker products of the assembled 1D P1 matrices, the
Robin facets left out: < 1 % of the rows), the hierarchy and smoother those
of tests/gmg_reference.py (every other node, linear P, R = P^T, damped Jacobi
with the Gershgorin weight, one Jacobi step on the coarsest level), PCG with
rtol 1e-5 on the preconditioned norm (PETSc KSPCG defaults), right-hand side
a smooth thermal-shock-like residual (boundary layer) plus noise.

    python tools/mg_coupling_model.py [--cells 100,100,50] [--parts 1,2,4,8]
"""
import argparse
import json

import numpy as np
import scipy.sparse as sp


def axis_mats(x):
    n = len(x)
    h = np.diff(x)
    M = sp.lil_matrix((n, n))
    K = sp.lil_matrix((n, n))
    for e in range(n - 1):
        M[e:e + 2, e:e + 2] += h[e] * np.array([[1 / 3, 1 / 6], [1 / 6, 1 / 3]])
        K[e:e + 2, e:e + 2] += np.array([[1.0, -1.0], [-1.0, 1.0]]) / h[e]
    return M.tocsr(), K.tocsr()


def kron3(z, y, x):
    return sp.kron(z, sp.kron(y, x, format="csr"), format="csr")


def operator(axes, da):
    (Mx, Kx), (My, Ky), (Mz, Kz) = [axis_mats(a) for a in axes]
    return (kron3(Mz, My, Mx) + da * (kron3(Mz, My, Kx) + kron3(Mz, Ky, Mx) + kron3(Kz, My, Mx))).tocsr()


def omega(A):
    b = float(np.max(np.asarray(abs(A).sum(axis=1)).ravel() / A.diagonal()))
    return 2.0 / (1.1 * (max(b, 2.25) * 1.05))


def hierarchy(axes, da):
    """levels along the partition axis (storage axis 2 = index 2 of `axes`)"""
    lev, Xp = [], [np.asarray(a, float) for a in axes]
    while True:
        A = operator(Xp, da)
        lev.append({"A": A, "d": A.diagonal(), "om": omega(A), "n": [len(a) for a in Xp]})
        cells = [len(a) - 1 for a in Xp]
        h = min((a[-1] - a[0]) / c for a, c in zip(Xp, cells) if c >= 1)
        if da / (h * h) <= 0.5:
            return lev
        keep, Ps = [], []
        for a in Xp:
            nf = len(a)
            k = (np.arange(nf) % 2 == 0) | (np.arange(nf) == nf - 1) if nf >= 3 else np.ones(nf, bool)
            cpos = np.cumsum(k) - 1
            rows, cols, vals = [], [], []
            for i in range(nf):
                if k[i]:
                    rows.append(i); cols.append(cpos[i]); vals.append(1.0)
                else:
                    wl = (a[i + 1] - a[i]) / (a[i + 1] - a[i - 1])
                    rows += [i, i]; cols += [cpos[i - 1], cpos[i + 1]]; vals += [wl, 1 - wl]
            Ps.append(sp.csr_matrix((vals, (rows, cols)), shape=(nf, int(k.sum()))))
            keep.append(k)
        lev[-1]["P"] = kron3(Ps[2], Ps[1], Ps[0])
        lev[-1]["keep2"] = keep[2]
        Xp = [a[k] for a, k in zip(Xp, keep)]


def local_blocks(lev, P):
    """per partition: the principal blocks (owned planes of every level)"""
    n2 = lev[0]["n"][2]
    owner = np.zeros(n2, dtype=int)
    for q in range(P):
        owner[n2 * q // P:n2 * (q + 1) // P] = q
    owners = []
    for L in lev:
        owners.append(owner)
        if "keep2" in L:
            owner = owner[L["keep2"]]
    parts = []
    for q in range(P):
        blk = []
        for l, L in enumerate(lev):
            sel = np.repeat(owners[l] == q, L["n"][0] * L["n"][1])
            e = {"A": L["A"][sel][:, sel], "d": L["d"][sel], "om": L["om"], "sel": sel}
            blk.append(e)
        for l in range(len(lev) - 1):
            blk[l]["P"] = lev[l]["P"][blk[l]["sel"]][:, blk[l + 1]["sel"]]
        parts.append(blk)
    return parts


def vcycle(lev, b, l=0):
    L = lev[l]
    x = L["om"] * b / L["d"]
    if l + 1 < len(lev):
        x = x + L["P"] @ vcycle(lev, L["P"].T @ (b - L["A"] @ x), l + 1)
        x = x + L["om"] * (b - L["A"] @ x) / L["d"]
    return x


def pcg(A, b, B, rtol=1e-5, maxit=500):
    x = np.zeros_like(b)
    r = b.copy()
    z = B(r)
    p = z.copy()
    rz = r @ z
    dp0 = np.sqrt(z @ z)
    for it in range(1, maxit + 1):
        w = A @ p
        a = rz / (p @ w)
        x += a * p
        r -= a * w
        z = B(r)
        if np.sqrt(z @ z) <= rtol * dp0:
            return it
        rz2 = r @ z
        p = z + (rz2 / rz) * p
        rz = rz2
    return maxit


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", default="100,50,100", help="x, z, y cells (y = the partition axis, last)")
    ap.add_argument("--h", default="0.125,0.1,0.125", help="cell sizes along the same axes (C4: 0.125 x 0.1 x 0.125)")
    ap.add_argument("--parts", default="1,2,4,8")
    ap.add_argument("--dt-alpha", type=float, default=0.1)
    a = ap.parse_args()
    nc = [int(v) for v in a.cells.split(",")]
    hs = [float(v) for v in a.h.split(",")]
    axes = [np.arange(n + 1) * h for n, h in zip(nc, hs)]
    lev = hierarchy(axes, a.dt_alpha)
    A = lev[0]["A"]
    n0, n1, n2 = lev[0]["n"]
    rng = np.random.default_rng(3)
    X, Z, Y = np.meshgrid(axes[0], axes[1], axes[2], indexing="ij")
    # a thermal-shock-like Newton residual: the surface layer of the plate (z faces) + noise
    shock = np.exp(-np.minimum(Z, Z.max() - Z) / 0.3) + 0.3 * np.exp(-np.minimum(X, X.max() - X) / 0.3)
    b = (shock.transpose(2, 1, 0).ravel() + 0.01 * rng.standard_normal(A.shape[0])) * 1e-2
    res = {"cells": nc, "h": hs, "levels": len(lev), "nodes": A.shape[0], "its": {}}
    for P in [int(v) for v in a.parts.split(",")]:
        if P == 1:
            its = pcg(A, b, lambda r: vcycle(lev, r))
        else:
            parts = local_blocks(lev, P)

            def B(r, parts=parts):
                z = np.zeros_like(r)
                for blk in parts:
                    s = blk[0]["sel"]
                    z[s] = vcycle(blk, r[s])
                return z
            its = pcg(A, b, B)
        res["its"][P] = its
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()


def hybrid(lev, parts, k, b, l=0):
    """levels < k: the global cycle; from level k on each partition's own block cycle"""
    if l == k:
        z = np.zeros_like(b)
        for blk in parts:
            s = blk[k]["sel"]
            z[s] = vcycle(blk, b[s], k)
        return z
    L = lev[l]
    x = L["om"] * b / L["d"]
    if l + 1 < len(lev):
        x = x + L["P"] @ hybrid(lev, parts, k, L["P"].T @ (b - L["A"] @ x), l + 1)
        x = x + L["om"] * (b - L["A"] @ x) / L["d"]
    return x


def main_hybrid():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", default="100,50,100")
    ap.add_argument("--h", default="0.125,0.1,0.125")
    ap.add_argument("--parts", default="2,4,8")
    ap.add_argument("--dt-alpha", type=float, default=0.1)
    a, _ = ap.parse_known_args()
    nc = [int(v) for v in a.cells.split(",")]
    hs = [float(v) for v in a.h.split(",")]
    axes = [np.arange(n + 1) * h for n, h in zip(nc, hs)]
    lev = hierarchy(axes, a.dt_alpha)
    A = lev[0]["A"]
    rng = np.random.default_rng(3)
    X, Z, Y = np.meshgrid(axes[0], axes[1], axes[2], indexing="ij")
    shock = np.exp(-np.minimum(Z, Z.max() - Z) / 0.3) + 0.3 * np.exp(-np.minimum(X, X.max() - X) / 0.3)
    b = (shock.transpose(2, 1, 0).ravel() + 0.01 * rng.standard_normal(A.shape[0])) * 1e-2
    for P in [int(v) for v in a.parts.split(",")]:
        parts = local_blocks(lev, P)
        out = {k: pcg(A, b, lambda r, k=k: hybrid(lev, parts, k, r)) for k in range(len(lev))}
        print(json.dumps({"P": P, "levels": len(lev), "its_local_from_level": out}), flush=True)


def hybrid_loc(lev, parts, k, b, l=0):
    """levels < k global; the transfer into level k and everything below it per
    partition (owned fine planes -> owned coarse planes: R = P^T of the blocks)"""
    L = lev[l]
    x = L["om"] * b / L["d"]
    if l + 1 < len(lev):
        if l + 1 == k:
            d = b - L["A"] @ x
            c = np.zeros_like(x)
            for blk in parts:
                s = blk[l]["sel"]
                Pl = blk[l]["P"]
                c[s] = Pl @ vcycle(blk, Pl.T @ d[s], l + 1)
            x = x + c
        else:
            x = x + L["P"] @ hybrid_loc(lev, parts, k, L["P"].T @ (b - L["A"] @ x), l + 1)
        x = x + L["om"] * (b - L["A"] @ x) / L["d"]
    return x


def main_hybrid_loc():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", default="100,50,100")
    ap.add_argument("--h", default="0.125,0.1,0.125")
    ap.add_argument("--parts", default="2,4,8")
    ap.add_argument("--dt-alpha", type=float, default=0.1)
    a, _ = ap.parse_known_args()
    nc = [int(v) for v in a.cells.split(",")]
    hs = [float(v) for v in a.h.split(",")]
    axes = [np.arange(n + 1) * h for n, h in zip(nc, hs)]
    lev = hierarchy(axes, a.dt_alpha)
    A = lev[0]["A"]
    rng = np.random.default_rng(3)
    X, Z, Y = np.meshgrid(axes[0], axes[1], axes[2], indexing="ij")
    shock = np.exp(-np.minimum(Z, Z.max() - Z) / 0.3) + 0.3 * np.exp(-np.minimum(X, X.max() - X) / 0.3)
    b = (shock.transpose(2, 1, 0).ravel() + 0.01 * rng.standard_normal(A.shape[0])) * 1e-2
    for P in [int(v) for v in a.parts.split(",")]:
        parts = local_blocks(lev, P)
        out = {k: pcg(A, b, lambda r, k=k: hybrid_loc(lev, parts, k, r)) for k in range(1, len(lev))}
        print(json.dumps({"P": P, "levels": len(lev), "its_local_transfer_into_level": out}), flush=True)
