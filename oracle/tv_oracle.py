"""CPU ORACLE — test infrastructure only.

This module is a plain numpy/scipy restatement of the reference algorithm of
pzimbrod/fem-glass-tempering (``/root/reference``, snapshot 2025-01-14).  It is
the *checker* for the HIP path and nothing else: only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import it.  The product path (``fem-glass-tempering_amd/``) never imports it and
fails loudly when its HIP library is missing.

What it restates (file:line of the reference):

* ``ThermoViscoProblem._setup_weak_form``  (ThermoViscoProblem.py:280-327) —
  residual ``F`` incl. the SIPG branch for DG temperature, assembled generically
  cell-by-cell / facet-by-facet with isoparametric Q1/P1 geometry and Gauss
  quadrature (no tensor-product shortcuts, unlike the HIP path).
* ``NonlinearProblem.J = ufl.derivative(F)`` (ThermoViscoProblem.py:331) —
  assembled CSR Jacobian (hand-derived derivative of ``F``).
* dolfinx ``NewtonSolver`` with ``convergence_criterion="incremental"``,
  ``rtol=1e-12`` (ThermoViscoProblem.py:334-337) and the dolfinx-0.7.3 defaults
  ``atol=1e-10``, ``max_it=50``; iteration 1 only records ``||dx_1||``.
* the time loop and the exact per-step call order incl. every
  ``_update_values`` copy (ThermoViscoProblem.py:367-381, 393-595, 598-611).
* the 17 viscoelastic expressions (ViscoelasticModel.py:86-242) evaluated with
  dolfinx ``fem::interpolate`` semantics (per cell, at the target element's
  interpolation points = cell vertices for degree 1, last cell written wins).
* the Prony tableaux and constants (ViscoelasticModel.py:15-83,
  ThermalModel.py:18-27).

Parity status: **parity against dolfinx outputs is unpinned** — dolfinx / UFL /
FFCx / PETSc are not installable offline and the reference ships no tests,
fixtures or recorded outputs.  This oracle is pinned
instead by analytic known-answer tests (tests/test_oracle_kat.py: 50-digit
mpmath pointwise update, exact energy balance, uniform state, Jacobian vs
finite differences, MMS O(h^2) convergence, SIPG symmetry/SPD).
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

# ---------------------------------------------------------------------------
# Constants of the reference (ViscoelasticModel.py:19-68, main.py:29-55)
# ---------------------------------------------------------------------------
PRONY = {
    "m_n": [5.523e-2, 8.205e-2, 1.215e-1, 2.286e-1, 2.860e-1, 2.265e-1],
    "lambda_m": [5.965e-4, 1.077e-2, 1.362e-1, 1.505e-1, 6.747e+0, 2.963e+1],
    "g_n": [1.585, 2.354, 3.486, 6.558, 8.205, 6.498],
    "lambda_g": [6.658e-5, 1.197e-3, 1.514e-2, 1.672e-1, 7.497e-1, 3.292e+0],
    "k_n": [7.588e-1, 7.650e-1, 9.806e-1, 7.301e+0, 1.347e+1, 1.090e+1],
    "lambda_k": [5.009e-5, 9.945e-4, 2.022e-3, 1.925e-2, 1.199e-1, 2.033e+0],
}
TABLEAU_SIZE = 6

MAIN_MODEL_PARAMS = {
    "f": 0.0, "epsilon": 0.93, "sigma": 5.670e-8, "T_ambient": 600.0, "T_0": 800.0,
    "alpha": 1.0, "htc": 280.1, "rho": 2500.0, "cp": 1433.0, "k": 1.0,
    "H": 627.8e3, "Tb": 869.0e0, "Rg": 8.314, "alpha_solid": 9.10e-6,
    "alpha_liquid": 25.10e-6, "Tf_init": 873.0,
}


# ---------------------------------------------------------------------------
# Mesh: rectilinear grids expressed as a generic cell/vertex mesh
# ---------------------------------------------------------------------------
@dataclass
class Mesh:
    """Generic mesh: vertex coordinates + cell->vertex connectivity.

    Cells are intervals (d=1), quadrilaterals (d=2) or hexahedra (d=3) with the
    tensor-product local vertex order ``l = a + 2 b + 4 c`` (basix/dolfinx order
    for quadrilaterals and hexahedra).
    """
    dim: int
    x: np.ndarray          # (n_vertices, dim)
    cells: np.ndarray      # (n_cells, 2**dim) int64

    @property
    def n_vertices(self):
        return self.x.shape[0]

    @property
    def n_cells(self):
        return self.cells.shape[0]


def rectilinear_mesh(axes):
    """Rectilinear grid from per-axis node coordinates (1 to 3 axes).

    Vertex index = i + n0*(j + n1*k) (x fastest); cell index likewise.
    """
    axes = [np.asarray(a, dtype=np.float64) for a in axes]
    d = len(axes)
    n = [len(a) for a in axes]
    grids = np.meshgrid(*axes, indexing="ij")
    # flatten with x fastest
    x = np.stack([g.transpose(list(range(d))[::-1]).ravel() for g in grids], axis=1)
    nc = [m - 1 for m in n]
    cell_ijk = np.stack(np.meshgrid(*[np.arange(m) for m in nc], indexing="ij"), axis=-1)
    cell_ijk = cell_ijk.transpose(list(range(d))[::-1] + [d]).reshape(-1, d)
    strides = [1]
    for m in n[:-1]:
        strides.append(strides[-1] * m)
    cells = np.zeros((cell_ijk.shape[0], 2 ** d), dtype=np.int64)
    for l in range(2 ** d):
        off = np.zeros(cell_ijk.shape[0], dtype=np.int64)
        for a in range(d):
            bit = (l >> a) & 1
            off += (cell_ijk[:, a] + bit) * strides[a]
        cells[:, l] = off
    return Mesh(dim=d, x=x, cells=cells)


def box_mesh(lengths, ncells):
    return rectilinear_mesh([np.linspace(0.0, L, n + 1) for L, n in zip(lengths, ncells)])


# ---------------------------------------------------------------------------
# Reference element (degree-1 Lagrange, tensor product) and quadrature
# ---------------------------------------------------------------------------
def gauss01(n):
    p, w = np.polynomial.legendre.leggauss(n)
    return 0.5 * (p + 1.0), 0.5 * w


def tensor_rule(d, n):
    p1, w1 = gauss01(n)
    if d == 0:
        return np.zeros((1, 0)), np.ones(1)
    grids = np.meshgrid(*([p1] * d), indexing="ij")
    wgrids = np.meshgrid(*([w1] * d), indexing="ij")
    pts = np.stack([g.ravel() for g in grids], axis=1)
    w = np.prod(np.stack([g.ravel() for g in wgrids], axis=1), axis=1)
    return pts, w


def q1_basis(xi):
    """Values (nq, nl) and reference gradients (nq, nl, d) of Q1/P1 at xi (nq, d)."""
    nq, d = xi.shape
    nl = 2 ** d
    phi = np.ones((nq, nl))
    dphi = np.ones((nq, nl, d))
    for l in range(nl):
        for a in range(d):
            bit = (l >> a) & 1
            fa = xi[:, a] if bit else 1.0 - xi[:, a]
            dfa = 1.0 if bit else -1.0
            phi[:, l] *= fa
            for b in range(d):
                if b == a:
                    dphi[:, l, b] *= dfa
                else:
                    dphi[:, l, b] *= fa
    return phi, dphi


def cell_diameter(mesh):
    """ufl.CellDiameter: max distance between any two vertices of the cell."""
    X = mesh.x[mesh.cells]  # (nc, nl, d)
    diff = X[:, :, None, :] - X[:, None, :, :]
    return np.sqrt((diff ** 2).sum(-1)).max(axis=(1, 2))


# ---------------------------------------------------------------------------
# Function spaces (degree 1, CG or DG), dof maps
# ---------------------------------------------------------------------------
class Space:
    """Degree-1 Lagrange space on ``mesh``: CG dof = vertex, DG dof = cell*nl + l."""

    def __init__(self, mesh: Mesh, family: str, degree: int = 1):
        assert family in ("CG", "DG"), "Only CG and DG elements are supported"
        if degree != 1:
            raise NotImplementedError("oracle restates degree-1 Lagrange only")
        self.mesh = mesh
        self.family = family
        nl = 2 ** mesh.dim
        if family == "CG":
            self.dofmap = mesh.cells.copy()
            self.n = mesh.n_vertices
        else:
            self.dofmap = np.arange(mesh.n_cells * nl, dtype=np.int64).reshape(mesh.n_cells, nl)
            self.n = mesh.n_cells * nl

    def dof_coordinates(self):
        X = np.zeros((self.n, self.mesh.dim))
        X[self.dofmap.ravel()] = self.mesh.x[self.mesh.cells].reshape(-1, self.mesh.dim)
        return X


# ---------------------------------------------------------------------------
# Facets
# ---------------------------------------------------------------------------
def _local_facets(d):
    """Local facets of the tensor cell: list of (axis, side, local vertex ids sorted)."""
    out = []
    for a in range(d):
        for s in (0, 1):
            lv = [l for l in range(2 ** d) if ((l >> a) & 1) == s]
            out.append((a, s, lv))
    return out


def facet_topology(mesh, plus_side="lower"):
    """Exterior facets [(cell, lf)] and interior facet pairs [(c+, lf+, c-, lf-)].

    '+' is the lower cell index of the pair by default (``plus_side="higher"``
    flips it).  dolfinx orders the two cells of an interior facet by its
    facet->cell connectivity after its own cell reordering [3P, unpinned]: on a
    uniform mesh the choice does not change the form, on a graded one it moves
    h('+') in the SIPG penalty p/h('+') (ThermoViscoProblem.py:313-325), which
    tests/test_oracle_kat.py::test_sipg_plus_side_sensitivity measures.
    """
    d = mesh.dim
    lfs = _local_facets(d)
    keys = []
    owners = []
    for lf, (a, s, lv) in enumerate(lfs):
        vids = np.sort(mesh.cells[:, lv], axis=1)
        keys.append(vids)
        owners.append(np.stack([np.arange(mesh.n_cells), np.full(mesh.n_cells, lf)], axis=1))
    keys = np.concatenate(keys, axis=0)
    owners = np.concatenate(owners, axis=0)
    nk = keys.shape[1]
    if mesh.n_vertices < (1 << 21):
        # a facet is identified by its lowest min(nk, 3) sorted vertex ids (three
        # corners of a conforming quad facet belong to no other facet): one int64
        # key per facet, in the same lexicographic order as the rows
        packed = np.zeros(len(keys), dtype=np.int64)
        for q in range(min(nk, 3)):
            packed = (packed << 21) | keys[:, q].astype(np.int64)
        _, inv, counts = np.unique(packed, return_inverse=True, return_counts=True)
    else:
        _, inv, counts = np.unique(keys, axis=0, return_inverse=True, return_counts=True)
    inv = inv.ravel()
    ext_mask = counts[inv] == 1
    exterior = owners[ext_mask]
    exterior = exterior[np.lexsort((exterior[:, 1], exterior[:, 0]))]
    order = np.argsort(inv, kind="stable")
    inv_sorted = inv[order]
    idx = np.nonzero(counts[inv_sorted] == 2)[0]
    # consecutive pairs of the sorted shared facets: (owner 0, owner 1), '+' first
    o0 = owners[order[idx[0::2]]]
    o1 = owners[order[idx[1::2]]]
    swap = (o0[:, 0] > o1[:, 0]) == (plus_side == "lower")
    p_, m_ = np.where(swap[:, None], o1, o0), np.where(swap[:, None], o0, o1)
    interior = np.concatenate([p_, m_], axis=1).astype(np.int64).reshape(-1, 4)
    return exterior, interior


def _facet_ref_points(d, lf, q):
    """Map facet reference points q (nq, d-1) to cell reference coords for facet lf."""
    a, s, _ = _local_facets(d)[lf]
    tang = [b for b in range(d) if b != a]
    xi = np.zeros((q.shape[0], d))
    xi[:, a] = float(s)
    for k, b in enumerate(tang):
        xi[:, b] = q[:, k]
    return xi


kBigMeshCells = 200_000  # meshes from this size on: the BLAS-backed forms of the cell set-up


def _geometry(Xc, dphi):
    """Jacobian (nc, nq, d, d) of the isoparametric map: J[ab] = dx_a/dxi_b
    (= einsum("cla,qlb->cqab", Xc, dphi); as one matrix product on big meshes)."""
    if len(Xc) < kBigMeshCells:
        return np.einsum("cla,qlb->cqab", Xc, dphi)
    nc, nl, d = Xc.shape
    nq = dphi.shape[0]
    # (nc*d, nl) @ (nl, nq*d) -> [c, a, q, b]
    J = Xc.transpose(0, 2, 1).reshape(nc * d, nl) @ dphi.transpose(1, 0, 2).reshape(nl, nq * d)
    return J.reshape(nc, d, nq, d).transpose(0, 2, 1, 3)


def _facet_measure_and_normal(J, axis, side):
    """Surface Jacobian and outward unit normal at facet points.

    J: (n, nq, d, d).  Facet = {xi_axis = side}.  Normal = J^{-T} e_axis
    normalised, oriented outward; measure = |det J| * |J^{-T} e_axis|.
    """
    d = J.shape[-1]
    if d == 1:
        n = np.full(J.shape[:2] + (1,), 1.0 if side == 1 else -1.0)
        return np.ones(J.shape[:2]), n
    Jinv = np.linalg.inv(J)
    g = Jinv[..., axis, :]  # row axis of J^{-1} = grad xi_axis
    gn = np.linalg.norm(g, axis=-1)
    detJ = np.abs(np.linalg.det(J))
    n = g / gn[..., None] * (1.0 if side == 1 else -1.0)
    return detJ * gn, n


# ---------------------------------------------------------------------------
# Thermal model: residual and Jacobian (ThermoViscoProblem.py:280-327)
# ---------------------------------------------------------------------------
@dataclass
class ThermalParams:
    f: float
    epsilon: float
    sigma: float
    alpha: float
    htc: float
    T_ambient: float

    @classmethod
    def from_dict(cls, p):
        return cls(f=p["f"], epsilon=p["epsilon"], sigma=p["sigma"], alpha=p["alpha"],
                   htc=p["htc"], T_ambient=p["T_ambient"])


class HeatForm:
    """Residual F(T) and Jacobian J(T) of the reference's heat weak form.

    F = (T - T_prev) v dx + dt*( alpha grad T.grad v dx - f v dx
          + 0.001 sigma eps (T^4 - Ta^4) v ds + 0.001 htc (T - Ta) v ds )
        [+ dt*alpha('+')*( p/h('+') jump(v,n).jump(T,n) - avg(grad v).jump(T,n)
                           - jump(v,n).avg(grad T) ) dS   if T is DG]
    (ThermoViscoProblem.py:293-325)
    """

    def __init__(self, space: Space, dt: float, params: ThermalParams, qdeg_cell=3, qdeg_facet=3,
                 penalty=5.0, plus_side="lower"):
        self.V = space
        self.mesh = space.mesh
        self.dt = dt
        self.p = params
        self.penalty = penalty
        d = self.mesh.dim
        self.d = d
        # cell quadrature
        xq, wq = tensor_rule(d, qdeg_cell)
        phi, dphi = q1_basis(xq)
        Xc = self.mesh.x[self.mesh.cells]
        # congruent cells (a uniform box): the cell geometry is that of cell 0
        # everywhere, so it is computed once and broadcast (the same element
        # matrices up to the rounding of the coordinate differences, ~1e-15)
        # (large meshes only: the einsum statements below stay the reference
        # arithmetic of every small test mesh, whose CG iteration counts on long
        # 1D bars move with the last bit of the element matrices)
        big = len(Xc) >= kBigMeshCells
        self.congruent = False
        if big:
            rel = Xc - Xc[:, :1, :]
            scale = np.abs(rel[0]).max()
            self.congruent = bool(np.abs(rel - rel[:1]).max() <= 1e-13 * scale)
            del rel
        nc_all = len(Xc)
        if self.congruent:
            Xc = Xc[:1]
        J = _geometry(Xc, dphi)
        detJ = np.linalg.det(J)
        Jinv = np.linalg.inv(J)
        # physical gradients (nc, nq, nl, d): grad phi = J^{-T} dphi
        # (the contractions below as batched matrix products -- the same sums as
        # the einsum statements in the comments, BLAS-backed so the oracle sets up
        # a 1M-cell plate in seconds instead of minutes)
        self.cw = wq[None, :] * np.abs(detJ)                   # (nc, nq)
        self.cphi = phi                                         # (nq, nl)
        if not big:
            gphi = np.einsum("cqba,qlb->cqla", Jinv, dphi)
            self.cgphi = gphi                                   # (nc, nq, nl, d)
            # local mass and stiffness matrices
            self.Me = np.einsum("cq,qi,qj->cij", self.cw, phi, phi)
            self.Ke = np.einsum("cq,cqia,cqja->cij", self.cw, gphi, gphi)
            self.be = np.einsum("cq,qi->ci", self.cw, phi)     # int phi_i
        else:
            gphi = np.matmul(dphi[None], Jinv)                  # einsum("cqba,qlb->cqla", Jinv, dphi)
            self.cgphi = gphi
            nc_, nq_, nl_ = gphi.shape[0], gphi.shape[1], gphi.shape[2]
            #   Me = einsum("cq,qi,qj->cij", cw, phi, phi)
            self.Me = (self.cw @ (phi[:, :, None] * phi[:, None, :]).reshape(nq_, nl_ * nl_)).reshape(nc_, nl_, nl_)
            #   Ke = einsum("cq,cqia,cqja->cij", cw, gphi, gphi)
            G = (gphi * np.sqrt(self.cw)[:, :, None, None]).transpose(0, 2, 1, 3).reshape(nc_, nl_, nq_ * d)
            self.Ke = np.matmul(G, G.transpose(0, 2, 1))
            del G
            self.be = self.cw @ phi                             # einsum("cq,qi->ci", cw, phi): int phi_i
        if self.congruent:
            bc = lambda a: np.broadcast_to(a, (nc_all,) + a.shape[1:])  # noqa: E731
            self.cw, self.cgphi, self.Me, self.Ke, self.be = (bc(self.cw), bc(self.cgphi), bc(self.Me), bc(self.Ke),
                                                              bc(self.be))
        # exterior facets
        ext, inter = facet_topology(self.mesh, plus_side)
        self.ext = ext
        self.inter = inter
        self._prep_exterior(qdeg_facet)
        if space.family == "DG":
            self._prep_interior(max(qdeg_facet, 2))

    # -- exterior facets ----------------------------------------------------
    def _prep_exterior(self, nqf):
        d = self.d
        qf, wf = tensor_rule(d - 1, nqf)
        self.ef_cells = self.ext[:, 0]
        self.ef_phi = []
        self.ef_w = []
        nef = len(self.ext)
        nl = 2 ** d
        phis = np.zeros((nef, len(wf), nl))
        ws = np.zeros((nef, len(wf)))
        for lf in range(2 * d):
            sel = np.nonzero(self.ext[:, 1] == lf)[0]
            if len(sel) == 0:
                continue
            a, s, _ = _local_facets(d)[lf]
            xi = _facet_ref_points(d, lf, qf)
            phi, dphi = q1_basis(xi)
            Xc = self.mesh.x[self.mesh.cells[self.ext[sel[:1] if self.congruent else sel, 0]]]
            J = _geometry(Xc, dphi)
            meas, _ = _facet_measure_and_normal(J, a, s)
            phis[sel] = phi[None]
            ws[sel] = wf[None, :] * meas
        self.ef_phi = phis   # (nef, nqf, nl)
        self.ef_w = ws       # (nef, nqf)

    # -- interior facets (SIPG) ---------------------------------------------
    def _prep_interior(self, nqf):
        d = self.d
        mesh = self.mesh
        qf, wf = tensor_rule(d - 1, nqf)
        nif = len(self.inter)
        nl = 2 ** d
        nq = len(wf)
        self.if_phi = np.zeros((nif, 2, nq, nl))
        self.if_gphi = np.zeros((nif, 2, nq, nl, d))
        self.if_w = np.zeros((nif, nq))
        self.if_n = np.zeros((nif, nq, d))   # normal of '+' (outward from '+')
        hdiam = cell_diameter(mesh)
        self.if_h = hdiam[self.inter[:, 0]]  # h('+')
        lfs = _local_facets(d)
        for k, (cp, lfp, cm, lfm) in enumerate(self.inter):
            # '+' side points
            ap, sp_, lvp = lfs[lfp]
            xip = _facet_ref_points(d, lfp, qf)
            phip, dphip = q1_basis(xip)
            Xp = mesh.x[mesh.cells[cp]][None]
            Jp = _geometry(Xp, dphip)
            meas, nrm = _facet_measure_and_normal(Jp, ap, sp_)
            xphys = np.einsum("ql,la->qa", phip, mesh.x[mesh.cells[cp]])
            # '-' side: find reference coordinates of the same physical points
            xim = self._inverse_map(cm, xphys, lfm)
            phim, dphim = q1_basis(xim)
            Xm = mesh.x[mesh.cells[cm]][None]
            Jm = _geometry(Xm, dphim)
            gp = np.einsum("qba,qlb->qla", np.linalg.inv(Jp[0]), dphip)
            gm = np.einsum("qba,qlb->qla", np.linalg.inv(Jm[0]), dphim)
            self.if_phi[k, 0] = phip
            self.if_phi[k, 1] = phim
            self.if_gphi[k, 0] = gp
            self.if_gphi[k, 1] = gm
            self.if_w[k] = wf * meas[0]
            self.if_n[k] = nrm[0]

    def _inverse_map(self, c, xphys, lf):
        """Reference coords of physical points on facet lf of cell c (Newton on the Q1 map)."""
        d = self.d
        Xc = self.mesh.x[self.mesh.cells[c]]
        a, s, _ = _local_facets(d)[lf]
        xi = np.full((xphys.shape[0], d), 0.5)
        xi[:, a] = s
        for _ in range(30):
            phi, dphi = q1_basis(xi)
            r = np.einsum("ql,la->qa", phi, Xc) - xphys
            J = np.einsum("la,qlb->qab", Xc, dphi)
            dxi = np.linalg.solve(J, r[..., None])[..., 0]
            xi = xi - dxi
            if np.abs(dxi).max() < 1e-15:
                break
        xi[:, a] = s
        return xi

    # -- assembly -----------------------------------------------------------
    def _g(self, T):
        p = self.p
        return 0.001 * (p.sigma * p.epsilon) * (T ** 4 - p.T_ambient ** 4) + 0.001 * p.htc * (T - p.T_ambient)

    def _dg(self, T):
        p = self.p
        return 0.001 * (p.sigma * p.epsilon) * 4.0 * T ** 3 + 0.001 * p.htc

    def residual(self, T, T_prev):
        V = self.V
        dm = V.dofmap
        dt, p = self.dt, self.p
        Te = T[dm]
        Tpe = T_prev[dm]
        Fe = np.einsum("cij,cj->ci", self.Me, Te - Tpe)
        Fe += dt * (p.alpha * np.einsum("cij,cj->ci", self.Ke, Te) - p.f * self.be)
        F = np.zeros(V.n)
        np.add.at(F, dm, Fe)
        # exterior facets
        if len(self.ext):
            cells = self.ext[:, 0]
            Tq = np.einsum("fql,fl->fq", self.ef_phi, T[dm[cells]])
            Ff = dt * np.einsum("fq,fq,fql->fl", self.ef_w, self._g(Tq), self.ef_phi)
            np.add.at(F, dm[cells], Ff)
        if V.family == "DG" and len(self.inter):
            F += self._sipg_matrix() @ T
        return F

    def jacobian(self, T):
        V = self.V
        dm = V.dofmap
        dt, p = self.dt, self.p
        Ae = self.Me + dt * p.alpha * self.Ke
        rows = np.repeat(dm, dm.shape[1], axis=1).ravel()
        cols = np.tile(dm, (1, dm.shape[1])).ravel()
        vals = Ae.ravel()
        R, C, Vv = [rows], [cols], [vals]
        if len(self.ext):
            cells = self.ext[:, 0]
            Tq = np.einsum("fql,fl->fq", self.ef_phi, T[dm[cells]])
            Af = dt * np.einsum("fq,fq,fqi,fqj->fij", self.ef_w, self._dg(Tq), self.ef_phi, self.ef_phi)
            dmf = dm[cells]
            R.append(np.repeat(dmf, dmf.shape[1], axis=1).ravel())
            C.append(np.tile(dmf, (1, dmf.shape[1])).ravel())
            Vv.append(Af.ravel())
        A = sp.coo_matrix((np.concatenate(Vv), (np.concatenate(R), np.concatenate(C))),
                          shape=(V.n, V.n)).tocsr()
        if V.family == "DG" and len(self.inter):
            A = A + self._sipg_matrix()
        return A.tocsr()

    def _sipg_matrix(self):
        if getattr(self, "_sipg", None) is not None:
            return self._sipg
        V = self.V
        dm = V.dofmap
        dt, p = self.dt, self.p
        nif = len(self.inter)
        nl = 2 ** self.d
        # basis traces on the facet for the 2*nl dofs of the pair: jumps and averages
        # jump(w, n) = (w+ - w-) n+ ; avg(grad w) = (grad w+ + grad w-)/2
        phi = self.if_phi          # (nif, 2, nq, nl)
        gphi = self.if_gphi        # (nif, 2, nq, nl, d)
        n = self.if_n              # (nif, nq, d)
        w = self.if_w              # (nif, nq)
        sgn = np.array([1.0, -1.0])
        jmp = np.einsum("s,fsql,fqa->fsqla", sgn, phi, n)     # jump(phi, n) vector
        avg = 0.5 * gphi                                      # avg(grad phi)
        jmp = jmp.reshape(nif, 2, -1, nl, self.d).transpose(0, 2, 1, 3, 4).reshape(nif, -1, 2 * nl, self.d)
        avg = avg.transpose(0, 2, 1, 3, 4).reshape(nif, -1, 2 * nl, self.d)
        pen = (self.penalty / self.if_h)[:, None]
        # A[i,j] = p/h jump(phi_i).jump(phi_j) - avg(grad phi_i).jump(phi_j) - jump(phi_i).avg(grad phi_j)
        A = (np.einsum("fq,fq,fqia,fqja->fij", w, pen * np.ones_like(w), jmp, jmp)
             - np.einsum("fq,fqia,fqja->fij", w, avg, jmp)
             - np.einsum("fq,fqia,fqja->fij", w, jmp, avg))
        A *= dt * p.alpha
        dofs = np.concatenate([dm[self.inter[:, 0]], dm[self.inter[:, 2]]], axis=1)  # (nif, 2nl)
        rows = np.repeat(dofs, dofs.shape[1], axis=1).ravel()
        cols = np.tile(dofs, (1, dofs.shape[1])).ravel()
        self._sipg = sp.coo_matrix((A.ravel(), (rows, cols)), shape=(V.n, V.n)).tocsr()
        return self._sipg


# ---------------------------------------------------------------------------
# Newton (dolfinx 0.7.3 NewtonSolver, incremental criterion)
# ---------------------------------------------------------------------------
class NewtonNotConverged(RuntimeError):
    pass


def pcg_jacobi(A, b, rtol=1e-5, atol=1e-50, dtol=1e5, max_it=10000):
    """PETSc KSPCG + PCJACOBI restated (preconditioned norm, zero initial guess)."""
    dinv = 1.0 / A.diagonal()
    x = np.zeros_like(b)
    r = b.copy()
    z = dinv * r
    dp = np.linalg.norm(z)
    rnorm0 = dp
    ttol = max(rtol * rnorm0, atol)
    if dp <= ttol:
        return x, 0
    beta = z @ r
    p = None
    betaold = beta
    i = 0
    while i < max_it:
        if beta == 0.0:
            return x, i
        if i == 0:
            p = z.copy()
        else:
            p = z + (beta / betaold) * p
        w = A @ p
        dpi = p @ w
        betaold = beta
        if dpi <= 0.0:
            raise RuntimeError("KSP diverged: indefinite matrix")
        a = beta / dpi
        x += a * p
        r -= a * w
        z = dinv * r
        dp = np.linalg.norm(z)
        if dp <= ttol:
            return x, i + 1
        if dp >= dtol * rnorm0 or not np.isfinite(dp):
            raise RuntimeError("KSP diverged")
        beta = z @ r
        i += 1
    raise RuntimeError("KSP did not converge (max_it)")


def _apply_dirichlet(A, b, T, bc):
    """dolfinx NonlinearProblem with bcs [3P]: J gets identity rows / columns
    at the constrained dofs, b is lifted (apply_lifting(b, [J], [bcs], x0=[x],
    scale=-1)) and set (set_bc(b, bcs, x, -1)): b_i -= J_iB (x_B - g) on free
    rows, b_B = x_B - g, so the Newton step x <- x - dx lands on g."""
    dofs, g = bc
    d = np.zeros(A.shape[0])
    d[dofs] = T[dofs] - g
    b = b - A @ d
    b[dofs] = T[dofs] - g
    keep = np.ones(A.shape[0])
    keep[dofs] = 0.0
    K = sp.diags(keep)
    A = (K @ A @ K + sp.diags(1.0 - keep)).tocsr()
    return A, b


def newton_solve(T, F_fn, J_fn, rtol=1e-12, atol=1e-10, max_it=50, linear="direct", bc=None,
                 error_on_nonconvergence=True, ksp=None):
    """Returns (n_iterations, converged, krylov_its); updates T in place.
    ``bc`` = (dofs, value): Dirichlet constraint applied as dolfinx does;
    ``ksp`` = keyword tolerances of pcg_jacobi (KSPSetTolerances)."""
    b = F_fn(T)
    it = 0
    kits = 0
    converged = False
    r0 = 0.0
    while not converged and it < max_it:
        A = J_fn(T)
        if bc is not None:
            A, b = _apply_dirichlet(A, b, T, bc)
        if linear == "direct":
            dx = spla.spsolve(A.tocsc(), b)
        else:
            dx, k = pcg_jacobi(A, b, **(ksp or {}))
            kits += k
        T -= dx           # x <- x - relaxation * dx
        it += 1
        b = F_fn(T)
        if it == 1:
            r0 = np.linalg.norm(dx)
            converged = False
        else:
            r = np.linalg.norm(dx)
            rel = r / r0 if r0 != 0.0 else (np.inf if r != 0.0 else np.nan)
            converged = bool(rel < rtol or r < atol)
    if not converged and error_on_nonconvergence:
        raise NewtonNotConverged("Newton solver did not converge because maximum number of iterations reached")
    return it, converged, kits


# ---------------------------------------------------------------------------
# Viscoelastic model: the 17 expressions (ViscoelasticModel.py:86-242)
# ---------------------------------------------------------------------------
def taylor_exponential(xi, lam):
    """ViscoelasticModel._taylor_exponential (ViscoelasticModel.py:233-242):
    sum_{k=0}^{2} 1/k! * (-xi/lam)**k, summed left to right as np.sum does."""
    t0 = (1.0 / math.factorial(0)) * (-xi / lam) ** 0
    t1 = (1.0 / math.factorial(1)) * (-xi / lam) ** 1
    t2 = (1.0 / math.factorial(2)) * (-xi / lam) ** 2
    return (t0 + t1) + t2


class ViscoParams:
    def __init__(self, mp):
        self.T_init = float(mp["T_0"])
        self.H = float(mp["H"])
        self.Rg = float(mp["Rg"])
        self.Tb = float(mp["Tb"])
        self.alpha_solid = float(mp["alpha_solid"])
        self.alpha_liquid = float(mp["alpha_liquid"])
        self.chi = 0.5
        self.m_n = np.array(PRONY["m_n"])
        self.lambda_m = np.array(PRONY["lambda_m"])
        self.g_n = np.array(PRONY["g_n"])
        self.lambda_g = np.array(PRONY["lambda_g"])
        self.k_n = np.array(PRONY["k_n"])
        self.lambda_k = np.array(PRONY["lambda_k"])


def shift_function(T, vp: ViscoParams):
    """Eq. 5 (ViscoelasticModel.py:156-161): exp(H/Rg * (1/Tb - 1/T))."""
    return np.exp(vp.H / vp.Rg * (1.0 / vp.Tb - 1.0 / T))


# ---------------------------------------------------------------------------
# Oracle problem driver (ThermoViscoProblem restated)
# ---------------------------------------------------------------------------
class OracleProblem:
    """Restatement of ThermoViscoProblem on the CPU (setup/solve_timestep/solve).

    Fields live in the reference's interleaved blocked layout
    (``x.array[dof*bs + comp]``), in dicts named like the reference's
    ``functions``, ``functions_current``, ``functions_previous``, ``functions_next``
    (ThermoViscoProblem.py:112-171).
    """

    def __init__(self, mesh: Mesh, time, dt, config, model_parameters, linear="direct", plus_side="lower",
                 model_mode="reference"):
        assert all(v["element"] in ("CG", "DG") for v in config.values()), \
            "Only CG and DG elements are supported"
        self.mesh = mesh
        self.dim = mesh.dim
        self.dt = dt
        self.time = time
        self.t = time[0]
        self.n_steps = math.ceil((time[1] - time[0]) / dt)
        self.mp = dict(model_parameters)
        self.vp = ViscoParams(model_parameters)
        self.tp = ThermalParams.from_dict(model_parameters)
        self.linear = linear
        assert model_mode in ("reference", "paper")
        self.model_mode = model_mode
        self.bc = None
        self.VT = Space(mesh, config["T"]["element"], config["T"]["degree"])
        self.VS = Space(mesh, config["sigma"]["element"], config["sigma"]["degree"])
        self.form = HeatForm(self.VT, dt, self.tp, plus_side=plus_side)
        d = self.dim
        nT, nS = self.VT.n, self.VS.n
        z = np.zeros
        self.functions_previous = {"T": z(nT), "Tf_partial": z(nT * 6), "Tf": z(nT)}
        self.functions_current = {
            "T": z(nT), "Tf_partial": z(nT * 6), "Tf": z(nT),
            "s_tilde_partial": z(nS * 6 * d * d), "sigma_tilde_partial": z(nS * 6 * d * d),
            "s_partial": z(nS * 6 * d * d), "sigma_partial": z(nS * 6 * d * d),
        }
        self.functions_next = {
            "T": z(nT), "phi": z(nT),
            "s_tilde_partial": z(nS * 6 * d * d), "sigma_tilde_partial": z(nS * 6 * d * d),
            "s_partial": z(nS * 6 * d * d), "sigma_partial": z(nS * 6 * d * d),
            "sigma": z(nS * d * d),
        }
        self.functions = {
            "phi": z(nT), "xi": z(nT),
            "thermal_strain": z(nS * d * d), "total_strain": z(nS * d * d),
            "deviatoric_strain": z(nS * d * d),
            "ds_partial": z(nS * 6 * d * d), "dsigma_partial": z(nS * 6 * d * d),
        }
        self.newton_history = []
        # problem.solver / problem.ksp settings (ThermoViscoProblem.py:334-346):
        # dolfinx NewtonSolver and PETSc KSP defaults
        self.newton = {"rtol": 1e-12, "atol": 1e-10, "max_it": 50, "error_on_nonconvergence": True}
        self.ksp = {}
        self._build_interp_maps()

    # -- fem::interpolate semantics -------------------------------------------
    def _build_interp_maps(self):
        """For target space S and source space V: per (cell, vertex) evaluation,
        writes in cell order (last cell wins).  Return, per target dof, the
        source dof of the winning (cell, vertex)."""
        self._maps = {}
        for tname, tgt in (("T", self.VT), ("S", self.VS)):
            for sname, src in (("T", self.VT), ("S", self.VS)):
                tdofs = tgt.dofmap.ravel()
                sdofs = src.dofmap.ravel()
                # last occurrence of each target dof in cell order
                rev = tdofs[::-1]
                _, first_in_rev = np.unique(rev, return_index=True)
                last_idx = len(tdofs) - 1 - first_in_rev
                m = np.empty(tgt.n, dtype=np.int64)
                m[tdofs[last_idx]] = sdofs[last_idx]
                self._maps[(tname, sname)] = m

    def _src(self, tgt, src, arr, bs=1):
        m = self._maps[(tgt, src)]
        if bs == 1:
            return arr[m]
        return arr.reshape(-1, bs)[m]

    # -- setup --------------------------------------------------------------
    def setup(self, dirichlet_bc=False):
        if dirichlet_bc:
            # the reference's own path cannot run (ThermoViscoProblem.py:236-243:
            # material_model.T_ambient and self.fs do not exist, and the bc never
            # reaches NonlinearProblem at :331); paper mode runs what it intends:
            # T = T_ambient on every dof of the exterior boundary.  For DG the
            # dofs belong to cells, not facets, so locate_dofs_topological finds
            # none [3P] and the constraint is empty.
            if self.model_mode != "paper":
                raise AttributeError("'ViscoelasticModel' object has no attribute 'T_ambient' "
                                     "(Dirichlet path of the reference is broken)")
            if self.VT.family == "CG":
                dofs = np.unique(self.VT.dofmap[self.form.ext[:, 0]][
                    np.array([[((l >> (lf // 2)) & 1) == (lf % 2) for l in range(2 ** self.dim)]
                              for lf in self.form.ext[:, 1]])])
                self.bc = (dofs, float(self.tp.T_ambient))
        T0 = self.vp.T_init
        self.functions_previous["T"][:] = T0
        self.functions_current["T"][:] = T0
        self.functions_previous["Tf"][:] = self.functions_previous["T"]
        self.functions_current["Tf"][:] = self.functions_current["T"]
        tv = self.functions_current["T"][0]
        self.functions_previous["Tf_partial"][:] = tv
        self.functions_current["Tf_partial"][:] = tv

    # -- time step ----------------------------------------------------------
    def solve_T(self):
        T = self.functions_current["T"]
        Tp = self.functions_previous["T"]
        it, conv, kits = newton_solve(T, lambda u: self.form.residual(u, Tp), self.form.jacobian,
                                      linear=self.linear, bc=self.bc, ksp=self.ksp, **self.newton)
        self.newton_history.append((it, kits))
        assert conv or not self.newton["error_on_nonconvergence"]

    def visco_update(self):
        vp, dt, d = self.vp, self.dt, self.dim
        fc, fp, fn, f = self.functions_current, self.functions_previous, self.functions_next, self.functions
        I = np.eye(d)
        # --- _solve_Tf (TVP:393-407)
        T = fc["T"]
        paper = self.model_mode == "paper"
        Tf_old = fp["Tf"].copy()                                             # Tf_prev of the last step
        if paper:                                                            # VEM:100-108 (Eq.25) honoured
            f["phi"][:] = np.exp(vp.H / vp.Rg * (1.0 / vp.Tb - vp.chi / T - (1.0 - vp.chi) / Tf_old))
        else:
            f["phi"][:] = shift_function(T, vp)                              # VEM:156-161 (Eq.5), Q1
        Tfp_prev = fp["Tf_partial"].reshape(-1, 6)
        phi = f["phi"]
        Tfp = np.empty_like(Tfp_prev)
        for i in range(6):                                                   # VEM:111-119 (Eq.24)
            Tfp[:, i] = (vp.lambda_m[i] * Tfp_prev[:, i] + T * dt * phi) / (vp.lambda_m[i] + dt * phi)
        fc["Tf_partial"][:] = Tfp.ravel()
        fp["Tf_partial"][:] = fc["Tf_partial"]                               # TVP:469-470
        Tfp = fc["Tf_partial"].reshape(-1, 6)
        Tf = np.zeros(self.VT.n)
        for i in range(6):                                                   # VEM:122-125 inner(m, Tf_partial)
            Tf = Tf + vp.m_n[i] * Tfp[:, i]
        fc["Tf"][:] = Tf
        if not paper:
            fp["Tf"][:] = fc["Tf"]                                           # TVP:481-482 (Q2: before the strains)
        # --- _solve_strains (TVP:409-423), evaluated on the sigma space
        Ts = self._src("S", "T", fc["T"])
        Tps = self._src("S", "T", fp["T"])
        Tfs = self._src("S", "T", fc["Tf"])
        Tfps = self._src("S", "T", fp["Tf"])
        scal = vp.alpha_solid * (Ts - Tps) + (vp.alpha_liquid - vp.alpha_solid) * (Tfs - Tfps)
        th = I[None, :, :] * scal[:, None, None]                             # VEM:128-133 (Eq.9)
        f["thermal_strain"][:] = th.ravel()
        tot = -f["thermal_strain"].reshape(-1, d, d)                         # VEM:136-139 (Eq.28)
        f["total_strain"][:] = tot.ravel()
        tot = f["total_strain"].reshape(-1, d, d)
        tr = np.zeros(tot.shape[0])
        for i in range(d):
            tr = tr + tot[:, i, i]
        dev = tot - (1 / self.dim) * I[None] * tr[:, None, None]            # VEM:142-146 (Eq.29)
        f["deviatoric_strain"][:] = dev.ravel()
        if paper:
            fp["Tf"][:] = fc["Tf"]                                           # Tf_prev <- Tf after the strains
        # --- _solve_shifted_time (TVP:426-435)
        Tp = fp["T"]
        fn["T"][:] = T + (T - Tp)                                            # VEM:150-153
        f["phi"][:] = shift_function(T, vp)                                  # VEM:156-161
        fn["phi"][:] = shift_function(fn["T"], vp)                           # VEM:162-167
        if paper:
            f["xi"][:] = dt / 2 * (fn["phi"] + f["phi"])                    # Eq.19, trapezoidal "+"
        else:
            f["xi"][:] = dt / 2 * (fn["phi"] - f["phi"])                    # VEM:170-173 (Eq.19, "-"), Q4
        # --- _solve_stress (TVP:438-452), sigma space
        xi = self._src("S", "T", f["xi"])
        dev = f["deviatoric_strain"].reshape(-1, d, d)
        tot = f["total_strain"].reshape(-1, d, d)
        nS = self.VS.n
        ds = np.empty((nS, 6, d, d))
        for n in range(6):                                                   # VEM:176-182 (Eq.15a+20)
            lam, g = vp.lambda_g[n], vp.g_n[n]
            E = taylor_exponential(xi, lam)
            ds[:, n] = 2.0 * g * dev / xi[:, None, None] * lam * (1.0 - E)[:, None, None]
        f["ds_partial"][:] = ds.ravel()
        # Eq.16: reference feeds s~ from itself (Q3); paper mode from s
        st_cur = (fc["s_partial"] if paper else fc["s_tilde_partial"]).reshape(-1, 6, d, d)
        st_next = np.empty_like(st_cur)
        for n in range(6):                                                   # VEM:195-200 (Eq.16a)
            st_next[:, n] = st_cur[:, n] * taylor_exponential(xi, vp.lambda_g[n])[:, None, None]
        fn["s_tilde_partial"][:] = st_next.ravel()
        fn["s_partial"][:] = f["ds_partial"] + fn["s_tilde_partial"]         # VEM:212-215 (Eq.17a)
        fc["s_tilde_partial"][:] = fn["s_tilde_partial"]                     # TVP:559-562
        fc["s_partial"][:] = fn["s_partial"]
        trI = np.zeros(tot.shape[0])
        for i in range(d):
            trI = trI + tot[:, i, i]
        dsig = np.empty((nS, 6, d, d))
        for n in range(6):                                                   # VEM:185-191 (Eq.15b+20)
            lam, k = vp.lambda_k[n], vp.k_n[n]
            E = taylor_exponential(xi, lam)
            dsig[:, n] = k * (trI[:, None, None] * I[None]) / xi[:, None, None] * lam * (1.0 - E)[:, None, None]
        f["dsigma_partial"][:] = dsig.ravel()
        sg_cur = (fc["sigma_partial"] if paper else fc["sigma_tilde_partial"]).reshape(-1, 6, d, d)
        sg_next = np.empty_like(sg_cur)
        for n in range(6):                                                   # VEM:203-209 (Eq.16b)
            sg_next[:, n] = sg_cur[:, n] * taylor_exponential(xi, vp.lambda_k[n])[:, None, None]
        fn["sigma_tilde_partial"][:] = sg_next.ravel()
        fn["sigma_partial"][:] = f["dsigma_partial"] + fn["sigma_tilde_partial"]   # VEM:218-221
        fc["sigma_tilde_partial"][:] = fn["sigma_tilde_partial"]             # TVP:578-585
        fc["sigma_partial"][:] = fn["sigma_partial"]
        sN = fn["s_partial"].reshape(-1, 6, d, d)
        gN = fn["sigma_partial"].reshape(-1, 6, d, d)
        acc = sN[:, 0] + gN[:, 0]
        for n in range(1, 6):                                                # VEM:224-228 (Eq.18)
            acc = acc + (sN[:, n] + gN[:, n])
        fn["sigma"][:] = acc.ravel()

    def solve_timestep(self, t=None, thermal_only=False):
        self.solve_T()
        if not thermal_only:
            self.visco_update()
        # TVP:378-379: T_prev <- T at the very end of the step
        self.functions_previous["T"][:] = self.functions_current["T"]

    def solve(self, n_steps=None, thermal_only=False):
        n = self.n_steps if n_steps is None else n_steps
        for _ in range(n):
            self.t += self.dt
            self.solve_timestep(self.t, thermal_only=thermal_only)
