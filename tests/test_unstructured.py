"""General quadrilateral / hexahedral meshes:
the gmsh reader, the RCB partitioner, and the element-local isoparametric
kernels (csrc/tv_um.hip) against the oracle's generic isoparametric assembly
(oracle/tv_oracle.py:297-507), which the rectilinear cases already pin.

The meshes are distorted on purpose: interior vertices jittered, a shear and a
smooth warp applied (non-planar hex faces), vertex ids and cell order shuffled.

Tolerances (float64): operators F, J x, diag J rel. L2 <= 1e-12 (exact
quadrature on both sides: 3 Gauss points per direction); T per step rel. L2
<= 1e-10; stresses by parity_util.check_field (rel. 1e-6 on well-conditioned
dofs).
"""
import os

import numpy as np
import pytest

from oracle import tv_oracle as O
from parity_util import check_field, relerr

CG = {"element": "CG", "degree": 1}


def distorted_mesh(n, L, seed=0, amp=0.2, shuffle=True):
    from tvfem import distorted_box_mesh
    return distorted_box_mesh(L, n, amp=amp, seed=seed, shuffle=shuffle)


def oracle_mesh(m):
    return O.Mesh(dim=m.dim, x=m.x[:, :m.dim].copy(), cells=m.cells.copy())


# ---------------------------------------------------------------- CPU -------
def test_msh_roundtrip_hexahedra(tmp_path):
    from tvfem.mesh import read_msh, write_msh_unstructured
    m = distorted_mesh((3, 2, 2), (1.0, 1.0, 0.5), seed=3)
    path = os.path.join(tmp_path, "hex.msh")
    write_msh_unstructured(path, m)
    r = read_msh(path)
    assert type(r).__name__ == "UnstructuredMesh" and r.dim == 3
    assert np.array_equal(r.cells, m.cells)
    assert np.array_equal(r.x, m.x)


def test_msh_roundtrip_quadrilaterals(tmp_path):
    from tvfem.mesh import read_msh, write_msh_unstructured
    m = distorted_mesh((4, 3), (2.0, 1.0), seed=4)
    path = os.path.join(tmp_path, "quad.msh")
    write_msh_unstructured(path, m)
    r = read_msh(path)
    assert r.dim == 2 and np.array_equal(r.cells, m.cells) and np.array_equal(r.x, m.x)


def test_from_rectilinear_matches_oracle_numbering():
    from tvfem import RectilinearMesh, UnstructuredMesh
    axes = [np.linspace(0, 1, 4), np.linspace(0, 2, 3), np.array([0.0, 0.3, 1.0])]
    m = UnstructuredMesh.from_rectilinear(RectilinearMesh(axes))
    o = O.rectilinear_mesh(axes)
    assert np.array_equal(m.cells, o.cells) and np.array_equal(m.x[:, :3], o.x)


def test_oracle_isoparametric_known_answers():
    """Mass matrix sums to the volume (an affine image of a box: det(A) x box
    volume, exact under 3-point Gauss); stiffness rows sum to 0."""
    from tvfem import RectilinearMesh, UnstructuredMesh
    A = np.array([[1.0, 0.3, 0.1], [0.2, 1.5, -0.2], [0.0, 0.1, 0.8]])
    base = UnstructuredMesh.from_rectilinear(RectilinearMesh([np.linspace(0, 2, 5), np.linspace(0, 1, 4),
                                                              np.linspace(0, 1, 3)]))
    m = O.Mesh(dim=3, x=base.x @ A.T, cells=base.cells)
    form = O.HeatForm(O.Space(m, "CG"), 0.1, O.ThermalParams.from_dict(O.MAIN_MODEL_PARAMS))
    assert abs(form.Me.sum() - 2.0 * np.linalg.det(A)) < 1e-12
    assert np.abs(form.Ke.sum(axis=2)).max() < 1e-12
    dm = distorted_mesh((4, 3, 2), (2.0, 1.0, 1.0), seed=5)
    form = O.HeatForm(O.Space(oracle_mesh(dm), "CG"), 0.1, O.ThermalParams.from_dict(O.MAIN_MODEL_PARAMS))
    assert np.all(form.cw > 0.0)                      # valid (positive-Jacobian) distorted cells
    assert np.abs(form.Ke.sum(axis=2)).max() < 1e-12


def test_rcb_partition_balanced_and_deterministic():
    from tvfem.parallel import rcb_partition
    m = distorted_mesh((12, 6, 5), (4.0, 2.0, 1.0), seed=6)
    for n_parts in (1, 2, 3, 5, 8):
        part = rcb_partition(m, n_parts)
        cnt = np.bincount(part, minlength=n_parts)
        assert cnt.sum() == m.num_cells and cnt.min() > 0
        levels = int(np.ceil(np.log2(n_parts))) if n_parts > 1 else 0
        assert cnt.max() - cnt.min() <= max(1, levels), cnt
        assert np.array_equal(part, rcb_partition(m, n_parts))
    # the first cut is across the longest extent (x)
    part = rcb_partition(m, 2)
    cx = m.x[m.cells][:, :, 0].mean(axis=1)
    assert cx[part == 0].max() <= cx[part == 1].min() + 1e-12


def test_partition_submesh_covers_mesh():
    from tvfem.parallel import partition_submesh, rcb_partition
    m = distorted_mesh((6, 4, 3), (3.0, 2.0, 1.0), seed=7)
    part = rcb_partition(m, 4)
    owned = np.zeros(m.num_vertices, dtype=int)
    n_cells = 0
    for p in range(4):
        s = partition_submesh(m, part, p)
        sub, l2g = s["mesh"], s["l2g"]
        n_cells += sub.num_cells
        owned[l2g[:s["n_owned"]]] += 1
        assert np.array_equal(l2g[sub.cells], m.cells[part == p])
        assert np.array_equal(sub.x, m.x[l2g])
        assert np.all(s["ghost_owner"] != p)
    assert n_cells == m.num_cells and np.all(owned == 1)


def test_rcb_rejects_bad_counts():
    from tvfem.parallel import rcb_partition
    m = distorted_mesh((2, 2), (1.0, 1.0), seed=8)
    with pytest.raises(RuntimeError):
        rcb_partition(m, 0)
    with pytest.raises(RuntimeError):
        rcb_partition(m, 5)


# ---------------------------------------------------------------- GPU -------
def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


MESHES = {
    "quad": ((9, 5), (3.0, 1.0)),
    "hex": ((7, 5, 4), (2.0, 2.0, 1.0)),
    # numbered plane by plane (not shuffled), as gmsh and the box meshes number them
    "hex_ordered": ((7, 5, 4), (2.0, 2.0, 1.0)),
}


def make_pair(name, mode="reference", seed=0, **kw):
    from tvfem.problem import ThermoViscoProblem
    n, L = MESHES[name]
    m = distorted_mesh(n, L, seed=seed, shuffle=not name.endswith("_ordered"))
    cfg = {"T": CG, "sigma": CG}
    dev = ThermoViscoProblem(m, (0.0, 1.0), 0.1, cfg, dict(O.MAIN_MODEL_PARAMS), verbose=False, model_mode=mode, **kw)
    ref = O.OracleProblem(oracle_mesh(m), (0.0, 1.0), 0.1, cfg, dict(O.MAIN_MODEL_PARAMS), linear="pcg",
                          model_mode=mode)
    return m, dev, ref


@pytest.mark.gpu
@pytest.mark.parametrize("name", list(MESHES))
def test_unstructured_operators_match_oracle(name):
    torch = _torch()
    m, dev, ref = make_pair(name)
    dev.setup()
    ref.setup()
    assert np.array_equal(dev._dof_coordinates(0)[:, :m.dim], ref.VT.dof_coordinates())
    rng = np.random.default_rng(0)
    n = ref.VT.n
    X = ref.VT.dof_coordinates()
    T = 700.0 + 100.0 * np.cos(X[:, 0] / 0.7) + rng.uniform(-5, 5, n)
    Tp = T + rng.uniform(-3, 3, n)
    dev.set_field("T", T)
    dev.set_field("T_prev", Tp)
    lib, ctx = dev._lib, dev._ctx
    Td = torch.tensor(T, dtype=torch.float64, device="cuda")
    Fd = torch.zeros_like(Td)
    assert lib.tv_residual(ctx, Td.data_ptr(), Fd.data_ptr()) == 0
    assert relerr(Fd.cpu().numpy(), ref.form.residual(T, Tp)) < 1e-12
    x = rng.standard_normal(n)
    xd = torch.tensor(x, dtype=torch.float64, device="cuda")
    yd = torch.zeros_like(xd)
    assert lib.tv_jacobian_apply(ctx, xd.data_ptr(), yd.data_ptr()) == 0
    J = ref.form.jacobian(T)
    assert relerr(yd.cpu().numpy(), J @ x) < 1e-12
    dd = torch.zeros_like(xd)
    assert lib.tv_jacobian_diag(ctx, dd.data_ptr()) == 0
    assert relerr(dd.cpu().numpy(), J.diagonal()) < 1e-12
    dev.close()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["reference", "paper"])
@pytest.mark.parametrize("name", list(MESHES))
def test_unstructured_steps_match_oracle(name, mode):
    _torch()
    m, dev, ref = make_pair(name, mode)
    dev.setup()
    ref.setup()
    its = []
    for s in range(4):
        T_before = ref.functions_current["T"].copy()
        dev.solve_timestep()
        ref.solve_timestep()
        its.append((dev.last_newton_iterations, dev.last_krylov_iterations))
        assert relerr(dev.functions_current["T"].x.array, ref.functions_current["T"]) < 1e-10, s
    for (n_d, k_d), (n_r, k_r) in zip(its, ref.newton_history):
        assert n_d == n_r, (its, ref.newton_history)
        assert abs(k_d - k_r) <= max(n_r, int(np.ceil(0.05 * k_r))), (its, ref.newton_history)
    d2 = m.dim ** 2
    mT = np.abs(ref.functions_current["T"] - T_before) > 1e-6
    assert relerr(dev.functions_current["Tf"].x.array, ref.functions_current["Tf"]) < 1e-10
    check_field(f"sigma[{name},{mode}]", dev.functions_next["sigma"].x.array, ref.functions_next["sigma"], mT, d2,
                min_frac=0.9)
    dev.close()


@pytest.mark.gpu
def test_unstructured_dirichlet_matches_oracle():
    _torch()
    m, dev, ref = make_pair("hex", "paper")
    dev.setup(dirichlet_bc=True)
    ref.setup(dirichlet_bc=True)
    dofs, g = ref.bc
    for s in range(3):
        dev.solve_timestep()
        ref.solve_timestep()
        T = dev.functions_current["T"].x.array
        assert np.all(T[dofs] == g), s
        assert relerr(T, ref.functions_current["T"]) < 1e-10, s
        assert dev.last_newton_iterations == ref.newton_history[-1][0]
    dev.close()


@pytest.mark.gpu
def test_rectilinear_as_unstructured_matches_structured_path():
    """The same grid through both device paths (marching tensor-product
    kernels vs element-local kernels): T and sigma agree to rounding."""
    _torch()
    from tvfem import RectilinearMesh, UnstructuredMesh
    from tvfem.problem import ThermoViscoProblem
    axes = [np.linspace(0.0, 2.0, 9), np.linspace(0.0, 1.5, 7), np.array([0.0, 0.2, 0.5, 1.0])]
    cfg = {"T": CG, "sigma": CG}
    a = ThermoViscoProblem(RectilinearMesh(axes), (0.0, 1.0), 0.1, cfg, dict(O.MAIN_MODEL_PARAMS), verbose=False,
                           part_axis=2)
    b = ThermoViscoProblem(UnstructuredMesh.from_rectilinear(RectilinearMesh(axes)), (0.0, 1.0), 0.1, cfg,
                           dict(O.MAIN_MODEL_PARAMS), verbose=False)
    a.setup()
    b.setup()
    for s in range(3):
        a.solve_timestep()
        b.solve_timestep()
        assert relerr(b.functions_current["T"].x.array, a.functions_current["T"].x.array) < 1e-12, s
        assert a.last_newton_iterations == b.last_newton_iterations
    a.close()
    b.close()


@pytest.mark.gpu
def test_unstructured_output_series(tmp_path):
    _torch()
    from tvfem.xdmf import read_series
    out = os.path.join(tmp_path, "um_out")
    m, dev, ref = make_pair("hex", write_output=True, output_dir=out)
    dev.setup()
    for _ in range(2):
        dev.solve_timestep()
    T_last = dev.functions_current["T"].x.array.copy()
    dev.close()
    s = read_series(os.path.join(out, "T.xdmf"))
    assert len(s["times"]) == 3
    assert np.array_equal(s["geometry"], m.x)
    vtk = [0, 1, 3, 2, 4, 5, 7, 6]
    assert np.array_equal(s["topology"], m.cells[:, vtk])
    assert np.array_equal(s["values"][-1].ravel(), T_last)
