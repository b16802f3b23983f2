"""Geometric-multigrid preconditioner (options.preconditioner = GMG, tv_mg.hip)
on the box hierarchy -- SURVEY.md section 8(f) rank 3; the reference configures
PCGAMG (ThermoViscoProblem.py:343-346).

The preconditioner changes the Krylov iterates, not the Newton solution: every
linear solve still reaches rtol 1e-5 and Newton still stops at
||dx|| / ||dx_1|| < 1e-12, so T must match the oracle (its PETSc KSPCG + Jacobi
restatement) to the same 1e-10 as the Jacobi path, with the same Newton
iteration counts.  The Krylov count must drop (the point of the preconditioner).
Stresses follow T (pointwise update), checked with parity_util.check_field.
"""
import numpy as np
import pytest

from oracle import tv_oracle as O
from parity_util import check_field, relerr

CG = {"element": "CG", "degree": 1}


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _pair(axes, mode="reference", **kw):
    from tvfem import RectilinearMesh
    from tvfem.problem import ThermoViscoProblem
    cfg = {"T": CG, "sigma": CG}
    dev = ThermoViscoProblem(RectilinearMesh(axes), (0.0, 1.0), 0.1, cfg, dict(O.MAIN_MODEL_PARAMS), verbose=False,
                             part_axis=2, model_mode=mode, **kw)
    ref = O.OracleProblem(O.rectilinear_mesh(axes), (0.0, 1.0), 0.1, cfg, dict(O.MAIN_MODEL_PARAMS), linear="pcg",
                          model_mode=mode)
    return dev, ref


CASES = {
    # h = 0.125 as at C4 (dt alpha / h^2 = 6.4): three levels
    "plate": [np.linspace(0.0, 4.0, 33), np.linspace(0.0, 3.0, 25), np.linspace(0.0, 1.0, 9)],
    # graded axes (non-uniform interpolation weights), an odd cell count along z
    "graded": [np.concatenate([np.linspace(0.0, 0.5, 9), np.linspace(0.5, 2.5, 9)[1:]]),
               np.linspace(0.0, 2.0, 17), np.linspace(0.0, 0.75, 8)],
    # odd cell counts along x and y (the last fine node kept on every level: odd-tail transfers
    # of the row-wise prolongation), several 64-node x segments
    "oddx": [np.linspace(0.0, 16.375, 132), np.linspace(0.0, 1.875, 16), np.linspace(0.0, 0.5, 5)],
}


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(CASES) + ["plate+fused", "graded+fused"])
def test_gmg_steps_match_oracle(case, monkeypatch):
    """"+fused": level 0's fused residual restriction forced (k_mg_rrestrict, the
    default from 3M nodes)"""
    _torch()
    case, _, fused = case.partition("+")
    monkeypatch.setenv("TVFEM_MG_RR", "1" if fused else "0")
    axes = CASES[case]
    dev, ref = _pair(axes, preconditioner="gmg")
    jac, _ = _pair(axes)
    for p in (dev, ref, jac):
        p.setup()
    kd = kj = 0
    for s in range(4):
        T_before = ref.functions_current["T"].copy()
        for p in (dev, ref, jac):
            p.solve_timestep()
        kd += dev.last_krylov_iterations
        kj += jac.last_krylov_iterations
        assert relerr(dev.functions_current["T"].x.array, ref.functions_current["T"]) < 1e-10, s
        assert dev.last_newton_iterations == ref.newton_history[-1][0], s
    print(f"[gmg] {case}: Krylov iterations over 4 steps: GMG {kd}, Jacobi {kj}")
    assert kd * 3 <= kj, (kd, kj)
    mT = np.abs(ref.functions_current["T"] - T_before) > 1e-6
    check_field(f"sigma[gmg,{case}]", dev.functions_next["sigma"].x.array, ref.functions_next["sigma"], mT, 9,
                min_frac=0.9)
    for p in (dev, jac):
        p.close()


@pytest.mark.gpu
def test_gmg_newton_ahead_mispredicted(monkeypatch):
    """The next Newton iteration's solve is queued before the host reads the
    previous test when the last step took more iterations (newton(), gated on
    the device's test by k_set_state).  A looser Newton rtol makes step 2 end
    before the predicted count (the solve queued ahead is gated off), then the
    default rtol makes step 3 take more than predicted; every state field must
    be bitwise the one of a context that waits at every Newton boundary
    (TVFEM_NEWTON_AHEAD=0), with the same Newton and Krylov counts."""
    _torch()
    axes = CASES["plate"]
    monkeypatch.setenv("TVFEM_NEWTON_AHEAD", "1")
    dev, _ = _pair(axes, preconditioner="gmg")
    monkeypatch.setenv("TVFEM_NEWTON_AHEAD", "0")
    base, _ = _pair(axes, preconditioner="gmg")
    for p in (dev, base):
        p.setup()
    counts = []
    for step, rtol in enumerate((1e-12, 1e-6, 1e-12, 1e-12)):
        for p in (dev, base):
            p.solver.rtol = rtol
            p.solve_timestep()
        counts.append((dev.last_newton_iterations, base.last_newton_iterations))
        assert counts[-1][0] == counts[-1][1], (step, counts)
        assert dev.last_krylov_iterations == base.last_krylov_iterations, step
        for f in ("T", "T_prev", "phi", "Tf", "xi", "sigma"):
            assert np.array_equal(dev.get_field(f), base.get_field(f), equal_nan=True), (step, f)
    assert counts[1][0] < counts[0][0] and counts[2][0] > counts[1][0], counts  # both mispredictions happened
    print(f"[gmg] Newton counts with the solve queued ahead: {counts}")
    for p in (dev, base):
        p.close()


DG = {"element": "DG", "degree": 1}


@pytest.mark.gpu
@pytest.mark.parametrize("sig", ["DG", "CG"])
def test_gmg_dg_steps_match_oracle(sig):
    """DG1 temperature (C5's family): damped-Jacobi smoothing of the SIPG
    operator (weight from a power-iteration estimate of lambda_max(D^-1 J)),
    coarse correction on the CG1 space of the same box (vertex sums / injection)
    and the CG hierarchy below it."""
    _torch()
    from tvfem import RectilinearMesh
    from tvfem.problem import ThermoViscoProblem
    axes = [np.linspace(0.0, 3.0, 13), np.linspace(0.0, 2.5, 11), np.linspace(0.0, 1.0, 6)]
    cfg = {"T": DG, "sigma": DG if sig == "DG" else CG}
    mk = lambda pc: ThermoViscoProblem(RectilinearMesh(axes), (0.0, 1.0), 0.1, cfg, dict(O.MAIN_MODEL_PARAMS),  # noqa: E731
                                       verbose=False, part_axis=2, preconditioner=pc)
    dev, jac = mk("gmg"), mk("jacobi")
    ref = O.OracleProblem(O.rectilinear_mesh(axes), (0.0, 1.0), 0.1, cfg, dict(O.MAIN_MODEL_PARAMS), linear="pcg")
    for p in (dev, jac, ref):
        p.setup()
    kd = kj = 0
    for s in range(3):
        for p in (dev, jac, ref):
            p.solve_timestep()
        kd += dev.last_krylov_iterations
        kj += jac.last_krylov_iterations
        assert relerr(dev.functions_current["T"].x.array, ref.functions_current["T"]) < 1e-10, s
        assert dev.last_newton_iterations == ref.newton_history[-1][0], s
    print(f"[gmg] DG/{sig}: Krylov iterations over 3 steps: GMG {kd}, Jacobi {kj}")
    assert kd * 3 <= kj, (kd, kj)
    for p in (dev, jac):
        p.close()


@pytest.mark.gpu
@pytest.mark.parametrize("levels", [1, 2, 3])
def test_gmg_explicit_levels(levels):
    """Any depth is a valid preconditioner (1 level = two damped-Jacobi steps)."""
    _torch()
    axes = CASES["plate"]
    dev, ref = _pair(axes, preconditioner="gmg", mg_levels=levels)
    dev.setup()
    ref.setup()
    for s in range(2):
        dev.solve_timestep()
        ref.solve_timestep()
        assert relerr(dev.functions_current["T"].x.array, ref.functions_current["T"]) < 1e-10, (levels, s)
    dev.close()


@pytest.mark.gpu
def test_gmg_dirichlet_matches_oracle():
    _torch()
    axes = [np.linspace(0.0, 2.0, 17), np.linspace(0.0, 2.0, 17), np.linspace(0.0, 1.0, 9)]
    dev, ref = _pair(axes, mode="paper", preconditioner="gmg")
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
def test_gmg_vcycle_timing_and_bytes():
    """tv_time_kernel / tv_kernel_bytes id 11 (one V-cycle) run on a live context."""
    import ctypes as C
    _torch()
    dev, _ = _pair(CASES["plate"], preconditioner="gmg")
    dev.setup()
    dev.solve_timestep()
    ms, by = C.c_double(), C.c_double()
    assert dev._lib.tv_time_kernel(dev._ctx, 11, 3, C.byref(ms)) == 0
    assert dev._lib.tv_kernel_bytes(dev._ctx, 11, C.byref(by)) == 0
    assert ms.value > 0.0 and by.value > 0.0
    T = dev.functions_current["T"].x.array.copy()
    dev.solve_timestep()  # the timing left the solver state consistent
    assert np.all(np.isfinite(dev.functions_current["T"].x.array)) and not np.array_equal(T, dev.functions_current["T"].x.array)
    dev.close()


@pytest.mark.gpu
def test_gmg_rejects_unsupported_meshes():
    _torch()
    from tvfem import RectilinearMesh, UnstructuredMesh
    from tvfem._native import NativeError
    from tvfem.problem import ThermoViscoProblem
    cfg = {"T": CG, "sigma": CG}
    mp = dict(O.MAIN_MODEL_PARAMS)
    axes2 = [np.linspace(0, 1, 9), np.linspace(0, 1, 9)]
    with pytest.raises(NativeError):
        ThermoViscoProblem(RectilinearMesh(axes2), (0, 1), 0.1, cfg, mp, verbose=False, preconditioner="gmg")
    axes3 = CASES["plate"]
    # (partitioned boxes are supported: the distributed V-cycle, tests/test_partition.py)
    with pytest.raises(NativeError):  # the single-reduction form with GMG
        ThermoViscoProblem(RectilinearMesh(axes3), (0, 1), 0.1, cfg, mp, verbose=False, preconditioner="gmg",
                           pcg_variant="single")
    with pytest.raises(NativeError):
        ThermoViscoProblem(UnstructuredMesh.from_rectilinear(RectilinearMesh(axes3)), (0, 1), 0.1, cfg, mp,
                           verbose=False, preconditioner="gmg")
    with pytest.raises(NativeError):  # DG1 in 2D
        ThermoViscoProblem(RectilinearMesh(axes2), (0, 1), 0.1, {"T": DG, "sigma": CG}, mp, verbose=False,
                           preconditioner="gmg")


@pytest.mark.gpu
def test_gmg_failed_krylov_solve_leaves_state_untouched():
    """A Krylov solve that ends badly (here DIVERGED_ITS at ksp_max_it = 1)
    raises, and the post-solve group queued behind the multigrid batches
    (dx finish, T <- T - dx, ||dx||) must not have run: T bitwise as before."""
    _torch()
    from tvfem._native import NativeError
    dev, _ = _pair(CASES["plate"], preconditioner="gmg", ksp_max_it=1)
    dev.setup()
    T0 = dev.functions_current["T"].x.array.copy()
    with pytest.raises(NativeError, match="DIVERGED_ITS"):
        dev.solve_timestep()
    T1 = dev.functions_current["T"].x.array
    assert np.array_equal(T0.view(np.uint64), T1.view(np.uint64))
    dev.close()


def test_preconditioner_argument_checked():
    from tvfem import RectilinearMesh
    from tvfem.problem import ThermoViscoProblem
    with pytest.raises(ValueError):
        ThermoViscoProblem(RectilinearMesh(CASES["plate"]), (0, 1), 0.1, {"T": CG, "sigma": CG},
                           dict(O.MAIN_MODEL_PARAMS), verbose=False, preconditioner="gamg")


# ---- the V-cycle operator itself against a numpy restatement --------------------
# (tests/gmg_reference.py: the box hierarchy restated on the oracle's assembled Jacobians)
from gmg_reference import vcycle_reference as _vcycle_reference  # noqa: E402


VCYCLE_CASES = {
    # automatic depth (3 levels, as "plate" above)
    "plate_auto": ([np.linspace(0.0, 4.0, 33), np.linspace(0.0, 3.0, 25), np.linspace(0.0, 1.0, 9)], 0),
    # odd cell counts along all three axes (odd tails of the x-pair transfers, the
    # 2 x 2 prolongation blocks and the fused post-smoothing's side faces), graded x,
    # four explicit levels down to a 3-node axis (generic transfer kernels there)
    "odd_graded_4": ([np.concatenate([np.linspace(0.0, 0.6, 7), np.linspace(0.6, 3.0, 21)[1:]]),
                      np.linspace(0.0, 2.2, 12), np.linspace(0.0, 0.9, 10)], 4),
    # a thin x axis (4 -> 3 -> 2 nodes): the generic transfer kernels, the separate
    # coarse post-smoothing and k_cg_addfaces on the levels where the x-pair kernels
    # do not apply
    "thin_x_4": ([np.linspace(0.0, 0.3, 4), np.linspace(0.0, 2.0, 17), np.linspace(0.0, 1.0, 9)], 4),
}


@pytest.mark.gpu
@pytest.mark.parametrize("fused", [False, True], ids=["jx_restrict", "fused_restrict"])
@pytest.mark.parametrize("case", list(VCYCLE_CASES))
def test_gmg_vcycle_operator_matches_numpy_restatement(case, fused, monkeypatch):
    """tv_precond_apply (one V-cycle: the PCApply of the solve) against the numpy
    V-cycle above at a non-uniform T, to 1e-11; the operator is symmetric (CG
    needs it) and positive.  fused: level 0's restriction as the fused residual
    restriction b_1 = R (r - J x0) without J x0 (k_mg_rrestrict, on by default
    from 3M nodes; forced here, where the geometry allows it: thin_x_4 keeps the
    J x path)"""
    torch = _torch()
    monkeypatch.setenv("TVFEM_MG_RR", "1" if fused else "0")
    from tvfem import RectilinearMesh
    from tvfem.problem import ThermoViscoProblem
    axes, levels = VCYCLE_CASES[case]
    mp = dict(O.MAIN_MODEL_PARAMS)
    cfg = {"T": CG, "sigma": CG}
    p = ThermoViscoProblem(RectilinearMesh(axes), (0.0, 1.0), 0.1, cfg, mp, verbose=False, part_axis=2,
                           preconditioner="gmg", mg_levels=levels)
    p.setup()
    n = p.get_field("T").size
    rng = np.random.default_rng(11)
    T = 700.0 + rng.uniform(0.0, 150.0, n)
    p.set_field("T", T)
    p._flush()
    nlev = levels
    if nlev == 0:  # the automatic depth of mg_setup
        da, nlev, Xp = 0.1 * mp["alpha"], 1, [np.asarray(a) for a in axes]
        while True:
            cells = [len(a) - 1 for a in Xp]
            h = min((a[-1] - a[0]) / c for a, c in zip(Xp, cells) if c >= 1)
            if not any(c >= 2 for c in cells) or da / (h * h) <= 0.5:
                break
            Xp = [a[(np.arange(len(a)) % 2 == 0) | (np.arange(len(a)) == len(a) - 1)] if len(a) >= 3 else a
                  for a in Xp]
            nlev += 1
    B = _vcycle_reference(axes, T, mp, 0.1, nlev)
    r = rng.standard_normal(n)
    y = rng.standard_normal(n)
    out = []
    for v in (r, y):
        vd = torch.tensor(v, dtype=torch.float64, device="cuda")
        zd = torch.empty_like(vd)
        assert p._lib.tv_precond_apply(p._ctx, vd.data_ptr(), zd.data_ptr()) == 0, p._lib.tv_last_error(p._ctx)
        out.append(zd.cpu().numpy())
    z_r, z_y = out
    e = relerr(z_r, B(r))
    sym = abs(y @ z_r - r @ z_y) / abs(y @ z_r)
    print(f"[gmg] V-cycle {case} ({'fused' if fused else 'J x'} restriction): {nlev} levels, vs numpy {e:.2e}, "
          f"symmetry {sym:.1e}, r.Br {r @ z_r:.3e}")
    assert e < 1e-11, e
    assert sym < 1e-12, sym
    assert r @ z_r > 0.0
    p.close()


@pytest.mark.gpu
def test_gmg_zero_residual_step():
    """T_0 = T_ambient = 0 and f = 0: F(T_0) = 0 exactly, so every Krylov solve
    converges at its init (0 iterations) and dx must be exactly 0
    (launch_mg_dx_finish: the init pass leaves dx to iteration 1); T stays 0 and
    the Newton counts equal the oracle's (2 per step)."""
    _torch()
    axes = CASES["plate"]
    mp = dict(O.MAIN_MODEL_PARAMS)
    mp["T_0"] = 0.0
    mp["T_ambient"] = 0.0
    mp["f"] = 0.0
    from tvfem import RectilinearMesh
    from tvfem.problem import ThermoViscoProblem
    cfg = {"T": CG, "sigma": CG}
    dev = ThermoViscoProblem(RectilinearMesh(axes), (0.0, 1.0), 0.1, cfg, mp, verbose=False, part_axis=2,
                             preconditioner="gmg")
    ref = O.OracleProblem(O.rectilinear_mesh(axes), (0.0, 1.0), 0.1, cfg, mp, linear="pcg")
    dev.setup()
    ref.setup()
    for _ in range(2):
        dev.solve_timestep()
        ref.solve_timestep()
        assert dev.last_krylov_iterations == 0
        assert dev.last_newton_iterations == ref.newton_history[-1][0]
        assert ref.newton_history[-1][1] == 0
        T = dev.functions_current["T"].x.array
        assert np.array_equal(T, np.zeros_like(T)), np.abs(T).max()
    dev.close()


@pytest.mark.gpu
def test_precond_apply_jacobi_matches_oracle_diagonal():
    """tv_precond_apply with the Jacobi preconditioner: z = r / diag J(T), the
    diagonal of the oracle's assembled Jacobian at a non-uniform T (1e-13)."""
    torch = _torch()
    from tvfem import RectilinearMesh
    from tvfem.problem import ThermoViscoProblem
    axes = CASES["graded"]
    mp = dict(O.MAIN_MODEL_PARAMS)
    p = ThermoViscoProblem(RectilinearMesh(axes), (0.0, 1.0), 0.1, {"T": CG, "sigma": CG}, mp, verbose=False,
                           part_axis=2, preconditioner="jacobi")
    p.setup()
    n = p.get_field("T").size
    rng = np.random.default_rng(5)
    T = 700.0 + rng.uniform(0.0, 150.0, n)
    p.set_field("T", T)
    p._flush()
    r = rng.standard_normal(n)
    rd = torch.tensor(r, dtype=torch.float64, device="cuda")
    zd = torch.empty_like(rd)
    assert p._lib.tv_precond_apply(p._ctx, rd.data_ptr(), zd.data_ptr()) == 0
    J = O.HeatForm(O.Space(O.rectilinear_mesh(axes), "CG", 1), 0.1, O.ThermalParams.from_dict(mp)).jacobian(T)
    assert relerr(zd.cpu().numpy(), r / J.diagonal()) < 1e-13
    p.close()
