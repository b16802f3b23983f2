"""Parity at BASELINE.json's full sizes.

C3 (200 x 200 x 25 CG1 hex, 1.05M dofs, coupled): pinned to the oracle at full
size -- its own residual (HeatForm.residual, one vectorised assembly) at the
device's converged T, and its own visco_update (OracleProblem.visco_update)
applied to the device's T / T_prev / Tf / Tf_partial, against every state field
the device wrote (test_c3_fullsize_steps_pinned_to_oracle).

C3, C4 (400 x 400 x 50 CG1 hex, 8.2M dofs) and C5 (200 x 200 x 25 DG1, 8M dofs)
on the 50 x 50 x 5 plate of bench.py, through size-independent properties (the
oracle cannot run a Newton solve at these sizes in a test's time):
  * J(T) is symmetric: y.(J x) = x.(J y) for random x, y (SIPG and the Robin
    facet terms included);
  * J(T0) 1 sums to |Omega| + dt dg(T0) |dOmega| at a uniform T0: the stiffness
    and the SIPG terms annihilate constants, the mass and the boundary mass sum
    to the volume and the area (ThermoViscoProblem.py:293-325 with
    dg(T) = 0.001 (4 sigma eps T^3 + htc));
  * one coupled step with the geometric-multigrid preconditioner and one with
    Jacobi give the same T (Newton to 1e-12 either way, so only the Krylov
    iterates differ) and the same Newton count, and the converged residual is
    small against the first one.

C4 and C5 at full size are also pinned to the C/OpenMP port of the oracle
(oracle/tv_cpu.c, itself pinned to the numpy oracle by tests/test_cpu_port.py):
two coupled steps of the whole 8M-dof plate on both, the same Newton counts,
T, phi and Tf at 1e-10, xi and sigma by check_field
(test_fullsize_step_pinned_to_cpu_port).
"""
import numpy as np
import pytest

from oracle import tv_oracle as O

L = (50.0, 50.0, 5.0)
SIZES = {"C3": ("CG", (200, 200, 25)), "C4": ("CG", (400, 400, 50)), "C5": ("DG", (200, 200, 25))}
# the marching kernels' tile mapping (march_tile: face-chunk tiles first on
# every XCD) with THREE chunks along the march axis -- one interior chunk and
# uneven per-XCD shares: 401 x 33 x 1201 nodes, 7 x 151 tiles per chunk,
# 3 chunks of 11 planes (a tile left out or mapped twice breaks the sum or
# the symmetry below)
OPERATOR_SIZES = {**SIZES, "T3": ("CG", (400, 1200, 32))}


def _torch():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def _problem(fam, nc, pc, part_axis=1):
    from tvfem import box_mesh
    from tvfem.problem import ThermoViscoProblem
    cfg = {"T": {"element": fam, "degree": 1}, "sigma": {"element": fam, "degree": 1}}
    return ThermoViscoProblem(box_mesh(L, nc), (0.0, 1.0), 0.1, cfg, dict(O.MAIN_MODEL_PARAMS), verbose=False,
                              materialize=False, part_axis=part_axis, preconditioner=pc)


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(OPERATOR_SIZES))
def test_fullsize_jacobian_symmetry_and_constants(case):
    torch = _torch()
    fam, nc = OPERATOR_SIZES[case]
    p = _problem(fam, nc, "jacobi")
    p.setup()
    lib, ctx = p._lib, p._ctx
    n = p.get_field("T").size
    g = torch.Generator(device="cuda").manual_seed(7)
    x = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
    y = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
    jx, jy = torch.empty_like(x), torch.empty_like(y)
    assert lib.tv_jacobian_apply(ctx, x.data_ptr(), jx.data_ptr()) == 0
    assert lib.tv_jacobian_apply(ctx, y.data_ptr(), jy.data_ptr()) == 0
    a, b = float(torch.dot(y, jx)), float(torch.dot(x, jy))
    assert abs(a - b) <= 1e-12 * (abs(a) + abs(b)), (case, a, b)
    one = torch.ones(n, dtype=torch.float64, device="cuda")
    j1 = torch.empty_like(one)
    assert lib.tv_jacobian_apply(ctx, one.data_ptr(), j1.data_ptr()) == 0
    mp = O.MAIN_MODEL_PARAMS
    T0 = mp["T_0"]
    dg = 0.001 * (4.0 * mp["sigma"] * mp["epsilon"] * T0 ** 3 + mp["htc"])
    vol = L[0] * L[1] * L[2]
    area = 2.0 * (L[0] * L[1] + L[0] * L[2] + L[1] * L[2])
    want = vol + 0.1 * dg * area
    got = float(j1.sum())
    print(f"[fullsize] {case}: n {n}, sum J1 {got:.12e} vs {want:.12e}; symmetry {abs(a - b) / abs(a):.1e}")
    assert abs(got - want) <= 1e-10 * want, (case, got, want)
    p.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", list(SIZES))
def test_fullsize_gmg_step_matches_jacobi_step(case):
    import ctypes as C
    from tvfem import _native as N
    torch = _torch()
    fam, nc = SIZES[case]
    out = {}
    for pc in ("gmg", "jacobi"):
        p = _problem(fam, nc, pc)
        p.setup()
        T0 = p.get_field("T")
        lib, ctx = p._lib, p._ctx
        n = T0.size
        # residual at the start of the step (T = T_prev = T0: only the Robin and source terms)
        Td = torch.tensor(T0, dtype=torch.float64, device="cuda")
        F0 = torch.empty_like(Td)
        assert lib.tv_residual(ctx, Td.data_ptr(), F0.data_ptr()) == 0
        p.solve_timestep()
        T1 = p.get_field("T")
        # the converged step's residual, F(T1; T_prev = T0), against the initial one:
        # T1 from the context's own device field (device layout), T_prev reset to the
        # uniform T0 the visco update overwrote
        p.set_field("T_prev", T0)
        p._flush()
        ptr, stride = C.c_void_p(), C.c_int64()
        assert lib.tv_field_device_ptr(ctx, N.FIELD_ID["T"], C.byref(ptr), C.byref(stride)) == 0
        F1 = torch.empty_like(Td)
        assert lib.tv_residual(ctx, ptr.value, F1.data_ptr()) == 0
        ratio = float(torch.linalg.norm(F1) / torch.linalg.norm(F0))
        out[pc] = (T1, p.last_newton_iterations, p.last_krylov_iterations, ratio, n)
        p.close()
    Tg, ng, kg, rg, n = out["gmg"]
    Tj, nj, kj, rj, _ = out["jacobi"]
    rel = float(np.linalg.norm(Tg - Tj) / np.linalg.norm(Tj))
    print(f"[fullsize] {case}: n {n}, T gmg vs jacobi {rel:.2e}; Newton {ng} / {nj}, Krylov {kg} / {kj}; "
          f"|F(T1)| / |F(T0)| {rg:.1e} / {rj:.1e}")
    assert rel < 1e-10, rel
    assert ng == nj
    assert kg * 3 <= kj
    assert rg < 1e-6 and rj < 1e-6, (rg, rj)


@pytest.mark.gpu
@pytest.mark.parametrize("pc", ["jacobi", "gmg"])
def test_c3_fullsize_steps_pinned_to_oracle(pc):
    """C3 at full size (200 x 200 x 25 CG1/CG1, 1,050,426 T-dofs, coupled, 6-term
    Prony), three steps with the default (Jacobi) and the multigrid
    preconditioner.  After every step:
      * the oracle's residual F(T_dev; T_prev) (ThermoViscoProblem.py:293-306,
        oracle HeatForm.residual) is <= 1e-10 relative to F(T_prev; T_prev), the
        residual the step started from;
      * the oracle's viscoelastic pipeline (OracleProblem.visco_update,
        ViscoelasticModel.py:100-228 in the order of ThermoViscoProblem.py:393-595)
        run on the device's T, T_prev and pre-step Tf / Tf_partial reproduces
        the device's phi, Tf, Tf_partial (1e-12), xi and sigma (check_field:
        rel. 1e-6 on the dofs with |T - T_prev| > 1e-6 K, >= 90 % of them, the
        rest bounded in absolute terms).
    part_axis=2 keeps the device's storage order equal to the oracle's dof order."""
    _torch()
    from parity_util import check_field, cond_mask, relerr
    fam, nc = SIZES["C3"]
    dev = _problem(fam, nc, pc, part_axis=2)
    dev.setup()
    mesh = O.box_mesh(L, nc)
    cfg = {"T": {"element": "CG", "degree": 1}, "sigma": {"element": "CG", "degree": 1}}
    ref = O.OracleProblem(mesh, (0.0, 1.0), 0.1, cfg, dict(O.MAIN_MODEL_PARAMS))
    ref.setup()
    hf = ref.form
    assert hf.congruent and ref.VT.n == dev.num_dofs(0)[0] == 1_050_426
    for step in range(3):
        Tp = dev.get_field("T")  # T_prev of this step (T_prev <- T ended the last one)
        Tf0, Tfp0 = dev.get_field("Tf"), dev.get_field("Tf_partial")
        dev.solve_timestep()
        T1 = dev.get_field("T")
        F0 = np.linalg.norm(hf.residual(Tp, Tp))
        F1 = np.linalg.norm(hf.residual(T1, Tp))
        print(f"[c3 {pc}] step {step}: Newton {dev.last_newton_iterations}, Krylov {dev.last_krylov_iterations}, "
              f"|F(T1)| / |F(T0)| = {F1 / F0:.2e}, |T1 - T0| max {np.abs(T1 - Tp).max():.3e} K")
        assert F1 <= 1e-10 * F0, (step, F1, F0)
        # the oracle's visco pipeline on the device's inputs
        ref.functions_current["T"][:] = T1
        ref.functions_previous["T"][:] = Tp
        for fd in (ref.functions_current, ref.functions_previous):
            fd["Tf"][:] = Tf0
            fd["Tf_partial"][:] = Tfp0
        ref.visco_update()
        mT, _ = cond_mask(T1, Tp)
        assert relerr(dev.get_field("phi"), ref.functions["phi"]) < 1e-12
        assert relerr(dev.get_field("Tf"), ref.functions_current["Tf"]) < 1e-12
        assert relerr(dev.get_field("Tf_partial"), ref.functions_current["Tf_partial"]) < 1e-12
        check_field("xi", dev.get_field("xi"), ref.functions["xi"], mT, min_frac=0.9)
        check_field("sigma", dev.get_field("sigma"), ref.functions_next["sigma"], mT, bs=9, min_frac=0.9)
    dev.close()


@pytest.mark.gpu
@pytest.mark.parametrize("case", ["C4", "C5"])
def test_fullsize_step_pinned_to_cpu_port(case):
    """One coupled step of C4 (CG1, 8.2M dofs) / C5 (DG1, 8M dofs) on the GPU
    (the bench's GMG) and on the oracle's C/OpenMP port (GMG for CG1, Jacobi for
    DG1: the preconditioner moves only the Krylov iterates, Newton converges to
    1e-12 either way): the same Newton count, T / phi / Tf to 1e-10, xi and
    sigma on the dofs whose temperature moved (parity_util.check_field).
    part_axis=2 keeps the device's storage order equal to the port's dof order."""
    _torch()
    from parity_util import check_field, cond_mask, relerr
    from oracle import tv_cpu
    fam, nc = SIZES[case]
    p = _problem(fam, nc, "gmg", part_axis=2)
    p.setup()
    T0 = p.get_field("T")
    p.solve_timestep()
    dev = {k: p.get_field(k) for k in ("T", "phi", "xi", "Tf", "sigma")}
    nd = p.last_newton_iterations
    p.close()
    axes = [np.linspace(0.0, l, n + 1) for l, n in zip(L, nc)]
    cpu = tv_cpu.CpuProblem(axes, dict(O.MAIN_MODEL_PARAMS), 0.1, fam, pc="gmg" if fam == "CG" else "jacobi")
    try:
        nit, kit = cpu.step()
        nl = 8

        def host(a, bs=1):  # port layout (DG: l * ncell + cell) -> the problem's (cell-major)
            return a if fam == "CG" else a.reshape(nl, -1, bs).transpose(1, 0, 2).reshape(-1)
        ref = {k: host(cpu.get(k), 9 if k == "sigma" else 1) for k in ("T", "phi", "xi", "Tf", "sigma")}
    finally:
        cpu.close()
    errs = {k: relerr(dev[k], ref[k]) for k in ("T", "phi", "Tf")}
    print(f"[fullsize] {case} vs CPU port: Newton {nd} / {nit}, Krylov (port) {kit}, "
          + ", ".join(f"{k} {v:.1e}" for k, v in errs.items()))
    assert nd == nit, (nd, nit)
    for k, v in errs.items():
        assert v < 1e-10, (k, v)
    mT, _ = cond_mask(ref["T"], T0)
    check_field(f"xi[{case} full size, cpu port]", dev["xi"], ref["xi"], mT, min_frac=0.9)
    check_field(f"sigma[{case} full size, cpu port]", dev["sigma"], ref["sigma"], mT, bs=9, min_frac=0.9)
