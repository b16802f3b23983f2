"""problem.solver / problem.ksp (ThermoViscoProblem.py:330-346): the dolfinx
NewtonSolver and PETSc KSP attributes a caller of the reference sets after
setup(), against the oracle run with the same settings (its newton_solve /
pcg_jacobi restatements take the same tolerances), and the failure paths of a
Newton solve that reaches max_it (dolfinx raises RuntimeError; with
error_on_nonconvergence off _solve_T fails its assert(converged), :390).

Tolerances as tests/test_gpu_parity.py: T rel. L2 <= 1e-10 (1e-9 with the
looser linear solves), Newton counts equal, Krylov counts within
max(one per Newton solve, 5 %)."""
import numpy as np
import pytest

from oracle import tv_oracle as O
from test_gpu_parity import AXES, CG, check_counts, make_pair, _torch
from parity_util import relerr

pytestmark = pytest.mark.gpu

STATE = ("T", "T_prev", "phi", "Tf", "xi", "sigma")


def _state(dev):
    return {f: dev.get_field(f).copy() for f in STATE}


def _first_step_newton_count():
    r = O.OracleProblem(O.rectilinear_mesh(AXES["3d"]), (0.0, 1.0), 0.1, {"T": CG, "sigma": CG},
                        dict(O.MAIN_MODEL_PARAMS), linear="pcg")
    r.setup()
    r.solve_T()
    return r.newton_history[0][0]


def test_solver_objects_defaults_and_checks():
    _torch()
    dev, _ = make_pair(AXES["3d"], {"T": CG, "sigma": CG})
    s, k = dev.solver, dev.ksp
    assert k is s.krylov_solver
    assert (s.rtol, s.atol, s.max_it, s.error_on_nonconvergence) == (1e-12, 1e-10, 50, True)
    assert s.convergence_criterion == "incremental" and s.report
    assert k.getType() == "cg" and k.getPC().getType() == "jacobi"
    assert k.getTolerances() == (1e-5, 1e-50, 1e5, 10000)
    s.max_it = 7
    k.setTolerances(rtol=1e-7)
    assert s.max_it == 7 and k.getTolerances() == (1e-7, 1e-50, 1e5, 10000)
    from tvfem._native import NativeError
    with pytest.raises(NativeError):
        s.max_it = 0
    with pytest.raises(NativeError):
        k.setTolerances(rtol=-1.0)
    with pytest.raises(NotImplementedError):
        s.convergence_criterion = "residual"
    # _update_values (ThermoViscoProblem.py:349-354): previous <- current
    s.max_it = 50
    k.setTolerances(rtol=1e-5)
    dev.solve_timestep()
    dev._update_values(dev.functions_current["T"], dev.functions_next["T"])
    dev._flush()
    assert np.array_equal(dev.get_field("T_next"), dev.get_field("T"))
    dev.close()


def test_tolerances_match_oracle():
    """looser Newton test, tighter Krylov test: same counts and iterates"""
    _torch()
    dev, ref = make_pair(AXES["3d"], {"T": CG, "sigma": CG})
    dev.solver.rtol = 1e-6
    dev.ksp.setTolerances(rtol=1e-8)
    ref.newton["rtol"] = 1e-6
    ref.ksp = {"rtol": 1e-8}
    its = []
    for s in range(4):
        dev.solve_timestep()
        ref.solve_timestep()
        its.append((dev.last_newton_iterations, dev.last_krylov_iterations))
        assert relerr(dev.functions_current["T"].x.array, ref.functions_current["T"]) < 1e-9, s
    check_counts(its, ref.newton_history)
    # NewtonSolver.solve(u) -> (n, converged), the _solve_T call (:389)
    n, conv = dev.solver.solve(dev.functions_current["T"])
    ref.solve_T()
    assert conv and n == ref.newton_history[-1][0]
    assert relerr(dev.functions_current["T"].x.array, ref.functions_current["T"]) < 1e-9
    dev.close()


@pytest.mark.parametrize("after_converged_step", [False, True])
def test_newton_failure_keeps_step_state(after_converged_step):
    """max_it below the count the step needs, error_on_nonconvergence on:
    RuntimeError, and the step's end (visco update, T_prev <- T) not run.  A
    fresh context queues the end at every iteration from the second on, gated
    on the device's copy of the Newton test (all gated off here); after a
    converged step it predicts that step's count, beyond max_it (no end queued)"""
    _torch()
    n1 = _first_step_newton_count()
    assert n1 >= 3
    dev, ref = make_pair(AXES["3d"], {"T": CG, "sigma": CG})
    if after_converged_step:
        dev.solve_timestep()
        ref.solve_timestep()
        n2 = ref.newton_history[-1][0]
    else:
        n2 = n1
    before = _state(dev)
    dev.solver.max_it = n2 - 1
    with pytest.raises(RuntimeError, match="did not converge"):
        dev.solve_timestep()
    after = _state(dev)
    for f in ("T_prev", "phi", "Tf", "xi", "sigma"):
        assert np.array_equal(after[f], before[f], equal_nan=True), f
    # T holds the last Newton iterate, as the oracle's after the same iterations
    ref.newton.update(max_it=n2 - 1, error_on_nonconvergence=False)
    ref.solve_T()
    assert relerr(after["T"], ref.functions_current["T"]) < 1e-10
    dev.close()


def test_error_off_keeps_step_state_then_asserts():
    """error_on_nonconvergence off: dolfinx returns (max_it, False) and
    _solve_T's assert(converged) (ThermoViscoProblem.py:390) fires before
    _solve_Tf and the stress updates (:372-381) -- so T holds the last Newton
    iterate (the oracle's T after the same iterations) while T_prev and the
    viscoelastic state keep the previous step's values (the step end
    used to run ungated here)"""
    _torch()
    n1 = _first_step_newton_count()
    dev, ref = make_pair(AXES["3d"], {"T": CG, "sigma": CG})
    before = _state(dev)
    dev.solver.max_it = n1 - 1
    dev.solver.error_on_nonconvergence = False
    ref.newton.update(max_it=n1 - 1, error_on_nonconvergence=False)
    with pytest.raises(AssertionError):
        dev.solve_timestep()
    ref.solve_T()  # the oracle's Newton solve alone: the reference stops at the assert
    assert dev.last_newton_iterations == n1 - 1
    st = _state(dev)
    assert relerr(st["T"], ref.functions_current["T"]) < 1e-10
    for f in ("T_prev", "phi", "Tf", "xi", "sigma"):
        assert np.array_equal(st[f], before[f], equal_nan=True), f
    # the context stays usable: with the default max_it the next step converges
    dev.solver.max_it = 50
    dev.solver.error_on_nonconvergence = True
    dev.solve_timestep()
    dev.close()
