"""The solver objects the reference exposes on a set-up problem.

``ThermoViscoProblem._setup_solver`` (ThermoViscoProblem.py:330-346) creates
``problem.solver``, a dolfinx ``NewtonSolver`` (incremental criterion, rtol
1e-12, report on), and ``problem.ksp = solver.krylov_solver``, the PETSc KSP of
its linear solves.  A caller of the reference tunes them by attribute
(``problem.solver.max_it = 20``, ``problem.ksp.setTolerances(rtol=1e-8)``) and
``_solve_T`` (:384-391) runs ``solver.solve(T)``.  These two classes keep that
surface over the native context: the tolerances live in the context's options
(``tv_set_newton_tolerances`` / ``tv_set_ksp_tolerances``, read at the next
solve) and ``solve`` is ``tv_solve_T`` -- the whole Newton loop on the GPU.
"""
from __future__ import annotations

import ctypes as C

from . import _native as N


def _options(problem) -> N.Options:
    o = N.Options()
    N.check(problem._lib.tv_get_options(problem._ctx, C.byref(o)), problem._ctx)
    return o


class KrylovSolver:
    """``problem.ksp`` (ThermoViscoProblem.py:339-346): CG with the context's
    preconditioner; the petsc4py KSP calls a caller of the reference makes."""

    def __init__(self, problem):
        self._p = problem

    def getType(self) -> str:
        return "cg"  # ThermoViscoProblem.py:343

    def getPC(self):
        return _PC(self._p)

    def getOptionsPrefix(self) -> str:
        return "nls_solve_"  # dolfinx NewtonSolver's KSP prefix

    def setFromOptions(self) -> None:
        pass  # the options database is not read: the context's options are the configuration

    def getTolerances(self):
        o = _options(self._p)
        return o.ksp_rtol, o.ksp_atol, o.ksp_dtol, o.ksp_max_it

    def setTolerances(self, rtol=None, atol=None, divtol=None, max_it=None) -> None:
        """petsc4py KSP.setTolerances: an argument left None keeps its value."""
        r, a, d, m = self.getTolerances()
        p = self._p
        N.check(p._lib.tv_set_ksp_tolerances(p._ctx, float(r if rtol is None else rtol),
                                             float(a if atol is None else atol),
                                             float(d if divtol is None else divtol),
                                             int(m if max_it is None else max_it)), p._ctx)

    rtol = property(lambda self: self.getTolerances()[0], lambda self, v: self.setTolerances(rtol=v))
    atol = property(lambda self: self.getTolerances()[1], lambda self, v: self.setTolerances(atol=v))
    divtol = property(lambda self: self.getTolerances()[2], lambda self, v: self.setTolerances(divtol=v))
    max_it = property(lambda self: self.getTolerances()[3], lambda self, v: self.setTolerances(max_it=v))


class _PC:
    def __init__(self, problem):
        self._p = problem

    def getType(self) -> str:
        # the reference asks for "gamg" (ThermoViscoProblem.py:344); the context
        # runs point Jacobi, the box multigrid or the algebraic multigrid
        return {"jacobi": "jacobi", "gmg": "mg", "amg": "gamg"}[self._p.preconditioner]


class NewtonSolver:
    """``problem.solver`` (ThermoViscoProblem.py:334-337)."""

    def __init__(self, problem):
        self._p = problem
        self.report = True  # :337; the step's counts are in problem.last_newton_iterations
        self.krylov_solver = KrylovSolver(problem)

    @property
    def convergence_criterion(self) -> str:
        return "incremental"  # :335

    @convergence_criterion.setter
    def convergence_criterion(self, v: str) -> None:
        if v != "incremental":
            raise NotImplementedError("libtvfem's Newton test is the incremental criterion "
                                      "(ThermoViscoProblem.py:335)")

    def _get(self):
        o = _options(self._p)
        return o.newton_rtol, o.newton_atol, o.newton_max_it, o.error_on_nonconvergence

    def _set(self, i, v):
        t = list(self._get())
        t[i] = v
        p = self._p
        N.check(p._lib.tv_set_newton_tolerances(p._ctx, float(t[0]), float(t[1]), int(t[2]), int(bool(t[3]))),
                p._ctx)

    rtol = property(lambda self: self._get()[0], lambda self, v: self._set(0, v))
    atol = property(lambda self: self._get()[1], lambda self, v: self._set(1, v))
    max_it = property(lambda self: self._get()[2], lambda self, v: self._set(2, v))
    error_on_nonconvergence = property(lambda self: bool(self._get()[3]), lambda self, v: self._set(3, v))

    def solve(self, u=None):
        """dolfinx NewtonSolver.solve(u) -> (iterations, converged), on the
        problem's own temperature (``u``, when given, must be
        functions_current["T"], the only unknown the reference solves for).
        Raises RuntimeError when it does not converge and
        error_on_nonconvergence is set, as dolfinx does."""
        p = self._p
        if u is not None and u is not p.functions_current["T"]:
            raise ValueError("NewtonSolver.solve: the unknown is functions_current['T']")
        p._flush()
        nits, kits, conv = C.c_int(), C.c_int(), C.c_int()
        rc = p._lib.tv_solve_T(p._ctx, C.byref(nits), C.byref(kits), C.byref(conv))
        p._device_version += 1
        if rc == N.TV_ERR_NOT_CONVERGED:
            raise RuntimeError(p._lib.tv_last_error(p._ctx).decode())
        N.check(rc, p._ctx)
        p.last_newton_iterations = nits.value
        p.last_krylov_iterations = kits.value
        return nits.value, bool(conv.value)
