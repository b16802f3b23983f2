"""CPU ORACLE port (test infrastructure): ctypes wrapper of oracle/tv_cpu.c, the
C/OpenMP restatement of the reference time step timed as bench.py's
cpu_baseline ("kind": "port").  Never imported by the product path."""
import ctypes as C
import os
import subprocess
import time

import numpy as np

from . import tv_oracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libtvcpu.so")
_lib = None


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            subprocess.run(["make", "-C", HERE], check=True, capture_output=True)
        lib = C.CDLL(LIB)
        dp = C.POINTER(C.c_double)
        lib.tvcpu_create.restype = C.c_void_p
        lib.tvcpu_create.argtypes = [C.POINTER(C.c_int), dp, dp, dp, dp, dp]
        lib.tvcpu_create_dg.restype = C.c_void_p
        lib.tvcpu_create_dg.argtypes = [C.POINTER(C.c_int), dp, dp, dp, dp, dp]
        lib.tvcpu_step.argtypes = [C.c_void_p, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int)]
        lib.tvcpu_num_dofs.restype = C.c_longlong
        lib.tvcpu_num_dofs.argtypes = [C.c_void_p]
        lib.tvcpu_get.argtypes = [C.c_void_p, C.c_int, dp]
        lib.tvcpu_destroy.argtypes = [C.c_void_p]
        lib.tvcpu_set_gmg.argtypes = [C.c_void_p]
        lib.tvcpu_set_gmg.restype = C.c_int
        lib.tvcpu_precond_apply.argtypes = [C.c_void_p, dp, dp]
        _lib = lib
    return _lib


class CpuProblem:
    """Structured 3D plate on the CPU (axes: node coordinates per axis), CG1/CG1
    or (family "DG") DG1/DG1 with cell-local dofs at l * ncell + cell."""

    def __init__(self, axes, mp, dt, family="CG", pc="jacobi"):
        lib = load()
        self.axes = [np.ascontiguousarray(a, dtype=np.float64) for a in axes]
        nc = (C.c_int * 3)(*[len(a) - 1 for a in self.axes])
        params = np.array([mp["f"], mp["epsilon"], mp["sigma"], mp["T_ambient"], mp["T_0"], mp["alpha"],
                           mp["htc"], mp["H"], mp["Tb"], mp["Rg"], mp["alpha_solid"], mp["alpha_liquid"], dt])
        tabs = np.concatenate([O.PRONY[k] for k in ("m_n", "lambda_m", "g_n", "lambda_g", "k_n", "lambda_k")])
        dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
        self._keep = (params, tabs)
        create = lib.tvcpu_create_dg if family == "DG" else lib.tvcpu_create
        self.h = create(nc, dp(self.axes[0]), dp(self.axes[1]), dp(self.axes[2]), dp(params), dp(tabs))
        self.n = lib.tvcpu_num_dofs(self.h)
        self.lib = lib
        self.levels = 1
        if pc == "gmg":  # the GPU line's geometric multigrid (tv_cpu.c tvcpu_set_gmg)
            self.levels = lib.tvcpu_set_gmg(self.h)
            if self.levels < 1:
                raise ValueError("GMG: CG1 plates only in the CPU port")

    def precond_apply(self, r):
        """z = B r at the current T (Jacobi or one V-cycle)."""
        r = np.ascontiguousarray(r, dtype=np.float64)
        z = np.empty_like(r)
        dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))  # noqa: E731
        self.lib.tvcpu_precond_apply(self.h, dp(r), dp(z))
        return z

    def step(self, thermal_only=False):
        a, b = C.c_int(), C.c_int()
        rc = self.lib.tvcpu_step(self.h, 1 if thermal_only else 0, C.byref(a), C.byref(b))
        if rc:
            raise RuntimeError(f"CPU port step failed ({rc})")
        return a.value, b.value

    def get(self, which):
        n = self.n * (9 if which == "sigma" else 1)
        out = np.empty(n)
        idx = {"T": 0, "phi": 1, "xi": 2, "Tf": 3, "sigma": 4}[which]
        self.lib.tvcpu_get(self.h, idx, out.ctypes.data_as(C.POINTER(C.c_double)))
        return out

    def close(self):
        if self.h:
            self.lib.tvcpu_destroy(self.h)
            self.h = None


def cores():
    try:
        return len(os.sched_getaffinity(0))
    except Exception:
        return os.cpu_count() or 1


def time_baseline(nc, L, mp, seconds=15.0, thermal_only=False, family="CG", pc="jacobi"):
    """Bounded sample of the bench workload: the full mesh, as many whole time
    steps as fit about `seconds` (at least one, at most 10), with the GPU
    line's preconditioner where the port has it (GMG: CG1).  Returns the
    cpu_baseline record of bench.py."""
    axes = [np.linspace(0.0, l, n + 1) for l, n in zip(L, nc)]
    pc = pc if family == "CG" else "jacobi"
    P = CpuProblem(axes, mp, 0.1, family, pc=pc)
    t0 = time.perf_counter()
    steps = 0
    while True:
        P.step(thermal_only)
        steps += 1
        el = time.perf_counter() - t0
        if el >= seconds or steps >= 10 or el / steps * (steps + 1) > 2 * seconds:
            break
    n = P.n
    P_levels = P.levels
    P.close()
    return {"value": n * steps / el, "unit": "DOF-updates/s", "cores": int(os.environ.get("OMP_NUM_THREADS", cores())),
            "kind": "port",
            "sample": f"{steps} full time step(s) of the same {nc[0]}x{nc[1]}x{nc[2]} hex mesh "
                      f"({n} dofs, {'thermal-only' if thermal_only else 'coupled'}) in {el:.1f} s, "
                      f"oracle/tv_cpu.c (C/OpenMP port, {family}1: matrix-free "
                      + (f"GMG-preconditioned ({P_levels} levels) " if pc == "gmg" else "Jacobi-") + "PCG Newton "
                      "+ visco update)", "algorithm": "gmg" if pc == "gmg" else "jacobi"}
