"""Drive the hot-path kernels for a rocprofv3 --pmc pass.

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- \
        python3 tools/pmc_kernels.py [--cells 400,400,50] [--family CG|DG] [--mesh box|distorted] [--reps 5]

One coupled step (realistic state), then `reps` whole PCG iterations (CG: fused
matvec + update alternating as in the solve, tv_time_kernel id 5; DG: the
fused DG matvec, id 3), `reps` viscoelastic updates (id 1) and `reps` plain
J x launches with the Infinity Cache flushed before each (id 10), so the
counters see the kernels in the cache state of the solve.  ``--mesh
distorted``: the plate as a general hexahedral mesh (tv_um.hip), plain J x
(id 0) and the visco update.
"""
import argparse
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "fem-glass-tempering_amd"), ROOT]

from tvfem import _native as N, box_mesh, distorted_box_mesh  # noqa: E402
from tvfem.problem import ThermoViscoProblem  # noqa: E402

MP = {"f": 0.0, "epsilon": 0.93, "sigma": 5.670e-8, "T_ambient": 600.0, "T_0": 800.0, "alpha": 1.0,
      "htc": 280.1, "rho": 2500.0, "cp": 1433.0, "k": 1.0, "H": 627.8e3, "Tb": 869.0, "Rg": 8.314,
      "alpha_solid": 9.10e-6, "alpha_liquid": 25.10e-6, "Tf_init": 873.0}  # main.py:29-55

ap = argparse.ArgumentParser()
ap.add_argument("--cells", default="400,400,50")
ap.add_argument("--reps", type=int, default=5)
ap.add_argument("--family", choices=["CG", "DG"], default="CG")
ap.add_argument("--mesh", choices=["box", "distorted"], default="box")
ap.add_argument("--pc", choices=["jacobi", "gmg"], default="jacobi",
                help="gmg: the bench line's solver -- whole coupled steps under the counters (the fused "
                     "matvec and every V-cycle kernel in the cache state of the multigrid solve)")
ap.add_argument("--steps", type=int, default=2)
ap.add_argument("--jx-only", action="store_true",
                help="only `reps` plain J x launches with the Infinity Cache flushed (tv_time_kernel 10): the fine-grid "
                     "J x record (with --pc gmg at C4 the V-cycle no longer runs a fine J x: the fused restriction)")
a = ap.parse_args()
nc = [int(v) for v in a.cells.split(",")]
cfg = {"T": {"element": a.family, "degree": 1}, "sigma": {"element": a.family, "degree": 1}}
um = a.mesh == "distorted"
mesh = (distorted_box_mesh if um else box_mesh)([50.0, 50.0, 5.0], nc)
prob = ThermoViscoProblem(mesh, (0.0, 1.0), 0.1, cfg, dict(MP), materialize=False, write_output=False,
                          verbose=False, preconditioner=a.pc, **({} if um else {"part_axis": 1}))
prob.setup()
prob.solve_timestep()
lib, ctx = prob._lib, prob._ctx
if a.jx_only:
    ms = C.c_double()
    N.check(lib.tv_time_kernel(ctx, 10, a.reps, C.byref(ms)), ctx)
    print(10, ms.value, flush=True)
    prob.close()
    sys.exit(0)
if a.pc == "gmg":  # whole steps of the bench's solve and nothing else (the
    # V-cycle aggregate of pmc_summarize.py counts every level-0 J x launch)
    for _ in range(a.steps):
        prob.solve_timestep()
        print("step", prob.last_newton_iterations, prob.last_krylov_iterations, flush=True)
    prob.close()
    sys.exit(0)
for kid in ((0, 1) if um else (5, 1, 10) if a.family == "CG" else (3, 1, 10)):
    ms = C.c_double()
    N.check(lib.tv_time_kernel(ctx, kid, a.reps, C.byref(ms)), ctx)
    print(kid, ms.value, flush=True)
prob.close()
