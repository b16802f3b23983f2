"""A/B bit-equality helper: run a few coupled steps on a small box with the
library TVFEM_LIB selects (or the in-tree one) and save T and sigma, so two
library builds can be compared bit for bit (tools/_r7e.sh).  GPU only.
    python tools/bitcmp_step.py OUT.npz [jacobi|gmg]"""
import sys

import numpy as np

sys.path.insert(0, "fem-glass-tempering_amd")
from tvfem import RectilinearMesh  # noqa: E402
from tvfem.problem import ThermoViscoProblem  # noqa: E402

out, pc = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "gmg")
CG = {"element": "CG", "degree": 1}
MP = {  # main.py:29-55, as in bench.py
    "f": 0.0, "epsilon": 0.93, "sigma": 5.670e-8, "T_ambient": 600.0, "T_0": 800.0, "alpha": 1.0,
    "htc": 280.1, "rho": 2500.0, "cp": 1433.0, "k": 1.0, "H": 627.8e3, "Tb": 869.0e0, "Rg": 8.314,
    "alpha_solid": 9.10e-6, "alpha_liquid": 25.10e-6, "Tf_init": 873.0,
}
axes = [np.linspace(0.0, 8.0, 65), np.linspace(0.0, 6.0, 49), np.linspace(0.0, 1.0, 9)]
p = ThermoViscoProblem(RectilinearMesh(axes), (0.0, 1.0), 0.1, {"T": CG, "sigma": CG}, dict(MP),
                       verbose=False, preconditioner=pc)
p.setup()
its = []
for _ in range(3):
    p.solve_timestep()
    its.append((p.last_newton_iterations, p.last_krylov_iterations))
np.savez(out, T=p.functions_current["T"].x.array.copy(), sigma=p.functions_next["sigma"].x.array.copy(),
         its=np.array(its))
p.close()
print(out, its)
