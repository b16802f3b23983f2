"""Entry script with the reference's surface (main.py:1-62): the same
``jit_options``, time domain, ``fe_config`` and ``model_params`` dicts, then
ThermoViscoProblem(...).setup() / .solve() on the MI355X path.

Run from this directory:  python main.py
"""
import os

from geometry import create_mesh
from ThermoViscoProblem import ThermoViscoProblem

# accepted and ignored: nothing is JIT-compiled on this path (main.py:6-8)
jit_options = {
    "cffi_extra_compile_args": ["-O3", "-march=native"]
}

# Time domain
t_start = 0.0
t_end = 50.0
time = (0.0, 50.0)

dt = 0.1
t = t_start

mesh_path = "mesh1d.msh"
create_new_mesh = not os.path.exists(mesh_path)

if create_new_mesh:
    create_mesh(path=mesh_path)

fe_config = {
    "T":        {"element": "DG", "degree": 1},
    "sigma":    {"element": "CG", "degree": 1},
}

model_params = {
    "f": 0.0,
    "epsilon": 0.93,
    "sigma": 5.670e-8,
    "T_ambient": 600.0,
    "T_0": 800.0,
    "alpha": 1.0,
    "htc": 280.1,
    "rho": 2500.0,
    "cp": 1433.0,
    "k": 1.0,
    "H": 627.8e3,
    "Tb": 869.0e0,
    "Rg": 8.314,
    "alpha_solid": 9.10e-6,
    "alpha_liquid": 25.10e-6,
    "Tf_init": 873.0,
}

if __name__ == "__main__":
    model = ThermoViscoProblem(mesh_path=mesh_path, config=fe_config,
                               time=time, dt=dt, model_parameters=model_params,
                               jit_options=jit_options)
    model.setup(dirichlet_bc=False)
    model.solve()
