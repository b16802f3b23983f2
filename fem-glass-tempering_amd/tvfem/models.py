"""Material and thermal model constants (host side).

``ThermalModel`` mirrors ThermalModel.py:6-29 and ``ViscoelasticModel`` mirrors
ViscoelasticModel.py:9-242 of the reference.  In the reference these hold
dolfinx ``Constant`` objects and 17 JIT-compiled UFL ``Expression``s; here they
hold plain floats / numpy tableaux that are passed to the device once, and the
17 expressions are one fused HIP kernel (csrc/tv_visco.hip).
"""
from __future__ import annotations

from math import factorial

import numpy as np

# ViscoelasticModel.py:19-68
M_N = [5.523e-2, 8.205e-2, 1.215e-1, 2.286e-1, 2.860e-1, 2.265e-1]
LAMBDA_M = [5.965e-4, 1.077e-2, 1.362e-1, 1.505e-1, 6.747e+0, 2.963e+1]
G_N = [1.585, 2.354, 3.486, 6.558, 8.205, 6.498]
LAMBDA_G = [6.658e-5, 1.197e-3, 1.514e-2, 1.672e-1, 7.497e-1, 3.292e+0]
K_N = [7.588e-1, 7.650e-1, 9.806e-1, 7.301e+0, 1.347e+1, 1.090e+1]
LAMBDA_K = [5.009e-5, 9.945e-4, 2.022e-3, 1.925e-2, 1.199e-1, 2.033e+0]

# The 17 interpolation passes of one step, in the reference's call order
# (ThermoViscoProblem.py:455-591); all of them run inside the fused kernel.
EXPRESSIONS = [
    "phi", "Tf_partial", "Tf", "thermal_strain", "total_strain", "deviatoric_strain", "T_next", "phi",
    "phi_next", "xi", "ds_partial", "s_tilde_partial_next", "s_partial_next", "dsigma_partial",
    "sigma_tilde_partial_next", "sigma_partial_next", "sigma_next",
]


class ThermalModel:
    """Heat-equation coefficients (ThermalModel.py:7-29).  rho, cp and k are
    stored and unused, as in the reference."""

    def __init__(self, mesh, model_parameters: dict) -> None:
        self.f = float(model_parameters["f"])
        self.epsilon = float(model_parameters["epsilon"])
        self.sigma = float(model_parameters["sigma"])
        self.alpha = float(model_parameters["alpha"])
        self.htc = float(model_parameters["htc"])
        self.rho = float(model_parameters["rho"])
        self.cp = float(model_parameters["cp"])
        self.k = float(model_parameters["k"])
        self.T_ambient = float(model_parameters["T_ambient"])


class FusedExpression:
    """Placeholder for one of the reference's dolfinx ``Expression`` objects:
    records which stage of the fused device kernel computes it."""

    def __init__(self, name, stage):
        self.name = name
        self.stage = stage

    def __repr__(self):
        return f"FusedExpression({self.name!r}, stage={self.stage})"


class ViscoelasticModel:
    """Narayanaswamy / Prony viscoelastic model constants (ViscoelasticModel.py:10-84)."""

    def __init__(self, mesh, model_parameters: dict) -> None:
        self.chi = 0.5
        self.tableau_size = 6
        self.dim = mesh.dim
        self.m_n_tableau = np.array(M_N)
        self.lambda_m_n_tableau = np.array(LAMBDA_M)
        self.g_n_tableau = np.array(G_N)
        self.lambda_g_n_tableau = np.array(LAMBDA_G)
        self.k_n_tableau = np.array(K_N)
        self.lambda_k_n_tableau = np.array(LAMBDA_K)
        self.I = np.eye(self.dim)
        self.T_init = float(model_parameters["T_0"])
        self.H = float(model_parameters["H"])
        self.Rg = float(model_parameters["Rg"])
        self.Tb = float(model_parameters["Tb"])
        self.alpha_solid = float(model_parameters["alpha_solid"])
        self.alpha_liquid = float(model_parameters["alpha_liquid"])
        self.expressions = {}

    def _init_expressions(self, functions=None, functions_next=None, functions_current=None,
                          functions_previous=None, functionSpaces=None, dt=None) -> None:
        """ViscoelasticModel._init_expressions (ViscoelasticModel.py:86-230).

        Nothing is JIT-compiled: the 17 expressions are the stages of the fused
        per-dof kernel.  The dict is kept for introspection (same keys)."""
        self.expressions = {name: FusedExpression(name, k) for k, name in enumerate(EXPRESSIONS)}

    def _taylor_exponential(self, xi, lambda_value):
        """ViscoelasticModel._taylor_exponential (ViscoelasticModel.py:233-242) on numpy data."""
        xi = np.asarray(xi, dtype=np.float64)
        terms = [1.0 / factorial(k) * (-xi / lambda_value) ** k for k in range(0, 3)]
        return (terms[0] + terms[1]) + terms[2]
