"""Drop-in module name of the reference driver (ThermoViscoProblem.py).

``from ThermoViscoProblem import ThermoViscoProblem`` works exactly as in the
reference's main.py; the implementation is tvfem.problem (MI355X C-ABI host side).
"""
from tvfem.problem import Function, ThermoViscoProblem  # noqa: F401

__all__ = ["ThermoViscoProblem", "Function"]
