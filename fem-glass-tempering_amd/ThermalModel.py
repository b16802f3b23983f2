"""Drop-in module name of the reference's ThermalModel.py (constants only)."""
from tvfem.models import ThermalModel  # noqa: F401

__all__ = ["ThermalModel"]
