"""Drop-in module name of the reference's ViscoelasticModel.py (constants; the
17 expressions are the fused HIP kernel csrc/tv_visco.hip)."""
from tvfem.models import ViscoelasticModel  # noqa: F401

__all__ = ["ViscoelasticModel"]
