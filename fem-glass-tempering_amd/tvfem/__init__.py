"""tvfem — MI355X-native (gfx950) hot path of pzimbrod/fem-glass-tempering.

Host side of the thermo-viscoelastic time step: Python mirrors of the
reference's ``ThermoViscoProblem`` / ``ThermalModel`` / ``ViscoelasticModel``
over the C-ABI library ``libtvfem.so`` (hand-written HIP kernels for gfx950,
RCCL over xGMI).  There is no CPU fallback: importing works anywhere, but
creating a problem requires the built library and an MI355X GPU.
"""
from .mesh import RectilinearMesh, UnstructuredMesh, box_mesh, distorted_box_mesh, interval_mesh, read_msh  # noqa: F401
from ._native import lib_path, load_library, NativeError  # noqa: F401

__all__ = ["RectilinearMesh", "UnstructuredMesh", "box_mesh", "distorted_box_mesh", "interval_mesh", "read_msh", "lib_path", "load_library",
           "NativeError"]
