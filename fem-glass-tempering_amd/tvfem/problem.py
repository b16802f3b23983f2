"""``ThermoViscoProblem`` — drop-in host mirror of the reference driver
(ThermoViscoProblem.py:23-620) over the MI355X C-ABI library.

Same constructor arguments and meaning (``mesh_path, time, dt, config,
model_parameters, jit_options``), same ``setup`` / ``solve`` /
``solve_timestep`` methods and the same state dictionaries ``functions``,
``functions_current``, ``functions_previous``, ``functions_next`` whose values
expose ``.x.array`` in the reference's interleaved blocked layout
(``x.array[dof*bs + comp]``).  The FEniCSx stack underneath (UFL forms, FFCx
kernels, dolfinx assemblers, PETSc Newton/KSP) is replaced by libtvfem.so.

Differences that are part of the contract:
  * ``mesh_path`` may be a ``.msh`` file (1D line mesh, as the reference) or a
    ``RectilinearMesh`` (structured 1D / 2D / 3D grids);
  * the linear solver is matrix-free Jacobi-PCG (reference: CG + GAMG); T and
    sigma agree with the CPU restatement within the tolerances stated in
    tests/;
  * file output (:246-276, VTX / XDMF there) is XDMF over raw binary here,
    written by default as the reference does (T, phi, Tf, xi and sigma every
    step into ``output_dir`` = "output"); ``write_output=False`` opts out
    (the benchmark, tests).
"""
from __future__ import annotations

import ctypes as C
import time as _time
from math import ceil

import numpy as np

try:
    import xxhash as _xxhash
except Exception:  # pragma: no cover
    _xxhash = None

from . import _native as N
from .mesh import RectilinearMesh, UnstructuredMesh, read_msh
from .models import ThermalModel, ViscoelasticModel

_FAMILIES = {"CG": N.TV_CG, "DG": N.TV_DG}


def _digest(a: np.ndarray):
    if _xxhash is not None:
        return _xxhash.xxh3_64_intdigest(memoryview(np.ascontiguousarray(a)).cast("B"))
    return hash(a.tobytes())


class FunctionSpaceInfo:
    def __init__(self, problem, space, family, degree, bs):
        self._p = problem
        self.space = space
        self.family = family
        self.degree = degree
        self.bs = bs

    def tabulate_dof_coordinates(self):
        return self._p._dof_coordinates(self.space)


class _Vector:
    def __init__(self, fn):
        self._fn = fn

    @property
    def array(self):
        return self._fn._problem._host_array(self._fn.field)

    def scatter_forward(self):
        """Ghost values live on the device and are exchanged there (RCCL)."""
        return None


class Function:
    """Proxy of one device-resident field (a dolfinx ``Function`` of the reference)."""

    def __init__(self, problem, field, space: FunctionSpaceInfo, name=None):
        self._problem = problem
        self.field = field
        self.function_space = space
        self.name = name or field
        self.x = _Vector(self)

    def interpolate(self, f):
        """Interpolate a Python callable ``f(x) -> values`` (x of shape (3, n)) at the dofs."""
        if not callable(f):
            raise TypeError("only Python callables can be interpolated into device fields")
        X = self.function_space.tabulate_dof_coordinates()
        vals = np.asarray(f(X.T), dtype=np.float64)
        bs = self._problem._bs[self.field]
        if bs == 1:
            vals = vals.reshape(-1)
        else:
            vals = vals.reshape(bs, -1).T.reshape(-1)
        arr = self.x.array
        arr[:] = vals

    def __repr__(self):
        return f"Function({self.name!r})"


class ThermoViscoProblem:
    # setup() opens the output writers unless write_output=False is passed: the
    # reference always writes (ThermoViscoProblem.py:182, 246-276, 374).
    # tests/conftest.py turns the default off for the test session.
    WRITE_OUTPUT_DEFAULT = True

    def __init__(self, mesh_path, time: tuple, dt: float, config: dict, model_parameters: dict,
                 jit_options: dict | None = None, *, device: int = 0, materialize: bool = True,
                 ksp_rtol: float = 1e-5, n_parts: int = 1, part: int = 0, part_axis: int = -1,
                 verbose: bool = True, pcg_variant: str = "auto", model_mode: str = "reference",
                 write_output: bool | None = None, output_dir: str = "output", preconditioner: str = "jacobi",
                 mg_levels: int = 0, dg_kernel: str = "auto", dg_tile_chunk: int = 0,
                 mg_replicate_nodes: int = 0, ksp_fixed_its: int = 0, newton_fixed_its: int = 0,
                 cell_parts=None, mg_coupling: str = "auto", ksp_max_it: int = 10000) -> None:
        if isinstance(mesh_path, (RectilinearMesh, UnstructuredMesh)):
            self.mesh = mesh_path
        elif isinstance(mesh_path, str):
            self.mesh = read_msh(mesh_path)
        else:
            raise TypeError("mesh_path must be a .msh path, a tvfem.RectilinearMesh or a tvfem.UnstructuredMesh")
        self.dim = self.mesh.dim
        self.dt = dt
        self.time = time
        self.t = self.time[0]
        self.n_steps = ceil((self.time[1] - self.time[0]) / self.dt)
        self.verbose = verbose
        self.material_model = ViscoelasticModel(mesh=self.mesh, model_parameters=model_parameters)
        self.physical_model = ThermalModel(mesh=self.mesh, model_parameters=model_parameters)
        self._ctx = None
        self._cache = {}
        self._device_version = 0
        self.last_newton_iterations = 0
        self.last_krylov_iterations = 0
        self.__init_function_spaces(config=config)
        if model_mode not in ("reference", "paper"):
            raise ValueError("model_mode must be 'reference' (the reference as it runs) or 'paper'")
        self.model_mode = model_mode
        self.write_output = self.WRITE_OUTPUT_DEFAULT if write_output is None else bool(write_output)
        self.output_dir = output_dir
        self._output_open = False
        if preconditioner not in ("jacobi", "gmg", "amg"):
            raise ValueError("preconditioner must be 'jacobi' (PETSc PCJACOBI, the oracle's), 'gmg' (geometric "
                             "multigrid on the box hierarchy) or 'amg' (smoothed aggregation, unstructured meshes)")
        self.preconditioner = preconditioner
        self._mg_levels = int(mg_levels)
        if dg_kernel not in ("auto", "tile", "cells"):
            raise ValueError("dg_kernel must be 'auto' (= 'tile', the marching tile kernel) or 'cells' "
                             "(one thread per cell, the reference evaluation)")
        self._dg_kernel = {"auto": N.TV_DG_KERNEL_AUTO, "tile": N.TV_DG_KERNEL_TILE,
                           "cells": N.TV_DG_KERNEL_CELLS}[dg_kernel]
        self._dg_tile_chunk = int(dg_tile_chunk)
        self._mg_replicate_nodes = int(mg_replicate_nodes)
        if mg_coupling not in ("auto", "global", "local"):
            raise ValueError("mg_coupling must be 'auto', 'global' (the distributed V-cycle of the whole box) or "
                             "'local' (block Jacobi: each partition's own V-cycle)")
        self._mg_coupling = {"auto": N.TV_MG_COUPLING_AUTO, "global": N.TV_MG_COUPLING_GLOBAL,
                             "local": N.TV_MG_COUPLING_LOCAL}[mg_coupling]
        self._ksp_fixed_its = int(ksp_fixed_its)
        self._ksp_max_it = int(ksp_max_it)  # PETSc KSP max_it (default 10000)
        self._newton_fixed_its = int(newton_fixed_its)
        # partitioned unstructured mesh: cell -> part ids (default: tv_partition_rcb)
        self._cell_parts = None if cell_parts is None else np.asarray(cell_parts)
        self.__init_native(model_parameters, device, materialize, ksp_rtol, n_parts, part, part_axis, pcg_variant)
        self.__init_functions()
        self.material_model._init_expressions(functionSpaces=self.functionSpaces, functions=self.functions,
                                              functions_current=self.functions_current,
                                              functions_previous=self.functions_previous,
                                              functions_next=self.functions_next, dt=self.dt)
        self.jit_options = jit_options

    # ---------------------------------------------------------------------------------
    def __init_function_spaces(self, config: dict) -> None:
        # Only CG and DG are supported (ThermoViscoProblem.py:70-71)
        assert all(var["element"] in ["CG", "DG"] for var in config.values()), \
            "Only CG and DG elements are supported"
        for key in ("T", "sigma"):
            if config[key]["degree"] != 1:
                raise NotImplementedError("libtvfem implements degree-1 Lagrange spaces")
        self.config = config
        d = self.dim
        self._fam = {"T": config["T"]["element"], "sigma": config["sigma"]["element"]}
        self.functionSpaces = {
            "T": FunctionSpaceInfo(self, 0, config["T"]["element"], 1, 1),
            "Tf_partial": FunctionSpaceInfo(self, 0, config["T"]["element"], 1, 6),
            "sigma": FunctionSpaceInfo(self, 1, config["sigma"]["element"], 1, d * d),
            "sigma_partial": FunctionSpaceInfo(self, 1, config["sigma"]["element"], 1, 6 * d * d),
        }

    def __init_native(self, mp, device, materialize, ksp_rtol, n_parts, part, part_axis, pcg_variant):
        lib = N.load_library()
        self._lib = lib
        um = isinstance(self.mesh, UnstructuredMesh)
        if um:
            # general quadrilateral / hexahedral cells: element-local kernels
            # (csrc/tv_um.hip), CG1 spaces; partitioned: recursive coordinate
            # bisection of the cells + a ghost layer (tvfem.parallel.ghosted_partition,
            # the mesh distribution of gmshio.read_from_msh at ThermoViscoProblem.py:27-28)
            if self._fam["T"] != "CG" or self._fam["sigma"] != "CG":
                raise NotImplementedError("unstructured meshes: CG temperature and stress spaces")
            local = self.mesh
            self._upart = None
            if n_parts > 1:
                from .parallel import ghosted_partition, rcb_partition
                cp = rcb_partition(self.mesh, n_parts) if self._cell_parts is None else self._cell_parts
                self._upart = ghosted_partition(self.mesh, cp, part, n_parts)
                local = self._upart["mesh"]
            desc = N.UMeshDesc()
            desc.dim = self.dim
            xyz = np.zeros((local.num_vertices, 3))
            xyz[:, :self.dim] = local.x[:, :self.dim]
            cells = np.ascontiguousarray(local.cells, dtype=np.int64)
            self._coord_bufs = [xyz, cells]
            desc.n_vertices = xyz.shape[0]
            desc.coords = xyz.ctypes.data_as(C.POINTER(C.c_double))
            desc.n_cells = cells.shape[0]
            desc.cells = cells.ctypes.data_as(C.POINTER(C.c_int64))
        else:
            desc = N.MeshDesc()
            desc.dim = self.dim
            self._coord_bufs = []
            for a in range(3):
                if a < self.dim:
                    buf = np.ascontiguousarray(self.mesh.axes[a])
                    self._coord_bufs.append(buf)
                    desc.n_cells[a] = len(buf) - 1
                    desc.coords[a] = buf.ctypes.data_as(C.POINTER(C.c_double))
                else:
                    desc.n_cells[a] = 0
            desc.part_axis = part_axis
            desc.n_parts = n_parts
            desc.part = part
        self._n_parts, self._part = n_parts, part
        fe = N.FeConfig(_FAMILIES[self._fam["T"]], 1, _FAMILIES[self._fam["sigma"]], 1)
        params = N.default_params(mp, self.dt)
        opts = N.default_options()
        opts.materialize = 1 if materialize else 0
        opts.ksp_rtol = ksp_rtol
        opts.pcg_variant = {"auto": N.TV_PCG_AUTO, "kspcg": N.TV_PCG_KSPCG,
                            "single": N.TV_PCG_SINGLE_REDUCTION}[pcg_variant]
        opts.model_mode = N.TV_MODEL_PAPER if self.model_mode == "paper" else N.TV_MODEL_REFERENCE
        opts.preconditioner = {"jacobi": N.TV_PC_JACOBI, "gmg": N.TV_PC_GMG, "amg": N.TV_PC_AMG}[self.preconditioner]
        opts.mg_levels = self._mg_levels
        opts.dg_kernel = self._dg_kernel
        opts.dg_tile_chunk = self._dg_tile_chunk
        opts.mg_replicate_nodes = self._mg_replicate_nodes
        opts.ksp_fixed_its = self._ksp_fixed_its
        opts.ksp_max_it = self._ksp_max_it
        opts.mg_coupling = self._mg_coupling
        if self._newton_fixed_its > 0:  # timing runs only: exactly this many Newton iterations per step
            opts.newton_rtol = 0.0
            opts.newton_atol = 0.0
            opts.newton_max_it = self._newton_fixed_its
            opts.error_on_nonconvergence = 0
        ctx = C.c_void_p()
        if um and self._upart is not None:
            from .parallel import upart_desc
            pdesc, pbufs = upart_desc(self._upart)
            self._coord_bufs.append(pbufs)
            N.check(lib.tv_create_unstructured_part(C.byref(desc), C.byref(pdesc), C.byref(fe), C.byref(params),
                                                    C.byref(opts), device, C.byref(ctx)))
        else:
            create = lib.tv_create_unstructured if um else lib.tv_create
            N.check(create(C.byref(desc), C.byref(fe), C.byref(params), C.byref(opts), device, C.byref(ctx)))
        self._ctx = ctx
        self.materialize = materialize
        self._bs = {}
        for name, fid in N.FIELD_ID.items():
            bs = C.c_int()
            N.check(lib.tv_field_block_size(ctx, fid, C.byref(bs)), ctx)
            self._bs[name] = bs.value

    def __init_functions(self) -> None:
        S = self.functionSpaces
        mk = lambda field, sp, name=None: Function(self, field, S[sp], name)  # noqa: E731
        self.functions_previous = {"T": mk("T_prev", "T"), "Tf_partial": mk("Tf_partial_prev", "Tf_partial"),
                                   "Tf": mk("Tf_prev", "T")}
        self.functions_current = {
            "T": mk("T", "T", "Temperature"), "Tf_partial": mk("Tf_partial", "Tf_partial", "Fictive_temperature"),
            "Tf": mk("Tf", "T", "Fictive_Temperature"),
            "s_tilde_partial": mk("s_tilde_partial", "sigma_partial"),
            "sigma_tilde_partial": mk("sigma_tilde_partial", "sigma_partial"),
            "s_partial": mk("s_partial", "sigma_partial"), "sigma_partial": mk("sigma_partial", "sigma_partial"),
        }
        self.functions_next = {
            "T": mk("T_next", "T"), "phi": mk("phi_next", "T"),
            "s_tilde_partial": mk("s_tilde_partial_next", "sigma_partial"),
            "sigma_tilde_partial": mk("sigma_tilde_partial_next", "sigma_partial"),
            "s_partial": mk("s_partial_next", "sigma_partial"),
            "sigma_partial": mk("sigma_partial_next", "sigma_partial"),
            "sigma": mk("sigma", "sigma", "Stress_tensor"),
        }
        self.functions = {
            "phi": mk("phi", "T"), "xi": mk("xi", "T", "Shifted_time"),
            "thermal_strain": mk("thermal_strain", "sigma"), "total_strain": mk("total_strain", "sigma"),
            "deviatoric_strain": mk("deviatoric_strain", "sigma"),
            "ds_partial": mk("ds_partial", "sigma_partial", "Deviatoric_stress_increment"),
            "dsigma_partial": mk("dsigma_partial", "sigma_partial", "Hydrostatic_stress_increment"),
        }

    # ---- host mirrors of device fields -------------------------------------------------
    @property
    def pcg_variant(self) -> str:
        """Krylov form in use: "kspcg" (PETSc KSPSolve_CG as written, two
        reductions per iteration) or "single" (Chronopoulos-Gear, one)."""
        v = C.c_int()
        N.check(self._lib.tv_pcg_variant(self._ctx, C.byref(v)), self._ctx)
        return "single" if v.value == N.TV_PCG_SINGLE_REDUCTION else "kspcg"

    def num_dofs(self, space=0):
        n = C.c_int64()
        off = C.c_int64()
        N.check(self._lib.tv_num_dofs(self._ctx, space, C.byref(n), C.byref(off)), self._ctx)
        return n.value, off.value

    def _dof_coordinates(self, space):
        n, _ = self.num_dofs(space)
        X = np.zeros((n, 3))
        N.check(self._lib.tv_dof_coordinates(self._ctx, space, X.ctypes.data_as(C.POINTER(C.c_double)), n),
                self._ctx)
        return X

    def get_field(self, field: str) -> np.ndarray:
        fid = N.FIELD_ID[field]
        space = 1 if field in _SIGMA_FIELDS else 0
        n, _ = self.num_dofs(space)
        out = np.empty(n * self._bs[field])
        N.check(self._lib.tv_get_field(self._ctx, fid, out.ctypes.data_as(C.POINTER(C.c_double)), out.size),
                self._ctx)
        return out

    def set_field(self, field: str, values) -> None:
        fid = N.FIELD_ID[field]
        v = np.ascontiguousarray(values, dtype=np.float64).reshape(-1)
        N.check(self._lib.tv_set_field(self._ctx, fid, v.ctypes.data_as(C.POINTER(C.c_double)), v.size),
                self._ctx)
        self._cache.pop(field, None)

    def _host_array(self, field):
        ent = self._cache.get(field)
        if ent is not None and ent[2] == self._device_version:
            return ent[0]
        arr = self.get_field(field)
        self._cache[field] = [arr, _digest(arr), self._device_version]
        return arr

    def _flush(self):
        """Push host arrays that were modified in place back to the device."""
        for field, (arr, dig, ver) in list(self._cache.items()):
            if ver == self._device_version and _digest(arr) != dig:
                self.set_field(field, arr)
        self._cache.clear()

    # ---- reference API -------------------------------------------------------------------
    def setup(self, dirichlet_bc: bool = False, outfile_name: str = "visco", outfile_name1: str = "stresses") -> None:
        self._set_initial_condition(temp_value=self.material_model.T_init)
        if dirichlet_bc:
            if self.model_mode != "paper":
                # ThermoViscoProblem.py:180 reads material_model.T_ambient, which
                # ViscoelasticModel does not have (nor self.fs, :241), and the bc
                # never reaches NonlinearProblem (:331): the reference cannot run this
                raise AttributeError("'ViscoelasticModel' object has no attribute 'T_ambient' "
                                     "(Dirichlet path of the reference is broken; model_mode='paper' runs it)")
            # paper mode: T = T_ambient on the exterior boundary, in the Newton
            # solve as dolfinx NonlinearProblem(bcs=[bc]) applies it
            N.check(self._lib.tv_set_dirichlet(self._ctx, 1, float(self.physical_model.T_ambient)), self._ctx)
        self.dirichlet_bc = bool(dirichlet_bc)
        self._outfile_names = (outfile_name, outfile_name1)
        if self.write_output:
            self._write_initial_output(t=self.t)
        self._setup_solver()

    def _setup_solver(self) -> None:
        """ThermoViscoProblem.py:330-346: ``problem.solver`` (NewtonSolver:
        incremental criterion, rtol 1e-12, report) and ``problem.ksp`` (its CG
        KSP), whose tolerances reach the context (tvfem/solver.py)."""
        from .solver import NewtonSolver
        self.solver = NewtonSolver(self)
        self.ksp = self.solver.krylov_solver

    def _update_values(self, current: Function, previous: Function) -> None:
        """ThermoViscoProblem.py:349-354: ghost update, then previous <- current
        (host round trip; the step's own copies run on the device)."""
        current.x.scatter_forward()
        previous.x.array[:] = current.x.array[:]

    # the reference's five series (ThermoViscoProblem.py:246-276): T, phi, Tf,
    # xi and sigma, as XDMF over raw binary (tvfem.xdmf reads them back)
    OUTPUT_FIELDS = ("T", "phi", "Tf", "xi", "sigma")

    def series_names(self, outfile_name: str = "visco", outfile_name1: str = "stresses"):
        """File stems of the five series.  With setup()'s defaults they are the
        reference's own file names (output/T, phi, Tf, xi and sigma,
        ThermoViscoProblem.py:249-268, which never reads the two arguments);
        a non-default ``outfile_name`` prefixes the four scalar series
        (``<outfile_name>_T`` ...) and a non-default ``outfile_name1`` names the
        stress series."""
        pre = "" if outfile_name == "visco" else f"{outfile_name}_"
        sig = "sigma" if outfile_name1 == "stresses" else outfile_name1
        return [f"{pre}{f}" for f in self.OUTPUT_FIELDS[:4]] + [sig]

    def _write_initial_output(self, t: float = 0.0) -> None:
        import os
        d = self.output_dir
        n_parts = getattr(self, "_n_parts", 1)
        if n_parts > 1:
            d = os.path.join(d, f"part{self._part}")
        os.makedirs(d, exist_ok=True)
        ids = (C.c_int * len(self.OUTPUT_FIELDS))(*[N.FIELD_ID[f] for f in self.OUTPUT_FIELDS])
        names = (C.c_char_p * len(self.OUTPUT_FIELDS))(*[n.encode() for n in self.series_names(
            *getattr(self, "_outfile_names", ("visco", "stresses")))])
        N.check(self._lib.tv_output_open_named(self._ctx, d.encode(), ids, names, len(self.OUTPUT_FIELDS)),
                self._ctx)
        self._output_open = True
        self._write_output(t)

    def _write_output(self, t=None) -> None:
        """Queue this step's fields; the copy and the file writes overlap the next steps."""
        self._flush()
        N.check(self._lib.tv_output_write(self._ctx, float(self.t if t is None else t)), self._ctx)

    def _finalize(self) -> None:
        if self._output_open:
            self._output_open = False
            N.check(self._lib.tv_output_close(self._ctx), self._ctx)

    def _set_initial_condition(self, temp_value: float) -> None:
        self._cache.clear()
        N.check(self._lib.tv_set_initial_condition(self._ctx, float(temp_value)), self._ctx)
        self._device_version += 1

    def solve_timestep(self, t=None, thermal_only: bool = False) -> None:
        if self.verbose:
            print(f"t={self.t}")
        self._flush()
        nits = C.c_int()
        kits = C.c_int()
        rc = self._lib.tv_step(self._ctx, 1 if thermal_only else 0, C.byref(nits), C.byref(kits))
        self._device_version += 1
        if rc == N.TV_ERR_NOT_CONVERGED:
            msg = self._lib.tv_last_error(self._ctx).decode()
            raise RuntimeError(msg)
        N.check(rc, self._ctx)
        self.last_newton_iterations = nits.value
        self.last_krylov_iterations = kits.value
        if self._newton_fixed_its == 0:
            # solver.error_on_nonconvergence = False: dolfinx returns (n, False)
            # and _solve_T fails its assert(converged) (ThermoViscoProblem.py:390)
            conv = C.c_int()
            N.check(self._lib.tv_last_converged(self._ctx, C.byref(conv)), self._ctx)
            assert conv.value, "Newton solver did not converge"
        if self._output_open:  # ThermoViscoProblem.py:374
            self._write_output()

    def _solve_T(self):
        self._flush()
        nits, kits, conv = C.c_int(), C.c_int(), C.c_int()
        rc = self._lib.tv_solve_T(self._ctx, C.byref(nits), C.byref(kits), C.byref(conv))
        self._device_version += 1
        N.check(rc, self._ctx)
        assert conv.value
        return nits.value, kits.value

    def solve(self, n_steps: int | None = None) -> None:
        if self.verbose:
            print("Starting solve")
        t_start = _time.time()
        for _ in range(self.n_steps if n_steps is None else n_steps):
            self.t += self.dt
            self.solve_timestep(t=self.t)
        if self.verbose:
            print(f"Solve finished in {_time.time() - t_start} seconds.")
        self._finalize()  # ThermoViscoProblem.py:614-620

    def close(self):
        if self._ctx is not None:
            try:
                self._finalize()
            finally:
                self._lib.tv_destroy(self._ctx)
                self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_SIGMA_FIELDS = {"thermal_strain", "total_strain", "deviatoric_strain", "ds_partial", "dsigma_partial",
                 "s_tilde_partial", "s_tilde_partial_next", "sigma_tilde_partial", "sigma_tilde_partial_next",
                 "s_partial", "s_partial_next", "sigma_partial", "sigma_partial_next", "sigma"}
