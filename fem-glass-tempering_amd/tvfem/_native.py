"""ctypes binding of libtvfem.so (C-ABI declared in include/tvfem.h).

The product path has no fallback: if the library is missing or no GPU is
present, every entry point raises ``NativeError``.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_NAME = "libtvfem.so"

# status codes (tvfem.h)
TV_OK, TV_ERR_ARG, TV_ERR_HIP, TV_ERR_NOT_CONVERGED, TV_ERR_KSP, TV_ERR_STATE, TV_ERR_COMM = range(7)
TV_CG, TV_DG = 0, 1
TV_PCG_AUTO, TV_PCG_KSPCG, TV_PCG_SINGLE_REDUCTION = 0, 1, 2
TV_MODEL_REFERENCE, TV_MODEL_PAPER = 0, 1
TV_PC_JACOBI, TV_PC_GMG, TV_PC_AMG = 0, 1, 2
TV_DG_KERNEL_AUTO, TV_DG_KERNEL_TILE, TV_DG_KERNEL_CELLS = 0, 1, 2
TV_MG_COUPLING_AUTO, TV_MG_COUPLING_GLOBAL, TV_MG_COUPLING_LOCAL = 0, 1, 2
ABI_VERSION = 8

# field ids (tvfem.h enum, same order)
FIELDS = [
    "T", "T_prev", "T_next", "Tf", "Tf_prev", "Tf_partial", "Tf_partial_prev", "phi", "phi_next", "xi",
    "thermal_strain", "total_strain", "deviatoric_strain", "ds_partial", "dsigma_partial",
    "s_tilde_partial", "s_tilde_partial_next", "sigma_tilde_partial", "sigma_tilde_partial_next",
    "s_partial", "s_partial_next", "sigma_partial", "sigma_partial_next", "sigma", "residual", "dx",
]
FIELD_ID = {n: i for i, n in enumerate(FIELDS)}

# every C symbol include/tvfem.h declares (checked by tests/test_abi.py)
EXPORTS = [
    "tv_abi_version", "tv_last_error", "tv_default_options", "tv_default_params", "tv_create", "tv_create_unstructured", "tv_create_unstructured_part", "tv_partition_rcb", "tv_destroy",
    "tv_num_dofs", "tv_field_block_size", "tv_dof_coordinates", "tv_set_field", "tv_get_field",
    "tv_field_device_ptr", "tv_set_initial_condition", "tv_sync", "tv_residual", "tv_jacobian_apply",
    "tv_jacobian_diag", "tv_precond_apply", "tv_solve_T", "tv_visco_update", "tv_step", "tv_comm_unique_id_size",
    "tv_comm_get_unique_id", "tv_comm_init", "tv_comm_init_stub", "tv_comm_init_loopback", "tv_comm_check", "tv_comm_time", "tv_halo_exchange", "tv_time_kernel", "tv_kernel_bytes", "tv_kernel_timing", "tv_kernel_stats",
    "tv_last_stats", "tv_last_converged", "tv_comm_init_host", "tv_partition_layout", "tv_pcg_variant",
    "tv_set_dirichlet", "tv_get_options", "tv_set_newton_tolerances", "tv_set_ksp_tolerances",
    "tv_output_open", "tv_output_open_named", "tv_output_write", "tv_output_close", "tv_xdmf_open",
    "tv_xdmf_add_field", "tv_xdmf_append", "tv_xdmf_close",
]

HOST_ALLREDUCE_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_int, C.c_void_p)
HOST_SENDRECV_FN = C.CFUNCTYPE(C.c_int, C.POINTER(C.c_double), C.c_size_t, C.c_int, C.POINTER(C.c_double),
                               C.c_size_t, C.c_int, C.c_void_p)


class NativeError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(msg)
        self.code = code


class MeshDesc(C.Structure):
    _fields_ = [("dim", C.c_int), ("n_cells", C.c_int * 3), ("coords", C.POINTER(C.c_double) * 3),
                ("part_axis", C.c_int), ("n_parts", C.c_int), ("part", C.c_int)]


class UMeshDesc(C.Structure):
    _fields_ = [("dim", C.c_int), ("n_vertices", C.c_int64), ("coords", C.POINTER(C.c_double)),
                ("n_cells", C.c_int64), ("cells", C.POINTER(C.c_int64))]


class UPartDesc(C.Structure):
    _fields_ = [("n_parts", C.c_int), ("part", C.c_int), ("n_owned", C.c_int64), ("n_owned_cells", C.c_int64),
                ("global_offset", C.c_int64), ("n_neighbors", C.c_int), ("neighbors", C.POINTER(C.c_int)),
                ("recv_count", C.POINTER(C.c_int64)), ("send_count", C.POINTER(C.c_int64)),
                ("send_idx", C.POINTER(C.c_int64))]


class FeConfig(C.Structure):
    _fields_ = [("T_family", C.c_int), ("T_degree", C.c_int), ("sigma_family", C.c_int),
                ("sigma_degree", C.c_int)]


_PARAM_SCALARS = ["f", "epsilon", "sigma", "T_ambient", "T_0", "alpha", "htc", "rho", "cp", "k",
                  "H", "Tb", "Rg", "alpha_solid", "alpha_liquid", "Tf_init"]
_PARAM_TABLES = ["m_n", "lambda_m", "g_n", "lambda_g", "k_n", "lambda_k"]


class Params(C.Structure):
    _fields_ = ([(n, C.c_double) for n in _PARAM_SCALARS] + [(n, C.c_double * 6) for n in _PARAM_TABLES]
                + [("dt", C.c_double)])


class Options(C.Structure):
    _fields_ = [("newton_rtol", C.c_double), ("newton_atol", C.c_double), ("newton_max_it", C.c_int),
                ("error_on_nonconvergence", C.c_int), ("ksp_rtol", C.c_double), ("ksp_atol", C.c_double),
                ("ksp_dtol", C.c_double), ("ksp_max_it", C.c_int), ("materialize", C.c_int),
                ("pcg_batch", C.c_int), ("pcg_variant", C.c_int),
                ("model_mode", C.c_int), ("preconditioner", C.c_int), ("mg_levels", C.c_int),
                ("dg_kernel", C.c_int), ("dg_tile_chunk", C.c_int), ("mg_replicate_nodes", C.c_int),
                ("ksp_fixed_its", C.c_int), ("mg_coupling", C.c_int)]


_lib = None


def lib_path():
    return os.environ.get("TVFEM_LIB", os.path.join(_HERE, LIB_NAME))


def load_library():
    """Load libtvfem.so (built in-tree by __graft_entry__.build() / make)."""
    global _lib
    if _lib is not None:
        return _lib
    p = lib_path()
    if not os.path.exists(p):
        raise NativeError(TV_ERR_HIP, f"{p} not found: build it with `make -C fem-glass-tempering_amd` "
                                      "(there is no CPU fallback)")
    lib = C.CDLL(p)
    vp = C.c_void_p
    i64p = C.POINTER(C.c_int64)
    dp = C.POINTER(C.c_double)
    ip = C.POINTER(C.c_int)
    sig = {
        "tv_abi_version": (C.c_int, []),
        "tv_last_error": (C.c_char_p, [vp]),
        "tv_default_options": (None, [C.POINTER(Options)]),
        "tv_default_params": (None, [C.POINTER(Params)]),
        "tv_create_unstructured": (C.c_int, [C.POINTER(UMeshDesc), C.POINTER(FeConfig), C.POINTER(Params),
                                             C.POINTER(Options), C.c_int, C.POINTER(C.c_void_p)]),
        "tv_create_unstructured_part": (C.c_int, [C.POINTER(UMeshDesc), C.POINTER(UPartDesc), C.POINTER(FeConfig),
                                                  C.POINTER(Params), C.POINTER(Options), C.c_int,
                                                  C.POINTER(C.c_void_p)]),
        "tv_partition_rcb": (C.c_int, [C.POINTER(UMeshDesc), C.c_int, C.POINTER(C.c_int)]),
        "tv_create": (C.c_int, [C.POINTER(MeshDesc), C.POINTER(FeConfig), C.POINTER(Params), C.POINTER(Options),
                                C.c_int, C.POINTER(vp)]),
        "tv_destroy": (C.c_int, [vp]),
        "tv_num_dofs": (C.c_int, [vp, C.c_int, i64p, i64p]),
        "tv_field_block_size": (C.c_int, [vp, C.c_int, ip]),
        "tv_dof_coordinates": (C.c_int, [vp, C.c_int, dp, C.c_size_t]),
        "tv_set_field": (C.c_int, [vp, C.c_int, dp, C.c_size_t]),
        "tv_get_field": (C.c_int, [vp, C.c_int, dp, C.c_size_t]),
        "tv_field_device_ptr": (C.c_int, [vp, C.c_int, C.POINTER(vp), i64p]),
        "tv_set_initial_condition": (C.c_int, [vp, C.c_double]),
        "tv_sync": (C.c_int, [vp]),
        "tv_residual": (C.c_int, [vp, vp, vp]),
        "tv_jacobian_apply": (C.c_int, [vp, vp, vp]),
        "tv_jacobian_diag": (C.c_int, [vp, vp]),
        "tv_precond_apply": (C.c_int, [vp, vp, vp]),
        "tv_solve_T": (C.c_int, [vp, ip, ip, ip]),
        "tv_visco_update": (C.c_int, [vp]),
        "tv_step": (C.c_int, [vp, C.c_int, ip, ip]),
        "tv_comm_unique_id_size": (C.c_int, []),
        "tv_comm_get_unique_id": (C.c_int, [C.c_char_p]),
        "tv_comm_init": (C.c_int, [vp, C.c_char_p, C.c_int, C.c_int]),
        "tv_comm_init_stub": (C.c_int, [vp]),
        "tv_comm_init_loopback": (C.c_int, [vp, C.c_char_p]),
        "tv_comm_check": (C.c_int, [vp, i64p, i64p]),
        "tv_halo_exchange": (C.c_int, [vp, C.c_int]),
        "tv_comm_time": (C.c_int, [vp, C.c_int, C.c_int, C.POINTER(C.c_double)]),
        "tv_time_kernel": (C.c_int, [vp, C.c_int, C.c_int, dp]),
        "tv_kernel_bytes": (C.c_int, [vp, C.c_int, dp]),
        "tv_kernel_timing": (C.c_int, [vp, C.c_int]),
        "tv_kernel_stats": (C.c_int, [vp, C.c_int, dp, C.POINTER(C.c_int64)]),
        "tv_last_stats": (C.c_int, [vp, ip, ip, dp]),
        "tv_last_converged": (C.c_int, [vp, ip]),
        "tv_comm_init_host": (C.c_int, [vp, C.c_int, C.c_int, HOST_ALLREDUCE_FN, HOST_SENDRECV_FN, vp]),
        "tv_partition_layout": (C.c_int, [C.POINTER(MeshDesc), i64p]),
        "tv_pcg_variant": (C.c_int, [vp, ip]),
        "tv_set_dirichlet": (C.c_int, [vp, C.c_int, C.c_double]),
        "tv_get_options": (C.c_int, [vp, C.POINTER(Options)]),
        "tv_set_newton_tolerances": (C.c_int, [vp, C.c_double, C.c_double, C.c_int, C.c_int]),
        "tv_set_ksp_tolerances": (C.c_int, [vp, C.c_double, C.c_double, C.c_double, C.c_int]),
        "tv_output_open": (C.c_int, [vp, C.c_char_p, ip, C.c_int]),
        "tv_output_open_named": (C.c_int, [vp, C.c_char_p, ip, C.POINTER(C.c_char_p), C.c_int]),
        "tv_output_write": (C.c_int, [vp, C.c_double]),
        "tv_output_close": (C.c_int, [vp]),
        "tv_xdmf_open": (vp, [C.c_char_p, C.c_int, ip, C.POINTER(dp)]),
        "tv_xdmf_add_field": (C.c_int, [vp, C.c_char_p, C.c_int, C.c_int]),
        "tv_xdmf_append": (C.c_int, [vp, C.c_int, C.c_double, dp, C.c_size_t]),
        "tv_xdmf_close": (None, [vp]),
    }
    for name, (res, args) in sig.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.tv_abi_version() != ABI_VERSION:
        raise NativeError(TV_ERR_ARG, "libtvfem ABI version mismatch")
    _lib = lib
    return lib


def check(code, ctx=None):
    if code != TV_OK:
        lib = load_library()
        msg = lib.tv_last_error(ctx)
        msg = msg.decode() if msg else "unknown error"
        if code == TV_ERR_NOT_CONVERGED:
            raise NativeError(code, msg)
        raise NativeError(code, msg)
    return code


def default_params(model_parameters: dict | None, dt: float) -> Params:
    lib = load_library()
    p = Params()
    lib.tv_default_params(C.byref(p))
    if model_parameters is not None:
        for n in _PARAM_SCALARS:
            if n not in model_parameters:
                if n == "Tf_init":  # declared in main.py:54 but never read by the reference
                    continue
                raise KeyError(n)  # the reference indexes every other key (ThermalModel.py:18-27,
                #                     ViscoelasticModel.py:73-83)
            setattr(p, n, float(model_parameters[n]))
    p.dt = float(dt)
    return p


def default_options() -> Options:
    lib = load_library()
    o = Options()
    lib.tv_default_options(C.byref(o))
    return o
