"""The C-ABI boundary: libtvfem.so builds, loads and exports every function
include/tvfem.h declares; without a GPU the library fails loudly (there is no
CPU fallback on the product path)."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "tvfem.h")
PKG = os.path.join(ROOT, "fem-glass-tempering_amd")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?(?:int|void|char)\s*\*?\s+(tv_\w+)\s*\(", src, flags=re.M)
    return sorted(set(names))


@pytest.fixture(scope="module")
def lib():
    so = os.path.join(PKG, "tvfem", "libtvfem.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, capture_output=True)
    from tvfem import _native as N
    return N.load_library()


def test_header_declares_the_boundary():
    names = _declared()
    for must in ("tv_create", "tv_residual", "tv_jacobian_apply", "tv_jacobian_diag", "tv_solve_T",
                 "tv_visco_update", "tv_step", "tv_comm_init", "tv_halo_exchange"):
        assert must in names


def test_library_exports_every_declared_symbol(lib):
    from tvfem import _native as N
    declared = _declared()
    missing = [n for n in declared if not hasattr(lib, n)]
    assert not missing, missing
    assert sorted(N.EXPORTS) == declared  # the Python binding covers exactly the header


def test_abi_version_and_defaults(lib):
    from tvfem import _native as N
    assert lib.tv_abi_version() == 8
    o = N.default_options()
    assert o.newton_rtol == 1e-12 and o.newton_atol == 1e-10 and o.newton_max_it == 50
    assert o.ksp_rtol == 1e-5 and o.ksp_max_it == 10000
    p = N.default_params(None, 0.1)
    assert p.T_0 == 800.0 and p.htc == 280.1 and list(p.lambda_k)[-1] == 2.033


def test_missing_parameter_key_raises(lib):
    from tvfem import _native as N
    with pytest.raises(KeyError):
        N.default_params({"f": 0.0}, 0.1)


def test_create_without_gpu_fails_loudly(lib):
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except Exception:
        pass
    import numpy as np
    from tvfem import _native as N
    desc = N.MeshDesc()
    desc.dim = 1
    x = np.linspace(0, 1, 5)
    desc.n_cells[0] = 4
    desc.coords[0] = x.ctypes.data_as(C.POINTER(C.c_double))
    desc.n_parts = 1
    fe = N.FeConfig(N.TV_CG, 1, N.TV_CG, 1)
    params = N.default_params(None, 0.1)
    ctx = C.c_void_p()
    rc = lib.tv_create(C.byref(desc), C.byref(fe), C.byref(params), None, 0, C.byref(ctx))
    assert rc == N.TV_ERR_HIP
    assert b"GPU" in lib.tv_last_error(None) or b"HIP" in lib.tv_last_error(None)


def test_problem_requires_gpu(lib):
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("GPU present")
    except Exception:
        pass
    from tvfem import interval_mesh
    from tvfem.problem import ThermoViscoProblem
    from tvfem._native import NativeError
    from oracle.tv_oracle import MAIN_MODEL_PARAMS
    cfg = {"T": {"element": "CG", "degree": 1}, "sigma": {"element": "CG", "degree": 1}}
    with pytest.raises(NativeError):
        ThermoViscoProblem(interval_mesh(50.0, 10), (0, 1), 0.1, cfg, dict(MAIN_MODEL_PARAMS))


def test_only_cg_dg_accepted(lib):
    from tvfem import interval_mesh
    from tvfem.problem import ThermoViscoProblem
    from oracle.tv_oracle import MAIN_MODEL_PARAMS
    with pytest.raises(AssertionError):
        ThermoViscoProblem(interval_mesh(50.0, 10), (0, 1), 0.1,
                           {"T": {"element": "N1curl", "degree": 1}, "sigma": {"element": "CG", "degree": 1}},
                           dict(MAIN_MODEL_PARAMS))
