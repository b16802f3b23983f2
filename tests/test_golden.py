"""Golden time-step fixtures (tests/golden/*.npz, made by make_golden.py).

CPU: the oracle reproduces its committed vectors (guards the checker itself).
GPU: the HIP path reproduces them without running the oracle.  Tolerances as
in test_gpu_parity.py: T / Tf rel. L2 <= 1e-10, phi <= 1e-9, xi and the stress
tensors <= 1e-6 on the well-conditioned dofs (|T - T_prev| > 1e-6 K; stored
masks), NaN positions equal there.
"""
import glob
import json
import os

import numpy as np
import pytest

HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
FILES = sorted(glob.glob(os.path.join(HERE, "*.npz")))
IDS = [os.path.basename(f)[:-4] for f in FILES]


def load(path):
    z = np.load(path)  # allow_pickle=False
    meta = json.loads(str(z["meta"]))
    axes = [z[f"axis{a}"] for a in range(3) if f"axis{a}" in z]
    return meta, axes, {k: z[k] for k in z.files}


def relerr(a, b, mask=None, scale=None):
    """relative L2 error; ``scale`` (optional) replaces ||b|| in the denominator."""
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    if mask is not None:
        a, b = a[mask], b[mask]
    na, nb = np.isnan(a), np.isnan(b)
    assert np.array_equal(na, nb), f"NaN pattern differs: {na.sum()} vs {nb.sum()}"
    a, b = a[~na], b[~nb]
    den = np.linalg.norm(b) if scale is None else scale
    return np.linalg.norm(a - b) / den if den else np.linalg.norm(a - b)


def _checks(z, d, get):
    """(name, got, want, tol, mask, scale).  The deviatoric partial stresses
    s_partial are rounding noise (the thermal strain is isotropic, so dev = tot -
    tr/d I is 0 up to an ulp in 3D): they are measured against the volumetric
    stress scale ||sigma_partial|| instead of their own norm."""
    d2 = d * d
    mT, mS = z["mask_T"], z["mask_S"]
    m6 = np.repeat(mS, 6 * d2)
    sg = z["sigma_partial"][m6]
    sg_scale = float(np.linalg.norm(sg[~np.isnan(sg)]))
    return [
        ("T", get("T"), z["T"], 1e-10, None, None),
        ("Tf", get("Tf"), z["Tf"], 1e-10, None, None),
        ("Tf_partial", get("Tf_partial"), z["Tf_partial"], 1e-10, None, None),
        ("phi", get("phi"), z["phi"], 1e-9, None, None),
        ("xi", get("xi"), z["xi"], 1e-6, mT, None),
        ("sigma", get("sigma"), z["sigma"], 1e-6, np.repeat(mS, d2), None),
        ("s_partial", get("s_partial"), z["s_partial"], 1e-6, m6, sg_scale),
        ("sigma_partial", get("sigma_partial"), z["sigma_partial"], 1e-6, m6, None),
    ]


def test_fixtures_present():
    assert len(FILES) >= 5


@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_oracle_reproduces_golden(path):
    from oracle import tv_oracle as O
    meta, axes, z = load(path)
    ref = O.OracleProblem(O.rectilinear_mesh(axes), (0.0, meta["steps"] * meta["dt"]), meta["dt"],
                          meta["config"], meta["model_parameters"])
    ref.setup()
    with np.errstate(invalid="ignore", divide="ignore"):
        for _ in range(meta["steps"]):
            ref.solve_timestep()
    src = {"T": ref.functions_current["T"], "Tf": ref.functions_current["Tf"],
           "Tf_partial": ref.functions_current["Tf_partial"], "phi": ref.functions["phi"],
           "xi": ref.functions["xi"], "sigma": ref.functions_next["sigma"],
           "s_partial": ref.functions_current["s_partial"], "sigma_partial": ref.functions_current["sigma_partial"]}
    for name, got, want, tol, m, sc in _checks(z, len(axes), src.__getitem__):
        assert relerr(got, want, m, sc) < min(tol, 1e-9), name
    assert [h[0] for h in ref.newton_history] == list(z["newton_its"])


@pytest.mark.gpu
@pytest.mark.parametrize("path", FILES, ids=IDS)
def test_hip_path_reproduces_golden(path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tvfem import RectilinearMesh
    from tvfem.problem import ThermoViscoProblem
    meta, axes, z = load(path)
    dev = ThermoViscoProblem(RectilinearMesh(axes), (0.0, meta["steps"] * meta["dt"]), meta["dt"],
                             meta["config"], meta["model_parameters"], materialize=True, verbose=False,
                             part_axis=2 if len(axes) == 3 else -1)  # storage order = oracle dof order
    dev.setup()
    for _ in range(meta["steps"]):
        dev.solve_timestep()
    groups = {"T": dev.functions_current, "Tf": dev.functions_current, "Tf_partial": dev.functions_current,
              "phi": dev.functions, "xi": dev.functions, "sigma": dev.functions_next,
              "s_partial": dev.functions_current, "sigma_partial": dev.functions_current}
    get = lambda k: groups[k][k].x.array  # noqa: E731
    for name, got, want, tol, m, sc in _checks(z, len(axes), get):
        e = relerr(got, want, m, sc)
        assert e < tol, (name, e, tol)
    dev.close()
