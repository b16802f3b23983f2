"""Generate the golden time-step fixtures under tests/golden/ from the CPU
oracle (oracle/tv_oracle.py, the restatement of ThermoViscoProblem.solve_timestep,
ThermoViscoProblem.py:349-379).

    python tests/golden/make_golden.py

The reference itself (dolfinx 0.7.3 + PETSc 3.20, as the reference pins them) is not installed in this image, so
these vectors pin regressions of the oracle and give the GPU tests a fixed
target that does not need the oracle at run time; they are not dolfinx output
(parity to dolfinx is unpinned).  Each .npz holds the inputs
(axes, element config, parameters, dt, steps) and the outputs after `steps`
coupled steps from the uniform T_0 initial state, plus the well-conditioned
masks (|T - T_prev| > 1e-6 K) used for the stress comparison.
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import tv_oracle as O  # noqa: E402

CG = {"element": "CG", "degree": 1}
DG = {"element": "DG", "degree": 1}
GRADED_1D = np.concatenate([np.linspace(0, 5, 11), np.linspace(5, 45, 9)[1:], np.linspace(45, 50, 11)[1:]])

CASES = {
    "g1d_cg_graded": ([GRADED_1D], CG, CG, 6, 0.1),
    "g1d_dg_cg": ([GRADED_1D], DG, CG, 6, 0.1),
    "g2d_cg_dg": ([np.linspace(0, 3, 9), np.linspace(0, 1, 4)], CG, DG, 3, 0.1),
    "g3d_cg": ([np.linspace(0, 2, 7), np.linspace(0, 1.5, 5), np.array([0.0, 0.2, 0.5, 1.0])], CG, CG, 3, 0.1),
    "g3d_dg": ([np.linspace(0, 1, 4), np.linspace(0, 1, 4), np.linspace(0, 0.5, 3)], DG, DG, 2, 0.05),
}

OUT_FIELDS = {
    "T": ("functions_current", "T"),
    "Tf": ("functions_current", "Tf"), "Tf_partial": ("functions_current", "Tf_partial"),
    "phi": ("functions", "phi"), "xi": ("functions", "xi"),
    "sigma": ("functions_next", "sigma"),
    "s_partial": ("functions_current", "s_partial"), "sigma_partial": ("functions_current", "sigma_partial"),
}


def run_case(axes, tf, sf, steps, dt):
    mp = dict(O.MAIN_MODEL_PARAMS)
    ref = O.OracleProblem(O.rectilinear_mesh(axes), (0.0, steps * dt), dt, {"T": tf, "sigma": sf}, mp)
    ref.setup()
    Tlast = None
    for _ in range(steps):
        Tlast = ref.functions_current["T"].copy()
        ref.solve_timestep()
    mT = np.abs(ref.functions_current["T"] - Tlast) > 1e-6
    mS = mT[ref._maps[("S", "T")]]
    out = {k: getattr(ref, a)[n].copy() for k, (a, n) in OUT_FIELDS.items()}
    out["mask_T"] = mT
    out["mask_S"] = mS
    out["newton_its"] = np.array([h[0] for h in ref.newton_history])
    return mp, out


def main():
    for name, (axes, tf, sf, steps, dt) in CASES.items():
        mp, out = run_case(axes, tf, sf, steps, dt)
        meta = json.dumps({"config": {"T": tf, "sigma": sf}, "model_parameters": mp, "dt": dt, "steps": steps})
        arrs = {f"axis{a}": np.asarray(x, dtype=np.float64) for a, x in enumerate(axes)}
        np.savez_compressed(os.path.join(HERE, name + ".npz"), meta=np.array(meta), **arrs, **out)
        print(name, {k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
