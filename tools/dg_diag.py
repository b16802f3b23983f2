"""DG1 tile J x against the cell kernel for both partition axes (diagnostic).
Usage: python tools/dg_diag.py"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fem-glass-tempering_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from oracle import tv_oracle as O  # noqa: E402
from tvfem import box_mesh  # noqa: E402
from tvfem.problem import ThermoViscoProblem  # noqa: E402

DG = {"element": "DG", "degree": 1}


def japply(nc, L, pa, tile):
    os.environ["TVFEM_EXPERIMENTS"] = "1"
    os.environ["TVFEM_DG_TILE"] = str(tile)
    p = ThermoViscoProblem(box_mesh(L, nc), (0.0, 1.0), 0.1, {"T": DG, "sigma": DG}, dict(O.MAIN_MODEL_PARAMS),
                           part_axis=pa, materialize=False, verbose=False)
    p.setup()
    n = p.get_field("T").size
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.randn(n, dtype=torch.float64, device="cuda", generator=g)
    one = torch.ones(n, dtype=torch.float64, device="cuda")
    y, y1 = torch.empty_like(x), torch.empty_like(x)
    assert p._lib.tv_jacobian_apply(p._ctx, x.data_ptr(), y.data_ptr()) == 0
    assert p._lib.tv_jacobian_apply(p._ctx, one.data_ptr(), y1.data_ptr()) == 0
    p.close()
    return y.cpu().numpy(), y1.cpu().numpy()


mp = O.MAIN_MODEL_PARAMS
dg = 0.001 * (4.0 * mp["sigma"] * mp["epsilon"] * mp["T_0"] ** 3 + mp["htc"])
for nc, L in (((64, 13, 7), (6.4, 1.3, 0.7)), ((20, 20, 5), (5.0, 5.0, 1.0)), ((40, 40, 10), (5.0, 5.0, 1.0)),
              ((200, 200, 25), (50.0, 50.0, 5.0))):
    want = L[0] * L[1] * L[2] + 0.1 * dg * 2 * (L[0] * L[1] + L[0] * L[2] + L[1] * L[2])
    for pa in (2, 1):
        yc, yc1 = japply(nc, L, pa, 0)
        yt, yt1 = japply(nc, L, pa, 2)
        e = np.linalg.norm(yt - yc) / np.linalg.norm(yc)
        bad = np.nonzero(np.abs(yt1 - yc1) > 1e-9 * np.abs(yc1).max())[0]
        print(f"nc {nc} part_axis {pa}: tile vs cell {e:.2e}; sum J1 cell {yc1.sum():.10e} tile {yt1.sum():.10e} "
              f"want {want:.10e}; {bad.size} differing dofs, first {bad[:8]}", flush=True)
