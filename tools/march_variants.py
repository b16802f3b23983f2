"""Isolated timings of the box march kernels for library variants (A/B builds
of tools/build_variant.sh), without a solve: the C4 context is set up, then
tv_time_kernel times the fused PCG matvec (id 3, back to back), the plain
J x (id 0, back to back) and the flushed J x (id 10, median of 21).  Prints
one MARCH line per library given in TVFEM_LIB.

    TVFEM_LIB=... python tools/march_variants.py [--cells 400,400,50] [--reps 20]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fem-glass-tempering_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from tvfem import box_mesh  # noqa: E402
from tvfem import _native as N  # noqa: E402
from tvfem.problem import ThermoViscoProblem  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", default="400,400,50")
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    from partition_check import MP
    nc = [int(v) for v in a.cells.split(",")]
    cfg = {"T": {"element": "CG", "degree": 1}, "sigma": {"element": "CG", "degree": 1}}
    p = ThermoViscoProblem(box_mesh([50.0, 50.0, 5.0], nc), (0, 10), 0.1, cfg, MP, verbose=False,
                           write_output=False, materialize=False, part_axis=1, pcg_variant="kspcg")
    p.setup()
    lib, ctx = p._lib, p._ctx
    res = {"lib": os.path.basename(os.environ.get("TVFEM_LIB", "libtvfem.so"))}
    for kid, name, reps in ((3, "fused_us", a.reps), (0, "jx_us", a.reps), (10, "jx_flushed_us", 21),
                            (3, "fused_us_again", a.reps)):
        ms = C.c_double()
        N.check(lib.tv_time_kernel(ctx, kid, reps, C.byref(ms)), ctx)
        res[name] = round(ms.value * 1e3, 2)
    print("MARCH " + json.dumps(res), flush=True)
    p.close()


if __name__ == "__main__":
    main()
