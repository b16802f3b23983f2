"""The visco update's two speeds: one process, the C4
bench configuration (lean state, coupled, 8.2M CG1 nodes), a few time steps,
then the isolated update timed back to back (tv_time_kernel id 1, HIP events)
and the J x for comparison; prints one VISCO_MODE json line with the timings
and the device addresses of the streams the update touches (alignment / page
offsets), so fast and slow processes can be compared -- run it in several
processes, alone or under rocprofv3 --pmc.

    python tools/visco_modes.py [--cells 400,400,50] [--steps 2] [--reps 30]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fem-glass-tempering_amd"))
sys.path.insert(0, ROOT)

from tvfem import box_mesh  # noqa: E402
from tvfem import _native as N  # noqa: E402
from tvfem.problem import ThermoViscoProblem  # noqa: E402

FIELDS = {"T": 0, "T_prev": 1, "Tf": 3, "Tf_partial": 5, "phi": 7, "xi": 9, "s_tilde": 15, "sigma_tilde": 17,
          "sigma": 23}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", default="400,400,50")
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--reps", type=int, default=30)
    a = ap.parse_args()
    nc = [int(v) for v in a.cells.split(",")]
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from partition_check import MP
    cfg = {"T": {"element": "CG", "degree": 1}, "sigma": {"element": "CG", "degree": 1}}
    p = ThermoViscoProblem(box_mesh([50.0, 50.0, 5.0], nc), (0, 10), 0.1, cfg, MP, verbose=False,
                           write_output=False, materialize=False, part_axis=1, preconditioner="gmg")
    p.setup()
    for _ in range(a.steps):
        p.solve_timestep()
    lib, ctx = p._lib, p._ctx
    res = {"pid": os.getpid(), "cells": nc}
    for kid, name in ((1, "visco_ms"), (0, "jx_ms"), (1, "visco_ms_again")):
        ms = C.c_double()
        N.check(lib.tv_time_kernel(ctx, kid, a.reps, C.byref(ms)), ctx)
        res[name] = round(ms.value, 5)
    addrs = {}
    for nm, fid in FIELDS.items():
        ptr, stride = C.c_void_p(), C.c_int64()
        if lib.tv_field_device_ptr(ctx, fid, C.byref(ptr), C.byref(stride)) == 0 and ptr.value:
            addrs[nm] = {"addr": hex(ptr.value), "mod_2MiB": ptr.value % (2 << 20), "mod_1GiB": ptr.value % (1 << 30)}
    res["fields"] = addrs
    print("VISCO_MODE " + json.dumps(res), flush=True)
    p.close()


if __name__ == "__main__":
    main()
