#!/usr/bin/env python3
"""Launch audit (VERDICT r5 "next" item 1a): the unprofiled cost of one
dependent launch of the library's own small kernels, on the C4 context and on
one rank's share of an N-way partition (the context bench.py --share N builds).

For each kernel id of tv_time_kernel 12-17 (include/tvfem.h) it queues `reps`
back-to-back launches behind a spin kernel and reads HIP events around the
chain: per launch = elapsed / reps, as the GPU runs them.  Compare with the
rocprofv3 kernel-trace durations of the same kernels (profiles/r05_trace_*).

    python tools/launch_audit.py [--share 8] [--reps 400] [--out FILE]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fem-glass-tempering_amd"))

IDS = {12: "empty one-thread kernel", 13: "k_set_state (one thread, 160-B argument)",
       14: "one-block reduce (k_reduce)", 15: "k_mg_jacobi, coarsest GMG level",
       16: "J x of GMG level 1 (march)", 17: "fine-grid J x (march + side faces)"}


def audit(share, reps, cells):
    from tvfem import box_mesh
    from tvfem import _native as N
    from tvfem.problem import ThermoViscoProblem
    mp = {"f": 0.0, "epsilon": 0.93, "sigma": 5.670e-8, "T_ambient": 600.0, "T_0": 800.0, "alpha": 1.0,
          "htc": 280.1, "rho": 2500.0, "cp": 1433.0, "k": 1.0, "H": 627.8e3, "Tb": 869.0e0, "Rg": 8.314,
          "alpha_solid": 9.10e-6, "alpha_liquid": 25.10e-6, "Tf_init": 873.0}
    cfg = {"T": {"element": "CG", "degree": 1}, "sigma": {"element": "CG", "degree": 1}}
    kw = {}
    if share > 1:
        kw = {"n_parts": share, "part": share // 2, "part_axis": 1, "newton_fixed_its": 4, "ksp_fixed_its": 5}
    prob = ThermoViscoProblem(box_mesh([50.0, 50.0, 5.0], cells), (0.0, 50.0), 0.1, cfg, mp, materialize=False,
                              verbose=False, preconditioner="gmg", write_output=False, **kw)
    lib, ctx = prob._lib, prob._ctx
    if share > 1:
        N.check(lib.tv_comm_init_stub(ctx), ctx)
    prob.setup()
    prob.solve_timestep()
    prob.solve_timestep()
    out = {}
    for kid, name in IDS.items():
        ms = C.c_double()
        rc = lib.tv_time_kernel(ctx, kid, reps, C.byref(ms))
        if rc != 0:
            out[name] = None
            continue
        out[name] = round(ms.value * 1e3, 3)
    prob.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--share", type=int, nargs="*", default=[1, 8])
    ap.add_argument("--reps", type=int, default=400)
    ap.add_argument("--cells", default="400,400,50")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cells = [int(v) for v in a.cells.split(",")]
    res = {"method": f"{a.reps} back-to-back launches queued behind a spin kernel, HIP events around the chain "
                     "(tv_time_kernel 12-17): us per launch, unprofiled", "contexts": {}}
    for s in a.share:
        key = "C4 single GPU" if s <= 1 else f"share/{s} (middle slab, transport stubbed)"
        res["contexts"][key] = audit(s, a.reps, cells)
        print(key, json.dumps(res["contexts"][key]), flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            json.dump(res, fh, indent=1)


if __name__ == "__main__":
    main()
