"""Time the fused PCG matvec (tv_time_kernel id 3) and the other hot kernels
under several env configurations, one subprocess per configuration.

    python tools/sweep_matvec.py [--cells 400,400,50] "TVFEM_MARCH_ROWS=8" "TVFEM_MARCH_ROWS=16 TVFEM_MARCH_MINBLK=1024" ...
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MP = {"f": 0.0, "epsilon": 0.93, "sigma": 5.670e-8, "T_ambient": 600.0, "T_0": 800.0, "alpha": 1.0,
      "htc": 280.1, "rho": 2500.0, "cp": 1433.0, "k": 1.0, "H": 627.8e3, "Tb": 869.0, "Rg": 8.314,
      "alpha_solid": 9.10e-6, "alpha_liquid": 25.10e-6, "Tf_init": 873.0}


def child(cells, reps, kernels, part_axis):
    sys.path[:0] = [os.path.join(ROOT, "fem-glass-tempering_amd"), ROOT]
    from tvfem import _native as N, box_mesh
    from tvfem.problem import ThermoViscoProblem
    nc = [int(v) for v in cells.split(",")]
    cfg = {"T": {"element": "CG", "degree": 1}, "sigma": {"element": "CG", "degree": 1}}
    prob = ThermoViscoProblem(box_mesh([50.0, 50.0, 5.0], nc), (0.0, 1.0), 0.1, cfg, dict(MP),
                              materialize=False, part_axis=part_axis, verbose=False)
    prob.setup()
    try:
        prob.solve_timestep(thermal_only=True)
    except Exception as e:  # timing-only experiments may break the solve
        print("solve failed:", e, flush=True)
    lib, ctx = prob._lib, prob._ctx
    out = {}
    for kid in kernels:
        ms = C.c_double()
        by = C.c_double()
        N.check(lib.tv_time_kernel(ctx, kid, reps, C.byref(ms)), ctx)
        N.check(lib.tv_kernel_bytes(ctx, kid, C.byref(by)), ctx)
        out[kid] = (round(ms.value * 1e3, 2), round(by.value / ms.value / 1e6, 1))
    out["newton"] = getattr(prob, "last_newton_iterations", None)
    out["krylov"] = getattr(prob, "last_krylov_iterations", None)
    prob.close()
    print("RESULT " + json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", default="400,400,50")
    ap.add_argument("--reps", type=int, default=30)
    ap.add_argument("--kernels", default="3,0,4")
    ap.add_argument("--part-axis", type=int, default=1)
    ap.add_argument("--child", action="store_true")
    ap.add_argument("configs", nargs="*")
    a = ap.parse_args()
    kernels = [int(k) for k in a.kernels.split(",")]
    if a.child:
        child(a.cells, a.reps, kernels, a.part_axis)
        return
    for cfg in a.configs or [""]:
        env = dict(os.environ)
        for kv in cfg.split():
            k, v = kv.split("=", 1)
            env[k] = v
        cmd = [sys.executable, os.path.abspath(__file__), "--child", "--cells", a.cells, "--reps", str(a.reps),
               "--kernels", a.kernels, "--part-axis", str(a.part_axis)]
        p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
        res = [ln for ln in p.stdout.splitlines() if ln.startswith("RESULT ")]
        print(f"{cfg or 'default':50s} rc={p.returncode} {res[0][7:] if res else p.stderr[-400:]}", flush=True)
        if p.returncode != 0:
            sys.exit(p.returncode)


if __name__ == "__main__":
    main()
