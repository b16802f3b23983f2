"""Measured cost of every exchange pattern of the partitioned C4 solve, and the
N-GPU step projection built from it.

For N = 2, 4, 8 a middle partition of the C4 plate (400 x 400 x 50 CG1, slabs
along y, the distributed GMG of the bench) is created on ONE GPU and given a
one-rank RCCL loopback communicator (tv_comm_init_loopback: every neighbour is
the rank itself, so the production RCCL groups run with self send/recv pairs
and one-rank all-reduces).  tv_comm_time times each pattern (back-to-back
calls on the stream, mean per call).  That is the fixed cost of the RCCL group
on one GPU -- enqueue, kernel launch, the copies -- and so a LOWER bound of the
same group between two GPUs over xGMI (which adds the peer round trip).

The projection: step(N) = the per-rank compute floor (bench.py --share N, the
launch sequence with the transport stubbed, read from profiles/) + the
exchange points of one step x their measured cost - the stub's own stand-ins.

    python tools/comm_latency.py [--reps 200] [--floors profiles/r05_bench_n{N}.json]
prints COMM_LATENCY <json>"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fem-glass-tempering_amd"))
sys.path.insert(0, ROOT)
os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")

from tvfem import box_mesh  # noqa: E402
from tvfem import _native as N  # noqa: E402
from tvfem.problem import ThermoViscoProblem  # noqa: E402

MP = {"f": 0.0, "epsilon": 0.93, "sigma": 5.670e-8, "T_ambient": 600.0, "T_0": 800.0, "alpha": 1.0, "htc": 280.1,
      "rho": 2500.0, "cp": 1433.0, "k": 1.0, "H": 627.8e3, "Tb": 869.0, "Rg": 8.314, "alpha_solid": 9.1e-6,
      "alpha_liquid": 25.1e-6}
CFG = {"T": {"element": "CG", "degree": 1}, "sigma": {"element": "CG", "degree": 1}}
PATTERNS = ["halo", "allreduce1", "close", "vec", "halo_l1", "halo_l2"]


def measure(world, reps, transport):
    lib = N.load_library()
    kw = {"ksp_fixed_its": 5} if transport == "stub" else {}
    p = ThermoViscoProblem(box_mesh([50.0, 50.0, 5.0], [400, 400, 50]), (0, 1), 0.1, CFG, MP, n_parts=world,
                           part=world // 2, part_axis=1, verbose=False, materialize=False, preconditioner="gmg",
                           write_output=False, **kw)
    if transport == "rccl":
        uid = C.create_string_buffer(lib.tv_comm_unique_id_size())
        N.check(lib.tv_comm_get_unique_id(uid))
        N.check(lib.tv_comm_init_loopback(p._ctx, uid.raw), p._ctx)
    else:
        N.check(lib.tv_comm_init_stub(p._ctx), p._ctx)
    p.setup()
    us = {}
    for k, name in enumerate(PATTERNS):
        v = C.c_double()
        rc = lib.tv_comm_time(p._ctx, k, reps, C.byref(v))
        us[name] = v.value if rc == 0 else None
    p.close()
    return us


def exchanges_per_step(us, newton=4, krylov=20, form="cgs"):
    """Exchange points of one C4 step of the distributed GMG-PCG as tv_mgdist.cpp
    / tv_solver.cpp issue them (each entry: pattern -> calls per step).
    form "kspcg1": KSPCG with one ghost plane (rounds 3-4); "kspcg": KSPCG on
    deep-ghost slabs; "cgs": the single-reduction form on deep-ghost slabs."""
    dist_l1 = us["halo_l1"] is not None
    dist_l2 = us["halo_l2"] is not None
    rep = us["vec"] is not None
    vcyc = [] if form != "kspcg1" else [("halo", 1)]   # pre-smoothed x0 (deep ghosts: computed on the ghosts)
    if dist_l1:
        vcyc += [] if form != "kspcg1" else [("halo", 1)]  # the residual d0
        vcyc += [("halo_l1", 2)]                             # x1 pre- and post-smoothed
        if dist_l2:
            vcyc += [("halo_l1", 1), ("halo_l2", 2)]
    if rep:
        vcyc += [("vec", 1)]
    if form == "cgs":
        per_it = [("close", 1)] + vcyc          # (z.z, z.r, z.u) + u ghosts; the V-cycle
    else:
        per_it = [("allreduce1", 1), ("close", 1)] + vcyc  # p.w; (z.z, z.r) + z ghosts; the V-cycle
    per_newton = [("close", 1)] + vcyc + [("allreduce1", 1), ("halo", 1)]  # the solve's init; ||dx||; T ghosts
    cnt = {}
    for name, n in per_it:
        cnt[name] = cnt.get(name, 0) + n * krylov
    for name, n in per_newton:
        cnt[name] = cnt.get(name, 0) + n * newton
    cnt["halo"] = cnt.get("halo", 0) + 2  # T, T_prev at the step's start
    points_it = sum(n for _, n in per_it)
    return cnt, points_it


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--worlds", type=str, default="2,4,8")
    ap.add_argument("--form", choices=["cgs", "kspcg", "kspcg1"], default="cgs",
                    help="the Krylov form whose exchange points are counted (the contexts measured are this "
                         "library's: deep ghosts on the fine grid)")
    ap.add_argument("--floors", type=str, default=os.path.join(ROOT, "profiles", "r05_bench_n{N}.json"))
    a = ap.parse_args()
    out = {"transport": "RCCL one-rank loopback on one MI355X (self send/recv, one-rank all-reduce)",
           "reps": a.reps, "worlds": {}}
    for w in (int(v) for v in a.worlds.split(",")):
        rc = measure(w, a.reps, "rccl")
        st = measure(w, a.reps, "stub")
        cnt, pts = exchanges_per_step(rc, form=a.form)
        comm_ms = sum(cnt[k] * rc[k] for k in cnt) * 1e-3
        stub_ms = sum(cnt[k] * (st[k] or 0.0) for k in cnt) * 1e-3
        rec = {"us_rccl_loopback": rc, "us_stub": st, "exchanges_per_step": cnt, "points_per_krylov_it": pts,
               "comm_ms_per_step_lower_bound": comm_ms, "stub_ms_per_step": stub_ms}
        fp = a.floors.replace("{N}", str(w))
        if os.path.exists(fp):
            floor = json.load(open(fp))["ms_per_step"]
            rec["share_floor_ms"] = floor
            rec["projected_step_ms_lower_bound"] = floor - stub_ms + comm_ms
        out["worlds"][str(w)] = rec
        print(f"[comm] N={w}: " + json.dumps(rec), flush=True)
    print("COMM_LATENCY " + json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
