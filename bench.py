#!/usr/bin/env python3
"""Benchmark of the hot path: coupled thermo-viscoelastic time steps
(Newton + matrix-free Jacobi-PCG heat solve, fused viscoelastic update) on the
structured 3D CG1 hexahedral plate of BASELINE.json configs[3] (C4: 50 x 50 x 5
plate, 400 x 400 x 50 = 8M hex, 8,200,851 temperature dofs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--scaling strong|weak]

One process per GPU (torch.distributed.run sets RANK / LOCAL_RANK /
WORLD_SIZE); the mesh is sliced along y into N partitions with one ghost node
plane per interface; RCCL exchanges the ghost planes and all-reduces the PCG /
Newton dot products.  ``--scaling strong`` (default) partitions the fixed 8M-hex
mesh; ``weak`` gives every rank its own 400 x 400 x 50 slab of a 400 x 400N x 50
plate.  Rank 0 prints one JSON line (metric, value, roofline, cpu_baseline ...).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "fem-glass-tempering_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip table)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong")
    ap.add_argument("--cells", type=str, default="400,400,50", help="hex cells per axis (per rank for weak)")
    ap.add_argument("--lengths", type=str, default="50,50,5")
    ap.add_argument("--thermal-only", action="store_true")
    ap.add_argument("--family", choices=["CG", "DG"], default="CG",
                    help="element family of T and sigma (degree 1): CG (C1-C4) or DG (C5)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0, help="target CPU-baseline sample length")
    ap.add_argument("--kernel-reps", type=int, default=20)
    ap.add_argument("--comm", choices=["rccl", "host", "loopback"], default="rccl",
                    help="rccl (production) or host-staged gloo transport (rehearsal on one GPU); with --share: "
                         "loopback = the share's solve with the production RCCL groups on a one-rank communicator "
                         "(tv_comm_init_loopback: the neighbours are the slab's periodic images) instead of the stub")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="no HIP events around the hot kernels inside the timed steps")
    ap.add_argument("--output", default=None, metavar="DIR",
                    help="write the reference's five output series (T, phi, Tf, xi, sigma) every step "
                         "into DIR (asynchronous XDMF writer), to measure the step cost with output on")
    ap.add_argument("--mesh", choices=["box", "distorted"], default="box",
                    help="box: the rectilinear plate (tensor-product kernels); distorted: the same plate as a "
                         "general hexahedral mesh (jittered, sheared, warped; element-local kernels, one GPU)")
    ap.add_argument("--pc", choices=["auto", "jacobi", "gmg", "amg"], default="auto",
                    help="preconditioner: gmg (geometric multigrid on the box hierarchy, 3D box; distributed "
                         "over the ranks when partitioned), amg (smoothed-aggregation AMG, --mesh distorted on "
                         "one GPU), jacobi, or auto (gmg where it applies and the mesh has >= 4M T-dofs, at "
                         "every rank count; amg for --mesh distorted on one GPU)")
    ap.add_argument("--mg-levels", type=int, default=0, help="GMG levels incl. the fine one (0: automatic)")
    ap.add_argument("--dg-tile-chunk", type=int, default=0, help="DG1 J x tile: planes per march chunk (0: automatic)")
    ap.add_argument("--mg-coupling", choices=["auto", "global", "local"], default="auto",
                    help="partitioned GMG: global = the distributed V-cycle of the whole box (the N = 1 "
                         "preconditioner), local = each slab's own V-cycle (block Jacobi, no exchange inside the "
                         "preconditioner, ~2.4x the Krylov iterations); auto = global")
    ap.add_argument("--share", type=int, default=0, metavar="N",
                    help="time ONE rank's share of an N-way partition of the mesh on this GPU with the "
                         "communication stubbed (halos and all-reduces are no-ops) and the iteration counts "
                         "fixed (--share-its): the per-rank compute floor of an N-GPU run")
    ap.add_argument("--share-its", type=str, default="4,5", metavar="NEWTON,KRYLOV",
                    help="--share: Newton iterations per step, Krylov iterations per Newton solve")
    ap.add_argument("--pcg", choices=["auto", "kspcg", "single"], default="auto",
                    help="Krylov form: single-reduction (Chronopoulos-Gear, 3D CG) or PETSc KSPCG as written")
    return ap.parse_args()


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if a.gpus != world and world > 1:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE {world}")
    dist = None
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("gloo", rank=rank, world_size=world)

    from tvfem import box_mesh, distorted_box_mesh
    from tvfem import _native as N
    from tvfem.problem import ThermoViscoProblem

    nc = [int(v) for v in a.cells.split(",")]
    L = [float(v) for v in a.lengths.split(",")]
    if a.scaling == "weak":
        nc[1] *= world
        L[1] *= world
    um = a.mesh == "distorted"
    if um and a.family != "CG":
        raise SystemExit("--mesh distorted: CG1 (unstructured meshes)")
    mesh = distorted_box_mesh(L, nc) if um else box_mesh(L, nc)
    mp = {
        "f": 0.0, "epsilon": 0.93, "sigma": 5.670e-8, "T_ambient": 600.0, "T_0": 800.0, "alpha": 1.0,
        "htc": 280.1, "rho": 2500.0, "cp": 1433.0, "k": 1.0, "H": 627.8e3, "Tb": 869.0e0, "Rg": 8.314,
        "alpha_solid": 9.10e-6, "alpha_liquid": 25.10e-6, "Tf_init": 873.0,
    }  # main.py:29-55
    cfg = {"T": {"element": a.family, "degree": 1}, "sigma": {"element": a.family, "degree": 1}}
    device = local_rank
    if a.comm == "host":  # rehearsal of several ranks on fewer GPUs (host-staged transport)
        import torch
        device = local_rank % max(1, torch.cuda.device_count())
    pc = a.pc
    if pc == "auto":
        # GMG where it applies and pays: below ~4M T-dofs the V-cycle's ~25 launches are
        # latency-bound and Jacobi-PCG is faster per step (measured: C2 1.48 vs 1.29 ms,
        # C3 4.06 vs 3.19 ms; C4 13.4 vs 19.8 ms, C5 16.5 vs 32.5 ms)
        cells = nc[0] * nc[1] * nc[2]
        big = cells * (8 if a.family == "DG" else 1) >= 4_000_000
        # the same solver at every rank count: partitioned boxes run the distributed
        # V-cycle (tv_mgdist.cpp), so N = 1 and N > 1 lines compare like with like
        pc = "gmg" if (not um and a.pcg != "single" and big) else "jacobi"
        if um and world == 1:  # general hexahedra: the smoothed-aggregation AMG (distorted C4: 71.9 vs 127.0 ms)
            pc = "amg"
    # unstructured: RCB cell partition + ghost layer (tvfem.parallel.ghosted_partition)
    kw = {"n_parts": world, "part": rank} if um else {"n_parts": world, "part": rank, "part_axis": 1}
    if a.share > 1:  # a middle rank's slab (ghost planes both sides), no communicator
        if world > 1 or um:
            raise SystemExit("--share: one process, box mesh")
        nn, kk = (int(v) for v in a.share_its.split(","))
        kw = {"n_parts": a.share, "part": a.share // 2, "part_axis": 1, "newton_fixed_its": nn,
              "ksp_fixed_its": kk}
    prob = ThermoViscoProblem(mesh, (0.0, 50.0), 0.1, cfg, mp, device=device, materialize=False,
                              verbose=False, pcg_variant=a.pcg, preconditioner=pc, mg_levels=a.mg_levels,
                              mg_coupling=a.mg_coupling, dg_tile_chunk=a.dg_tile_chunk,
                              write_output=a.output is not None, output_dir=a.output or "output", **kw)
    mg_single = pc == "gmg" and prob.pcg_variant == "single"  # GMG-PCG, Chronopoulos-Gear form (deep-ghost slabs)
    single = prob.pcg_variant == "single" and not mg_single
    lib, ctx = prob._lib, prob._ctx
    if a.share > 1 and a.comm == "loopback":  # the production RCCL groups, self send / receive pairs
        os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
        uid = C.create_string_buffer(lib.tv_comm_unique_id_size())
        with _StdoutToStderr():
            N.check(lib.tv_comm_get_unique_id(uid))
            N.check(lib.tv_comm_init_loopback(ctx, uid.raw), ctx)
    elif a.share > 1:  # the multi-rank launch sequence with the transport stubbed (tv_comm_init_stub)
        N.check(lib.tv_comm_init_stub(ctx), ctx)
    if world > 1:
        from tvfem.parallel import init_host_comm, init_rccl
        if a.comm == "host":  # explicit opt-in only (rehearsal of several ranks on one GPU)
            init_host_comm(prob, rank, world, dist)
        else:
            # production transport; no silent fallback: a failed RCCL init ends the run
            try:
                with _StdoutToStderr():
                    init_rccl(prob, rank, world, dist)
            except Exception as e:
                print(f"[bench rank {rank}] RCCL init failed: {e}", file=sys.stderr, flush=True)
                raise SystemExit(3)
        # pre-flight: every exchange pattern of the solve on id-valued vectors
        # (tv_comm_check, collective); a wrong ghost or sum ends the run here
        nchk, nbad = C.c_int64(), C.c_int64()
        rc = lib.tv_comm_check(ctx, C.byref(nchk), C.byref(nbad))
        if rc != 0 or nbad.value:
            print(f"[bench rank {rank}] transport check failed: rc {rc}, {nbad.value} of {nchk.value} wrong: "
                  f"{lib.tv_last_error(ctx)}", file=sys.stderr, flush=True)
            raise SystemExit(3)
    prob.setup()
    n_owned, _ = prob.num_dofs(0)
    n_global = int(np.prod([n + 1 for n in nc])) if a.family == "CG" else 8 * int(np.prod(nc))
    cname = {("CG", (100, 100, 10)): "C2", ("CG", (200, 200, 25)): "C3", ("CG", (400, 400, 50)): "C4",
             ("DG", (200, 200, 25)): "C5"}.get((a.family, tuple(nc)), "custom")

    def barrier_sync():
        N.check(lib.tv_sync(ctx), ctx)
        if dist is not None:
            dist.barrier()

    step = lambda: prob.solve_timestep(thermal_only=a.thermal_only)  # noqa: E731
    for _ in range(a.warmup):
        step()
    barrier_sync()
    # the hot kernels are timed inside the timed steps themselves: the fused
    # matvec and the update of every converging PCG iteration write device clock
    # stamps (first workgroup's start, reduction tail's end), the visco update is
    # bracketed by HIP events
    if not a.no_kernel_timing:
        N.check(lib.tv_kernel_timing(ctx, 1), ctx)
    t0 = time.perf_counter()
    nits = kits = 0
    for _ in range(a.steps):
        step()
        nits += prob.last_newton_iterations
        kits += prob.last_krylov_iterations
    if a.output is not None:  # the timed region includes draining the writer
        prob._finalize()
    barrier_sync()
    dt_local = time.perf_counter() - t0
    if dist is not None:
        import torch
        t = torch.tensor([dt_local], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    else:
        elapsed = dt_local

    # ---- per-kernel timing and algorithmic bytes ----
    # "ms": mean launch duration inside the timed steps (device clock stamps of
    # every launch of the converging PCG iterations / HIP events around the visco
    # update); "ms_isolated":
    # back-to-back launches after the timed region (inputs partly Infinity-Cache
    # resident, so faster than in the solve; reported for reference only)
    kern = {}
    names = {3: "pcg_matvec_fused", 4: "pcg_update", 0: "jacobian_apply", 2: "residual"}
    if single:  # one fused launch per Krylov iteration, no separate update
        names = {3: "pcg_iteration_single_reduction", 0: "jacobian_apply", 2: "residual"}
    if pc == "gmg":  # the update is k_mg_update (no stamps); the V-cycle is timed as a whole
        names = {3: "pcg_matvec_fused", 11: "mg_vcycle", 0: "jacobian_apply", 2: "residual"}
    if um:  # element-local kernels: J x (coloured cell + facet launches) is the roofline kernel
        names = {0: "jacobian_apply_unstructured", 3: "pcg_matvec_unstructured", 4: "pcg_update", 2: "residual"}
        if pc == "amg":  # the update is k_mg_update (no stamps); the algebraic V-cycle timed as a whole
            names = {0: "jacobian_apply_unstructured", 3: "pcg_matvec_unstructured", 11: "mg_vcycle",
                     2: "residual"}
    if not a.thermal_only:
        names[1] = "visco_update"
    for kid, name in names.items():
        ms = C.c_double()
        by = C.c_double()
        N.check(lib.tv_time_kernel(ctx, kid, a.kernel_reps, C.byref(ms)), ctx)
        N.check(lib.tv_kernel_bytes(ctx, kid, C.byref(by)), ctx)
        rec = {"ms_isolated": ms.value, "bytes": by.value}
        live = C.c_double()
        cnt = C.c_int64()
        if kid in (1, 3, 4) and not a.no_kernel_timing:
            N.check(lib.tv_kernel_stats(ctx, kid, C.byref(live), C.byref(cnt)), ctx)
        if cnt.value > 0:
            rec.update({"ms": live.value, "launches_timed": cnt.value})
        else:
            rec.update({"ms": ms.value, "launches_timed": 0})
        rec["GBps"] = by.value / (rec["ms"] * 1e-3) / 1e9
        kern[name] = rec

    # the plain J x behind the C-ABI (tv_jacobian_apply) with the Infinity Cache
    # flushed before every launch: the HBM figure, next to
    # the effective in-solve figure of the roofline kernel
    # (the median over >= 20 flushed reps)
    fl_ms, fl_by = C.c_double(), C.c_double()
    N.check(lib.tv_time_kernel(ctx, 10, 21, C.byref(fl_ms)), ctx)
    N.check(lib.tv_kernel_bytes(ctx, 10, C.byref(fl_by)), ctx)
    flushed = {"kernel": "jacobian_apply (J(T) x, tv_jacobian_apply: the march + the side-face pass)",
               "bytes_per_launch": fl_by.value,
               "ms_per_launch": fl_ms.value, "achieved": fl_by.value / (fl_ms.value * 1e-3) / 1e9,
               "unit": "GB/s", "frac": fl_by.value / (fl_ms.value * 1e-3) / 1e9 / HBM_PEAK_GBS,
               "timing": "HBM (flushed): 512 MiB write + read sweep before each of 21 launches, HIP events "
                         "around each launch (dispatch included), median"}
    # the same flushed launches under the rocprofv3 kernel trace of this command
    # (kernel time, no dispatch), from the committed profile summary of the
    # bench default (tools/profile_summary.py; the trace cannot run inside the
    # timed process)
    prof_file = latest_profile_summary()
    prof = None
    if not um and a.share <= 1 and nc == [400, 400, 50] and a.family == "CG" and prof_file:
        with open(prof_file) as fh:
            prof = json.load(fh)
        pf = prof.get("hbm_flushed")
        if pf:
            flushed["rocprof_median_us"] = pf["rocprof_median_us"]
            flushed["rocprof_frac"] = pf["rocprof_frac"]
            flushed["rocprof_source"] = ("committed rocprofv3 --kernel-trace of the C4 bench default, median of "
                                         f"{pf['launches']} flushed launches: " + os.path.relpath(prof_file, ROOT))
    dom = kern[names[0] if um else names[3]]
    # traffic: HBM bytes per launch of this kernel from the rocprofv3 --pmc passes
    # (FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md HBM section) of this same
    # bench command, committed under profiles/ (counters cannot be read inside
    # the timed run); traffic_source names the file
    traffic, traffic_src = None, None
    dname = names[0] if um else names[3]
    pmc_file = os.path.join(ROOT, "profiles", f"pmc_{dname}_{a.family}_{nc[0]}x{nc[1]}x{nc[2]}_n{world}"
                            + ("_gmg" if pc == "gmg" else "") + ".json")
    pmc = None
    if os.path.exists(pmc_file) and a.share <= 1:  # a share's slab is not the recorded command
        with open(pmc_file) as fh:
            pmc = json.load(fh)
        traffic = pmc.get("hbm_bytes_per_launch")
        traffic_src = "committed rocprofv3 --pmc record " + os.path.relpath(pmc_file, ROOT)
    # per-kernel traffic from the same PMC record (working dispatches only) and
    # its ratio to the algorithmic bytes: > 1 means re-reads
    for name, rec in kern.items():
        pk = (pmc or {}).get("kernels", {}).get(name)
        if pk and rec.get("bytes"):
            rec["traffic"] = pk["hbm_bytes_per_launch"]
            rec["traffic_over_algorithmic"] = pk["hbm_bytes_per_launch"] / rec["bytes"]
    roofline = {"bound": "hbm", "achieved": dom["GBps"], "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": dom["GBps"] / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                "kernel": ("jacobian_apply_unstructured (y <- J(T) x; structured topology: the 14 upper slots of "
                           "the symmetric 27-point stencil of J(T) per row, 128 B/vertex with x and y; else SELL-64, "
                           "12 B per stored entry + 16 B/vertex)" if um else
                           "pcg_iteration_single_reduction (s, p, x, r, z updates; w <- J(T) z; (r,z), (z,w), (z,z))"
                           if single else "pcg_matvec_fused (p <- z + b p; w <- J(T) p; p.w)"),
                "bytes_per_launch": dom["bytes"], "ms_per_launch": dom["ms"],
                "timing": ("effective (in-solve, Infinity-Cache assisted)" if dom["launches_timed"]
                           else "isolated"),
                "hbm_flushed": flushed}
    # the same kernel's kernel-trace mean from the committed rocprofv3 record of
    # the bench default (the in-kernel clock stamps above read ~3 % below it)
    pk = (prof or {}).get("kernels", {}).get(names[3] if not um else "")
    if pk and pk.get("rocprof_timed_steps_working_mean_us"):
        us = pk["rocprof_timed_steps_working_mean_us"]
        roofline["rocprof"] = {"ms_per_launch": us * 1e-3, "achieved": dom["bytes"] / (us * 1e-6) / 1e9,
                               "frac": dom["bytes"] / (us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                               "source": "committed rocprofv3 --kernel-trace of the bench default, working "
                                         "dispatches of the timed steps: " + os.path.relpath(prof_file, ROOT)}
    if "mg_vcycle" in kern:  # the multigrid V-cycle as a whole (every launch of one application, all levels)
        v = kern["mg_vcycle"]
        vt = (pmc or {}).get("kernels", {}).get("mg_vcycle", {}).get("hbm_bytes_per_launch")
        roofline["vcycle"] = {"achieved": v["GBps"], "frac": v["GBps"] / HBM_PEAK_GBS, "unit": "GB/s",
                              "bytes_per_cycle": v["bytes"], "ms_per_cycle": v["ms"], "traffic": vt,
                              "traffic_source": traffic_src if vt else None,
                              "timing": "isolated: back-to-back V-cycles on the current state (tv_time_kernel 11)"}

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline and a.share <= 1:
        if um:
            cpu = {"value": None, "unit": "DOF-updates/s", "cores": 0, "kind": "port",
                   "sample": "no unstructured path in oracle/tv_cpu.c (the numpy oracle covers its parity only)"}
        else:
            cpu = cpu_baseline(nc, L, mp, a.cpu_seconds, a.thermal_only, a.family, pc)

    prob.close()
    if rank == 0:
        value = n_global * a.steps / elapsed
        out = {
            "metric": f"DOF-updates/sec ({'thermal Newton' if a.thermal_only else 'coupled thermo-visco'} "
                      f"time step, 3D {a.family}1 hex)",
            "value": value,
            "unit": "DOF-updates/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": a.scaling,
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (uniform T_0 = 800 K initial state, main.py parameters)",
            "config": {"workload": ("distorted-hex " if um else "")
                                   + f"{cname} 3D plate {a.family}1/{a.family}1 {nc[0]}x{nc[1]}x{nc[2]} hex "
                                   f"({n_global} T-dofs), dt 0.1, "
                                   + ("thermal-only" if a.thermal_only else "coupled 6-term Prony"),
                       "parallelism": (f"ONE rank's share (partition {a.share // 2} of {a.share}, its slab of "
                                       f"{n_owned} owned T-dofs) on one GPU, "
                                       + ("the production RCCL groups on a one-rank loopback communicator "
                                          "(self send/receive pairs; one-rank all-reduces are local copies)"
                                          if a.comm == "loopback" else "communication stubbed")
                                       + f", iterations fixed at {a.share_its} (Newton per step, Krylov per solve): "
                                       "the per-rank step without cross-GPU transfer time, not a multi-GPU "
                                       "measurement"
                                       if a.share > 1 else
                                       "single GPU, one partition (no communication)" if world == 1 else
                                       (f"RCB cell partition x{world} with a ghost-cell layer ("
                                        if um else f"mesh partition along y x{world} (")
                                       + ("RCCL halo + allreduce" if a.comm == "rccl" else "host-staged gloo") + ")"),
                       "newton_its_per_step": nits / a.steps, "krylov_its_per_step": kits / a.steps,
                       "output": (f"T, phi, Tf, xi, sigma written every step (async XDMF) to {a.output}"
                                  if a.output else "none (reference writes VTX/XDMF every step)"),
                       "krylov_form": ("single-reduction (Chronopoulos-Gear) Jacobi-PCG" if single
                                       else "PETSc KSPCG Jacobi-PCG" if pc == "jacobi"
                                       else "PETSc KSPCG, smoothed-aggregation AMG preconditioner (additive "
                                       "level 0)" if pc == "amg"
                                       else "single-reduction (Chronopoulos-Gear) CG, geometric-multigrid V-cycle "
                                       "preconditioner, three ghost planes per slab interface" if mg_single
                                       else "PETSc KSPCG, geometric-multigrid V-cycle preconditioner"),
                       "preconditioner": pc,
                       "visco_fields": "state (T, Tf, Tf_partial, phi, xi, s_tilde, sigma_tilde, sigma)"},
            "roofline": roofline,
            "kernels": kern,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))


class _StdoutToStderr:
    """fd 1 -> fd 2 while RCCL initialises (its version banner goes to stdout;
    the bench's stdout must hold the JSON line only)"""
    def __enter__(self):
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        sys.stdout.flush()
        os.dup2(self.saved, 1)
        os.close(self.saved)


def latest_profile_summary():
    """the newest committed profiles/rNN_profile_summary.json (tools/profile_summary.py)"""
    import glob
    fs = sorted(glob.glob(os.path.join(ROOT, "profiles", "r[0-9][0-9]_profile_summary.json")))
    return fs[-1] if fs else None


def cpu_baseline(nc, L, mp, seconds, thermal_only, family="CG", pc="jacobi"):
    """Time the oracle's C/OpenMP restatement (oracle/tv_cpu.c, a port of the same
    algorithm) on a bounded sample of the same workload: the same mesh and
    physics, as many full time steps as fit ~`seconds` (at least one)."""
    try:
        from oracle import tv_cpu
    except Exception as e:  # the baseline is reported, never required
        return {"value": None, "unit": "DOF-updates/s", "cores": 0, "kind": "port", "sample": f"unavailable: {e}"}
    return tv_cpu.time_baseline(nc, L, mp, seconds, thermal_only, family, pc)


if __name__ == "__main__":
    main()
