"""Partitioned run vs the single-partition run of the same mesh: T, phi, xi and
sigma must agree, and the Newton / Krylov iteration counts too.  Launched by
tests/test_partition.py as `torch.distributed.run --nproc-per-node P`.

    --comm host   every rank on GPU 0, host-staged transport over gloo (one GPU)
    --comm rccl   rank r on GPU r (LOCAL_RANK), RCCL send/recv + allreduce over
                  xGMI: the production transport (needs P GPUs)
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fem-glass-tempering_amd"))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from tvfem import box_mesh, distorted_box_mesh  # noqa: E402
from tvfem.parallel import init_host_comm, init_rccl  # noqa: E402
from tvfem.problem import ThermoViscoProblem  # noqa: E402

MP = {"f": 0.0, "epsilon": 0.93, "sigma": 5.670e-8, "T_ambient": 600.0, "T_0": 800.0, "alpha": 1.0, "htc": 280.1,
      "rho": 2500.0, "cp": 1433.0, "k": 1.0, "H": 627.8e3, "Tb": 869.0, "Rg": 8.314, "alpha_solid": 9.1e-6,
      "alpha_liquid": 25.1e-6}
CFG = {"T": {"element": "CG", "degree": 1}, "sigma": {"element": "CG", "degree": 1}}


def run(mesh, n_parts, part, steps, comm=None, device=0, pcg="auto", edit=False, pc="jacobi", mg_rep=0,
        outdir=None, dirichlet=False, edit_field="T", mg_coupling="auto", family="CG", dg_kernel="auto",
        edit_box=(0.0, 0.6, 0.0, 0.6), paper=False):
    fam_T, fam_S = family.split("-") if "-" in family else (family, family)  # "DG-CG": DG T, CG sigma (main.py)
    cfg = {"T": {"element": fam_T, "degree": 1}, "sigma": {"element": fam_S, "degree": 1}}
    p = ThermoViscoProblem(mesh, (0, 1), 0.1, cfg, MP, device=device, n_parts=n_parts, part=part, part_axis=1,
                           dg_kernel=dg_kernel,
                           verbose=False, pcg_variant=pcg, write_output=outdir is not None,
                           output_dir=outdir or "output", preconditioner=pc, mg_replicate_nodes=mg_rep,
                           model_mode="paper" if (dirichlet or paper) else "reference", mg_coupling=mg_coupling)
    if comm is not None:
        comm(p)
        if n_parts > 1:  # every exchange pattern on id-valued vectors first (collective)
            import ctypes as C
            nchk, nbad = C.c_int64(), C.c_int64()
            rc = p._lib.tv_comm_check(p._ctx, C.byref(nchk), C.byref(nbad))
            if rc != 0 or nbad.value or not nchk.value:
                raise SystemExit(f"tv_comm_check: rc {rc}, {nbad.value} of {nchk.value} values wrong")
    if dirichlet:  # paper mode with T = T_ambient on the boundary (tv_set_dirichlet)
        p.setup(dirichlet_bc=True)
    else:
        p.setup()
    if edit:
        # a local hot spot written in place on the host by the ranks that own it
        # (rank 0 only when partitioned): the ghost planes must still follow
        X = p._dof_coordinates(0)
        x0, x1, y0, y1 = edit_box
        m = (X[:, 0] >= x0) & (X[:, 0] < x1) & (X[:, 1] >= y0) & (X[:, 1] < y1)
        if m.any():
            if edit_field == "T":
                p.functions_current["T"].x.array[m] += 20.0
            else:  # a T-space state field other than T: its ghost copies must follow too
                arr = (p.functions_current if edit_field in p.functions_current else p.functions)[edit_field].x.array
                bs = arr.size // m.size
                arr.reshape(-1, bs)[m] += 20.0
    its = []
    for _ in range(steps):
        p.solve_timestep()
        its.append((p.last_newton_iterations, p.last_krylov_iterations))
    out = {k: p.get_field(k) for k in ("T", "phi", "xi", "sigma")}
    import ctypes as C
    for sp in (0, 1):  # global offset of the part's first owned dof per space (its written series start there)
        no, go = C.c_int64(), C.c_int64()
        p._lib.tv_num_dofs(p._ctx, sp, C.byref(no), C.byref(go))
        out["goff%d" % sp] = np.array([go.value])
    up = getattr(p, "_upart", None)
    if up is not None:  # unstructured partition: owned vertices -> global ids
        out["l2g"] = up["l2g"][:up["n_owned"]]
    p.close()
    if outdir is not None:  # the last step of the written T and sigma series (this part's directory)
        from tvfem.xdmf import read_series
        d = os.path.join(outdir, f"part{part}") if n_parts > 1 else outdir
        out["outT"] = np.asarray(read_series(os.path.join(d, "T.xdmf"))["values"][-1]).ravel()
        out["outS"] = np.asarray(read_series(os.path.join(d, "sigma.xdmf"))["values"][-1]).ravel()
        if up is not None:
            out["l2g_local"] = up["l2g"]
    return out, its


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--comm", choices=["host", "rccl"], default="host")
    ap.add_argument("--cells", default="10,30,5")
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--pcg", choices=["auto", "kspcg", "single"], default="auto")
    ap.add_argument("--edit", action="store_true", help="host edit of T on the owning rank only, after setup()")
    ap.add_argument("--edit-field", default="T", help="--edit: the field edited (T, Tf, Tf_partial, phi, xi)")
    ap.add_argument("--edit-box", default="0,0.6,0,0.6",
                    help="--edit: x0,x1,y0,y1 of the edited nodes (an interface plane inside: the ghost copies follow)")
    ap.add_argument("--paper", action="store_true",
                    help="paper model mode (Tf_partial / Tf feed the stress; the reference mode's stress reads T only)")
    ap.add_argument("--dirichlet", action="store_true", help="paper mode with the Dirichlet condition T = T_ambient")
    ap.add_argument("--family", choices=["CG", "DG", "DG-CG", "CG-DG"], default="CG",
                    help="element family of T and sigma (one name: both; DG-CG: DG T and CG sigma, main.py's pairing)")
    ap.add_argument("--dg-kernel", choices=["auto", "tile", "cells"], default="auto")
    ap.add_argument("--mg-coupling", choices=["auto", "global", "local"], default="auto",
                    help="partitioned GMG: the distributed V-cycle of the whole box, or each slab's own (block Jacobi)")
    ap.add_argument("--pc", choices=["jacobi", "gmg", "amg"], default="jacobi")
    ap.add_argument("--mesh", choices=["box", "distorted"], default="box",
                    help="distorted: the box as a general hexahedral mesh (tv_um.hip), RCB cell partition + ghost layer")
    ap.add_argument("--output", action="store_true",
                    help="write the five series (per-part directories) and check them against the gathered state")
    ap.add_argument("--mg-replicate", type=int, default=0,
                    help="GMG: coarse levels of at most this many nodes replicated (0: the library default)")
    a = ap.parse_args()
    rank = int(os.environ["RANK"])
    world = int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", rank))
    dist.init_process_group("gloo")
    eb = tuple(float(v) for v in a.edit_box.split(","))
    nc = [int(v) for v in a.cells.split(",")]
    mesh = (distorted_box_mesh if a.mesh == "distorted" else box_mesh)([2.0, 6.0, 1.0], nc)
    steps = a.steps
    outdir = None
    if a.output:
        import tempfile
        outdir = tempfile.mkdtemp(prefix=f"pcheck{rank}_")
    if a.comm == "rccl":
        if torch.cuda.device_count() < world:
            raise SystemExit(f"--comm rccl needs {world} GPUs, {torch.cuda.device_count()} visible")
        loc, its = run(mesh, world, rank, steps, comm=lambda p: init_rccl(p, rank, world, dist), device=local,
                       pcg=a.pcg, edit=a.edit, pc=a.pc, mg_rep=a.mg_replicate, outdir=outdir,
                       dirichlet=a.dirichlet, edit_field=a.edit_field, mg_coupling=a.mg_coupling, family=a.family,
                       dg_kernel=a.dg_kernel, edit_box=eb, paper=a.paper)
    else:
        loc, its = run(mesh, world, rank, steps, comm=lambda p: init_host_comm(p, rank, world), pcg=a.pcg,
                       edit=a.edit, pc=a.pc, mg_rep=a.mg_replicate, outdir=outdir, dirichlet=a.dirichlet,
                       edit_field=a.edit_field, mg_coupling=a.mg_coupling, family=a.family, dg_kernel=a.dg_kernel,
                       edit_box=eb, paper=a.paper)
    gathered = [None] * world
    dist.all_gather_object(gathered, {k: v.tolist() for k, v in loc.items()})
    if rank == 0:
        ref, its_ref = run(mesh, 1, 0, steps, edit=a.edit, pc=a.pc, dirichlet=a.dirichlet, edit_field=a.edit_field,
                           family=a.family, dg_kernel=a.dg_kernel, edit_box=eb, paper=a.paper)
        res = {"comm": a.comm, "pcg": a.pcg, "pc": a.pc, "mesh": a.mesh, "its_parts": its, "its_single": its_ref}
        for k in ("T", "phi", "xi", "sigma"):
            if "l2g" in gathered[0]:  # scatter every part's owned vertices to their global ids
                full = np.zeros_like(ref[k]).reshape(mesh.num_vertices, -1)
                for g in gathered:
                    full[np.asarray(g["l2g"], dtype=np.int64)] = np.asarray(g[k]).reshape(len(g["l2g"]), -1)
                full = full.ravel()
            else:
                full = np.concatenate([np.asarray(g[k]) for g in gathered])
            e = np.linalg.norm(full - ref[k]) / np.linalg.norm(ref[k])
            res[k] = float(e)
            if a.output and k in ("T", "sigma"):  # every part's written series vs the gathered state
                key = "outT" if k == "T" else "outS"
                if "l2g_local" in gathered[0]:  # unstructured: the part's local vertices, ghosts included
                    fr = full.reshape(mesh.num_vertices, -1)
                    errs = [np.abs(np.asarray(g[key]) - fr[np.asarray(g["l2g_local"], dtype=np.int64)].ravel()).max()
                            for g in gathered]
                else:  # box: each part's series is the global range from its first owned dof (owned planes or
                    # cell layers, plus the shared plane above of a mixed-family slab)
                    bs = 1 if k == "T" else mesh.dim * mesh.dim
                    errs = []
                    for g in gathered:
                        wv = np.asarray(g[key])
                        o0 = int(g["goff0" if k == "T" else "goff1"][0]) * bs
                        errs.append(np.abs(wv - full[o0:o0 + wv.size]).max() if wv.size else 0.0)
                res["output_" + k] = float(max(errs) / np.abs(full).max())
        print("PARTITION_CHECK " + json.dumps(res), flush=True)
    dist.barrier()


if __name__ == "__main__":
    main()
