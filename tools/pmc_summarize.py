"""Summarise two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) into HBM bytes
per launch for the hot-path kernels, with the gfx950 correction of
/opt/skills/guides/MI355X_MICROARCH.md §HBM (FETCH_SIZE counts half of wide
streaming reads: doubled here; WRITE_SIZE taken as is).  Counter values are in
KB (rocprofv3 derived-counter unit) -> bytes x1024.

    python tools/pmc_summarize.py FETCH_DIR WRITE_DIR OUT.json [DOMINANT [JX_FETCH_DIR JX_WRITE_DIR]]

JX_*: passes of `pmc_kernels.py --jx-only` (flushed plain J x launches): the
jacobian_apply record comes from them (the multigrid solve itself may run no
fine-grid J x: the fused residual restriction).

DOMINANT (default pcg_matvec_fused) names the group whose per-launch bytes are
the record's top-level hbm_bytes_per_launch (bench.py's roofline.traffic).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

GROUPS = {
    "pcg_matvec_fused": ("k_cg_march<1, true",),  # marching tiles + face workgroups, one launch
    "pcg_update": ("k_pcg_update",),
    "visco_update": ("k_visco_fused",),
    "jacobian_apply": ("k_cg_march<1, false, 8, 1, 2, false",),  # the FINE-grid plain J x (largest grid; V-cycle x0)
    "dg_matvec_fused": ("k_dg_tile<true",),
    "pcg_iteration_single_reduction": ("k_cgs_march<false",),
    "jacobian_apply_unstructured": ("k_um_march14<1>",),  # half-stencil J x (structured topology, tv_um.hip)
    "jacobian_apply_unstructured_sell": ("k_um_rows<3, 1>",),  # SELL-64 J x (general meshes)
    # multigrid kernels (pmc_kernels.py --pc gmg)
    "mg_update": ("k_mg_update",),
    "mg_post_march": ("k_cg_march<1, false, 8, 1, 2, true",),
    "mg_restrict": ("k_mg_restrict_pairs",),
    "mg_prolong": ("k_mg_prolong_blk",),
}
# one V-cycle (tv_mgsolve.cpp mg_apply0): every launch of these, all levels, per
# k_mg_post_faces dispatch (one per V-cycle)
VCYCLE = ("k_cg_march<1, false", "k_cg_addfaces", "k_mg_restrict", "k_mg_rrestrict", "k_cg_faces_all", "k_mg_prolong",
          "k_mg_jacobi", "k_mg_post_faces")


# a dispatch that did no work: a gated-off step-end launch (the visco update
# queued behind a Newton iteration that did not converge exits at its first
# instruction) or a launch queued behind a converged Krylov solve.  Such
# dispatches are dropped: below this fraction of the group's largest dispatch
IDLE_FRAC = 0.02


def per_kernel(d, counter):
    """{kernel name: [(grid size, value), ...]} in dispatch order"""
    vals = defaultdict(list)
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                grid = int(float(row.get("Grid_Size") or row.get("Grid_Size_X") or 0))
                vals[row["Kernel_Name"]].append((grid, float(row["Counter_Value"])))
    return vals


def group_avg(vals, pats, grid_sel=None):
    """mean per dispatch of each pattern's working dispatches (idle ones dropped),
    summed over the patterns; grid_sel: "max" keeps the largest grid only (the
    fine-grid launch of a kernel that also runs on the coarse multigrid levels)"""
    tot = 0.0
    found = []
    for pat in pats:
        ks = [k for k in vals if pat in k]
        if not ks:
            return None, found
        v = [x for k in ks for x in vals[k]]
        if grid_sel == "max":
            gmax = max(g for g, _ in v)
            v = [x for x in v if x[0] == gmax]
        top = max(x for _, x in v)
        work = [x for _, x in v if x >= IDLE_FRAC * top]
        found.append((ks[0][:80], len(work), len(v) - len(work)))
        tot += sum(work) / len(work)
    return tot, found


def main():
    fdir, wdir, out = sys.argv[1:4]
    fetch = per_kernel(fdir, "FETCH_SIZE")
    write = per_kernel(wdir, "WRITE_SIZE")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate passes), tools/pmc_kernels.py",
           "correction": "FETCH_SIZE x2 (gfx950 wide-read halving), KB -> bytes x1024", "kernels": {}}
    for name, pats in GROUPS.items():
        sel = "max" if name == "jacobian_apply" else None
        fb, ff = group_avg(fetch, pats, sel)
        wb, wf = group_avg(write, pats, sel)
        if fb is None or wb is None:
            continue
        rd = 2.0 * fb * 1024.0
        wr = wb * 1024.0
        res["kernels"][name] = {"fetch_bytes": rd, "write_bytes": wr, "hbm_bytes_per_launch": rd + wr,
                                "dispatches": ff,
                                "dispatch_note": "(name, working dispatches averaged, idle dispatches dropped)"
                                                 + ("; the largest grid only (the fine level)" if sel else "")}
    ncyc = sum(len(v) for k, v in fetch.items() if "k_mg_post_faces" in k)
    if ncyc:  # (idle dispatches of a converged solve add ~0 bytes to the sums)
        fsum = sum(x for k, v in fetch.items() if any(p in k for p in VCYCLE) for _, x in v)
        wsum = sum(x for k, v in write.items() if any(p in k for p in VCYCLE) for _, x in v)
        res["kernels"]["mg_vcycle"] = {"fetch_bytes": 2.0 * fsum * 1024.0 / ncyc, "write_bytes": wsum * 1024.0 / ncyc,
                                       "hbm_bytes_per_launch": (2.0 * fsum + wsum) * 1024.0 / ncyc,
                                       "dispatches": [("V-cycles (k_mg_post_faces dispatches)", ncyc)]}
    # the code the counters were collected on (the GPU box's copy has no .git:
    # the caller passes the commit in TVFEM_GIT_HEAD)
    res["git_head"] = os.environ.get("TVFEM_GIT_HEAD")
    if len(sys.argv) > 6:  # the fine J x from its own (flushed) passes
        jf = per_kernel(sys.argv[5], "FETCH_SIZE")
        jw = per_kernel(sys.argv[6], "WRITE_SIZE")
        pats = GROUPS["jacobian_apply"]
        if not any(pats[0] in k for k in jf):  # DG1: the plain J x tile
            pats = ("k_dg_tile<false",)
        fb, ff = group_avg(jf, pats, "max")
        wb, _ = group_avg(jw, pats, "max")
        if fb is not None and wb is not None:
            res["kernels"]["jacobian_apply"] = {
                "fetch_bytes": 2.0 * fb * 1024.0, "write_bytes": wb * 1024.0,
                "hbm_bytes_per_launch": (2.0 * fb + wb) * 1024.0, "dispatches": ff,
                "dispatch_note": "pmc_kernels.py --jx-only: plain fine-grid J x, Infinity Cache flushed before each"}
    dom = sys.argv[4] if len(sys.argv) > 4 else "pcg_matvec_fused"
    if dom in res["kernels"]:
        res["dominant"] = dom
        res["hbm_bytes_per_launch"] = res["kernels"][dom]["hbm_bytes_per_launch"]
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
