"""The partitioned (multi-GPU) path.

CPU (gloo, world size 2): the host-only partition layout of every rank tiles
the global dof range, ghost planes match the neighbours' owned boundary
planes, and the host-staged transport callbacks move the right bytes.
GPU: P partitions on one GPU (host-staged comm) reproduce the single-partition
solution (tools/partition_check.py).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _have_lib():
    try:
        from tvfem import load_library
        load_library()
        return True
    except Exception:
        return False


@pytest.mark.parametrize("cells,world,axis", [((8, 30, 5), 3, 1), ((400, 400, 50), 8, 1), ((6, 5, 40), 4, 2),
                                              ((12, 9), 2, -1)])
def test_partition_layout_tiles_global_range(cells, world, axis):
    if not _have_lib():
        pytest.skip("libtvfem.so not built")
    from tvfem import box_mesh
    from tvfem.parallel import partition_layout
    mesh = box_mesh([1.0] * len(cells), list(cells))
    lays = [partition_layout(mesh, world, p, axis) for p in range(world)]
    total = int(np.prod([c + 1 for c in cells]))
    off = 0
    for p, L in enumerate(lays):
        assert L["global_offset"] == off
        off += L["n_owned"]
        assert L["ghost_lo"] == (p > 0) and L["ghost_hi"] == (p < world - 1)
        plane = L["nodes"][0] * L["nodes"][1]
        assert L["n_local"] == L["n_owned"] + plane * (L["ghost_lo"] + L["ghost_hi"])
        if p > 0:
            assert lays[p - 1]["planes"][1] == L["planes"][0]
    assert off == total


def _gloo_worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sys.path.insert(0, os.path.join(ROOT, "fem-glass-tempering_amd"))
    import ctypes as C
    from tvfem import box_mesh
    from tvfem.parallel import partition_layout
    from tvfem import _native as N
    mesh = box_mesh([1.0, 2.0, 1.0], [4, 9, 3])
    L = partition_layout(mesh, world, rank, 1)
    plane = L["nodes"][0] * L["nodes"][1]
    # emulate one halo exchange through the same callbacks init_host_comm installs
    import numpy as np
    import torch
    glob = np.arange(int(np.prod(L["nodes"])), dtype=np.float64)
    b0, b1 = L["planes"]
    lo = b0 - (1 if L["ghost_lo"] else 0)
    local = np.full(L["n_local"], -1.0)
    local[(b0 - lo) * plane:(b1 - lo) * plane] = glob[b0 * plane:b1 * plane]
    holder = type("P", (), {})()
    holder._lib = None

    def sendrecv(s, peer):
        t = torch.from_numpy(s.copy())
        r = torch.empty_like(t)
        for qq in (dist.isend(t, peer), dist.irecv(r, peer)):
            qq.wait()
        return r.numpy()
    if L["ghost_lo"]:
        local[:plane] = sendrecv(local[plane:2 * plane], rank - 1)
    if L["ghost_hi"]:
        local[-plane:] = sendrecv(local[-2 * plane:-plane], rank + 1)
    ok = bool(np.array_equal(local, glob[lo * plane:lo * plane + L["n_local"]]))
    # allreduce callback semantics
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t)
    ok = ok and t.item() == world * (world + 1) / 2
    q.put((rank, ok))
    dist.destroy_process_group()


def test_gloo_two_rank_halo_exchange_cpu():
    if not _have_lib():
        pytest.skip("libtvfem.so not built")
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29600 + os.getpid() % 200
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok in res), res


def _partition_check(world, comm, port, extra=(), krylov_slack=1):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tools", "partition_check.py"),
           "--comm", comm, *extra]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("PARTITION_CHECK ")]
    assert line, out.stdout[-2000:] + out.stderr[-2000:]
    res = json.loads(line[0].split(" ", 1)[1])
    print("[partition] " + json.dumps(res))
    assert res["T"] < 1e-12, res
    assert res["phi"] < 1e-11, res
    assert res["xi"] < 1e-6, res
    assert res["sigma"] < 1e-6, res
    # the global reductions make the partitioned solve take the same iterations
    # up to the summation order of the dot products: within max(krylov_slack per
    # Newton solve, 5 %) -- the rule the oracle comparisons use (check_counts);
    # DG Jacobi-PCG runs ~50 iterations per solve, where rounding moves the
    # threshold crossing by a few (krylov_slack None: a partition-dependent
    # preconditioner, Newton counts only)
    for (n1, k1), (n2, k2) in zip(res["its_parts"], res["its_single"]):
        assert n1 == n2 and (krylov_slack is None or abs(k1 - k2) <= max(krylov_slack * n1, 0.05 * k2)), res
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("pcg", ["single", "kspcg"])
@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_run_matches_single_partition(world, pcg):
    """P partitions on one GPU (host-staged transport) vs one partition, with
    the single-reduction iteration (the partitioned default: lagged logic, one
    all-reduce + packed w halo per iteration) and with PETSc KSPCG as written."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _partition_check(world, "host", 29700 + world + (10 if pcg == "kspcg" else 0), ("--pcg", pcg))


@pytest.mark.gpu
@pytest.mark.parametrize("pcg", ["kspcg", "auto"])
@pytest.mark.parametrize("world,rep", [(2, 0), (3, 0), (2, 200), (3, 200), (3, 1)])
def test_partitioned_gmg_matches_single_partition(world, rep, pcg):
    """The geometric-multigrid preconditioner on a partitioned box (the solver
    of the single-GPU line, distributed: tv_mgdist.cpp) reproduces the
    single-partition GMG run: T <= 1e-12, equal Newton counts, Krylov counts
    within one per Newton solve.  On the 10 x 30 x 5 box of partition_check the
    hierarchy has three levels (31 -> 16 -> 9 planes along the partition axis);
    `rep` is the replication bound: 0 (default) keeps only level 0
    distributed, 200 levels 0-1 (level 2 replicated, 108 nodes), 1 all three
    (the coarsest level's solve distributed too).  Both Krylov forms run on
    deep-ghost slabs (three ghost planes: the V-cycle's level-0 vectors are
    computed on them and need no exchange of their own): KSPCG as written, and
    AUTO -- the single-reduction form, one all-reduce + ghost group per
    iteration (tv_mgdist.cpp pcg_solve_mg_dist_cgs)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _partition_check(world, "host", 29750 + 10 * world + (rep % 7) + (pcg == "auto") * 100,
                     ("--pc", "gmg", "--mg-replicate", str(rep), "--pcg", pcg, "--mg-coupling", "global"))


@pytest.mark.gpu
def test_partitioned_output_series():
    """The writers on a slab-partitioned box, one directory per part holding
    its owned planes: the written T and sigma equal the gathered state."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _partition_check(2, "host", 29748, ("--steps", "2", "--output"))
    assert res["output_T"] == 0.0 and res["output_sigma"] == 0.0, res


@pytest.mark.gpu
@pytest.mark.parametrize("coupling,world,rep", [("global", 2, 0), ("global", 3, 0), ("global", 3, 1),
                                                ("local", 2, 0), ("local", 3, 0)])
def test_partitioned_vcycle_operator_matches_restatement(coupling, world, rep):
    """The partitioned V-cycle in isolation (tv_precond_apply on every rank,
    host-staged transport): GLOBAL coupling -- its per-level ghost exchanges and
    the replicated levels' all-reduce -- reproduces the single-partition V-cycle
    of the whole box; LOCAL coupling (block Jacobi) each rank's block of the
    numpy restatement (tests/gmg_reference.py).  1e-11, symmetric, positive."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(29770 + 3 * world + rep + (coupling == "local") * 20),
           os.path.join(ROOT, "tests", "vcycle_part_check.py"), "--coupling", coupling, "--mg-replicate", str(rep)]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("VCYCLE_CHECK ")]
    assert line, out.stdout[-2000:] + out.stderr[-3000:]
    res = json.loads(line[0].split(" ", 1)[1])
    print("[vcycle-part]", json.dumps(res), flush=True)
    assert res["err"] < 1e-11 and res["sym"] < 1e-12 and res["rBr"] > 0.0, res


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_local_gmg_solves(world):
    """LOCAL coupling (block-Jacobi V-cycle, opt-in; AUTO = GLOBAL): the
    Newton solution equals the single partition's (T <= 1e-12; the Krylov
    tolerance is met either way), the Newton counts too; the Krylov counts may
    differ (they depend on the partition count, as PCGAMG's do)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _partition_check(world, "host", 29790 + world, ("--pc", "gmg", "--pcg", "kspcg", "--mg-coupling", "local"),
                           krylov_slack=None)
    print("[local-gmg]", json.dumps(res), flush=True)


@pytest.mark.gpu
@pytest.mark.parametrize("world,kernel", [(2, "tile"), (3, "tile"), (3, "cells")])
def test_partitioned_dg_matches_single_partition(world, kernel):
    """DG1 temperature and stress on slabs of cell layers (the SIPG facets of
    the interfaces read one ghost cell layer, exchanged with all 8 cell-local
    dofs): Jacobi-PCG on 2 / 3 partitions reproduces the single partition --
    T <= 1e-12, equal Newton counts -- with the marching tile kernel and the
    one-thread-per-cell kernel (ThermoViscoProblem.py:308-325 under mpiexec)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _partition_check(world, "host", 29780 + world + (kernel == "cells") * 5,
                     ("--family", "DG", "--dg-kernel", kernel, "--pcg", "kspcg", "--steps", "3"))


@pytest.mark.gpu
@pytest.mark.parametrize("world,family", [(2, "DG"), (3, "DG"), (2, "DG-CG"), (3, "DG-CG")])
def test_partitioned_dg_gmg_matches_single_partition(world, family):
    """The DG1 -> CG1 multigrid on slabs of cell layers (tv_mgsolve.cpp
    mg_setup: the CG levels replicated, the owned cells restricted into the
    vertex planes they touch and summed by one all-reduce, the prolongation
    into every local cell): DG/DG and the reference's main.py pairing DG T /
    CG sigma reproduce the single-partition DG multigrid run (T <= 1e-12,
    equal Newton counts, Krylov within one per Newton solve -- the level-1
    sums add in another order, and the smoother weight's power iteration starts
    from the partition-major vector); the reference runs this under mpiexec
    with PCGAMG (ThermoViscoProblem.py:343-346, main.py:24-27)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _partition_check(world, "host", 29810 + world + (family == "DG-CG") * 5,
                     ("--family", family, "--pc", "gmg", "--pcg", "kspcg", "--steps", "3"))


@pytest.mark.gpu
def test_partitioned_dg_output_series():
    """The writers on a DG1 slab partition: each part writes the discontinuous
    fields of its owned cell layers; concatenated they equal the gathered state."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _partition_check(2, "host", 29777, ("--family", "DG", "--steps", "2", "--output"))
    assert res["output_T"] == 0.0 and res["output_sigma"] == 0.0, res


@pytest.mark.gpu
@pytest.mark.parametrize("family", ["DG-CG", "CG-DG"])
@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_mixed_families_match_single_partition(world, family):
    """Mixed element families on slabs: DG1 T / CG1 sigma -- the reference's own
    main.py pairing (main.py:24-27) under mpiexec -- and CG1 T / DG1 sigma.  The
    T space is partitioned as on its own, the sigma space follows without ghosts
    (setup_mixed_part): each sigma dof reads the T-space state of the dof that
    fem::interpolate's last-writer rule picks, an owned dof or one of the ghost
    layer above.  2 / 3 partitions reproduce the single partition (T <= 1e-12,
    sigma <= 1e-6, equal Newton counts), and every part's written series equals
    the gathered state over its output mesh (the nodes of its owned cell layers)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _partition_check(world, "host", 29790 + world + (family == "CG-DG") * 7,
                           ("--family", family, "--pcg", "kspcg", "--steps", "3", "--output"))
    assert res["output_T"] == 0.0 and res["output_sigma"] == 0.0, res


@pytest.mark.gpu
def test_partitioned_mixed_families_host_edit():
    """A host edit of a T-space state field (Tf_partial: Tf itself is recomputed
    from it every step) on one rank of a CG T / DG sigma
    slab pair: the sigma pass reads that field at the ghost plane above, so the
    edited values must reach the neighbour's ghost copy before the next update."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    # nodes on both sides of the interface planes (y = 3.0 / 3.2 of the 10 x 30 x 5 slab pair) are edited;
    # paper mode, where Tf (from Tf_partial) enters the thermal strain -- the
    # reference mode's stress reads T alone (Q2), which is exchanged every step
    _partition_check(2, "host", 29805, ("--family", "CG-DG", "--pcg", "kspcg", "--steps", "2", "--edit", "--paper",
                                        "--edit-field", "Tf_partial", "--edit-box", "0,0.6,2.5,3.5"))


@pytest.mark.gpu
@pytest.mark.parametrize("pc", ["jacobi", "gmg"])
def test_partitioned_dirichlet_matches_single_partition(pc):
    """Paper mode with T = T_ambient on the exterior boundary on 2 slabs: the
    lifting vector dB is exchanged before J dB, each slab masks its own
    constrained rows; Jacobi and the distributed multigrid reproduce the
    single partition."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _partition_check(2, "host", 29760 + (pc == "gmg"), ("--dirichlet", "--steps", "2", "--pc", pc, "--pcg", "kspcg",
                                                        "--mg-coupling", "global"))


@pytest.mark.gpu
def test_auto_krylov_form_agrees_across_ranks():
    """pcg_variant AUTO must pick the same Krylov form on every rank (the two
    forms issue different collectives).  A 400 x 292 x 50 plate on 2 ranks gives
    slabs of 146 and 147 planes of 401 x 51 nodes, 2.986M and 3.006M owned nodes,
    on both sides of the 3M single-reduction bound: the choice follows the
    largest slab, so both ranks take KSPCG."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tvfem import box_mesh
    from tvfem.problem import ThermoViscoProblem
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from partition_check import CFG, MP
    mesh = box_mesh([50.0, 36.5, 5.0], [400, 292, 50])
    forms, owned = [], []
    for part in range(2):
        p = ThermoViscoProblem(mesh, (0, 1), 0.1, CFG, MP, n_parts=2, part=part, part_axis=1, verbose=False,
                               materialize=False, pcg_variant="auto")
        forms.append(p.pcg_variant)
        owned.append(p.num_dofs(0)[0])
        p.close()
    assert owned[0] < 3_000_000 < owned[1], owned
    assert forms == ["kspcg", "kspcg"], forms


@pytest.mark.gpu
def test_partitioned_host_edit_on_one_rank():
    """A host-side in-place edit of T made by one rank only (a local hot spot
    after setup()) must neither hang the other rank nor leave stale ghost
    planes: tv_set_field is local, and every rank refreshes the T / T_prev
    ghosts collectively at the start of the step (ThermoViscoProblem.py:351's
    scatter_forward).  Compared with the same edit on one partition."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _partition_check(2, "host", 29745, ("--edit", "--steps", "3"))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_rccl_partitioned_run_matches_single_partition(world):
    """The production transport: one rank per GPU, RCCL grouped send/recv of the
    ghost planes and ncclAllReduce of the PCG / Newton sums over xGMI (replaces
    dolfinx scatter_forward, ThermoViscoProblem.py:351, and PETSc's MPI
    reductions).  Needs `world` GPUs; skipped on smaller boxes."""
    import torch
    n = torch.cuda.device_count()  # does not initialise the GPU in this process
    if n < world:
        pytest.skip(f"{world} GPUs needed, {n} visible")
    _partition_check(world, "rccl", 29720 + world, ("--cells", "12,48,6"))
    _partition_check(world, "rccl", 29730 + world, ("--cells", "12,48,6", "--pc", "gmg", "--pcg", "kspcg",
                                                     "--mg-coupling", "global"))
    _partition_check(world, "rccl", 29740 + world, ("--cells", "12,48,6", "--pc", "gmg", "--pcg", "kspcg",
                                                     "--mg-coupling", "local"), krylov_slack=None)


@pytest.mark.gpu
def test_bench_two_rank_rehearsal():
    """bench.py's distributed flow (barriers, max-over-ranks timing, rank-0 JSON
    line) at world size 2 with the host-staged transport, both ranks on GPU 0."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", "29711", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--comm", "host", "--cells", "40,40,10", "--steps", "2", "--warmup", "1",
           "--kernel-reps", "2", "--no-cpu-baseline"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stdout[-2000:] + out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]  # rank 0 only
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 2 and rec["steps"] == 2 and rec["value"] > 0
    assert "host-staged" in rec["config"]["parallelism"]
    assert rec["config"]["newton_its_per_step"] >= 2
