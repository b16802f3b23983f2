"""Distributed unstructured meshes: the ghosted partition plan
(tvfem.parallel.ghosted_partition, the layout tv_create_unstructured_part
takes) on CPU -- ownership, ghost layer completeness, halo plans that match
pairwise -- and the partitioned solve on the GPU (tools/partition_check.py
--mesh distorted; host-staged transport, several partitions on one GPU).

Reference: the mesh distribution of gmshio.read_from_msh(..., MPI.COMM_WORLD,
0) (ThermoViscoProblem.py:27-28) and the ghost update scatter_forward (:351)."""
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


def _plans(mesh, P):
    from tvfem.parallel import ghosted_partition, rcb_partition
    part = rcb_partition(mesh, P)
    return part, [ghosted_partition(mesh, part, p, P) for p in range(P)]


@pytest.mark.parametrize("n_cells,P,shuffle", [((6, 5, 4), 2, False), ((7, 6, 5), 3, True), ((9, 8), 4, True),
                                              ((5, 4, 6), 5, False)])
def test_ghosted_partition_plan(n_cells, P, shuffle):
    if not _have_lib():
        pytest.skip("libtvfem.so not built")
    from tvfem import distorted_box_mesh
    mesh = distorted_box_mesh([1.0] * len(n_cells), list(n_cells), shuffle=shuffle, seed=3)
    part, plans = _plans(mesh, P)
    nv = mesh.num_vertices
    cells = mesh.cells
    # owned vertices tile the global vertex set; the partition-major offsets add up
    owned = np.concatenate([g["l2g"][:g["n_owned"]] for g in plans])
    assert np.array_equal(np.sort(owned), np.arange(nv))
    offs = np.cumsum([0] + [g["n_owned"] for g in plans])[:-1]
    assert [g["global_offset"] for g in plans] == list(offs)
    owner = np.empty(nv, dtype=np.int64)
    for p, g in enumerate(plans):
        owner[g["l2g"][:g["n_owned"]]] = p
    for p, g in enumerate(plans):
        sub, l2g, no = g["mesh"], g["l2g"], g["n_owned"]
        # own cells first, in global order
        assert g["n_owned_cells"] == np.count_nonzero(part == p)
        gcells = l2g[sub.cells]
        assert np.array_equal(gcells[:g["n_owned_cells"]], cells[part == p])
        # ghost layer: every cell around an owned vertex is local (complete rows)
        need = np.flatnonzero((owner[cells] == p).any(axis=1) | (part == p))
        have = {tuple(c) for c in gcells}
        assert all(tuple(c) in have for c in cells[need])
        assert len(have) == len(need)
        # geometry carried along
        assert np.allclose(sub.x, mesh.x[l2g])
        # ghosts grouped by owner in neighbour order, ascending global ids inside a group
        go = owner[l2g[no:]]
        assert np.all(np.diff(go) >= 0)
        nb = list(g["neighbors"])
        assert nb == sorted(nb) and p not in nb
        pos = no
        for q, rc in zip(nb, g["recv_count"]):
            grp = l2g[pos:pos + rc]
            assert np.all(owner[grp] == q) and np.all(np.diff(grp) > 0)
            pos += rc
        assert pos == len(l2g)
    # pairwise: p's send list to q is q's ghost group from p, value for value
    for p, g in enumerate(plans):
        soff = np.concatenate([[0], np.cumsum(g["send_count"])])
        for k, q in enumerate(g["neighbors"]):
            h = plans[q]
            assert p in list(h["neighbors"])  # symmetric neighbour relation
            kq = list(h["neighbors"]).index(p)
            roff = h["n_owned"] + int(np.sum(h["recv_count"][:kq]))
            recv_g = h["l2g"][roff:roff + h["recv_count"][kq]]
            sent_g = g["l2g"][g["send_idx"][soff[k]:soff[k + 1]]]
            assert np.array_equal(recv_g, sent_g)
            assert np.all(g["send_idx"][soff[k]:soff[k + 1]] < g["n_owned"])


def test_ghosted_partition_single_part_is_whole_mesh():
    if not _have_lib():
        pytest.skip("libtvfem.so not built")
    from tvfem import distorted_box_mesh
    from tvfem.parallel import ghosted_partition
    mesh = distorted_box_mesh([1.0, 1.0, 1.0], [3, 4, 2], seed=1)
    g = ghosted_partition(mesh, np.zeros(mesh.num_cells, dtype=np.int32), 0, 1)
    assert g["n_owned"] == mesh.num_vertices and len(g["neighbors"]) == 0
    assert np.array_equal(g["l2g"], np.arange(mesh.num_vertices))
    assert np.array_equal(g["mesh"].cells, mesh.cells)


def _partition_check(world, port, extra=(), krylov_slack=1):
    import json
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tools", "partition_check.py"),
           "--comm", "host", "--mesh", "distorted", *extra]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("PARTITION_CHECK ")]
    assert line, out.stdout[-2000:] + out.stderr[-2000:]
    res = json.loads(line[0].split(" ", 1)[1])
    print("[upartition]", json.dumps(res), flush=True)
    assert res["T"] < 1e-12, res
    assert res["phi"] < 1e-11, res
    assert res["xi"] < 1e-6, res
    assert res["sigma"] < 1e-6, res
    for (n1, k1), (n2, k2) in zip(res["its_parts"], res["its_single"]):
        assert n1 == n2 and (krylov_slack is None or abs(k1 - k2) <= krylov_slack * n1), res
    return res


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_unstructured_matches_single_partition(world):
    """P partitions of a distorted hexahedral plate (RCB + ghost layer, one GPU,
    host-staged halo of the ghost vertices) reproduce the single-partition
    unstructured solve: T <= 1e-12, equal Newton counts, Krylov within one per
    Newton solve (the reductions sum in a different order)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _partition_check(world, 29810 + world, ("--cells", "10,30,5"))


@pytest.mark.gpu
def test_partitioned_unstructured_output():
    """The writers on a partitioned unstructured mesh (ThermoViscoProblem.py:
    246-276, one directory per part): each part writes its own cells over its
    local vertices, and the written T and sigma -- ghost vertices included,
    whose visco state evolves on the part itself -- equal the gathered
    owners' values exactly."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _partition_check(2, 29817, ("--cells", "10,30,5", "--steps", "2", "--output"))
    assert res["output_T"] == 0.0 and res["output_sigma"] == 0.0, res


@pytest.mark.gpu
def test_partitioned_unstructured_host_edit():
    """A host edit of T on the owning rank only, then the collective ghost
    refresh at the start of the step (as the box partition does)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _partition_check(2, 29816, ("--cells", "10,30,5", "--edit", "--steps", "3"))


@pytest.mark.gpu
@pytest.mark.parametrize("field", ["Tf", "Tf_partial", "xi"])
def test_partitioned_unstructured_host_edit_state_field(field):
    """A host edit of a viscoelastic state field on the owning rank only: the
    ghost copies of that field are refreshed from their owners at the next
    step (one all-reduce of the per-field write flags, then the halo of the
    written fields), so every part's ghost vertices keep evolving as their
    owners do and the written series agree at shared vertices."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _partition_check(2, 29830, ("--cells", "10,30,5", "--edit", "--edit-field", field, "--steps", "2",
                                      "--output"))
    assert res["output_T"] == 0.0 and res["output_sigma"] == 0.0, res


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_unstructured_amg(world):
    """The smoothed-aggregation AMG on a distributed distorted mesh: every rank
    gathers the global fine operator (partition-major numbering) at its first
    solve and builds the same hierarchy; level 0 restricts its owned rows, one
    all-reduce forms the level-1 right-hand side, the coarse cycle runs
    replicated.  T reproduces the single-partition AMG run (<= 1e-12, equal
    Newton counts) and the Krylov counts stay within 1.5x of it (its aggregates
    follow the input numbering, the partitioned ones the partition-major)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    res = _partition_check(world, 29840 + world, ("--cells", "16,30,10", "--steps", "2", "--pc", "amg"),
                           krylov_slack=None)
    print("[upartition-amg]", res["its_parts"], res["its_single"], flush=True)
    ka = sum(k for _, k in res["its_parts"])
    ks = sum(k for _, k in res["its_single"])
    assert ka <= 1.5 * ks, res


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 3])
def test_partitioned_unstructured_dirichlet(world):
    """Paper mode with T = T_ambient on the exterior boundary on a distributed
    distorted mesh: each part constrains its owned boundary vertices, the
    lifting vector's ghosts come from their owners before J dB; the parts
    reproduce the single partition."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    _partition_check(world, 29833 + world, ("--cells", "10,30,5", "--dirichlet", "--steps", "2"))


@pytest.mark.gpu
@pytest.mark.parametrize("world", [2, 4, 8])
def test_rccl_partitioned_unstructured(world):
    """The production transport for the unstructured partition: one rank per
    GPU, RCCL grouped send / recv of the packed ghost values per neighbour
    and ncclAllReduce of the PCG / Newton sums.  Needs `world` GPUs."""
    import json
    import torch
    n = torch.cuda.device_count()  # does not initialise the GPU in this process
    if n < world:
        pytest.skip(f"{world} GPUs needed, {n} visible")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(29820 + world),
           os.path.join(ROOT, "tools", "partition_check.py"), "--comm", "rccl", "--mesh", "distorted",
           "--cells", "12,48,6"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("PARTITION_CHECK ")]
    assert line, out.stdout[-2000:] + out.stderr[-2000:]
    res = json.loads(line[0].split(" ", 1)[1])
    assert res["T"] < 1e-12 and res["sigma"] < 1e-6, res
