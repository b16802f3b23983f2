"""Multi-GPU plumbing: one process per GPU, mesh sliced along the slowest
storage axis (one ghost node plane per interface), RCCL over xGMI for the ghost
planes and the PCG / Newton dot products.

Replaces the reference's MPI layer (mpi4py COMM_WORLD at
ThermoViscoProblem.py:28, dolfinx Scatterer::scatter_forward at :351 and the
PETSc MPI_Allreduce inside VecNorm / VecDot).  ``torch.distributed`` is used
only to bootstrap (broadcast the RCCL unique id) — it is plumbing, not the
data path.  ``init_host_comm`` stages through host memory over a gloo process
group instead (for running several partitions on one GPU in tests).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _native as N


def partition_layout(mesh, n_parts: int, part: int, part_axis: int = -1) -> dict:
    """Host-only layout of one partition (no GPU needed)."""
    lib = N.load_library()
    desc = N.MeshDesc()
    desc.dim = mesh.dim
    bufs = []
    for a in range(3):
        if a < mesh.dim:
            b = np.ascontiguousarray(mesh.axes[a])
            bufs.append(b)
            desc.n_cells[a] = len(b) - 1
            desc.coords[a] = b.ctypes.data_as(C.POINTER(C.c_double))
    desc.part_axis = part_axis
    desc.n_parts = n_parts
    desc.part = part
    out = (C.c_int64 * 13)()
    N.check(lib.tv_partition_layout(C.byref(desc), out))
    v = list(out)
    return {"perm": v[0:3], "nodes": v[3:6], "planes": (v[6], v[7]), "global_offset": v[8], "n_owned": v[9],
            "n_local": v[10], "ghost_lo": bool(v[11]), "ghost_hi": bool(v[12])}


def umesh_desc(mesh):
    """(tv_umesh_desc, buffers to keep alive) of a tvfem.UnstructuredMesh."""
    desc = N.UMeshDesc()
    desc.dim = mesh.dim
    xyz = np.ascontiguousarray(mesh.x, dtype=np.float64)
    cells = np.ascontiguousarray(mesh.cells, dtype=np.int64)
    desc.n_vertices = xyz.shape[0]
    desc.coords = xyz.ctypes.data_as(C.POINTER(C.c_double))
    desc.n_cells = cells.shape[0]
    desc.cells = cells.ctypes.data_as(C.POINTER(C.c_int64))
    return desc, (xyz, cells)


def rcb_partition(mesh, n_parts: int) -> np.ndarray:
    """Cell -> part ids (int32) of an unstructured mesh by recursive coordinate
    bisection (tv_partition_rcb, host only).  Parts differ in size by at most
    one cell per bisection level."""
    lib = N.load_library()
    desc, keep = umesh_desc(mesh)
    part = np.empty(mesh.num_cells, dtype=np.int32)
    N.check(lib.tv_partition_rcb(C.byref(desc), int(n_parts), part.ctypes.data_as(C.POINTER(C.c_int))))
    del keep
    return part


def partition_submesh(mesh, part: np.ndarray, p: int):
    """Local mesh of part ``p``: its cells, the vertices they touch (owned
    vertices first, then ghosts) and the local -> global vertex map.  A vertex
    is owned by the lowest part among the cells that touch it (the dolfinx
    convention is the owner rank chosen by its distributed vertex numbering)."""
    from .mesh import UnstructuredMesh
    nv = mesh.num_vertices
    owner = np.full(nv, np.iinfo(np.int32).max, dtype=np.int64)
    np.minimum.at(owner, mesh.cells.ravel(), np.repeat(part.astype(np.int64), mesh.cells.shape[1]))
    cells = mesh.cells[part == p]
    used = np.unique(cells.ravel())
    own = used[owner[used] == p]
    ghost = used[owner[used] != p]
    l2g = np.concatenate([own, ghost])
    g2l = np.full(nv, -1, dtype=np.int64)
    g2l[l2g] = np.arange(len(l2g))
    sub = UnstructuredMesh(mesh.dim, mesh.x[l2g], g2l[cells])
    return {"mesh": sub, "l2g": l2g, "n_owned": len(own), "ghost_owner": owner[ghost]}


def ghosted_partition(mesh, part: np.ndarray, p: int, n_parts: int | None = None) -> dict:
    """Partition ``p`` of an unstructured mesh with its ghost layer and halo
    plan, as tv_create_unstructured_part takes it (include/tvfem.h
    tv_upart_desc).  ``part``: cell -> part ids (rcb_partition).

    A vertex is owned by the lowest part among the cells around it.  Local
    cells: the part's own cells, then every other cell that touches one of its
    owned vertices, so each owned row of F and J is complete on the part (the
    ghost layer dolfinx keeps for ThermoViscoProblem.py:351's scatter_forward).
    Local vertices: owned first (ascending global id), then the ghosts grouped
    by owner (ascending rank), each group ascending -- the order in which the
    owner packs them.  Neighbours: the parts this one receives from or sends
    to (the relation is symmetric by construction, so both sides of every pair
    call the exchange).  Every rank computes the plan from the global mesh."""
    from .mesh import UnstructuredMesh
    cells = np.asarray(mesh.cells, dtype=np.int64)
    part = np.asarray(part, dtype=np.int64)
    nv, nl = mesh.num_vertices, cells.shape[1]
    P = int(part.max()) + 1 if n_parts is None else int(n_parts)
    owner = np.full(nv, np.iinfo(np.int64).max, dtype=np.int64)
    for q in range(P - 1, -1, -1):  # lowest part last: owner = min over the cells around a vertex
        owner[cells[part == q].ravel()] = q
    counts = np.bincount(owner, minlength=P)
    ocell = owner[cells]                                   # (nc, nl) owners of each cell's vertices
    own_c = np.flatnonzero(part == p)
    ghost_c = np.flatnonzero((part != p) & (ocell == p).any(axis=1))
    lc = np.concatenate([own_c, ghost_c])
    used = np.unique(cells[lc].ravel())
    own_v = used[owner[used] == p]
    gv = used[owner[used] != p]
    gv = gv[np.lexsort((gv, owner[gv]))]
    l2g = np.concatenate([own_v, gv])
    g2l = np.full(nv, -1, dtype=np.int64)
    g2l[l2g] = np.arange(len(l2g))
    # sends: owned vertex v goes to every part q != p for which a cell around v
    # is local: q = the cell's part or an owner of one of its vertices
    cand = lc[(np.concatenate([part[lc, None], ocell[lc]], axis=1) != p).any(axis=1)]
    lp = np.concatenate([part[cand, None], ocell[cand]], axis=1)   # (m, nl + 1) parts the cell is local to
    cv = cells[cand]                                                 # (m, nl)
    qq = np.repeat(lp[:, :, None], nl, axis=2)                       # (m, nl + 1, nl)
    vv = np.repeat(cv[:, None, :], lp.shape[1], axis=1)
    ok = (qq != p) & (owner[vv] == p)
    pairs = np.unique(np.stack([qq[ok], vv[ok]], axis=1), axis=0) if ok.any() else np.zeros((0, 2), np.int64)
    recv_from = np.unique(owner[gv])
    nbrs = np.union1d(recv_from, np.unique(pairs[:, 0])).astype(np.int64)
    recv_count = np.array([np.count_nonzero(owner[gv] == q) for q in nbrs], dtype=np.int64)
    send_idx, send_count = [], []
    for q in nbrs:
        sv = pairs[pairs[:, 0] == q, 1]                              # ascending global ids (np.unique order)
        send_idx.append(g2l[sv])
        send_count.append(len(sv))
    sub = UnstructuredMesh(mesh.dim, mesh.x[l2g], g2l[cells[lc]])
    return {"mesh": sub, "l2g": l2g, "n_owned": len(own_v), "n_owned_cells": len(own_c),
            "global_offset": int(counts[:p].sum()), "neighbors": nbrs.astype(np.int32),
            "recv_count": recv_count, "send_count": np.array(send_count, dtype=np.int64),
            "send_idx": (np.concatenate(send_idx) if send_idx else np.zeros(0, np.int64)).astype(np.int64),
            "n_parts": P, "part": int(p)}


def upart_desc(gp: dict):
    """(tv_upart_desc, buffers to keep alive) of a ghosted_partition record."""
    d = N.UPartDesc()
    bufs = [np.ascontiguousarray(gp[k]) for k in ("neighbors", "recv_count", "send_count", "send_idx")]
    d.n_parts, d.part = gp["n_parts"], gp["part"]
    d.n_owned, d.n_owned_cells, d.global_offset = gp["n_owned"], gp["n_owned_cells"], gp["global_offset"]
    d.n_neighbors = len(bufs[0])
    d.neighbors = bufs[0].ctypes.data_as(C.POINTER(C.c_int))
    d.recv_count = bufs[1].ctypes.data_as(C.POINTER(C.c_int64))
    d.send_count = bufs[2].ctypes.data_as(C.POINTER(C.c_int64))
    d.send_idx = bufs[3].ctypes.data_as(C.POINTER(C.c_int64))
    return d, bufs


def init_rccl(problem, rank: int, world: int, dist=None):
    """Create the RCCL communicator of a partitioned problem (rank 0 makes the id)."""
    if dist is None:
        import torch.distributed as dist
    lib, ctx = problem._lib, problem._ctx
    buf = C.create_string_buffer(lib.tv_comm_unique_id_size())
    if rank == 0:
        N.check(lib.tv_comm_get_unique_id(buf))
    obj = [buf.raw if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0)
    N.check(lib.tv_comm_init(ctx, C.c_char_p(obj[0]), world, rank), ctx)


def init_host_comm(problem, rank: int, world: int, dist=None):
    """Host-staged communicator over a torch.distributed (gloo) group."""
    if dist is None:
        import torch.distributed as dist
    import torch

    def allreduce(ptr, n, user):
        try:
            a = np.ctypeslib.as_array(ptr, shape=(n,))
            t = torch.from_numpy(a.copy())
            dist.all_reduce(t)
            a[:] = t.numpy()
            return 0
        except Exception:  # pragma: no cover
            return 1

    def sendrecv(sptr, ns, peer_s, rptr, nr, peer_r, user):
        try:
            s = torch.from_numpy(np.ctypeslib.as_array(sptr, shape=(ns,)).copy())
            r = torch.empty(nr, dtype=torch.float64)
            reqs = [dist.isend(s, peer_s), dist.irecv(r, peer_r)]
            for q in reqs:
                q.wait()
            np.ctypeslib.as_array(rptr, shape=(nr,))[:] = r.numpy()
            return 0
        except Exception:  # pragma: no cover
            return 1

    problem._host_cbs = (N.HOST_ALLREDUCE_FN(allreduce), N.HOST_SENDRECV_FN(sendrecv))
    N.check(problem._lib.tv_comm_init_host(problem._ctx, world, rank, problem._host_cbs[0], problem._host_cbs[1],
                                           None), problem._ctx)
