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
