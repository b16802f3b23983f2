"""Meshes of the hot path: rectilinear grids (tensor products of per-axis node
coordinates) in 1, 2 or 3 dimensions.

They cover the reference's own mesh (a 1D graded interval written by gmsh,
geometry.py:3-29, read with gdim=1 at ThermoViscoProblem.py:27-28) and the
structured hexahedral plates of the benchmark configurations.  ``read_msh``
reads gmsh ASCII files (MSH 2.2 / 4.1) of 1D line meshes.
"""
from __future__ import annotations

import numpy as np


class RectilinearMesh:
    """Tensor-product grid.  ``axes[a]`` holds the strictly increasing node
    coordinates along physical axis ``a``."""

    def __init__(self, axes):
        self.axes = [np.ascontiguousarray(a, dtype=np.float64) for a in axes]
        if not 1 <= len(self.axes) <= 3:
            raise ValueError("1 to 3 axes")
        for a in self.axes:
            if a.ndim != 1 or len(a) < 2 or not np.all(np.diff(a) > 0):
                raise ValueError("axis coordinates must be 1D, strictly increasing, >= 2 nodes")

    @property
    def dim(self):
        return len(self.axes)

    @property
    def n_cells(self):
        return [len(a) - 1 for a in self.axes]

    @property
    def num_cells(self):
        return int(np.prod(self.n_cells))

    @property
    def num_vertices(self):
        return int(np.prod([len(a) for a in self.axes]))

    def __repr__(self):
        return f"RectilinearMesh(dim={self.dim}, n_cells={self.n_cells})"


def box_mesh(lengths, n_cells):
    """Uniform box [0, L0] x ... with n_cells[a] cells along axis a."""
    return RectilinearMesh([np.linspace(0.0, float(L), int(n) + 1) for L, n in zip(lengths, n_cells)])


def interval_mesh(length, n_cells):
    return box_mesh([length], [n_cells])


def _read_msh_nodes_and_lines(path):
    with open(path, "r") as fh:
        lines = [ln.strip() for ln in fh]
    try:
        fmt = lines.index("$MeshFormat")
    except ValueError as e:
        raise ValueError(f"{path}: not a gmsh ASCII .msh file") from e
    version = float(lines[fmt + 1].split()[0])
    if int(lines[fmt + 1].split()[1]) != 0:
        raise ValueError("binary .msh files are not supported")
    ni = lines.index("$Nodes")
    ei = lines.index("$Elements")
    nodes = {}
    segs = []
    if version < 3:
        n = int(lines[ni + 1])
        for k in range(n):
            t = lines[ni + 2 + k].split()
            nodes[int(t[0])] = float(t[1])
        m = int(lines[ei + 1])
        for k in range(m):
            t = [int(v) for v in lines[ei + 2 + k].split()]
            if t[1] == 1:  # 2-node line
                ntags = t[2]
                segs.append((t[3 + ntags], t[4 + ntags]))
    else:
        hdr = lines[ni + 1].split()
        nblocks = int(hdr[0])
        pos = ni + 2
        for _ in range(nblocks):
            _, _, param, nb = (int(v) for v in lines[pos].split()[:4])
            tags = [int(lines[pos + 1 + q]) for q in range(nb)]
            for q in range(nb):
                nodes[tags[q]] = float(lines[pos + 1 + nb + q].split()[0])
            pos += 1 + 2 * nb
        hdr = lines[ei + 1].split()
        nblocks = int(hdr[0])
        pos = ei + 2
        for _ in range(nblocks):
            _, _, etype, nb = (int(v) for v in lines[pos].split()[:4])
            for q in range(nb):
                t = [int(v) for v in lines[pos + 1 + q].split()]
                if etype == 1:
                    segs.append((t[1], t[2]))
            pos += 1 + nb
    return nodes, segs


def read_msh(path):
    """Read a gmsh ASCII 1D line mesh (what geometry.create_mesh writes) as a
    RectilinearMesh; the reference reads it with gdim=1 (ThermoViscoProblem.py:28)."""
    nodes, segs = _read_msh_nodes_and_lines(path)
    if not segs:
        raise ValueError(f"{path}: no 2-node line elements (only 1D meshes are supported, as in the reference)")
    used = sorted({v for s in segs for v in s})
    x = np.array(sorted(nodes[v] for v in used))
    if len(np.unique(x)) != len(x):
        raise ValueError("duplicate vertex coordinates")
    if len(segs) != len(x) - 1:
        raise ValueError("line mesh is not a single connected interval")
    return RectilinearMesh([x])


def write_msh(path, mesh: RectilinearMesh):
    """Write a 1D RectilinearMesh as a gmsh MSH 2.2 ASCII file."""
    if mesh.dim != 1:
        raise ValueError("only 1D meshes are written")
    x = mesh.axes[0]
    with open(path, "w") as fh:
        fh.write("$MeshFormat\n2.2 0 8\n$EndMeshFormat\n$Nodes\n%d\n" % len(x))
        for i, v in enumerate(x):
            fh.write(f"{i + 1} {float(v)!r} 0 0\n")
        fh.write("$EndNodes\n$Elements\n%d\n" % (len(x) - 1))
        for i in range(len(x) - 1):
            fh.write(f"{i + 1} 1 2 0 1 {i + 1} {i + 2}\n")
        fh.write("$EndElements\n")
