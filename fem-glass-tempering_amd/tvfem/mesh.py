"""Meshes of the hot path.

* ``RectilinearMesh``: tensor products of per-axis node coordinates in 1, 2 or
  3 dimensions -- the reference's own mesh (a 1D graded interval written by
  gmsh, geometry.py:3-29, read with gdim=1 at ThermoViscoProblem.py:27-28) and
  the structured hexahedral plates of the benchmark configurations; the
  operators factorise on them (the fast path).
* ``UnstructuredMesh``: vertices + quadrilateral / hexahedral cells of any
  shape (gmsh .msh files with 2D / 3D elements), assembled by the
  element-local kernels (csrc/tv_um.hip).

``read_msh`` reads gmsh ASCII files (MSH 2.2 / 4.1): line meshes as a
RectilinearMesh, quadrilateral / hexahedral meshes as an UnstructuredMesh.
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


class UnstructuredMesh:
    """Vertices ``x`` (n_vertices, 3; unused coordinates 0) and cells ``cells``
    (n_cells, 2**dim) of quadrilaterals (dim 2) or hexahedra (dim 3) in the
    tensor-product local vertex order l = a + 2 b + 4 c (basix / dolfinx order
    for quadrilaterals and hexahedra)."""

    def __init__(self, dim, x, cells):
        if dim not in (2, 3):
            raise ValueError("unstructured meshes are quadrilateral (2D) or hexahedral (3D)")
        x = np.asarray(x, dtype=np.float64)
        if x.ndim != 2 or x.shape[1] < dim:
            raise ValueError("x must be (n_vertices, >= dim)")
        self.x = np.zeros((x.shape[0], 3))
        self.x[:, :x.shape[1]] = x[:, :3]
        self.cells = np.ascontiguousarray(cells, dtype=np.int64)
        if self.cells.ndim != 2 or self.cells.shape[1] != 2 ** dim:
            raise ValueError(f"cells must be (n_cells, {2 ** dim})")
        if self.cells.size and (self.cells.min() < 0 or self.cells.max() >= self.x.shape[0]):
            raise ValueError("cell vertex index out of range")
        self.dim = dim

    @property
    def num_cells(self):
        return int(self.cells.shape[0])

    @property
    def num_vertices(self):
        return int(self.x.shape[0])

    def __repr__(self):
        return f"UnstructuredMesh(dim={self.dim}, vertices={self.num_vertices}, cells={self.num_cells})"

    @classmethod
    def from_rectilinear(cls, mesh: "RectilinearMesh"):
        """The same grid as an unstructured mesh (vertex i + n0 (j + n1 k))."""
        axes = mesh.axes
        d = mesh.dim
        n = [len(a) for a in axes]
        grids = np.meshgrid(*axes, indexing="ij")
        x = np.stack([g.transpose(list(range(d))[::-1]).ravel() for g in grids], axis=1)
        nc = [m - 1 for m in n]
        ijk = np.stack(np.meshgrid(*[np.arange(m) for m in nc], indexing="ij"), axis=-1)
        ijk = ijk.transpose(list(range(d))[::-1] + [d]).reshape(-1, d)
        strides = [1]
        for m in n[:-1]:
            strides.append(strides[-1] * m)
        cells = np.zeros((ijk.shape[0], 2 ** d), dtype=np.int64)
        for l in range(2 ** d):
            for a in range(d):
                cells[:, l] += (ijk[:, a] + ((l >> a) & 1)) * strides[a]
        return cls(d, x, cells)


def box_mesh(lengths, n_cells):
    """Uniform box [0, L0] x ... with n_cells[a] cells along axis a."""
    return RectilinearMesh([np.linspace(0.0, float(L), int(n) + 1) for L, n in zip(lengths, n_cells)])


def distorted_box_mesh(lengths, n_cells, amp=0.2, seed=0, shuffle=False):
    """Box of n_cells quadrilaterals / hexahedra made general: interior vertices
    jittered by up to ``amp`` x the smallest spacing, then a shear and a smooth
    warp applied to all vertices (curved boundary, non-planar hex faces);
    ``shuffle`` also permutes vertex ids and cell order.  A stand-in for a gmsh
    mesh of the plate (ThermoViscoProblem.py:27-28) that exercises the
    element-local kernels' geometry."""
    L = [float(v) for v in lengths]
    n = [int(v) for v in n_cells]
    d = len(n)
    m = UnstructuredMesh.from_rectilinear(box_mesh(L, n))
    x = m.x
    rng = np.random.default_rng(seed)
    h = min(L[a] / n[a] for a in range(d))
    inner = np.ones(len(x), dtype=bool)
    for a in range(d):
        inner &= (x[:, a] > 1e-12 * L[a]) & (x[:, a] < L[a] * (1 - 1e-12))
    x[inner, :d] += rng.uniform(-amp * h, amp * h, (int(inner.sum()), d))
    x0 = x.copy()
    x[:, 1] += 0.15 * x0[:, 0]
    x[:, 0] += 0.1 * h * np.sin(np.pi * x0[:, 1] / L[1])
    if d == 3:
        x[:, 2] += 0.1 * h * np.cos(np.pi * x0[:, 0] / L[0]) * x0[:, 1] / L[1]
    cells = m.cells
    if shuffle:
        perm = rng.permutation(len(x))
        xn = np.empty_like(x)
        xn[perm] = x
        x = xn
        cells = perm[cells][rng.permutation(len(cells))]
    return UnstructuredMesh(d, x, cells)


def interval_mesh(length, n_cells):
    return box_mesh([length], [n_cells])


# gmsh element types and the gmsh -> tensor (l = a + 2b + 4c) vertex order
_GMSH_TYPES = {1: (1, 2, [0, 1]), 3: (2, 4, [0, 1, 3, 2]), 5: (3, 8, [0, 1, 3, 2, 4, 5, 7, 6])}
# topological dimension of the gmsh element types this reader does NOT support
# (triangles, tetrahedra, prisms, pyramids, higher-order lines / quads / hexes)
_GMSH_UNSUPPORTED = {2: 2, 4: 3, 6: 3, 7: 3, 8: 1, 9: 2, 10: 2, 11: 3, 12: 3, 13: 3, 14: 3, 16: 2, 17: 3, 18: 3,
                     19: 3, 20: 2, 21: 2, 22: 2, 23: 2, 24: 2, 25: 2, 26: 1, 27: 1, 28: 1, 29: 3, 30: 3, 31: 3,
                     36: 2, 37: 2, 38: 2, 92: 3, 93: 3}
_GMSH_NAMES = {2: "3-node triangle", 4: "4-node tetrahedron", 6: "6-node prism", 7: "5-node pyramid",
               8: "3-node line", 9: "6-node triangle", 10: "9-node quadrilateral", 11: "10-node tetrahedron",
               12: "27-node hexahedron", 16: "8-node quadrilateral", 17: "20-node hexahedron"}


def _elem_dim(etype):
    """Topological dimension of a gmsh element type (0 for points), None if unknown."""
    if etype == 15:
        return 0
    if etype in _GMSH_TYPES:
        return _GMSH_TYPES[etype][0]
    return _GMSH_UNSUPPORTED.get(etype)


def _read_msh_raw(path):
    """nodes {tag: (x, y, z)} and elements {dim: [node tags in gmsh order]}.

    Every element type in the file is recorded: a top-dimension element that is
    not a 2-node line, 4-node quadrilateral or 8-node hexahedron (a triangle,
    tetrahedron, prism, pyramid or a second-order cell) raises ValueError rather
    than being skipped, which would leave a hole in the domain with spurious
    Robin boundaries (or read a triangle mesh as its boundary lines)."""
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
    elems = {1: [], 2: [], 3: []}
    seen = set()  # every element type in the file
    if version < 3:
        n = int(lines[ni + 1])
        for k in range(n):
            t = lines[ni + 2 + k].split()
            nodes[int(t[0])] = tuple(float(v) for v in t[1:4])
        m = int(lines[ei + 1])
        for k in range(m):
            t = [int(v) for v in lines[ei + 2 + k].split()]
            seen.add(t[1])
            if t[1] in _GMSH_TYPES:
                d, nn, _ = _GMSH_TYPES[t[1]]
                ntags = t[2]
                elems[d].append(t[3 + ntags:3 + ntags + nn])
    else:
        hdr = lines[ni + 1].split()
        nblocks = int(hdr[0])
        pos = ni + 2
        for _ in range(nblocks):
            _, _, param, nb = (int(v) for v in lines[pos].split()[:4])
            tags = [int(lines[pos + 1 + q]) for q in range(nb)]
            for q in range(nb):
                nodes[tags[q]] = tuple(float(v) for v in lines[pos + 1 + nb + q].split()[:3])
            pos += 1 + 2 * nb
        hdr = lines[ei + 1].split()
        nblocks = int(hdr[0])
        pos = ei + 2
        for _ in range(nblocks):
            _, _, etype, nb = (int(v) for v in lines[pos].split()[:4])
            if nb > 0:
                seen.add(etype)
            for q in range(nb):
                t = [int(v) for v in lines[pos + 1 + q].split()]
                if etype in _GMSH_TYPES:
                    d, nn, _ = _GMSH_TYPES[etype]
                    elems[d].append(t[1:1 + nn])
            pos += 1 + nb
    dims = {}
    for et in seen:
        d = _elem_dim(et)
        if d is None:
            raise ValueError(f"{path}: unsupported gmsh element type {et}")
        dims.setdefault(d, set()).add(et)
    top = max(dims, default=0)
    bad = sorted(et for et in dims.get(top, ()) if et not in _GMSH_TYPES)
    if bad:
        names = ", ".join(_GMSH_NAMES.get(et, f"type {et}") for et in bad)
        raise ValueError(f"{path}: {top}D cells of unsupported element types ({names}); "
                         "libtvfem reads 2-node lines, 4-node quadrilaterals and 8-node hexahedra")
    return nodes, elems


def _read_msh_nodes_and_lines(path):
    nodes, elems = _read_msh_raw(path)
    return {k: v[0] for k, v in nodes.items()}, [tuple(e) for e in elems[1]]


def read_msh(path):
    """Read a gmsh ASCII mesh (MSH 2.2 / 4.1).  The cells are the elements of
    the highest dimension present: 2-node lines give a RectilinearMesh (what
    geometry.create_mesh writes; the reference reads it with gdim=1,
    ThermoViscoProblem.py:28), 4-node quadrilaterals / 8-node hexahedra an
    UnstructuredMesh (vertices numbered in increasing gmsh tag order)."""
    nodes, elems = _read_msh_raw(path)
    dim = max((d for d in (3, 2, 1) if elems[d]), default=0)
    if dim == 0:
        raise ValueError(f"{path}: no line, quadrilateral or hexahedral elements")
    if dim == 1:
        segs = elems[1]
        used = sorted({v for s in segs for v in s})
        x = np.array(sorted(nodes[v][0] for v in used))
        if len(np.unique(x)) != len(x):
            raise ValueError("duplicate vertex coordinates")
        if len(segs) != len(x) - 1:
            raise ValueError("line mesh is not a single connected interval")
        return RectilinearMesh([x])
    perm = _GMSH_TYPES[{2: 3, 3: 5}[dim]][2]
    cells_g = np.array(elems[dim], dtype=np.int64)
    used = np.unique(cells_g)
    index = {int(t): i for i, t in enumerate(used)}
    x = np.array([nodes[int(t)] for t in used])
    cells = np.vectorize(index.__getitem__)(cells_g)[:, perm]
    return UnstructuredMesh(dim, x, cells)


def write_msh_unstructured(path, mesh: UnstructuredMesh):
    """Write an UnstructuredMesh as a gmsh MSH 4.1 ASCII file (one entity)."""
    d = mesh.dim
    etype = {2: 3, 3: 5}[d]
    inv = np.argsort(_GMSH_TYPES[etype][2])  # tensor -> gmsh order
    with open(path, "w") as fh:
        fh.write("$MeshFormat\n4.1 0 8\n$EndMeshFormat\n")
        nv, nc = mesh.num_vertices, mesh.num_cells
        fh.write(f"$Nodes\n1 {nv} 1 {nv}\n{d} 1 0 {nv}\n")
        for i in range(nv):
            fh.write(f"{i + 1}\n")
        for p in mesh.x:
            fh.write(f"{float(p[0])!r} {float(p[1])!r} {float(p[2])!r}\n")
        fh.write("$EndNodes\n")
        fh.write(f"$Elements\n1 {nc} 1 {nc}\n{d} 1 {etype} {nc}\n")
        for e, c in enumerate(mesh.cells):
            fh.write(f"{e + 1} " + " ".join(str(int(v) + 1) for v in c[inv]) + "\n")
        fh.write("$EndElements\n")


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
