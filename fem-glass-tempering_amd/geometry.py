"""Mesh generation entry point with the reference's name (geometry.py:3-29).

The reference builds a graded 1D bar on [0, 50] with gmsh (target sizes 0.1 at
both ends, 1.0 at x = 5 and 45, 3.0 at x = 25).  gmsh is not available, so this
writes an equivalent graded line mesh: node spacing follows the same piecewise
linear size field, integrated the way a 1D advancing mesher would.  The node
positions are this framework's own (not gmsh's).
"""
import numpy as np

from tvfem.mesh import RectilinearMesh, write_msh

_POINTS = [(0.0, 0.1), (5.0, 1.0), (25.0, 3.0), (45.0, 1.0), (50.0, 0.1)]


def graded_bar():
    xs = [0.0]
    while xs[-1] < 50.0:
        x = xs[-1]
        for (a, ha), (b, hb) in zip(_POINTS[:-1], _POINTS[1:]):
            if a <= x <= b:
                h = ha + (hb - ha) * (x - a) / (b - a)
                break
        xs.append(min(50.0, x + h))
    xs = np.array(xs)
    if xs[-1] - xs[-2] < 0.5 * 0.1:  # merge a sliver at the end
        xs = np.delete(xs, -2)
    return RectilinearMesh([xs])


def create_mesh(path: str):
    write_msh(path, graded_bar())
