"""Reader of the XDMF time series libtvfem writes (tv_output_* / tv_xdmf_*).

One series per field: ``<dir>/<name>.xdmf`` indexes raw little-endian float64
arrays in ``<name>.bin`` (one block per time, ``Seek`` byte offsets) over the
mesh in ``mesh_geometry.bin`` / ``mesh_topology.bin`` (``mesh_dg_*`` for DG
fields).  The reference writes the same fields through dolfinx.io
(ThermoViscoProblem.py:246-276, 357-364): VTX/BP4 for T, phi, Tf and xi, and
XDMF/HDF5 for sigma.
"""
from __future__ import annotations

import os
import xml.etree.ElementTree as ET

import numpy as np


def _item(dirname, di):
    dims = [int(v) for v in di.attrib["Dimensions"].split()]
    dtype = np.float64 if di.attrib.get("DataType", "Float") == "Float" else np.int64
    assert di.attrib.get("Format") == "Binary" and di.attrib.get("Endian", "Little") == "Little"
    assert int(di.attrib.get("Precision", "8")) == 8
    off = int(di.attrib.get("Seek", "0"))
    n = int(np.prod(dims))
    a = np.fromfile(os.path.join(dirname, di.text.strip()), dtype=dtype, count=n, offset=off)
    if a.size != n:
        raise ValueError(f"{di.text.strip()}: expected {n} values at offset {off}, got {a.size}")
    return a.reshape(dims)


def read_series(path):
    """-> dict(times=[...], values=[array (n_nodes, ncomp), ...], geometry=(n, 3),
    topology=(n_cells, 2**d), topology_type=str, name=str)."""
    dirname = os.path.dirname(os.path.abspath(path))
    root = ET.parse(path).getroot()
    coll = root.find("Domain").find("Grid")
    out = {"name": coll.attrib["Name"], "times": [], "values": []}
    for g in coll.findall("Grid"):
        out["times"].append(float(g.find("Time").attrib["Value"]))
        att = g.find("Attribute")
        out["values"].append(_item(dirname, att.find("DataItem")))
        if "geometry" not in out:
            out["geometry"] = _item(dirname, g.find("Geometry").find("DataItem"))
            topo = g.find("Topology")
            out["topology"] = _item(dirname, topo.find("DataItem"))
            out["topology_type"] = topo.attrib["TopologyType"]
            out["attribute_type"] = att.attrib["AttributeType"]
    return out
