"""Time-series output (ThermoViscoProblem.py:246-276 _write_initial_output,
:357-364 _write_output, :614-620 _finalize): XDMF 3 over raw binary.

CPU: the file format layer (tv_xdmf_*, no GPU) round-trips through the reader
(tvfem.xdmf) for 1D / 2D / 3D and CG / DG fields.  GPU: a coupled run with
write_output=True writes the five series asynchronously; every written step
equals the field values read back from the device at that step.
"""
import ctypes as C

import numpy as np
import pytest


def _lib():
    try:
        from tvfem import load_library
        return load_library()
    except Exception:
        pytest.skip("libtvfem.so not built")


@pytest.mark.parametrize("axes", [
    [np.linspace(0.0, 5.0, 7)],
    [np.array([0.0, 0.5, 2.0]), np.linspace(0.0, 1.0, 4)],
    [np.linspace(0.0, 1.0, 3), np.array([0.0, 0.2, 0.7, 1.0]), np.linspace(0.0, 0.5, 3)],
])
def test_xdmf_round_trip_cpu(tmp_path, axes):
    from tvfem.xdmf import read_series
    lib = _lib()
    d = len(axes)
    nc = (C.c_int * 3)(*[len(a) - 1 for a in axes], *([0] * (3 - d)))
    bufs = [np.ascontiguousarray(a) for a in axes]
    cp = (C.POINTER(C.c_double) * 3)(*[b.ctypes.data_as(C.POINTER(C.c_double)) for b in bufs],
                                     *([None] * (3 - d)))
    h = lib.tv_xdmf_open(str(tmp_path).encode(), d, nc, cp)
    assert h
    nn = int(np.prod([len(a) for a in axes]))
    ncell = int(np.prod([len(a) - 1 for a in axes]))
    assert lib.tv_xdmf_add_field(h, b"T", 1, 0) == 0
    assert lib.tv_xdmf_add_field(h, b"sigma", d * d, 0) == 0
    assert lib.tv_xdmf_add_field(h, b"Tdg", 1, 1) == 0
    rng = np.random.default_rng(0)
    written = []
    for step in range(3):
        T = rng.standard_normal(nn)
        S = rng.standard_normal(nn * d * d)
        G = rng.standard_normal(ncell * 2 ** d)
        for k, v in enumerate((T, S, G)):
            assert lib.tv_xdmf_append(h, k, 0.1 * step, v.ctypes.data_as(C.POINTER(C.c_double)), v.size) == 0
        written.append((T, S, G))
    assert lib.tv_xdmf_append(h, 0, 0.0, T.ctypes.data_as(C.POINTER(C.c_double)), T.size - 1) != 0  # size check
    lib.tv_xdmf_close(h)
    sT = read_series(str(tmp_path / "T.xdmf"))
    sS = read_series(str(tmp_path / "sigma.xdmf"))
    sG = read_series(str(tmp_path / "Tdg.xdmf"))
    assert sT["times"] == pytest.approx([0.0, 0.1, 0.2])
    assert sT["topology_type"] == {1: "Polyline", 2: "Quadrilateral", 3: "Hexahedron"}[d]
    assert sS["attribute_type"] == ("Scalar" if d == 1 else ("Tensor" if d == 3 else "Matrix"))
    for step, (T, S, G) in enumerate(written):
        assert np.array_equal(sT["values"][step].ravel(), T)
        assert np.array_equal(sS["values"][step].ravel(), S)
        assert np.array_equal(sG["values"][step].ravel(), G)
    # geometry: node v = i + n0 (j + n1 k) at (x_i, y_j, z_k); topology in VTK order
    X = sT["geometry"]
    grids = np.meshgrid(*axes, indexing="ij")
    for a in range(d):
        assert np.array_equal(X[:, a], grids[a].transpose(list(range(d))[::-1]).ravel())
    topo = sT["topology"]
    assert topo.shape == (ncell, 2 ** d) and topo.min() == 0 and topo.max() == nn - 1
    # every cell's vertices span exactly one cell of the grid (VTK-ordered corners)
    corners = X[topo]
    span = corners.max(axis=1) - corners.min(axis=1)
    for a in range(d):
        assert np.all(span[:, a] > 0)
    # DG copy: node (cell e, local l) at the cell's vertex l
    assert sG["geometry"].shape == (ncell * 2 ** d, 3)


@pytest.mark.gpu
def test_async_output_matches_device_fields(tmp_path):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tvfem import box_mesh
    from tvfem.problem import ThermoViscoProblem
    from tvfem.xdmf import read_series
    from oracle import tv_oracle as O
    cfg = {"T": {"element": "CG", "degree": 1}, "sigma": {"element": "CG", "degree": 1}}
    p = ThermoViscoProblem(box_mesh([2.0, 2.0, 1.0], [12, 10, 5]), (0.0, 0.4), 0.1, cfg, dict(O.MAIN_MODEL_PARAMS),
                           part_axis=1, verbose=False, write_output=True, output_dir=str(tmp_path))
    p.setup()
    snaps = [{f: p.get_field(f) for f in p.OUTPUT_FIELDS}]
    for _ in range(4):
        p.t += p.dt
        p.solve_timestep()
        snaps.append({f: p.get_field(f) for f in p.OUTPUT_FIELDS})
    p.close()  # drains the writer
    X = None
    for f in p.OUTPUT_FIELDS:
        s = read_series(str(tmp_path / f"{f}.xdmf"))
        assert len(s["times"]) == 5
        assert s["times"] == pytest.approx([0.0, 0.1, 0.2, 0.3, 0.4])
        for k in range(5):
            assert np.array_equal(s["values"][k].ravel(), snaps[k][f], equal_nan=True), (f, k)
        X = s["geometry"]
    # geometry in physical coordinates for the (x, z, y) storage order of part_axis=1
    assert np.isclose(X[:, 0].max(), 2.0) and np.isclose(X[:, 1].max(), 2.0) and np.isclose(X[:, 2].max(), 1.0)


@pytest.mark.gpu
@pytest.mark.parametrize("fam", ["CG", "DG"])
def test_output_series_match_oracle(tmp_path, fam):
    """The five written series (T, phi, Tf, xi, sigma: ThermoViscoProblem.py:246-276
    at setup, :357-364 after every step) against the ORACLE's fields of the same
    steps (oracle/tv_oracle.py OracleProblem, run alongside): T and Tf rel. L2
    <= 1e-10, phi <= 1e-9, xi and sigma by check_field (rel. 1e-6 on the dofs
    whose T changed by more than 1e-6 K in that step, the rest bounded), at the
    initial output and after each of four steps.  part_axis=2 keeps the written
    node order equal to the oracle's dof order.  Also checks setup()'s default
    series names (the reference's T, phi, Tf, xi, sigma)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tvfem import box_mesh
    from tvfem.problem import ThermoViscoProblem
    from tvfem.xdmf import read_series
    from oracle import tv_oracle as O
    from parity_util import check_field, cond_mask, relerr
    cfg = {"T": {"element": fam, "degree": 1}, "sigma": {"element": fam, "degree": 1}}
    L, nc = [2.0, 2.0, 1.0], [10, 8, 5]
    dev = ThermoViscoProblem(box_mesh(L, nc), (0.0, 0.4), 0.1, cfg, dict(O.MAIN_MODEL_PARAMS), part_axis=2,
                             verbose=False, write_output=True, output_dir=str(tmp_path))
    ref = O.OracleProblem(O.box_mesh(L, nc), (0.0, 0.4), 0.1, cfg, dict(O.MAIN_MODEL_PARAMS), linear="pcg")
    dev.setup()
    ref.setup()
    snaps = [{"T": ref.functions_current["T"].copy(), "phi": ref.functions["phi"].copy(),
              "Tf": ref.functions_current["Tf"].copy(), "xi": ref.functions["xi"].copy(),
              "sigma": ref.functions_next["sigma"].copy(), "T_before": ref.functions_current["T"].copy()}]
    with np.errstate(all="ignore"):
        for _ in range(4):
            T_before = ref.functions_current["T"].copy()
            dev.t += dev.dt
            dev.solve_timestep()
            ref.solve_timestep()
            snaps.append({"T": ref.functions_current["T"].copy(), "phi": ref.functions["phi"].copy(),
                          "Tf": ref.functions_current["Tf"].copy(), "xi": ref.functions["xi"].copy(),
                          "sigma": ref.functions_next["sigma"].copy(), "T_before": T_before})
    dev.close()  # drains the writer
    series = {f: read_series(str(tmp_path / f"{f}.xdmf")) for f in ("T", "phi", "Tf", "xi", "sigma")}
    for f, s in series.items():
        assert s["times"] == pytest.approx([0.0, 0.1, 0.2, 0.3, 0.4]), f
    for k, sn in enumerate(snaps):
        got = {f: series[f]["values"][k].ravel() for f in series}
        assert relerr(got["T"], sn["T"]) <= 1e-10, k
        assert relerr(got["Tf"], sn["Tf"]) <= 1e-10, k
        assert relerr(got["phi"], sn["phi"]) <= 1e-9, k
        if k == 0:  # the initial output: xi and sigma are the zero-initialised functions
            assert not got["xi"].any() and not got["sigma"].any()
            continue
        mT, _ = cond_mask(sn["T"], sn["T_before"])
        check_field(f"xi step {k}", got["xi"], sn["xi"], mT)
        check_field(f"sigma step {k}", got["sigma"], sn["sigma"], mT, bs=9)


@pytest.mark.gpu
def test_output_series_names_follow_setup_arguments(tmp_path):
    """setup(outfile_name=..., outfile_name1=...) (ThermoViscoProblem.py:176-178):
    the defaults give the reference's file names; other values prefix the four
    scalar series and name the stress series."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from tvfem import box_mesh
    from tvfem.problem import ThermoViscoProblem
    from tvfem.xdmf import read_series
    from oracle import tv_oracle as O
    cfg = {"T": {"element": "CG", "degree": 1}, "sigma": {"element": "CG", "degree": 1}}
    p = ThermoViscoProblem(box_mesh([1.0, 1.0, 1.0], [4, 4, 4]), (0.0, 0.2), 0.1, cfg, dict(O.MAIN_MODEL_PARAMS),
                           verbose=False, write_output=True, output_dir=str(tmp_path))
    assert p.series_names() == ["T", "phi", "Tf", "xi", "sigma"]
    p.setup(outfile_name="run1", outfile_name1="stress_run1")
    p.solve()
    for stem in ("run1_T", "run1_phi", "run1_Tf", "run1_xi", "stress_run1"):
        s = read_series(str(tmp_path / f"{stem}.xdmf"))
        assert len(s["times"]) == 3, stem
    p.close()
