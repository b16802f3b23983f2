"""The production RCCL path on one GPU (tools/loopback_check.py): a partition
on a one-rank RCCL communicator whose neighbours are itself.

Every RCCL group the partitioned solver issues runs in the real library --
grouped ncclSend / ncclRecv of ghost planes (fine grid and distributed
multigrid levels), ncclAllReduce mixed with send / receive pairs in one group
(the closing group of a KSPCG iteration, the single-reduction group), the
replicated multigrid level's vector all-reduce, and the per-neighbour groups of
the unstructured halo (ThermoViscoProblem.py:351 scatter_forward, PETSc's
all-reduces inside :389).  The received values are checked against the sent
ones (tv_comm_check), and whole coupled steps are compared bitwise with the
host-staged transport under the same loopback semantics.

Also the guards around the transport: a partitioned context refuses to solve
without a communicator, and the measurement stub refuses unless the Krylov
iteration count is fixed (it solves a decoupled block).
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.gpu
def test_rccl_loopback_groups_match_host_transport():
    _gpu()
    cmd = [sys.executable, "-u", os.path.join(ROOT, "tools", "loopback_check.py")]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    lines = [json.loads(ln.split(" ", 1)[1]) for ln in out.stdout.splitlines() if ln.startswith("LOOPBACK ")]
    assert out.returncode == 0 and len(lines) == 9, out.stdout[-3000:] + out.stderr[-3000:]
    for r in lines:
        print(f"[loopback] {r['case']}: {r['checked']} values checked, {r['bad']} wrong; its {r['its_rccl']} "
              f"(host {r['its_host']}); form {r['krylov_form']}, pc {r['pc']}; err {r['err_rccl']}")
        assert r["checked"] > 0 and r["bad"] == 0, r
        assert r["err_rccl"] == r["err_host"], r
        # the CG slabs' mirrored-ghost problem is symmetric: every CG step converges,
        # the distributed multigrid ones (three deep ghost planes, single-reduction
        # GMG-PCG) included; the DG ghost layer is a shifted copy
        # of the cell layer (its local vertex order is not mirrored): agreement counts
        assert r["err_rccl"] is None or r["case"].startswith("dg"), r
        if r["pc"] == "gmg":  # the distributed V-cycle itself, every exchange of it, through both transports
            assert r["vcycle_bitwise"] and r["vcycle_norm"] > 0.0, r
        assert r["its_rccl"] == r["its_host"], r
        for k in ("T", "phi", "xi", "sigma"):
            assert r["bitwise_" + k], r
    forms = {(r["krylov_form"], r["pc"]) for r in lines}
    assert ("single", "jacobi") in forms and ("kspcg", "gmg") in forms, forms


def _box_problem(**kw):
    sys.path.insert(0, os.path.join(ROOT, "fem-glass-tempering_amd"))
    from tvfem import box_mesh
    from tvfem.problem import ThermoViscoProblem
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from loopback_check import CFG, MP
    mesh = box_mesh([2.0, 6.0, 1.0], [6, 12, 3])
    return ThermoViscoProblem(mesh, (0, 1), 0.1, CFG, MP, part_axis=1, verbose=False, write_output=False, **kw)


@pytest.mark.gpu
def test_partitioned_context_without_communicator_refuses_to_solve():
    """a partition stepped before tv_comm_init would solve a
    decoupled block on stale ghosts and return success."""
    _gpu()
    from tvfem import _native as N
    p = _box_problem(n_parts=2, part=0)
    p.setup()
    with pytest.raises(N.NativeError) as e:
        p.solve_timestep()
    assert e.value.code == N.TV_ERR_STATE and "communicator" in str(e.value)
    p.close()


@pytest.mark.gpu
def test_measurement_stub_is_timing_only():
    _gpu()
    import ctypes as C
    from tvfem import _native as N
    p = _box_problem(n_parts=2, part=1)
    assert p._lib.tv_comm_init_stub(p._ctx) == N.TV_ERR_ARG  # no fixed Krylov count: refused
    p.close()
    p = _box_problem(n_parts=2, part=1, ksp_fixed_its=3, newton_fixed_its=2)
    N.check(p._lib.tv_comm_init_stub(p._ctx), p._ctx)
    p.setup()
    p.solve_timestep()
    out = np.empty(p.num_dofs(0)[0])
    rc = p._lib.tv_get_field(p._ctx, N.FIELD_ID["T"], out.ctypes.data_as(C.POINTER(C.c_double)), out.size)
    assert rc == N.TV_ERR_STATE  # the decoupled block is no solution to read
    n, b = C.c_int64(), C.c_int64()
    assert p._lib.tv_comm_check(p._ctx, C.byref(n), C.byref(b)) == N.TV_ERR_STATE
    p.close()
