"""Workgroup timeline of the box march kernels (C4), from the timing build of
tools/wgtrace/build.py: per kind (plain tile / face-chunk tile / face
workgroup) the start, end and duration of the workgroups relative to the
launch, per XCC the last end, the last workgroups to finish and the number of
workgroups in flight over time.  s_memrealtime ticks at 100 MHz (10 ns).

    TVFEM_LIB=.../libtvfem_wgt.so python tools/wgtrace/run.py [--kernel 3] [--reps 5]
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "fem-glass-tempering_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

from tvfem import box_mesh  # noqa: E402
from tvfem import _native as N  # noqa: E402
from tvfem.problem import ThermoViscoProblem  # noqa: E402

KINDS = {0: "tile", 1: "face-chunk tile", 2: "face workgroup"}


def analyse(buf, label):
    t0, t1, xcc, kind = buf[0], buf[1], buf[2] & 0xF, buf[3]
    ok = t0 > 0
    last = t0[ok].max()
    ok &= t0 >= last - 100000  # this launch only (1 ms)
    idx = np.nonzero(ok)[0]
    s, e = t0[idx].astype(np.int64), t1[idx].astype(np.int64)
    base = s.min()
    s = (s - base) / 100.0
    e = (e - base) / 100.0  # us
    k = kind[idx]
    x = xcc[idx]
    span = e.max()
    out = {"kernel": label, "workgroups": int(idx.size), "span_us": round(float(span), 2)}
    for kk, name in KINDS.items():
        m = k == kk
        if m.any():
            out[name] = {"n": int(m.sum()), "start_us": [round(float(np.percentile(s[m], q)), 2) for q in (0, 50, 100)],
                         "end_us": [round(float(np.percentile(e[m], q)), 2) for q in (0, 50, 100)],
                         "dur_us": [round(float(np.percentile(e[m] - s[m], q)), 2) for q in (10, 50, 90)]}
    out["xcc_last_end_us"] = [round(float(e[x == c].max()), 2) if (x == c).any() else None for c in range(8)]
    order = np.argsort(-e)[:16]
    out["last16"] = [(int(idx[i]), KINDS[int(k[i])], int(x[i]), round(float(s[i]), 2), round(float(e[i]), 2)) for i in order]
    bins = np.arange(0.0, span + 2.0, 2.0)
    out["in_flight_per_2us"] = [int(((s < b + 2.0) & (e > b)).sum()) for b in bins]
    print("WGT " + json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cells", default="400,400,50")
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from partition_check import MP
    nc = [int(v) for v in a.cells.split(",")]
    cfg = {"T": {"element": "CG", "degree": 1}, "sigma": {"element": "CG", "degree": 1}}
    p = ThermoViscoProblem(box_mesh([50.0, 50.0, 5.0], nc), (0, 10), 0.1, cfg, MP, verbose=False,
                           write_output=False, materialize=False, part_axis=1, pcg_variant="kspcg")
    p.setup()
    lib, ctx = p._lib, p._ctx
    lib.tv_wgt_read.argtypes = [C.c_void_p]
    buf = np.zeros((4, 16384), dtype=np.uint64)
    for kid, label in ((3, "fused matvec"), (0, "J x (march part)")):
        ms = C.c_double()
        N.check(lib.tv_time_kernel(ctx, kid, a.reps, C.byref(ms)), ctx)
        assert lib.tv_wgt_read(buf.ctypes.data) == 0
        print(f"[{label}] tv_time_kernel mean {ms.value * 1e3:.2f} us", flush=True)
        analyse(buf, label)
    p.close()


if __name__ == "__main__":
    main()
