"""Collect the bench lines of the per-rank strong-scaling shapes of C4 (run as
single-GPU problems, no halo or allreduce) and the C2-C5 lines into one record.

    python tools/strong_shapes.py OUT.json tag=bench.json [tag=bench.json ...]
"""
import json
import sys


def main():
    out = {}
    for arg in sys.argv[2:]:
        tag, path = arg.split("=", 1)
        d = json.load(open(path))
        out[tag] = {"ms_per_step": d["ms_per_step"], "value": d["value"],
                    "krylov_its_per_step": d["config"]["krylov_its_per_step"],
                    "workload": d["config"]["workload"],
                    "kernels_us": {k: round(v["ms"] * 1e3, 2) for k, v in d["kernels"].items()}}
    rec = {"source": "bench.py on one MI355X, --steps 10 --no-cpu-baseline (C5: --steps 5); the n*_share shapes "
                     "are the per-rank slabs of C4 under strong scaling along y, run as single-GPU problems "
                     "(no halo or allreduce)",
           "runs": out}
    with open(sys.argv[1], "w") as fh:
        json.dump(rec, fh, indent=1)


if __name__ == "__main__":
    main()
