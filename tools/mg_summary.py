"""Summarise a gpu_mg.sh run: bench line and per-(kernel, grid size) trace means."""
import collections
import csv
import json
import sys

out = sys.argv[1]
d = json.load(open(f"{out}/b_gmg.json"))
print(round(d["ms_per_step"], 2), "ms/step", d["config"]["newton_its_per_step"], d["config"]["krylov_its_per_step"],
      "its", {k: (round(v["ms"] * 1e3, 1), round(v["GBps"])) for k, v in d["kernels"].items()})
g = collections.defaultdict(list)
for r in csv.DictReader(open(f"{out}/prof/run_kernel_trace.csv")):
    n = r["Kernel_Name"].replace("void ", "").replace("tv::(anonymous namespace)::", "").split("(")[0]
    g[(n, r["Grid_Size_X"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
for k, v in sorted(g.items(), key=lambda kv: -sum(kv[1]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 24]:
    print(f"{k[0][:40]:40s} grid {k[1]:>10s} n {len(v):5d} mean {sum(v) / len(v) / 1e3:8.1f} us")
