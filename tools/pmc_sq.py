"""Mean SQ counters per dispatch for the kernels matching the given patterns,
from one rocprofv3 --pmc pass (SQ_* cycle counters are quad-cycles on gfx950,
MI355X_MICROARCH.md; WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES):

    python tools/pmc_sq.py PMC_DIR PATTERN [PATTERN ...]
"""
import csv
import glob
import os
import sys
from collections import defaultdict

d, pats = sys.argv[1], sys.argv[2:]
vals = defaultdict(lambda: defaultdict(list))
for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            for p in pats:
                if p in row["Kernel_Name"]:
                    vals[p][row["Counter_Name"]].append(float(row["Counter_Value"]))
for p in pats:
    print(p)
    c = vals[p]
    for k in sorted(c):
        v = c[k]
        print(f"  {k:24s} {sum(v) / len(v):16.1f}  ({len(v)} dispatches)")
    w = c.get("SQ_WAVE_CYCLES")
    if w:
        W = sum(w) / len(w)
        for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
            if k in c:
                print(f"  {k:24s} {sum(c[k]) / len(c[k]) / W:8.3f} of SQ_WAVE_CYCLES")
