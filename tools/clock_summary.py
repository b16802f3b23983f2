"""Effective GPU clock of the hot kernels per process, from one rocprofv3 run
with --kernel-trace and --pmc GRBM_GUI_ACTIVE GRBM_COUNT (GPU-clock cycle
counts per dispatch): clock = cycles / kernel duration.  Used to tell the visco
update's fast and slow processes apart.

    python tools/clock_summary.py DIR [DIR ...]     (one rocprofv3 -d DIR per process)
"""
import csv
import glob
import os
import sys
from collections import defaultdict

KERNELS = {"visco": "k_visco_fused", "march": "k_cg_march<1, false"}


def one(d):
    tr = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    cc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not tr or not cc:
        return None
    dur = {}
    name = {}
    for r in csv.DictReader(open(tr[0])):
        k = r.get("Dispatch_Id") or r.get("Correlation_Id")
        dur[k] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        name[k] = r["Kernel_Name"]
    cyc = defaultdict(dict)
    for r in csv.DictReader(open(cc[0])):
        k = r.get("Dispatch_Id") or r.get("Correlation_Id")
        cyc[k][r["Counter_Name"]] = float(r["Counter_Value"])
        name.setdefault(k, r["Kernel_Name"])
    out = {}
    for tag, pat in KERNELS.items():
        ks = [k for k in cyc if pat in name.get(k, "") and k in dur and dur[k] > 0]
        if not ks:
            continue
        ds = [dur[k] for k in ks]
        ga = [cyc[k].get("GRBM_GUI_ACTIVE", 0.0) / dur[k] * 1e3 for k in ks]  # MHz
        gc = [cyc[k].get("GRBM_COUNT", 0.0) / dur[k] * 1e3 for k in ks]
        out[tag] = (len(ks), sum(ds) / len(ds) / 1e3, sum(ga) / len(ga), sum(gc) / len(gc))
    return out


for d in sys.argv[1:]:
    r = one(d)
    if r is None:
        print(d, "no trace / counters")
        continue
    print(os.path.basename(d.rstrip("/")), "  ".join(
        f"{t}: n {n} {us:7.1f} us  GUI_ACTIVE {a:6.0f} MHz  COUNT {c:6.0f} MHz" for t, (n, us, a, c) in r.items()))
