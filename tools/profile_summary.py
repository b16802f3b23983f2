"""Cross-check of bench.py's in-solve kernel timing against a rocprofv3 kernel
trace of the same command:

    python tools/profile_summary.py PROF_DIR BENCH_JSON OUT_JSON

For each hot kernel: the rocprofv3 mean over all dispatches, and the mean over
the dispatches of bench.py's timed steps that do work.  The timed steps are
located by the visco update launches (one per step: `warmup` of them precede
the timed region, which ends with the `steps`-th after them); "do work" means
> 20 us: after the PCG has converged, the launches queued behind the
convergence poll exit at their first instruction in ~5-7 us, and bench.py's
in-solve timing covers the converging iterations only."""
import csv
import json
import os
import statistics
import sys

prof, bench_json, out = sys.argv[1:4]
bench = json.load(open(bench_json))
rows = list(csv.DictReader(open(os.path.join(prof, "run_kernel_trace.csv"))))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
pats = {"pcg_matvec_fused": "k_cg_march<1, true", "pcg_update": "k_pcg_update<", "visco_update": "k_visco_fused<"}

vis = [r for r in rows if pats["visco_update"] in r["Kernel_Name"]]
dur = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in vis]
# the updates that ran: a step's end is queued speculatively, gated on the
# device's Newton test, and a gated-off launch exits at once
visco_end = [int(r["End_Timestamp"]) for r, d in zip(vis, dur) if d > 0.2 * max(dur)]
w, k = bench["warmup"], bench["steps"]
window = (visco_end[w - 1] if w > 0 else 0, visco_end[w + k - 1]) if len(visco_end) >= w + k else None

res = {"source": f"rocprofv3 --kernel-trace --stats ({prof}) vs bench.py in-solve timing "
                 "(device clock stamps for the PCG kernels, HIP events for the visco update)",
       "timed_window_ns": window, "kernels": {}}
for name, pat in pats.items():
    sel = [r for r in rows if pat in r["Kernel_Name"]]
    d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in sel]
    if not d:
        continue
    timed = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in sel
             if window and window[0] < int(r["Start_Timestamp"]) < window[1]]
    work = [x for x in timed if x > 20.0]
    kb = bench["kernels"].get(name, {})
    bus = kb.get("ms", 0.0) * 1e3
    wm = sum(work) / len(work) if work else None
    res["kernels"][name] = {
        "rocprof_dispatches": len(d), "rocprof_mean_us": sum(d) / len(d),
        "rocprof_timed_steps_working_dispatches": len(work), "rocprof_timed_steps_working_mean_us": wm,
        "rocprof_timed_steps_working_median_us": statistics.median(work) if work else None,
        "bench_in_solve_us": bus, "bench_isolated_us": kb.get("ms_isolated", 0.0) * 1e3,
        "bench_launches_timed": kb.get("launches_timed"),
        "bench_over_rocprof": bus / wm if wm else None,
    }
# the flushed J x of bench.py's hbm_flushed record under the same trace: the
# kernels between each Infinity-Cache sweep (k_read_sweep) and the next one
# (the march + k_cg_addfaces), their durations summed -- the rocprof
# counterpart of bench.py's HIP-event median, which includes the dispatch
sweeps = [i for i, r in enumerate(rows) if "k_read_sweep" in r["Kernel_Name"]]
fl = []
for i in sweeps:
    ks = []
    j = i + 1
    while j < len(rows) and len(ks) < 3 and "k_read_sweep" not in rows[j]["Kernel_Name"] \
            and "fillBuffer" not in rows[j]["Kernel_Name"]:
        ks.append(rows[j])
        j += 1
    if ks:
        fl.append(sum(int(k["End_Timestamp"]) - int(k["Start_Timestamp"]) for k in ks) / 1e3)
hf = bench.get("roofline", {}).get("hbm_flushed")
if fl and hf:
    med = statistics.median(fl)
    res["hbm_flushed"] = {"launches": len(fl), "rocprof_median_us": round(med, 2),
                          "bench_hip_event_median_us": round(hf["ms_per_launch"] * 1e3, 2),
                          "bytes_per_launch": hf["bytes_per_launch"],
                          "rocprof_frac": round(hf["bytes_per_launch"] / (med * 1e-6) / 8e12, 4),
                          "bench_frac": round(hf["frac"], 4)}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
