"""Busy / idle accounting of a rocprofv3 kernel trace (one time step window).

    python tools/trace_gaps.py run_kernel_trace.csv [first_visco_index]

Takes the window between two consecutive k_visco_fused launches (one coupled
time step), sums kernel time per kernel name and reports the idle gaps."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
def dur(r):
    return int(r["End_Timestamp"]) - int(r["Start_Timestamp"])


vis = [i for i, r in enumerate(rows) if "k_visco_fused" in r["Kernel_Name"]]
if not vis:  # thermal only: the step ends with T_prev <- T
    vis = [i for i, r in enumerate(rows) if "k_copy" in r["Kernel_Name"]]
# step boundaries: visco launches that did the update (a speculative launch the
# device's Newton test gated off exits at once), and windows that hold a whole
# step (not the back-to-back timing launches after the timed region)
dmax = max(dur(rows[i]) for i in vis)
vis = [i for i in vis if dur(rows[i]) > 0.2 * dmax]
wins = [(a, b) for a, b in zip(vis, vis[1:]) if b - a > 20] or list(zip(vis, vis[1:]))
k = int(sys.argv[2]) if len(sys.argv) > 2 else max(0, len(wins) // 2)
a, b = wins[k]
win = rows[a + 1:b + 1]
t0 = int(rows[a]["End_Timestamp"])
t1 = int(rows[b]["End_Timestamp"])
busy = defaultdict(float)
cnt = defaultdict(int)
gaps = []
prev = t0
for r in win:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("tv::(anonymous namespace)::", "").split("(")[0][:60]
    busy[name] += (e - s) / 1e3
    cnt[name] += 1
    if s > prev:
        gaps.append(((s - prev) / 1e3, name))
    prev = max(prev, e)
wall = (t1 - t0) / 1e3
tot = sum(busy.values())
print(f"step window {wall:.1f} us, kernel busy {tot:.1f} us, idle {wall - tot:.1f} us in {len(gaps)} gaps")
for n, v in sorted(busy.items(), key=lambda x: -x[1]):
    print(f"  {n:60s} {cnt[n]:5d} x {v / cnt[n]:8.1f} us = {v:9.1f} us")
gaps.sort(reverse=True)
print("largest gaps (us, next kernel):")
for g, n in gaps[:12]:
    print(f"  {g:8.1f}  {n}")
print(f"gaps > 10 us: {sum(g for g, _ in gaps if g > 10):.1f} us; <= 10 us: {sum(g for g, _ in gaps if g <= 10):.1f} us")
