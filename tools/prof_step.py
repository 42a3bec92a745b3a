"""Summarise the decode steps of a rocprofv3 kernel_trace.csv: per-kernel time and launch gaps.

Steps are the kernel runs between consecutive sample_kernel launches; every step with the modal
kernel count contributes, and each position's duration / gap is the MEDIAN over those steps (one
step alone is noisy, and the last one is followed by host work)."""
import csv
import statistics
import sys
from collections import Counter, defaultdict

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "sample_kernel" in r["Kernel_Name"]]
steps = [rows[a + 1:b + 1] for a, b in zip(idx, idx[1:])]
n_mode = Counter(len(s) for s in steps).most_common(1)[0][0]
steps = [s for s in steps if len(s) == n_mode][2:]  # drop the first (warm-up) ones
name = lambda r: r["Kernel_Name"].split("(")[0][:70]
dur = [[(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in s] for s in steps]
gap = [[0.0] + [(int(s[i]["Start_Timestamp"]) - int(s[i - 1]["End_Timestamp"])) / 1e3 for i in range(1, len(s))]
       for s in steps]
med_d = [statistics.median(d[i] for d in dur) for i in range(n_mode)]
med_g = [statistics.median(g[i] for g in gap) for i in range(n_mode)]
walls = [(int(s[-1]["End_Timestamp"]) - int(s[0]["Start_Timestamp"])) / 1e3 for s in steps]
print(f"{len(steps)} steps of {n_mode} kernels: median wall {statistics.median(walls):.1f} us, "
      f"sum of median kernel times {sum(med_d):.1f} us, sum of median gaps {sum(med_g):.1f} us")
agg = defaultdict(lambda: [0, 0.0])
for i, r in enumerate(steps[0]):
    agg[name(r)][0] += 1
    agg[name(r)][1] += med_d[i]
for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{v[1]:9.1f} us {v[0]:4d}x  avg {v[1] / v[0]:7.2f}  {k}")
print("--- layer 1 (median over steps)")
s0 = steps[0]
# layer 1 starts where layer 0 did (the step's second kernel seen again); none: print from kernel 1
first = next((i for i, r in enumerate(s0) if i > 2 and name(r) == name(s0[1])), 1)
for i in range(first, min(first + 9, n_mode)):
    r = s0[i]
    print(f"  +{med_g[i]:5.2f} gap  {med_d[i]:7.2f} us  grid={r['Grid_Size_X']:>7} wg={r['Workgroup_Size_X']:>4} "
          f"vgpr={r['VGPR_Count']:>3} lds={r['LDS_Block_Size']:>6}  {name(r)[:60]}")
