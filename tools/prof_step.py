"""Summarise one decode step from a rocprofv3 kernel_trace.csv: per-kernel time, gaps, bandwidth."""
import csv
import sys
from collections import defaultdict

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof/run_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "sample_kernel" in r["Kernel_Name"]]
a, b = idx[-2], idx[-1]
step = rows[a + 1:b + 1]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in step)
print(f"step wall {(t1 - t0) / 1e3:.1f} us, busy {busy / 1e3:.1f} us, {len(step)} kernels")
agg = defaultdict(lambda: [0, 0])
for r in step:
    n = r["Kernel_Name"].split("(")[0][:70]
    d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    agg[n][0] += 1
    agg[n][1] += d
for k, v in sorted(agg.items(), key=lambda x: -x[1][1]):
    print(f"{v[1] / 1e3:9.1f} us {v[0]:4d}x  avg {v[1] / v[0] / 1e3:7.2f}  {k}")
print("--- first layer")
prev = t0
for r in step[:9]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"  +{(s - prev) / 1e3:6.2f} gap  {(e - s) / 1e3:7.2f} us  grid={r['Grid_Size_X']:>7} wg={r['Workgroup_Size_X']:>4} "
          f"vgpr={r['VGPR_Count']:>3} lds={r['LDS_Block_Size']:>6}  {r['Kernel_Name'].split('(')[0][:60]}")
    prev = e
