"""Mean PMC counter values per dispatch, grouped by kernel name, from rocprofv3 counter_collection CSVs."""
import csv
import glob
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
agg = defaultdict(lambda: defaultdict(list))
for path in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].split("(")[0][:64]
        agg[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name, cs in sorted(agg.items(), key=lambda kv: -kv[1].get("SQ_BUSY_CYCLES", [0])[0] if kv[1].get("SQ_BUSY_CYCLES") else 0):
    print(name)
    for c, v in sorted(cs.items()):
        print(f"    {c:24s} {sum(v) / len(v):16.1f}  (n={len(v)})")
