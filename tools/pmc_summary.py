#!/usr/bin/env python3
"""Per-kernel averages of a rocprofv3 --pmc counter_collection.csv (one row per dispatch x counter).

  python tools/pmc_summary.py gpurun_out/pmc/run_counter_collection.csv [--top 12]
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=12)
    args = ap.parse_args()
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    with open(args.csv) as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"]
            acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add(r["Dispatch_Id"])
    rows = sorted(acc.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0.0))[:args.top]
    for k, c in rows:
        n = len(disp[k])
        avg = {name: v / n for name, v in sorted(c.items())}
        line = " ".join(f"{name}={v:.4g}" for name, v in avg.items())
        extra = ""
        if avg.get("SQ_WAVE_CYCLES"):
            wc = avg["SQ_WAVE_CYCLES"]
            extra = (f" | valu_active/wave_cyc={avg.get('SQ_ACTIVE_INST_VALU', 0) / wc:.3f}"
                     f" wait_any/wave_cyc={avg.get('SQ_WAIT_ANY', 0) / wc:.3f}"
                     f" wait_inst/wave_cyc={avg.get('SQ_WAIT_INST_ANY', 0) / wc:.3f}")
        print(f"{k[:70]:70s} x{n}: {line}{extra}")


if __name__ == "__main__":
    main()
