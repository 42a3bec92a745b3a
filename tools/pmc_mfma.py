#!/usr/bin/env python3
"""MFMA busy fraction and LDS bank-conflict share per kernel from one rocprofv3 --pmc pass with
--kernel-trace (tools/gpu_r6_pmc.sh): SQ_VALU_MFMA_BUSY_CYCLES (chip-wide MFMA busy cycles, 32 per
32x32x16 bf16 MFMA) over the dispatch's duration x 1,024 SIMDs x the clock, and
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE.

  python tools/pmc_mfma.py <run>_counter_collection.csv <run>_kernel_trace.csv [--grep gemm_pf] [--ghz 2.4]
"""
import argparse
import csv
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("counters")
    ap.add_argument("trace")
    ap.add_argument("--grep", default="")
    ap.add_argument("--ghz", type=float, default=2.4)
    ap.add_argument("--simds", type=int, default=1024)
    a = ap.parse_args()
    dur = {r["Dispatch_Id"]: int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in csv.DictReader(open(a.trace))}
    per = defaultdict(lambda: defaultdict(float))  # (kernel, dispatch) -> counter -> value
    for r in csv.DictReader(open(a.counters)):
        if a.grep and a.grep not in r["Kernel_Name"]:
            continue
        per[(r["Kernel_Name"].split("(")[0], r["Dispatch_Id"])][r["Counter_Name"]] += float(r["Counter_Value"])
    agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0, 0.0])  # n, ns, mfma busy, lds conflict, lds active
    for (k, d), c in per.items():
        if d not in dur:
            continue
        g = agg[k]
        g[0] += 1
        g[1] += dur[d]
        g[2] += c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        g[3] += c.get("SQ_LDS_BANK_CONFLICT", 0.0)
        g[4] += c.get("SQ_LDS_IDX_ACTIVE", 0.0)
    print(f"{'kernel':60s} {'n':>4s} {'avg_us':>8s} {'mfma_busy':>9s} {'lds_confl':>9s}")
    for k, (n, ns, mb, lc, la) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
        cyc = ns * a.ghz * a.simds
        print(f"{k[:60]:60s} {n:4d} {ns / n / 1e3:8.1f} {mb / cyc if cyc else 0:9.3f} {lc / la if la else 0:9.3f}")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
