"""Inter-step idle time of a pipelined decode from a rocprofv3 kernel trace (+ memory-copy trace):
for consecutive decode steps (delimited by sample_kernel), the GPU idle time between a step's sampler
and the next step's first forward kernel, and which copies ran in that window.

  python tools/step_gaps.py gpurun_out/gp/run_kernel_trace.csv [gpurun_out/gp/run_memory_copy_trace.csv]
"""
import csv
import statistics
import sys


def main():
    kt = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
    copies = []
    if len(sys.argv) > 2:
        copies = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Direction", r.get("Operation", "")))
                         for r in csv.DictReader(open(sys.argv[2]))))
    samp = [i for i, r in enumerate(kt) if "sample_kernel" in r["Kernel_Name"]]
    gaps, steps, before = [], [], []
    for a, b in zip(samp, samp[1:]):
        if b - a < 20:  # not a full forward between the two samplers
            continue
        s_end = int(kt[a]["End_Timestamp"])
        nxt = int(kt[a + 1]["Start_Timestamp"])
        gaps.append((nxt - s_end) / 1e3)
        steps.append((int(kt[b]["End_Timestamp"]) - int(kt[a]["End_Timestamp"])) / 1e3)
        # idle inside the step: sum of gaps between its kernels
        before.append(sum(max(0, int(kt[i]["Start_Timestamp"]) - int(kt[i - 1]["End_Timestamp"])) for i in range(a + 2, b + 1)) / 1e3)
    if not gaps:
        print("no decode steps found")
        return
    q = lambda v, p: sorted(v)[int(p * (len(v) - 1))]
    print(f"{len(gaps)} steps: step period median {statistics.median(steps):.1f} us (p90 {q(steps, 0.9):.1f}); "
          f"sampler -> next forward idle median {statistics.median(gaps):.1f} us (p90 {q(gaps, 0.9):.1f}); "
          f"idle between the step's own kernels median {statistics.median(before):.1f} us")
    # kernel time per step by name (the forward's GEMV / attention kernels vs copies / sampler / others)
    from collections import defaultdict
    per = defaultdict(float)
    n = 0
    for a, b in zip(samp, samp[1:]):
        if b - a < 20:
            continue
        n += 1
        for i in range(a + 1, b + 1):
            per[kt[i]["Kernel_Name"].split("(")[0][:60]] += (int(kt[i]["End_Timestamp"]) - int(kt[i]["Start_Timestamp"])) / 1e3
    tot = sum(per.values()) / max(n, 1)
    print(f"kernel time per step {tot:.1f} us:")
    for k, v in sorted(per.items(), key=lambda x: -x[1])[:12]:
        print(f"  {v / n:8.1f} us  {k}")
    if copies:
        lat = [(e - s) / 1e3 for s, e, _ in copies]
        print(f"{len(copies)} copies, median duration {statistics.median(lat):.1f} us")


if __name__ == "__main__":
    main()
