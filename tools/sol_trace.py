"""One-launch streaming-read speed of light from a kernel trace of `mall_probe --sol MB...`
(tools/mall_probe.hip): per size, the median kernel time of a cold-cache read with the default and the
non-temporal policy, and the rate.

  rocprofv3 --kernel-trace --output-format csv -d gpurun_out/sol -- /tmp/mall_probe --sol 9.4 14.2 48 66
  python tools/sol_trace.py gpurun_out/sol/.../*_kernel_trace.csv 9.4 14.2 48 66
"""
import csv
import statistics
import sys


def main():
    path, sizes = sys.argv[1], [float(x) for x in sys.argv[2:]]
    kt = sorted((r for r in csv.DictReader(open(path)) if "stream_read" in r["Kernel_Name"]),
                key=lambda r: int(r["Start_Timestamp"]))
    if len(kt) != 20 * len(sizes):
        raise SystemExit(f"expected {20 * len(sizes)} stream_read dispatches, found {len(kt)}")
    us = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in kt]
    print(f"{'MB':>7} {'default_us':>11} {'TB/s':>6} {'nt_us':>8} {'TB/s':>6}")
    for i, mb in enumerate(sizes):
        blk = us[20 * i: 20 * (i + 1)]
        d, n = statistics.median(blk[1::4]), statistics.median(blk[3::4])  # [flush, default, flush, nt] x 5
        b = mb * 1048576
        print(f"{mb:7.1f} {d:11.2f} {b / d / 1e6:6.2f} {n:8.2f} {b / n / 1e6:6.2f}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
