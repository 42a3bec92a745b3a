"""Streaming-read floor of the decode projections (graph-replayed single-read kernels over
rotating HBM-resident buffers) against the GEMVs' in-step times.  python tools/stream_probe.py"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aios_amd.runtime import native

SHAPES = {"qkv": 15.2e6, "o": 9.4e6, "gate_up": 66.1e6, "down_q4k": 33.0e6, "down_q6k": 48.2e6, "lm_head": 107.5e6}


def main():
    E = native.require()
    only = os.environ.get("STREAM_SHAPES", "")
    for name, b in SHAPES.items():
        if only and name not in only.split(","):
            continue
        b = int(b) // 4096 * 4096
        nbuf = max(4, (768 << 20) // b + 1)
        best = None
        for wg in (1, 2, 4, 8):
            for u in (1, 2, 4, 8):
                for th in (256, 512):
                    us = E.bench_stream_read(b, nbuf, wg, u, th, 20)
                    row = dict(shape=name, mb=round(b / 1e6, 1), wg_per_cu=wg, u=u, threads=th, us=round(us, 2),
                               tbs=round(b / us / 1e6, 2))
                    if best is None or us < best["us"]:
                        best = row
                    if os.environ.get("STREAM_ALL"):
                        print(json.dumps(row), flush=True)
        print(json.dumps(dict(best, best=True)), flush=True)
        # access pattern at the decode GEMV geometry (1 workgroup per CU, U = 4): grid-strided 16 B
        # pieces vs per-CU contiguous slices vs 2 KB pieces dealt round-robin
        for th in (512, 1024):
            row = dict(shape=name, threads=th, strided=round(E.bench_stream_read(b, nbuf, 1, 4, th, 20), 2))
            for mode, tag in ((1, "slices"), (2, "pieces2k")):
                row[tag] = round(E.bench_stream_read_part(b, nbuf, mode, th, 20), 2)
            print(json.dumps(row), flush=True)
    print(json.dumps({"launch_chain_us": round(E.bench_launch_chain(200, 256, 1, 20), 2)}))


if __name__ == "__main__":
    main()
