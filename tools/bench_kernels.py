"""Kernel microbenchmarks on the GPU: launch overhead + GEMV bandwidth per shape/format/path.

python tools/bench_kernels.py [--json out.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from aios_amd.gguf.quants import BLOCK_INFO, GGMLType, quantize
from aios_amd.runtime import native


def time_fn(fn, reps=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--sweep", action="store_true", help="grid/U sweep of the q8 GEMV")
    args = ap.parse_args()
    E = native.require()
    out = {"launch": [], "gemv": []}
    for g in (0, 1):
        for blocks in (1, 256, 2048):
            us = E.bench_launch_chain(200, blocks, g, 20)
            out["launch"].append(dict(graph=g, blocks=blocks, us_per_kernel=round(us, 3)))
            print(f"launch chain graph={g} blocks={blocks:5d}: {us:.2f} us/kernel", flush=True)
    st = torch.cuda.current_stream().cuda_stream
    shapes = [("qkv", 6144, 4096), ("o", 4096, 4096), ("gate_up", 28672 * 2, 4096), ("down", 4096, 14336),
              ("lm_head", 32000, 4096), ("tl_gate_up", 5632 * 2, 2048), ("tl_down", 2048, 5632)]
    for t in (GGMLType.Q4_K, GGMLType.Q6_K):
        for name, N, K in shapes:
            if K % 256:
                continue
            raw = np.random.default_rng(0).integers(0, 256, BLOCK_INFO[t][1] * N * K // 256, dtype=np.uint8)
            m = E.QMatrix(int(t), N, K, raw)
            m.fill_random(1, 0.02)
            x = torch.randn(1, K, device="cuda")
            y = torch.zeros(1, N, device="cuda")
            nbytes = N * K // 256 * BLOCK_INFO[t][1]
            for mode in ("v2", "q8"):
                us = time_fn(lambda: E.gemv([m], 1, x.data_ptr(), K, 0, 1e-5, y.data_ptr(), N, E.EPI_STORE, st, 0,
                                            int(mode == "q8")))
                tbs = nbytes / us / 1e6
                out["gemv"].append(dict(fmt=t.name, shape=name, N=N, K=K, mode=mode, us=round(us, 2),
                                        tb_s=round(tbs, 2)))
                print(f"gemv {t.name:5s} {name:10s} N={N:6d} K={K:6d} {mode}: {us:7.2f} us  {tbs:5.2f} TB/s",
                      flush=True)
            del m
    if args.sweep:
        for name, N, K in shapes:
            for t in (GGMLType.Q4_K, GGMLType.Q6_K):
                raw = np.zeros(BLOCK_INFO[t][1] * N * K // 256, dtype=np.uint8)
                m = E.QMatrix(int(t), N, K, raw)
                m.fill_random(1, 0.02)
                x = torch.randn(1, K, device="cuda")
                y = torch.zeros(1, N, device="cuda")
                nbytes = N * K // 256 * BLOCK_INFO[t][1]
                best = None
                for u in (1, 2, 4):
                    for g in (1, 2, 3, 4, 6, 8):
                        us = time_fn(lambda: E.gemv([m], 1, x.data_ptr(), K, 0, 1e-5, y.data_ptr(), N, E.EPI_STORE,
                                                    st, 0, 1, g, u))
                        out.setdefault("sweep", []).append(dict(fmt=t.name, shape=name, u=u, grid=g, us=round(us, 2)))
                        if best is None or us < best[0]:
                            best = (us, u, g)
                print(f"sweep {t.name} {name:10s}: best {best[0]:.2f} us ({nbytes / best[0] / 1e6:.2f} TB/s) "
                      f"U={best[1]} grid/CU={best[2]}", flush=True)
                del m
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
