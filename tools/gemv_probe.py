"""Where does a decode GEMV's time go?  Times the q8 GEMV per Mistral shape with the x staging
and/or the dot compute disabled (tune_dbg bits), back to back in a hipGraph-free loop.

python tools/gemv_probe.py [--json gpurun_out/gemv_probe.json]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np
import torch

from aios_amd.gguf.quants import BLOCK_INFO, GGMLType
from aios_amd.runtime import native
from tools.bench_kernels import time_fn


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--u", type=int, default=0)
    ap.add_argument("--sweep", action="store_true", help="U x blocks-per-CU sweep per shape")
    args = ap.parse_args()
    E = native.require()
    st = torch.cuda.current_stream().cuda_stream
    shapes = [("qkv", 6144, 4096, True), ("o", 4096, 4096, False), ("gate_up", 28672, 4096, True),
              ("down", 4096, 14336, False), ("lm_head", 32000, 4096, True)]
    res = []
    for t in (GGMLType.Q4_K, GGMLType.Q6_K):
        for name, N, K, norm in shapes:
            raw = np.zeros(BLOCK_INFO[t][1] * N * K // 256, dtype=np.uint8)
            m = E.QMatrix(int(t), N, K, raw)
            m.fill_random(1, 0.02)
            x = torch.randn(1, K, device="cuda")
            nw = torch.ones(K, device="cuda")
            y = torch.zeros(1, N, device="cuda")
            nbytes = N * K // 256 * BLOCK_INFO[t][1]
            line = []
            for dbg in (0, 1, 2, 3, 4, 8, 12):
                us = time_fn(lambda: E.gemv([m], 1, x.data_ptr(), K, nw.data_ptr() if norm else 0, 1e-5, y.data_ptr(),
                                            N, E.EPI_STORE, st, 0, 1, 0, args.u, 0, dbg), reps=100)
                res.append(dict(fmt=t.name, shape=name, dbg=dbg, us=round(us, 2), tb_s=round(nbytes / us / 1e6, 2)))
                line.append(f"dbg{dbg} {us:6.2f}us {nbytes / us / 1e6:4.2f}TB/s")
            print(f"{t.name:5s} {name:8s} N={N:6d} K={K:6d} {nbytes / 1e6:6.1f}MB | " + " | ".join(line), flush=True)
            del m
    # Q4_K_M mixed QKV (Q,K rows Q4_K + V rows Q6_K): one launch, one x staging
    mq = E.QMatrix(int(GGMLType.Q4_K), 5120, 4096, np.zeros(144 * 5120 * 16, dtype=np.uint8))
    mv = E.QMatrix(int(GGMLType.Q6_K), 1024, 4096, np.zeros(210 * 1024 * 16, dtype=np.uint8))
    mq.fill_random(1, 0.02)
    mv.fill_random(2, 0.02)
    x = torch.randn(1, 4096, device="cuda")
    nw = torch.ones(4096, device="cuda")
    y = torch.zeros(1, 6144, device="cuda")
    nbytes = 144 * 5120 * 16 + 210 * 1024 * 16
    line = []
    for dbg in (0, 1, 2, 3):
        us = time_fn(lambda: E.gemv([mq, mv], 1, x.data_ptr(), 4096, nw.data_ptr(), 1e-5, y.data_ptr(), 6144,
                                    E.EPI_STORE, st, 0, 1, 0, args.u, 0, dbg), reps=100)
        res.append(dict(fmt="Q4_K+Q6_K", shape="qkv_mixed", dbg=dbg, us=round(us, 2)))
        line.append(f"dbg{dbg} {us:6.2f}us {nbytes / us / 1e6:4.2f}TB/s")
    print(f"Q4K+Q6K qkv_mix N=  6144 K=  4096 {nbytes / 1e6:6.1f}MB | " + " | ".join(line), flush=True)
    if args.sweep:
        for t in (GGMLType.Q4_K, GGMLType.Q6_K):
            for name, N, K, norm in shapes:
                raw = np.zeros(BLOCK_INFO[t][1] * N * K // 256, dtype=np.uint8)
                m = E.QMatrix(int(t), N, K, raw)
                m.fill_random(1, 0.02)
                x = torch.randn(1, K, device="cuda")
                nw = torch.ones(K, device="cuda")
                y = torch.zeros(1, N, device="cuda")
                cells = []
                for u in list(range(1, 9)) + [13, 14, 21, 22, 31]:
                    uu = {13: 3, 14: 4, 21: 1, 22: 2, 31: 1}.get(u, u)
                    if (K // 32 + 64 * uu - 1) // (64 * uu) > 4:
                        continue
                    for g in (1, 2, 3, 4):
                        us = time_fn(lambda: E.gemv([m], 1, x.data_ptr(), K, nw.data_ptr() if norm else 0, 1e-5,
                                                    y.data_ptr(), N, E.EPI_STORE, st, 0, 1, g, u, 0, 0), reps=60)
                        cells.append((us, u, g))
                        res.append(dict(fmt=t.name, shape=name, sweep_u=u, sweep_grid=g, us=round(us, 2)))
                cells.sort()
                print(f"sweep {t.name} {name}: best " + ", ".join(f"u{u}/g{g} {us:.2f}us" for us, u, g in cells[:4]),
                      flush=True)
                del m
    # pure launch/boundary floor for reference
    for blocks in (256, 1024):
        print(f"empty-chain eager blocks={blocks}: {E.bench_launch_chain(200, blocks, 0, 20):.2f} us/kernel")
    if args.json:
        with open(args.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
