"""Batched-decode skinny MFMA GEMM anatomy on MI355X (kernels/gemm_skinny.hip): per Mistral-7B
projection at B rows, the graph-replayed launch time over rotating HBM-resident weight copies, the
bytes it moves per us, and one cold launch's in-kernel phase stamps (s_memrealtime, 10 ns ticks)
across workgroups: start, prologue loads issued, first X chunk staged, main loop done, split-K slab
published + ticket, last arriver done.

python tools/skinny_probe.py [--batch 8] [--only qkv,o,gate_up,down]
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

Q4, Q6 = GGMLType.Q4_K, GGMLType.Q6_K
SHAPES = [  # name, [(fmt, rows)], K, epilogue
    ("qkv", [(Q4, 5120), (Q6, 1024)], 4096, "STORE"),
    ("o", [(Q4, 4096)], 4096, "ACCUM"),
    ("gate_up", [(Q4, 28672)], 4096, "SWIGLU_BF16"),
    ("down", [(Q6, 4096)], 14336, "ACCUM"),
]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--only", default="")
    args = ap.parse_args()
    E = native.require()
    B = args.batch
    for name, segs, K, epi in SHAPES:
        if args.only and name not in args.only.split(","):
            continue
        nbytes = sum(BLOCK_INFO[t][1] * r * K // 256 for t, r in segs)
        nrot = max(2, (640 << 20) // nbytes + 1)
        mats = []
        for i in range(nrot):
            ms = []
            for j, (t, r) in enumerate(segs):
                m = E.QMatrix(int(t), r, K, np.zeros(BLOCK_INFO[t][1] * r * K // 256, dtype=np.uint8))
                m.fill_random(11 + 3 * i + j, 0.02)
                ms.append(m)
            mats.append(ms)
        N = sum(r for _, r in segs)
        A = (torch.randn(B, K, device="cuda") * 0.5).to(torch.bfloat16)
        C = torch.zeros(B, N, device="cuda")
        C16 = torch.zeros(B, N // 2, dtype=torch.bfloat16, device="cuda")
        ldc = N // 2 if epi == "SWIGLU_BF16" else N
        e = getattr(E, "GEPI_" + epi)

        def launch(ms, ts=0):
            E.gemm_q(A.data_ptr(), K, ms, B, C.data_ptr(), C16.data_ptr(), ldc, e,
                     torch.cuda.current_stream().cuda_stream, 0, dbg_ts=ts)

        for ms in mats:
            launch(ms)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for ms in mats:
                launch(ms)
        g.replay()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 20
        e0.record()
        for _ in range(reps):
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / (reps * nrot)
        row = dict(shape=name, B=B, mb=round(nbytes / 1e6, 1), us=round(us, 2), tbs=round(nbytes / us / 1e6, 2))
        G = 4096
        ts = torch.zeros(G * 8, dtype=torch.int64, device="cuda")
        launch(mats[0], ts.data_ptr())
        torch.cuda.synchronize()
        t = ts.view(G, 8).cpu().numpy().astype(np.float64)
        t = t[t[:, 0] > 0]
        row["workgroups"] = int(len(t))
        if not len(t):  # the ring GEMM (gemm_ring.hip) writes no stamps
            print(json.dumps(row), flush=True)
            del mats
            torch.cuda.empty_cache()
            continue
        t0 = t[:, 0].min()
        rel = (t - t0) / 100.0
        names = ["start", "loads_issued", "x_staged", "loop_done", "done_slice", "done_epilogue"]
        st = {}
        for i, nm in enumerate(names):
            v = rel[:, i][t[:, i] > 0]
            if len(v):
                st[nm] = [round(float(np.percentile(v, q)), 2) for q in (0, 50, 100)]
        row["stamps_us"] = st
        print(json.dumps(row), flush=True)
        del mats
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
