"""Cold-cache (HBM-resident) per-kernel probe of the decode projections at B = 1 and small B.

Every variant is timed over R rotating copies of its weight matrix (> 512 MB in total, so no call
finds its weights in the 256 MB Infinity Cache), i.e. the bytes come from HBM as they do inside
the decode step.  Variants: the int8-activation GEMV (grid knob), the skinny MFMA GEMM (RB x S),
and torch's streaming sum over a buffer of the same size as the cold-read floor.

python tools/decode_probe.py [--json gpurun_out/decode_probe.jsonl] [--ms 1,4]
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

SHAPES = [("qkv", 6144, 4096, GGMLType.Q4_K), ("o", 4096, 4096, GGMLType.Q4_K),
          ("gate_up", 28672, 4096, GGMLType.Q4_K), ("down_q4k", 4096, 14336, GGMLType.Q4_K),
          ("down_q6k", 4096, 14336, GGMLType.Q6_K), ("lm_head", 32000, 4096, GGMLType.Q6_K)]


def time_rot(fns, reps):
    n = len(fns)
    for i in range(n):
        fns[i]()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for i in range(reps):
        fns[i % n]()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default=None)
    ap.add_argument("--ms", default="1,4")
    ap.add_argument("--shapes", default="")
    ap.add_argument("--dbg", action="store_true", help="GEMV anatomy: prologue off (1) / compute off (2) x U")
    ap.add_argument("--no-skinny", action="store_true")
    args = ap.parse_args()
    E = native.require()
    st = torch.cuda.current_stream().cuda_stream
    out = open(args.json, "w") if args.json else None
    ms = [int(x) for x in args.ms.split(",")]

    def emit(row):
        print(json.dumps(row), flush=True)
        if out:
            out.write(json.dumps(row) + "\n")

    for name, N, K, t in SHAPES:
        if args.shapes and name not in args.shapes.split(","):
            continue
        nbytes = N * K // 256 * BLOCK_INFO[t][1]
        R = max(2, (640 << 20) // nbytes + 1)
        mats = []
        for r in range(R):
            m = E.QMatrix(int(t), N, K, np.zeros(nbytes, dtype=np.uint8))
            m.fill_random(r + 1, 0.02)
            mats.append(m)
        bufs = [torch.empty(nbytes // 4, dtype=torch.int32, device="cuda") for _ in range(R)]
        us = time_rot([lambda b=b: b.sum() for b in bufs], 4 * R)
        emit(dict(shape=name, variant="torch_sum_floor", us=round(us, 2), gbs=round(nbytes / us / 1e3, 1)))
        del bufs
        x = torch.randn(1, K, device="cuda")
        nw = torch.ones(K, device="cuda")
        y = torch.zeros(64, N, device="cuda")
        if args.dbg:
            for u in (0, 1, 2, 3, 4, 13, 14, 21, 22):
                for dbg in (0, 1, 2, 3):
                    fns = [lambda m=m: E.gemv([m], 1, x.data_ptr(), K, nw.data_ptr(), 1e-5, y.data_ptr(), N,
                                              E.EPI_STORE, st, 0, 1, 0, u, 0, dbg) for m in mats]
                    us = time_rot(fns, 4 * R)
                    emit(dict(shape=name, variant="gemv_q8", u=u, dbg=dbg, us=round(us, 2),
                              gbs=round(nbytes / us / 1e3, 1)))
        else:
            for g in (0, 1, 2, 3, 4):
                fns = [lambda m=m: E.gemv([m], 1, x.data_ptr(), K, nw.data_ptr(), 1e-5, y.data_ptr(), N, E.EPI_STORE,
                                          st, 0, 1, g, 0, 0, 0) for m in mats]
                us = time_rot(fns, 4 * R)
                emit(dict(shape=name, variant="gemv_q8", grid=g, us=round(us, 2), gbs=round(nbytes / us / 1e3, 1)))
        for M in ([] if args.no_skinny else ms):
            A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            for rb in (4, 8):
                os.environ["AIOS_SKINNY_RB"] = str(rb)
                for S in (1, 2, 4, 8):
                    fns = [lambda m=m: E.gemm_q(A.data_ptr(), K, [m], M, y.data_ptr(), 0, N, E.GEPI_STORE, st, S)
                           for m in mats]
                    us = time_rot(fns, 4 * R)
                    emit(dict(shape=name, variant="skinny", M=M, RB=rb, S=S, us=round(us, 2),
                              gbs=round(nbytes / us / 1e3, 1)))
            os.environ.pop("AIOS_SKINNY_RB", None)
        del mats
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
