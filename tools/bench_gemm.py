"""Matrix-core GEMM benchmark on one GPU: the engine's dequant-fused GEMMs (skinny M <= 64 for
batched decode, big-M tiles for prefill) on the Mistral-7B projection shapes, next to torch's bf16
matmul (hipBLASLt / rocBLAS on an unquantised bf16 copy) as the library yardstick.

python tools/bench_gemm.py [--ms 2,4,8,16,32,64,512,2048] [--json out.jsonl]
Per row: us per call, TFLOP/s, effective weight-stream GB/s (quantised bytes / time).
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

SHAPES = [  # name, N, K, qtype, epilogue
    ("qkv", 6144, 4096, GGMLType.Q4_K, "store"),
    ("o", 4096, 4096, GGMLType.Q4_K, "accum"),
    ("gate_up", 28672, 4096, GGMLType.Q4_K, "swiglu"),
    ("down_q4k", 4096, 14336, GGMLType.Q4_K, "accum"),
    ("down_q6k", 4096, 14336, GGMLType.Q6_K, "accum"),
]


def time_fn(fn, reps=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ms", default="1,2,4,8,16,32,64,512,2048")
    ap.add_argument("--json", default=None)
    ap.add_argument("--no-torch", action="store_true")
    ap.add_argument("--sweep", action="store_true", help="skinny kernel: RB x split-K sweep per shape")
    ap.add_argument("--pf-sweep", action="store_true", help="prefill GEMM: tile x split-K sweep per shape")
    ap.add_argument("--pf-probe", action="store_true", help="prefill GEMM 256x256 Q4_K: timing-anatomy probes")
    ap.add_argument("--shapes", default=None, help="comma list of shape names (default: all)")
    args = ap.parse_args()
    E = native.require()
    st = torch.cuda.current_stream().cuda_stream
    ms = [int(x) for x in args.ms.split(",")]
    out = open(args.json, "w") if args.json else None
    for name, N, K, t, epi in SHAPES:
        if args.shapes and name not in args.shapes.split(","):
            continue
        nbytes = N * K // 256 * BLOCK_INFO[t][1]
        raw = np.random.default_rng(0).integers(0, 256, nbytes, dtype=np.uint8)
        m = E.QMatrix(int(t), N, K, raw)
        m.fill_random(1, 0.02)
        wb = torch.randn(N, K, device="cuda", dtype=torch.bfloat16) * 0.02 if not args.no_torch else None
        if args.pf_probe:
            if t != GGMLType.Q4_K:
                continue
            for M in ms:
                A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
                C = torch.zeros(M, N, device="cuda")
                for probe in (300, 301, 304, 308, 313, 364, 368, 377):
                    us = time_fn(lambda: E.gemm_pf_probe(A.data_ptr(), K, m, M, C.data_ptr(), probe, st), reps=10)
                    row = dict(probe=probe, shape=name, M=M, us=round(us, 2), tflops=round(2 * M * N * K / us / 1e6, 1))
                    print(json.dumps(row), flush=True)
            continue
        if args.pf_sweep:
            for M in ms:
                A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
                C = torch.zeros(M, N, device="cuda")
                C16 = torch.zeros(M, N // 2, device="cuda", dtype=torch.bfloat16)
                plan = E.gemm_pf_plan([m], M, E.GEPI_ACCUM, 0)
                for tile in ("256x256", "128x256", "64x256", "256x128", "128x128", "64x128"):
                    os.environ["AIOS_GEMM_PF_TILE"] = tile
                    for S in ((1,) if epi == "swiglu" else (1, 2, 4, 8)):
                        if epi == "swiglu":
                            fn = lambda: E.gemm_q(A.data_ptr(), K, [m], M, 0, C16.data_ptr(), N // 2, E.GEPI_SWIGLU_BF16, st)
                        else:
                            fn = lambda: E.gemm_q(A.data_ptr(), K, [m], M, C.data_ptr(), 0, N, E.GEPI_ACCUM, st, S)
                        us = time_fn(fn, reps=10)
                        row = dict(pf=1, shape=name, M=M, tile=tile, S=S, us=round(us, 2),
                                   tflops=round(2 * M * N * K / us / 1e6, 1), auto=list(plan))
                        print(json.dumps(row), flush=True)
                        if out:
                            out.write(json.dumps(row) + "\n")
                os.environ.pop("AIOS_GEMM_PF_TILE", None)
            continue
        if args.sweep:
            for M in ms:
                A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
                C = torch.zeros(M, N, device="cuda")
                for rb in (4, 8):
                    os.environ["AIOS_SKINNY_RB"] = str(rb)
                    for S in (1, 2, 3, 4, 6, 8):
                        us = time_fn(lambda: E.gemm_q(A.data_ptr(), K, [m], M, C.data_ptr(), 0, N, E.GEPI_STORE, st, S),
                                     reps=50)
                        row = dict(sweep=1, shape=name, M=M, RB=rb, S=S, us=round(us, 2),
                                   weight_gbs=round(nbytes / us / 1e3, 1))
                        print(json.dumps(row), flush=True)
                        if out:
                            out.write(json.dumps(row) + "\n")
                os.environ.pop("AIOS_SKINNY_RB", None)
            continue
        for M in ms:
            A = torch.randn(M, K, device="cuda").to(torch.bfloat16)
            C = torch.zeros(M, N, device="cuda")
            C16 = torch.zeros(M, N // 2, device="cuda", dtype=torch.bfloat16)
            if epi == "swiglu":
                fn = lambda: E.gemm_q(A.data_ptr(), K, [m], M, 0, C16.data_ptr(), N // 2, E.GEPI_SWIGLU_BF16, st)
            else:
                e = E.GEPI_STORE if epi == "store" else E.GEPI_ACCUM
                fn = lambda: E.gemm_q(A.data_ptr(), K, [m], M, C.data_ptr(), 0, N, e, st)
            us = time_fn(fn, reps=50 if M <= 64 else 10)
            row = dict(shape=name, M=M, N=N, K=K, qtype=int(t), us=round(us, 2),
                       tflops=round(2 * M * N * K / us / 1e6, 1), weight_gbs=round(nbytes / us / 1e3, 1))
            if wb is not None:
                ut = time_fn(lambda: torch.matmul(A, wb.T), reps=50 if M <= 64 else 10)
                row.update(torch_bf16_us=round(ut, 2), torch_tflops=round(2 * M * N * K / ut / 1e6, 1))
            print(json.dumps(row), flush=True)
            if out:
                out.write(json.dumps(row) + "\n")
        del wb
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
