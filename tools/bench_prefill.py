"""Prefill (TTFT) benchmark on one GPU: time to prefill T prompt tokens of a random-init model,
GEMM path (MFMA GEMMs + flash attention) vs the batched-GEMV path.
python tools/bench_prefill.py [--model mistral-7b] [--lens 128,512,2048]"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--recipe", default="Q4_K_M")
    ap.add_argument("--lens", default="128,512,2048")
    ap.add_argument("--gemv", action="store_true", help="also time the GEMV path")
    args = ap.parse_args()
    from aios_amd.models.config import get_preset
    from aios_amd.runtime.loader import random_engine

    cfg = get_preset(args.model)
    lens = [int(x) for x in args.lens.split(",")]
    rows = []
    for path in (["gemm", "gemv"] if args.gemv else ["gemm"]):
        os.environ["AIOS_PREFILL_GEMM"] = "1" if path == "gemm" else "0"
        eng = random_engine(cfg, args.recipe, seed=3, max_ctx=max(lens) + 64, max_slots=1, max_batch=1)
        for T in lens:
            if path == "gemv" and T > 512:
                continue
            p = [cfg.bos_id] + [(11 * i) % (cfg.vocab_size - 3) + 3 for i in range(T - 1)]
            eng.prefill(0, p, 0, True)  # warm (graph-free path; kernels loaded)
            n = 3
            t0 = time.perf_counter()
            for _ in range(n):
                eng.prefill(0, p, 0, True)
            dt = (time.perf_counter() - t0) / n
            r = dict(path=path, model=args.model,
                     recipe=args.recipe, prompt_tokens=T, ms=round(dt * 1e3, 2),
                     tok_per_s=round(T / dt, 1))
            rows.append(r)
            print(json.dumps(r), flush=True)
        del eng


if __name__ == "__main__":
    main()
