#!/usr/bin/env python3
"""GGUF load time (reference target "TinyLlama loaded in < 5 s",
docs/phases/04-AI-RUNTIME.md:331): writes a synthetic GGUF file of the named architecture (exact
per-tensor Q4_K_M layout, random values), then times `load_engine` from that FILE -- mmap, upload
through the pinned staging pipeline, on-device repack, KV/workspace allocation -- and one prefill
as a readiness check.  The file was just written, so it is read from the page cache (warm load).

  python tools/bench_load.py [--models tinyllama-1.1b,mistral-7b] [--json out.jsonl]
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--models", default="tinyllama-1.1b,mistral-7b")
    ap.add_argument("--recipe", default="Q4_K_M")
    ap.add_argument("--dir", default="")
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    import numpy as np

    from aios_amd.models.config import get_preset
    from aios_amd.models.synthetic import write_synthetic_gguf
    from aios_amd.runtime.loader import load_engine

    d = args.dir or tempfile.mkdtemp(prefix="aios_load_")
    for name in args.models.split(","):
        cfg = get_preset(name)
        path = os.path.join(d, f"{name}.{args.recipe}.gguf")
        t = time.time()
        write_synthetic_gguf(path, cfg, args.recipe, seed=1)
        write_s = time.time() - t
        size = os.path.getsize(path)
        t = time.time()
        eng, _, _ = load_engine(path, max_ctx=4096, max_slots=4, max_batch=8)
        load_s = time.time() - t
        t = time.time()
        logits = np.asarray(eng.prefill(0, [cfg.bos_id, 5, 6, 7], 0, True))
        first_s = time.time() - t
        row = {"bench": "gguf load", "model": name, "recipe": args.recipe, "file_gb": round(size / 1e9, 3),
               "load_s": round(load_s, 3), "load_gb_per_s": round(size / 1e9 / load_s, 2),
               "first_prefill_s": round(first_s, 3), "write_s": round(write_s, 2),
               "weight_gb": round(eng.weight_bytes / 1e9, 3), "finite_logits": bool(np.isfinite(logits).all())}
        print(json.dumps(row), flush=True)
        if args.json:
            with open(args.json, "a") as f:
                f.write(json.dumps(row) + "\n")
        del eng
        os.remove(path)


if __name__ == "__main__":
    main()
