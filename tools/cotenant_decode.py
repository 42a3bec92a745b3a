#!/usr/bin/env python3
"""Co-tenant load for the shared-GPU TP test: a TinyLlama-1.1B (random-init Q4_K_M) batch-1 decode
loop replaying its captured graph on its own stream until --seconds pass or --stop-file appears.
Prints 'ready' once the loop runs, then one JSON line at the end with the steps and tok/s."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=120.0)
    ap.add_argument("--stop-file", default="")
    ap.add_argument("--device", type=int, default=0)
    args = ap.parse_args()
    os.environ.setdefault("AIOS_GEMM_PF_TUNE", "0")
    from aios_amd.models.config import get_preset
    from aios_amd.runtime.loader import random_engine

    cfg = get_preset("tinyllama-1.1b")
    eng = random_engine(cfg, "Q4_K_M", seed=5, max_ctx=4096, max_slots=1, max_batch=1, device=args.device)
    tok = int(eng.prefill(0, [1, 5, 6, 7, 8], 0, True).argmax())
    pos = 5
    eng.decode_loop_prepare([0], [tok], [pos])
    eng.decode_loop_run(1, 8, True)
    eng.synchronize()
    print("ready", flush=True)
    t0 = time.perf_counter()
    steps, chunk = 0, 64
    while time.perf_counter() - t0 < args.seconds and not (args.stop_file and os.path.exists(args.stop_file)):
        eng.decode_loop_run(1, chunk, True)
        eng.synchronize()
        steps += chunk
        if steps % (chunk * 40) == 0:  # restart the sequence long before the context fills
            eng.decode_loop_prepare([0], [tok], [pos])
    dt = time.perf_counter() - t0
    print(json.dumps({"cotenant": "tinyllama-1.1b Q4_K_M B=1 decode", "steps": steps, "seconds": round(dt, 2),
                      "tok_s": round(steps / dt, 1)}), flush=True)


if __name__ == "__main__":
    main()
