#!/usr/bin/env python3
"""Co-resident tiers on ONE MI355X (BASELINE.json config 4): TinyLlama-1.1B (operational) and
Mistral-7B (tactical), both Q4_K_M, random-init weights of those architectures, resident in HBM
together; each engine owns a non-blocking HIP stream and replays its captured decode graph.
Measures B=1 decode tok/s of each model alone, then both decoding at the same time from two host
threads (the agent router dispatching to two tiers concurrently), and the aggregate.

python tools/bench_coresident.py [--steps 512]"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=512)
    ap.add_argument("--prompt", type=int, default=128)
    ap.add_argument("--cu-split", type=int, default=0,
                    help="CUs for the TinyLlama tier's stream (the rest for Mistral; 0: both tiers on every CU)")
    ap.add_argument("--priority", default="",
                    help="tier whose stream gets the high priority (unmasked streams only): tinyllama | mistral")
    print(json.dumps(run(ap.parse_args())), flush=True)


def run(args):
    """the measurement (bench.py's `coresident` secondary calls this); returns the summary dict"""
    import torch  # noqa: F401  (HIP runtime init order as in bench.py)

    from aios_amd.models.config import get_preset
    from aios_amd.runtime.loader import random_engine
    from aios_amd.runtime.native import cu_mask_words, require

    # CU partition: each tier's stream gets its own CUs (hipExtStreamCreateWithCUMask)
    # and the engine sizes its one-workgroup-per-CU grids to them, so the tiers stop trampling each
    # other's dispatch rounds
    split = int(getattr(args, "cu_split", 0) or 0)
    total = require().device_cu_count() if split else 0
    masks = {"tinyllama": cu_mask_words(split, 0, total), "mistral": cu_mask_words(total - split, split // 8, total)} \
        if split else {}
    models = {}
    for name, preset, seed in (("tinyllama", "tinyllama-1.1b", 1), ("mistral", "mistral-7b", 2)):
        cfg = get_preset(preset)
        prio = -1 if (not split and getattr(args, "priority", "") == name) else 0
        eng = random_engine(cfg, "Q4_K_M", seed=seed, max_ctx=((args.prompt + 3 * args.steps + 64) // 128 + 1) * 128,
                            max_slots=1, max_batch=1, cu_mask=masks.get(name), stream_priority=prio)
        models[name] = (cfg, eng)

    pos = {}

    def prep(name):
        cfg, eng = models[name]
        p = [cfg.bos_id] + [(7 * i + 11) % (cfg.vocab_size - 3) + 3 for i in range(args.prompt - 1)]
        first = int(eng.prefill(0, p, 0, True).argmax())
        eng.decode_loop_prepare([0], [first], [args.prompt])
        eng.decode_loop_run(1, 8, True)  # graph capture + warm-up
        eng.synchronize()

    steps = {n: args.steps for n in models}

    def run(name, res):
        _, eng = models[name]
        t0 = time.perf_counter()
        eng.decode_loop_run(1, steps[name], True)
        eng.synchronize()
        res[name] = time.perf_counter() - t0

    out = {"bench": "co-resident tiers, B=1 decode on one GPU", "steps": args.steps, "prompt": args.prompt,
           "cu_split": {"tinyllama": split, "mistral": total - split} if split else None,
           "high_priority_tier": (getattr(args, "priority", "") or None) if not split else None,
           "data": "synthetic (random-init Q4_K_M weights, synthetic prompts)",
           "hbm_weights_gb": round(sum(e.weight_bytes for _, e in models.values()) / 1e9, 3),
           "hbm_gb_per_tier": {n: {"weights": round(e.weight_bytes / 1e9, 3), "kv": round(e.kv_bytes / 1e9, 3),
                                   "workspace": round(e.workspace_bytes / 1e9, 3)} for n, (_, e) in models.items()}}
    for name in models:
        prep(name)
        r = {}
        run(name, r)
        out[f"{name}_alone_tok_s"] = round(args.steps / r[name], 1)
    # concurrent phase: step counts in the ratio of the solo rates, so both streams run for about the
    # same wall time and the aggregate is not a solo tail of the slower model
    for name in models:
        steps[name] = max(16, int(round(args.steps * out[f"{name}_alone_tok_s"] / out["mistral_alone_tok_s"])))
        prep(name)
    r = {}
    ts = [threading.Thread(target=run, args=(n, r)) for n in models]
    t0 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    wall = time.perf_counter() - t0
    for name in models:
        out[f"{name}_concurrent_tok_s"] = round(steps[name] / r[name], 1)
        out[f"{name}_concurrent_steps"] = steps[name]
    out["concurrent_aggregate_tok_s"] = round(sum(steps.values()) / wall, 1)
    # the same token counts run one model after the other (a single decode stream time-sharing the GPU)
    out["time_shared_aggregate_tok_s"] = round(
        sum(steps.values()) / sum(steps[n] / out[f"{n}_alone_tok_s"] for n in models), 1)
    for name in list(models):
        del models[name]
    return out


if __name__ == "__main__":
    main()
