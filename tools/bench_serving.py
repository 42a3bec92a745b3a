#!/usr/bin/env python3
"""Serving benchmark of the reference's hottest inference pattern: N concurrent
JSON-mode streams whose prompts share a long prefix -- the autonomy loop resends its tool catalogue
and format rules every round (`agent-core/src/autonomy.rs:988-1036`) with up to 3 reasoning loops
at once (`:376,632`).

Runs the real serving path: ModelManager -> Scheduler (admission with paged-KV prefix sharing,
chunked prefill interleaved with batched decode, per-step JSON grammar masks, device sampling with
temperature / top-k / top-p) -> native Engine, on a random-init model of the named architecture.

Reports TTFT p50/p90, inter-token latency (ITL) p50, aggregate decode tok/s, prefix-shared tokens,
and the bare decode-step time of the same engine at the same batch (the ITL floor).

  python tools/bench_serving.py [--model mistral-7b] [--streams 8] [--prompt 3072] [--shared 2048]
                                [--max-tokens 128] [--json out.json]
"""
import argparse
import asyncio
import json
import os
import statistics
import sys
import threading
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="mistral-7b")
    ap.add_argument("--recipe", default="Q4_K_M")
    ap.add_argument("--streams", type=int, default=8)
    ap.add_argument("--prompt", type=int, default=3072)
    ap.add_argument("--shared", type=int, default=2048)
    ap.add_argument("--max-tokens", type=int, default=128)
    ap.add_argument("--temperature", type=float, default=0.7)
    ap.add_argument("--ctx", type=int, default=4096)
    ap.add_argument("--tp", type=int, default=1, help="tensor-parallel ranks (#tp=N model spec; ranks share the GPU "
                    "when the box has fewer GPUs)")
    ap.add_argument("--json", default="")
    args = ap.parse_args()

    import numpy as np

    from aios_amd.runtime.model_manager import ModelManager
    from aios_amd.runtime.scheduler import GenRequest

    mgr = ModelManager(max_batch=args.streams, max_slots=2 * args.streams)
    spec = f"synthetic:{args.model}:{args.recipe}" + (f"#tp={args.tp}" if args.tp > 1 else "")
    t0 = time.time()
    m = asyncio.run(mgr.load_model("bench", spec, context_length=args.ctx))
    if m.status != "ready":
        raise SystemExit(f"load failed: {m.error}")
    load_s = time.time() - t0
    V = m.tokenizer.vocab_size
    rng = np.random.default_rng(0)
    prefix = [m.tokenizer.bos_id] + [int(t) for t in rng.integers(100, V - 100, args.shared - 1)]

    def prompt(i):
        own = [int(t) for t in np.random.default_rng(100 + i).integers(100, V - 100, args.prompt - args.shared)]
        return prefix + own

    def run_round(n, json_mode=True):
        done = [threading.Event() for _ in range(n)]
        res = [None] * n
        for i in range(n):
            def cb(r, i=i):
                res[i] = r
                done[i].set()
            m.scheduler.submit(GenRequest(prompt_ids=prompt(i), max_tokens=args.max_tokens,
                                          temperature=args.temperature, top_k=40, top_p=0.95, json_mode=json_mode,
                                          seed=i + 1, on_done=cb))
        t = time.time()
        for e in done:
            if not e.wait(600):
                raise SystemExit("serving bench timed out")
        return res, time.time() - t

    run_round(2)  # warm-up: graphs captured, kernels loaded
    sched = m.scheduler
    st0 = dict(sched.stats)
    tm0 = dict(sched.timing)
    sched.step_log.clear()
    res, wall = run_round(args.streams)
    st1 = dict(sched.stats)
    tm1 = dict(sched.timing)
    log = list(sched.step_log)
    # steady-state ITL: gaps between consecutive full-batch decode steps with no prefill chunk
    # in between (admission-time gaps are in TTFT / itl_p50)
    gaps = sorted((b[0] - a[0]) * 1e3 for a, b in zip(log, log[1:]) if a[1] > 0 and b[1] > 0)
    steps_in_round = st1["steps"] - st0["steps"]
    errs = [r.error for r in res if r.finish_reason == "error"]
    if errs:
        raise SystemExit(f"requests failed: {errs[:2]}")
    ttft = sorted(r.ttft_ms for r in res)
    itl = sorted((r.latency_ms - r.ttft_ms) / (r.completion_tokens - 1) for r in res if r.completion_tokens > 1)
    toks = sum(r.completion_tokens for r in res)

    # the ITL floor: bare decode steps of the same engine at the same batch (graph replay)
    eng = m.engine
    B = args.streams
    slots = list(range(B))
    eng.decode_loop_prepare(slots, [5] * B, [args.prompt] * B)
    eng.decode_loop_run(B, 4, True)
    eng.synchronize()
    t = time.time()
    eng.decode_loop_run(B, 32, True)
    eng.synchronize()
    step_ms = (time.time() - t) / 32 * 1e3
    # the scheduler's engine call at the same batch: host upload + graph launch + token readback
    toks_ = [5] * B
    pos_ = [args.prompt + 40] * B
    mask = m.grammar.mask(m.grammar.initial()) * B
    for label, mk in (("engine_decode_call_ms", b""), ("engine_decode_call_masked_ms", mask)):
        eng.decode(slots, toks_, pos_, [0.7] * B, [40] * B, 1, mk, [0.95] * B)
        t = time.time()
        for i in range(16):
            eng.decode(slots, toks_, [p + i for p in pos_], [0.7] * B, [40] * B, 1, mk, [0.95] * B)
        globals()[label] = (time.time() - t) / 16 * 1e3

    out = {
        "bench": "serving: concurrent JSON-mode streams sharing a prompt prefix",
        "model": f"{args.model} {args.recipe} (random-init weights, synthetic prompts)",
        "tp": args.tp, "streams": args.streams, "prompt_tokens": args.prompt, "shared_prefix_tokens": args.shared,
        "max_tokens": args.max_tokens, "temperature": args.temperature, "top_k": 40, "top_p": 0.95,
        "json_mode": True,
        "ttft_p50_ms": round(ttft[len(ttft) // 2], 2), "ttft_p90_ms": round(ttft[min(len(ttft) - 1, int(len(ttft) * 0.9))], 2),
        "itl_p50_ms": round(itl[len(itl) // 2], 3) if itl else None,
        "steady_itl_p50_ms": round(gaps[len(gaps) // 2], 3) if gaps else None,
        "steady_itl_over_step": round(gaps[len(gaps) // 2] / step_ms, 3) if gaps else None,
        "host_breakdown_s": {k: round(tm1[k] - tm0[k], 4) for k in tm1},
        "decode_step_ms_same_batch": round(step_ms, 3),
        "engine_decode_call_ms": round(globals()["engine_decode_call_ms"], 3),
        "engine_decode_call_masked_ms": round(globals()["engine_decode_call_masked_ms"], 3),
        "scheduler_engine_ms_per_step": round((tm1["engine_decode_s"] - tm0["engine_decode_s"]) * 1e3 /
                                              max(1, steps_in_round), 3),
        "decode_steps": steps_in_round,
        "itl_over_step": round(itl[len(itl) // 2] / step_ms, 3) if itl else None,
        "aggregate_tok_s": round(toks / wall, 1), "completion_tokens": toks, "wall_s": round(wall, 3),
        "prefill_tokens": st1["prefill_tokens"] - st0["prefill_tokens"],
        "prefix_reused_tokens": st1["cached_tokens"] - st0["cached_tokens"],
        "finish_reasons": sorted({r.finish_reason for r in res}),
        "load_s": round(load_s, 2),
    }
    print(json.dumps(out), flush=True)
    if args.json:
        with open(args.json, "a") as f:
            f.write(json.dumps(out) + "\n")
    asyncio.run(mgr.unload_model("bench"))


if __name__ == "__main__":
    main()
