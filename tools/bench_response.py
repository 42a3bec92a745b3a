#!/usr/bin/env python3
"""Whole-response latency over gRPC against the reference's inference targets: a 50-token response from
TinyLlama in < 200 ms and from Mistral-7B (GPU) in < 100 ms (docs/phases/04-AI-RUNTIME.md:332-334,
SURVEY.md §6).

Both tiers (random-init Q4_K_M weights of each architecture) are loaded in one ModelManager and served
by the AIRuntime service on loopback; each request is the reference's unary AIRuntime.Infer (chat
template, JSON mode) routed by intelligence level (operational -> TinyLlama, tactical -> Mistral), timed
client-side from the call to the response: prompt prefill + every decoded token + detokenisation + gRPC.
AIOS_JSON_MIN_TOKENS=max keeps every response at exactly --tokens tokens (random weights would close the
JSON object at arbitrary points); the completion length is checked from tokens_used.

python tools/bench_response.py [--tokens 50] [--reps 10] [--json out.json]"""
import argparse
import asyncio
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TARGET_MS = {"tinyllama-1.1b": 200.0, "mistral-7b": 100.0}
LEVEL = {"tinyllama-1.1b": "operational", "mistral-7b": "tactical"}
PROMPT = ("The disk usage on /var crossed 90 percent twenty minutes ago and the nginx error log is growing "
          "quickly. List the checks to run and the safe cleanup steps, as JSON.")


async def main_async(args):
    os.environ["AIOS_JSON_MIN_TOKENS"] = "max"
    from aios_amd.rpc.client import Stub, channel, close_all
    from aios_amd.rpc.schema import pb
    from aios_amd.rpc.server import RpcServer
    from aios_amd.runtime.chat_template import build_messages
    from aios_amd.runtime.model_manager import ModelManager
    from aios_amd.runtime.service import AIRuntimeService

    mgr = ModelManager(max_batch=4, max_slots=4)
    for name in TARGET_MS:
        m = await mgr.load_model(name, f"synthetic:{name}:{args.recipe}", context_length=2048)
        assert m.status == "ready", m.error
    server = await RpcServer("127.0.0.1:0", {"aios.runtime.AIRuntime": AIRuntimeService(mgr, http=False)}).start()
    stub = Stub(channel(f"127.0.0.1:{server.port}"), "aios.runtime.AIRuntime", timeout=120)
    out = {"metric": f"{args.tokens}-token response latency over gRPC (AIRuntime.Infer, loopback)",
           "tokens": args.tokens, "reps": args.reps, "prompt": PROMPT,
           "data": f"synthetic (random-init {args.recipe} weights of each architecture)", "models": {}}
    try:
        for name, target in TARGET_MS.items():
            req = pb.runtime.InferRequest(prompt=PROMPT, max_tokens=args.tokens, temperature=-1.0,
                                          intelligence_level=LEVEL[name], requesting_agent="bench")
            r = await stub.Infer(req)  # warm-up: graph capture, first prefill
            assert r.model_used == name, (r.model_used, name)
            lat, server_ms, used = [], [], []
            for _ in range(args.reps):
                t = time.perf_counter()
                r = await stub.Infer(req)
                lat.append((time.perf_counter() - t) * 1e3)
                server_ms.append(r.latency_ms)
                used.append(r.tokens_used)
            mm = next(x for x in mgr.list_models() if x.name == name)
            prompt_tokens = len(mm.tokenizer.encode(mm.template.render(build_messages(PROMPT, ""), add_generation_prompt=True)))
            lat.sort()
            out["models"][name] = {
                "intelligence_level": LEVEL[name], "prompt_tokens": prompt_tokens,
                "completion_tokens": sorted({u - prompt_tokens for u in used}),
                "p50_ms": round(statistics.median(lat), 2), "p90_ms": round(lat[int(0.9 * len(lat)) - 1], 2),
                "server_p50_ms": statistics.median(server_ms), "target_ms": target,
                "meets_target": statistics.median(lat) < target}
    finally:
        await server.stop(0)
        await close_all()
        for name in TARGET_MS:
            await mgr.unload_model(name)
    return out


def main():
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--tokens", type=int, default=50)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--recipe", default="Q4_K_M")
    ap.add_argument("--json", default="")
    args = ap.parse_args()
    out = asyncio.run(main_async(args))
    print(json.dumps(out), flush=True)
    if args.json:
        with open(args.json, "w") as f:
            json.dump(out, f, indent=1)
    return 0


if __name__ == "__main__":
    sys.exit(main())
