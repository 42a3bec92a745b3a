#!/usr/bin/env python3
"""Operational tier over gRPC (BASELINE.json config 2): TinyLlama-1.1B with BF16 weights (random
init of that architecture), served by the AIRuntime service on loopback; tokens/s of
AIRuntime.StreamInfer and AIRuntime.Infer with intelligence_level="operational" (routed by the
ModelManager like the reference's runtime, grpc_service.rs:33-177), next to the bare engine's decode
rate that bench.py measures on the same weights.

Random weights mostly run to the --tokens cap, but may sample EOS early; stream rate = (chunks - 1) /
(last chunk - first chunk) (one chunk per decoded token) over however many tokens the request
produced (stream_chunks), TTFT = request -> first chunk.  (The unary Infer is JSON-mode -- grammar-constrained like the reference's -- and with
random weights closes its object after a few tokens, so it is only the routing check here.)

python tools/bench_grpc.py [--tokens 256] [--reps 3] [--recipe BF16]"""
import argparse
import asyncio
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


async def main_async(args):
    from aios_amd.rpc.client import Stub, channel, close_all
    from aios_amd.rpc.schema import pb
    from aios_amd.rpc.server import RpcServer
    from aios_amd.runtime.model_manager import ModelManager
    from aios_amd.runtime.service import AIRuntimeService

    mgr = ModelManager(max_batch=4, max_slots=4)
    t0 = time.time()
    m = await mgr.load_model("tinyllama-1.1b", f"synthetic:tinyllama-1.1b:{args.recipe}", context_length=2048)
    assert m.status == "ready", m.error
    load_s = time.time() - t0
    server = await RpcServer("127.0.0.1:0", {"aios.runtime.AIRuntime": AIRuntimeService(mgr, http=False)}).start()
    stub = Stub(channel(f"127.0.0.1:{server.port}"), "aios.runtime.AIRuntime", timeout=120)
    req = pb.runtime.InferRequest(prompt="Check the status of the nginx service and report any failed units.",
                                  max_tokens=args.tokens, temperature=0.0, intelligence_level="operational",
                                  requesting_agent="bench")
    r = await stub.Infer(req)  # warm-up (graph capture, first prefill)
    assert r.model_used.startswith("tinyllama"), r.model_used
    stream, ttft, chunks = [], [], []
    for _ in range(args.reps):
        t = time.perf_counter()
        first = last = None
        n = 0
        async for ch in stub.StreamInfer(req):
            now = time.perf_counter()
            if ch.done:
                break
            if first is None:
                first = now
            last = now
            n += 1
        ttft.append((first - t) * 1e3)
        stream.append((n - 1) / max(last - first, 1e-9))  # one chunk per decoded token
        chunks.append(n)
    out = {"metric": "operational tier tokens/s over gRPC (TinyLlama-1.1B " + args.recipe + ", loopback)",
           "service_stream_tok_s": round(statistics.median(stream), 1),
           "stream_ttft_ms": round(statistics.median(ttft), 2),
           "max_tokens": args.tokens, "stream_chunks": chunks, "reps": args.reps,
           "intelligence_level": "operational", "model_used": r.model_used, "model_load_s": round(load_s, 1),
           "data": f"synthetic (random-init {args.recipe} weights of the TinyLlama-1.1B architecture)"}
    await server.stop(0)
    await close_all()
    await mgr.unload_model("tinyllama-1.1b")
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tokens", type=int, default=256)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--recipe", default="BF16")
    print(json.dumps(asyncio.run(main_async(ap.parse_args()))), flush=True)


if __name__ == "__main__":
    main()
