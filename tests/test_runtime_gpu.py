"""GPU end-to-end tests of the runtime on the native engine (synthetic random-init models).

* continuous batching returns the same greedy tokens as one-at-a-time generation,
* prefix-KV reuse (partial prefill into a slot with cached tokens) is token-exact,
* JSON mode on a random model still yields grammar-valid output (device-side masks),
* the AIRuntime gRPC service serves Infer/StreamInfer from a ModelManager-loaded model.
"""
import asyncio
import json
import threading

import pytest

pytestmark = pytest.mark.gpu


def _run_all(sched, reqs, timeout=60):
    from aios_amd.runtime.scheduler import GenRequest

    out = [None] * len(reqs)
    evs = [threading.Event() for _ in reqs]
    for i, (ids, kw) in enumerate(reqs):
        def done(r, i=i):
            out[i] = r
            evs[i].set()
        sched.submit(GenRequest(prompt_ids=ids, on_done=done, **kw))
    for e in evs:
        assert e.wait(timeout)
    return out


@pytest.fixture(scope="module")
def model():
    from aios_amd.runtime.model_manager import ModelManager

    mgr = ModelManager(max_batch=8, max_slots=8)
    m = asyncio.run(mgr.load_model("test-small", "synthetic:test-small:Q4_K_M", context_length=512))
    assert m.status == "ready", m.error
    yield m
    asyncio.run(mgr.unload_model("test-small"))


def test_batched_equals_sequential(model):
    tok, sched = model.tokenizer, model.scheduler
    prompts = [tok.encode(p) for p in ["alpha beta gamma", "the quick brown fox", "json { } [ ]", "aiOS goal"]]
    seq = [_run_all(sched, [(p, dict(max_tokens=12))])[0] for p in prompts]
    bat = _run_all(sched, [(p, dict(max_tokens=12)) for p in prompts])
    for a, b in zip(seq, bat):
        assert a.token_ids == b.token_ids


@pytest.mark.parametrize("json_mode", [False, True])
def test_pipelined_decode_matches_sync(model, json_mode):
    """The scheduler's pipelined decode on the native engine (Engine.decode_submit / decode_sample /
    decode_collect: step t+1's forward queued from the device-resident token before step t's token
    reaches the host) against the synchronous decode() path: the same greedy tokens for one and for
    three concurrent requests (rows finishing at different lengths), JSON mode with the masks."""
    tok, sched = model.tokenizer, model.scheduler
    prompts = [tok.encode(p) for p in ["alpha beta gamma", "the quick brown fox jumps", "aiOS goal"]]
    kw = [dict(max_tokens=n, temperature=0.0, json_mode=json_mode) for n in (20, 9, 31)]
    res = {}
    try:
        for pipe in (False, True):
            sched.pipeline = pipe
            one = [_run_all(sched, [(p, k)])[0] for p, k in zip(prompts, kw)]
            many = _run_all(sched, list(zip(prompts, kw)))
            res[pipe] = [(r.token_ids, r.finish_reason) for r in one + many]
    finally:
        sched.pipeline = True
    assert res[False] == res[True]
    assert all(len(t) > 0 for t, _ in res[True])


def test_prefix_reuse_is_exact(model):
    tok, sched = model.tokenizer, model.scheduler
    base = tok.encode("system: you are the aiOS planner. tools: fs.read fs.write net.ping " * 2)
    r1 = _run_all(sched, [(base + tok.encode("goal one", add_bos=False), dict(max_tokens=8))])[0]
    r2 = _run_all(sched, [(base + tok.encode("goal two", add_bos=False), dict(max_tokens=8))])[0]
    assert r2.cached_prompt_tokens >= len(base) - 1
    # fresh engine state for the same prompt: evict by filling every slot with unrelated prompts
    _run_all(sched, [(tok.encode(f"unrelated {i} " * 5), dict(max_tokens=1)) for i in range(8)])
    r2b = _run_all(sched, [(base + tok.encode("goal two", add_bos=False), dict(max_tokens=8))])[0]
    assert r2b.token_ids == r2.token_ids
    assert r1.completion_tokens == 8


def test_json_mode_random_model(model):
    tok, sched, g = model.tokenizer, model.scheduler, model.grammar
    res = _run_all(sched, [(tok.encode(f"reply in json {i}"), dict(max_tokens=96, json_mode=True, temperature=t))
                           for i, t in enumerate([0.0, 0.8, 1.2])])
    for r in res:
        st = g.initial()
        assert g.accept_bytes(st, r.text.encode()), r.text
        if r.finish_reason == "grammar":
            assert isinstance(json.loads(r.text), dict)


def test_runtime_service_grpc(model):
    from aios_amd.rpc.client import Stub, channel
    from aios_amd.rpc.schema import pb
    from aios_amd.rpc.server import RpcServer
    from aios_amd.runtime.model_manager import ModelManager
    from aios_amd.runtime.service import AIRuntimeService

    async def run():
        mgr = ModelManager()
        mgr.models[model.name] = model          # share the loaded model
        svc = AIRuntimeService(mgr, http=False)
        srv = RpcServer("127.0.0.1:0", {"aios.runtime.AIRuntime": svc})
        await srv.start()
        ch = channel(f"127.0.0.1:{srv.port}", fresh=True)
        stub = Stub(ch, "aios.runtime.AIRuntime")
        try:
            r = await stub.Infer(pb.runtime.InferRequest(prompt="plan", max_tokens=48, temperature=-1))
            assert r.model_used == model.name and r.tokens_used > 0 and r.latency_ms >= 0
            chunks = [c async for c in stub.StreamInfer(pb.runtime.InferRequest(prompt="s", max_tokens=16,
                                                                                 temperature=-1))]
            assert chunks[-1].done
        finally:
            await ch.close()
            await srv.stop()

    asyncio.run(run())
