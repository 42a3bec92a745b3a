"""CPU tests of the AI runtime: tokenizer, chat templates, JSON grammar, scheduler, gRPC + HTTP.

The scheduler and services run against `FakeEngine` (same Python surface as the native Engine:
prefill/decode with per-row masks) so the control flow -- batching, prefix-KV reuse, JSON mode,
streaming, routing errors -- is pinned without a GPU.  GPU end-to-end runs of the same paths on
the native engine live in test_runtime_gpu.py.
"""
import asyncio
import json

import grpc
import numpy as np
import pytest

from aios_amd.models.config import get_preset
from aios_amd.models.synthetic import synthetic_vocab
from aios_amd.runtime import chat_template, native
from aios_amd.runtime.sampler import all_allowed, mask_to_bool, sample
from aios_amd.runtime.tokenizer import SpmTokenizer

E = native.load()
needs_native = pytest.mark.skipif(E is None, reason="native extension not built")


@pytest.fixture(scope="module")
def tok():
    t, s, ty = synthetic_vocab(1024)
    return SpmTokenizer(t, s, ty, 1, 2)


# ---------------------------------------------------------------------------- tokenizer / template
def test_tokenizer_roundtrip(tok):
    for text in ["hello world", '{"goal": "list files", "n": 3}', "tab\tand\nnewline", "ünïcødé ✓ 日本"]:
        ids = tok.encode(text, add_bos=False)
        assert tok.decode(ids) == text
    ids = tok.encode("hi", add_bos=True)
    assert ids[0] == tok.bos_id


def test_chat_templates_render(tok):
    msgs = chat_template.build_messages("do X", "you are aiOS")
    assert msgs[0]["role"] == "system" and msgs[1]["content"] == "do X"
    z = chat_template.for_model("zephyr", tok).render(msgs)
    assert "<|system|>" in z and z.rstrip().endswith("<|assistant|>")
    m = chat_template.for_model("mistral", tok).render(msgs)
    assert "[INST]" in m and "you are aiOS" in m
    l3 = chat_template.for_model("llama3", tok).render(msgs)
    assert "<|start_header_id|>assistant<|end_header_id|>" in l3
    c = chat_template.for_model("chatml", tok).render(msgs)
    assert c.endswith("<|im_start|>assistant\n")


# ---------------------------------------------------------------------------- sampler
def test_host_sampler():
    logits = np.array([0.0, 5.0, 1.0, 4.0], np.float32)
    assert sample(logits) == 1
    mask = bytes([0b1101])  # tokens 0,2,3 allowed
    assert sample(logits, mask=mask) == 3
    assert list(mask_to_bool(all_allowed(4), 4)) == [True] * 4
    rng = np.random.default_rng(0)
    draws = [sample(logits, 1.0, top_k=2, rng=rng) for _ in range(400)]
    assert set(draws) <= {1, 3}
    frac = draws.count(1) / len(draws)
    assert abs(frac - 1 / (1 + np.exp(-1))) < 0.08


# ---------------------------------------------------------------------------- grammar
@needs_native
def test_json_grammar_accepts_and_masks(tok):
    g = E.JsonGrammar(tok.all_token_bytes(), tok.eos_id)
    st = g.initial()
    for t in tok.encode('{"a": [1, 2.5e3, "x\\n", true, null], "b": {}}', add_bos=False):
        assert g.accept_token(st, t)
    assert g.complete(st)
    # the object is closed: nothing but eos may follow
    allowed = np.flatnonzero(mask_to_bool(g.mask(st), tok.vocab_size))
    assert list(allowed) == [tok.eos_id]
    # the first token of a JSON-mode reply must open an object (require_object)
    st0 = g.initial()
    allowed0 = mask_to_bool(g.mask(st0), tok.vocab_size)
    for t in np.flatnonzero(allowed0):
        assert tok.token_bytes(int(t)).lstrip(b" \t\n\r")[:1] in (b"{", b"")
    bad = g.initial()
    assert not g.accept_bytes(bad, b'{"a" 1}')


@needs_native
def test_json_grammar_rejects_structural_errors(tok):
    g = E.JsonGrammar(tok.all_token_bytes(), tok.eos_id)
    for s in [b'{"a":}', b'{"a":1,}', b'{a:1}', b'{"a":[1,]}', b'{"a":01}', b'[]']:
        assert not g.accept_bytes(g.initial(), s), s
    for s in [b'{}', b'{"k": -0.5E-2}', b'{"u": "\\u00e9"}', b'{"n": [[], {}, [1]]}']:
        st = g.initial()
        assert g.accept_bytes(st, s) and g.complete(st), s


@needs_native
def test_json_grammar_open_mask_keeps_object_open(tok):
    g = E.JsonGrammar(tok.all_token_bytes(), tok.eos_id)
    st = g.initial()
    for t in tok.encode('{"a": 1', add_bos=False):
        assert g.accept_token(st, t)
    full = mask_to_bool(g.mask(st), tok.vocab_size)
    opn = mask_to_bool(g.mask_open(st), tok.vocab_size)
    assert not (opn & ~full).any()                   # a subset of the grammar's mask
    closing = [t for t in np.flatnonzero(full) if g.accept_token(s2 := st.copy(), int(t)) and g.complete(s2)]
    assert closing                                   # '}' (and '}'-ending tokens) close the object here
    assert not opn[closing].any() and opn.sum() > 0  # ... but not under the open mask
    # nothing but a closing token left: the open mask falls back to the full one
    done = g.initial()
    assert g.accept_bytes(done, b'{}') and g.complete(done)
    assert g.mask_open(done) == g.mask(done)


# ---------------------------------------------------------------------------- fake engine
class FakeEngine:
    """Deterministic stand-in for the native Engine: the next token is a function of the last one,
    or the next byte-compatible token of a scripted JSON answer when a mask is in force."""

    def __init__(self, tokenizer, script='{"ok": true}'):
        self.tok = tokenizer
        self.V = tokenizer.vocab_size
        self.script = tokenizer.encode(script, add_bos=False)
        self.prefills = []
        self.batches = []
        self.progress = {}
        self.weight_bytes = 1 << 20
        self.kv_bytes = 1 << 20

    def _logits(self, last):
        l = np.zeros(self.V, np.float32)
        l[(last * 7 + 3) % self.V] = 10.0
        l[self.tok.eos_id] = -10.0
        return l

    def prefill(self, slot, ids, start, want_logits=True):
        self.prefills.append((slot, len(ids), start))
        self.progress[slot] = 1
        l = self._logits(ids[-1] if ids else 0)
        l[self.script[0]] = 5.0   # wins only when a grammar mask removes the free-running token
        return l

    def decode(self, slots, toks, pos, temps, topk, seed, mask, top_p=None, seeds=None):
        self.batches.append(len(slots))
        out = []
        row = (self.V + 7) // 8
        for b, (slot, t) in enumerate(zip(slots, toks)):
            if mask:
                allowed = mask_to_bool(mask[b * row:(b + 1) * row], self.V)
                k = self.progress.get(slot, 0)
                nxt = self.script[k] if k < len(self.script) else self.tok.eos_id
                self.progress[slot] = k + 1
                out.append(nxt if allowed[nxt] else int(np.flatnonzero(allowed)[0]))
            else:
                out.append(int(np.argmax(self._logits(t))))
        return out


class PipeFakeEngine(FakeEngine):
    """FakeEngine with the pipelined decode surface: decode_submit without tokens takes the ones the
    last sampler left 'on the device'; every call is logged, so the test sees the overlap order."""

    def __init__(self, tokenizer, script='{"ok": true}'):
        super().__init__(tokenizer, script)
        self.dev_tokens = {}
        self.log = []
        self._sub = None
        self._out = None

    def decode_submit(self, slots, toks, pos, temps, topk, seed, top_p, seeds):
        self.log.append(("submit", tuple(slots), bool(toks), tuple(pos)))
        toks = list(toks) if toks else [self.dev_tokens[s] for s in slots]
        self._sub = (list(slots), toks, list(pos))

    def decode_sample(self, mask=b""):
        slots, toks, pos = self._sub
        self.log.append(("sample", tuple(slots)))
        self._out = FakeEngine.decode(self, slots, toks, pos, [], [], 0, mask)
        for s_, t in zip(slots, self._out):
            self.dev_tokens[s_] = t

    def decode_collect(self):
        self.log.append(("collect",))
        return list(self._out)


@needs_native
@pytest.mark.parametrize("n_req", [1, 3])
def test_scheduler_pipelined_decode_matches_sync(tok, n_req, monkeypatch):
    """The pipelined decode (forward of step t+1 queued before step t's token reaches the host) gives
    the same tokens, texts and finish reasons as the synchronous path, for JSON-mode and free text,
    with rows finishing at different steps; the speculative forward is issued before the collect."""
    import threading

    from aios_amd.runtime.scheduler import GenRequest, Scheduler

    res = {}
    for pipe in ("0", "1"):
        monkeypatch.setenv("AIOS_DECODE_PIPELINE", pipe)
        eng = PipeFakeEngine(tok)
        g = E.JsonGrammar(tok.all_token_bytes(), tok.eos_id)
        sched = Scheduler(eng, tok, max_batch=4, max_slots=4, max_ctx=256, grammar=g)
        assert sched.pipeline == (pipe == "1")
        done, evs = {}, [threading.Event() for _ in range(n_req)]
        try:
            for i in range(n_req):
                sched.submit(GenRequest(prompt_ids=tok.encode(f"req {i}"), max_tokens=[12, 7, 30][i],
                                        json_mode=i != 1, min_tokens=[0, 0, 20][i],
                                        on_done=lambda r, i=i: (done.__setitem__(i, r), evs[i].set())))
            for e in evs:
                assert e.wait(10)
        finally:
            sched.close()
        res[pipe] = ([(done[i].text, done[i].finish_reason, done[i].completion_tokens) for i in range(n_req)], eng)
    assert res["0"][0] == res["1"][0]
    log = res["1"][1].log
    # overlap: a device-token submit (the next step's forward) is queued before the previous collect
    spec = [k for k, e in enumerate(log) if e[0] == "submit" and not e[2]]
    assert spec and all(log[k + 1][0] == "collect" for k in spec)


@needs_native
def test_scheduler_batches_streams_and_reuses_prefix(tok):
    from aios_amd.runtime.scheduler import GenRequest, Scheduler

    eng = FakeEngine(tok)
    g = E.JsonGrammar(tok.all_token_bytes(), tok.eos_id)
    sched = Scheduler(eng, tok, max_batch=4, max_slots=4, max_ctx=256, grammar=g)
    try:
        import threading

        done = {}
        evs = [threading.Event() for _ in range(4)]
        deltas = {i: [] for i in range(4)}
        prompt = tok.encode("shared system prompt with tool catalogue " * 3)

        def mk(i, json_mode=False, max_tokens=6):
            def on_done(r):
                done[i] = r
                evs[i].set()
            return GenRequest(prompt_ids=prompt + [100 + i], max_tokens=max_tokens, json_mode=json_mode,
                              on_delta=deltas[i].append, on_done=on_done)

        for i in range(3):
            sched.submit(mk(i))
        for e in evs[:3]:
            assert e.wait(10)
        for i in range(3):
            r = done[i]
            assert r.completion_tokens == 6 and r.finish_reason == "length"
            assert "".join(deltas[i]) == r.text
        assert max(eng.batches) >= 2            # continuous batching shared decode steps
        # a 4th request sharing the prompt prefix reuses a finished slot's KV
        sched.submit(mk(3, json_mode=True, max_tokens=64))
        assert evs[3].wait(10)
        r = done[3]
        assert r.cached_prompt_tokens == len(prompt)
        assert eng.prefills[-1][2] == len(prompt) and eng.prefills[-1][1] == 1
        assert r.finish_reason == "grammar"
        assert json.loads(r.text) == {"ok": True}
    finally:
        sched.close()


@needs_native
def test_scheduler_min_tokens_pins_json_length(tok):
    """min_tokens: the grammar may not close the object before it (bench plans of a fixed length)."""
    import threading

    from aios_amd.runtime.scheduler import GenRequest, Scheduler

    eng = FakeEngine(tok)  # scripted '{"ok": true}' closes after a few tokens when allowed
    g = E.JsonGrammar(tok.all_token_bytes(), tok.eos_id)
    sched = Scheduler(eng, tok, max_batch=2, max_slots=2, max_ctx=256, grammar=g)
    try:
        res, ev = {}, threading.Event()
        for n in (0, 24):
            ev.clear()
            sched.submit(GenRequest(prompt_ids=tok.encode("plan"), max_tokens=24, min_tokens=n, json_mode=True,
                                    on_done=lambda r, n=n: (res.__setitem__(n, r), ev.set())))
            assert ev.wait(10)
        assert res[0].finish_reason == "grammar" and res[0].completion_tokens < 24
        assert res[24].finish_reason == "length" and res[24].completion_tokens == 24
    finally:
        sched.close()


# ---------------------------------------------------------------------------- services
def _fake_manager(tok):
    from aios_amd.runtime import model_manager as mm
    from aios_amd.runtime.scheduler import Scheduler

    class Mgr(mm.ModelManager):
        def _load_blocking(self, m, context_length):
            if "missing" in m.path:
                raise FileNotFoundError(m.path)
            m.engine = FakeEngine(tok)
            m.tokenizer = tok
            m.template = chat_template.for_model("zephyr", tok)
            m.grammar = E.JsonGrammar(tok.all_token_bytes(), tok.eos_id)
            m.context_length = context_length or 512
            m.scheduler = Scheduler(m.engine, tok, self.max_batch, self.max_slots, m.context_length, m.grammar, m.name)

    return Mgr(base_port=18080)


@needs_native
def test_runtime_grpc_service_end_to_end(tok):
    from aios_amd.rpc.client import Stub, channel
    from aios_amd.rpc.schema import pb
    from aios_amd.rpc.server import RpcServer
    from aios_amd.runtime.service import AIRuntimeService

    async def run():
        svc = AIRuntimeService(_fake_manager(tok), http=False)
        srv = RpcServer("127.0.0.1:0", {"aios.runtime.AIRuntime": svc})
        await srv.start()
        ch = channel(f"127.0.0.1:{srv.port}", fresh=True)
        stub = Stub(ch, "aios.runtime.AIRuntime")
        try:
            # no model loaded -> UNAVAILABLE (grpc_service.rs)
            with pytest.raises(grpc.aio.AioRpcError) as ei:
                await stub.Infer(pb.runtime.InferRequest(prompt="x"))
            assert ei.value.code() == grpc.StatusCode.UNAVAILABLE
            st = await stub.LoadModel(pb.runtime.LoadModelRequest(model_name="tinyllama-1.1b", model_path="fake.gguf"))
            assert st.status == "ready" and st.port == 18080
            bad = await stub.LoadModel(pb.runtime.LoadModelRequest(model_name="x", model_path="missing.gguf"))
            assert bad.status.startswith("error:")
            lst = await stub.ListModels(pb.common.Empty())
            assert {m.model_name for m in lst.models} == {"tinyllama-1.1b", "x"}
            r = await stub.Infer(pb.runtime.InferRequest(prompt="plan", intelligence_level="operational", max_tokens=0))
            assert json.loads(r.text) == {"ok": True}          # Infer always runs JSON mode
            assert r.model_used == "tinyllama-1.1b" and r.tokens_used > 0
            with pytest.raises(grpc.aio.AioRpcError) as ei:
                await stub.Infer(pb.runtime.InferRequest(prompt="x", intelligence_level="reactive"))
            assert ei.value.code() == grpc.StatusCode.INVALID_ARGUMENT
            with pytest.raises(grpc.aio.AioRpcError) as ei:
                await stub.Infer(pb.runtime.InferRequest(prompt="x", intelligence_level="strategic"))
            assert ei.value.code() == grpc.StatusCode.FAILED_PRECONDITION
            chunks = [c async for c in stub.StreamInfer(pb.runtime.InferRequest(prompt="s", max_tokens=5,
                                                                                 temperature=-1))]
            assert chunks[-1].done and len(chunks) >= 3
            assert all(not c.done for c in chunks[:-1])
            h = await stub.HealthCheck(pb.common.Empty())
            assert h.healthy and "model:tinyllama-1.1b" in h.details
            u = await stub.UnloadModel(pb.runtime.UnloadModelRequest(model_name="tinyllama-1.1b"))
            assert u.success
        finally:
            await ch.close()
            await srv.stop()
            await svc.close()

    asyncio.run(run())


@needs_native
def test_openai_http_endpoint(tok):
    import aiohttp

    from aios_amd.runtime.service import AIRuntimeService

    async def run():
        mgr = _fake_manager(tok)
        svc = AIRuntimeService(mgr, http=True)
        m = await mgr.load_model("tiny", "fake.gguf", port=18931)
        await svc.start_http(m)
        try:
            async with aiohttp.ClientSession() as s:
                async with s.get("http://127.0.0.1:18931/health") as r:
                    assert (await r.json())["status"] == "ok"
                body = {"messages": [{"role": "user", "content": "hi"}], "max_tokens": 64,
                        "response_format": {"type": "json_object"}}
                async with s.post("http://127.0.0.1:18931/v1/chat/completions", json=body) as r:
                    js = await r.json()
                assert json.loads(js["choices"][0]["message"]["content"]) == {"ok": True}
                assert js["usage"]["completion_tokens"] > 0
                body = {"messages": [{"role": "user", "content": "hi"}], "max_tokens": 4, "stream": True}
                async with s.post("http://127.0.0.1:18931/v1/chat/completions", json=body) as r:
                    raw = (await r.read()).decode()
                events = [l[6:] for l in raw.split("\n") if l.startswith("data: ")]
                assert events[-1] == "[DONE]"
                text = "".join(json.loads(e)["choices"][0]["delta"].get("content", "") for e in events[:-1])
                assert len(text) > 0
        finally:
            await svc.close()

    asyncio.run(run())


def test_level_routing_table():
    from aios_amd.runtime.model_manager import LEVEL_CANDIDATES, ManagedModel, ModelManager, RoutingError

    mgr = ModelManager()
    mgr.models["mistral-7b-instruct"] = ManagedModel("mistral-7b-instruct", "p", status="ready", port=8080)
    mgr.models["tinyllama-1.1b-chat"] = ManagedModel("tinyllama-1.1b-chat", "p", status="ready", port=8081)
    assert mgr.resolve("", "operational").name == "tinyllama-1.1b-chat"
    assert mgr.resolve("", "tactical").name == "mistral-7b-instruct"
    assert mgr.resolve("", "strategic").name == "mistral-7b-instruct"   # mistral is a strategic fallback
    with pytest.raises(RoutingError):
        mgr.resolve("", "reactive")
    assert mgr.resolve("tinyllama-1.1b-chat", "").request_count >= 1
    assert LEVEL_CANDIDATES["strategic"][0] == "llama3-70b"
    assert mgr.allocate_port() == 8082


def test_tier_context_follows_reference_size_heuristic(tmp_path):
    """reference runtime/src/main.rs:86-98: > 8 GB -> 8192, 2-8 GB -> 4096, else 2048; synthetic
    tiers (the TP strategic tier included) use their preset's estimated Q4_K_M size"""
    from aios_amd.runtime.model_manager import tier_context

    assert tier_context(get_preset("llama3-70b")) == 8192
    assert tier_context(get_preset("qwen3-14b")) == 8192
    assert tier_context(get_preset("mistral-7b")) == 4096
    assert tier_context(get_preset("tinyllama-1.1b")) == 2048
    f = tmp_path / "big.gguf"
    with open(f, "wb") as fh:
        fh.truncate(9 * 10**9)  # sparse: only the size is read
    assert tier_context(get_preset("mistral-7b").__class__(**{**get_preset("mistral-7b").__dict__}), str(f)) == 8192
