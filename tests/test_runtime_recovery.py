"""Runtime robustness on CPU: the CPU engine backend (BASELINE config #1 plumbing), fault
injection, engine-failure -> error -> bounded auto-reload, decode-stall watchdog and metrics.
Reference semantics: runtime/src/model_manager.rs:393-447 (health -> Error, no restart); the
reload, the stall watchdog and the fault hooks are additions."""
import asyncio
import time

import numpy as np
import pytest

from aios_amd.models.config import get_preset
from aios_amd.models.reference import ReferenceModel
from aios_amd.models.synthetic import write_synthetic_gguf
from aios_amd.runtime import faults
from aios_amd.runtime.cpu_engine import CpuEngine


@pytest.fixture(scope="module")
def small_gguf(tmp_path_factory):
    p = tmp_path_factory.mktemp("cpu") / "small_q4_0.gguf"
    write_synthetic_gguf(str(p), get_preset("test-small"), "Q4_0", seed=5)
    return str(p)


def test_cpu_engine_greedy_matches_reference(small_gguf):
    eng = CpuEngine.from_gguf(small_gguf, max_ctx=128, max_slots=2, max_batch=2)
    ref = ReferenceModel.from_gguf(small_gguf)
    prompt = [1, 17, 29, 31, 5]
    want = ref.greedy(prompt, 8)
    tok = int(np.argmax(eng.prefill(0, prompt, 0, True)))
    got, pos = [tok], len(prompt)
    for _ in range(7):
        tok = eng.decode([0], [tok], [pos], [0.0], [0], 0, b"")[0]
        pos += 1
        got.append(tok)
    assert got == want
    # prefix reuse: re-prefill from position 3 on the same slot gives the same first token
    assert int(np.argmax(eng.prefill(0, prompt[3:], 3, True))) == want[0]
    # batched decode of two slots equals per-slot decode
    eng.prefill(1, prompt, 0, True)
    two = eng.decode([0, 1], [want[0], want[0]], [len(prompt)] * 2, [0.0, 0.0], [0, 0], 0, b"")
    assert two[0] == two[1] == want[1]


def test_fault_spec_parsing_and_triggers():
    s = faults.FaultSpec("decode:after=2,prefill:once=1")
    s.check("decode"); s.check("decode")
    with pytest.raises(faults.InjectedFault):
        s.check("decode")
    s.check("prefill")
    with pytest.raises(faults.InjectedFault):
        s.check("prefill")
    s.check("prefill")  # once: only the 2nd call
    s.check("load")     # no rule
    with pytest.raises(ValueError):
        faults.FaultSpec("gpu:explode")
    t0 = time.time()
    faults.FaultSpec("decode:stall=0.05").check("decode")
    assert time.time() - t0 >= 0.05


def _run(coro):
    return asyncio.run(coro)


def _infer(m, prompt="hello", max_tokens=6):
    from aios_amd.runtime.scheduler import GenRequest

    done = {}
    ev = __import__("threading").Event()

    def on_done(res):
        done["r"] = res
        ev.set()

    ids = m.tokenizer.encode(prompt, add_bos=True)
    m.scheduler.submit(GenRequest(prompt_ids=ids, max_tokens=max_tokens, temperature=0.0, on_done=on_done))
    assert ev.wait(60)
    return done["r"]


def test_manager_cpu_backend_serves(small_gguf, monkeypatch):
    from aios_amd.runtime.model_manager import ModelManager

    monkeypatch.delenv("AIOS_FAULT_INJECT", raising=False)
    mgr = ModelManager(max_batch=2, max_slots=2)
    m = _run(mgr.load_model("tiny", small_gguf + "#cpu", 256))
    assert m.status == "ready" and m.backend == "cpu", m.error
    r = _infer(m)
    assert r.finish_reason in ("length", "stop") and r.completion_tokens > 0
    det = mgr.health()["model:tiny"]
    assert "backend=cpu" in det and "ttft_p50_ms=" in det and "tok_s=" in det
    assert mgr.metrics()["runtime.models_ready"] == 1.0
    _run(mgr.unload_model("tiny"))


def test_injected_decode_fault_marks_error_and_autorecovers(small_gguf, monkeypatch):
    from aios_amd.runtime.model_manager import ModelManager

    monkeypatch.setenv("AIOS_FAULT_INJECT", "decode:after=2")
    mgr = ModelManager(max_batch=2, max_slots=2)
    m = _run(mgr.load_model("tiny", small_gguf + "#cpu", 256))
    assert m.status == "ready"
    r = _infer(m, max_tokens=10)
    assert r.finish_reason == "error" and "injected decode fault" in r.error
    monkeypatch.delenv("AIOS_FAULT_INJECT")  # the reload gets a healthy engine
    recovered = _run(mgr.supervise(stall_timeout_s=30))
    assert recovered == ["tiny"]
    m2 = mgr.models["tiny"]
    assert m2.status == "ready" and m2.port == m.port and len(m2.restarts) == 1
    assert _infer(m2).finish_reason in ("length", "stop")
    _run(mgr.unload_model("tiny"))


def test_restart_budget_and_no_autorecover(small_gguf, monkeypatch):
    from aios_amd.runtime.model_manager import ModelManager

    monkeypatch.setenv("AIOS_FAULT_INJECT", "load:always")
    mgr = ModelManager(max_batch=1, max_slots=1)
    m = _run(mgr.load_model("bad", small_gguf + "#cpu", 128))
    assert m.status == "error" and "injected load fault" in m.error
    assert _run(mgr.supervise(auto_recover=False)) == []
    for _ in range(5):
        _run(mgr.supervise(max_restarts=2))
    assert mgr.models["bad"].status == "error" and len(mgr.models["bad"].restarts) == 2  # budget exhausted


def test_decode_stall_watchdog_fails_requests(small_gguf, monkeypatch):
    from aios_amd.runtime.model_manager import ModelManager
    from aios_amd.runtime.scheduler import GenRequest

    monkeypatch.setenv("AIOS_FAULT_INJECT", "decode:stall=1.5")
    mgr = ModelManager(max_batch=1, max_slots=1)
    m = _run(mgr.load_model("slow", small_gguf + "#cpu", 128))
    results = []
    ids = m.tokenizer.encode("x", add_bos=True)
    m.scheduler.submit(GenRequest(prompt_ids=ids, max_tokens=50, temperature=0.0, on_done=results.append))
    t_end = time.time() + 20  # admitted, now inside a stalled decode call (polled: a loaded host
    while not m.scheduler.stalled(0.3) and time.time() < t_end:  # may take longer to get there)
        time.sleep(0.02)
    monkeypatch.delenv("AIOS_FAULT_INJECT")
    recovered = _run(mgr.supervise(stall_timeout_s=0.3))
    assert results and results[0].finish_reason == "error" and "stalled" in results[0].error
    assert recovered == ["slow"] and mgr.models["slow"].status == "ready"
    assert mgr.join_abandoned(30) == 0  # the stuck thread drains once its stalled call returns
    _run(mgr.unload_model("slow"))


def test_airuntime_grpc_on_cpu_engine_json_mode(small_gguf, monkeypatch):
    """BASELINE config #1 plumbing: LoadModel of a Q4_0 GGUF on the CPU backend, JSON-mode Infer and
    token StreamInfer over the real gRPC contract (the reference's default CPU deployment)."""
    import json

    from aios_amd.rpc.client import Stub, channel
    from aios_amd.rpc.schema import pb
    from aios_amd.rpc.server import RpcServer
    from aios_amd.runtime.model_manager import ModelManager
    from aios_amd.runtime.service import AIRuntimeService

    monkeypatch.setenv("AIOS_RUNTIME_DEVICE", "cpu")
    monkeypatch.delenv("AIOS_FAULT_INJECT", raising=False)

    async def run():
        svc = AIRuntimeService(ModelManager(max_batch=2, max_slots=2, base_port=18180), http=False)
        srv = RpcServer("127.0.0.1:0", {"aios.runtime.AIRuntime": svc})
        await srv.start()
        ch = channel(f"127.0.0.1:{srv.port}", fresh=True)
        stub = Stub(ch, "aios.runtime.AIRuntime", timeout=120)
        try:
            st = await stub.LoadModel(pb.runtime.LoadModelRequest(model_name="tinyllama-1.1b", model_path=small_gguf,
                                                                  context_length=256))
            assert st.status == "ready", st.status
            r = await stub.Infer(pb.runtime.InferRequest(prompt="plan the task", intelligence_level="operational",
                                                         max_tokens=24))
            assert r.model_used == "tinyllama-1.1b" and r.tokens_used > 0
            if r.text.strip():
                json.loads(r.text) if r.text.strip().endswith(("}", "]")) else None  # grammar-constrained prefix
            chunks = [c async for c in stub.StreamInfer(pb.runtime.InferRequest(prompt="s", max_tokens=4))]
            assert chunks[-1].done
            h = await stub.HealthCheck(pb.common.Empty())
            assert h.healthy and "backend=cpu" in h.details["model:tinyllama-1.1b"]
        finally:
            await ch.close()
            await srv.stop()
            await svc.close()

    asyncio.run(run())


def test_failed_strategic_tier_is_torn_down_and_request_rerouted(small_gguf, monkeypatch):
    """A strategic-tier engine failure mid-request (what a TP rank timeout raises) takes that
    tier out of routing, tears its engine down (abort: TP worker ranks killed) and the same
    Infer is answered by the next ready model of the level."""
    from aios_amd.rpc.schema import pb
    from aios_amd.runtime.model_manager import ModelManager
    from aios_amd.runtime.service import AIRuntimeService

    monkeypatch.setenv("AIOS_RUNTIME_DEVICE", "cpu")
    monkeypatch.setenv("AIOS_FAULT_INJECT", "decode:always")
    monkeypatch.setenv("AIOS_FAULT_MODELS", "llama3-70b")

    class Ctx:
        async def abort(self, code, msg):
            raise AssertionError(f"aborted: {code} {msg}")

    async def run():
        mgr = ModelManager(max_batch=2, max_slots=2, base_port=18190)
        svc = AIRuntimeService(mgr, http=False)
        try:
            big = await mgr.load_model("llama3-70b", small_gguf, 256)
            mid = await mgr.load_model("mistral-7b", small_gguf, 256)
            assert big.status == mid.status == "ready"
            aborted = []
            big.engine.abort = lambda: aborted.append(True)  # the TPEngine teardown hook
            r = await svc.Infer(pb.runtime.InferRequest(prompt="plan the migration", intelligence_level="strategic",
                                                        max_tokens=8), Ctx())
            assert r.model_used == "mistral-7b"
            assert big.status == "error" and aborted == [True]
            assert mgr.select_model_for_level("strategic") == "mistral-7b"
        finally:
            await svc.close()

    asyncio.run(run())
