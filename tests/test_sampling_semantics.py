"""Sampling semantics of the serving path (CPU engine; the GPU engine's device sampler keys its RNG
the same way, tests/test_runtime_gpu.py): every request samples from its own stream keyed by
(seed, position) -- unseeded requests draw a fresh seed as llama-server does, a seeded request
reproduces at any batch row and next to any other requests, and the first token is drawn by the
engine's sampler with the same stream as the decode steps."""
import threading

import pytest

from aios_amd.models.config import get_preset
from aios_amd.models.synthetic import synthetic_vocab, write_synthetic_gguf
from aios_amd.runtime.cpu_engine import CpuEngine
from aios_amd.runtime.scheduler import GenRequest, Scheduler
from aios_amd.runtime.tokenizer import SpmTokenizer


@pytest.fixture(scope="module")
def setup(tmp_path_factory):
    p = tmp_path_factory.mktemp("smp") / "small.gguf"
    write_synthetic_gguf(str(p), get_preset("test-small"), "Q8_0", seed=11)
    t, s, ty = synthetic_vocab(1024)
    return str(p), SpmTokenizer(t, s, ty, 1, 2)


def _run(path, tok, reqs, max_batch=4):
    eng = CpuEngine.from_gguf(path, max_ctx=128, max_slots=4, max_batch=max_batch)
    calls = []
    orig = eng.decode

    def spy(*a):
        calls.append(a)
        return orig(*a)

    eng.decode = spy
    sched = Scheduler(eng, tok, max_batch=max_batch, max_slots=4, max_ctx=128)
    out, evs = {}, []
    try:
        for i, (prompt, seed) in enumerate(reqs):
            ev = threading.Event()
            evs.append(ev)

            def done(r, i=i, ev=ev):
                out[i] = r.token_ids
                ev.set()
            sched.submit(GenRequest(prompt_ids=prompt, max_tokens=12, temperature=1.3, top_k=0, top_p=1.0,
                                    seed=seed, on_done=done))
        for ev in evs:
            assert ev.wait(60)
    finally:
        sched.close()
    return [out[i] for i in range(len(reqs))], calls


def test_unseeded_requests_differ(setup):
    path, tok = setup
    prompt = [1, 40, 41, 42, 43]
    (a, b), calls = _run(path, tok, [(prompt, 0), (prompt, 0)])
    assert a != b
    # every decode call carried one seed per row
    assert all(len(c) >= 9 and len(c[8]) == len(c[0]) for c in calls)


def test_seeded_request_reproduces_at_any_row(setup):
    path, tok = setup
    target = [1, 70, 71, 72]
    others = [[1, 5, 6, 7, 8], [1, 300, 301]]
    (solo,), _ = _run(path, tok, [(target, 1234)])
    (x0, t_row1, x2), _ = _run(path, tok, [(others[0], 7), (target, 1234), (others[1], 9)])
    (t_row0, y1), _ = _run(path, tok, [(target, 1234), (others[1], 0)])
    assert solo == t_row1 == t_row0


def test_first_token_from_engine_sampler(setup):
    path, tok = setup
    eng = CpuEngine.from_gguf(path, max_ctx=128, max_slots=2, max_batch=2)
    eng.prefill(0, [1, 40, 41], 0, True)
    a = eng.sample_first(2, 1.3, 0, 1.0, 99)
    b = eng.sample_first(2, 1.3, 0, 1.0, 99)
    assert a == b
    draws = {eng.sample_first(2, 1.3, 0, 1.0, s) for s in range(1, 40)}
    assert len(draws) > 1
