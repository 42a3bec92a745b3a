"""Serving-path scheduling on CPU with a recording fake engine: prefix sharing from a slot that
is still decoding (paged-KV copy_slot, csrc/engine.hip) and chunked prefill interleaved with the
batched decode steps of running streams (the autonomy loop resends its ~2-4k-token
tool catalogue every round with up to 3 concurrent loops, `agent-core/src/autonomy.rs:988-1036`)."""
import threading
import time

import numpy as np

from aios_amd.runtime.scheduler import GenRequest, Scheduler


class Tok:
    vocab_size = 1000
    eos_id = 2
    vocab = {}

    def decode(self, ids):
        return " ".join(str(i) for i in ids)

    def encode(self, text):
        return [1] + [int(t) for t in text.split()]


class RecEngine:
    def __init__(self, step_s=0.002):
        self.log = []
        self.step_s = step_s
        self.lock = threading.Lock()

    def _logits(self, last):
        l = np.zeros(1000, np.float32)
        l[(int(last) * 7 + 3) % 997 + 3] = 10.0
        return l

    def prefill(self, slot, ids, start, want_logits=True):
        with self.lock:
            self.log.append(("prefill", slot, len(ids), start))
        return self._logits(ids[-1]) if want_logits else []

    def decode(self, slots, toks, pos, temps, topk, seed, mask=b"", top_p=None, seeds=None):
        time.sleep(self.step_s)
        with self.lock:
            self.log.append(("decode", len(slots)))
        return [int(np.argmax(self._logits(t))) for t in toks]

    def copy_slot(self, src, dst, n):
        with self.lock:
            self.log.append(("copy", src, dst, n))


def _run(sched, req):
    ev = threading.Event()
    box = {}

    def done(r):
        box["r"] = r
        ev.set()

    req.on_done = done
    sched.submit(req)
    return ev, box


def test_prefix_shared_from_a_decoding_slot_and_chunked_prefill(monkeypatch):
    monkeypatch.setenv("AIOS_PREFILL_CHUNK", "256")
    eng = RecEngine()
    sched = Scheduler(eng, Tok(), max_batch=4, max_slots=4, max_ctx=4096)
    try:
        catalogue = [1] + [int(t) for t in np.random.default_rng(0).integers(3, 900, 899)]  # 900-token prefix
        first = threading.Event()
        a = GenRequest(prompt_ids=catalogue + [5, 6, 7], max_tokens=200, on_delta=lambda d: first.set())
        ev_a, box_a = _run(sched, a)
        assert first.wait(10)
        # a second reasoning loop with the same tool catalogue and its own 700-token task
        b = GenRequest(prompt_ids=catalogue + [int(t) for t in np.random.default_rng(1).integers(3, 900, 700)],
                       max_tokens=8)
        ev_b, box_b = _run(sched, b)
        assert ev_b.wait(20) and ev_a.wait(20)
    finally:
        sched.close()
    rb = box_b["r"]
    assert rb.finish_reason == "length" and rb.cached_prompt_tokens == 900
    copies = [e for e in eng.log if e[0] == "copy"]
    assert len(copies) == 1 and copies[0][3] == 900  # shared from A's slot, no recompute
    src, dst = copies[0][1], copies[0][2]
    assert src != dst
    b_prefills = [e for e in eng.log if e[0] == "prefill" and e[1] == dst]
    # 700 suffix tokens in 256-token chunks, starting at the shared prefix
    assert [e[2] for e in b_prefills] == [256, 256, 188] and b_prefills[0][3] == 900
    # A kept decoding between B's chunks (ITL bounded by one chunk, not the whole prompt)
    i0 = eng.log.index(b_prefills[0])
    i2 = eng.log.index(b_prefills[-1])
    assert any(e[0] == "decode" for e in eng.log[i0:i2])
    assert box_a["r"].finish_reason == "length"


def test_idle_scheduler_prefills_whole_prompt_at_once(monkeypatch):
    monkeypatch.setenv("AIOS_PREFILL_CHUNK", "128")
    eng = RecEngine(step_s=0.0)
    sched = Scheduler(eng, Tok(), max_batch=2, max_slots=2, max_ctx=4096)
    try:
        ev, box = _run(sched, GenRequest(prompt_ids=[1] + list(range(3, 603)), max_tokens=3))
        assert ev.wait(10)
    finally:
        sched.close()
    assert [e for e in eng.log if e[0] == "prefill"] == [("prefill", 0, 601, 0)]
    assert box["r"].completion_tokens == 3
