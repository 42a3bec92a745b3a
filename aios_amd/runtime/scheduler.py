"""Continuous-batching generation scheduler for one model.

Replaces the per-request HTTP round trip to llama-server (`runtime/src/inference.rs:94-186`)
with an in-process worker per model that owns the native Engine:

* admission: a waiting request takes a free KV slot and inherits the longest cached prefix of
  ANY slot -- free or still decoding: the engine's paged KV shares that prefix's full blocks
  with the new slot (refcounted, no copy; csrc/engine.hip copy_slot) and only the remainder is
  prefilled (the autonomy loop resends the tool catalogue and format rules every round, with up
  to 3 concurrent loops);
* chunked prefill interleaved with decode: while sequences are decoding, a new prompt is
  prefilled AIOS_PREFILL_CHUNK tokens (default 512) per scheduler iteration between batched
  decode steps, so a 3k-token admission does not stall every running stream for its whole
  prefill; with nothing decoding the prompt goes through in one call;
* each iteration runs ONE batched decode step (hipGraph replay) for every decoding sequence, so
  concurrent agents/reasoning loops share each weight pass;
* JSON mode (the reference's `response_format: json_object`) builds the allowed-token mask per
  row with the native JsonGrammar and the device sampler applies it; generation stops as soon as
  the top-level object is complete;
* true token streaming: every step pushes text deltas to the request's callback (the reference
  buffered the whole SSE body, App. A #2).

The worker is a thread: engine calls release the GIL, asyncio callers get results through
thread-safe callbacks.
"""
from __future__ import annotations

import collections
import dataclasses
import logging
import os
import threading
import time
from typing import Callable, Deque, Dict, List, Optional

import numpy as np

from . import sampler as host_sampler

log = logging.getLogger("aios.runtime.scheduler")


def _fresh_seed() -> int:
    return int.from_bytes(os.urandom(8), "little") | 1


@dataclasses.dataclass
class GenRequest:
    prompt_ids: List[int]
    max_tokens: int = 512
    temperature: float = 0.0
    top_k: int = 40
    top_p: float = 0.95
    json_mode: bool = False
    # JSON mode: the grammar may not close the object before this many tokens (bench runs pin the
    # plan length with it: random weights close a JSON object at arbitrary points)
    min_tokens: int = 0
    seed: int = 0
    stop_ids: Optional[List[int]] = None
    on_delta: Optional[Callable[[str], None]] = None
    on_done: Optional[Callable[["GenResult"], None]] = None
    deadline: float = 0.0             # absolute time.time(); 0 = none
    cancelled: bool = False
    submitted_at: float = dataclasses.field(default_factory=time.time)


@dataclasses.dataclass
class GenResult:
    text: str
    token_ids: List[int]
    prompt_tokens: int
    completion_tokens: int
    finish_reason: str                # stop | length | grammar | cancelled | error | deadline
    ttft_ms: float = 0.0
    latency_ms: float = 0.0
    cached_prompt_tokens: int = 0
    error: str = ""


class _Seq:
    __slots__ = ("req", "slot", "pos", "last", "out", "grammar_state", "emitted", "t_first", "cached", "todo",
                 "p_off", "r_off", "seed")

    def __init__(self, req, slot):
        self.req, self.slot = req, slot
        # the request's sampling seed; unseeded requests draw a fresh one (llama-server does the
        # same), so two identical T > 0 requests do not return identical "samples"
        self.seed = int(req.seed) & 0xFFFFFFFFFFFFFFFF if req.seed else _fresh_seed()
        self.pos = 0                 # next position to write (prefill cursor, then decode position)
        self.last = 0
        self.out: List[int] = []
        self.grammar_state = None
        self.emitted = ""
        self.t_first = 0.0
        self.cached = 0
        self.todo: List[int] = []    # prompt tokens still to prefill
        self.p_off = 0               # incremental detokenization window [p_off, r_off) already emitted
        self.r_off = 0


class Scheduler:
    def __init__(self, engine, tokenizer, max_batch: int, max_slots: int, max_ctx: int, grammar=None,
                 name: str = "model"):
        self.engine = engine
        self.tok = tokenizer
        self.max_batch = max_batch
        self.max_ctx = max_ctx
        self.grammar = grammar
        self.name = name
        self.vocab = tokenizer.vocab_size
        self.eos = {tokenizer.eos_id}
        for extra in ("<|eot_id|>", "<|im_end|>", "<|end|>"):
            if extra in tokenizer.vocab:
                self.eos.add(tokenizer.vocab[extra])
        self.slot_cache: Dict[int, List[int]] = {s: [] for s in range(max_slots)}
        self.free_slots = list(range(max_slots))
        self.queue: Deque[GenRequest] = collections.deque()
        self.active: List[_Seq] = []          # decoding
        self.prefilling: List[_Seq] = []      # admitted, prompt not fully prefilled yet
        self.prefill_chunk = int(os.environ.get("AIOS_PREFILL_CHUNK", "512"))
        self._full_mask = None
        # host-side cost breakdown of the decode loop (bench_serving / HealthCheck)
        self.timing = dict(mask_s=0.0, engine_decode_s=0.0, accept_s=0.0, prefill_s=0.0)
        self.step_log: Deque = collections.deque(maxlen=4096)  # (end time, batch) per decode step
        self.share_prefix = hasattr(engine, "copy_slot")
        self.min_shared_prefix = int(os.environ.get("AIOS_MIN_SHARED_PREFIX", "128"))
        self.cv = threading.Condition()
        self.stop_flag = False
        self.stats = dict(requests=0, tokens=0, prefill_tokens=0, cached_tokens=0, steps=0, batch_sum=0, errors=0)
        # health / metrics (ModelManager.supervise and HealthCheck details)
        self.max_slots = max_slots
        self.last_progress = time.time()   # last completed admission or decode step
        self.failed = ""                   # last engine error (a device fault leaves the engine unusable)
        self._ttft = collections.deque(maxlen=256)
        self._step_ms = collections.deque(maxlen=256)
        self._tok_times = collections.deque(maxlen=4096)
        # pipelined decode (Engine.decode_submit / decode_sample / decode_collect): the forward of step
        # t+1 is queued before the host has seen step t's token, so the host's per-token work (grammar
        # mask, accept, detokenize, callbacks) overlaps the device step instead of adding to it
        self.pipeline = hasattr(engine, "decode_submit") and os.environ.get("AIOS_DECODE_PIPELINE", "1") != "0"
        self._pending: Optional[List[_Seq]] = None  # rows whose sampled step is in flight
        self.thread = threading.Thread(target=self._run, name=f"sched-{name}", daemon=True)
        self.thread.start()

    # ------------------------------------------------------------------ public
    def submit(self, req: GenRequest):
        with self.cv:
            self.queue.append(req)
            self.stats["requests"] += 1
            self.cv.notify()

    def close(self):
        with self.cv:
            self.stop_flag = True
            self.cv.notify()
        self.thread.join(timeout=10)

    @property
    def load(self) -> int:
        return len(self.queue) + len(self.active) + len(self.prefilling)

    # ------------------------------------------------------------------ worker
    def _run(self):
        while True:
            with self.cv:
                while not self.stop_flag and not self.queue and not self.active and not self.prefilling:
                    self.cv.wait(timeout=1.0)
                if self.stop_flag:
                    self._discard_pending()
                    for s in list(self.active) + list(self.prefilling):
                        self._finish(s, "cancelled")
                    while self.queue:
                        r = self.queue.popleft()
                        self._done(r, GenResult("", [], len(r.prompt_ids), 0, "cancelled"))
                    return
                admit = []
                while (self.queue and self.free_slots and
                       len(self.active) + len(self.prefilling) + len(admit) < self.max_batch):
                    admit.append(self.queue.popleft())
            if admit or self.prefilling:
                self._drain()  # (no other engine call while a pipelined step is in flight)
            for r in admit:
                try:
                    self._admit(r)
                    self.last_progress = time.time()
                except ValueError as e:  # request error (e.g. prompt too long): the engine is fine
                    self._done(r, GenResult("", [], len(r.prompt_ids), 0, "error", error=str(e)))
                except Exception as e:  # noqa: BLE001 - engine failure: reported to the caller
                    log.exception("admission failed")
                    self._engine_failed(e)
                    self._done(r, GenResult("", [], len(r.prompt_ids), 0, "error", error=str(e)))
            if self.prefilling:
                seq = self.prefilling[0]
                try:
                    self._prefill_chunk(seq)
                    self.last_progress = time.time()
                except ValueError as e:
                    self._finish(seq, "error", str(e))
                except Exception as e:  # noqa: BLE001
                    log.exception("prefill failed")
                    self._engine_failed(e)
                    self._finish(seq, "error", str(e))
            if self.active:
                try:
                    t0 = time.time()
                    self._step()
                    self.last_progress = time.time()
                    self._step_ms.append((self.last_progress - t0) * 1e3)
                except Exception as e:  # noqa: BLE001
                    log.exception("decode step failed")
                    self._engine_failed(e)
                    self._pending = None
                    for s in list(self.active):
                        self._finish(s, "error", str(e))

    @staticmethod
    def _common(c: List[int], ids: List[int]) -> int:
        n, lim = 0, min(len(c), len(ids) - 1)  # >= 1 token is always prefilled (its logits)
        while n < lim and c[n] == ids[n]:
            n += 1
        return n

    def _pick_slot(self, ids: List[int]):
        """(slot, reused tokens): the free slot whose own cache matches best, or -- when another
        slot (free or decoding) holds a longer matching prefix -- the free slot with the least
        cached content, which then shares that prefix through the paged KV."""
        best, best_len = None, -1
        for s in self.free_slots:
            n = self._common(self.slot_cache[s], ids)
            if n > best_len:
                best, best_len = s, n
        best_len = max(best_len, 0)
        if self.share_prefix:
            src, src_len = None, best_len
            for s, c in self.slot_cache.items():
                if s != best:
                    n = self._common(c, ids)
                    if n > src_len:
                        src, src_len = s, n
            if src is not None and src_len >= best_len + self.min_shared_prefix:
                dst = min(self.free_slots, key=lambda f: len(self.slot_cache[f]))
                self.engine.copy_slot(src, dst, src_len)
                self.slot_cache[dst] = list(ids[:src_len])
                self.stats["shared_prefix_tokens"] = self.stats.get("shared_prefix_tokens", 0) + src_len
                return dst, src_len
        return best, best_len

    def _admit(self, r: GenRequest):
        ids = r.prompt_ids
        if len(ids) >= self.max_ctx:
            raise ValueError(f"prompt of {len(ids)} tokens exceeds the context window ({self.max_ctx})")
        r.max_tokens = max(1, min(r.max_tokens, self.max_ctx - len(ids)))
        r.min_tokens = min(r.min_tokens, r.max_tokens)
        slot, common = self._pick_slot(ids)
        self.free_slots.remove(slot)
        seq = _Seq(r, slot)
        seq.cached = common
        seq.pos = common
        seq.todo = list(ids[common:])
        self.slot_cache[slot] = list(ids[:common])
        self.stats["cached_tokens"] += common
        self.prefilling.append(seq)
        if not self.active:  # nothing decoding: no stream to protect, prefill it right away
            try:
                self._prefill_chunk(seq, whole=True)
            except Exception:
                if seq in self.prefilling:  # the caller reports the error; the slot goes back
                    self.prefilling.remove(seq)
                    self.free_slots.append(slot)
                raise

    def _prefill_chunk(self, seq: _Seq, whole: bool = False):
        """Prefill the next chunk of seq's prompt; the last chunk samples the first token and
        moves the sequence to the decoding set."""
        r = seq.req
        if r.cancelled:
            self._finish(seq, "cancelled")
            return
        n = len(seq.todo) if (whole or not self.active) else min(len(seq.todo), max(1, self.prefill_chunk))
        chunk, last = seq.todo[:n], n == len(seq.todo)
        tp0 = time.perf_counter()
        logits = self.engine.prefill(seq.slot, chunk, seq.pos, last)
        self.timing["prefill_s"] += time.perf_counter() - tp0
        self.step_log.append((time.perf_counter(), -n))  # a prefill chunk between decode steps
        seq.todo = seq.todo[n:]
        seq.pos += n
        self.slot_cache[seq.slot].extend(chunk)
        self.stats["prefill_tokens"] += n
        if not last:
            return
        self.prefilling.remove(seq)
        mask = None
        if r.json_mode and self.grammar is not None:
            seq.grammar_state = self.grammar.initial()
            mask = self._mask(seq)
        topk = int(r.top_k) if r.temperature > 0 else 0
        topp = float(r.top_p) if 0.0 < r.top_p < 1.0 else 1.0
        if hasattr(self.engine, "sample_first"):
            # on the device, the decode steps' sampler and RNG stream (seed, position)
            tok = int(self.engine.sample_first(seq.pos - 1, float(r.temperature), topk, topp, seq.seed,
                                               bytes(mask) if mask is not None else b""))
        else:
            rng = np.random.default_rng([seq.seed & 0xFFFFFFFF, seq.pos - 1])
            tok = host_sampler.sample(logits, r.temperature, r.top_k, r.top_p, mask, rng)
        seq.t_first = time.time()
        self.active.append(seq)
        self._accept(seq, tok)

    def _accept(self, seq: _Seq, tok: int) -> bool:
        """Record a sampled token; returns False when the sequence finished."""
        r = seq.req
        if r.cancelled:
            self._finish(seq, "cancelled")
            return False
        if tok in self.eos or (r.stop_ids and tok in r.stop_ids):
            self._finish(seq, "stop")
            return False
        if seq.grammar_state is not None:
            if not self.grammar.accept_token(seq.grammar_state, tok):
                self._finish(seq, "stop")
                return False
        seq.out.append(tok)
        seq.last = tok
        self.stats["tokens"] += 1
        self._tok_times.append(time.time())
        if r.on_delta is not None:
            # incremental detokenization over a short window (decoding the whole output every
            # token is O(n^2) per stream and dominated the host side of a step)
            prev = self.tok.decode(seq.out[seq.p_off:seq.r_off])
            text = self.tok.decode(seq.out[seq.p_off:])
            if len(text) > len(prev) and not text.endswith("�"):
                delta = text[len(prev):]
                seq.emitted += delta
                seq.p_off, seq.r_off = seq.r_off, len(seq.out)
                r.on_delta(delta)
        if seq.grammar_state is not None and self.grammar.complete(seq.grammar_state):
            self._finish(seq, "grammar")
            return False
        if len(seq.out) >= r.max_tokens or seq.pos + 1 >= self.max_ctx:
            self._finish(seq, "length")
            return False
        if r.deadline and time.time() > r.deadline:
            self._finish(seq, "deadline")
            return False
        return True

    def _engine_failed(self, e: BaseException):
        self.stats["errors"] += 1
        self.failed = f"{type(e).__name__}: {e}"

    def stalled(self, timeout_s: float) -> bool:
        """Work is pending but nothing completed for timeout_s (a hung device call)."""
        return bool(self.active or self.queue) and time.time() - self.last_progress > timeout_s

    def metrics(self) -> dict:
        now = time.time()
        while self._tok_times and now - self._tok_times[0] > 10.0:
            self._tok_times.popleft()
        ttft = sorted(self._ttft)
        st = self.stats
        return {"tokens_per_s": len(self._tok_times) / 10.0,
                "ttft_p50_ms": ttft[len(ttft) // 2] if ttft else 0.0,
                "itl_ms": sum(self._step_ms) / len(self._step_ms) if self._step_ms else 0.0,
                # a sequence mid chunked-prefill holds a slot and is work in flight: it
                # counts as active for idle-unload and replica routing
                "active": len(self.active) + len(self.prefilling), "decoding": len(self.active),
                "prefilling": len(self.prefilling), "queued": len(self.queue),
                "kv_slot_util": (len(self.active) + len(self.prefilling)) / max(1, self.max_slots),
                "avg_batch": st["batch_sum"] / st["steps"] if st["steps"] else 0.0,
                "prefix_hit_tokens": st["cached_tokens"], "errors": st["errors"]}

    def _mask(self, seq: _Seq) -> bytes:
        if len(seq.out) + 1 < seq.req.min_tokens:  # the next token may not complete the object
            return self.grammar.mask_open(seq.grammar_state)
        return self.grammar.mask(seq.grammar_state)

    def _drain(self):
        """Collect and accept a pipelined step still in flight (before any other engine call)."""
        rows = self._pending
        if rows is None:
            return
        self._pending = None
        try:
            out = self.engine.decode_collect()
        except Exception as e:  # noqa: BLE001
            log.exception("decode step failed")
            self._engine_failed(e)
            for s in list(self.active):
                self._finish(s, "error", str(e))
            return
        self._take(rows, out)

    def _discard_pending(self):
        if self._pending is not None:
            self._pending = None
            try:
                self.engine.decode_collect()
            except Exception:  # noqa: BLE001
                pass

    def _take(self, rows, out):
        self.stats["steps"] += 1
        self.stats["batch_sum"] += len(rows)
        for s, t in zip(rows, out):
            s.pos += 1
            self.slot_cache[s.slot].append(s.last)
            self._accept(s, int(t))

    def _can_speculate(self, rows) -> bool:
        """Whether step t+1 of the same rows can be queued before step t's tokens are known: no
        admission or prefill will interleave, and no row is certain to finish at step t."""
        if self.prefilling or (self.queue and self.free_slots and
                               len(self.active) + len(self.prefilling) < self.max_batch):
            return False
        now = time.time()
        for s in rows:
            r = s.req
            if r.cancelled or len(s.out) + 1 >= r.max_tokens or s.pos + 2 >= self.max_ctx:
                return False
            if r.deadline and now > r.deadline:
                return False
        return True

    def _submit(self, rows, first: bool):
        """Queue the forward of the rows' next step: `first` with the host's tokens at s.pos, else
        with the tokens the in-flight sampler leaves on the device, at s.pos + 1."""
        self.engine.decode_submit([s.slot for s in rows], [s.last for s in rows] if first else [],
                                  [s.pos + (0 if first else 1) for s in rows],
                                  [float(s.req.temperature) for s in rows],
                                  [int(s.req.top_k) if s.req.temperature > 0 else 0 for s in rows], 0,
                                  [float(s.req.top_p) if 0.0 < s.req.top_p < 1.0 else 1.0 for s in rows],
                                  [s.seed for s in rows])

    def _masks(self, rows) -> bytes:
        if not any(s.grammar_state is not None for s in rows):
            return b""
        if self._full_mask is None:
            self._full_mask = host_sampler.all_allowed(self.vocab)
        return b"".join(self._mask(s) if s.grammar_state is not None else self._full_mask for s in rows)

    def _step_pipelined(self):
        t0 = time.perf_counter()
        rows = self._pending
        if rows is None:  # a batch's first step (or after an admission / finish): host tokens
            rows = list(self.active)
            self._submit(rows, True)
            self.engine.decode_sample(self._masks(rows))
        self._pending = None
        spec = self._can_speculate(rows)
        if spec:
            self._submit(rows, False)
        t1 = time.perf_counter()
        out = self.engine.decode_collect()
        t2 = time.perf_counter()
        self._take(rows, out)
        t2b = time.perf_counter()
        if spec and self.active == rows:
            # nobody finished or joined: sample the queued forward with the masks of the new tokens
            self.engine.decode_sample(self._masks(rows))
            self._pending = rows
        # (spec and a row finished: the queued forward is dropped -- its KV writes at the next
        # position are rewritten by whatever runs there next)
        t3 = time.perf_counter()
        tm = self.timing
        tm["mask_s"] += (t3 - t2b) + (t1 - t0)   # masks + submit / sampler enqueue
        tm["engine_decode_s"] += t2 - t1          # waiting for the device
        tm["accept_s"] += t2b - t2
        self.step_log.append((t3, len(rows)))

    def _step(self):
        if self.pipeline:
            return self._step_pipelined()
        B = len(self.active)
        slots = [s.slot for s in self.active]
        toks = [s.last for s in self.active]
        pos = [s.pos for s in self.active]
        temps = [float(s.req.temperature) for s in self.active]
        topk = [int(s.req.top_k) if s.req.temperature > 0 else 0 for s in self.active]
        seeds = [s.seed for s in self.active]  # per row: a request samples the same at any batch row
        t0 = time.perf_counter()
        mask = b""
        if any(s.grammar_state is not None for s in self.active):
            if self._full_mask is None:
                self._full_mask = host_sampler.all_allowed(self.vocab)
            mask = b"".join(self._mask(s) if s.grammar_state is not None else self._full_mask for s in self.active)
        topp = [float(s.req.top_p) if 0.0 < s.req.top_p < 1.0 else 1.0 for s in self.active]
        t1 = time.perf_counter()
        out = self.engine.decode(slots, toks, pos, temps, topk, 0, mask, topp, seeds)
        t2 = time.perf_counter()
        self.stats["steps"] += 1
        self.stats["batch_sum"] += B
        for s, t in zip(list(self.active), out):
            s.pos += 1
            self.slot_cache[s.slot].append(s.last)
            self._accept(s, int(t))
        t3 = time.perf_counter()
        tm = self.timing
        tm["mask_s"] += t1 - t0
        tm["engine_decode_s"] += t2 - t1
        tm["accept_s"] += t3 - t2
        self.step_log.append((t3, B))

    def _finish(self, seq: _Seq, reason: str, error: str = ""):
        if seq in self.active:
            self.active.remove(seq)
        if seq in self.prefilling:
            self.prefilling.remove(seq)
        self.free_slots.append(seq.slot)
        r = seq.req
        text = self.tok.decode(seq.out)
        if r.on_delta is not None and len(text) > len(seq.emitted) and text.startswith(seq.emitted):
            r.on_delta(text[len(seq.emitted):])
        now = time.time()
        if seq.t_first:
            self._ttft.append((seq.t_first - r.submitted_at) * 1e3)
        self._done(r, GenResult(
            text=text, token_ids=list(seq.out), prompt_tokens=len(r.prompt_ids), completion_tokens=len(seq.out),
            finish_reason=reason, ttft_ms=(seq.t_first - r.submitted_at) * 1e3 if seq.t_first else 0.0,
            latency_ms=(now - r.submitted_at) * 1e3, cached_prompt_tokens=seq.cached, error=error))

    @staticmethod
    def _done(r: GenRequest, res: GenResult):
        if r.on_done is not None:
            try:
                r.on_done(res)
            except Exception:  # noqa: BLE001
                log.exception("on_done callback failed")
