"""CPU inference engine: the runtime's no-GPU backend (BASELINE config #1 -- "TinyLlama Q4_0 greedy
decode via the runtime on CPU, plumbing, no GPU"; the reference's default deployment is
llama-server with `gpu_layers: 0`, `runtime/src/main.rs:108-115`).

Same Python surface as the native `Engine` (prefill / decode / config / weight_bytes / kv_bytes /
close), so the scheduler, the AIRuntime gRPC service and the OpenAI HTTP endpoint run unchanged
on it.  Numerics are the fp32 reference forward (`aios_amd.models.reference`) over the exact
dequantised GGUF weights with a per-slot KV cache; sampling uses the host sampler (same
semantics as the device sampler, incl. the JSON-grammar bitmask).
"""
from __future__ import annotations

import dataclasses
from typing import Dict, List, Optional

import numpy as np
import torch

from ..models.reference import ReferenceModel
from . import sampler as host_sampler


@dataclasses.dataclass
class CpuEngineConfig:
    max_ctx: int
    max_slots: int
    max_batch: int
    vocab_size: int
    n_layers: int
    device: str = "cpu"


class CpuEngine:
    def __init__(self, model: ReferenceModel, max_ctx: int = 2048, max_slots: int = 4, max_batch: int = 4,
                 threads: int = 0):
        if threads > 0:
            torch.set_num_threads(threads)
        self.model = model
        self.cfg = model.cfg
        self.config = CpuEngineConfig(max_ctx=max_ctx, max_slots=max_slots, max_batch=max_batch,
                                      vocab_size=model.cfg.vocab_size, n_layers=model.cfg.n_layers)
        self.caches: Dict[int, dict] = {}
        self.weight_bytes = int(sum(t.numel() * t.element_size() for t in model.w.values()))
        c = model.cfg
        self.kv_bytes = 2 * c.n_layers * max_slots * max_ctx * c.n_kv_heads * c.head_dim * 4
        self.last: Optional[np.ndarray] = None

    @classmethod
    def from_gguf(cls, path: str, max_ctx: int = 2048, max_slots: int = 4, max_batch: int = 4,
                  threads: int = 0) -> "CpuEngine":
        return cls(ReferenceModel.from_gguf(path, kv_bf16=False), max_ctx, max_slots, max_batch, threads)

    # ------------------------------------------------------------------ cache
    def _cache_at(self, slot: int, start: int) -> dict:
        if not 0 <= slot < self.config.max_slots:
            raise ValueError(f"bad slot {slot}")
        c = self.caches.get(slot)
        if c is None or start == 0:
            c = self.model.new_cache()
            self.caches[slot] = c
        if start > c["len"]:
            raise ValueError(f"slot {slot}: position {start} beyond the cached {c['len']} tokens")
        if start < c["len"]:  # prefix reuse: drop the cached tail
            for l in range(self.cfg.n_layers):
                c["k"][l] = c["k"][l][:start]
                c["v"][l] = c["v"][l][:start]
            c["len"] = start
        return c

    def copy_slot(self, src: int, dst: int, n: int):
        s = self.caches.get(src)
        if s is None:
            return
        self.caches[dst] = {"k": [k[:n].clone() for k in s["k"]], "v": [v[:n].clone() for v in s["v"]], "len": n}

    # ------------------------------------------------------------------ inference
    def prefill(self, slot: int, ids: List[int], start: int = 0, want_logits: bool = True):
        if start + len(ids) > self.config.max_ctx:
            raise ValueError("prefill: context overflow")
        c = self._cache_at(slot, start)
        logits = self.model.forward(list(ids), c)[-1].numpy()
        self.last = logits[None]
        return logits if want_logits else []

    def decode(self, slots, toks, pos, temps, topk, seed, mask: bytes = b"", top_p=None, seeds=None):
        V = self.config.vocab_size
        row = (V + 7) // 8
        out, rows = [], []
        for b, (slot, tok, p) in enumerate(zip(slots, toks, pos)):
            if p >= self.config.max_ctx:
                raise ValueError("decode: position out of range")
            c = self._cache_at(slot, p)
            logits = self.model.forward([int(tok)], c)[-1].numpy()
            rows.append(logits)
            m = mask[b * row:(b + 1) * row] if mask else None
            t = float(temps[b]) if b < len(temps) else 0.0
            k = int(topk[b]) if b < len(topk) else 0
            # per-row seed: the row's stream depends on (seed, position) only, as on the GPU
            rng = (np.random.default_rng([int(seeds[b]) & 0xFFFFFFFF, p]) if seeds else
                   np.random.default_rng((int(seed) << 20) ^ (slot << 12) ^ p))
            tp = float(top_p[b]) if top_p is not None and b < len(top_p) else 1.0
            out.append(host_sampler.sample(logits, t, k, tp, m, rng))
        self.last = np.stack(rows) if rows else None
        return out

    def sample_first(self, pos, temperature, top_k, top_p, seed, mask: bytes = b""):
        """the token after a prefill, from its last logits, with the decode steps' RNG stream"""
        logits = self.last[0]
        rng = np.random.default_rng([int(seed) & 0xFFFFFFFF, int(pos)])
        return host_sampler.sample(logits, float(temperature), int(top_k), float(top_p), mask or None, rng)

    def last_logits(self, B: int):
        return self.last[:B].reshape(-1) if self.last is not None else np.zeros(0, np.float32)

    def synchronize(self):
        pass

    def close(self):
        self.caches.clear()
