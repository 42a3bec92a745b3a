"""Host-side sampling for the first token after prefill (the decode steps sample on device).

Semantics match the device sampler (aios::sample_kernel): temperature <= 0 -> greedy argmax,
else sample from softmax(logits / T) restricted to the top-k (if k > 0) and nucleus top-p (if
0 < p < 1), always within the grammar's allowed-token bitmask when one is given.
"""
from __future__ import annotations

from typing import Optional

import numpy as np


def mask_to_bool(mask: bytes, vocab: int) -> np.ndarray:
    bits = np.unpackbits(np.frombuffer(mask, dtype=np.uint8), bitorder="little")
    return bits[:vocab].astype(bool)


def sample(logits: np.ndarray, temperature: float = 0.0, top_k: int = 0, top_p: float = 1.0,
           mask: Optional[bytes] = None, rng: Optional[np.random.Generator] = None) -> int:
    l = np.asarray(logits, dtype=np.float64).copy()
    if mask is not None:
        allowed = mask_to_bool(mask, l.shape[0])
        if not allowed.any():
            return int(np.argmax(l))
        l[~allowed] = -np.inf
    if temperature <= 0.0:
        return int(np.argmax(l))
    rng = rng or np.random.default_rng()
    l = l / temperature
    if top_k and 0 < top_k < l.shape[0]:
        kth = np.partition(l, -top_k)[-top_k]
        l[l < kth] = -np.inf
    l -= np.max(l)
    p = np.exp(l)
    p /= p.sum()
    if 0.0 < top_p < 1.0:
        order = np.argsort(-p)
        cum = np.cumsum(p[order])
        cut = order[np.searchsorted(cum, top_p) + 1:]
        p[cut] = 0.0
        p /= p.sum()
    return int(rng.choice(p.shape[0], p=p))


def all_allowed(vocab: int) -> bytes:
    m = np.zeros((vocab + 7) // 8, np.uint8) + 0xFF
    return m.tobytes()
