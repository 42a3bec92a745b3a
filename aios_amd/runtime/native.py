"""Loader for the native engine extension (`aios_amd/_engine*.so`).

torch is imported first on purpose: torch-ROCm bundles `libamdhip64.so.7`; importing it before
the extension makes the dynamic loader resolve our DT_NEEDED entry to that same runtime, so one
process never holds two HIP runtimes.

On a machine with a GPU the extension is mandatory: `require()` raises instead of silently
falling back to a Python path (the round-end checks record which .so files were loaded).
"""
from __future__ import annotations

import importlib
import os
from typing import Optional

_mod = None
_err: Optional[BaseException] = None


def load(build_if_missing: bool = True):
    global _mod, _err
    if _mod is not None:
        return _mod
    try:
        import torch  # noqa: F401  (see module docstring)
    except Exception:  # pragma: no cover - torch is present in this image
        pass
    try:
        _mod = importlib.import_module("aios_amd._engine")
        return _mod
    except ImportError as e:
        _err = e
    if build_if_missing and os.environ.get("AIOS_NO_AUTOBUILD") != "1":
        from .. import _build

        _build.build(verbose=False)
        importlib.invalidate_caches()
        _mod = importlib.import_module("aios_amd._engine")
        return _mod
    raise ImportError(f"aios_amd native engine not built: {_err}")


def available() -> bool:
    try:
        load(build_if_missing=False)
        return True
    except Exception:
        return False


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available() and torch.cuda.device_count() > 0
    except Exception:
        return False


def require():
    """The native engine, loudly: on a GPU box a missing extension is an error."""
    return load(build_if_missing=True)


KV_DTYPES = ("bf16", "fp8", "fp8_e4m3")


def kv_fp8_flag(kv_dtype: str) -> int:
    """KV cache dtype name -> EngineConfig.kv_fp8: 'bf16' (default) or 'fp8' / 'fp8_e4m3' (OCP e4m3
    with per-layer K / V scales, half the cache bytes)."""
    k = (kv_dtype or "bf16").strip().lower()
    if k not in KV_DTYPES:
        raise ValueError(f"kv_dtype must be one of {KV_DTYPES}, not {kv_dtype!r}")
    return 0 if k == "bf16" else 1


def cu_mask_words(n: int, first: int = 0, total: int = 256) -> list:
    """A CU mask (32 CUs per word) of n CUs for one co-resident tier: CU slots [first, first + n/8) of
    every aligned group of 32 CU ids.  Whether the driver numbers CUs XCD-major (32 per XCD) or
    XCD-minor (id % 8), every XCD then keeps CUs of the tier (no XCD left without any -- each XCD has
    its own L2 and dispatcher) and two tiers with disjoint [first, first + n/8) ranges never share a CU.
    n must be a multiple of 8 between 64 and total."""
    if n % 8 or not (64 <= n <= total) or total % 32:
        raise ValueError(f"cu mask: {n} CUs (multiple of 8, 64..{total})")
    per = n // (total // 32)
    if first < 0 or first + per > 32:
        raise ValueError("cu mask: slot range outside the 32-CU group")
    words = [0] * (total // 32)
    for i in range(total):
        if first <= i % 32 < first + per:
            words[i // 32] |= 1 << (i % 32)
    return words


def engine_config(cfg, max_ctx: Optional[int] = None, max_slots: int = 4, max_batch: int = 8, device: int = 0,
                  tp_rank: int = 0, tp_size: int = 1, act_q8: bool = True, vocab_parallel: bool = True,
                  cu_mask: Optional[list] = None, kv_dtype: str = "bf16", stream_priority: int = 0):
    """aios_amd.models.config.ModelConfig -> native EngineConfig (per-rank shapes under TP).
    Under TP the lm_head is vocab-parallel (V/tp rows per rank + logits all-gather) unless the
    embeddings are tied or V is not divisible by tp."""
    m = require()
    ec = m.EngineConfig()
    ec.name = cfg.name
    ec.vocab_size = cfg.vocab_size
    ec.d_model = cfg.d_model
    ec.n_layers = cfg.n_layers
    if cfg.n_heads % tp_size or cfg.n_kv_heads % tp_size or cfg.d_ff % tp_size:
        raise ValueError(f"TP={tp_size} does not divide heads/kv_heads/d_ff of {cfg.name}")
    ec.n_heads = cfg.n_heads // tp_size
    ec.n_kv_heads = cfg.n_kv_heads // tp_size
    ec.head_dim = cfg.head_dim
    ec.d_ff = cfg.d_ff // tp_size
    ec.rope_theta = float(cfg.rope_theta)
    ec.rope_neox = 1 if cfg.rope_mode == 2 else 0
    ec.norm_eps = float(cfg.norm_eps)
    ec.max_ctx = int(max_ctx or cfg.max_ctx)
    ec.max_slots = max_slots
    ec.max_batch = max_batch
    ec.tie_embeddings = int(cfg.tie_embeddings)
    ec.qk_norm = int(cfg.qk_norm)
    ec.qkv_bias = int(cfg.qkv_bias)
    ec.tp_rank = tp_rank
    ec.tp_size = tp_size
    ec.vocab_parallel = int(bool(vocab_parallel) and tp_size > 1 and not cfg.tie_embeddings
                            and cfg.vocab_size % tp_size == 0)
    ec.device = device
    if cu_mask:
        ec.cu_mask = [int(w) & 0xFFFFFFFF for w in cu_mask]
    ec.kv_fp8 = kv_fp8_flag(kv_dtype)
    ec.stream_priority = int(stream_priority)
    ec.act_q8 = int(act_q8)
    return ec
