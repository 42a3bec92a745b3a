"""GGUF -> native engine loader (SURVEY.md §3.4 `load`, §2.7 K12).

Replaces `ModelManager::load_model` spawning llama-server (`runtime/src/model_manager.rs:149-277`):
the file is memory-mapped, each tensor's raw block bytes are handed zero-copy to the engine,
which uploads them to HBM and repacks them into the GEMV/MFMA layout.  Under tensor
parallelism each rank receives only its shard: column-parallel Q/K/V/gate/up (whole heads /
rows), row-parallel attn_output/ffn_down (whole quant blocks along K), vocab-parallel lm_head
(output.weight rows, the logits completed by an xGMI all-gather), replicated embeddings and norms
(SURVEY.md §2.9 TP row).
"""
from __future__ import annotations

import logging
import os
import time
from typing import Optional

import numpy as np

from ..gguf.quants import BLOCK_INFO, GGMLType
from ..gguf.reader import GGUFReader
from ..models.config import ModelConfig
from . import native

log = logging.getLogger("aios.runtime.loader")

COLUMN_PARALLEL = ("attn_q.weight", "attn_k.weight", "attn_v.weight", "ffn_gate.weight", "ffn_up.weight",
                   "attn_q.bias", "attn_k.bias", "attn_v.bias")
ROW_PARALLEL = ("attn_output.weight", "ffn_down.weight")


def shard_tensor(name: str, raw: np.ndarray, ggml_type: int, rows: int, cols: int, rank: int, tp: int,
                 vocab_parallel: bool = False):
    """Return (raw_shard, rows, cols) of this rank's slice of a GGUF tensor."""
    if tp == 1:
        return raw, rows, cols
    short = name.split(".", 2)[-1] if name.startswith("blk.") else name
    blk, bpb = BLOCK_INFO[GGMLType(ggml_type)]
    if short in COLUMN_PARALLEL or (vocab_parallel and name == "output.weight"):
        if short.endswith(".bias"):  # 1-D: rows == 1, cols == n
            n = cols // tp
            return raw.view(np.uint8).reshape(cols, -1)[rank * n:(rank + 1) * n].ravel(), 1, n
        if rows % tp:
            raise ValueError(f"{name}: {rows} rows not divisible by TP={tp}")
        n = rows // tp
        rb = raw.size // rows
        return raw[rank * n * rb:(rank + 1) * n * rb], n, cols
    if short in ROW_PARALLEL:
        nblk = cols // blk
        if nblk % tp:
            raise ValueError(f"{name}: K={cols} not divisible into whole {blk}-blocks for TP={tp}")
        nb = nblk // tp
        r = raw.reshape(rows, nblk, bpb)[:, rank * nb:(rank + 1) * nb, :]
        return np.ascontiguousarray(r).ravel(), rows, nb * blk
    return raw, rows, cols


def load_engine(path: str, max_ctx: Optional[int] = None, max_slots: int = 4, max_batch: int = 8, device: int = 0,
                tp_rank: int = 0, tp_size: int = 1, name: Optional[str] = None, verbose: bool = False,
                act_q8: bool = True, cu_mask: Optional[list] = None, kv_dtype: str = "bf16"):
    """Load a GGUF file into a native Engine on `device`. Returns (engine, ModelConfig, reader)."""
    m = native.require()
    t0 = time.time()
    r = GGUFReader(path)
    cfg = ModelConfig.from_gguf(r, name=name)
    ec = native.engine_config(cfg, max_ctx=max_ctx or min(cfg.max_ctx, 4096), max_slots=max_slots,
                              max_batch=max_batch, device=device, tp_rank=tp_rank, tp_size=tp_size,
                              act_q8=act_q8, cu_mask=cu_mask, kv_dtype=kv_dtype)
    eng = m.Engine(ec)
    vp = bool(ec.vocab_parallel)
    for tname, ti in r.tensors.items():
        raw = r.tensor_array(tname)
        rows, cols = ti.rows, ti.cols
        raw, rows, cols = shard_tensor(tname, raw, int(ti.ggml_type), rows, cols, tp_rank, tp_size, vp)
        eng.set_tensor(tname, int(ti.ggml_type), rows, cols, raw)
    finalize(eng)
    if verbose:
        print(f"[loader] {cfg.name}: {eng.weight_bytes / 1e9:.2f} GB weights, {eng.kv_bytes / 1e9:.2f} GB KV, "
              f"{time.time() - t0:.1f}s")
    return eng, cfg, r


def finalize(eng):
    """Engine.finalize with the prefill-GEMM plans persisted when AIOS_GEMM_PF_PLANS names a file:
    plans saved by an earlier process are installed first (finalize then times only shapes it does
    not hold), and the process's plans are written back -- every process serving a model runs the
    same tile / split plans (per-process tuning noise changed prefill numerics)."""
    import json

    m = native.require()
    path = os.environ.get("AIOS_GEMM_PF_PLANS", "")
    if path and os.path.exists(path):
        try:
            with open(path) as f:
                m.gemm_pf_import([int(v) for v in json.load(f)])
        except (OSError, ValueError, RuntimeError) as e:
            log.warning("ignoring prefill plan file %s: %s", path, e)
    eng.finalize()
    if path:
        tmp = f"{path}.{os.getpid()}.tmp"
        try:
            with open(tmp, "w") as f:
                json.dump(list(m.gemm_pf_export()), f)
            os.replace(tmp, path)
        except OSError as e:
            log.warning("cannot persist prefill plans to %s: %s", path, e)


def random_engine(cfg: ModelConfig, recipe: str = "Q4_K_M", seed: int = 0, max_ctx: Optional[int] = None,
                  max_slots: int = 4, max_batch: int = 8, device: int = 0, tp_rank: int = 0, tp_size: int = 1,
                  act_q8: bool = True, cu_mask: Optional[list] = None, kv_dtype: str = "bf16",
                  stream_priority: int = 0):
    """Engine with random-init weights of `cfg`'s architecture generated directly in HBM (cu_mask: the
    CUs its stream may use, native.cu_mask_words)."""
    m = native.require()
    ec = native.engine_config(cfg, max_ctx=max_ctx or min(cfg.max_ctx, 4096), max_slots=max_slots,
                              max_batch=max_batch, device=device, tp_rank=tp_rank, tp_size=tp_size,
                              act_q8=act_q8, cu_mask=cu_mask, kv_dtype=kv_dtype, stream_priority=stream_priority)
    eng = m.Engine(ec)
    eng.init_random(recipe, seed)
    finalize(eng)
    return eng
