"""GPU: the fused batch-1 attention block (kernels/attn_block.hip) against the three-launch path.

QKV GEMV -> attention -> O GEMV run as workgroup roles of ONE launch wired by in-launch
hand-offs (AIOS_FUSE_ATTN=1: attention + O fused, 2: all three).  The roles run the same device
code as the separate kernels, so tokens must be identical and logits equal to rounding, in the
short-context mode (<= 512 keys, one workgroup per head) and the split-K long mode (last-arriver
combine), for GQA groups 4 (Mistral) and 8 (TinyLlama / Llama-3), head_dim 128 and 64, and for
mixed Q4_K/Q6_K QKV layers.  A reference-model check is in test_engine_gpu.py (its batch-1
decode runs the fused path by default).
"""
import dataclasses

import numpy as np
import pytest

from aios_amd.models.config import get_preset

pytestmark = pytest.mark.gpu

SHAPES = {
    "mistral_g4_hd128": dataclasses.replace(get_preset("test-mistral-shape"), max_ctx=1024),
    "tinyllama_g8_hd64": dataclasses.replace(get_preset("test-mistral-shape"), name="t8", n_heads=16, n_kv_heads=2,
                                             head_dim=64, max_ctx=1024),
}


def _run(cfg, mode, prompt_len, steps, monkeypatch, graph=True):
    from aios_amd.runtime.loader import random_engine

    monkeypatch.setenv("AIOS_FUSE_ATTN", str(mode))
    eng = random_engine(cfg, "Q4_K_M", seed=3, max_ctx=cfg.max_ctx, max_slots=1, max_batch=1)
    prompt = [cfg.bos_id] + [(11 * i + 5) % (cfg.vocab_size - 3) + 3 for i in range(prompt_len - 1)]
    first = int(np.argmax(eng.prefill(0, prompt, 0, True)))
    eng.decode_loop_prepare([0], [first], [prompt_len])
    eng.decode_loop_run(1, steps, graph)
    eng.synchronize()  # raises if an in-launch hand-off gave up
    toks = list(eng.decode_loop_history(1, prompt_len + 1, steps))
    logits = np.asarray(eng.last_logits(1)).reshape(-1)
    del eng
    return toks, logits


@pytest.mark.parametrize("shape", sorted(SHAPES))
@pytest.mark.parametrize("prompt_len", [37, 300, 700])
@pytest.mark.parametrize("mode", [1, 2])
def test_fused_attention_block_matches_three_launches(shape, prompt_len, mode, monkeypatch):
    cfg = SHAPES[shape]
    ref_t, ref_l = _run(cfg, 0, prompt_len, 12, monkeypatch)
    t, lg = _run(cfg, mode, prompt_len, 12, monkeypatch)
    assert t == ref_t
    scale = max(1.0, float(np.abs(ref_l).max()))
    assert float(np.abs(lg - ref_l).max()) <= 1e-3 * scale


def test_fused_attention_block_eager_and_graph_agree(monkeypatch):
    cfg = SHAPES["mistral_g4_hd128"]
    g, _ = _run(cfg, 2, 130, 8, monkeypatch, graph=True)
    e, _ = _run(cfg, 2, 130, 8, monkeypatch, graph=False)
    assert g == e
