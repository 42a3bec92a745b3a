"""GPU: the persistent batch-1 decode kernel (kernels/decode_mk.hip) against the launch-per-op path
and the fp32 reference model.

The persistent step must produce the same logits as the 5-launches-per-layer path (same int8
activation precision, row sums in a different order: tolerance, not bit equality), keep doing so
over graph replays (its arrival counters re-arm themselves), handle contexts that split the
attention into several pieces per KV head (last-arriver combine), and the paged block table.
"""
import numpy as np
import pytest
import torch

from aios_amd.models.config import ModelConfig, get_preset

pytestmark = pytest.mark.gpu


def _cfg(name):
    if name == "g8-hd64":  # TinyLlama's head layout (32 q / 4 kv heads of 64) at test size
        return ModelConfig(name="g8-hd64", vocab_size=1024, d_model=1024, n_layers=2, n_heads=16, n_kv_heads=2,
                           head_dim=64, d_ff=2048, rope_theta=10000.0, max_ctx=1024)
    if name == "mistral-k":  # Mistral's K widths (chunk rows >= 64: groups straddle <= 2 rows)
        return ModelConfig(name="mistral-k", vocab_size=2048, d_model=2048, n_layers=2, n_heads=16, n_kv_heads=4,
                           head_dim=128, d_ff=4096, rope_theta=1e6, max_ctx=2048)
    return get_preset(name)


def _engine(name, recipe="Q4_K_M", max_ctx=1024, seed=3):
    from aios_amd.runtime.loader import random_engine

    cfg = _cfg(name)
    eng = random_engine(cfg, recipe, seed=seed, max_ctx=max_ctx, max_slots=2, max_batch=4)
    return eng, cfg


def _steps(eng, cfg, prompt, n, mk):
    eng.mk_enabled = mk
    logits = np.asarray(eng.prefill(0, prompt, 0, True))
    tok = int(np.argmax(logits))
    pos = len(prompt)
    out_l, out_t = [], []
    for _ in range(n):
        nxt = eng.decode([0], [tok], [pos])[0]
        out_l.append(np.asarray(eng.last_logits(1)).copy())
        out_t.append(nxt)
        tok = nxt
        pos += 1
    return out_l, out_t


@pytest.mark.parametrize("name", ["test-mistral-shape", "test-small", "g8-hd64", "mistral-k"])
@pytest.mark.parametrize("recipe", ["Q4_K_M", "Q5_K_M"])
def test_mk_matches_launch_path(name, recipe):
    eng, cfg = _engine(name, recipe)
    assert eng.mk_available, "persistent decode kernel not available for this shape"
    prompt = [1] + list(np.random.default_rng(0).integers(3, cfg.vocab_size, 20))
    l_on, t_on = _steps(eng, cfg, prompt, 6, True)
    l_off, t_off = _steps(eng, cfg, prompt, 6, False)
    # compare step logits while the token paths agree (the first steps must)
    for i, (a, b) in enumerate(zip(l_on, l_off)):
        scale = max(1.0, float(np.abs(b).max()))
        err = float(np.abs(a - b).max())
        assert err < 2e-3 * scale, (i, err, scale)
        if t_on[i] != t_off[i]:
            break
    assert t_on[:3] == t_off[:3]


@pytest.mark.parametrize("name", ["test-mistral-shape", "g8-hd64"])
@pytest.mark.parametrize("ctx", [300, 700])
def test_mk_long_context_pieces(name, ctx):
    """contexts of 3-6 attention pieces per KV head: partials + last-arriver combine"""
    eng, cfg = _engine(name, max_ctx=1024)
    rng = np.random.default_rng(1)
    prompt = [1] + list(rng.integers(3, cfg.vocab_size, ctx - 1))
    l_on, _ = _steps(eng, cfg, prompt, 3, True)
    l_off, _ = _steps(eng, cfg, prompt, 3, False)
    a, b = l_on[0], l_off[0]
    err = float(np.abs(a - b).max())
    assert err < 2e-3 * max(1.0, float(np.abs(b).max())), err


def test_mk_graph_loop_replays_match():
    """many captured replays (counters re-armed by the last workgroup) == the launch path"""
    eng, cfg = _engine("test-mistral-shape")
    prompt = [1, 17, 29, 31, 400, 5, 6]
    first = int(np.argmax(np.asarray(eng.prefill(0, prompt, 0, True))))
    hist = {}
    for mk in (True, False):
        eng.mk_enabled = mk
        eng.prefill(0, prompt, 0, False)
        eng.decode_loop_prepare([0], [first], [len(prompt)])
        eng.decode_loop_run(1, 40, True)
        eng.synchronize()
        hist[mk] = eng.decode_loop_history(1, len(prompt) + 1, 40)
    # greedy paths on random weights are chaotic; the first tokens must agree
    assert hist[True][:8] == hist[False][:8]


def test_mk_matches_reference_model(tmp_path):
    """teacher-forced: every persistent step's logits against the fp32 reference forward of the
    same token sequence (greedy paths on random weights can part at near-ties, logits cannot)"""
    from aios_amd.models.reference import ReferenceModel
    from aios_amd.models.synthetic import write_synthetic_gguf
    from aios_amd.runtime.loader import load_engine

    path = write_synthetic_gguf(str(tmp_path / "ms.gguf"), get_preset("test-mistral-shape"), "Q4_K_M", seed=9)
    eng, cfg, _ = load_engine(path, max_ctx=256)
    assert eng.mk_available
    eng.mk_enabled = True
    ref = ReferenceModel.from_gguf(path, kv_bf16=True, act_q8=True)
    prompt = [1, 30, 40, 50, 60, 70, 80]
    n = 10
    seq = prompt + ref.greedy(prompt, n)
    rl = ref.forward(seq)
    eng.prefill(0, prompt, 0, False)
    for i in range(n):
        p = len(prompt) + i
        eng.decode([0], [seq[p]], [p])
        el = torch.from_numpy(np.asarray(eng.last_logits(1)).reshape(-1))
        err = (el - rl[p]).abs().max().item()
        assert err < 2e-2 * max(1.0, rl[p].abs().max().item()), (i, err)
