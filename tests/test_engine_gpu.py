"""GPU end-to-end: native engine vs the fp32 reference model on synthetic GGUF checkpoints."""
import time

import numpy as np
import pytest
import torch

from aios_amd.models.config import get_preset
from aios_amd.models.reference import ReferenceModel
from aios_amd.models.synthetic import write_synthetic_gguf

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def model_files(tmp_path_factory):
    d = tmp_path_factory.mktemp("eng")
    out = {}
    for recipe in ("Q4_K_M", "Q4_0", "Q8_0", "BF16", "Q5_K_M", "Q3_K_M", "Q2_K", "Q4_1", "Q5_0", "Q5_1", "IQ4_NL", "IQ4_XS"):
        out[recipe] = write_synthetic_gguf(str(d / f"small_{recipe}.gguf"), get_preset("test-small"), recipe, seed=7)
    out["mistral_shape"] = write_synthetic_gguf(str(d / "ms.gguf"), get_preset("test-mistral-shape"), "Q4_K_M", seed=9)
    return out


def _load(path, **kw):
    from aios_amd.runtime.loader import load_engine

    eng, cfg, r = load_engine(path, max_ctx=256, **kw)
    return eng, cfg


@pytest.mark.parametrize("recipe", ["Q4_K_M", "Q4_0", "Q8_0", "BF16", "mistral_shape"])
@pytest.mark.parametrize("q8", [False, True])
def test_prefill_logits_match_reference(model_files, recipe, q8):
    path = model_files[recipe]
    eng, cfg = _load(path, act_q8=q8)
    ref = ReferenceModel.from_gguf(path, kv_bf16=True, act_q8=q8)
    prompt = [1] + list(np.random.default_rng(0).integers(3, cfg.vocab_size, 40))
    logits = torch.from_numpy(np.asarray(eng.prefill(0, prompt, 0, True)))
    rl = ref.forward(prompt)[-1]
    err = (logits - rl).abs().max().item()
    scale = rl.abs().max().item()
    assert err < 2e-2 * max(scale, 1.0), (err, scale)


@pytest.mark.parametrize("recipe", ["Q3_K_M", "Q2_K", "Q4_1", "Q5_0", "Q5_1", "IQ4_NL", "IQ4_XS"])
def test_load_time_expanded_formats_match_reference(model_files, recipe):
    """Q2_K / Q3_K (and the legacy Q4_1 / Q5_0 / Q5_1) matrices are expanded to bf16 on the GPU at load
    (quant_pack.hip legacy_to_bf16_kernel): prefill logits against the fp32 reference over the host
    dequantisation of the same blocks (quants.py; the engine's copy is that, rounded to bf16), then a few
    decode steps with finite logits"""
    path = model_files[recipe]
    eng, cfg = _load(path, act_q8=False)
    ref = ReferenceModel.from_gguf(path, kv_bf16=True, act_q8=False)
    prompt = [1] + list(np.random.default_rng(0).integers(3, cfg.vocab_size, 40))
    logits = torch.from_numpy(np.asarray(eng.prefill(0, prompt, 0, True)))
    rl = ref.forward(prompt)[-1]
    err, scale = (logits - rl).abs().max().item(), rl.abs().max().item()
    assert err < 2e-2 * max(scale, 1.0), (err, scale)
    tok, pos = int(torch.argmax(logits)), len(prompt)
    for _ in range(4):
        tok = eng.decode([0], [tok], [pos])[0]
        pos += 1
        assert 0 <= tok < cfg.vocab_size


@pytest.mark.parametrize("recipe", ["Q4_K_M", "BF16"])
@pytest.mark.parametrize("q8", [False, True])
def test_greedy_decode_token_exact(model_files, recipe, q8):
    path = model_files[recipe]
    eng, cfg = _load(path, act_q8=q8)
    ref = ReferenceModel.from_gguf(path, kv_bf16=True, act_q8=q8)
    prompt = [1, 30, 40, 50, 60, 70, 80]
    n = 12
    want = ref.greedy(prompt, n)
    logits = np.asarray(eng.prefill(0, prompt, 0, True))
    tok = int(np.argmax(logits))
    got = [tok]
    pos = len(prompt)
    for _ in range(n - 1):
        tok = eng.decode([0], [tok], [pos])[0]
        pos += 1
        got.append(tok)
    assert got == want


@pytest.mark.parametrize("recipe", ["Q4_K_M", "mistral_shape"])
@pytest.mark.parametrize("gemm_prefill", ["0", "1"])
def test_fp8_kv_cache_matches_reference(model_files, monkeypatch, recipe, gemm_prefill):
    """the fp8 e4m3 KV cache (kv_dtype='fp8_e4m3', per-layer K / V scales) against the
    fp32 reference model with the same fp8 rounding of K / V (fp32 GEMV activations on both sides, so
    the KV cache is the only approximation): prefill logits (GEMV and MFMA prefill paths, 70-token
    prompt) within the bf16-KV tolerance; the fp8 cache's own error against the bf16-KV engine within 5 %
    of the logit scale; 64 teacher-forced decode steps (the reference's greedy tokens fed back, so one
    near-tie does not cascade) with every step's logits within tolerance and >= 62 of 63 argmaxes equal."""
    from aios_amd.runtime.loader import load_engine

    monkeypatch.setenv("AIOS_PREFILL_GEMM", gemm_prefill)
    path = model_files[recipe]
    eng, cfg, _ = load_engine(path, max_ctx=256, kv_dtype="fp8_e4m3", act_q8=False)
    assert eng.kv_fp8 == 1 and len(eng.kv_scales) == 2 * cfg.n_layers
    scales = [0.05 if i % 2 == 0 else 0.02 for i in range(2 * cfg.n_layers)]
    eng.set_kv_scales(scales)
    ref = ReferenceModel.from_gguf(path, kv_fp8=True, kv_scales=scales)
    prompt = [1] + list(np.random.default_rng(3).integers(3, cfg.vocab_size, 69))
    logits = torch.from_numpy(np.asarray(eng.prefill(0, prompt, 0, True)))
    rl = ref.forward(prompt)[-1]
    sc = rl.abs().max().item()
    assert (logits - rl).abs().max().item() < 2e-2 * max(sc, 1.0)
    bf, _, _ = load_engine(path, max_ctx=256, act_q8=False)
    lb = torch.from_numpy(np.asarray(bf.prefill(0, prompt, 0, True)))
    assert (logits - lb).abs().max().item() < 5e-2 * max(sc, 1.0)
    # 64 decode steps, teacher-forced with the fp8-emulating reference's greedy tokens
    want = ref.greedy(prompt[:8], 64)
    assert int(np.argmax(np.asarray(eng.prefill(1, prompt[:8], 0, True)))) == want[0]
    ctx = list(prompt[:8])
    agree, worst = 0, 0.0
    for i in range(63):
        eng.decode([1], [want[i]], [8 + i])
        el = torch.from_numpy(np.asarray(eng.last_logits(1))[0])
        ctx.append(want[i])
        rl = ref.forward(ctx)[-1]
        worst = max(worst, (el - rl).abs().max().item() / max(rl.abs().max().item(), 1.0))
        agree += int(el.argmax()) == want[i + 1]
    assert worst < 2e-2 and agree >= 62, (worst, agree)


def test_batched_decode_matches_single(model_files):
    path = model_files["Q4_K_M"]
    eng, cfg = _load(path, max_slots=4, max_batch=4)
    prompts = [[1, 5, 6, 7], [1, 9, 10, 11, 12, 13], [1, 100, 200]]
    firsts, poss = [], []
    for s, p in enumerate(prompts):
        firsts.append(int(np.argmax(eng.prefill(s, p, 0, True))))
        poss.append(len(p))
    # batched step
    toks = eng.decode([0, 1, 2], firsts, poss)
    # single steps on fresh copies (slot 3) must agree
    for s, p in enumerate(prompts):
        eng.prefill(3, p, 0, False)
        t = eng.decode([3], [firsts[s]], [poss[s]])[0]
        assert t == toks[s]


def test_graph_loop_matches_eager(model_files):
    path = model_files["Q4_K_M"]
    eng, cfg = _load(path, max_slots=2, max_batch=2)
    prompt = [1, 42, 43, 44]
    first = int(np.argmax(eng.prefill(0, prompt, 0, True)))
    eng.prefill(1, prompt, 0, False)
    n = 10
    eng.decode_loop_prepare([0], [first], [len(prompt)])
    eng.decode_loop_run(1, n, True)
    g = eng.decode_loop_history(1, len(prompt) + 1, n)
    eng.decode_loop_prepare([1], [first], [len(prompt)])
    eng.decode_loop_run(1, n, False)
    e = eng.decode_loop_history(1, len(prompt) + 1, n)
    assert list(g) == list(e)


def test_capture_graphs_precaptures_every_batch_size(model_files):
    """capture_graphs(max_b) captures (without running) the masked and unmasked step graph of every
    B; later decode calls replay them and give the same tokens as a fresh engine's lazily captured
    graphs."""
    path = model_files["Q4_K_M"]
    prompts = [[1, 5, 6, 7], [1, 9, 10, 11, 12, 13], [1, 100, 200]]
    outs = []
    for pre in (False, True):
        eng, cfg = _load(path, max_slots=4, max_batch=4)
        if pre:
            # 4 B x (masked, unmasked) step graphs + the pipelined decode's 4 forward graphs
            assert eng.capture_graphs(4) == 12
            assert eng.capture_graphs(4) == 12  # idempotent
        firsts = [int(np.argmax(eng.prefill(s, p, 0, True))) for s, p in enumerate(prompts)]
        outs.append(eng.decode([0, 1, 2], firsts, [len(p) for p in prompts]))
        del eng
    assert outs[0] == outs[1]


def test_random_init_engine_runs():
    from aios_amd.runtime.loader import random_engine

    eng = random_engine(get_preset("test-mistral-shape"), "Q4_K_M", seed=1, max_ctx=256, max_batch=2)
    logits = np.asarray(eng.prefill(0, [1, 2, 3, 4], 0, True))
    assert np.isfinite(logits).all()
    eng.decode_loop_prepare([0], [5], [4])
    eng.decode_loop_run(1, 8, True)
    eng.synchronize()
    h = eng.decode_loop_history(1, 5, 8)
    assert all(0 <= t < 1024 for t in h)


@pytest.mark.parametrize("recipe", ["Q4_K_M", "mistral_shape"])
def test_prefill_gemm_chunks_match_reference(model_files, recipe, monkeypatch):
    # 64-row GEMM chunks: a 150-token prompt crosses two chunk boundaries (flash attention over
    # the previous chunks' cached keys), and a prefill continued at start_pos > 0 matches too
    monkeypatch.setenv("AIOS_PREFILL_GEMM_ROWS", "64")
    path = model_files[recipe]
    eng, cfg = _load(path)
    ref = ReferenceModel.from_gguf(path, kv_bf16=True)
    prompt = [1] + list(np.random.default_rng(3).integers(3, cfg.vocab_size, 149))
    rl = ref.forward(prompt)[-1]
    logits = torch.from_numpy(np.asarray(eng.prefill(0, prompt, 0, True)))
    scale = max(rl.abs().max().item(), 1.0)
    assert (logits - rl).abs().max().item() < 2e-2 * scale
    eng.prefill(1, prompt[:100], 0, False)
    logits2 = torch.from_numpy(np.asarray(eng.prefill(1, prompt[100:], 100, True)))
    assert (logits2 - rl).abs().max().item() < 2e-2 * scale


@pytest.mark.parametrize("recipe", ["Q4_K_M", "mistral_shape", "Q5_K_M", "Q4_0", "Q8_0"])
@pytest.mark.parametrize("tile", ["", "256x256", "128x256", "64x128"])
def test_prefill_gemm_pf_chunks_match_reference(model_files, recipe, tile, monkeypatch):
    """prefill chunks on the hand-written prefill GEMM (kernels/gemm_pf.hip, M >= 33): 64-row chunks of
    a 150-token prompt -- two 64-row chunks on gemm_pf (each tile shape), the 22-row tail on the ring
    GEMM -- against the fp32 reference, continued at start_pos > 0 too (round 6: the Q5_K_M / Q4_0 / Q8_0
    recipes' stacks as well, on the pf4 / pf8 bodies)"""
    monkeypatch.setenv("AIOS_PREFILL_GEMM_ROWS", "64")
    if tile:
        monkeypatch.setenv("AIOS_GEMM_PF_TILE", tile)
    path = model_files[recipe]
    eng, cfg = _load(path)
    ref = ReferenceModel.from_gguf(path, kv_bf16=True)
    prompt = [1] + list(np.random.default_rng(5).integers(3, cfg.vocab_size, 149))
    rl = ref.forward(prompt)[-1]
    logits = torch.from_numpy(np.asarray(eng.prefill(0, prompt, 0, True)))
    scale = max(rl.abs().max().item(), 1.0)
    assert (logits - rl).abs().max().item() < 2e-2 * scale
    eng.prefill(1, prompt[:70], 0, False)
    logits2 = torch.from_numpy(np.asarray(eng.prefill(1, prompt[70:], 70, True)))
    assert (logits2 - rl).abs().max().item() < 2e-2 * scale


@pytest.mark.parametrize("T", [3, 4, 5, 8, 15])
@pytest.mark.parametrize("q8", [False, True])
def test_short_prompt_prefill_matches_reference(model_files, monkeypatch, T, q8):
    """2-4-token prompts go through the batched LDS-DMA GEMV engine (B = T rows), 5-15-token ones
    through the skinny MFMA GEMM (gm_min_rows_ = 5): their logits against the fp32 reference for both
    GEMV activation settings (the decode steps' precision differs from the GEMM's bf16 operands; the
    reference bounds both)"""
    monkeypatch.setenv("AIOS_PREFILL_GEMM", "1")
    path = model_files["mistral_shape"]
    eng, cfg = _load(path, act_q8=q8)
    ref = ReferenceModel.from_gguf(path, kv_bf16=True, act_q8=q8)
    prompt = [1] + list(np.random.default_rng(T).integers(3, cfg.vocab_size, T - 1))
    logits = torch.from_numpy(np.asarray(eng.prefill(0, prompt, 0, True)))
    rl = ref.forward(prompt)[-1]
    assert (logits - rl).abs().max().item() < 2e-2 * max(rl.abs().max().item(), 1.0)


@pytest.mark.parametrize("recipe", ["Q4_K_M", "mistral_shape"])
@pytest.mark.parametrize("fuse", ["0", "1"])
def test_short_chunk_prefill_fusions_match_reference(model_files, monkeypatch, recipe, fuse):
    """chunks of <= 64 rows take the decode step's fusions (RoPE + KV write in the QKV GEMM epilogue,
    split RMSNorm through the residual GEMMs, AIOS_PREFILL_SHORT_FUSE): a 30-token prompt in one chunk
    and its continuation at start_pos 30 (34 more rows: the hand-written prefill GEMM's
    smallest M window, 33..64 rows), then the whole 64-token prompt, against the fp32 reference, fused and not"""
    monkeypatch.setenv("AIOS_PREFILL_GEMM", "1")
    monkeypatch.setenv("AIOS_PREFILL_SHORT_FUSE", fuse)
    path = model_files[recipe]
    eng, cfg = _load(path, max_batch=1)
    ref = ReferenceModel.from_gguf(path, kv_bf16=True)
    prompt = [1] + list(np.random.default_rng(11).integers(3, cfg.vocab_size, 63))
    rl = ref.forward(prompt)[-1]
    scale = max(rl.abs().max().item(), 1.0)
    eng.prefill(0, prompt[:30], 0, False)
    logits = torch.from_numpy(np.asarray(eng.prefill(0, prompt[30:], 30, True)))
    assert (logits - rl).abs().max().item() < 2e-2 * scale
    logits1 = torch.from_numpy(np.asarray(eng.prefill(1, prompt, 0, True)))
    assert (logits1 - rl).abs().max().item() < 2e-2 * scale


def test_prefill_gemm_vs_gemv_path(model_files, monkeypatch):
    path = model_files["Q4_K_M"]
    prompt = [1] + list(np.random.default_rng(4).integers(3, 200, 60))
    monkeypatch.setenv("AIOS_PREFILL_GEMM", "0")
    e1, _ = _load(path)
    l1 = np.asarray(e1.prefill(0, prompt, 0, True))
    del e1
    monkeypatch.setenv("AIOS_PREFILL_GEMM", "1")
    e2, _ = _load(path)
    l2 = np.asarray(e2.prefill(0, prompt, 0, True))
    assert np.abs(l1 - l2).max() < 2e-2 * max(np.abs(l1).max(), 1.0)


@pytest.mark.parametrize("B", [2, 3, 4])
@pytest.mark.parametrize("graph", [False, True])
def test_batched_decode_gemm_path_matches_gemv_path(model_files, monkeypatch, B, graph):
    """B >= AIOS_DECODE_GEMM_MIN_B runs the projections through the skinny MFMA GEMM (split-K
    slabs reduced in-launch, SwiGLU in the gate/up epilogue, residual accumulate in O/down); its
    logits must match the fp32-activation GEMV path's for the same batch, eager and replayed from
    the captured decode graph."""
    path = model_files["Q4_K_M"]
    prompts = [[1, 5, 6, 7], [1, 9, 10, 11, 12, 13], [1, 100, 200], [1, 3, 4]][:B]
    outs = {}
    for mode, min_b in (("gemv", "0"), ("gemm", "2")):
        monkeypatch.setenv("AIOS_DECODE_GEMM_MIN_B", min_b)
        eng, cfg = _load(path, max_slots=4, max_batch=4, act_q8=False)
        firsts = [int(np.argmax(eng.prefill(s, p, 0, True))) for s, p in enumerate(prompts)]
        if graph:
            eng.decode_loop_prepare(list(range(B)), firsts, [len(p) for p in prompts])
            eng.decode_loop_run(B, 3, True)
            toks = None
        else:
            toks = eng.decode(list(range(B)), firsts, [len(p) for p in prompts])
        outs[mode] = (toks, np.asarray(eng.last_logits(B)).reshape(B, -1))
        del eng
    l0, l1 = outs["gemv"][1], outs["gemm"][1]
    scale = max(np.abs(l0).max(), 1.0)
    assert np.abs(l0 - l1).max() < 2e-2 * scale


@pytest.mark.parametrize("B", [2, 3, 4])
def test_batched_int8_gemv_engine_matches_single_rows(model_files, monkeypatch, B):
    """B = 2..4 on the int8-activation path: every projection through the LDS-DMA GEMV engine
    serving the B rows from ONE weight stream (kernels/gemv_lds.h, B-row consumers); each row's
    logits must equal that sequence decoded alone (B = 1 engine) up to fp32 summation order."""
    monkeypatch.setenv("AIOS_DECODE_GEMM_MIN_B", "0")
    path = model_files["Q4_K_M"]
    prompts = [[1, 5, 6, 7], [1, 9, 10, 11, 12, 13], [1, 100, 200], [1, 3, 4]][:B]
    eng, cfg = _load(path, max_slots=4, max_batch=4, act_q8=True)
    firsts = [int(np.argmax(eng.prefill(s, p, 0, True))) for s, p in enumerate(prompts)]
    toks = eng.decode(list(range(B)), firsts, [len(p) for p in prompts])
    batched = np.asarray(eng.last_logits(B)).reshape(B, -1)
    del eng
    for b in range(B):
        e1, _ = _load(path, max_slots=4, max_batch=4, act_q8=True)
        f = int(np.argmax(e1.prefill(0, prompts[b], 0, True)))
        assert f == firsts[b]
        t1 = e1.decode([0], [f], [len(prompts[b])])
        single = np.asarray(e1.last_logits(1)).reshape(-1)
        del e1
        assert t1[0] == toks[b]
        assert np.abs(single - batched[b]).max() < 2e-3 * max(np.abs(single).max(), 1.0)


@pytest.mark.parametrize("recipe,rb,split", [("Q4_K_M", "0", "0"), ("Q4_K_M", "4", "1"),
                                             ("mistral_shape", "0", "1"), ("mistral_shape", "4", "0")])
def test_batched_decode_split_rmsnorm_matches_explicit(model_files, monkeypatch, recipe, rb, split):
    """AIOS_GEMM_NORM_FUSE: the residual GEMMs (O, down) emit bf16(x * g_next) plus per-tile row
    sums of squares and the next GEMM scales its rows by the inverse RMS -- the explicit
    normalisation launches' result to bf16 rounding, with the reduction tiles over 4..16 parts
    (AIOS_SKINNY_RB) on both the split-K last-arriver and the one-slice epilogue (AIOS_SKINNY_S)."""
    monkeypatch.setenv("AIOS_DECODE_GEMM_MIN_B", "2")
    monkeypatch.setenv("AIOS_SKINNY_RB", rb)
    if split == "1":
        monkeypatch.setenv("AIOS_SKINNY_S", "1")
    path = model_files[recipe]
    B = 4
    prompts = [[1, 5, 6, 7], [1, 9, 10, 11, 12, 13], [1, 100, 200], [1, 3, 4]]
    outs = {}
    for fuse in ("0", "1"):
        monkeypatch.setenv("AIOS_GEMM_NORM_FUSE", fuse)
        eng, cfg = _load(path, max_slots=4, max_batch=4, act_q8=False)
        want_parts = cfg.d_model // (16 * (4 if rb == "4" else 8)) if fuse == "1" else 0
        assert eng.norm_fused_parts == want_parts
        firsts = [int(np.argmax(eng.prefill(s, p, 0, True))) for s, p in enumerate(prompts)]
        eng.decode_loop_prepare(list(range(B)), firsts, [len(p) for p in prompts])
        eng.decode_loop_run(B, 3, True)
        outs[fuse] = np.asarray(eng.last_logits(B)).reshape(B, -1)
        del eng
    l0, l1 = outs["0"], outs["1"]
    assert np.isfinite(l1).all()
    assert np.abs(l0 - l1).max() < 1e-2 * max(np.abs(l0).max(), 1.0)


@pytest.mark.parametrize("recipe", ["Q4_K_M", "mistral_shape"])
def test_batched_decode_mixed_format_qkv_launch(model_files, monkeypatch, recipe):
    """AIOS_SKINNY_MIXED: the Q4_K_M QKV stack (Q|K Q4_K, V Q6_K) as ONE skinny launch whose V
    tiles run the Q6_K body -- the same logits as one launch per format."""
    monkeypatch.setenv("AIOS_DECODE_GEMM_MIN_B", "2")
    path = model_files[recipe]
    B = 4
    prompts = [[1, 5, 6, 7], [1, 9, 10, 11, 12, 13], [1, 100, 200], [1, 3, 4]]
    outs = {}
    for mixed in ("0", "1"):
        monkeypatch.setenv("AIOS_SKINNY_MIXED", mixed)
        eng, cfg = _load(path, max_slots=4, max_batch=4, act_q8=False)
        firsts = [int(np.argmax(eng.prefill(s, p, 0, True))) for s, p in enumerate(prompts)]
        eng.decode_loop_prepare(list(range(B)), firsts, [len(p) for p in prompts])
        eng.decode_loop_run(B, 3, True)
        outs[mixed] = np.asarray(eng.last_logits(B)).reshape(B, -1)
        del eng
    assert np.abs(outs["0"] - outs["1"]).max() < 1e-3 * max(np.abs(outs["0"]).max(), 1.0)


@pytest.mark.parametrize("recipe", ["Q4_K_M", "mistral_shape"])
def test_prefill_one_chunk_matches_reference(model_files, recipe):
    """A 140-token prompt prefills as ONE GEMM chunk (big-M MFMA kernel, dequant fused; no bf16
    weight copy exists) and matches the fp32 reference."""
    path = model_files[recipe]
    ref = ReferenceModel.from_gguf(path, kv_bf16=True)
    prompt = [1] + list(np.random.default_rng(5).integers(3, 200, 140))
    rl = ref.forward(prompt)[-1]
    scale = max(rl.abs().max().item(), 1.0)
    eng, cfg = _load(path)
    got = torch.from_numpy(np.asarray(eng.prefill(0, prompt, 0, True)))
    assert (got - rl).abs().max().item() < 2e-2 * scale


@pytest.mark.parametrize("gemm_prefill", ["0", "1"])
def test_paged_kv_prefix_sharing_and_copy_on_write(model_files, monkeypatch, gemm_prefill):
    """Paged KV: slot 1 inherits slot 0's first 300 tokens (two full 128-token blocks shared by
    reference, the partial third block copied), prefills only its own suffix, and its logits and
    greedy continuation equal a fresh full prefill of the same prompt in slot 2.  Then slot 0 is
    re-prefilled from position 100 -- inside a shared block -- which must un-share (copy-on-write)
    instead of corrupting slot 1."""
    monkeypatch.setenv("AIOS_PREFILL_GEMM", gemm_prefill)
    path = model_files["mistral_shape"]
    from aios_amd.runtime.loader import load_engine

    eng, cfg, _ = load_engine(path, max_ctx=512, max_slots=4, max_batch=2, act_q8=False)
    rng = np.random.default_rng(11)
    a = [1] + [int(t) for t in rng.integers(3, 900, 399)]
    b = a[:300] + [int(t) for t in rng.integers(3, 900, 60)]
    total = eng.kv_blocks_total
    eng.prefill(0, a, 0, False)
    assert eng.kv_blocks_free == total - 4  # 400 tokens -> 4 blocks
    eng.copy_slot(0, 1, 300)
    t0, t1 = eng.block_table(0), eng.block_table(1)
    assert t1[:2] == t0[:2] and t1[2] not in t0 and t1[3] == -1
    lb = np.asarray(eng.prefill(1, b[300:], 300, True))
    lf = np.asarray(eng.prefill(2, b, 0, True))
    scale = max(np.abs(lf).max(), 1.0)
    assert np.abs(lb - lf).max() < 2e-2 * scale
    # greedy continuation of the shared-prefix slot and the fresh slot, batched in one step
    nb = int(np.argmax(lb))
    toks = eng.decode([1, 2], [nb, nb], [len(b), len(b)])
    l2 = np.asarray(eng.last_logits(2)).reshape(2, -1)
    assert np.abs(l2[0] - l2[1]).max() < 2e-2 * scale
    # copy-on-write: rewriting slot 0 from position 100 must not touch slot 1's shared blocks
    c = a[:100] + [int(t) for t in rng.integers(3, 900, 50)]
    eng.prefill(0, c[100:], 100, False)
    assert eng.block_table(0)[0] != eng.block_table(1)[0]
    eng.decode([1, 2], [int(toks[0]), int(toks[1])], [len(b) + 1, len(b) + 1])
    l3 = np.asarray(eng.last_logits(2)).reshape(2, -1)
    assert np.abs(l3[0] - l3[1]).max() < 2e-2 * scale
    eng.release_slot(0)
    eng.release_slot(1)
    eng.release_slot(2)
    assert eng.kv_blocks_free == total


def test_per_row_seeds_are_row_independent(model_files):
    """a row's sample depends on (its seed, its position), not on its batch row (verdict r2 #7)"""
    eng, cfg = _load(model_files["Q4_K_M"], max_slots=4, max_batch=4)
    prompt = [1, 5, 6, 7]
    for s in range(3):
        eng.prefill(s, prompt, 0, False)
    t = int(np.argmax(eng.prefill(3, prompt, 0, True)))
    a = eng.decode([0, 1], [t, t], [4, 4], [1.0, 1.0], [0, 0], 0, b"", [1.0, 1.0], [77, 5])
    b = eng.decode([2, 0], [t, t], [4, 4], [1.0, 1.0], [0, 0], 0, b"", [1.0, 1.0], [5, 77])
    assert a[0] == b[1] and a[1] == b[0]
    draws = {eng.decode([0], [t], [4], [1.0], [0], 0, b"", [1.0], [s])[0] for s in range(1, 30)}
    assert len(draws) > 1


def test_sample_first_on_device(model_files):
    eng, cfg = _load(model_files["Q4_K_M"], max_slots=2, max_batch=2)
    logits = np.asarray(eng.prefill(0, [1, 9, 10, 11], 0, True))
    assert eng.sample_first(3, 0.0, 0, 1.0, 5) == int(np.argmax(logits))  # T = 0: greedy
    x = eng.sample_first(3, 1.0, 0, 1.0, 1234)
    assert x == eng.sample_first(3, 1.0, 0, 1.0, 1234)
    assert len({eng.sample_first(3, 1.0, 0, 1.0, s) for s in range(1, 30)}) > 1




_PLAN_PROC = r"""
import json, sys, numpy as np
from aios_amd.models.config import get_preset
from aios_amd.runtime import native
from aios_amd.runtime.loader import random_engine
eng = random_engine(get_preset("test-mistral-shape"), "Q4_K_M", seed=3, max_ctx=512, max_batch=2)
prompt = [1] + list(np.random.default_rng(5).integers(3, 1024, 299))
np.save(sys.argv[1], np.asarray(eng.prefill(0, [int(t) for t in prompt], 0, True), dtype=np.float32))
print(json.dumps(sorted(native.require().gemm_pf_export())))
"""


@pytest.mark.parametrize("deterministic", [False, True])
def test_prefill_plans_persist_across_processes(tmp_path, deterministic):
    """with AIOS_GEMM_PF_PLANS naming a file, a second process installs the first's
    tuned prefill-GEMM plans instead of timing its own (the same plan list in both).  Split-K / stream-K
    plans add partial tiles with fp32 atomics in arrival order, so their last bits may still differ:
    the logits agree to float rounding and on the argmax; AIOS_GEMM_PF_DETERMINISTIC=1 keeps those plans
    out, and the two processes' prefill logits are then bit-identical."""
    import json
    import os
    import subprocess
    import sys

    env = dict(os.environ, AIOS_GEMM_PF_PLANS=str(tmp_path / "plans.json"))
    if deterministic:
        env["AIOS_GEMM_PF_DETERMINISTIC"] = "1"
    outs, plans = [], []
    for i in range(2):
        out = tmp_path / f"logits{i}.npy"
        r = subprocess.run([sys.executable, "-c", _PLAN_PROC, str(out)], env=env, capture_output=True, text=True,
                           timeout=240, cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        assert r.returncode == 0, r.stderr[-2000:]
        plans.append(json.loads(r.stdout.strip().splitlines()[-1]))
        outs.append(np.load(out))
    assert (tmp_path / "plans.json").exists() and plans[0] and plans[1] == plans[0]
    assert np.isfinite(outs[0]).all() and int(np.argmax(outs[0])) == int(np.argmax(outs[1]))
    if deterministic:
        assert np.array_equal(outs[0], outs[1])
    else:
        assert np.allclose(outs[0], outs[1], rtol=1e-4, atol=1e-5)
