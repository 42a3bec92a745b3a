"""CPU tests: GGUF reader/writer and synthetic model generation."""
import numpy as np
import pytest

from aios_amd.gguf.quants import GGMLType, dequantize, quantize
from aios_amd.gguf.reader import GGUFReader, GGUFWriter
from aios_amd.models.config import ModelConfig, get_preset
from aios_amd.models.synthetic import synthetic_vocab, write_synthetic_gguf


def test_roundtrip(tmp_path):
    p = str(tmp_path / "a.gguf")
    w = GGUFWriter(p)
    w.add("general.architecture", "llama")
    w.add("llama.block_count", 3)
    w.add("some.float", 1.5)
    w.add("some.list", ["a", "bc"])
    w.add("some.arr", np.arange(5, dtype=np.int32))
    x = np.random.default_rng(0).standard_normal((4, 256)).astype(np.float32)
    w.add_tensor("t.q4k", (256, 4), GGMLType.Q4_K, quantize(x, GGMLType.Q4_K))
    w.add_tensor("t.f32", (7,), GGMLType.F32, np.arange(7, dtype=np.float32).view(np.uint8))
    w.write()
    r = GGUFReader(p)
    assert r.get("llama.block_count") == 3
    assert abs(r.get("some.float") - 1.5) < 1e-6
    assert r.get("some.list") == ["a", "bc"]
    assert list(r.get("some.arr")) == [0, 1, 2, 3, 4]
    assert r.tensors["t.q4k"].shape == (256, 4)
    assert r.tensors["t.q4k"].rows == 4 and r.tensors["t.q4k"].cols == 256
    y = r.dequantize("t.q4k")
    assert y.shape == (4, 256)
    assert np.allclose(y, dequantize(quantize(x, GGMLType.Q4_K), GGMLType.Q4_K).reshape(4, 256))
    assert np.array_equal(r.dequantize("t.f32"), np.arange(7, dtype=np.float32))
    assert r.data_offset % 32 == 0
    r.close()


def test_synthetic_model(tmp_path):
    cfg = get_preset("test-tiny")
    p = write_synthetic_gguf(str(tmp_path / "m.gguf"), cfg, "Q4_K_M")
    r = GGUFReader(p)
    c2 = ModelConfig.from_gguf(r)
    assert (c2.d_model, c2.n_layers, c2.n_heads, c2.n_kv_heads, c2.head_dim, c2.d_ff) == (256, 2, 4, 2, 64, 512)
    assert r.tensors["output.weight"].ggml_type == GGMLType.Q6_K
    assert r.tensors["blk.1.ffn_down.weight"].ggml_type == GGMLType.Q6_K  # last 1/8 of layers: more bits
    assert r.tensors["blk.0.attn_q.weight"].ggml_type == GGMLType.Q4_K
    assert len(r.get("tokenizer.ggml.tokens")) == cfg.vocab_size
    r.close()


def test_vocab_has_bytes_and_ascii():
    toks, scores, types = synthetic_vocab(2000)
    assert len(toks) == 2000 and toks[3] == "<0x00>" and types[3] == 6
    assert "{" in toks and '"' in toks and "▁the" in toks


@pytest.mark.parametrize("recipe,tol", [("Q5_1", 0.08), ("Q5_0", 0.1), ("Q4_1", 0.15), ("Q3_K_M", 0.3), ("Q2_K", 0.5),
                                        ("IQ4_NL", 0.15), ("IQ4_XS", 0.15)])
def test_low_bit_and_legacy_recipes_run(tmp_path, recipe, tol):
    """GGUF files in the legacy 32-block formats and the 2- / 3-bit K-quant mixes (expanded to bf16 by the
    GPU loader; dequantised exactly by the CPU engine's reference forward): the same random weights as an
    F32 file give logits within the format's quantisation error and the same argmax"""
    from aios_amd.models.config import get_preset
    from aios_amd.models.reference import ReferenceModel
    from aios_amd.models.synthetic import write_synthetic_gguf

    cfg = get_preset("test-small")
    prompt = [1] + list(range(5, 40))
    lg = {}
    for r in ("F32", recipe):
        m = ReferenceModel.from_gguf(write_synthetic_gguf(str(tmp_path / f"m_{r}.gguf"), cfg, r, seed=7))
        lg[r] = m.forward(prompt)[-1].numpy()
    rel = np.linalg.norm(lg[recipe] - lg["F32"]) / np.linalg.norm(lg["F32"])
    assert rel < tol and int(np.argmax(lg[recipe])) == int(np.argmax(lg["F32"])), rel
