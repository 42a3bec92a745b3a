"""The routing candidates' families on the CPU: synthetic Qwen3 / Llama-3 GGUFs carry their real
tokenizer kind (byte-level BPE with ranked merges, 151,936 / 128,256 tokens, control tokens at
the real ids) and architecture keys; they load into the tokenizer, the config and the fp32
reference model (GPU engine numerics: test_model_families_gpu.py)."""
import pytest

from aios_amd.gguf.reader import GGUFReader
from aios_amd.models.config import ModelConfig, get_preset
from aios_amd.models.synthetic import write_synthetic_gguf
from aios_amd.runtime.tokenizer import Gpt2Tokenizer, from_gguf


@pytest.fixture(scope="module", params=["test-qwen3-shape", "test-llama3-shape"])
def fam(request, tmp_path_factory):
    cfg = get_preset(request.param)
    p = write_synthetic_gguf(str(tmp_path_factory.mktemp("fam") / f"{cfg.name}.gguf"), cfg, "Q4_K_M", seed=2)
    return cfg, p


def test_family_gguf_roundtrip(fam):
    cfg, path = fam
    r = GGUFReader(path)
    c2 = ModelConfig.from_gguf(r)
    assert (c2.vocab_size, c2.qk_norm, c2.rope_mode, c2.tokenizer_model) == \
        (cfg.vocab_size, cfg.qk_norm, cfg.rope_mode, "gpt2")
    tok = from_gguf(r)
    assert isinstance(tok, Gpt2Tokenizer) and tok.vocab_size == cfg.vocab_size
    text = "the agent checked the system status and wrote json"
    ids = tok.encode(text, add_bos=False)
    assert tok.decode(ids) == text
    assert len(ids) < len(text.encode()) // 2  # merges applied: whole words, not bytes
    assert tok.tokens[cfg.eos_id] in ("<|eot_id|>", "<|im_end|>")


def test_family_reference_model_runs(fam):
    from aios_amd.models.reference import ReferenceModel

    cfg, path = fam
    ref = ReferenceModel.from_gguf(path)
    out = ref.greedy([5, 6, 7, 300], 3)
    assert len(out) == 3 and all(0 <= t < cfg.vocab_size for t in out)
