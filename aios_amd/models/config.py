"""Model architecture configs for the Llama-family decoders the runtime serves.

Reference roles:
  * TinyLlama-1.1B-Chat   — operational tier (`scripts/download-models.sh:70-72`)
  * Mistral-7B-Instruct   — tactical tier    (`scripts/download-models.sh:75-77`)
  * Qwen3-8B / Qwen3-14B  — tactical/strategic routing candidates
                             (`runtime/src/model_manager.rs:471-492`)
  * Llama-3-70B           — local strategic tier, TP=8 (BASELINE.json config 5)

At load time the values are read from the GGUF metadata (`from_gguf`); the
presets here are used to emit random-init synthetic GGUF files of the named
shapes (no network: checkpoints cannot be downloaded).
"""
from __future__ import annotations

import dataclasses
from typing import Dict, Optional

from ..gguf.quants import GGMLType

ROPE_NORM = 0   # llama/mistral GGUF: adjacent pairs (x[2i], x[2i+1]) (converter pre-permutes Q/K)
ROPE_NEOX = 2   # qwen: (x[i], x[i + rot/2])


@dataclasses.dataclass
class ModelConfig:
    name: str
    arch: str = "llama"
    vocab_size: int = 32000
    d_model: int = 2048
    n_layers: int = 22
    n_heads: int = 32
    n_kv_heads: int = 4
    head_dim: int = 64
    d_ff: int = 5632
    rope_theta: float = 10000.0
    rope_mode: int = ROPE_NORM
    norm_eps: float = 1e-5
    max_ctx: int = 2048
    tie_embeddings: bool = False
    qk_norm: bool = False          # Qwen3
    qkv_bias: bool = False         # Qwen2
    bos_id: int = 1
    eos_id: int = 2
    tokenizer_model: str = "llama"  # "llama" (SPM) or "gpt2" (byte-level BPE)
    chat_template: str = "zephyr"

    @property
    def q_dim(self) -> int:
        return self.n_heads * self.head_dim

    @property
    def kv_dim(self) -> int:
        return self.n_kv_heads * self.head_dim

    @property
    def qkv_dim(self) -> int:
        return self.q_dim + 2 * self.kv_dim

    def n_params(self) -> int:
        per_layer = self.d_model * (self.qkv_dim + self.q_dim) + 3 * self.d_model * self.d_ff + 2 * self.d_model
        emb = self.vocab_size * self.d_model * (1 if self.tie_embeddings else 2)
        return self.n_layers * per_layer + emb + self.d_model

    def scaled(self, **kw) -> "ModelConfig":
        return dataclasses.replace(self, **kw)

    # ------------------------------------------------------------------------------
    @classmethod
    def from_gguf(cls, reader, name: Optional[str] = None) -> "ModelConfig":
        arch = reader.architecture
        g = reader.arch_get
        d = int(g("embedding_length"))
        nh = int(g("attention.head_count"))
        nkv = int(g("attention.head_count_kv", nh))
        hd = int(g("attention.key_length", d // nh))
        tokens = reader.get("tokenizer.ggml.tokens")
        vocab = int(g("vocab_size", len(tokens) if tokens is not None else 32000))
        tmpl = reader.get("tokenizer.chat_template")
        return cls(
            name=name or str(reader.get("general.name", "model")),
            arch=arch,
            vocab_size=vocab,
            d_model=d,
            n_layers=int(g("block_count")),
            n_heads=nh,
            n_kv_heads=nkv,
            head_dim=hd,
            d_ff=int(g("feed_forward_length")),
            rope_theta=float(g("rope.freq_base", 10000.0)),
            rope_mode=ROPE_NEOX if arch in ("qwen2", "qwen3", "qwen2moe", "phi3", "gptneox") else ROPE_NORM,
            norm_eps=float(g("attention.layer_norm_rms_epsilon", 1e-5)),
            max_ctx=int(g("context_length", 2048)),
            tie_embeddings="output.weight" not in reader.tensors,
            qk_norm="blk.0.attn_q_norm.weight" in reader.tensors,
            qkv_bias="blk.0.attn_q.bias" in reader.tensors,
            bos_id=int(reader.get("tokenizer.ggml.bos_token_id", 1)),
            eos_id=int(reader.get("tokenizer.ggml.eos_token_id", 2)),
            tokenizer_model=str(reader.get("tokenizer.ggml.model", "llama")),
            chat_template=tmpl if isinstance(tmpl, str) else "zephyr",
        )


PRESETS: Dict[str, ModelConfig] = {
    "tinyllama-1.1b": ModelConfig(
        name="tinyllama-1.1b", vocab_size=32000, d_model=2048, n_layers=22, n_heads=32, n_kv_heads=4,
        head_dim=64, d_ff=5632, rope_theta=10000.0, max_ctx=2048, chat_template="zephyr"),
    "mistral-7b": ModelConfig(
        name="mistral-7b", vocab_size=32000, d_model=4096, n_layers=32, n_heads=32, n_kv_heads=8,
        head_dim=128, d_ff=14336, rope_theta=1e6, max_ctx=32768, chat_template="mistral"),
    "llama3-70b": ModelConfig(
        name="llama3-70b", vocab_size=128256, d_model=8192, n_layers=80, n_heads=64, n_kv_heads=8,
        head_dim=128, d_ff=28672, rope_theta=5e5, max_ctx=8192, bos_id=128000, eos_id=128009,
        tokenizer_model="gpt2", chat_template="llama3"),
    "llama3-8b": ModelConfig(
        name="llama3-8b", vocab_size=128256, d_model=4096, n_layers=32, n_heads=32, n_kv_heads=8,
        head_dim=128, d_ff=14336, rope_theta=5e5, max_ctx=8192, bos_id=128000, eos_id=128009,
        tokenizer_model="gpt2", chat_template="llama3"),
    "qwen3-8b": ModelConfig(
        name="qwen3-8b", arch="qwen3", vocab_size=151936, d_model=4096, n_layers=36, n_heads=32,
        n_kv_heads=8, head_dim=128, d_ff=12288, rope_theta=1e6, rope_mode=ROPE_NEOX, norm_eps=1e-6,
        max_ctx=32768, qk_norm=True, bos_id=151643, eos_id=151645, tokenizer_model="gpt2",
        chat_template="chatml"),
    "qwen3-14b": ModelConfig(
        name="qwen3-14b", arch="qwen3", vocab_size=151936, d_model=5120, n_layers=40, n_heads=40,
        n_kv_heads=8, head_dim=128, d_ff=17408, rope_theta=1e6, rope_mode=ROPE_NEOX, norm_eps=1e-6,
        max_ctx=32768, qk_norm=True, bos_id=151643, eos_id=151645, tokenizer_model="gpt2",
        chat_template="chatml"),
    # small shapes for unit tests (K dims multiples of 256 so every K-quant applies)
    "test-tiny": ModelConfig(
        name="test-tiny", vocab_size=512, d_model=256, n_layers=2, n_heads=4, n_kv_heads=2, head_dim=64,
        d_ff=512, rope_theta=10000.0, max_ctx=256),
    "test-small": ModelConfig(
        name="test-small", vocab_size=1024, d_model=512, n_layers=3, n_heads=8, n_kv_heads=2,
        head_dim=64, d_ff=1536, rope_theta=10000.0, max_ctx=512),
    # smallest llama-3-style shape that shards over TP=2/4/8 in whole Q4_K blocks (8 KV heads,
    # q_dim/8 and d_ff/8 multiples of 256) -- the TP tests' stand-in for Llama-3-70B
    "test-tp8-shape": ModelConfig(
        name="test-tp8-shape", vocab_size=1024, d_model=2048, n_layers=2, n_heads=16, n_kv_heads=8,
        head_dim=128, d_ff=4096, rope_theta=5e5, max_ctx=512),
    # the router's other families at test size, full vocabularies and tokenizers (verdict r2 #9):
    # Qwen3 (NeoX RoPE, QK-norm, 151,936-token byte-level BPE) and Llama-3 (128,256-token BPE)
    "test-qwen3-shape": ModelConfig(
        name="test-qwen3-shape", arch="qwen3", vocab_size=151936, d_model=512, n_layers=2, n_heads=4, n_kv_heads=1,
        head_dim=128, d_ff=1536, rope_theta=1e6, rope_mode=ROPE_NEOX, norm_eps=1e-6, max_ctx=512, qk_norm=True,
        bos_id=151643, eos_id=151645, tokenizer_model="gpt2", chat_template="chatml"),
    "test-llama3-shape": ModelConfig(
        name="test-llama3-shape", vocab_size=128256, d_model=512, n_layers=2, n_heads=4, n_kv_heads=1, head_dim=128,
        d_ff=1536, rope_theta=5e5, max_ctx=512, bos_id=128000, eos_id=128009, tokenizer_model="gpt2",
        chat_template="llama3"),
    "test-mistral-shape": ModelConfig(
        name="test-mistral-shape", vocab_size=1024, d_model=1024, n_layers=2, n_heads=8, n_kv_heads=2,
        head_dim=128, d_ff=2048, rope_theta=1e6, max_ctx=512, chat_template="mistral"),
}


def get_preset(name: str) -> ModelConfig:
    key = name.lower()
    if key not in PRESETS:
        raise KeyError(f"unknown model preset {name!r}; have {sorted(PRESETS)}")
    return PRESETS[key]


# ---------------------------------------------------------------------------------------
# Quantization recipes (which ggml type each tensor gets), mirroring the public llama.cpp
# "Q4_K_M" mix: Q6_K for output + attn_v/ffn_down in "more bits" layers, Q4_K elsewhere.
# ---------------------------------------------------------------------------------------

def _use_more_bits(i: int, n: int) -> bool:
    return i < n // 8 or i >= 7 * n // 8 or (i - n // 8) % 3 == 2


def tensor_type(recipe: str, name: str, layer: int, n_layers: int) -> GGMLType:
    r = recipe.upper()
    if name.endswith("norm.weight") or name.endswith(".bias"):
        return GGMLType.F32
    if r in ("F32",):
        return GGMLType.F32
    if r in ("F16",):
        return GGMLType.F16
    if r in ("BF16",):
        return GGMLType.BF16
    if r == "Q8_0":
        return GGMLType.Q8_0
    if r == "Q4_0":
        return GGMLType.Q6_K if name == "output.weight" else GGMLType.Q4_0
    if r == "Q4_K_M":
        if name == "output.weight":
            return GGMLType.Q6_K
        if name.endswith("attn_v.weight") or name.endswith("ffn_down.weight"):
            return GGMLType.Q6_K if _use_more_bits(layer, n_layers) else GGMLType.Q4_K
        return GGMLType.Q4_K
    if r == "Q5_K_M":
        if name == "output.weight":
            return GGMLType.Q6_K
        if name.endswith("attn_v.weight") or name.endswith("ffn_down.weight"):
            return GGMLType.Q6_K if _use_more_bits(layer, n_layers) else GGMLType.Q5_K
        return GGMLType.Q5_K
    if r in ("IQ4_NL", "IQ4_XS"):  # non-linear 4-bit levels (expanded to bf16 at load)
        return GGMLType.Q6_K if name == "output.weight" else GGMLType[r]
    if r in ("Q4_1", "Q5_0", "Q5_1"):  # legacy 32-block files: expanded to bf16 at load
        return GGMLType.Q6_K if name == "output.weight" else GGMLType[r]
    if r == "Q3_K_M":  # 3-bit K-quant mix (expanded to bf16 at load, like Q2_K)
        if name == "output.weight":
            return GGMLType.Q6_K
        if name.endswith("attn_v.weight") or name.endswith("ffn_down.weight"):
            return GGMLType.Q5_K if _use_more_bits(layer, n_layers) else GGMLType.Q4_K
        return GGMLType.Q4_K if name.endswith("attn_output.weight") else GGMLType.Q3_K
    if r == "Q2_K":
        if name == "output.weight":
            return GGMLType.Q6_K
        if name.endswith("attn_v.weight") or name.endswith("ffn_down.weight"):
            return GGMLType.Q4_K if _use_more_bits(layer, n_layers) else GGMLType.Q3_K
        return GGMLType.Q2_K
    if r == "Q6_K":
        return GGMLType.Q6_K
    if r == "Q4_K":
        return GGMLType.Q4_K
    if r == "Q5_K":
        return GGMLType.Q5_K
    raise ValueError(f"unknown quant recipe {recipe}")
