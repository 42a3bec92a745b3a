"""Random-init synthetic GGUF models of a named architecture (SURVEY.md §7.5 "Synthetic models").

No network: real checkpoints cannot be fetched, so tests and benchmarks use random weights of
the exact TinyLlama / Mistral / Llama-3 / Qwen3 shapes, quantized with the same per-tensor
recipe as the public Q4_K_M / Q4_0 / ... files, plus a synthetic SentencePiece-style vocabulary
(byte-fallback tokens, printable ASCII, word pieces with '▁' prefixes) and a chat template.
"""
from __future__ import annotations

import itertools
import string
from typing import List, Optional

import numpy as np

from ..gguf.quants import GGMLType, quantize
from ..gguf.reader import GGUFValueType, GGUFWriter
from .config import ModelConfig, tensor_type

CHAT_TEMPLATES = {
    "zephyr": "{% for message in messages %}{% if message['role'] == 'user' %}{{ '<|user|>\n' + message['content'] + eos_token }}{% elif message['role'] == 'system' %}{{ '<|system|>\n' + message['content'] + eos_token }}{% elif message['role'] == 'assistant' %}{{ '<|assistant|>\n'  + message['content'] + eos_token }}{% endif %}{% if loop.last and add_generation_prompt %}{{ '<|assistant|>' }}{% endif %}{% endfor %}",
    "mistral": "{{ bos_token }}{% for message in messages %}{% if message['role'] == 'user' %}{{ '[INST] ' + message['content'] + ' [/INST]' }}{% elif message['role'] == 'assistant' %}{{ message['content'] + eos_token}}{% endif %}{% endfor %}",
}

_WORDS = (
    "the of and to in is that for it as with was on be by this are or from at an have not which "
    "but all were can has one their more will if other its would been also about into do only time "
    "system task goal tool agent memory service file process network status error json true false null "
    "plan step steps tools_needed reasoning done result output input name type value path cpu disk "
    "check monitor restart install security package scan log logs health report data"
).split()


def synthetic_vocab(n: int):
    """SPM-style vocab: (tokens, scores, token_types)."""
    toks: List[str] = ["<unk>", "<s>", "</s>"]
    types: List[int] = [2, 3, 3]
    for b in range(256):
        toks.append(f"<0x{b:02X}>")
        types.append(6)
    seen = set(toks)

    def add(t):
        if t not in seen and len(toks) < n:
            seen.add(t)
            toks.append(t)
            types.append(1)

    for ch in string.printable[:-5]:  # printable ASCII (no \t\n\r\x0b\x0c)
        add(ch.replace(" ", "▁"))
    add("▁")
    for w in _WORDS:
        add("▁" + w)
        add(w)
    letters = string.ascii_lowercase
    for a, b in itertools.product(letters, repeat=2):
        add(a + b)
        add("▁" + a + b)
    for p in ['{"', '":', '",', '"}', '":▁"', '▁{', '▁}', '▁[', ']', '},', '▁"', '"']:
        add(p)
    for a, b, c in itertools.product(letters, repeat=3):
        if len(toks) >= n:
            break
        add(a + b + c)
        add("▁" + a + b + c)
    i = 0
    while len(toks) < n:
        add(f"▁tok{i}")
        i += 1
    scores = [0.0] * 3 + [0.0] * 256 + [-(float(i)) for i in range(len(toks) - 259)]
    return toks, np.array(scores, np.float32), np.array(types, np.int32)


# the control tokens of the byte-level BPE families the router serves (Llama-3 / Qwen3 GGUF ids)
BPE_SPECIALS = {
    128000: "<|begin_of_text|>", 128001: "<|end_of_text|>", 128006: "<|start_header_id|>",
    128007: "<|end_header_id|>", 128009: "<|eot_id|>",
    151643: "<|endoftext|>", 151644: "<|im_start|>", 151645: "<|im_end|>",
}


def synthetic_bpe_vocab(n: int):
    """GPT-2 style byte-level BPE vocab of n tokens: (tokens, merges, token_types) -- the 256 byte
    symbols, ranked merges that build the common words (with and without a leading space), the
    Llama-3 / Qwen control tokens at their real ids, reserved fillers elsewhere."""
    from ..runtime.tokenizer import bytes_to_unicode

    b2u = bytes_to_unicode()
    toks: List[str] = [b2u[b] for b in range(256)]
    types: List[int] = [1] * 256
    seen = set(toks)
    merges: List[str] = []
    for w in _WORDS:
        for word in (w, " " + w):
            sym = [b2u[b] for b in word.encode()]
            cur = sym[0]
            for c in sym[1:]:
                nxt = cur + c
                if nxt not in seen and len(toks) < min(n, 100000):
                    merges.append(f"{cur} {c}")
                    seen.add(nxt)
                    toks.append(nxt)
                    types.append(1)
                cur = nxt
    while len(toks) < n:
        i = len(toks)
        toks.append(BPE_SPECIALS.get(i, f"<|reserved_{i}|>"))
        types.append(3 if i in BPE_SPECIALS else 5)
    return toks, merges, types


def write_synthetic_gguf(path: str, cfg: ModelConfig, recipe: str = "Q4_K_M", seed: int = 0,
                         weight_std: float = 0.02, vocab: Optional[tuple] = None) -> str:
    rng = np.random.default_rng(seed)
    w = GGUFWriter(path)
    arch = cfg.arch
    w.add("general.architecture", arch)
    w.add("general.name", cfg.name)
    w.add(f"{arch}.context_length", cfg.max_ctx)
    w.add(f"{arch}.embedding_length", cfg.d_model)
    w.add(f"{arch}.block_count", cfg.n_layers)
    w.add(f"{arch}.feed_forward_length", cfg.d_ff)
    w.add(f"{arch}.attention.head_count", cfg.n_heads)
    w.add(f"{arch}.attention.head_count_kv", cfg.n_kv_heads)
    w.add(f"{arch}.attention.key_length", cfg.head_dim)
    w.add(f"{arch}.attention.layer_norm_rms_epsilon", float(cfg.norm_eps), GGUFValueType.FLOAT32)
    w.add(f"{arch}.rope.freq_base", float(cfg.rope_theta), GGUFValueType.FLOAT32)
    w.add(f"{arch}.rope.dimension_count", cfg.head_dim)
    w.add(f"{arch}.vocab_size", cfg.vocab_size)
    if cfg.tokenizer_model == "gpt2" and vocab is None:  # Llama-3 / Qwen: byte-level BPE
        toks, merges, types = synthetic_bpe_vocab(cfg.vocab_size)
        w.add("tokenizer.ggml.model", "gpt2")
        w.add("tokenizer.ggml.pre", "qwen2" if cfg.arch == "qwen3" else "llama-bpe")
        w.add("tokenizer.ggml.tokens", toks)
        w.add("tokenizer.ggml.merges", merges)
        w.add("tokenizer.ggml.token_type", types)
        w.add("tokenizer.ggml.add_bos_token", cfg.arch != "qwen3")
    else:
        toks, scores, types = vocab if vocab is not None else synthetic_vocab(cfg.vocab_size)
        w.add("tokenizer.ggml.model", "llama")
        w.add("tokenizer.ggml.tokens", toks)
        w.add("tokenizer.ggml.scores", scores)
        w.add("tokenizer.ggml.token_type", types)
        w.add("tokenizer.ggml.add_bos_token", True)
    w.add("tokenizer.ggml.bos_token_id", cfg.bos_id)
    w.add("tokenizer.ggml.eos_token_id", cfg.eos_id)
    tmpl = CHAT_TEMPLATES.get(cfg.chat_template)
    if tmpl:
        w.add("tokenizer.chat_template", tmpl)

    def mat(name: str, rows: int, cols: int, layer: int, std: float):
        t = tensor_type(recipe, name, layer, cfg.n_layers)
        x = rng.standard_normal((rows, cols), dtype=np.float32) * std
        w.add_tensor(name, (cols, rows), t, quantize(x, t))

    def vec(name: str, n: int, base: float = 1.0, amp: float = 0.1):
        x = (base + amp * rng.standard_normal(n)).astype(np.float32)
        w.add_tensor(name, (n,), GGMLType.F32, x.view(np.uint8))

    d, qd, kvd = cfg.d_model, cfg.q_dim, cfg.kv_dim
    mat("token_embd.weight", cfg.vocab_size, d, 0, 1.0)
    vec("output_norm.weight", d)
    if not cfg.tie_embeddings:
        mat("output.weight", cfg.vocab_size, d, 0, weight_std)
    for i in range(cfg.n_layers):
        p = f"blk.{i}."
        vec(p + "attn_norm.weight", d)
        vec(p + "ffn_norm.weight", d)
        mat(p + "attn_q.weight", qd, d, i, weight_std)
        mat(p + "attn_k.weight", kvd, d, i, weight_std)
        mat(p + "attn_v.weight", kvd, d, i, weight_std)
        mat(p + "attn_output.weight", d, qd, i, weight_std)
        mat(p + "ffn_gate.weight", cfg.d_ff, d, i, weight_std)
        mat(p + "ffn_up.weight", cfg.d_ff, d, i, weight_std)
        mat(p + "ffn_down.weight", d, cfg.d_ff, i, weight_std)
        if cfg.qk_norm:
            vec(p + "attn_q_norm.weight", cfg.head_dim)
            vec(p + "attn_k_norm.weight", cfg.head_dim)
        if cfg.qkv_bias:
            vec(p + "attn_q.bias", qd, 0.0, 0.02)
            vec(p + "attn_k.bias", kvd, 0.0, 0.02)
            vec(p + "attn_v.bias", kvd, 0.0, 0.02)
    w.write()
    return path
