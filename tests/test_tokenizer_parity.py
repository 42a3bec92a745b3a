"""Tokenizer parity against the two reference tokenizer libraries, trained offline here.

aios_amd.runtime.tokenizer re-implements the GGUF tokenizers instead of
linking sentencepiece / HF tokenizers.  With no network there is no real checkpoint vocab to check
against, so each library trains a small vocabulary on a local corpus (this repository's own docs
plus generated mixed-script text), the vocabulary is written into a GGUF with the repo's own
writer (the `tokenizer.ggml.*` keys llama.cpp's converters emit), read back through the engine's
loader path (GGUFReader -> from_gguf), and encode() must agree token for token with the library on
>= 1000 strings:

* SentencePiece BPE with byte fallback (Llama-2 / Mistral / TinyLlama style, model "llama"),
* HF tokenizers byte-level BPE with the GPT-2 and the Llama-3 pre-tokenizer regex (model "gpt2").
"""
import random
from pathlib import Path

import pytest

from aios_amd.gguf.reader import GGUFReader, GGUFWriter
from aios_amd.runtime.tokenizer import (TOKEN_BYTE, TOKEN_CONTROL, TOKEN_NORMAL, TOKEN_UNKNOWN, PRE_PATTERNS,
                                        bytes_to_unicode, from_gguf)

ROOT = Path(__file__).resolve().parents[1]
N_STRINGS = 1200


def _words(rng):
    text = " ".join((ROOT / f).read_text(errors="ignore") for f in ("README.md", "SURVEY.md") if (ROOT / f).exists())
    words = [w for w in text.split() if len(w) < 24]
    extra = ["naïve", "café", "Zürich", "über", "東京", "数据", "模型", "Ωμέγα", "привет", "😀", "🚀🔥", "ﬁ", "ǅ",
             "x²", "½", "é", "\t", "  ", "\n\n", "1234567", "3.14159", "$100", "foo_bar", "CamelCase",
             "don't", "WE'LL", "it's", "<tag>", "a​b", " nbsp", "\r\n"]
    return words, extra


def _corpus(rng, n):
    words, extra = _words(rng)
    out = []
    for _ in range(n):
        k = rng.randint(1, 14)
        parts = []
        for _ in range(k):
            r = rng.random()
            if r < 0.70 and words:
                parts.append(rng.choice(words))
            elif r < 0.85:
                parts.append(rng.choice(extra))
            else:
                parts.append("".join(chr(rng.choice([rng.randint(0x21, 0x7e), rng.randint(0xa0, 0x24f),
                                                     rng.randint(0x4e00, 0x4fff), rng.randint(0x1f300, 0x1f5ff)]))
                                     for _ in range(rng.randint(1, 5))))
        sep = rng.choice([" ", " ", " ", "  ", "\n", " \n", "\t"])
        out.append(sep.join(parts))
    return out


@pytest.fixture(scope="module")
def corpus(tmp_path_factory):
    rng = random.Random(1234)
    train = _corpus(rng, 4000)
    test = _corpus(random.Random(99), N_STRINGS)
    d = tmp_path_factory.mktemp("tokpar")
    f = d / "corpus.txt"
    f.write_text("\n".join(train), encoding="utf-8")
    return d, f, train, test


def _read(path):
    return from_gguf(GGUFReader(str(path)))


def test_sentencepiece_bpe_byte_fallback_parity(corpus):
    spm = pytest.importorskip("sentencepiece")
    d, f, _, test = corpus
    prefix = str(d / "spm")
    spm.SentencePieceTrainer.train(
        input=str(f), model_prefix=prefix, model_type="bpe", vocab_size=1500, byte_fallback=True,
        character_coverage=0.98, normalization_rule_name="identity", remove_extra_whitespaces=False,
        add_dummy_prefix=True, split_digits=False, allow_whitespace_only_pieces=True, num_threads=4,
        unk_id=0, bos_id=1, eos_id=2, pad_id=-1, minloglevel=2)
    sp = spm.SentencePieceProcessor(model_file=prefix + ".model")
    tokens, scores, types = [], [], []
    for i in range(sp.get_piece_size()):
        tokens.append(sp.id_to_piece(i))
        scores.append(float(sp.get_score(i)))
        types.append(TOKEN_UNKNOWN if sp.is_unknown(i) else TOKEN_CONTROL if sp.is_control(i)
                     else TOKEN_BYTE if sp.is_byte(i) else TOKEN_NORMAL)
    g = d / "spm.gguf"
    w = GGUFWriter(str(g))
    w.add("general.architecture", "llama")
    w.add("tokenizer.ggml.model", "llama")
    w.add("tokenizer.ggml.tokens", tokens)
    w.add("tokenizer.ggml.scores", scores)
    w.add("tokenizer.ggml.token_type", types)
    w.add("tokenizer.ggml.bos_token_id", 1)
    w.add("tokenizer.ggml.eos_token_id", 2)
    w.add("tokenizer.ggml.add_bos_token", True)
    w.add("tokenizer.ggml.add_space_prefix", True)
    w.write()
    tok = _read(g)
    assert sum(t == TOKEN_BYTE for t in types) == 256
    bad = []
    for s in test:
        want = sp.encode(s)
        got = tok.encode(s, add_bos=False, parse_special=False)
        if got != want:
            bad.append((s, want, got))
    assert not bad, f"{len(bad)}/{len(test)} mismatches, first: {bad[0]!r}"
    # byte fallback really exercised (characters outside the trained pieces)
    assert any(sp.is_byte(i) for s in test for i in sp.encode(s))
    # round trip through the engine's decoder
    for s in test[:200]:
        assert tok.decode(tok.encode(s, add_bos=False, parse_special=False)) == s


@pytest.mark.parametrize("pre", ["gpt2", "llama3"])
def test_hf_byte_level_bpe_parity(corpus, pre):
    tk = pytest.importorskip("tokenizers")
    from tokenizers import Regex, Tokenizer, decoders, models, pre_tokenizers, trainers

    d, f, train, test = corpus
    t = Tokenizer(models.BPE())
    if pre == "gpt2":
        t.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=True)
    else:
        t.pre_tokenizer = pre_tokenizers.Sequence([
            pre_tokenizers.Split(Regex(PRE_PATTERNS["llama3"]), behavior="isolated", invert=False),
            pre_tokenizers.ByteLevel(add_prefix_space=False, use_regex=False)])
    t.decoder = decoders.ByteLevel()
    trainer = trainers.BpeTrainer(vocab_size=1500, min_frequency=2, show_progress=False,
                                  special_tokens=["<|begin_of_text|>", "<|end_of_text|>"],
                                  initial_alphabet=pre_tokenizers.ByteLevel.alphabet())
    t.train_from_iterator(train, trainer=trainer)
    vocab = t.get_vocab()
    itos = sorted(vocab.items(), key=lambda kv: kv[1])
    assert [i for _, i in itos] == list(range(len(itos)))
    tokens = [s for s, _ in itos]
    import json
    merges = json.loads(t.to_str())["model"]["merges"]
    merges = [m if isinstance(m, str) else " ".join(m) for m in merges]
    types = [TOKEN_CONTROL if s.startswith("<|") and s.endswith("|>") else TOKEN_NORMAL for s in tokens]
    g = d / f"bpe_{pre}.gguf"
    w = GGUFWriter(str(g))
    w.add("general.architecture", "llama")
    w.add("tokenizer.ggml.model", "gpt2")
    w.add("tokenizer.ggml.pre", pre)
    w.add("tokenizer.ggml.tokens", tokens)
    w.add("tokenizer.ggml.merges", merges)
    w.add("tokenizer.ggml.token_type", types)
    w.add("tokenizer.ggml.bos_token_id", vocab["<|begin_of_text|>"])
    w.add("tokenizer.ggml.eos_token_id", vocab["<|end_of_text|>"])
    w.add("tokenizer.ggml.add_bos_token", False)
    w.write()
    tok = _read(g)
    b2u = bytes_to_unicode()
    assert all(b2u[b] in vocab for b in range(256))  # byte-level: every byte has a token
    bad = []
    for s in test:
        want = t.encode(s, add_special_tokens=False).ids
        got = tok.encode(s, add_bos=False, parse_special=False)
        if got != want:
            bad.append((s, want, got))
    assert not bad, f"{len(bad)}/{len(test)} mismatches, first: {bad[0]!r}"
    for s in test[:200]:
        assert tok.decode(tok.encode(s, add_bos=False, parse_special=False)) == s
    # control tokens in text are matched whole (chat templates), like the library's added tokens
    s = "<|begin_of_text|>hello world<|end_of_text|>"
    assert tok.encode(s, add_bos=False) == t.encode(s, add_special_tokens=False).ids
