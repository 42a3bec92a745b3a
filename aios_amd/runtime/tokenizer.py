"""Tokenizers read from GGUF metadata.

* `SpmTokenizer`  -- `tokenizer.ggml.model == "llama"` (TinyLlama / Mistral): SentencePiece-style
  BPE driven by piece scores, '▁' space marker, optional space prefix, byte fallback via the
  `<0xXX>` pieces.
* `Gpt2Tokenizer` -- `tokenizer.ggml.model == "gpt2"` (Llama-3 / Qwen): byte-level BPE with the
  GGUF merge list and a regex pre-tokenizer chosen by `tokenizer.ggml.pre`.

Control tokens (token_type 3, e.g. `<s>`, `<|im_start|>`) appearing in text are matched whole
before BPE (chat templates emit them as text), like llama.cpp's parse_special.
"""
from __future__ import annotations

import heapq
from functools import lru_cache
from typing import Dict, List, Optional, Sequence

import regex

TOKEN_NORMAL, TOKEN_UNKNOWN, TOKEN_CONTROL, TOKEN_USER, TOKEN_UNUSED, TOKEN_BYTE = 1, 2, 3, 4, 5, 6

PRE_PATTERNS = {
    "llama3": r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}{1,3}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+",
    "qwen2": r"(?i:'s|'t|'re|'ve|'m|'ll|'d)|[^\r\n\p{L}\p{N}]?\p{L}+|\p{N}| ?[^\s\p{L}\p{N}]+[\r\n]*|\s*[\r\n]+|\s+(?!\S)|\s+",
    "gpt2": r"'s|'t|'re|'ve|'m|'ll|'d| ?\p{L}+| ?\p{N}+| ?[^\s\p{L}\p{N}]+|\s+(?!\S)|\s+",
}
PRE_PATTERNS["llama-bpe"] = PRE_PATTERNS["llama3"]  # the name Llama-3 GGUFs carry in tokenizer.ggml.pre


@lru_cache(maxsize=1)
def bytes_to_unicode() -> Dict[int, str]:
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("¡"), ord("¬") + 1)) + list(range(ord("®"), ord("ÿ") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, map(chr, cs)))


class BaseTokenizer:
    def __init__(self, tokens: Sequence[str], types: Optional[Sequence[int]], bos_id: int, eos_id: int,
                 add_bos: bool = True):
        self.tokens = list(tokens)
        self.types = list(types) if types is not None else [TOKEN_NORMAL] * len(self.tokens)
        self.vocab = {t: i for i, t in enumerate(self.tokens)}
        self.bos_id, self.eos_id, self.add_bos = bos_id, eos_id, add_bos
        self.specials = sorted((t for t, ty in zip(self.tokens, self.types) if ty in (TOKEN_CONTROL, TOKEN_USER) and t),
                               key=len, reverse=True)
        self._special_re = regex.compile("|".join(regex.escape(s) for s in self.specials)) if self.specials else None

    @property
    def vocab_size(self) -> int:
        return len(self.tokens)

    def _split_special(self, text: str, parse_special: bool):
        if not parse_special or self._special_re is None:
            return [(text, False)]
        out, pos = [], 0
        for m in self._special_re.finditer(text):
            if m.start() > pos:
                out.append((text[pos:m.start()], False))
            out.append((m.group(0), True))
            pos = m.end()
        if pos < len(text):
            out.append((text[pos:], False))
        return out

    def encode(self, text: str, add_bos: Optional[bool] = None, parse_special: bool = True) -> List[int]:
        ids: List[int] = []
        if (self.add_bos if add_bos is None else add_bos) and self.bos_id >= 0:
            ids.append(self.bos_id)
        first = True
        for frag, special in self._split_special(text, parse_special):
            if special:
                ids.append(self.vocab[frag])
            else:
                ids.extend(self._encode_fragment(frag, first))
            first = False
        return ids

    def _encode_fragment(self, text: str, first: bool) -> List[int]:
        raise NotImplementedError

    def token_bytes(self, tid: int) -> bytes:
        raise NotImplementedError

    def decode(self, ids: Sequence[int], skip_special: bool = True) -> str:
        out = bytearray()
        for i in ids:
            if skip_special and self.types[i] == TOKEN_CONTROL:
                continue
            out += self.token_bytes(i)
        return out.decode("utf-8", errors="replace")

    def all_token_bytes(self) -> List[bytes]:
        return [b"" if self.types[i] == TOKEN_CONTROL else self.token_bytes(i) for i in range(len(self.tokens))]


class SpmTokenizer(BaseTokenizer):
    """Score-driven BPE over UTF-8 characters with byte fallback (llama/mistral GGUF vocab)."""

    def __init__(self, tokens, scores, types, bos_id=1, eos_id=2, add_bos=True, add_space_prefix=True):
        super().__init__(tokens, types, bos_id, eos_id, add_bos)
        self.scores = [float(s) for s in scores] if scores is not None else [0.0] * len(self.tokens)
        self.add_space_prefix = add_space_prefix
        self.byte_ids = {}
        for i, t in enumerate(self.tokens):
            if self.types[i] == TOKEN_BYTE and len(t) == 6 and t.startswith("<0x"):
                self.byte_ids[int(t[3:5], 16)] = i
        self.unk_id = next((i for i, ty in enumerate(self.types) if ty == TOKEN_UNKNOWN), 0)

    def _encode_fragment(self, text: str, first: bool) -> List[int]:
        if not text:
            return []
        if self.add_space_prefix and first:
            text = " " + text
        text = text.replace(" ", "▁")
        syms = list(text)
        n = len(syms)
        prev = list(range(-1, n - 1))
        nxt = list(range(1, n + 1))
        nxt[-1] = -1
        alive = [True] * n
        heap = []

        def push(i, j):
            piece = syms[i] + syms[j]
            tid = self.vocab.get(piece)
            if tid is not None and self.types[tid] != TOKEN_CONTROL:
                heapq.heappush(heap, (-self.scores[tid], i, j, piece))

        for i in range(n - 1):
            push(i, i + 1)
        while heap:
            _, i, j, piece = heapq.heappop(heap)
            if not (alive[i] and alive[j]) or nxt[i] != j or syms[i] + syms[j] != piece:
                continue
            syms[i] = piece
            alive[j] = False
            nxt[i] = nxt[j]
            if nxt[j] != -1:
                prev[nxt[j]] = i
            if prev[i] != -1:
                push(prev[i], i)
            if nxt[i] != -1:
                push(i, nxt[i])
        out = []
        i = 0
        while i != -1 and i < n:
            if alive[i]:
                tid = self.vocab.get(syms[i])
                if tid is not None:
                    out.append(tid)
                else:
                    for byte in syms[i].encode("utf-8"):
                        out.append(self.byte_ids.get(byte, self.unk_id))
            i = nxt[i]
        return out

    def token_bytes(self, tid: int) -> bytes:
        t = self.tokens[tid]
        if self.types[tid] == TOKEN_BYTE:
            return bytes([int(t[3:5], 16)])
        return t.replace("▁", " ").encode("utf-8")

    def decode(self, ids: Sequence[int], skip_special: bool = True) -> str:
        s = super().decode(ids, skip_special)
        if self.add_space_prefix and s.startswith(" "):
            s = s[1:]
        return s


class Gpt2Tokenizer(BaseTokenizer):
    """Byte-level BPE with ranked merges (Llama-3 / Qwen GGUF vocab)."""

    def __init__(self, tokens, merges, types, bos_id, eos_id, add_bos=False, pre: str = "llama3"):
        super().__init__(tokens, types, bos_id, eos_id, add_bos)
        self.ranks = {}
        for r, m in enumerate(merges or []):
            a, _, b = m.partition(" ")
            self.ranks[(a, b)] = r
        self.pat = regex.compile(PRE_PATTERNS.get(pre, PRE_PATTERNS["llama3"]))
        self.b2u = bytes_to_unicode()
        self.u2b = {v: k for k, v in self.b2u.items()}
        self._cache: Dict[str, List[int]] = {}

    def _bpe(self, word: str) -> List[int]:
        if word in self._cache:
            return self._cache[word]
        parts = list(word)
        while len(parts) > 1:
            best, bi = None, -1
            for i in range(len(parts) - 1):
                r = self.ranks.get((parts[i], parts[i + 1]))
                if r is not None and (best is None or r < best):
                    best, bi = r, i
            if best is None:
                break
            parts[bi:bi + 2] = [parts[bi] + parts[bi + 1]]
        ids = []
        for p in parts:
            tid = self.vocab.get(p)
            if tid is None:
                ids.extend(self.vocab[c] for c in p if c in self.vocab)
            else:
                ids.append(tid)
        if len(self._cache) < 100_000:
            self._cache[word] = ids
        return ids

    def _encode_fragment(self, text: str, first: bool) -> List[int]:
        out = []
        for w in self.pat.findall(text):
            out.extend(self._bpe("".join(self.b2u[b] for b in w.encode("utf-8"))))
        return out

    def token_bytes(self, tid: int) -> bytes:
        t = self.tokens[tid]
        try:
            return bytes(self.u2b[c] for c in t)
        except KeyError:
            return t.encode("utf-8")


def from_gguf(reader) -> BaseTokenizer:
    g = reader.get
    model = str(g("tokenizer.ggml.model", "llama"))
    tokens = g("tokenizer.ggml.tokens")
    if tokens is None:
        raise ValueError("GGUF has no tokenizer.ggml.tokens")
    types = g("tokenizer.ggml.token_type")
    types = [int(t) for t in types] if types is not None else None
    bos = int(g("tokenizer.ggml.bos_token_id", 1))
    eos = int(g("tokenizer.ggml.eos_token_id", 2))
    if model == "gpt2":
        return Gpt2Tokenizer(tokens, g("tokenizer.ggml.merges"), types, bos, eos,
                             add_bos=bool(g("tokenizer.ggml.add_bos_token", False)),
                             pre=str(g("tokenizer.ggml.pre", "llama3")))
    return SpmTokenizer(tokens, g("tokenizer.ggml.scores"), types, bos, eos,
                        add_bos=bool(g("tokenizer.ggml.add_bos_token", True)),
                        add_space_prefix=bool(g("tokenizer.ggml.add_space_prefix", True)))
