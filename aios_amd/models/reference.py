"""fp32 PyTorch reference forward of the Llama-family decoder -- the CPU numerics oracle
("a CPU numerics oracle", "greedy decode must be token-exact against the
CPU engine over N tokens") and the CPU backend of BASELINE config #1 ("TinyLlama Q4_0 greedy
decode ... on CPU, plumbing, no GPU").

Weights are the exact dequantized GGUF values (aios_amd.gguf.quants), so differences against the
HIP engine measure only kernel arithmetic (fp32 accumulation order, bf16 KV cache).
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import numpy as np
import torch

from ..gguf.reader import GGUFReader
from .config import ROPE_NEOX, ModelConfig


class ReferenceModel:
    def __init__(self, cfg: ModelConfig, weights: Dict[str, torch.Tensor], kv_bf16: bool = False,
                 device: str = "cpu", act_q8: bool = False, quantized: Optional[set] = None, kv_fp8: bool = False,
                 kv_scales: Optional[list] = None):
        self.cfg = cfg
        self.w = weights
        self.kv_bf16 = kv_bf16
        # the engine's fp8 KV cache (EngineConfig::kv_fp8): K / V rounded to OCP e4m3 (saturating at
        # 448) after division by the layer's scale (kv_scales: [K0, V0, K1, V1, ...], default 1)
        self.kv_fp8 = kv_fp8
        self.kv_scales = kv_scales
        self.device = device
        self.act_q8 = act_q8                     # emulate the engine's int8 activation path
        self.quantized = quantized or set()      # weight names stored in a block-quant format

    @classmethod
    def from_gguf(cls, path: str, kv_bf16: bool = False, device: str = "cpu", act_q8: bool = False,
                  kv_fp8: bool = False, kv_scales: Optional[list] = None) -> "ReferenceModel":
        from ..gguf.quants import GGMLType

        r = GGUFReader(path)
        cfg = ModelConfig.from_gguf(r)
        w = {}
        quant = set()
        for name, ti in r.tensors.items():
            w[name] = torch.from_numpy(np.ascontiguousarray(r.dequantize(name))).to(device)
            if ti.ggml_type not in (GGMLType.F32, GGMLType.F16, GGMLType.BF16):
                quant.add(name)
        r.close()
        return cls(cfg, w, kv_bf16=kv_bf16, device=device, act_q8=act_q8, quantized=quant, kv_fp8=kv_fp8,
                   kv_scales=kv_scales)

    @staticmethod
    def fp8(x: torch.Tensor, scale: float = 1.0) -> torch.Tensor:
        """OCP e4m3 round trip (round-to-nearest-even, saturating at +-448) of x / scale, times scale."""
        return (x / scale).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).to(torch.float32) * scale

    @staticmethod
    def q8(x: torch.Tensor) -> torch.Tensor:
        """Per-32-block int8 round trip of activations (amax/127 scale, round-half-even)."""
        shp = x.shape
        xb = x.reshape(-1, 32).to(torch.float32)
        amax = xb.abs().amax(-1, keepdim=True)
        inv = torch.where(amax > 0, 127.0 / amax, torch.zeros_like(amax))
        q = torch.round(xb * inv).clamp(-127, 127)
        return (q * (amax / 127.0)).reshape(shp)

    def _mm(self, x: torch.Tensor, name: str) -> torch.Tensor:
        if self.act_q8 and name in self.quantized:
            x = self.q8(x)
        return x @ self.w[name].T

    # ------------------------------------------------------------------------------------------
    def _rms(self, x, w):
        return x * torch.rsqrt((x * x).mean(-1, keepdim=True) + self.cfg.norm_eps) * w

    def _rope(self, x, pos):
        # x [T, H, hd]; pos [T]
        hd = x.shape[-1]
        p = torch.arange(hd // 2, dtype=torch.float32, device=x.device)
        freq = torch.pow(torch.tensor(self.cfg.rope_theta, dtype=torch.float32), -2.0 * p / hd)
        ang = pos.to(torch.float32)[:, None] * freq[None, :]
        c, s = torch.cos(ang)[:, None, :], torch.sin(ang)[:, None, :]
        if self.cfg.rope_mode == ROPE_NEOX:
            a, b = x[..., : hd // 2], x[..., hd // 2:]
            return torch.cat([a * c - b * s, a * s + b * c], dim=-1)
        a, b = x[..., 0::2], x[..., 1::2]
        out = torch.empty_like(x)
        out[..., 0::2] = a * c - b * s
        out[..., 1::2] = a * s + b * c
        return out

    def new_cache(self):
        return {"k": [None] * self.cfg.n_layers, "v": [None] * self.cfg.n_layers, "len": 0}

    @torch.no_grad()
    def forward(self, tokens: List[int], cache: Optional[dict] = None) -> torch.Tensor:
        """Logits [T, V] for `tokens` appended after `cache` (created if None)."""
        cfg = self.cfg
        if cache is None:
            cache = self.new_cache()
        T = len(tokens)
        start = cache["len"]
        pos = torch.arange(start, start + T, device=self.device)
        tok = torch.tensor(tokens, dtype=torch.long, device=self.device)
        x = self.w["token_embd.weight"][tok]
        H, Hkv, hd = cfg.n_heads, cfg.n_kv_heads, cfg.head_dim
        G = H // Hkv
        for l in range(cfg.n_layers):
            p = f"blk.{l}."
            h = self._rms(x, self.w[p + "attn_norm.weight"])
            q = self._mm(h, p + "attn_q.weight")
            k = self._mm(h, p + "attn_k.weight")
            v = self._mm(h, p + "attn_v.weight")
            if p + "attn_q.bias" in self.w:
                q = q + self.w[p + "attn_q.bias"]
                k = k + self.w[p + "attn_k.bias"]
                v = v + self.w[p + "attn_v.bias"]
            q = q.view(T, H, hd)
            k = k.view(T, Hkv, hd)
            v = v.view(T, Hkv, hd)
            if cfg.qk_norm:
                q = self._rms(q, self.w[p + "attn_q_norm.weight"])
                k = self._rms(k, self.w[p + "attn_k_norm.weight"])
            q = self._rope(q, pos)
            k = self._rope(k, pos)
            if self.kv_fp8:
                sk, sv = (self.kv_scales[2 * l], self.kv_scales[2 * l + 1]) if self.kv_scales else (1.0, 1.0)
                k = self.fp8(k, sk)
                v = self.fp8(v, sv)
            elif self.kv_bf16:
                k = k.to(torch.bfloat16).to(torch.float32)
                v = v.to(torch.bfloat16).to(torch.float32)
            if cache["k"][l] is not None:
                k = torch.cat([cache["k"][l], k], 0)
                v = torch.cat([cache["v"][l], v], 0)
            cache["k"][l], cache["v"][l] = k, v
            S = k.shape[0]
            kk = k.repeat_interleave(G, dim=1)  # [S, H, hd]
            vv = v.repeat_interleave(G, dim=1)
            att = torch.einsum("thd,shd->hts", q, kk) / math.sqrt(hd)
            qpos = pos[:, None]
            kpos = torch.arange(S, device=self.device)[None, :]
            att = att.masked_fill((kpos > qpos)[None], float("-inf"))
            att = torch.softmax(att, dim=-1)
            o = torch.einsum("hts,shd->thd", att, vv).reshape(T, H * hd)
            x = x + self._mm(o, p + "attn_output.weight")
            h = self._rms(x, self.w[p + "ffn_norm.weight"])
            g = self._mm(h, p + "ffn_gate.weight")
            u = self._mm(h, p + "ffn_up.weight")
            x = x + self._mm(torch.nn.functional.silu(g) * u, p + "ffn_down.weight")
        cache["len"] = start + T
        x = self._rms(x, self.w["output_norm.weight"])
        return self._mm(x, "output.weight" if "output.weight" in self.w else "token_embd.weight")

    @torch.no_grad()
    def greedy(self, prompt: List[int], n_new: int) -> List[int]:
        cache = self.new_cache()
        logits = self.forward(prompt, cache)
        out = []
        nxt = int(torch.argmax(logits[-1]))
        for _ in range(n_new):
            out.append(nxt)
            logits = self.forward([nxt], cache)
            nxt = int(torch.argmax(logits[-1]))
        return out
