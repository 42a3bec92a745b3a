"""GGML block-quant formats: CPU reference (numpy) dequantizers and simple quantizers.

This is the bit-exact oracle the HIP dequant kernels are tested against.  The
byte layouts are the public GGUF/ggml block formats that the reference's
llama-server consumes (`runtime/src/model_manager.rs:187-204` spawns it on
Q4_K_M GGUF files, `scripts/download-models.sh:70-77`).  SURVEY.md §2.7 K3/K12
lists the formats a Q4_K_M file contains (Q4_K, Q6_K, plus Q5_K/Q8_0/Q4_0/F16/BF16).

Quantizers here are deliberately simple (min/max per sub-block): they produce
valid blocks for synthetic random-init models; only dequantization has to match
ggml exactly.
"""
from __future__ import annotations

import enum

import numpy as np


class GGMLType(enum.IntEnum):
    F32 = 0
    F16 = 1
    Q4_0 = 2
    Q4_1 = 3
    Q5_0 = 6
    Q5_1 = 7
    Q8_0 = 8
    Q8_1 = 9
    Q2_K = 10
    Q3_K = 11
    Q4_K = 12
    Q5_K = 13
    Q6_K = 14
    Q8_K = 15
    IQ4_NL = 20
    IQ4_XS = 23
    BF16 = 30


QK_K = 256

# (elements per block, bytes per block)
BLOCK_INFO = {
    GGMLType.F32: (1, 4),
    GGMLType.F16: (1, 2),
    GGMLType.BF16: (1, 2),
    GGMLType.Q4_0: (32, 18),
    GGMLType.Q4_1: (32, 20),
    GGMLType.Q5_0: (32, 22),
    GGMLType.Q5_1: (32, 24),
    GGMLType.Q8_0: (32, 34),
    GGMLType.IQ4_NL: (32, 18),
    GGMLType.IQ4_XS: (256, 136),
    GGMLType.Q2_K: (256, 84),
    GGMLType.Q3_K: (256, 110),
    GGMLType.Q4_K: (256, 144),
    GGMLType.Q5_K: (256, 176),
    GGMLType.Q6_K: (256, 210),
}


def type_size(t: GGMLType, n_elements: int) -> int:
    blk, nbytes = BLOCK_INFO[GGMLType(t)]
    if n_elements % blk:
        raise ValueError(f"{GGMLType(t).name}: {n_elements} not a multiple of {blk}")
    return n_elements // blk * nbytes


def _f16(b: np.ndarray) -> np.ndarray:
    """View trailing 2 bytes as float16 -> float32."""
    return np.ascontiguousarray(b).view(np.float16).astype(np.float32)


# ----------------------------------------------------------------------------------
# dequantizers: raw bytes [n_blocks * block_bytes] -> float32 [n_blocks * block_elems]
# ----------------------------------------------------------------------------------

def _blocks(raw: np.ndarray, t: GGMLType) -> np.ndarray:
    _, nb = BLOCK_INFO[t]
    raw = np.frombuffer(raw, dtype=np.uint8) if not isinstance(raw, np.ndarray) else raw.view(np.uint8)
    assert raw.size % nb == 0, (raw.size, nb)
    return raw.reshape(-1, nb)


def dequant_q4_0(raw) -> np.ndarray:
    b = _blocks(raw, GGMLType.Q4_0)
    d = _f16(b[:, 0:2]).reshape(-1, 1)
    qs = b[:, 2:18]
    lo = (qs & 0x0F).astype(np.int32) - 8
    hi = (qs >> 4).astype(np.int32) - 8
    return (np.concatenate([lo, hi], axis=1) * d).astype(np.float32).ravel()


def dequant_q4_1(raw) -> np.ndarray:
    b = _blocks(raw, GGMLType.Q4_1)
    d = _f16(b[:, 0:2]).reshape(-1, 1)
    m = _f16(b[:, 2:4]).reshape(-1, 1)
    qs = b[:, 4:20]
    q = np.concatenate([qs & 0x0F, qs >> 4], axis=1).astype(np.float32)
    return (q * d + m).astype(np.float32).ravel()


def _q5_high(b: np.ndarray, off: int) -> np.ndarray:
    qh = np.ascontiguousarray(b[:, off:off + 4]).view(np.uint32).reshape(-1, 1)
    j = np.arange(16, dtype=np.uint32).reshape(1, -1)
    h0 = ((qh >> j) << 4) & 0x10
    h1 = (qh >> (j + 12)) & 0x10
    return h0.astype(np.int32), h1.astype(np.int32)


def dequant_q5_0(raw) -> np.ndarray:
    b = _blocks(raw, GGMLType.Q5_0)
    d = _f16(b[:, 0:2]).reshape(-1, 1)
    h0, h1 = _q5_high(b, 2)
    qs = b[:, 6:22].astype(np.int32)
    x0 = ((qs & 0x0F) | h0) - 16
    x1 = ((qs >> 4) | h1) - 16
    return (np.concatenate([x0, x1], axis=1) * d).astype(np.float32).ravel()


def dequant_q5_1(raw) -> np.ndarray:
    b = _blocks(raw, GGMLType.Q5_1)
    d = _f16(b[:, 0:2]).reshape(-1, 1)
    m = _f16(b[:, 2:4]).reshape(-1, 1)
    h0, h1 = _q5_high(b, 4)
    qs = b[:, 8:24].astype(np.int32)
    x0 = (qs & 0x0F) | h0
    x1 = (qs >> 4) | h1
    return (np.concatenate([x0, x1], axis=1) * d + m).astype(np.float32).ravel()


def dequant_q8_0(raw) -> np.ndarray:
    b = _blocks(raw, GGMLType.Q8_0)
    d = _f16(b[:, 0:2]).reshape(-1, 1)
    q = b[:, 2:34].view(np.int8).astype(np.float32)
    return (q * d).astype(np.float32).ravel()


# the IQ4 formats' 16 non-linear levels (the public GGUF definition), scaled by the block's d
IQ4_LEVELS = np.array([-127, -104, -83, -65, -49, -35, -22, -10, 1, 13, 25, 38, 53, 69, 89, 113], np.float32)


def dequant_iq4_nl(raw) -> np.ndarray:
    """IQ4_NL: f16 d, 16 bytes of 4-bit level indices (element j < 16: low nibble of byte j, j >= 16: high
    nibble of byte j - 16, as Q4_0); y = d * level."""
    b = _blocks(raw, GGMLType.IQ4_NL)
    d = _f16(b[:, 0:2]).reshape(-1, 1)
    qs = b[:, 2:18]
    return (d * IQ4_LEVELS[np.concatenate([qs & 0xF, qs >> 4], axis=1)]).astype(np.float32).ravel()


def iq4xs_scales(b: np.ndarray) -> np.ndarray:
    """[nb, 136] IQ4_XS blocks -> [nb, 8] signed sub-block scales: 4 low bits from nibble (i & 1) of byte
    4 + i // 2, 2 high bits at bits 2 i of the u16 at byte 2; stored value - 32."""
    sh = np.ascontiguousarray(b[:, 2:4]).view(np.uint16).astype(np.int32).reshape(-1, 1)
    i = np.arange(8)
    lo = (b[:, 4 + i // 2].astype(np.int32) >> (4 * (i % 2))) & 0xF
    return (lo | (((sh >> (2 * i)) & 3) << 4)) - 32


def dequant_iq4_xs(raw) -> np.ndarray:
    """IQ4_XS: f16 d, u16 high scale bits, 4 bytes of low scale nibbles, 128 bytes of level indices (eight
    32-element sub-blocks, each laid out as an IQ4_NL block's nibbles); y = d * scale(j >> 5) * level."""
    b = _blocks(raw, GGMLType.IQ4_XS)
    d = _f16(b[:, 0:2]).reshape(-1, 1)
    qs = b[:, 8:136].reshape(-1, 8, 16)
    idx = np.concatenate([qs & 0xF, qs >> 4], axis=2).reshape(-1, 256)
    return (d * np.repeat(iq4xs_scales(b), 32, axis=1) * IQ4_LEVELS[idx]).astype(np.float32).ravel()


def _kq_low2(qs: np.ndarray) -> np.ndarray:
    """2-bit fields of the Q2_K / Q3_K quant bytes [nb, 64] -> [nb, 256] in element order: element
    j = 128 n + 32 g + t sits in byte 32 n + t at bits 2 g."""
    g = (2 * np.arange(4, dtype=np.uint8)).reshape(1, 1, 4, 1)
    return ((qs.reshape(-1, 2, 1, 32) >> g) & 3).reshape(-1, 256).astype(np.int32)


def dequant_q2_k(raw) -> np.ndarray:
    """Q2_K: 16 (4-bit scale, 4-bit min) bytes, 64 bytes of 2-bit quants, f16 d, f16 dmin;
    y = d * scale(j >> 4) * q - dmin * min(j >> 4)."""
    b = _blocks(raw, GGMLType.Q2_K)
    sc = b[:, :16].astype(np.int32)
    d = _f16(b[:, 80:82]).reshape(-1, 1)
    dmin = _f16(b[:, 82:84]).reshape(-1, 1)
    q = _kq_low2(b[:, 16:80])
    return (d * np.repeat(sc & 0xF, 16, axis=1) * q - dmin * np.repeat(sc >> 4, 16, axis=1)).astype(np.float32).ravel()


def q3k_scales(scb: np.ndarray) -> np.ndarray:
    """The 12-byte table of sixteen 6-bit Q3_K scales -> [nb, 16] signed (stored value - 32): scale s
    (g = s >> 2, k = s & 3) has its low 4 bits in byte k (g even) or 4 + k (g odd), low or high nibble
    for g < 2 / g >= 2, and its top 2 bits at bits 2 g of byte 8 + k."""
    scb = scb.astype(np.int32)
    out = np.empty((scb.shape[0], 16), np.int32)
    for s_ in range(16):
        g, k = s_ >> 2, s_ & 3
        low = (scb[:, (4 if g & 1 else 0) + k] >> (4 if g & 2 else 0)) & 0xF
        out[:, s_] = (low | (((scb[:, 8 + k] >> (2 * g)) & 3) << 4)) - 32
    return out


def dequant_q3_k(raw) -> np.ndarray:
    """Q3_K: 32 bytes of high bits, 64 bytes of 2-bit quants, 12 bytes of 6-bit scales, f16 d;
    y = d * scale(j >> 4) * (low2 - (high bit ? 0 : 4)), the high bit of element j at bit j >> 5 of
    byte j & 31."""
    b = _blocks(raw, GGMLType.Q3_K)
    hm = b[:, :32]
    low = _kq_low2(b[:, 32:96])
    hb = ((hm.reshape(-1, 1, 32) >> np.arange(8, dtype=np.uint8).reshape(1, 8, 1)) & 1).reshape(-1, 256).astype(np.int32)
    sc = np.repeat(q3k_scales(b[:, 96:108]), 16, axis=1)
    d = _f16(b[:, 108:110]).reshape(-1, 1)
    return (d * sc * (low - 4 * (1 - hb))).astype(np.float32).ravel()


def kquant_scale_min(scales: np.ndarray):
    """Unpack the 12-byte 6-bit (scale, min) table of Q4_K/Q5_K -> two [nb, 8] int arrays."""
    q = scales.astype(np.int32)
    sc = np.empty((q.shape[0], 8), np.int32)
    mn = np.empty((q.shape[0], 8), np.int32)
    for j in range(8):
        if j < 4:
            sc[:, j] = q[:, j] & 63
            mn[:, j] = q[:, j + 4] & 63
        else:
            sc[:, j] = (q[:, j + 4] & 0xF) | ((q[:, j - 4] >> 6) << 4)
            mn[:, j] = (q[:, j + 4] >> 4) | ((q[:, j] >> 6) << 4)
    return sc, mn


def kquant_pack_scale_min(sc: np.ndarray, mn: np.ndarray) -> np.ndarray:
    """Inverse of kquant_scale_min: [nb,8] 6-bit values -> [nb,12] bytes."""
    sc = sc.astype(np.int32)
    mn = mn.astype(np.int32)
    out = np.zeros((sc.shape[0], 12), np.int32)
    for j in range(8):
        if j < 4:
            out[:, j] |= sc[:, j] & 63
            out[:, j + 4] |= mn[:, j] & 63
        else:
            out[:, j + 4] |= (sc[:, j] & 0xF) | ((mn[:, j] & 0xF) << 4)
            out[:, j - 4] |= (sc[:, j] >> 4) << 6
            out[:, j] |= (mn[:, j] >> 4) << 6
    return out.astype(np.uint8)


def dequant_q4_k(raw) -> np.ndarray:
    b = _blocks(raw, GGMLType.Q4_K)
    d = _f16(b[:, 0:2]).reshape(-1, 1)
    dmin = _f16(b[:, 2:4]).reshape(-1, 1)
    sc, mn = kquant_scale_min(b[:, 4:16])
    qs = b[:, 16:144].reshape(-1, 4, 32)
    out = np.empty((b.shape[0], 4, 2, 32), np.float32)
    for g in range(4):
        d1 = d * sc[:, 2 * g:2 * g + 1]
        m1 = dmin * mn[:, 2 * g:2 * g + 1]
        d2 = d * sc[:, 2 * g + 1:2 * g + 2]
        m2 = dmin * mn[:, 2 * g + 1:2 * g + 2]
        out[:, g, 0] = d1 * (qs[:, g] & 0xF) - m1
        out[:, g, 1] = d2 * (qs[:, g] >> 4) - m2
    return out.ravel()


def dequant_q5_k(raw) -> np.ndarray:
    b = _blocks(raw, GGMLType.Q5_K)
    d = _f16(b[:, 0:2]).reshape(-1, 1)
    dmin = _f16(b[:, 2:4]).reshape(-1, 1)
    sc, mn = kquant_scale_min(b[:, 4:16])
    qh = b[:, 16:48]
    qs = b[:, 48:176].reshape(-1, 4, 32)
    out = np.empty((b.shape[0], 4, 2, 32), np.float32)
    for g in range(4):
        d1 = d * sc[:, 2 * g:2 * g + 1]
        m1 = dmin * mn[:, 2 * g:2 * g + 1]
        d2 = d * sc[:, 2 * g + 1:2 * g + 2]
        m2 = dmin * mn[:, 2 * g + 1:2 * g + 2]
        h1 = ((qh >> (2 * g)) & 1).astype(np.int32) * 16
        h2 = ((qh >> (2 * g + 1)) & 1).astype(np.int32) * 16
        out[:, g, 0] = d1 * ((qs[:, g] & 0xF) + h1) - m1
        out[:, g, 1] = d2 * ((qs[:, g] >> 4) + h2) - m2
    return out.ravel()


def dequant_q6_k(raw) -> np.ndarray:
    b = _blocks(raw, GGMLType.Q6_K)
    ql = b[:, 0:128].astype(np.int32)
    qh = b[:, 128:192].astype(np.int32)
    sc = b[:, 192:208].view(np.int8).astype(np.float32)
    d = _f16(b[:, 208:210]).reshape(-1, 1)
    out = np.empty((b.shape[0], 2, 4, 32), np.float32)
    for n in range(2):
        l0 = ql[:, 64 * n:64 * n + 32]
        l1 = ql[:, 64 * n + 32:64 * n + 64]
        h = qh[:, 32 * n:32 * n + 32]
        s = sc[:, 8 * n:8 * n + 8]
        q1 = ((l0 & 0xF) | (((h >> 0) & 3) << 4)) - 32
        q2 = ((l1 & 0xF) | (((h >> 2) & 3) << 4)) - 32
        q3 = ((l0 >> 4) | (((h >> 4) & 3) << 4)) - 32
        q4 = ((l1 >> 4) | (((h >> 6) & 3) << 4)) - 32
        # scale index is = l/16 (+0,+2,+4,+6)
        for k, q in enumerate((q1, q2, q3, q4)):
            sidx = np.repeat(np.array([0, 1]) + 2 * k, 16)
            out[:, n, k] = d * s[:, sidx] * q
    return out.ravel()


def dequant_f16(raw) -> np.ndarray:
    return np.frombuffer(raw, dtype=np.float16).astype(np.float32) if not isinstance(raw, np.ndarray) \
        else raw.view(np.float16).astype(np.float32).ravel()


def dequant_bf16(raw) -> np.ndarray:
    u = (np.frombuffer(raw, dtype=np.uint16) if not isinstance(raw, np.ndarray) else raw.view(np.uint16).ravel())
    return (u.astype(np.uint32) << 16).view(np.float32)


def dequant_f32(raw) -> np.ndarray:
    return (np.frombuffer(raw, dtype=np.float32) if not isinstance(raw, np.ndarray) else raw.view(np.float32).ravel()).copy()


DEQUANT = {
    GGMLType.F32: dequant_f32,
    GGMLType.F16: dequant_f16,
    GGMLType.BF16: dequant_bf16,
    GGMLType.Q4_0: dequant_q4_0,
    GGMLType.Q4_1: dequant_q4_1,
    GGMLType.Q5_0: dequant_q5_0,
    GGMLType.Q5_1: dequant_q5_1,
    GGMLType.Q8_0: dequant_q8_0,
    GGMLType.Q2_K: dequant_q2_k,
    GGMLType.Q3_K: dequant_q3_k,
    GGMLType.IQ4_NL: dequant_iq4_nl,
    GGMLType.IQ4_XS: dequant_iq4_xs,
    GGMLType.Q4_K: dequant_q4_k,
    GGMLType.Q5_K: dequant_q5_k,
    GGMLType.Q6_K: dequant_q6_k,
}


def dequantize(raw, t: GGMLType, shape=None) -> np.ndarray:
    out = DEQUANT[GGMLType(t)](raw)
    return out.reshape(shape) if shape is not None else out


# ----------------------------------------------------------------------------------
# quantizers (float32 [n] -> raw bytes)
# ----------------------------------------------------------------------------------

def _to_f16_bytes(x: np.ndarray) -> np.ndarray:
    return x.astype(np.float16).reshape(-1, 1).view(np.uint8).reshape(-1, 2)


def quant_q4_0(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float32).reshape(-1, 32)
    amax_idx = np.argmax(np.abs(x), axis=1)
    mx = x[np.arange(x.shape[0]), amax_idx]
    d = mx / -8.0
    dh = d.astype(np.float16).astype(np.float32)
    inv = np.where(dh != 0, 1.0 / np.where(dh == 0, 1, dh), 0.0).reshape(-1, 1)
    q = np.clip(np.floor(x * inv + 8.5), 0, 15).astype(np.uint8)
    qs = (q[:, :16] | (q[:, 16:] << 4)).astype(np.uint8)
    return np.concatenate([_to_f16_bytes(dh), qs], axis=1).ravel()


def quant_q8_0(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float32).reshape(-1, 32)
    amax = np.abs(x).max(axis=1)
    d = (amax / 127.0).astype(np.float16).astype(np.float32)
    inv = np.where(d != 0, 1.0 / np.where(d == 0, 1, d), 0.0).reshape(-1, 1)
    q = np.clip(np.round(x * inv), -127, 127).astype(np.int8)
    return np.concatenate([_to_f16_bytes(d), q.view(np.uint8)], axis=1).ravel()


def _affine32(x: np.ndarray, nmax: int):
    """x [nb, 32] -> (d, m f16-rounded [nb, 1], q [nb, 32] in 0..nmax): y = d * q + m."""
    mn, mx = x.min(axis=1, keepdims=True), x.max(axis=1, keepdims=True)
    d = ((mx - mn) / nmax).astype(np.float16).astype(np.float32)
    m = mn.astype(np.float16).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        q = np.where(d > 0, np.round((x - m) / d), 0)
    return d, m, q.clip(0, nmax).astype(np.int32)


def _q5_pack(q: np.ndarray) -> np.ndarray:
    """5-bit q [nb, 32] -> qh (bit i = high bit of element i, 4 bytes) + 16 nibble-pair bytes."""
    qh = np.zeros(q.shape[0], np.uint32)
    for i in range(32):
        qh |= ((q[:, i] >> 4) & 1).astype(np.uint32) << np.uint32(i)
    qs = ((q[:, :16] & 0xF) | ((q[:, 16:] & 0xF) << 4)).astype(np.uint8)
    return np.concatenate([qh.reshape(-1, 1).view(np.uint8), qs], axis=1)


def quant_q4_1(x: np.ndarray) -> np.ndarray:
    d, m, q = _affine32(x.astype(np.float32).reshape(-1, 32), 15)
    qs = (q[:, :16] | (q[:, 16:] << 4)).astype(np.uint8)
    return np.concatenate([_to_f16_bytes(d), _to_f16_bytes(m), qs], axis=1).ravel()


def quant_q5_0(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float32).reshape(-1, 32)
    mx = x[np.arange(x.shape[0]), np.argmax(np.abs(x), axis=1)]
    d = (mx / -16.0).astype(np.float16).astype(np.float32)
    inv = np.where(d != 0, 1.0 / np.where(d == 0, 1, d), 0.0).reshape(-1, 1)
    q = np.clip(np.floor(x * inv + 16.5), 0, 31).astype(np.int32)
    return np.concatenate([_to_f16_bytes(d), _q5_pack(q)], axis=1).ravel()


def quant_q5_1(x: np.ndarray) -> np.ndarray:
    d, m, q = _affine32(x.astype(np.float32).reshape(-1, 32), 31)
    return np.concatenate([_to_f16_bytes(d), _to_f16_bytes(m), _q5_pack(q)], axis=1).ravel()


def _iq4_index(v: np.ndarray) -> np.ndarray:
    """Nearest IQ4 level index of each value (in level units)."""
    return np.abs(v[..., None] - IQ4_LEVELS).argmin(axis=-1).astype(np.uint8)


def quant_iq4_nl(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float32).reshape(-1, 32)
    d = (np.abs(x).max(axis=1) / 127.0).astype(np.float16).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        q = _iq4_index(np.where(d[:, None] > 0, x / d[:, None], 0.0))
    return np.concatenate([_to_f16_bytes(d), q[:, :16] | (q[:, 16:] << 4)], axis=1).ravel()


def quant_iq4_xs(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float32).reshape(-1, 8, 32)
    s_f = np.abs(x).max(axis=2) / 127.0
    d = (s_f.max(axis=1) / 31.0).astype(np.float16).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        ls = np.where(d[:, None] > 0, np.round(s_f / d[:, None]), 0).clip(0, 31).astype(np.int32)
        dl = d[:, None] * ls
        q = _iq4_index(np.where(dl[..., None] > 0, x / dl[..., None], 0.0))
    v = ls + 32  # stored 6-bit scales
    sh = np.zeros(x.shape[0], np.uint16)
    sl = np.zeros((x.shape[0], 4), np.uint8)
    for i in range(8):
        sh |= ((v[:, i] >> 4) & 3).astype(np.uint16) << np.uint16(2 * i)
        sl[:, i // 2] |= ((v[:, i] & 0xF) << (4 * (i % 2))).astype(np.uint8)
    qs = (q[:, :, :16] | (q[:, :, 16:] << 4)).reshape(-1, 128)
    return np.concatenate([_to_f16_bytes(d), sh.reshape(-1, 1).view(np.uint8), sl, qs], axis=1).ravel()


def _kq_pack_low2(q: np.ndarray) -> np.ndarray:
    """[nb, 256] values 0..3 -> the 64 quant bytes (inverse of _kq_low2)."""
    q4 = q.reshape(-1, 2, 4, 32).astype(np.uint8)
    out = np.zeros((q.shape[0], 2, 32), np.uint8)
    for g in range(4):
        out |= q4[:, :, g, :] << np.uint8(2 * g)
    return out.reshape(-1, 64)


def quant_q2_k(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float32).reshape(-1, 16, 16)
    lo = np.minimum(x.min(axis=2), 0.0)
    scale, mins = (x.max(axis=2) - lo) / 3.0, -lo
    d = (scale.max(axis=1) / 15.0).astype(np.float16).astype(np.float32)
    dmin = (mins.max(axis=1) / 15.0).astype(np.float16).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        sc = np.where(d[:, None] > 0, np.round(scale / d[:, None]), 0).clip(0, 15).astype(np.int32)
        mn = np.where(dmin[:, None] > 0, np.round(mins / dmin[:, None]), 0).clip(0, 15).astype(np.int32)
        eff_d, eff_m = d[:, None] * sc, dmin[:, None] * mn
        q = np.where(eff_d[..., None] > 0, np.round((x + eff_m[..., None]) / eff_d[..., None]), 0)
    q = q.clip(0, 3).astype(np.int32).reshape(-1, 256)
    return np.concatenate([(sc | (mn << 4)).astype(np.uint8), _kq_pack_low2(q), _to_f16_bytes(d),
                           _to_f16_bytes(dmin)], axis=1).ravel()


def quant_q3_k(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float32).reshape(-1, 16, 16)
    s_f = np.abs(x).max(axis=2) / 4.0
    d = (s_f.max(axis=1) / 31.0).astype(np.float16).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        sc = np.where(d[:, None] > 0, np.round(s_f / d[:, None]), 0).clip(0, 31).astype(np.int32)
        eff = d[:, None] * sc
        q = np.where(eff[..., None] > 0, np.round(x / eff[..., None]), 0)
    u = (q.clip(-4, 3) + 4).astype(np.int32).reshape(-1, 256)
    nb = u.shape[0]
    hm = np.zeros((nb, 32), np.uint8)
    hbit = (u >> 2).reshape(nb, 8, 32).astype(np.uint8)
    for bit in range(8):
        hm |= hbit[:, bit, :] << np.uint8(bit)
    v = sc + 32  # stored 6-bit scales
    scb = np.zeros((nb, 12), np.int32)
    for s_ in range(16):
        g, k = s_ >> 2, s_ & 3
        scb[:, (4 if g & 1 else 0) + k] |= (v[:, s_] & 0xF) << (4 if g & 2 else 0)
        scb[:, 8 + k] |= (v[:, s_] >> 4) << (2 * g)
    return np.concatenate([hm, _kq_pack_low2(u & 3), scb.astype(np.uint8), _to_f16_bytes(d)], axis=1).ravel()


def _kquant_affine(x: np.ndarray, nmax: int):
    """x [nb, 8, 32] -> (d, dmin f16-rounded [nb], sc6, mn6 [nb,8], q [nb,8,32] in 0..nmax)."""
    lo = np.minimum(x.min(axis=2), 0.0)  # min is stored as a positive offset: y = d*sc*q - dmin*m
    hi = x.max(axis=2)
    scale = (hi - lo) / nmax
    mins = -lo
    max_scale = scale.max(axis=1)
    max_min = mins.max(axis=1)
    d = (max_scale / 63.0).astype(np.float16).astype(np.float32)
    dmin = (max_min / 63.0).astype(np.float16).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        sc = np.where(d[:, None] > 0, np.round(scale / d[:, None]), 0).clip(0, 63).astype(np.int32)
        mn = np.where(dmin[:, None] > 0, np.round(mins / dmin[:, None]), 0).clip(0, 63).astype(np.int32)
        eff_d = d[:, None] * sc
        eff_m = dmin[:, None] * mn
        q = np.where(eff_d[..., None] > 0, np.round((x + eff_m[..., None]) / eff_d[..., None]), 0)
    q = q.clip(0, nmax).astype(np.int32)
    return d, dmin, sc, mn, q


def quant_q4_k(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float32).reshape(-1, 8, 32)
    d, dmin, sc, mn, q = _kquant_affine(x, 15)
    qs = np.empty((x.shape[0], 4, 32), np.uint8)
    for g in range(4):
        qs[:, g] = (q[:, 2 * g] | (q[:, 2 * g + 1] << 4)).astype(np.uint8)
    return np.concatenate([_to_f16_bytes(d), _to_f16_bytes(dmin), kquant_pack_scale_min(sc, mn),
                           qs.reshape(-1, 128)], axis=1).ravel()


def quant_q5_k(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float32).reshape(-1, 8, 32)
    d, dmin, sc, mn, q = _kquant_affine(x, 31)
    qs = np.empty((x.shape[0], 4, 32), np.uint8)
    qh = np.zeros((x.shape[0], 32), np.int32)
    for g in range(4):
        a, b = q[:, 2 * g], q[:, 2 * g + 1]
        qs[:, g] = ((a & 0xF) | ((b & 0xF) << 4)).astype(np.uint8)
        qh |= ((a >> 4) & 1) << (2 * g)
        qh |= ((b >> 4) & 1) << (2 * g + 1)
    return np.concatenate([_to_f16_bytes(d), _to_f16_bytes(dmin), kquant_pack_scale_min(sc, mn),
                           qh.astype(np.uint8), qs.reshape(-1, 128)], axis=1).ravel()


def quant_q6_k(x: np.ndarray) -> np.ndarray:
    x = x.astype(np.float32).reshape(-1, 16, 16)
    amax_idx = np.argmax(np.abs(x), axis=2)
    mx = np.take_along_axis(x, amax_idx[..., None], axis=2)[..., 0]
    scale = mx / -32.0  # per 16-elem sub-block
    amax_s_idx = np.argmax(np.abs(scale), axis=1)
    smax = scale[np.arange(x.shape[0]), amax_s_idx]
    d = (smax / -128.0).astype(np.float16).astype(np.float32)
    with np.errstate(divide="ignore", invalid="ignore"):
        sc = np.where(d[:, None] != 0, np.round(scale / d[:, None]), 0).clip(-128, 127).astype(np.int32)
        eff = d[:, None] * sc
        q = np.where(eff[..., None] != 0, np.round(x / eff[..., None]), 0)
    q = (q.clip(-32, 31) + 32).astype(np.int32).reshape(-1, 256)
    nb = x.shape[0]
    ql = np.zeros((nb, 128), np.int32)
    qh = np.zeros((nb, 64), np.int32)
    for n in range(2):
        base = 128 * n
        q1 = q[:, base + 0:base + 32]
        q2 = q[:, base + 32:base + 64]
        q3 = q[:, base + 64:base + 96]
        q4 = q[:, base + 96:base + 128]
        ql[:, 64 * n:64 * n + 32] = (q1 & 0xF) | ((q3 & 0xF) << 4)
        ql[:, 64 * n + 32:64 * n + 64] = (q2 & 0xF) | ((q4 & 0xF) << 4)
        qh[:, 32 * n:32 * n + 32] = (q1 >> 4) | ((q2 >> 4) << 2) | ((q3 >> 4) << 4) | ((q4 >> 4) << 6)
    return np.concatenate([ql.astype(np.uint8), qh.astype(np.uint8), sc.astype(np.int8).view(np.uint8),
                           _to_f16_bytes(d)], axis=1).ravel()


def quant_f16(x):
    return x.astype(np.float16).view(np.uint8).ravel()


def quant_bf16(x):
    u = x.astype(np.float32).view(np.uint32)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)
    return r.view(np.uint8).ravel()


def quant_f32(x):
    return x.astype(np.float32).view(np.uint8).ravel()


QUANT = {
    GGMLType.F32: quant_f32,
    GGMLType.F16: quant_f16,
    GGMLType.BF16: quant_bf16,
    GGMLType.Q4_0: quant_q4_0,
    GGMLType.Q4_1: quant_q4_1,
    GGMLType.Q5_0: quant_q5_0,
    GGMLType.Q5_1: quant_q5_1,
    GGMLType.Q8_0: quant_q8_0,
    GGMLType.Q2_K: quant_q2_k,
    GGMLType.Q3_K: quant_q3_k,
    GGMLType.IQ4_NL: quant_iq4_nl,
    GGMLType.IQ4_XS: quant_iq4_xs,
    GGMLType.Q4_K: quant_q4_k,
    GGMLType.Q5_K: quant_q5_k,
    GGMLType.Q6_K: quant_q6_k,
}


def quantize(x: np.ndarray, t: GGMLType) -> np.ndarray:
    return QUANT[GGMLType(t)](np.ascontiguousarray(x, dtype=np.float32).ravel())
