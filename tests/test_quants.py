"""CPU tests: GGML block formats (bit-exact layouts the HIP kernels mirror)."""
import numpy as np
import pytest

from aios_amd.gguf.quants import (BLOCK_INFO, GGMLType, dequantize, kquant_pack_scale_min, kquant_scale_min,
                                  quantize, type_size)

FORMATS = [GGMLType.Q4_0, GGMLType.Q8_0, GGMLType.Q4_K, GGMLType.Q5_K, GGMLType.Q6_K, GGMLType.F16, GGMLType.BF16,
           GGMLType.Q4_1, GGMLType.Q5_0, GGMLType.Q5_1, GGMLType.Q2_K, GGMLType.Q3_K, GGMLType.IQ4_NL,
           GGMLType.IQ4_XS]
TOL = {GGMLType.Q4_0: 0.2, GGMLType.Q8_0: 0.01, GGMLType.Q4_K: 0.12, GGMLType.Q5_K: 0.06, GGMLType.Q6_K: 0.03,
       GGMLType.F16: 1e-3, GGMLType.BF16: 1e-2, GGMLType.Q4_1: 0.12, GGMLType.Q5_0: 0.06, GGMLType.Q5_1: 0.06,
       GGMLType.Q2_K: 0.4, GGMLType.Q3_K: 0.22, GGMLType.IQ4_NL: 0.12, GGMLType.IQ4_XS: 0.12}


@pytest.mark.parametrize("t", FORMATS)
def test_roundtrip_error(t):
    rng = np.random.default_rng(0)
    x = rng.standard_normal(256 * 16).astype(np.float32)
    raw = quantize(x, t)
    assert raw.size == type_size(t, x.size)
    y = dequantize(raw, t)
    rel = np.sqrt(np.mean((x - y) ** 2)) / np.sqrt(np.mean(x ** 2))
    assert rel < TOL[t], (t, rel)


def test_scale_min_pack_roundtrip():
    rng = np.random.default_rng(1)
    sc = rng.integers(0, 64, (50, 8))
    mn = rng.integers(0, 64, (50, 8))
    s2, m2 = kquant_scale_min(kquant_pack_scale_min(sc, mn))
    assert (s2 == sc).all() and (m2 == mn).all()


def test_q4k_hand_block():
    # d=1, dmin=0.5, all scales 1, mins 2, nibble pattern known
    d = np.array([1.0], np.float16).view(np.uint8)
    dmin = np.array([0.5], np.float16).view(np.uint8)
    scales = kquant_pack_scale_min(np.ones((1, 8), int), np.full((1, 8), 2))[0]
    qs = np.arange(128, dtype=np.uint8) % 16 | ((np.arange(128, dtype=np.uint8) % 7) << 4)
    blk = np.concatenate([d, dmin, scales, qs])
    y = dequantize(blk, GGMLType.Q4_K)
    # group 0 low nibbles -> elements 0..31
    assert np.allclose(y[:32], (np.arange(32) % 16) * 1.0 - 1.0)
    assert np.allclose(y[32:64], (np.arange(32) % 7) * 1.0 - 1.0)


def test_q6k_matches_formula():
    rng = np.random.default_rng(2)
    raw = rng.integers(0, 256, 210 * 3, dtype=np.uint8)
    raw.reshape(3, 210)[:, 208:210] = np.array([0.01], np.float16).view(np.uint8)
    y = dequantize(raw, GGMLType.Q6_K).reshape(3, 256)
    b = raw.reshape(3, 210)
    # scalar reimplementation of the published reference loop
    for i in range(3):
        ql, qh, sc = b[i, :128].astype(int), b[i, 128:192].astype(int), b[i, 192:208].view(np.int8).astype(int)
        d = float(b[i, 208:210].view(np.float16)[0])
        out = np.zeros(256)
        for n in range(2):
            for l in range(32):
                is_ = l // 16
                q1 = ((ql[64 * n + l] & 0xF) | (((qh[32 * n + l] >> 0) & 3) << 4)) - 32
                q2 = ((ql[64 * n + l + 32] & 0xF) | (((qh[32 * n + l] >> 2) & 3) << 4)) - 32
                q3 = ((ql[64 * n + l] >> 4) | (((qh[32 * n + l] >> 4) & 3) << 4)) - 32
                q4 = ((ql[64 * n + l + 32] >> 4) | (((qh[32 * n + l] >> 6) & 3) << 4)) - 32
                out[128 * n + l] = d * sc[8 * n + is_] * q1
                out[128 * n + l + 32] = d * sc[8 * n + is_ + 2] * q2
                out[128 * n + l + 64] = d * sc[8 * n + is_ + 4] * q3
                out[128 * n + l + 96] = d * sc[8 * n + is_ + 6] * q4
        assert np.allclose(y[i], out, atol=1e-6)


def test_block_info_sizes():
    assert BLOCK_INFO[GGMLType.Q4_K] == (256, 144)
    assert BLOCK_INFO[GGMLType.Q6_K] == (256, 210)
    assert BLOCK_INFO[GGMLType.Q5_K] == (256, 176)
    assert BLOCK_INFO[GGMLType.Q8_0] == (32, 34)
    assert BLOCK_INFO[GGMLType.Q4_0] == (32, 18)


def test_q2k_hand_block():
    """Q2_K layout: 16 (scale | min << 4) bytes, 64 quant bytes (element j = 128 n + 32 g + t at bits 2 g of
    byte 32 n + t), f16 d, f16 dmin; y = d * scale(j >> 4) * q - dmin * min(j >> 4).  (Parity with llama.cpp's
    own files unpinned: no Q2_K fixture or independent decoder is available offline.)"""
    sc = np.arange(16, dtype=np.uint8) % 15 + 1
    mn = (np.arange(16, dtype=np.uint8) * 3) % 16
    q = (np.arange(256) * 7 + 3) % 4
    qs = np.zeros(64, np.uint8)
    for j in range(256):
        n, g, t = j >> 7, (j >> 5) & 3, j & 31
        qs[32 * n + t] |= q[j] << (2 * g)
    blk = np.concatenate([sc | (mn << 4), qs, np.array([0.5], np.float16).view(np.uint8),
                          np.array([0.25], np.float16).view(np.uint8)])
    y = dequantize(blk, GGMLType.Q2_K)
    want = np.array([0.5 * sc[j >> 4] * q[j] - 0.25 * mn[j >> 4] for j in range(256)], np.float32)
    np.testing.assert_array_equal(y, want)


def test_q3k_hand_block():
    """Q3_K layout: 32 high-bit bytes (bit j >> 5 of byte j & 31), 64 quant bytes (as Q2_K), twelve bytes of
    sixteen 6-bit scales stored + 32 (low nibbles in bytes 0-7, top 2 bits in bytes 8-11), f16 d;
    y = d * (scale - 32) * (low2 - (high ? 0 : 4)).  (Parity with llama.cpp's own files unpinned.)"""
    from aios_amd.gguf.quants import q3k_scales

    v = (np.arange(16) * 5 + 1) % 64  # stored 6-bit scales
    scb = np.zeros(12, np.int64)
    for s_ in range(16):
        g, k = s_ >> 2, s_ & 3
        scb[(4 if g & 1 else 0) + k] |= (v[s_] & 0xF) << (4 if g & 2 else 0)
        scb[8 + k] |= (v[s_] >> 4) << (2 * g)
    np.testing.assert_array_equal(q3k_scales(scb.astype(np.uint8).reshape(1, 12))[0], v - 32)
    u = (np.arange(256) * 5 + 1) % 8  # value + 4
    hm, qs = np.zeros(32, np.uint8), np.zeros(64, np.uint8)
    for j in range(256):
        hm[j & 31] |= (u[j] >> 2) << (j >> 5)
        qs[32 * (j >> 7) + (j & 31)] |= (u[j] & 3) << (2 * ((j >> 5) & 3))
    blk = np.concatenate([hm, qs, scb.astype(np.uint8), np.array([0.125], np.float16).view(np.uint8)])
    y = dequantize(blk, GGMLType.Q3_K)
    want = np.array([0.125 * (v[j >> 4] - 32) * (u[j] - 4) for j in range(256)], np.float32)
    np.testing.assert_array_equal(y, want)


def test_iq4_hand_blocks():
    """IQ4_NL (f16 d + Q4_0-ordered nibbles indexing 16 fixed levels) and IQ4_XS (eight 32-element runs of the
    same, each scaled by d x (6-bit scale - 32): low nibbles in bytes 4-7, top bits in the u16 at byte 2).
    (Parity with llama.cpp's own files unpinned.)"""
    from aios_amd.gguf.quants import IQ4_LEVELS

    idx = (np.arange(32) * 5 + 3) % 16
    qs = (idx[:16] | (idx[16:] << 4)).astype(np.uint8)
    y = dequantize(np.concatenate([np.array([0.5], np.float16).view(np.uint8), qs]), GGMLType.IQ4_NL)
    np.testing.assert_array_equal(y, 0.5 * IQ4_LEVELS[idx])
    v = (np.arange(8) * 9 + 5) % 64
    sh = sum(int((v[i] >> 4) & 3) << (2 * i) for i in range(8))
    sl = np.zeros(4, np.uint8)
    for i in range(8):
        sl[i // 2] |= (v[i] & 0xF) << (4 * (i % 2))
    idx = (np.arange(256) * 7 + 1) % 16
    q = idx.reshape(8, 32)
    qs = (q[:, :16] | (q[:, 16:] << 4)).astype(np.uint8).ravel()
    blk = np.concatenate([np.array([0.25], np.float16).view(np.uint8), np.array([sh], np.uint16).view(np.uint8), sl, qs])
    y = dequantize(blk, GGMLType.IQ4_XS)
    np.testing.assert_array_equal(y, (0.25 * np.repeat(v - 32, 32) * IQ4_LEVELS[idx]).astype(np.float32))
