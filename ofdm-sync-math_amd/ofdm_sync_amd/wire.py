"""The RTL detector's sample wire formats (host-side packing; the kernels decode OFS_CP12 words
themselves, 3 bytes per sample and channel instead of 4 for int16 I/Q).

* AXIS word (ref/test_minn_preamble_detector.py:41-47 ``_pack_axis_samples``,
  ref/minn_preamble_detector.sv:152-155): per time index one word of the channels' 24-bit
  groups, channel c at bit 24*c with I in bits 0-11 and Q in 12-23 (two's complement).  In
  memory: [.., T, 3 * n_ch] uint8, little-endian (OFS_CP12).
* ``docs/preamble_test_vector.hex``: one sample per line, ``(re12 << 12) | im12`` as 6 hex
  digits (Re in the UPPER 12 bits, the opposite order of the AXIS group), ``//`` comments.
"""
from __future__ import annotations

import numpy as np

MASK12 = 0xFFF


def _sext12(v: np.ndarray) -> np.ndarray:
    v = np.asarray(v, np.int64) & MASK12
    return np.where(v >= 0x800, v - 0x1000, v)


def pack_axis(iq: np.ndarray) -> np.ndarray:
    """int12 I/Q [.., n_ch, T, 2] (int16 values in [-2048, 2047]) -> AXIS words
    [.., T, 3 * n_ch] uint8 (ofdm's _pack_axis_samples, one word per time index)."""
    iq = np.asarray(iq)
    if iq.shape[-1] != 2 or iq.ndim < 3:
        raise ValueError("iq must be [.., n_ch, T, 2]")
    if iq.min(initial=0) < -2048 or iq.max(initial=0) > 2047:
        raise ValueError("samples must fit 12 bits")
    n_ch = iq.shape[-3]
    i = np.moveaxis(iq[..., 0].astype(np.int64) & MASK12, -2, -1)     # [.., T, n_ch]
    q = np.moveaxis(iq[..., 1].astype(np.int64) & MASK12, -2, -1)
    g = (i | (q << 12)).astype(np.uint32)                              # 24-bit group per channel
    out = np.empty(g.shape[:-1] + (3 * n_ch,), np.uint8)
    for c in range(n_ch):
        for k in range(3):
            out[..., 3 * c + k] = (g[..., c] >> (8 * k)) & 0xFF
    return out


def unpack_axis(words: np.ndarray) -> np.ndarray:
    """AXIS words [.., T, 3 * n_ch] uint8 -> int16 I/Q [.., n_ch, T, 2]."""
    w = np.asarray(words, np.uint32)
    n_ch = w.shape[-1] // 3
    out = []
    for c in range(n_ch):
        g = w[..., 3 * c] | (w[..., 3 * c + 1] << 8) | (w[..., 3 * c + 2] << 16)
        out.append(np.stack([_sext12(g), _sext12(g >> 12)], axis=-1))
    return np.stack(out, axis=-3).astype(np.int16)


def read_hex_vector(path: str) -> np.ndarray:
    """docs/preamble_test_vector.hex -> int12 I/Q [T, 2] (int16)."""
    vals = []
    for line in open(path):
        s = line.split("//", 1)[0].strip()               # trailing comments name the values
        if not s:
            continue
        v = int(s, 16)
        vals.append((_sext12(v >> 12), _sext12(v)))
    return np.array(vals, np.int16).reshape(-1, 2)
