"""CPU: host-side logic of the Python mirror that needs no GPU."""
import pytest
import numpy as np

from ofdm_sync_amd import zc, zc_v2


def test_zc_build_pss_symbol_leaves_zc_v2_globals_alone():
    """zc.build_pss_symbol uses zc's own N_FFT / CYCLIC_PREFIX (read at call time) without
    overwriting zc_v2's module globals (a caller who re-parameterised zc_v2 keeps it)."""
    n0, cp0 = zc_v2.N_FFT, zc_v2.CYCLIC_PREFIX
    zc_v2.N_FFT, zc_v2.CYCLIC_PREFIX = 256, 16
    zc.N_FFT, zc.CYCLIC_PREFIX = 512, 64
    try:
        s = zc.build_pss_symbol(include_cp=True)
        assert s.shape == (512 + 64,)
        assert (zc_v2.N_FFT, zc_v2.CYCLIC_PREFIX) == (256, 16)
        assert zc_v2.build_pss_symbol(include_cp=True).shape == (256 + 16,)
        np.testing.assert_allclose(s[64:], zc_v2.build_pss_symbol(n_fft=512, cyclic_prefix=0))
    finally:
        zc_v2.N_FFT, zc_v2.CYCLIC_PREFIX = n0, cp0
        zc.N_FFT, zc.CYCLIC_PREFIX = 2048, 512


# ---- input builders of the synthesis, pinned to the reference's own outputs -----------------
import os  # noqa: E402

from conftest import GOLDEN  # noqa: E402
from ofdm_sync_amd import synth  # noqa: E402


def _syn():
    return np.load(os.path.join(GOLDEN, "synth_builders.npz"), allow_pickle=False)


def test_load_cir_matches_reference():
    d = _syn()
    for name in ("cir1", "cir2"):
        assert np.array_equal(synth.load_cir(name), d[name])          # channel.load_measured_cir


def test_aa_preamble_matches_reference():
    d = _syn()
    for ln in (1024, 512, 256):
        np.testing.assert_allclose(synth.aa_preamble(ln), d[f"pre{ln}"], rtol=0, atol=1e-12)
    g = np.load(os.path.join(GOLDEN, "aa_clean_L512.npz"))
    np.testing.assert_allclose(synth.aa_preamble(1024), g["x"][0, 500:1524], rtol=0, atol=1e-12)


def test_qpsk_symbol_and_frame_chain_match_reference():
    d = _syn()
    N, cp, K, pre, post = (int(v) for v in d["geometry"])
    assert (N, cp, K, pre, post) == (synth.N_FFT, synth.CYCLIC_PREFIX, synth.NUM_ACTIVE, synth.PRE_PAD, synth.POST_PAD)
    syms = []
    for q, ref in zip(d["qpsk_values"], d["qpsk_symbols"]):
        ph = np.mod(np.round((np.angle(q * np.sqrt(2)) / (np.pi / 4) - 1) / 2), 4).astype(int)
        s = synth.qpsk_symbol(ph)
        np.testing.assert_allclose(s, ref, rtol=0, atol=1e-12)
        syms.append(s)
    fr = synth.frame(synth.aa_preamble(1024), syms[:2])
    cir = synth.load_cir("cir1")[:2]
    rx = np.stack([np.convolve(fr, cir[a]) for a in range(2)])
    n = np.arange(rx.shape[1])
    rx = rx * np.exp(1j * 2 * np.pi * 500.0 * n / 15.36e6)
    np.testing.assert_allclose(rx, d["frame_cir1_cfo500"], rtol=0, atol=1e-12)


# ---- wire formats (OFS_CP12 packing, the reference's .hex test vector) ----------------------
from ofdm_sync_amd import wire  # noqa: E402


def test_axis_pack_matches_reference_packing():
    """Bit layout of ref/test_minn_preamble_detector.py:41-47 (_pack_axis_samples), restated:
    word = ch0_i | ch0_q << 12 | ch1_i << 24 | ch1_q << 36 (12-bit two's complement fields)."""
    rng = np.random.default_rng(1)
    iq = rng.integers(-2048, 2048, size=(3, 2, 17, 2)).astype(np.int16)    # [B, ch, T, IQ]
    w = wire.pack_axis(iq)
    assert w.shape == (3, 17, 6) and w.dtype == np.uint8
    m = (1 << 12) - 1
    for b in range(3):
        for n in range(17):
            word = ((int(iq[b, 0, n, 0]) & m) | ((int(iq[b, 0, n, 1]) & m) << 12) |
                    ((int(iq[b, 1, n, 0]) & m) << 24) | ((int(iq[b, 1, n, 1]) & m) << 36))
            assert int.from_bytes(bytes(w[b, n]), "little") == word
    assert np.array_equal(wire.unpack_axis(w), iq)


def test_hex_vector_is_the_preamble():
    """docs/preamble_test_vector.hex = (re12 << 12) | im12 of round(preamble * 1024)."""
    iq = wire.read_hex_vector(os.path.join(GOLDEN, "preamble_test_vector.hex"))
    pre = synth.aa_preamble(1024)
    assert iq.shape == (1024, 2)
    assert np.array_equal(iq[:, 0], np.round(pre.real * 1024)) and np.array_equal(iq[:, 1], np.round(pre.imag * 1024))


from ofdm_sync_amd import zc_freq  # noqa: E402


def test_rocfft_default_chunk_sizing():
    """Chunked rocFFT plans (zc_freq.default_chunk): a multiple of the branch count, sized to
    about CHUNK_BYTES of spectrum, 0 (one execution) when one chunk would cover the batch."""
    N, esz = 4096, 8
    per = zc_freq.CHUNK_BYTES // (N * esz)
    assert zc_freq.default_chunk(1 << 20, 1, N, esz) == per
    c = zc_freq.default_chunk(1 << 20, 3, N, esz)
    assert c % 3 == 0 and 0 < c <= per
    assert zc_freq.default_chunk(per, 1, N, esz) == 0
    assert zc_freq.default_chunk(10, 2, N, esz) == 0
    assert zc_freq.default_chunk(1 << 20, 2, 1 << 26, 16) == 2        # never below one stream's branches


def test_rocfft_auto_layout_prices_the_rows_plan():
    """layout="auto" takes the rows plan only where its extra FFT work (about T / offsets) is small:
    the reference's sliding shape (T 4242, N 2048 + cp 512: 1683 offsets) yes; few offsets on a long
    row (N 4096, cp 0, T 4103: 8 offsets, ~500x the FFTs) no; never when chunk (windows of the
    offsets layout) is given; rows_per_execution (the rows layout's size) selects rows under auto and is
    refused with "offsets"; the rows layout refuses chunk and unprunable templates."""
    pick = zc_freq.pick_rows_layout
    assert pick("auto", True, None, 4242, 4242 - 2560 + 1)
    assert not pick("auto", True, None, 4103, 8)
    assert not pick("auto", True, 2048, 4242, 1683)
    assert not pick("auto", False, None, 4242, 1683)
    assert not pick("auto", True, None, 100, 7)                       # below ROWS_MIN_OFFSETS
    assert pick("auto", True, None, 4 * 1000, 1000) and not pick("auto", True, None, 4 * 1000 + 1, 1000)
    assert pick("rows", True, None, 4103, 8) and not pick("offsets", True, None, 4242, 1683)
    assert pick("auto", True, None, 4103, 8, rows_per_execution=4)     # the rows-only size selects rows
    for bad in (dict(layout="rows", prunable=True, chunk=64), dict(layout="rows", prunable=False, chunk=None),
                dict(layout="dense", prunable=True, chunk=None),
                dict(layout="offsets", prunable=True, chunk=None, rows_per_execution=4),
                dict(layout="auto", prunable=True, chunk=64, rows_per_execution=4),
                dict(layout="auto", prunable=False, chunk=None, rows_per_execution=4)):
        with pytest.raises(ValueError):
            pick(bad["layout"], bad["prunable"], bad["chunk"], 4242, 1683, bad.get("rows_per_execution"))
    assert zc_freq.rows_per_exec(10, 2, 4242, 62, 8) == 10
    assert zc_freq.rows_per_exec(1 << 20, 2, 4242, 62, 8) % 2 == 0
