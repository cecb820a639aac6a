"""GPU: the packed 12-bit AXIS wire format (OFS_CP12, 3 bytes per sample and channel) decoded
inside the integer-exact kernels.  The reference's own word layout (ref/test_minn_preamble_
detector.py:41-47) and its preamble test vector (docs/preamble_test_vector.hex) drive the
detector; every output must be BIT-IDENTICAL to the int16 I/Q path on the same samples (same
integer arithmetic, only the load differs), and the int16 path is pinned to the reference by
test_gpu_parity / test_gpu_exact."""
import os

import numpy as np
import pytest

import ofdm_oracle as O
from conftest import GOLDEN

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from ofdm_sync_amd import _lib, minn_rtl, sync_aa, synth, wire  # noqa: E402


def _both(iq, **kw):
    """iq int16 [B, n_ch, T, 2] -> (int16-path result, CP12-path result)."""
    a = sync_aa.aa_detect_streaming_batched(torch.from_numpy(iq).cuda(), **kw)
    p = wire.pack_axis(iq)
    b = sync_aa.aa_detect_streaming_batched(torch.from_numpy(p).cuda(), **kw)
    return a, b


def _same_aa(a, b):
    for k in ("P", "R", "M", "valid", "n_events"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    n = a.n_events.cpu().numpy()
    for s in range(len(n)):
        assert torch.equal(a.ev_int[s, :n[s]], b.ev_int[s, :n[s]])
        assert torch.equal(a.ev_real[s, :n[s]], b.ev_real[s, :n[s]])


@pytest.mark.parametrize("n_ch", [1, 2])
def test_hex_preamble_vector_through_the_detector(n_ch):
    """docs/preamble_test_vector.hex between 500-sample pads (the docs CSV geometry, L = 512):
    CP12 == int16 I/Q bit for bit, P and R equal the oracle's exact integers, and the event is
    the reference's (peak 1523, frame_start 500)."""
    pre = wire.read_hex_vector(os.path.join(GOLDEN, "preamble_test_vector.hex"))     # [1024, 2]
    x = np.zeros((n_ch, 2024, 2), np.int16)
    for c in range(n_ch):
        x[c, 500:1524] = pre if c == 0 else -pre                       # second channel: sign flip
    iq = x[None]
    assert _lib.lib().ofs_aa_plan(_lib.CP12, _lib.FP64, n_ch, 2024, 512) >= 2000
    a, b = _both(iq, L=512)
    _same_aa(a, b)
    xc = (x[..., 0] + 1j * x[..., 1]).astype(np.complex128)
    P, R, M, valid = O.aa_metric(xc, 512)
    assert np.array_equal(b.P[0].cpu().numpy(), P) and np.array_equal(b.R[0].cpu().numpy(), R)
    assert int(b.n_events[0]) == 1
    pk, gs, ge, fs = b.ev_int[0, 0].tolist()
    assert pk == 1523 and fs == 500


@pytest.mark.parametrize("n_ch,T,L", [(2, 5315, 512), (2, 5315, 128), (1, 1023, 128), (1, 4096, 256), (2, 7, 64)])
def test_cp12_equals_int16_on_adc_frames(n_ch, T, L):
    """run_single_test-style frames (12-bit ADC at FS 1.0, ofs_synth_frames) through both formats:
    bit-identical P, R, M, valid, events (odd T and a stream shorter than a row included)."""
    fr = synth.frames_batch(33, T, n_br=n_ch, snr_db=(5.0, 15.0), full_scale_ratio=1.0, seed=T + L,
                            dtype=torch.int16)
    iq = fr.x.cpu().numpy()
    a, b = _both(iq, L=L)
    _same_aa(a, b)
    assert _lib.lib().ofs_aa_plan(_lib.CP12, _lib.FP64, n_ch, T, L) >= 2000


@pytest.mark.parametrize("n_br,Q", [(1, 64), (2, 64), (2, 512), (1, 128)])
def test_cp12_minn_rtl_equals_int16(n_br, Q):
    fr = synth.frames_batch(21, 4 * Q + 2000, n_br=n_br, snr_db=(5.0, 15.0), full_scale_ratio=1.0, seed=Q + n_br,
                            dtype=torch.int16)
    iq = fr.x.cpu().numpy()
    assert _lib.lib().ofs_rtl_plan(_lib.CP12, n_br, iq.shape[2], Q) > 2000
    a = minn_rtl.minn_rtl_batched(torch.from_numpy(iq).cuda(), Q)
    b = minn_rtl.minn_rtl_batched(torch.from_numpy(wire.pack_axis(iq)).cuda(), Q)
    for k in ("corr_total", "corr_positive", "smooth_metric", "energy_total", "corr_scaled", "energy_scaled",
              "metric_valid", "above_threshold", "n_events", "open_gate_start"):
        assert torch.equal(getattr(a, k), getattr(b, k)), k
    n = a.n_events.cpu().numpy()
    for s in range(len(n)):
        assert torch.equal(a.events[s, :n[s]], b.events[s, :n[s]])


def test_cp12_rejected_where_unsupported():
    iq = np.zeros((2, 1, 64, 2), np.int16)
    p = torch.from_numpy(wire.pack_axis(iq)).cuda()
    with pytest.raises(ValueError):
        sync_aa.aa_detect_streaming_batched(p, L=100)                       # L not a whole row
    with pytest.raises(ValueError):
        sync_aa.aa_detect_streaming_batched(p, L=64, precision="fp32")      # fp32 engine: no CP12
    assert _lib.lib().ofs_aa_plan(_lib.CP12, _lib.FP32, 1, 64, 64) < 0
