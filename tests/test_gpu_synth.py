"""GPU: batched stream synthesis (csrc/synth.hip).  RNG parity with numpy is
not a goal (distribution only): the tests check determinism, the noiseless signal path
(shift + CFO tone, against a numpy restatement of core.apply_cfo), the noise statistics, the
int12 ADC, and that the sync detector recovers the drawn CFO and offset."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from ofdm_sync_amd import synth, sync_aa  # noqa: E402


def test_deterministic_per_seed():
    base = synth.faded_base(512, "cir1", (0, 1))
    a = synth.synth_batch(base, 64, 1024, seed=7)
    b = synth.synth_batch(base, 64, 1024, seed=7)
    c = synth.synth_batch(base, 64, 1024, seed=8)
    assert torch.equal(a, b) and not torch.equal(a, c)
    assert a.shape == (64, 2, 1024) and a.dtype == torch.complex64


def test_noiseless_path_is_shift_times_tone():
    base = synth.faded_base(256, "cir2", (1,))
    B, T, fs = 40, 700, 15.36e6
    x, p = synth.synth_batch(base, B, T, snr_db=(400.0, 400.0), cfo_hz=(-3000.0, 3000.0), fs=fs, seed=3,
                             dtype=torch.complex128, return_params=True)
    x, p = x.cpu().numpy(), p.cpu().numpy()
    n = np.arange(T)
    pad = np.concatenate([base[0], np.zeros(T + 200)])
    for b in range(B):
        off, snr, cfo = int(p[b, 0]), p[b, 1], p[b, 2]
        assert 0 <= off < 128 and snr == 400.0 and -3000.0 <= cfo <= 3000.0
        ref = pad[off:off + T] * np.exp(1j * 2 * np.pi * cfo * n / fs)      # core.apply_cfo
        assert np.max(np.abs(x[b, 0] - ref)) < 1e-12
    assert len(set(p[:, 0].astype(int))) > 10                               # offsets spread


def test_noise_statistics():
    base = np.zeros((1, 16), complex)
    B, T = 256, 4096
    x, p = synth.synth_batch(base, B, T, snr_db=(0.0, 20.0), cfo_hz=(0.0, 0.0), seed=11, dtype=torch.complex128,
                             return_params=True)
    x, p = x.cpu().numpy()[:, 0], p.cpu().numpy()
    var = np.mean(np.abs(x) ** 2, axis=1)
    expect = 10 ** (-p[:, 1] / 10)
    assert np.all(np.abs(var / expect - 1) < 0.1)                           # 4096 samples: ~2 % sd
    z = (x / np.sqrt(expect / 2)[:, None]).ravel()
    for comp in (z.real, z.imag):
        assert abs(np.mean(comp)) < 0.01 and abs(np.var(comp) - 1) < 0.01
        assert abs(np.mean(comp ** 4) - 3) < 0.05                           # Gaussian kurtosis
    assert abs(np.mean(z.real * z.imag)) < 0.01
    assert np.all((p[:, 1] >= 0) & (p[:, 1] <= 20)) and np.std(p[:, 1]) > 4


def test_int12_adc():
    base = synth.faded_base(512, "cir1", (1,))
    x = synth.synth_batch(base, 16, 1024, seed=5, dtype=torch.int16, adc_scale=600.0)
    assert x.shape == (16, 1, 1024, 2) and x.dtype == torch.int16
    assert int(x.min()) >= -2048 and int(x.max()) <= 2047 and int(x.abs().max()) > 1000


def test_detector_recovers_drawn_cfo_and_offset():
    L, fs = 512, 15.36e6
    base = synth.faded_base(L, None, (0,))
    x, p = synth.synth_batch(base, 32, 1024 + 128, snr_db=(30.0, 30.0), cfo_hz=(-4000.0, 4000.0), fs=fs, seed=9,
                             return_params=True)
    out = sync_aa.aa_detect_streaming_batched(x, L=L)
    p = p.cpu().numpy()
    assert bool((out.n_events >= 1).all())
    cfo = out.ev_real[:, 0, 3].cpu().numpy()
    assert np.max(np.abs(cfo - p[:, 2])) < 30.0                              # Hz, at 30 dB
    # no offset: the [A][A] |P|^2 peak sits at the end of the second half, n = 2L - 1
    x0 = synth.synth_batch(base, 8, 1024 + 128, max_offset=0, snr_db=(30.0, 30.0), cfo_hz=(-4000.0, 4000.0),
                           fs=fs, seed=10)
    o0 = sync_aa.aa_detect_streaming_batched(x0, L=L)
    peak = o0.ev_int[:, 0, 0].cpu().numpy()
    assert np.max(np.abs(peak - (2 * L - 1))) <= 2
