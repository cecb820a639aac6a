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
    assert bool((o0.n_events >= 1).all())                   # slot 0 is stored (slots past n_events are not)
    peak = o0.ev_int[:, 0, 0].cpu().numpy()
    assert np.max(np.abs(peak - (2 * L - 1))) <= 2


# ---------------- ofs_synth_frames: the whole run_single_test chain per stream -----------------
def _host_frame(fr, b, n_sym=2, fs=15.36e6):
    """numpy restatement of sync_aa.run_single_test's chain for stream b without noise/ADC, from
    the QPSK draws the GPU reports (synth.qpsk_symbol / frame pinned to the reference)."""
    ph = fr.phases[b].cpu().numpy()
    syms = [synth.qpsk_symbol(ph[s]) for s in range(n_sym)]
    f = synth.frame(fr.preamble, syms)
    rx = np.stack([np.convolve(f, fr.cir[br]) for br in range(fr.cir.shape[0])])
    cfo = float(fr.params[b, 2])
    return rx * np.exp(1j * 2 * np.pi * cfo * np.arange(rx.shape[1]) / fs)


def test_frames_noiseless_equal_host_restatement():
    B = 12
    fr = synth.frames_batch(B, snr_db=(400.0, 400.0), seed=11, dtype=torch.complex128, return_phases=True)
    x = fr.x.cpu().numpy()
    assert x.shape == (B, 2, 500 + 1024 + 2 * 1096 + 500 + 1099)
    for b in range(B):
        ref = _host_frame(fr, b)
        assert np.max(np.abs(x[b] - ref)) < 1e-11
    ph = fr.phases.cpu().numpy()
    assert ph.max() <= 3 and len(np.unique(ph[:, 0, :10], axis=0)) == B      # every stream its own payload


def test_frames_noise_level_and_window():
    B, fs = 64, 15.36e6
    kw = dict(cir="cir2", seed=5, dtype=torch.complex128, cfo_hz=(700.0, 700.0))
    clean = synth.frames_batch(B, snr_db=(400.0, 400.0), **kw)
    noisy = synth.frames_batch(B, snr_db=(6.0, 6.0), **kw)
    y, r = clean.x.cpu().numpy(), noisy.x.cpu().numpy()
    Lout = y.shape[-1]
    tone = np.exp(1j * 2 * np.pi * 700.0 * np.arange(Lout) / fs)
    w = (r - y) * np.conj(tone)                                  # sd * g per branch
    p_sig = np.mean(np.abs(y) ** 2, axis=-1)                     # mean |y_br|^2 (channel.py-style)
    ratio = np.mean(np.abs(w) ** 2, axis=-1) / (p_sig / 10 ** 0.6)
    assert abs(float(ratio.mean()) - 1.0) < 0.01 and float(ratio.std()) < 0.05
    # a window: same samples, shifted by the drawn offset
    win = synth.frames_batch(B, 1024, snr_db=(6.0, 6.0), win_start=300, max_offset=200, **kw)
    st = win.params[:, 0].cpu().numpy().astype(int)
    assert st.min() >= 300 and st.max() < 500 and len(set(st)) > 20
    xw = win.x.cpu().numpy()
    for b in range(B):
        assert np.max(np.abs(xw[b] - r[b, :, st[b]:st[b] + 1024])) < 1e-12


def test_frames_adc_codes():
    B = 32
    codes = synth.frames_batch(B, snr_db=(10.0, 10.0), full_scale_ratio=1.0, seed=9, dtype=torch.int16)
    deq = synth.frames_batch(B, snr_db=(10.0, 10.0), full_scale_ratio=1.0, seed=9, dtype=torch.complex128)
    c = codes.x.cpu().numpy().astype(np.float64)
    assert c.min() >= -2048 and c.max() <= 2047
    fsc = deq.params[:, 3].cpu().numpy()
    d = deq.x.cpu().numpy()
    assert np.array_equal(d.real, c[..., 0] / 2048 * fsc[:, None, None])       # quantize_adc's values
    assert np.array_equal(d.imag, c[..., 1] / 2048 * fsc[:, None, None])
    # full scale = rms over both branches: with ratio 1 about 16 % of the I/Q values clip
    clipped = np.mean((c == -2048) | (c == 2047))
    assert 0.05 < clipped < 0.35


def test_frames_detected_like_run_single_test():
    """2 antennas, cir1, 10 dB, 1024 preamble, 12-bit ADC at FS 1.0: the detector finds every frame,
    timing within the reference's multipath range of the true start (sync_aa design doc: +77..+94
    samples on multipath; grid golden cir1 +83)."""
    B = 64
    fr = synth.frames_batch(B, snr_db=(10.0, 10.0), full_scale_ratio=1.0, seed=21, dtype=torch.complex64)
    out = sync_aa.aa_detect_streaming_batched(fr.x, L=512, outputs=())
    n = out.n_events.cpu().numpy()
    assert (n >= 1).all()
    agg = np.sum(np.abs(fr.cir) ** 2, axis=0)
    true_start = 500 + int(np.argmax(agg))                       # sync_aa.py:631-634, :718-719
    fs_ = out.ev_int[:, 0, 3].cpu().numpy()
    assert np.all(np.abs(fs_ - true_start) < 150)
    cfo = out.ev_real[:, 0, 3].cpu().numpy()
    assert np.all(np.abs(cfo - fr.params[:, 2].cpu().numpy()) < 300.0)
