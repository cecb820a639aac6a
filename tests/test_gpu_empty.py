"""Empty batches through the batched device entry points: B = 0 streams must give empty
results of the right shape (the C ABI returns OFS_OK without launching), like the
reference's empty-array returns for short inputs (sc.py:50-52, minn.py:81-82)."""
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from ofdm_sync_amd import combined_sc_min, minn, minn_rtl, park, sc, sync_aa, zc_freq  # noqa: E402


def _x(B, nb, T, dtype=torch.complex64):
    return torch.zeros((B, nb, T), dtype=dtype, device="cuda")


@pytest.mark.parametrize("dtype", [torch.complex64, torch.complex128])
def test_aa_empty_batch(dtype):
    r = sync_aa.aa_detect_streaming_batched(_x(0, 1, 1024, dtype), 512)
    assert r.M.shape == (0, 1024) and r.n_events.shape == (0,)
    r = sync_aa.aa_detect_streaming_batched(_x(3, 1, 0, dtype), 512)
    assert r.M.shape == (3, 0)


def test_window_metrics_empty_batch():
    for fn in (sc.sc_streaming_metric_batched, combined_sc_min.schmidl_cox_streaming_metric_batched,
               minn.minn_streaming_metric_batched):
        M, P, R = fn(_x(0, 1, 4096), 2048)
        assert M.shape == (0, 2049) and P.shape == (0, 2049) and R.shape == (0, 2049)
    ds, M, P, E = park.park_streaming_metric_batched(_x(0, 1, 4096), 256)
    assert M.shape[0] == 0 and P.shape[0] == 0 and E.shape[0] == 0


def test_minn_rtl_and_zc_freq_empty_batch():
    x16 = torch.zeros((0, 1, 1024, 2), dtype=torch.int16, device="cuda")
    b = minn_rtl.minn_rtl_batched(x16, 64)
    assert b.corr_total.shape == (0, 1024)
    m = zc_freq.compute_frequency_metric_batched(_x(0, 1, 4096), N=4096, cp=0)
    assert m.shape == (0, 1)
    m, pk, pv = zc_freq.compute_frequency_metric_rocfft_batched(_x(0, 1, 4096), N=4096, cp=0, return_peak=True)
    assert m.shape == (0, 1) and pk.shape == (0,)
