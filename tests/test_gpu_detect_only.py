"""Detect-only mode of the sync_aa detector (8 B/sample + per-stream events): with
P/R/M/valid not requested the kernels skip those stores and keep the events on chip.  The
events must be identical to the ones of the full call on every dispatch plan (fp32 fast path,
int12 integer-exact path, general engine with fused events); the general engine's multi-tile
plan still gets P/M buffers from the mirror.  Exact equality: same kernel, same arithmetic (the
register-staged fp32 detect-only kernel runs 4 samples per lane per row with fp32 row scans,
aa_fast.hip pick_e_do / scan32, so its full call is compared at that row width and scan precision:
OFS_FAST_E=4, OFS_FAST_SCAN=32; with OFS_FAST_SCAN_DO=64 it equals the fp64-scan storing kernel)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from ofdm_sync_amd import _lib, synth, sync_aa  # noqa: E402


def _batch(kind, B, T, L):
    x = synth.make_aa_batch(B, T, L, seed=99, device="cuda")
    if kind == "c64":
        return x
    if kind == "c128":
        return x.to(torch.complex128)
    s = 2046.0 / float(x.abs().amax())
    re = torch.clamp(torch.round(x.real * s), -2048, 2047).to(torch.int16)
    im = torch.clamp(torch.round(x.imag * s), -2048, 2047).to(torch.int16)
    return torch.stack([re, im], dim=-1).contiguous()


@pytest.mark.parametrize("kind,T,L,plan_lo,plan_hi", [("c64", 1024, 512, 1000, 2000), ("ci16", 1024, 128, 2000, 3000),
                                                       ("c128", 1024, 512, 3000, 4000),
                                                       ("c128", 3000, 256, 3000, 4000), ("c128", 9000, 512, 3000, 4000),
                                                       ("c64", 4096, 512, 1100, 1200), ("c64", 5315, 256, 1100, 1200),
                                                       ("c64", 9000, 100, 2, 2)])
def test_detect_only_events_equal_full(kind, T, L, plan_lo, plan_hi, monkeypatch):
    B = 512
    x = _batch(kind, B, T, L)
    b = _lib.as_batch(x, batched=True)
    plan = _lib.lib().ofs_aa_plan(b.fmt, _lib.resolve_precision(b, None), 1, T, L)
    assert plan_lo <= plan <= plan_hi
    reg = 1000 <= plan < 1100                      # register-staged fp32 kernel: DO arithmetic
    for scan in ("32", "64") if reg else ("",):
        if reg:
            monkeypatch.setenv("OFS_FAST_E", "4")
            monkeypatch.setenv("OFS_FAST_SCAN", scan)
            monkeypatch.setenv("OFS_FAST_SCAN_DO", scan)
        full = sync_aa.aa_detect_streaming_batched(x, L)
        monkeypatch.delenv("OFS_FAST_E", raising=False)
        monkeypatch.delenv("OFS_FAST_SCAN", raising=False)
        det = sync_aa.aa_detect_streaming_batched(x, L, outputs=())
        monkeypatch.delenv("OFS_FAST_SCAN_DO", raising=False)
        assert det.P is None and det.M is None and det.R is None
        assert torch.equal(full.n_events, det.n_events)
        assert int(full.n_events.sum()) > B // 4
        E = min(full.ev_int.shape[1], det.ev_int.shape[1])
        mask = (torch.arange(E, device="cuda")[None, :] < torch.clamp(full.n_events, max=E)[:, None])
        assert torch.equal(full.ev_int[:, :E][mask], det.ev_int[:, :E][mask])
        assert torch.equal(full.ev_real[:, :E][mask], det.ev_real[:, :E][mask])
