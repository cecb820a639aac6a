"""Receiver back-end (sc.py:274-311 over core.py:123-138, 171-176, 339-370, 443-469) at full
occupancy against the oracle, every frame.

The fast kernel (csrc/backend.hip rx_backend_fast_kernel) overlays the unwrap phases and the
block-sum reduction slots on its sample buffer (OFS_BE_LDS40) and alternates two slot sets with
one barrier per reduction (OFS_BE_RED2).  A cross-wave ordering slip in that overlay only shows
when waves of different workgroups drift, i.e. with many more frames than resident workgroups,
each workgroup looping over several frames.  So: 4096 frames x 2 branches (4-5 workgroups per
CU x 256 CUs = 1024-1280 resident, 3-4 frames per workgroup), the largest used-bin count the
fast path takes (n_used = 3/5/10 x 256 at N = 1024/2048/4096: the phase array reaches as far
into the buffer as it can), and every frame checked against ofdm_oracle.rx_backend at the
tolerances of test_gpu_parity.py's per-frame test.
"""
import numpy as np
import pytest

import ofdm_oracle as O

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("needs a GPU", allow_module_level=True)

from ofdm_sync_amd import core  # noqa: E402

BW = 256                       # the back-end's workgroup width (csrc/backend.hip)
FAST_MAX_USED = {1024: 3 * BW, 2048: 5 * BW, 4096: 10 * BW}


def relerr(a, b):
    """as test_gpu_parity.relerr: max |a - b| over max(1, max |b|)"""
    a, b = np.asarray(a), np.asarray(b)
    return float(np.max(np.abs(a - b)) / max(1.0, float(np.max(np.abs(b)))))


@pytest.mark.parametrize("fmt,N", [("c64", 1024), ("c64", 2048), ("c64", 4096), ("c128", 2048), ("int16", 1024)])
def test_fast_backend_every_frame_vs_oracle_at_full_occupancy(fmt, N):
    rng = np.random.default_rng(7 * N + len(fmt))
    B, nb, cp = 4096, 2, min(N // 4, 512)
    U = FAST_MAX_USED[N]
    assert cp <= 2 * BW and U <= FAST_MAX_USED[N]          # the fast kernel's dispatch conditions
    k = core.centered_subcarrier_indices(U)
    assert k.size == U
    T = 2 * (N + cp) + 300
    x = np.round((rng.standard_normal((B, nb, T)) + 1j * rng.standard_normal((B, nb, T))) * 300)
    ps = rng.integers(0, 300, B)
    ds = ps + N + cp
    pil = np.exp(2j * np.pi * rng.random((B, U)))           # per-frame pilots
    dat = np.exp(2j * np.pi * rng.random(U))
    if fmt == "int16":
        xd = torch.from_numpy(np.stack([x.real, x.imag], -1).astype(np.int16)).cuda()
    else:
        xd = torch.from_numpy(x.astype(np.complex64 if fmt == "c64" else np.complex128)).cuda()
    out = core.receiver_backend_batched(xd, ps, ds, pil, dat, n_fft=N, cp_len=cp, fs_hz=1e6, bins=k)
    o = {key: v.cpu().numpy() for key, v in out.items()}
    del out, xd
    bad = []
    for b in range(B):
        r = O.rx_backend(x[b], int(ps[b]), int(ds[b]), N, cp, 1e6, k, pil[b], dat)
        ok = (abs(o["cfo"][b] - r["cfo"]) < 1e-6 and relerr(o["h"][b], r["h"]) < 1e-9
              and relerr(o["xa"][b], r["xa"]) < 1e-8 and abs(o["evm"][b] - r["evm"]) < 1e-8 * max(1.0, r["evm"])
              and abs(o["slope"][b] - r["slope"]) < 1e-9 * max(1.0, abs(r["slope"])))
        if not ok:
            bad.append(b)
    assert not bad, f"{len(bad)} of {B} frames differ from the oracle, first {bad[:8]}"


def test_fast_backend_given_cfo_every_frame_vs_oracle_at_full_occupancy():
    """The cfo_in branch (no CP reduction: one block sum fewer per frame shifts the alternating
    slot sets) at N = 2048, c64, every frame."""
    N, U = 2048, FAST_MAX_USED[2048]
    rng = np.random.default_rng(99)
    B, nb, cp = 4096, 2, 512
    k = core.centered_subcarrier_indices(U)
    T = 2 * (N + cp) + 128
    x = np.round((rng.standard_normal((B, nb, T)) + 1j * rng.standard_normal((B, nb, T))) * 300)
    ps = rng.integers(0, 128, B)
    ds = ps + N + cp
    cfo = rng.uniform(-200.0, 200.0, B)
    pil = np.exp(2j * np.pi * rng.random(U))
    dat = np.exp(2j * np.pi * rng.random((B, U)))           # per-frame data symbols
    xd = torch.from_numpy(x.astype(np.complex64)).cuda()
    out = core.receiver_backend_batched(xd, ps, ds, pil, dat, n_fft=N, cp_len=cp, fs_hz=1e6, bins=k, cfo_hz=cfo)
    o = {key: v.cpu().numpy() for key, v in out.items()}
    bad = []
    for b in range(B):
        r = O.rx_backend(x[b], int(ps[b]), int(ds[b]), N, cp, 1e6, k, pil, dat[b], cfo=float(cfo[b]))
        ok = (o["cfo"][b] == cfo[b] and relerr(o["h"][b], r["h"]) < 1e-9 and relerr(o["xa"][b], r["xa"]) < 1e-8
              and abs(o["evm"][b] - r["evm"]) < 1e-8 * max(1.0, r["evm"])
              and abs(o["slope"][b] - r["slope"]) < 1e-9 * max(1.0, abs(r["slope"])))
        if not ok:
            bad.append(b)
    assert not bad, f"{len(bad)} of {B} frames differ from the oracle, first {bad[:8]}"
