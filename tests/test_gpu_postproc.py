"""Detection post-processing on the GPU (csrc/postproc.hip) against the reference's own decisions.

Goldens (tests/golden/post_*.npz, made by tests/golden/make_golden.py from the reference):
sc.find_plateau_end_from_metric (sc.py:81-146), minn.find_minn_peak (minn.py:131-205),
minn._trailing_average (minn.py:115-128), combined_sc_min.find_minn_peak +
_streaming_peak_detector (combined_sc_min.py:183-259) and the S&C gate of run_simulation
(combined_sc_min.py:337-358).  Tolerances: indices, gates and error behaviour exact; the trailing
average is the reference's float64 recursion (bit-identical); the plateau's smoothed metric is a
window sum whose order differs from numpy's (BLAS) dot: 1e-15 relative.
"""
from __future__ import annotations

import glob
import os

import numpy as np
import pytest

import ofdm_oracle as O
from conftest import GOLDEN

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

from ofdm_sync_amd import _postproc, combined_sc_min, minn, sc  # noqa: E402


def cases(prefix):
    return sorted(os.path.basename(p)[:-4] for p in glob.glob(os.path.join(GOLDEN, prefix + "*.npz")))


def G(name):
    return np.load(os.path.join(GOLDEN, name + ".npz"))


@pytest.mark.parametrize("name", cases("post_plateau_"))
def test_plateau_end_vs_reference_golden(name):
    d = G(name)
    la = None if int(d["lookahead"]) < 0 else int(d["lookahead"])
    if int(d["error"]):
        with pytest.raises(ValueError):
            sc.find_plateau_end_from_metric(d["M"], int(d["cp"]), lookahead=la, smooth_win=int(d["smooth_win"]))
        return
    got = sc.find_plateau_end_from_metric(d["M"], int(d["cp"]), lookahead=la, smooth_win=int(d["smooth_win"]))
    assert got == int(d["index"])


def test_plateau_end_batched_vs_oracle():
    """Batch of metric streams (S&C-shaped plateaus, noise, ramps) through one launch; index and
    branch per stream equal the oracle's, the smoothed metric within 1e-15 relative."""
    rng = np.random.default_rng(5)
    B, n, cp, w = 96, 1500, 64, 16
    M = np.abs(rng.normal(0, 0.05, (B, n)))
    for b in range(B):
        s = int(rng.integers(0, n - 300))
        ln = int(rng.integers(5, 250))
        M[b, s:s + ln] += rng.uniform(0.3, 1.0) * np.hanning(ln) ** (0.1 + (b % 4))
    M[7] = np.linspace(0, 1, n)
    M[8] = 0.0
    M[9, 200:900] = 0.9                                  # plateau longer than cp: no 95 % drop
    M[10, 100:160] = 0.8                                 # in reach -> the earliest long run
    for dt in (torch.float64, torch.float32):
        Mt = torch.from_numpy(M).to("cuda", dt)
        idx, Ms, st = sc.find_plateau_end_batched(Mt, cp, lookahead=None, smooth_win=w)
        Mh = Mt.double().cpu().numpy()
        branches = set()
        for b in range(B):
            oi, ob, oMs = O.plateau_end(Mh[b], cp, None, w)
            assert int(idx[b]) == oi and int(st[b]) == ob, b
            assert np.allclose(Ms[b].cpu().numpy(), oMs, rtol=1e-15, atol=1e-17)
            branches.add(ob)
        assert {1, 2} <= branches


@pytest.mark.parametrize("name", cases("post_minnpeak_"))
def test_minn_peak_vs_reference_golden(name):
    d = G(name)
    b = None if int(d["bounds"][0]) < 0 else (int(d["bounds"][0]), int(d["bounds"][1]))
    if int(d["error"]):
        with pytest.raises(ValueError):
            minn.find_minn_peak(d["M"], smooth_win=int(d["smooth_win"]), gate_threshold=float(d["thr"]),
                                search_bounds=b)
        return
    pk, gate, Ms = minn.find_minn_peak(d["M"], smooth_win=int(d["smooth_win"]), gate_threshold=float(d["thr"]),
                                       search_bounds=b)
    assert pk == int(d["peak"])
    assert np.array_equal(gate, d["gate"])
    assert np.array_equal(Ms, d["Ms"])                   # the reference's recursion, bit for bit


def test_minn_peak_batched_vs_oracle():
    rng = np.random.default_rng(9)
    B, n = 64, 2049
    M = rng.normal(0, 0.02, (B, n))
    for b in range(B):
        for _ in range(int(rng.integers(1, 4))):
            s = int(rng.integers(0, n - 200))
            M[b, s:s + int(rng.integers(3, 200))] += rng.uniform(0.1, 1.0)
    M[3] = -np.abs(M[3])                                 # no positive peak -> status -2
    peak, glo, ghi, Ms, st = minn.find_minn_peak_batched(torch.from_numpy(M).cuda(), smooth_win=16,
                                                         gate_threshold=0.5, search_bounds=(100, 1900))
    for b in range(B):
        if b == 3:
            assert int(st[b]) == -2
            continue
        pk, gate, oMs = O.minn_peak(M[b], 16, 0.5, (100, 1900))
        assert int(st[b]) == 0 and int(peak[b]) == pk
        g = np.zeros(n, bool)
        g[int(glo[b]):int(ghi[b])] = True
        assert np.array_equal(g, gate)
        assert np.array_equal(Ms[b].cpu().numpy(), oMs)


def test_trailing_average_vs_reference_golden():
    d = G("post_trailing_avg")
    assert np.array_equal(minn._trailing_average(d["x"], 16), d["y16"])
    assert np.array_equal(combined_sc_min._trailing_average(d["x"], 16), d["y16"])
    assert np.array_equal(minn._trailing_average(d["x"], 1), d["y1"])
    assert np.array_equal(minn._trailing_average(d["x3"], 3), d["y3"])
    x32 = torch.from_numpy(d["x"]).float().cuda()         # f32 metric: recursion on its f64 values
    y = _postproc.trailing_average(torch.stack([x32, x32.flip(0)]), 16)
    assert np.array_equal(y[0].cpu().numpy(), O.trailing_average(x32.double().cpu().numpy(), 16))
    assert np.array_equal(y[1].cpu().numpy(), O.trailing_average(x32.flip(0).double().cpu().numpy(), 16))


def test_combined_detector_back_end_vs_reference_golden():
    d = G("post_comb_detect")
    mask, span = combined_sc_min.sc_gate_mask(d["M_sc"])
    assert np.array_equal(mask, d["gate"]) and span == tuple(int(v) for v in d["span"])
    pk = combined_sc_min.find_minn_peak(d["M_minn"], smooth_win=int(d["smooth_win"]), gate_mask=mask)
    assert pk == int(d["peak"])
    # batched: the same decision for a batch of (M_minn, M_sc) pairs (shifted copies)
    Mm = np.stack([np.roll(d["M_minn"], s) for s in (0, 37, -120)])
    Msc = np.stack([np.roll(d["M_sc"], s) for s in (0, 37, -120)])
    peak, st, spans = combined_sc_min.detect_batched(torch.from_numpy(Mm).cuda(), torch.from_numpy(Msc).cuda())
    for b in range(3):
        m, sp = O.sc_gate(Msc[b])
        assert int(st[b]) == 0 and int(peak[b]) == O.comb_minn_peak(Mm[b], 16, m)
        assert tuple(int(v) for v in spans[b]) == sp


def test_streaming_peak_vs_reference_golden():
    d = G("post_streaming_peak")
    for j in range(4):
        r = combined_sc_min._streaming_peak_detector(d["metric"], d[f"mask{j}"])
        assert (-1 if r is None else r) == int(d[f"peak{j}"])
    g = G("post_comb_detect")
    mask = g["gate"]
    first, last = int(np.argmax(mask)), int(mask.size - np.argmax(mask[::-1]) - 1)
    pk = combined_sc_min.find_minn_peak(g["M_minn"], smooth_win=4, gate_mask=mask,
                                        search_bounds=(first + 5, last - 5))
    assert pk == int(d["peak_bounded"])


def test_post_processing_errors_like_reference():
    with pytest.raises(ValueError):
        minn.find_minn_peak(np.zeros(0))
    with pytest.raises(ValueError):
        combined_sc_min.find_minn_peak(np.ones(10), gate_mask=None)
    with pytest.raises(ValueError):
        combined_sc_min.find_minn_peak(np.ones(10), gate_mask=np.zeros(9, bool))
    with pytest.raises(ValueError):
        combined_sc_min.find_minn_peak(np.ones(10), gate_mask=np.zeros(10, bool))
    assert combined_sc_min.find_minn_peak(np.zeros(0), gate_mask=np.zeros(0, bool)) == 0
    assert sc.find_plateau_end_from_metric(np.zeros(0), 16) == 0
