"""Diagnostic: the fused zc_v2 CFAR + gate (zc_v2._detect_run) from several library builds on the
same |corr| rows (4096 x 16384 f64 with bursts, near-threshold samples and gaps around the
hysteresis), every output compared bit for bit with the first build's - for layout / role variants
that must not change a bit.  Each build runs in its own process (one tuning library per process).

    python tools/zc_check.py build/libofdmsync_a.so build/libofdmsync_b.so ...
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def one(lib, out):
    sys.path.insert(0, os.path.join(ROOT, "ofdm-sync-math_amd"))
    import torch
    from ofdm_sync_amd import _lib, zc_v2
    _lib.use_tuning_library(lib)
    dev = torch.device("cuda", 0)
    B, n = 4096, 16384
    g = torch.Generator(device=dev).manual_seed(7)
    mag = torch.rand((B, n), dtype=torch.float64, device=dev, generator=g) * 0.5
    mag[:, 5000:5100] += 2.0
    for k in range(0, B, 7):                          # gate gaps around the hysteresis, late bursts
        s = 9000 + (k % 300)
        mag[k, s:s + 20] += 3.0
        mag[k, s + zc_v2.HYSTERESIS + (k % 3) - 1 + 20:s + zc_v2.HYSTERESIS + (k % 3) + 40] += 3.0
    res = {}
    for want_state in (False, True):
        st, gate, n_ev, ev_i, ev_v = zc_v2._detect_run(mag, zc_v2.CORR_WINDOW_SIZE, zc_v2.THRESH_VALUE,
                                                       zc_v2.THRESH_FRAC_BITS, zc_v2.MIN_CORR_MAG, 2048,
                                                       zc_v2.HYSTERESIS, 4, want_state=want_state)
        torch.cuda.synchronize()
        tag = "s" if want_state else "e"
        res[tag + "gate"] = gate.cpu().numpy()
        res[tag + "nev"] = n_ev.cpu().numpy()
        ne = n_ev.cpu().numpy()
        evi = ev_i.cpu().numpy()
        evv = ev_v.cpu().numpy()
        m = np.arange(evi.shape[1])[None, :] < ne[:, None]      # live event slots only
        res[tag + "evi"] = np.where(m[:, :, None], evi, 0)
        res[tag + "evv"] = np.where(m, evv, 0).view(np.int64)
        if want_state:
            for k, v in st.items():
                if v is not None:
                    a = v.cpu().numpy()
                    res["st_" + k] = a.view(np.int64) if a.dtype == np.float64 else a
    np.savez(out, **res)


def main():
    if sys.argv[1] == "--one":
        return one(sys.argv[2], sys.argv[3])
    libs = sys.argv[1:]
    outs = []
    with tempfile.TemporaryDirectory() as td:
        for i, lib in enumerate(libs):
            out = os.path.join(td, f"{i}.npz")
            subprocess.run([sys.executable, __file__, "--one", os.path.abspath(lib), out], check=True, timeout=300)
            outs.append(dict(np.load(out)))
    base = outs[0]
    for lib, o in zip(libs[1:], outs[1:]):
        diff = [k for k in base if not np.array_equal(base[k], o[k])]
        print(json.dumps({"lib": os.path.basename(lib), "vs": os.path.basename(libs[0]), "bit_identical": not diff,
                          "differs": diff, "events": int(base["enev"].sum())}), flush=True)


if __name__ == "__main__":
    main()
