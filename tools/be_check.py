"""Diagnostic: the receiver back-end's outputs from several library builds on the same inputs
(the backend config's shape: 16384 frames x 2 branches, N 2048, CP 512, c64), compared bit for bit
with the first library's - for layout / scheduling variants that must not change a single bit.

    python tools/be_check.py build/libofdmsync_a.so build/libofdmsync_b.so ...
"""
from __future__ import annotations

import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ofdm-sync-math_amd"))
from ofdm_sync_amd import _lib, core  # noqa: E402


def run(lib, dev, st, B=16384, nb=2, N=2048, cp=512, seed=11, n_used=1200):
    T = 2 * (N + cp) + 64
    g = torch.Generator(device=dev).manual_seed(seed)
    x = torch.randn((B, nb, T), dtype=torch.complex64, device=dev, generator=g)
    k = core.centered_subcarrier_indices(n_used)
    U = k.size
    ps = torch.randint(0, 60, (B,), dtype=torch.int64, device=dev, generator=g)
    ds = ps + N + cp
    pil = torch.exp(2j * np.pi * torch.rand((B, U), dtype=torch.float64, device=dev, generator=g))
    dat = torch.exp(2j * np.pi * torch.rand((U,), dtype=torch.float64, device=dev, generator=g))
    kb = torch.as_tensor(k.astype(np.int32)).to(dev)
    outs = [torch.full((B,), -7.0, dtype=torch.float64, device=dev) for _ in range(5)]
    h = torch.full((B, U), -7.0, dtype=torch.complex128, device=dev)
    xa = torch.full_like(h, -7.0)
    gain = torch.full((B,), -7.0, dtype=torch.complex128, device=dev)
    rc = lib.ofs_rx_backend(_lib.C64, x.data_ptr(), B, nb, T, N, cp, 30.72e6, ps.data_ptr(), ds.data_ptr(), None, U,
                            kb.data_ptr(), pil.data_ptr(), U, dat.data_ptr(), 0, outs[0].data_ptr(), h.data_ptr(),
                            xa.data_ptr(), gain.data_ptr(), outs[1].data_ptr(), outs[2].data_ptr(),
                            outs[3].data_ptr(), outs[4].data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    assert rc == 0, rc
    return [o.cpu() for o in outs] + [h.cpu(), xa.cpu(), gain.cpu()]


def main():
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    res = []
    N = int(os.environ.get("BE_N", "2048"))                 # BE_N=1024 / 4096: the other fast shapes
    shape = dict(N=N, cp=min(N // 4, 512), n_used=int(N * 1200 / 2048), B=16384 * 2048 // N)
    for path in sys.argv[1:]:
        lib = ctypes.CDLL(os.path.abspath(path))
        _lib._declare(lib)
        res.append((os.path.basename(path), run(lib, dev, st, **shape)))
    base = res[0][1]
    for name, r in res[1:]:
        same = [torch.equal(a.view(torch.int64) if a.dtype == torch.float64 else torch.view_as_real(a).view(torch.int64),
                            b.view(torch.int64) if b.dtype == torch.float64 else torch.view_as_real(b).view(torch.int64))
                for a, b in zip(base, r)]
        print(json.dumps({"lib": name, "vs": res[0][0], "bit_identical": all(same), "per_output": same}), flush=True)


if __name__ == "__main__":
    main()
