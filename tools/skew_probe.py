"""cfg4 (fused S&C + Minn, 32768 x 4096 c64) on ONE physically contiguous allocation with the
seven streams (x, Ms, Ps, Rs, Mm, Pm, Rm) carved at 2 MiB-aligned offsets plus a per-stream skew
i*S: does a sub-2 MiB skew between the concurrently written streams change the time?  Separate
plain allocations are timed alongside.  Diagnostic only.

    python tools/skew_probe.py [--skews 0,4096,...] [--steps K]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ofdm-sync-math_amd"))

import torch  # noqa: E402

from ofdm_sync_amd import _lib, synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--skews", default="0,4096,8448,69632,528384,1060864")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    B, T, N = 32768, 4096, 2048
    n_out = T - N + 1
    x0 = synth.make_aa_batch(B, T, N // 2, seed=4, device=dev)
    sizes = [B * T * 8] + [B * n_out * s for s in (4, 8, 4) * 2]
    dts = [torch.complex64] + [torch.float32, torch.complex64, torch.float32] * 2
    shapes = [(B, 1, T)] + [(B, n_out)] * 6
    big = 2 << 20
    L_ = _lib.lib()

    def run(bufs):
        x = bufs[0]
        x.copy_(x0)
        args = (_lib.C64, x.data_ptr(), B, 1, T, N, _lib.FP32, *[t.data_ptr() for t in bufs[1:]], st.cuda_stream)
        for _ in range(a.warmup):
            L_.ofs_sc_minn_metric(*args)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(a.steps):
            rc = L_.ofs_sc_minn_metric(*args)
        e1.record(st)
        torch.cuda.synchronize()
        assert rc == 0
        return e0.elapsed_time(e1) / a.steps

    for rep in range(2):
        bufs = [torch.empty(sh, dtype=dt, device=dev) for sh, dt in zip(shapes, dts)]
        print(json.dumps({"rep": rep, "layout": "separate", "ms": round(run(bufs), 4)}), flush=True)
        del bufs
        torch.cuda.empty_cache()
        for S in [int(v) for v in a.skews.split(",")]:
            offs, tot = [], 0
            for i, n in enumerate(sizes):
                tot = (tot + big - 1) // big * big + i * S
                offs.append(tot)
                tot += n
            blk = _lib._DeviceBlock(tot + big, _lib.HIP_MALLOC_CONTIGUOUS)
            with torch.cuda.device(dev):
                raw = torch.as_tensor(blk, device=dev)
            shift = (-raw.data_ptr()) % big
            bufs = [raw[shift + o:shift + o + n].view(dt).view(sh) for o, n, dt, sh in zip(offs, sizes, dts, shapes)]
            print(json.dumps({"rep": rep, "layout": "contiguous", "skew": S, "ms": round(run(bufs), 4)}), flush=True)
            del bufs, raw, blk
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
