"""Diagnostic: time of the fp64 zc_freq sliding DFT (zc_slide.hip) against the stream count, to
separate per-workgroup throughput from dispatch quantisation (one 14-16-wave workgroup per CU).
    python tools/zs_sweep.py [--T 16384] [--B 64,128,...] [--nb 1] [--fmt c128]
Prints one JSON line per B: ms per call (HIP events over --steps calls), us per stream."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "ofdm-sync-math_amd"))
from ofdm_sync_amd import _lib, zc_freq  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--T", type=int, default=16384)
    ap.add_argument("--N", type=int, default=2048)
    ap.add_argument("--cp", type=int, default=512)
    ap.add_argument("--nb", type=int, default=1)
    ap.add_argument("--fmt", default="c128", choices=("c128", "c64"))
    ap.add_argument("--B", default="32,64,128,192,224,240,248,256,264,288,320,384,448,512,768,1024")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--ab", default="", help="K=V[,K2=V2][;K=V...]: interleaved in-process A/B of knob sets the "
                                             "library reads per launch as debug variants (e.g. 'ZS_PAIR=0;ZS_PAIR=1'); "
                                             "medians of --reps")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--prec", default="fp64", choices=("fp64", "fp32"), help="metric precision (fp32: float out)")
    a = ap.parse_args()
    dt = torch.complex128 if a.fmt == "c128" else torch.complex64
    idx, tb, e = zc_freq.make_pss_frequency_template()
    for B in [int(v) for v in a.B.split(",")]:
        g = torch.Generator(device="cuda").manual_seed(B)
        x = torch.randn((B, a.nb, a.T), dtype=dt, device="cuda", generator=g)
        for _ in range(3):
            zc_freq.compute_frequency_metric_batched(x, idx, tb, e, N=a.N, cp=a.cp, precision=a.prec)
        torch.cuda.synchronize()

        def run():
            t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            t0.record()
            for _ in range(a.steps):
                zc_freq.compute_frequency_metric_batched(x, idx, tb, e, N=a.N, cp=a.cp, precision=a.prec)
            t1.record()
            torch.cuda.synchronize()
            return t0.elapsed_time(t1) / a.steps

        rec = {"B": B, "T": a.T, "nb": a.nb, "fmt": a.fmt}
        if a.ab:
            sets = [dict(kv.split("=") for kv in cfg.split(",")) for cfg in a.ab.split(";")]
            keys = sorted({k for st in sets for k in st})
            ts = {i: [] for i in range(len(sets))}
            for _ in range(a.reps):
                for i, st in enumerate(sets):
                    for k in keys:
                        _lib.set_variant(k.removeprefix("OFS_"), None)
                    for k, v in st.items():
                        _lib.set_variant(k.removeprefix("OFS_"), int(v))
                    run()
                    ts[i].append(run())
            _lib.reset_variants()
            for i, st in enumerate(sets):
                rec[",".join(f"{k}={v}" for k, v in st.items())] = round(sorted(ts[i])[len(ts[i]) // 2], 4)
        else:
            ms = run()
            rec.update(ms=round(ms, 4), us_per_stream=round(1000 * ms / B, 3), defer=_lib.get_variant("ZS_DEFER"))
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
