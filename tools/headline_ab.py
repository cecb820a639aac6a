"""Interleaved in-process A/B of debug variants on the headline detector (cfg3: 65536 x 1024 c64,
L = 512, P/R/M + events) through the product's AABatchDetector, same buffers for every arm.
Diagnostic tooling (not the product).

    python tools/headline_ab.py --ab "FAST_SCAN=64;FAST_SCAN=32" [--reps 7] [--steps 20]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ofdm-sync-math_amd"))
from ofdm_sync_amd import _lib, synth, sync_aa  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ab", required=True, help="K=V[,K2=V2][;K=V...] variant sets (ofs_debug_set_variant names)")
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--B", type=int, default=65536)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    det = sync_aa.AABatchDetector(a.B, 1024, 1, 512, outputs=("P", "R", "M"), max_events=4, device=dev)
    det.x.copy_(synth.headline_batch(a.B, 1024, 512, seed=2026, device=dev))
    sets = [dict(kv.split("=") for kv in cfg.split(",")) for cfg in a.ab.split(";")]
    keys = sorted({k for st in sets for k in st})
    st = torch.cuda.current_stream()
    times = {i: [] for i in range(len(sets))}
    for _ in range(a.reps):
        for i, vs in enumerate(sets):
            for k in keys:
                _lib.set_variant(k, None)
            for k, v in vs.items():
                _lib.set_variant(k, int(v))
            for _ in range(3):
                det.run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(a.steps):
                det.run()
            e1.record(st)
            torch.cuda.synchronize()
            times[i].append(round(e0.elapsed_time(e1) / a.steps, 5))
    _lib.reset_variants()
    out = {"placement": det.placement, "plan": det.plan()}
    for i, vs in enumerate(sets):
        name = ",".join(f"{k}={v}" for k, v in vs.items())
        out[name] = {"median_ms": sorted(times[i])[len(times[i]) // 2], "ms": times[i]}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
