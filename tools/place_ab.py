"""Paired A/B of the sync_aa buffer placement (sync_aa.allocate: "plain" caching-allocator arena vs
"contiguous" per-buffer physically contiguous blocks) on the fp32 shapes, through the product's
AABatchDetector: per round and shape a FRESH detector of each placement (order rotated per round),
the same input copied in, 20 timed launches (HIP events on the launch stream).  Prints one JSON line
per shape with the per-round times and medians.  Diagnostic tooling (not the product).

    python tools/place_ab.py [--rounds 5] [--shapes cfg3,cfg3_2ant,cfg3_T4096,aa_refshape_c64]
"""
import argparse
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ofdm-sync-math_amd"))
from ofdm_sync_amd import synth, sync_aa  # noqa: E402

SHAPES = {                       # name: (B, n_ant, T, L, cir branches)
    "cfg3": (65536, 1, 1024, 512, (1,)),
    "cfg3_2ant": (65536, 2, 1024, 512, (0, 1)),
    "cfg3_T4096": (65536, 1, 4096, 512, (1,)),
    "aa_refshape_c64": (16384, 2, 5315, 512, (0, 1)),
    "aa_1ant_T5315": (16384, 1, 5315, 512, (1,)),
    "aa_2ant_T4096": (16384, 2, 4096, 512, (0, 1)),
    "aa_2ant_T5316": (16384, 2, 5316, 512, (0, 1)),
    "aa_1ant_T4095": (65536, 1, 4095, 512, (1,)),
}


def time_one(det, steps, warmup):
    st = torch.cuda.current_stream()
    for _ in range(warmup):
        det.run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(steps):
        det.run()
    e1.record(st)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--shapes", default=",".join(SHAPES))
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    for name in a.shapes.split(","):
        B, na, T, L, br = SHAPES[name]
        x = synth.synth_batch(synth.faded_base(L, "cir1", br), B, T, seed=11, device=dev, dtype=torch.complex64)
        times = {"plain": [], "contiguous": []}
        for r in range(a.rounds):
            order = ("plain", "contiguous") if r % 2 == 0 else ("contiguous", "plain")
            for p in order:
                det = sync_aa.AABatchDetector(B, T, na, L, outputs=("P", "R", "M"), max_events=4, placement=p,
                                              device=dev)
                det.x.copy_(x.reshape(det.x.shape))
                times[p].append(round(time_one(det, a.steps, 3), 4))
                del det
                torch.cuda.empty_cache()
        med = {p: sorted(v)[len(v) // 2] for p, v in times.items()}
        print(json.dumps({"shape": name, "B": B, "n_ant": na, "T": T, "L": L, "times_ms": times,
                          "median_ms": med, "contiguous_over_plain": round(med["contiguous"] / med["plain"], 4)}),
              flush=True)


if __name__ == "__main__":
    main()
