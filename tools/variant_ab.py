"""Interleaved A/B of the library's runtime debug variants (ofs_debug_set_variant) over
tools/bench_configs.py configs, one process, same buffers per config call.  Diagnostic only.

    python tools/variant_ab.py --configs zc_freq_refshape --rounds 3 --variants "base" "ZS_DEFER=1" "ZS_C=256"
A variant spec is "base" (nothing forced) or comma-separated NAME=VALUE pairs.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "ofdm-sync-math_amd"))
import torch  # noqa: E402

import bench_configs as BC  # noqa: E402
from ofdm_sync_amd import _lib  # noqa: E402


def parse(spec):
    if spec == "base":
        return {}
    return {k: int(v) for k, v in (p.split("=") for p in spec.split(","))}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", required=True)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--variants", nargs="+", required=True)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev)
    for cfg in a.configs.split(","):
        fn = BC.CONFIGS[cfg]
        for r in range(a.rounds):
            order = a.variants[r % len(a.variants):] + a.variants[:r % len(a.variants)]
            for spec in order:
                with _lib.variants(**parse(spec)):
                    res = fn(dev, st, a.steps, 3)
                print(json.dumps({"config": cfg, "round": r, "variant": spec, "ms": res["ms"]}), flush=True)


if __name__ == "__main__":
    main()
