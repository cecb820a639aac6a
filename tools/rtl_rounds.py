"""Diagnostic: speculation rounds of rtl_exact_kernel's exact float IIR (aa_exact.hip phase B) on
the cfg2b batch.  Needs a library built with -DOFS_RTL_ROUNDS_DEBUG=1
(``python tools/variants.py aa_exact.hip "rr=-DOFS_RTL_ROUNDS_DEBUG=1"``), which writes each stream's total
rounds over its segments into open_gate_start instead of the gate state.  Not the product.

    OFS_LIB=build/libofdmsync_rr.so python tools/rtl_rounds.py [--B 4096]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "ofdm-sync-math_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import bench_configs as BC  # noqa: E402
from ofdm_sync_amd import _lib, synth  # noqa: E402
if os.environ.get("OFS_LIB"):   # a tools/variants.py tuning build, named explicitly (not a product switch)
    _lib.use_tuning_library(os.environ["OFS_LIB"])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--shift", type=int, default=3)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, T, Q = a.B, 1024, 64
    x = BC.int12(synth.make_aa_batch(B, T, 128, seed=9, device=dev))
    o = [torch.empty((B, T), dtype=torch.float64, device=dev) for _ in range(6)]
    o += [torch.empty((B, T), dtype=torch.bool, device=dev) for _ in range(2)]
    E = 16
    n_ev = torch.zeros(B, dtype=torch.int32, device=dev)
    ev = torch.empty((B, E, 4), dtype=torch.int64, device=dev)
    og = torch.full((B,), -7, dtype=torch.int64, device=dev)
    L_ = _lib.lib()
    st = torch.cuda.current_stream()
    rc = L_.ofs_minn_rtl(_lib.CI16, x.data_ptr(), B, 1, T, Q, a.shift, 0, 3276, 15,
                         *[t.data_ptr() for t in o], 1, 2, 0, E, n_ev.data_ptr(), ev.data_ptr(),
                         og.data_ptr(), st.cuda_stream)
    torch.cuda.synchronize()
    if rc:
        raise RuntimeError(f"ofs_minn_rtl status {rc}")
    r = og.double()
    nseg = (T + 255) // 256
    h = torch.bincount(og.clamp(0, 64 * nseg)).tolist()
    print(json.dumps({"B": B, "T": T, "Q": Q, "shift": a.shift, "plan": L_.ofs_rtl_plan(_lib.CI16, 1, T, Q),
                      "segments_per_stream": nseg,
                      "rounds_per_segment_mean": round(float(r.mean()) / nseg, 3),
                      "rounds_per_segment_max_stream": round(float(r.max()) / nseg, 3),
                      "rounds_per_segment_min_stream": round(float(r.min()) / nseg, 3),
                      "hist_total_rounds": {i: c for i, c in enumerate(h) if c}}))


if __name__ == "__main__":
    main()
