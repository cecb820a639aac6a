"""Diagnostic: per-phase cycles of the fast receiver back-end kernel (OFS_BE_TIMING build).
    python tools/variants.py backend.hip "betime=-DOFS_BE_TIMING=1"
    OFS_LIB=build/libofdmsync_betime.so python tools/be_phase.py"""
import ctypes
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, os.path.join(ROOT, "ofdm-sync-math_amd"))
import bench_configs as BC  # noqa: E402
from ofdm_sync_amd import _lib  # noqa: E402
if os.environ.get("OFS_LIB"):   # a tools/variants.py tuning build, named explicitly (not a product switch)
    _lib.use_tuning_library(os.environ["OFS_LIB"])

PHASES = ["cfo (CP loads + 2 block sums)", "pilot window -> LDS", "pilot FFT", "LS + atan2 (1200 bins)",
          "unwrap + slope", "data window -> LDS", "data FFT", "EQ + gain sums", "gain, EVM, outputs"]


def main():
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        BC.backend("cuda", st, 2, 1)
        torch.cuda.synchronize()
        L = _lib.lib()
        f = L.ofs_be_prof
        f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
        buf = (ctypes.c_ulonglong * 9)()
        f(buf)
        r = BC.backend("cuda", st, 5, 0)
        torch.cuda.synchronize()
        f(buf)
    tot = sum(buf)
    print(json.dumps({"ms": r["ms"], "phases": {p: round(buf[i] / tot, 4) for i, p in enumerate(PHASES)}}))


if __name__ == "__main__":
    main()
