"""Diagnostic: per-phase cycles of the persistent matched-filter kernel (OFS_MP_TIMING build).
    python tools/variants.py zc_fftcorr.hip "mptime=-DOFS_MP_TIMING=1"
    OFS_LIB=build/libofdmsync_mptime.so python tools/mp_phase.py
Cycles (s_memtime) summed over every wave of the launch, per phase of a block."""
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

PHASES = ["A: regs DIF (spans 4096..512)", "A: LDS write + barrier", "B: spans 256..32 (wave-local)",
          "mid: H wait, spans 16..1, xH, 1..16", "B': spans 32..256 + barrier", "A': read + regs DIT",
          "extract: energy prefix (4 barriers), next-block swap", "extract: outputs + stores"]


def main():
    st = torch.cuda.Stream()
    f = _lib.lib().ofs_mp_prof
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * 8)()
    with torch.cuda.stream(st):
        BC.zc_mf("cuda", st, 2, 1)
        torch.cuda.synchronize()
        f(buf)
        r = BC.zc_mf("cuda", st, 5, 0)
        torch.cuda.synchronize()
        f(buf)
    tot = sum(buf) or 1
    print(json.dumps({"config": r["config"], "ms": r["ms"], "build": _lib.TUNING_BUILD,
                      "phases": {p: round(buf[i] / tot, 4) for i, p in enumerate(PHASES)},
                      "note": "cycle shares over all waves; calls include the warm-up loop"}), flush=True)


if __name__ == "__main__":
    main()
