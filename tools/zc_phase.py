"""Diagnostic: per-role cycles of the fused zc_v2 CFAR + gate kernel (OFS_ZC_TIMING build).
    python tools/variants.py zc_cfar.hip "zctime=-DOFS_ZC_TIMING=1"
    OFS_LIB=build/libofdmsync_zctime.so python tools/zc_phase.py
Cycles are summed over the waves of each role (1 walker, ZH helpers per workgroup)."""
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

ROLES = ["walker: DMA issue + wait", "walker: chain", "walker: barrier", "helpers: work", "helpers: barrier"]


def main():
    st = torch.cuda.Stream()
    f = _lib.lib().ofs_zc_prof
    f.argtypes = [ctypes.POINTER(ctypes.c_ulonglong)]
    buf = (ctypes.c_ulonglong * 5)()
    nw = int(os.environ.get("ZC_WAVES", "8"))
    nwg = int(os.environ.get("ZC_WGS", "256"))
    for state in (False, True):
        with torch.cuda.stream(st):
            BC.zc_detect("cuda", st, 2, 1, state=state)
            torch.cuda.synchronize()
            f(buf)
            r = BC.zc_detect("cuda", st, 5, 0, state=state)
            torch.cuda.synchronize()
            f(buf)
        w = sum(buf[:3]) or 1
        h = sum(buf[3:]) or 1
        print(json.dumps({"config": r["config"], "ms": r["ms"],
                          "walker": {ROLES[i]: round(buf[i] / w, 4) for i in range(3)},
                          "helpers": {ROLES[i]: round(buf[i] / h, 4) for i in range(3, 5)},
                          "walker_cycles_per_wave_launch": w / (5 * nwg), "helper_cycles_per_wave_launch": h / (5 * nwg * (nw - 1))}),
              flush=True)
    # wave placement: HW_ID (gfx9: wave 3:0, simd 5:4, pipe 7:6, cu 11:8, sh 12, se 15:13) of every
    # wave of the first 512 workgroups -> which waves share a SIMD with the walker
    g = _lib.lib().ofs_zc_hwid
    g.argtypes = [ctypes.POINTER(ctypes.c_uint)]
    hw = (ctypes.c_uint * (4096 * 8))()
    g(hw)
    from collections import Counter, defaultdict
    nw = int(os.environ.get("ZC_WAVES", "8"))           # waves per workgroup of the build timed
    nwg = int(os.environ.get("ZC_WGS", "256"))          # workgroups (4096 streams / streams per workgroup)
    simd_of = {}
    per_cu = defaultdict(list)
    for wg in range(nwg):
        for w in range(nw):
            v = hw[wg * 8 + w]
            simd, cu, sh, se = (v >> 4) & 3, (v >> 8) & 15, (v >> 12) & 1, (v >> 13) & 7
            simd_of[(wg, w)] = simd
            per_cu[(se, sh, cu)].append((wg, w, simd))
    walker_simd = Counter(simd_of[(wg, 0)] for wg in range(nwg))
    shared = Counter()
    for key, lst in per_cu.items():
        wsimds = Counter(s for wg, w, s in lst if w == 0)
        hsimds = Counter(s for wg, w, s in lst if w != 0)
        shared[sum(hsimds[s] for s in wsimds)] += 1
    print(json.dumps({"walker_simd_hist": dict(walker_simd), "helper_waves_on_walker_simds_per_cu_hist": dict(shared),
                      "cus_seen": len(per_cu), "example": [per_cu[k] for k in list(per_cu)[:3]]}), flush=True)


if __name__ == "__main__":
    main()
