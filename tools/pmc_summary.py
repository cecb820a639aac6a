"""Summarise rocprofv3 --pmc counter_collection.csv files per kernel (average per dispatch).

    python tools/pmc_summary.py FILE.csv [FILE2.csv ...] [--match REGEX] [--json OUT]

Rows of one dispatch are merged across files by (kernel, dispatch order within the kernel), so
separate passes of the same command (one counter group each) combine.  Derived columns: VALU
per wave, waits as fractions of SQ_WAVE_CYCLES, mean resident waves per CU (SQ_WAVE_CYCLES /
(SQ_BUSY_CYCLES · 4 ... see below) and the kernel duration from the timestamps.
"""
from __future__ import annotations

import argparse
import csv
import json
import re
from collections import defaultdict


def short(name: str) -> str:
    name = name.replace("void ", "").replace("(anonymous namespace)::", "")
    name = re.sub(r"\(.*", "", name)
    name = re.sub(r"^.*::", "", name) if "<" not in name else name
    return name[:90]


def load(paths, match):
    per = defaultdict(lambda: defaultdict(dict))      # kernel -> dispatch ordinal -> counters
    for p in paths:
        seen = defaultdict(dict)
        with open(p) as fh:
            for r in csv.DictReader(fh):
                k = short(r["Kernel_Name"])
                if match and not re.search(match, k):
                    continue
                did = int(r["Dispatch_Id"])
                d = seen[k].setdefault(did, {"_dur_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                             "_vgpr": int(r["VGPR_Count"]), "_lds": int(r["LDS_Block_Size"]),
                                             "_grid": int(r["Grid_Size"]), "_wg": int(r["Workgroup_Size"])})
                d[r["Counter_Name"]] = d.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
        for k, ds in seen.items():
            for i, did in enumerate(sorted(ds)):
                per[k][i].update(ds[did])
    return per


def summarise(per):
    out = {}
    for k, ds in per.items():
        keys = set().union(*[d.keys() for d in ds.values()])
        avg = {c: sum(d.get(c, 0.0) for d in ds.values()) / len(ds) for c in keys}
        avg["_dispatches"] = len(ds)
        w = avg.get("SQ_WAVES")
        if w:
            if "SQ_INSTS_VALU" in avg:
                avg["valu_per_wave"] = avg["SQ_INSTS_VALU"] / w
            if "SQ_INSTS_LDS" in avg:
                avg["lds_per_wave"] = avg["SQ_INSTS_LDS"] / w
        wc = avg.get("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU"):
                if c in avg:
                    avg[c.lower() + "_frac"] = avg[c] / wc
            if avg.get("SQ_BUSY_CYCLES"):
                # SQ_WAVE_CYCLES sums quad-cycles over resident waves; SQ_BUSY_CYCLES counts
                # quad-cycles the SQs were busy, summed over the 32 SEs... the ratio is the mean
                # number of resident waves per SQ (per CU) while busy (relative occupancy)
                avg["waves_per_busy_sq"] = wc / avg["SQ_BUSY_CYCLES"]
        out[k] = avg
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("files", nargs="+")
    ap.add_argument("--match", default="")
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    s = summarise(load(a.files, a.match))
    for k, v in sorted(s.items(), key=lambda kv: -kv[1]["_dur_ns"]):
        print(f"{k}  [{v['_dispatches']} disp, {v['_dur_ns'] / 1e3:.1f} us, vgpr {v['_vgpr']:.0f}, lds {v['_lds']:.0f}]")
        for c in sorted(x for x in v if not x.startswith("_")):
            print(f"    {c:28s} {v[c]:.4g}")
    if a.json:
        json.dump(s, open(a.json, "w"), indent=1, sort_keys=True)


if __name__ == "__main__":
    main()
