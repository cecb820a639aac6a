"""Kernel durations of the TIMED calls from a rocprofv3 kernel trace of tools/bench_configs.py.

bench_configs times `steps` calls after >= 100 ms of warm-up calls (timed()); the trace's
kernel_stats average mixes both (the first calls run before the clocks settle).  This prints, per
kernel matching --match, the average / min / max duration of the last --last dispatches (the timed
calls) and of all of them.

    python tools/kt_tail.py gpurun_out/X_kt/cfg_kernel_trace.csv --match zc_pair --last 3
"""
import argparse
import csv
import json
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--match", required=True, help="substring of the kernel name")
    ap.add_argument("--last", type=int, default=3, help="dispatches at the end of the trace (the timed calls)")
    a = ap.parse_args()
    rows = [r for r in csv.DictReader(open(a.trace)) if a.match in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    tail = dur[-a.last:]
    print(json.dumps({"kernel": rows[-1]["Kernel_Name"][:120] if rows else None, "dispatches": len(dur),
                      "timed_last": len(tail), "timed_avg_us": round(statistics.mean(tail), 2) if tail else None,
                      "timed_min_us": round(min(tail), 2) if tail else None,
                      "timed_max_us": round(max(tail), 2) if tail else None,
                      "all_avg_us": round(statistics.mean(dur), 2) if dur else None,
                      "all_median_us": round(statistics.median(dur), 2) if dur else None}))


if __name__ == "__main__":
    main()
