#!/usr/bin/env python3
"""Per-kernel duration summary of a rocprofv3 --kernel-trace csv (measurement only).

For each yucsum kernel: dispatches, mean / median over all of them, and the mean over
the last K dispatches (the timed steps of a bench run, warm-up excluded), which is
what bench.py's HIP-event kernel time is compared against.

usage: tools/trace_summary.py run_kernel_trace.csv [K]
"""
import csv
import statistics
import sys
from collections import defaultdict


def main(path, k):
    d = defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "(anonymous namespace)::k_" not in name:
            continue
        d[name.split("(anonymous namespace)::")[1].split("(")[0]].append(
            (int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    out = {}
    for name, v in d.items():
        v.sort()
        durs = [x[1] / 1e3 for x in v]
        out[name] = {"dispatches": len(durs), "mean_us": round(statistics.mean(durs), 2),
                     "median_us": round(statistics.median(durs), 2),
                     f"mean_last{k}_us": round(statistics.mean(durs[-k:]), 2)}
        print(name, out[name])
    return out


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 20)
