#!/usr/bin/env python3
"""Per-launch HBM traffic of the checksum kernel from rocprofv3 PMC passes.

Reads the FETCH_SIZE and WRITE_SIZE counter CSVs written by tools/profile.sh and
applies MI355X_MICROARCH.md §HBM: counters are in KiB; on gfx950 FETCH_SIZE reports
exactly half the bytes of a wide (16 B/lane) coalesced streaming read, so it is
doubled. Writes profiles/pmc_traffic.json, which bench.py reports as
roofline.traffic.

usage: tools/pmc_traffic.py gpurun_out/prof_r01 profiles/pmc_traffic.json
"""
import csv
import json
import os
import statistics
import sys

import re


def short_name(full):
    """'void (anonymous namespace)::k_small<16, 6, 2>(...)' -> 'k_small<16,6>' (the
    name bench.py reports; the load-policy template argument is dropped)."""
    m = re.search(r"::(k_\w+)<([^>]*)>", full)
    if not m:
        return None
    k, args = m.group(1), [a.strip() for a in m.group(2).split(",")]
    if k == "k_small":
        return f"k_small<{args[0]},{args[1]}>"
    if k in ("k_tiny", "k_lane"):
        return f"{k}<{args[0]}>"
    if k == "k_loop":
        return f"k_loop<{args[0]},{'BE' if args[2] == 'true' else 'LE'}>"
    if k == "k_seg":
        kind = {"2": ",rx", "true": ",rx", "1": ",tx", "3": ",dg", "4": ",txw"}.get(args[2], "")  # template K
        ch = f",c{args[3]}" if len(args) > 3 and args[3] != "64" else ""  # packets per chunk
        return f"k_seg<{args[0]}{kind}{ch}>"
    if k == "k_rag":
        return f"k_rag<{args[0]},{args[1]}>"
    return k


def per_launch(path):
    """Median counter value per launch of the checksum kernel with the most
    dispatches in this CSV (the timed kernel)."""
    by = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            n = short_name(row["Kernel_Name"])
            if n:
                by.setdefault(n, []).append(float(row["Counter_Value"]))
    if not by:
        return None, None, 0
    name = max(by, key=lambda k: len(by[k]))
    return name, statistics.median(by[name]), len(by[name])


def main(prof_dir, out_path):
    res = {}
    if os.path.exists(out_path):  # merge: configs not profiled in prof_dir keep their record
        with open(out_path) as f:
            res = json.load(f)
    for c in ("2", "3", "4", "6", "7", "8", "9", "10", "11", "12", "13"):
        cfg = f"config{c}"
        fpath = os.path.join(prof_dir, f"pmc_FETCH_SIZE_c{c}", "run_counter_collection.csv")
        wpath = os.path.join(prof_dir, f"pmc_WRITE_SIZE_c{c}", "run_counter_collection.csv")
        if not (os.path.exists(fpath) and os.path.exists(wpath)):
            continue
        kern, fetch, nf = per_launch(fpath)
        kern_w, write, nw = per_launch(wpath)
        if fetch is None or write is None or kern != kern_w:
            continue
        res[cfg] = {
            "kernel": kern,
            "fetch_size_kib": fetch,
            "write_size_kib": write,
            "hbm_bytes_per_launch": int(round((2 * fetch + write) * 1024)),
            "launches": min(nf, nw),
            "source": f"{os.path.basename(prof_dir.rstrip('/'))}: rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE "
                      "(separate passes), median per launch, 2 x FETCH_SIZE (gfx950) + WRITE_SIZE, KiB",
        }
    with open(out_path, "w") as f:
        json.dump(res, f, indent=2)
    print(json.dumps(res, indent=2))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
