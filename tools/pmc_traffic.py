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

KERNELS = {"config2": "k_small<4, 1, true>", "config3": "k_small<16, 6, true>",
           "config4": "k_loop<4, true, true>"}
NAMES = {"k_small<4, 1, true>": "k_small<4,1>", "k_small<16, 6, true>": "k_small<16,6>",
         "k_loop<4, true, true>": "k_loop<4,BE>"}


def per_launch(path, kernel):
    vals = []
    with open(path) as f:
        for row in csv.DictReader(f):
            if kernel in row["Kernel_Name"]:
                vals.append(float(row["Counter_Value"]))
    return statistics.median(vals) if vals else None, len(vals)


def main(prof_dir, out_path):
    res = {}
    for cfg, kern in KERNELS.items():
        c = cfg[-1]
        fpath = os.path.join(prof_dir, f"pmc_FETCH_SIZE_c{c}", "run_counter_collection.csv")
        wpath = os.path.join(prof_dir, f"pmc_WRITE_SIZE_c{c}", "run_counter_collection.csv")
        if not (os.path.exists(fpath) and os.path.exists(wpath)):
            continue
        fetch, nf = per_launch(fpath, kern)
        write, nw = per_launch(wpath, kern)
        if fetch is None or write is None:
            continue
        res[cfg] = {
            "kernel": NAMES[kern],
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
