"""Median per-dispatch SQ counters of the yucsum kernels in a rocprofv3 --pmc csv tree."""
import csv, glob, statistics, sys
from collections import defaultdict

for d in sys.argv[1:]:
    vals = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"]
            if "k_" not in k:
                continue
            vals[k.split("(")[0].split("::")[-1]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, c in vals.items():
        m = {n: statistics.median(v) for n, v in c.items()}
        wc = m.get("SQ_WAVE_CYCLES", 1)
        print(d, k, {n: f"{v:.3g}" for n, v in sorted(m.items())})
        print("   wait_any %.2f  wait_inst %.2f  active %.2f  valu/active %.2f" % (
            m.get("SQ_WAIT_ANY", 0) / wc, m.get("SQ_WAIT_INST_ANY", 0) / wc,
            m.get("SQ_ACTIVE_INST_ANY", 0) / wc, m.get("SQ_ACTIVE_INST_VALU", 0) / max(1, m.get("SQ_ACTIVE_INST_ANY", 1))))
