#!/bin/bash
# Copies the summaries of a tools/profile.sh run (gpurun_out/prof_<tag>) into a
# tracked profiles/ directory: per-config kernel stats, the bench line run under
# the trace, the PMC counter CSVs, a trace summary of the timed launches, and the
# per-launch HBM traffic (tools/pmc_traffic.py, merged into profiles/pmc_traffic.json).
#   bash tools/collect_profile.sh r02a profiles/r02/prof_r02a
set -euo pipefail
TAG=$1
DST=$2
SRC=gpurun_out/prof_$TAG
mkdir -p "$DST"
for d in "$SRC"/trace_c*; do
  c=${d##*trace_c}
  cp "$d/run_kernel_stats.csv" "$DST/kernel_stats_config$c.csv"
  cp "$SRC/bench_c${c}_under_trace.json" "$DST/bench_config${c}_under_trace.json"
  python3 tools/trace_summary.py "$d/run_kernel_trace.csv" 30 > "$DST/trace_summary_config$c.txt"
  for ctr in FETCH_SIZE WRITE_SIZE; do
    f="$SRC/pmc_${ctr}_c$c/run_counter_collection.csv"
    [ -f "$f" ] && cp "$f" "$DST/pmc_${ctr}_config$c.csv"
  done
done
python3 tools/pmc_traffic.py "$SRC" profiles/pmc_traffic.json > "$DST/pmc_traffic.json"
